"""Autograd glue: each drop-in module's forward is one torch.autograd.Function whose forward and backward run
the explicit native programs of asrx.blocks.  Weight gradients are written by the kernels straight into the
flat gradient buffer that `p.grad` views (asrx.params); the Functions return None for parameters.

`model_forward` / `model_backward` are also used directly (no autograd) by the fused trainer (asrx.train).
"""
import os

import torch

from . import blocks as Bk
from . import kernels as K
from .kernels import MaskSpec
from .params import FlatParams


# ------------------------------------------------------------------------------------------- store / context

def root_of(m):
    r = m.__dict__.get("_asrx_root")
    r = r() if r is not None else None
    return r if r is not None else m


def param_order(root):
    """Module order, except that the decoder's per-layer cross-attention K/V projections are grouped into one
    contiguous [n_layers*2d, d] block (+ bias block): the all-layer K/V GEMM reads them as one matrix."""
    from .model import Decoder
    ps = list(root.parameters())
    decs = [m for m in root.modules() if isinstance(m, Decoder)]
    for dec in decs:
        wkv = [l._cross_attention.wkv for l in dec._layers]
        bkv = [l._cross_attention.bkv for l in dec._layers]
        if not wkv:
            continue
        ids = {id(p) for p in wkv + bkv}
        pos = min(i for i, p in enumerate(ps) if id(p) in ids)
        rest = [p for p in ps if id(p) not in ids]
        ps = rest[:pos] + wkv + bkv + rest[pos:]
    return ps


def get_store(m):
    root = root_of(m)
    st = root.__dict__.get("_asrx_store")
    try:
        dev = next(root.parameters()).device
    except StopIteration:
        raise RuntimeError("asrx: module has no parameters")
    if dev.type != "cuda":
        raise RuntimeError("asrx modules compute on the GPU only (libasrx.so, gfx950); move the model with .cuda()")
    if st is None or st.device != dev or not st.valid():
        st = FlatParams(param_order(root), dev)
        root.__dict__["_asrx_store"] = st
    return st


_SEED_FALLBACK = {}   # device index -> (initial seed, counter) when the CUDA generator cannot be read (capture)


def draw_seed(device):
    """Dropout seed base of one training call, taken where the reference's nn.Dropout takes its masks on the GPU:
    torch's CUDA generator of `device` — its seed and Philox offset, the offset advanced by 4 as a dropout kernel
    of torch would.  Runs are reproducible under torch.manual_seed / torch.cuda.manual_seed, and neither torch's
    CPU generator (DataLoader shuffling, other CPU RNG users) nor eval / no-dropout calls consume anything."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    gen = torch.cuda.default_generators[idx]
    seed = gen.initial_seed()
    if torch.cuda.is_current_stream_capturing():
        base, n = _SEED_FALLBACK.get(idx, (seed, 0))
        if base != seed:
            n = 0
        _SEED_FALLBACK[idx] = (seed, n + 1)
        off = (1 << 40) + n
    else:
        off = gen.get_offset()
        gen.set_offset(off + 4)
    return int((seed * 0x9E3779B97F4A7C15 + off * 0xBF58476D1CE4E5B9) & ((1 << 62) - 1))


def make_ctx(m, p_drop):
    root = root_of(m)
    st = get_store(m)
    prec = getattr(root, "precision", "bf16")
    cd = torch.bfloat16 if prec == "bf16" else torch.float32
    if cd == torch.bfloat16:
        st.refresh_shadow()
    train = m.training
    seeds = Bk.Seeds(draw_seed(st.device) if train and p_drop > 0 else 0)
    return Bk.Ctx(st, cd, train, p_drop, seeds, getattr(root, "attention", "fused"))


def _prepare_grads(C):
    st = C.store
    unbound = [p for p in st.params if p.grad is None or p.grad.data_ptr() != st._view(st.grad, p).data_ptr()]
    if not unbound:
        return
    if len(unbound) == len(st.params):
        st.zero_grad()
        for p in st.params:
            p.grad = st._view(st.grad, p)
    else:
        for p in unbound:
            st.ensure_grad(p)


def _params(m):
    return tuple(p for p in m.parameters())


# ------------------------------------------------------------------------------------------- programs

def encoder_input(C, x):
    """Accepts the FrontEnd's logical (B, 64, F'', T'') tensor (ideally the permuted view of its (B, T'', F'', 64)
    buffer) and returns (feats [B*T'', F''*64] compute dtype, B, T'')."""
    if x.dim() != 4:
        raise ValueError("Encoder expects the input_layer output (B, 64, F'', T'')")
    B, Cc, F2, T2 = x.shape
    buf = x.permute(0, 3, 2, 1)
    if not buf.is_contiguous() or buf.dtype != C.cd:
        buf = buf.to(C.cd).contiguous()
    return buf.reshape(B * T2, F2 * Cc), B, T2


def encoder_fwd(C, enc, feats, B, T):
    d = enc.emb_dim
    H = enc.num_heads
    x = torch.empty(B * T, d, dtype=torch.float32, device=feats.device)
    pe = enc._pe.pe[0]
    if T > pe.shape[0]:
        raise ValueError(f"encoder length {T} exceeds the PE table ({pe.shape[0]}) as in layers.py:73")
    K.linear(feats, C.W(enc._lin_in.weight), x, bias=enc._lin_in.bias.data, rowadd=pe, rowadd_mod=T, ld_rowadd=d)
    Ss = []
    for layer in enc._layers:
        x, S = Bk.enc_layer_fwd(C, x, layer, B, T, H)
        Ss.append(S)
    y, mean, rstd = Bk.ln_fwd(C, x, enc._norm_out)
    return y, dict(feats=feats, x=x, mean=mean, rstd=rstd, layers=Ss)


def _spans(C, params):
    """Maximal [start, end) element ranges of the flat gradient buffer covered by `params` (a module's params
    need not be adjacent: e.g. Encoder._norm_out is registered before the layers).  Two params merge only if
    the second starts at the first aligned offset after the first, so no other parameter lies in between."""
    from .params import ALIGN
    st = C.store
    iv = sorted((st.offset(p), st.offset(p) + p.numel()) for p in params)
    out = []
    for a, b in iv:
        if out and a == -(-out[-1][1] // ALIGN) * ALIGN:
            out[-1][1] = b
        else:
            out.append([a, b])
    return [tuple(x) for x in out]


def _release(C, ready, params):
    """Flush the queued weight-gradient / LayerNorm reductions, hand the finished ranges to the all-reduce and
    re-open the queues (multi-GPU backward only)."""
    if ready is None or C.wq is None:
        return
    C.flush_wgrad()
    if C.fresh is not None:   # unwritten (unzeroed) weight gradients must not reach the all-reduce
        C.fresh.drain(params, C.store)
    for a, b in _spans(C, params):
        ready(a, b)
    boundary = getattr(ready, "boundary", None)   # graph capture: the released ranges end a captured segment
    if boundary is not None:
        boundary()
    C.defer_wgrad()


# encoder layers per gradient release of the multi-GPU backward (ASRX_DP_RELEASE_LAYERS; 0 = by tile rounds, below).
# Every release ends a grouped weight-gradient launch, so finer releases trade all-reduce overlap for fuller launches.
RELEASE_LAYERS = int(os.environ.get("ASRX_DP_RELEASE_LAYERS", "0"))


def _wgrad_tile():
    """(rows, cols) of one weight-gradient tile of the grouped launch's kernel (kernels.WGRAD_KIND)."""
    return K._TILE_CODE.get(K.WGRAD_KIND, ((256, 256), 0))[0]


def _tiles(m, n):
    tm, tn = _wgrad_tile()
    return -(-m // tm) * -(-n // tn)


def _queued_tiles(C, start=0):
    """Output tiles of the weight gradients queued since queue position `start` (one tile per workgroup in the
    grouped launch, one workgroup per CU)."""
    return sum(_tiles(dy.shape[1], x.shape[1]) for (dy, x, _, _) in (C.wq or [])[start:])


def _num_cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 256


def release_groups(n, every=None):
    """The encoder layer ranges [lo, hi) released together, in backward order: groups of `every` layers from the
    top; the lowest group (with _lin_in and the front-end) is left to the reducer's finish()."""
    every = RELEASE_LAYERS if every is None else every
    k = every if every > 0 else max(1, n // 2)
    out, hi = [], n
    while hi - k > 0:
        out.append((hi - k, hi))
        hi -= k
    return out


def encoder_bwd(C, enc, S, dy, gate_feats, ready=None, release_every=None, carry=None):
    """dy: grad of the encoder output (fp32 or compute dtype). Returns dfeats (compute dtype).  With `ready`, the
    layers are released to the gradient all-reduce in groups (release_groups; the first with _norm_out) as soon as
    their gradients are final.  carry: parameters (the decoder's) released with the first group (else at finish)."""
    x = S["x"]
    dx_c = torch.empty(x.shape, dtype=C.cd, device=x.device)
    dx = Bk.ln_bwd(C, x, dy, enc._norm_out, S["mean"], S["rstd"], drop_out=dx_c)
    n = len(S["layers"])
    # by tile rounds (the default): ONE release, at the highest layer i whose lower layers 0..i-1 plus _lin_in fit
    # one round of weight-gradient tiles (one workgroup per CU).  The released launch carries the decoder's weight
    # gradients and layers n-1..i (c3: 7 layers; modelled makespan 626 K-steps), the finish() launch the rest (250
    # tiles, 249 K-steps): 875 in all, the single-GPU launch's makespan.  (Releases every 5 layers — one round each —
    # overlapped more of the all-reduce but made 505 + 249 + 249 K-steps.)
    by_rounds = ready is not None and C.wq is not None and release_every is None and RELEASE_LAYERS == 0
    groups = {} if by_rounds else {lo: hi for lo, hi in release_groups(n, release_every)}
    hi, q0, cus = n, len(C.wq or []), _num_cus(x.device)
    lw = enc._lin_in.weight
    tail = _tiles(lw.shape[0], lw.shape[1])
    for i, layer_S in reversed(list(enumerate(S["layers"]))):
        nxt = torch.empty(x.shape, dtype=C.cd, device=x.device)
        dx = Bk.enc_layer_bwd(C, layer_S, dx, dx_c, nxt)
        dx_c = nxt
        if by_rounds and i > 0 and C.wq is not None and hi == n:
            per = _queued_tiles(C, q0) // (n - i)
            if i * per + tail <= cus:
                groups[i] = hi
        if i in groups:
            extra = list(enc._norm_out.parameters()) if groups[i] == n else []
            _release(C, ready, [p for l in enc._layers[i:groups[i]] for p in l.parameters()] + extra + (carry or []))
            carry = None
            hi, q0 = i, len(C.wq or [])
    feats = S["feats"]
    dfeats = torch.empty(feats.shape, dtype=C.cd, device=x.device)
    w = enc._lin_in.weight
    if gate_feats:
        K.linear_dgrad(dx_c, C.W(w), dfeats, gate=feats, ld_gate=feats.shape[1])
    else:
        K.linear_dgrad(dx_c, C.W(w), dfeats)
    C.wgrad(dx_c, feats, C.G(w), C.G(enc._lin_in.bias))
    return dfeats


def _kv_block(C, dec):
    st = C.store
    n = len(dec._layers)
    first_w = dec._layers[0]._cross_attention.wkv
    first_b = dec._layers[0]._cross_attention.bkv
    d = dec.emb_dim
    buf = st.shadow if C.cd == torch.bfloat16 else st.flat
    W = st.span(first_w, n, buf)
    bias = st.span(first_b, n, st.flat)
    gW = st.span(first_w, n, st.grad)
    gb = st.span(first_b, n, st.grad)
    if W is None or bias is None:
        raise RuntimeError("asrx: cross-attention K/V parameters are not contiguous in the flat store")
    return W.view(n * 2 * d, d), bias, gW.view(n * 2 * d, d), gb


def decoder_fwd(C, dec, text, mask, enc_c, B, L, Te, final_norm=True, spec=None):
    d, H, n = dec.emb_dim, dec.num_heads, len(dec._layers)
    dev = enc_c.device
    Md = B * L
    text = text.to(device=dev, dtype=torch.int64).contiguous()
    if spec is None:
        spec = MaskSpec.decoder(mask.to(dev))
    pe = dec._pe.pe[0]
    if L > pe.shape[0]:
        raise ValueError(f"decoder length {L} exceeds the PE table ({pe.shape[0]})")
    x = torch.empty(Md, d, dtype=torch.float32, device=dev)
    s_emb = C.seed()
    K.embed_fwd(text, dec._embedding.weight.data, pe, x, L, C.p, s_emb)
    Wkv, bkv, _, _ = _kv_block(C, dec)
    kv = torch.empty(B * Te, n * 2 * d, dtype=C.cd, device=dev)
    K.linear(enc_c, Wkv, kv, bias=bkv)
    Ss = []
    for l, layer in enumerate(dec._layers):
        x, S = Bk.dec_layer_fwd(C, x, layer, B, L, H, spec, kv[:, l * 2 * d:], n * 2 * d, Te)
        Ss.append(S)
    cls = dec._classifier
    if final_norm:
        h, mean, rstd = Bk.ln_fwd(C, x, dec._norm_layer)
    else:
        h, mean, rstd = x.to(C.cd), None, None
    logits = torch.empty(Md, cls.Vp, dtype=torch.float32, device=dev)
    K.linear(h, C.W(cls.weight), logits)
    return logits, dict(text=text, x=x, h=h, mean=mean, rstd=rstd, kv=kv, enc=enc_c, layers=Ss, s_emb=s_emb,
                        dims=(B, L, Te))


def decoder_bwd(C, dec, S, dlogits_c):
    """dlogits_c: [B*L, Vp] compute dtype (padded columns zero). Returns d(encoder output) fp32 [B*Te, d]."""
    B, L, Te = S["dims"]
    d, n = dec.emb_dim, len(dec._layers)
    x, h = S["x"], S["h"]
    dev = x.device
    cls = dec._classifier
    dh = torch.empty(B * L, d, dtype=C.cd, device=dev)
    K.linear_dgrad(dlogits_c, C.W(cls.weight), dh)
    C.wgrad(dlogits_c, h, C.G(cls.weight))
    dx_c = torch.empty(B * L, d, dtype=C.cd, device=dev)
    dx = Bk.ln_bwd(C, x, dh, dec._norm_layer, S["mean"], S["rstd"], drop_out=dx_c)
    dkv = torch.empty(B * Te, n * 2 * d, dtype=C.cd, device=dev)
    for l in reversed(range(n)):
        nxt = torch.empty(B * L, d, dtype=C.cd, device=dev)
        dx = Bk.dec_layer_bwd(C, S["layers"][l], dx, dx_c, dkv[:, l * 2 * d:], nxt)
        dx_c = nxt
    K.embed_bwd(S["text"], dx, C.G(dec._embedding.weight), L, dec.pad_token_id if dec.pad_token_id is not None else -1,
                C.p, S["s_emb"])
    Wkv, _, gW, gb = _kv_block(C, dec)
    denc = torch.empty(B * Te, d, dtype=torch.float32, device=dev)
    K.linear_dgrad(dkv, Wkv, denc)
    C.wgrad(dkv, S["enc"], gW, gb)
    return denc


def model_forward(C, model, spectrum, text, mask, spec=None):
    """Transformer.forward (model.py:194-198) as one native program. Returns (logits [B*L, Vp] fp32, S).  spec:
    the decoder's self-attention mask when the caller already built it (mask is then unused)."""
    dev = C.store.device
    spectrum = spectrum.to(dev)
    feats, Sf = Bk.frontend_fwd(C, spectrum, model.input_layer[0], model.input_layer[2])
    B = spectrum.shape[0]
    T2 = Sf["dims"][-1]
    enc, Se = encoder_fwd(C, model.encoder, feats, B, T2)
    L = text.shape[1]
    logits, Sd = decoder_fwd(C, model.decoder, text, mask, enc, B, L, T2, spec=spec)
    return logits, dict(f=Sf, e=Se, d=Sd)


def model_backward(C, model, S, dlogits_c, ready=None):
    """Backward of model_forward.  ready(start, end): optional callback that receives flat-gradient ranges as
    they become final (decoder, then upper encoder half) so their all-reduce overlaps the rest of the backward;
    whatever is not released that way is final when this returns."""
    _prepare_grads(C)
    own = C.defer_wgrad()
    denc = decoder_bwd(C, model.decoder, S["d"], dlogits_c)
    # by tile rounds (the default release schedule): the decoder's weight gradients (the 96 long cross K/V tiles and
    # 672 short ones) are not a launch of their own but join the first encoder group's — one ~2-round launch instead
    # of a 313-K-step one plus a 249-K-step one (modelled with kernels.xcd_plan) and one segment boundary fewer;
    # their all-reduce then starts five encoder layers later, still overlapping the rest of the backward
    carry = ready is not None and own and RELEASE_LAYERS == 0
    if own:
        if not carry:
            _release(C, ready, list(model.decoder.parameters()))
    dfeats = encoder_bwd(C, model.encoder, S["e"], denc, gate_feats=True, ready=ready if own else None,
                         carry=list(model.decoder.parameters()) if carry else None)
    Bk.frontend_bwd(C, S["f"], dfeats, model.input_layer[0], model.input_layer[2])
    if own:
        C.flush_wgrad()


def _dlogits_padded(C, dlogits, rows, V, Vp):
    g = torch.zeros(rows, Vp, dtype=C.cd, device=dlogits.device)
    g[:, :V].copy_(dlogits.reshape(rows, V))
    return g


# ------------------------------------------------------------------------------------------- Functions

class _TransformerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, C, spectrum, text, mask, *params):
        logits, S = model_forward(C, model, spectrum, text, mask)
        ctx.model, ctx.C, ctx.S = model, C, S
        B, L = text.shape
        V = model.decoder._classifier.V
        ctx.shape = (B, L, V, logits.shape[1])
        out = logits.view(B, L, -1)
        return out[:, :, :V] if V != logits.shape[1] else out

    @staticmethod
    def backward(ctx, dlogits):
        B, L, V, Vp = ctx.shape
        C = ctx.C
        model_backward(C, ctx.model, ctx.S, _dlogits_padded(C, dlogits, B * L, V, Vp))
        ctx.S = None
        return (None,) * (5 + len(_params(ctx.model)))


def transformer(model, spectrum, text, mask):
    C = make_ctx(model, model.decoder.p)
    return _TransformerFn.apply(model, C, spectrum, text, mask, *_params(model))


class _FrontEndFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fe, C, spectrum, *params):
        feats, S = Bk.frontend_fwd(C, spectrum, fe[0], fe[2])
        ctx.fe, ctx.C, ctx.S = fe, C, S
        B, F, T, F1, T1, F2, T2 = S["dims"]
        return feats.view(B, T2, F2, 64).permute(0, 3, 2, 1)

    @staticmethod
    def backward(ctx, g):
        C, S = ctx.C, ctx.S
        _prepare_grads(C)
        buf = g.permute(0, 3, 2, 1).to(C.cd).contiguous()
        B, F, T, F1, T1, F2, T2 = S["dims"]
        dy2 = buf.view(B * T2, F2 * 64)
        K.ewise(K.EW_RELU_GRAD, dy2, dy2, b=S["feats"])   # the conv2 ReLU gate (model.py:170), in place
        Bk.frontend_bwd(C, S, dy2, ctx.fe[0], ctx.fe[2])
        return (None,) * (3 + len(_params(ctx.fe)))


def frontend(fe, spectrum):
    C = make_ctx(fe, 0.0)
    return _FrontEndFn.apply(fe, C, spectrum, *_params(fe))


class _EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, C, x, *params):
        feats, B, T = encoder_input(C, x)
        y, S = encoder_fwd(C, enc, feats, B, T)
        ctx.enc, ctx.C, ctx.S, ctx.xshape = enc, C, S, (B, T, x.shape[1], x.shape[2])
        return y.view(B, T, -1)

    @staticmethod
    def backward(ctx, g):
        C, S = ctx.C, ctx.S
        _prepare_grads(C)
        B, T, Cc, F2 = ctx.xshape
        own = C.defer_wgrad()
        dfeats = encoder_bwd(C, ctx.enc, S, g.reshape(B * T, -1).contiguous(), gate_feats=False)
        if own:
            C.flush_wgrad()
        dx = dfeats.view(B, T, F2, Cc).permute(0, 3, 2, 1)
        return (None, None, dx) + (None,) * len(_params(ctx.enc))


def encoder(enc, x):
    C = make_ctx(enc, enc.p)
    return _EncoderFn.apply(enc, C, x, *_params(enc))


class _DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dec, C, text, mask, enc_x, *params):
        B, Te, d = enc_x.shape
        enc_c = enc_x.reshape(B * Te, d).to(C.cd).contiguous()
        L = text.shape[1]
        logits, S = decoder_fwd(C, dec, text, mask, enc_c, B, L, Te)
        ctx.dec, ctx.C, ctx.S = dec, C, S
        V = dec._classifier.V
        ctx.shape = (B, L, V, logits.shape[1], Te, d)
        out = logits.view(B, L, -1)
        return out[:, :, :V] if V != logits.shape[1] else out

    @staticmethod
    def backward(ctx, dlogits):
        B, L, V, Vp, Te, d = ctx.shape
        C = ctx.C
        _prepare_grads(C)
        own = C.defer_wgrad()
        denc = decoder_bwd(C, ctx.dec, ctx.S, _dlogits_padded(C, dlogits, B * L, V, Vp))
        if own:
            C.flush_wgrad()
        return (None, None, None, None, denc.view(B, Te, d)) + (None,) * len(_params(ctx.dec))


def decoder(dec, x, mask, enc_x):
    C = make_ctx(dec, dec.p)
    return _DecoderFn.apply(dec, C, x, mask, enc_x, *_params(dec))


@torch.no_grad()
def decoder_evaluate(dec, x, enc_x):
    """Decoder.evaluate (model.py:125-151) with its quirks: causal-only mask, NO final LayerNorm before the
    classifier, no break on EOS (every sample runs seq_len steps), returns the LAST sample's token row and the list
    of logits snapshots `prob[:, :-1].squeeze()` (one per EOS hit or final step, samples in order).

    Eval mode: the whole batch decodes together with per-layer K/V caches (one position per step: causality makes
    the reference's full-prefix recomputation redundant), the cross-attention K/V of all layers projected once, and
    the next tokens chosen on the GPU (asrx_greedy_argmax) — no host round trip until the end.  Train mode with
    dropout (model.py:137 applies self._dropout, and every layer's dropouts are live): the reference's
    per-sample prefix recomputation, whose fresh masks a cache cannot reproduce."""
    if dec.training and dec.p > 0:
        return _decoder_evaluate_recompute(dec, x, enc_x)
    return _decoder_evaluate_cached(dec, x, enc_x)


def _decoder_evaluate_recompute(dec, x, enc_x):
    C = make_ctx(dec, dec.p)
    B, Te, d = enc_x.shape
    V = dec._classifier.V
    probs = []
    decoder_input = None
    for s in range(x.shape[0]):
        decoder_input = x[s].unsqueeze(0).to(enc_x.device)
        e = enc_x[s].reshape(Te, d).to(C.cd).contiguous()
        for i in range(1, dec._seq_len + 1):
            L = decoder_input.shape[1]
            spec = MaskSpec(1, True)
            logits, _ = decoder_fwd(C, dec, decoder_input, None, e, 1, L, Te, final_norm=False, spec=spec)
            prob = logits[:, :V].view(1, L, V)
            next_word = prob.argmax(dim=-1)[:, -1].unsqueeze(1)
            decoder_input = torch.cat([decoder_input, next_word.to(decoder_input.dtype)], dim=-1)
            if next_word.item() == dec._eos_token_id or i == dec._seq_len:
                probs.append(prob[:, :-1].squeeze())
    return decoder_input, probs


def _decoder_evaluate_cached(dec, x, enc_x):
    C = make_ctx(dec, 0.0)
    C.train, C.p = False, 0.0
    dev = enc_x.device
    B, Te, d = enc_x.shape
    n, H, steps = len(dec._layers), dec.num_heads, dec._seq_len
    dh = d // H
    cls = dec._classifier
    V, Vp = cls.V, cls.Vp
    L0 = x.shape[1]
    P = L0 - 1 + steps                      # positions processed (the last input has L0 + steps - 1 tokens)
    pe = dec._pe.pe[0]
    if P > pe.shape[0]:
        raise ValueError(f"decoder length {P} exceeds the PE table ({pe.shape[0]}) as in layers.py:73")
    if B == 0 or steps == 0:
        return x[-1:].to(dev) if B else x.to(dev), []
    enc_c = torch.empty(B * Te, d, dtype=C.cd, device=dev)
    K.cast(enc_x.reshape(B * Te, d).contiguous(), enc_c)
    Wkv, bkv, _, _ = _kv_block(C, dec)
    kvx = torch.empty(B * Te, n * 2 * d, dtype=C.cd, device=dev)      # every layer's cross-attention K/V
    K.linear(enc_c, Wkv, kvx, bias=bkv)
    kvs = torch.empty(n, B, P, 2 * d, dtype=C.cd, device=dev)          # self-attention K/V caches
    logits = torch.empty(B, P, Vp, dtype=torch.float32, device=dev)
    tokens = torch.empty(B, L0 + steps, dtype=torch.int64, device=dev)
    tokens[:, :L0] = x.to(device=dev, dtype=torch.int64)
    cur = tokens[:, 0].contiguous()
    scale = d ** -0.5
    for t in range(P):
        xs = torch.empty(B, d, dtype=torch.float32, device=dev)
        K.embed_fwd(cur, dec._embedding.weight.data, pe[t:t + 1], xs, 1)
        for l, layer in enumerate(dec._layers):
            mha, cr = layer._mask_attention, layer._cross_attention
            # masked self-attention: the new position's K/V join the cache, its query attends to positions 0..t
            h, _, _ = Bk.ln_fwd(C, xs, layer._norm1)
            q = torch.empty(B, d, dtype=C.cd, device=dev)
            wqkv, bqkv = C.W(mha.wqkv), mha.bqkv.data
            K.linear(h, wqkv[:d], q, bias=bqkv[:d])
            cache = kvs[l]
            K.gemm(h, wqkv[d:], cache[:, t], B, 2 * d, d, lda=d, ldb=d, ldc=P * 2 * d, bias=bqkv[d:])
            o = torch.empty(B, d, dtype=C.cd, device=dev)
            st = ((d, d), (2 * d, P * 2 * d), (2 * d, P * 2 * d), (d, d))
            Bk.attn_fwd(C, q, cache, cache[:, :, d:], o, B, H, 1, t + 1, dh, st, scale, MaskSpec())
            x1 = torch.empty(B, d, dtype=torch.float32, device=dev)
            K.linear(o, C.W(mha._out_linear.weight), x1, bias=mha._out_linear.bias.data, resid=xs, ld_resid=d)
            # cross-attention over the encoder output (no mask, model.py:71)
            h2, _, _ = Bk.ln_fwd(C, x1, layer._norm2)
            q2 = torch.empty(B, d, dtype=C.cd, device=dev)
            K.linear(h2, C.W(cr.wq), q2, bias=cr.bq.data)
            o2 = torch.empty(B, d, dtype=C.cd, device=dev)
            kv_l = kvx[:, l * 2 * d:]
            st2 = ((d, d), (n * 2 * d, Te * n * 2 * d), (n * 2 * d, Te * n * 2 * d), (d, d))
            Bk.attn_fwd(C, q2, kv_l, kv_l[:, d:], o2, B, H, 1, Te, dh, st2, scale, MaskSpec())
            x2 = torch.empty(B, d, dtype=torch.float32, device=dev)
            K.linear(o2, C.W(cr._out_linear.weight), x2, bias=cr._out_linear.bias.data, resid=x1, ld_resid=d)
            xs, _ = Bk.ffn_fwd(C, x2, layer._norm3, layer._feedforward)
        hc = torch.empty(B, d, dtype=C.cd, device=dev)       # no final LayerNorm in evaluate (model.py:142)
        K.cast(xs, hc)
        lg = logits[:, t]
        K.gemm(hc, C.W(cls.weight), lg, B, Vp, d, lda=d, ldb=d, ldc=P * Vp)
        if t + 1 >= L0:
            K.greedy_argmax(lg, V, tokens[:, t + 1], cur)
        else:
            cur = tokens[:, t + 1].contiguous()
    tok = tokens.cpu()
    eos = dec._eos_token_id
    probs = []
    for s in range(B):
        for i in range(1, steps + 1):
            Li = L0 + i - 1                                  # input length at step i
            if int(tok[s, Li]) == eos or i == steps:
                probs.append(logits[s:s + 1, :Li - 1, :V].squeeze())
    return tokens[B - 1:B].to(x.dtype), probs


@torch.no_grad()
def transformer_evaluate(model, spectrum, text):
    """Transformer.evaluate (model.py:201-206)."""
    feats = model.input_layer(spectrum)
    enc = model.encoder(feats)
    return model.decoder.evaluate(text, enc)


# ------------------------------------------------------------------------------------------- sub-modules

def _cd_input(C, x):
    return x.reshape(-1, x.shape[-1]).to(C.cd).contiguous()


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ln, C, x, *params):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        y, mean, rstd = Bk.ln_fwd(C, x2, ln, out_dtype=torch.float32)
        ctx.ln, ctx.C, ctx.S, ctx.shape = ln, C, (x2, mean, rstd), x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, g):
        C = ctx.C
        _prepare_grads(C)
        x2, mean, rstd = ctx.S
        dx = Bk.ln_bwd(C, x2, g.reshape(x2.shape).float().contiguous(), ctx.ln, mean, rstd)
        return (None, None, dx.view(ctx.shape)) + (None,) * len(_params(ctx.ln))


def layernorm(ln, x):
    C = make_ctx(ln, 0.0)
    return _LayerNormFn.apply(ln, C, x, *_params(ln))


class _MHAFn(torch.autograd.Function):
    """Standalone MHA: y = Drop(W_o . attn(x W_q, kv W_k, kv W_v) + b_o) — no LayerNorm, no residual."""

    @staticmethod
    def forward(ctx, m, C, x, enc_x, attention_mask, *params):
        B, Lq, d = x.shape
        kv_in = x if enc_x is None else enc_x
        Lk = kv_in.shape[1]
        H = m.num_heads
        dh = d // H
        xc = _cd_input(C, x)
        kc = xc if enc_x is None else _cd_input(C, enc_x)
        if m.cross:
            Wq, bq, Wkv, bkv = C.W(m.wq), m.bq.data, C.W(m.wkv), m.bkv.data
        else:
            Wq = C.W(m.wqkv)[:d]
            bq = m.bqkv.data[:d]
            Wkv, bkv = C.W(m.wqkv)[d:], m.bqkv.data[d:]
        q = torch.empty(B * Lq, d, dtype=C.cd, device=xc.device)
        K.linear(xc, Wq, q, bias=bq)
        kv = torch.empty(B * Lk, 2 * d, dtype=C.cd, device=xc.device)
        K.linear(kc, Wkv, kv, bias=bkv)
        spec = MaskSpec.from_attention_mask(attention_mask.to(xc.device) if attention_mask is not None else None,
                                            B, Lq, Lk)
        o = torch.empty(B * Lq, d, dtype=C.cd, device=xc.device)
        st = ((d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d), (d, Lq * d))
        A = Bk.attn_fwd(C, q, kv, kv[:, d:], o, B, H, Lq, Lk, dh, st, d ** -0.5, spec)
        y = torch.empty(B * Lq, d, dtype=torch.float32, device=xc.device)
        sd = C.seed()
        K.linear(o, C.W(m._out_linear.weight), y, bias=m._out_linear.bias.data, dropout_p=C.p, seed=sd)
        ctx.m, ctx.C = m, C
        ctx.S = dict(xc=xc, kc=kc, q=q, kv=kv, o=o, A=A, sd=sd, dims=(B, Lq, Lk, d), self_attn=enc_x is None,
                     xdtype=x.dtype, kdtype=kv_in.dtype)
        return y.view(B, Lq, d).to(x.dtype) if x.dtype != torch.float32 else y.view(B, Lq, d)

    @staticmethod
    def backward(ctx, g):
        C, S, m = ctx.C, ctx.S, ctx.m
        _prepare_grads(C)
        B, Lq, Lk, d = S["dims"]
        dev = S["xc"].device
        # dropout bwd of the output (same RNG stream as the forward epilogue)
        g2 = g.reshape(B * Lq, d).contiguous()
        dy_c = torch.empty(B * Lq, d, dtype=C.cd, device=dev)
        if C.p > 0:   # the forward epilogue's element mask (same seed), scaled, cast to the compute dtype
            K.ewise(K.EW_DROPOUT, g2, dy_c, p=C.p, seed=S["sd"])
        else:
            K.cast(g2, dy_c)
        do = torch.empty(B * Lq, d, dtype=C.cd, device=dev)
        K.linear_dgrad(dy_c, C.W(m._out_linear.weight), do)
        K.linear_wgrad(dy_c, S["o"], C.G(m._out_linear.weight), bias_grad=C.G(m._out_linear.bias))
        dq = torch.empty(B * Lq, d, dtype=C.cd, device=dev)
        dkv = torch.empty(B * Lk, 2 * d, dtype=C.cd, device=dev)
        q, kv = S["q"], S["kv"]
        gst = ((d, Lq * d), (d, Lq * d), (2 * d, Lk * 2 * d), (2 * d, Lk * 2 * d))
        Bk.attn_bwd(C, S["A"], q, kv, kv[:, d:], S["o"], do, dq, dkv, dkv[:, d:], gst)
        if m.cross:
            Wq, Wkv, gWq, gbq, gWkv, gbkv = C.W(m.wq), C.W(m.wkv), C.G(m.wq), C.G(m.bq), C.G(m.wkv), C.G(m.bkv)
        else:
            Wq, Wkv = C.W(m.wqkv)[:d], C.W(m.wqkv)[d:]
            gw, gb = C.G(m.wqkv), C.G(m.bqkv)
            gWq, gbq, gWkv, gbkv = gw[:d], gb[:d], gw[d:], gb[d:]
        dx = torch.empty(B * Lq, d, dtype=torch.float32, device=dev)
        K.linear_dgrad(dq, Wq, dx)
        K.linear_wgrad(dq, S["xc"], gWq, bias_grad=gbq)
        dk_in = torch.empty(B * Lk, d, dtype=torch.float32, device=dev)
        K.linear_dgrad(dkv, Wkv, dk_in)
        K.linear_wgrad(dkv, S["kc"], gWkv, bias_grad=gbkv)
        if S["self_attn"]:
            K.ewise(K.EW_ADD, dx, dx, b=dk_in)
            return (None, None, _as_dtype(dx.view(B, Lq, d), S["xdtype"]), None, None) + (None,) * len(_params(m))
        return (None, None, _as_dtype(dx.view(B, Lq, d), S["xdtype"]), _as_dtype(dk_in.view(B, Lk, d), S["kdtype"]),
                None) + (None,) * len(_params(m))


def _as_dtype(t, dtype):
    """t in `dtype` (the caller's input dtype): the native cast kernel when it differs."""
    if t.dtype == dtype:
        return t
    out = torch.empty(t.shape, dtype=dtype, device=t.device)
    K.cast(t.contiguous(), out)
    return out


def mha(m, x, enc_x=None, attention_mask=None):
    C = make_ctx(m, m.p)
    return _MHAFn.apply(m, C, x, enc_x, attention_mask, *_params(m))


class _FFNFn(torch.autograd.Function):
    """Standalone FeedForward (layers.py:53-58), no residual."""

    @staticmethod
    def forward(ctx, ff, C, x, *params):
        shape = x.shape
        xc = _cd_input(C, x)
        M = xc.shape[0]
        nf = ff.ff_dim
        f = torch.empty(M, nf, dtype=C.cd, device=xc.device)
        sf = C.seed()
        K.linear(xc, C.W(ff.squeeze.weight), f, bias=ff.squeeze.bias.data, relu=True, dropout_p=C.p, seed=sf)
        y = torch.empty(M, ff.emb_dim, dtype=torch.float32, device=xc.device)
        K.linear(f, C.W(ff.unsqueeze.weight), y, bias=ff.unsqueeze.bias.data)
        ctx.ff, ctx.C, ctx.S = ff, C, (xc, f, shape, x.dtype)
        return y.view(shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        C, ff = ctx.C, ctx.ff
        _prepare_grads(C)
        xc, f, shape, xdt = ctx.S
        M = xc.shape[0]
        g2 = g.reshape(M, -1).float().contiguous()
        g_c = g2.to(C.cd)
        dpre = torch.empty(M, ff.ff_dim, dtype=C.cd, device=xc.device)
        K.linear_dgrad(g_c, C.W(ff.unsqueeze.weight), dpre, alpha=1.0 / (1.0 - C.p) if C.p > 0 else 1.0, gate=f,
                       ld_gate=ff.ff_dim)
        K.linear_wgrad(g_c, f, C.G(ff.unsqueeze.weight), bias_grad=C.G(ff.unsqueeze.bias))
        dx = torch.empty(M, ff.emb_dim, dtype=torch.float32, device=xc.device)
        K.linear_dgrad(dpre, C.W(ff.squeeze.weight), dx)
        K.linear_wgrad(dpre, xc, C.G(ff.squeeze.weight), bias_grad=C.G(ff.squeeze.bias))
        return (None, None, dx.view(shape).to(xdt)) + (None,) * len(_params(ff))


def feed_forward(ff, x):
    C = make_ctx(ff, ff.p)
    return _FFNFn.apply(ff, C, x, *_params(ff))


class _EncLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, layer, C, x, *params):
        B, T, d = x.shape
        x32 = x.reshape(B * T, d).float().contiguous()
        y, S = Bk.enc_layer_fwd(C, x32, layer, B, T, layer.num_heads)
        ctx.layer, ctx.C, ctx.S, ctx.xdt = layer, C, S, x.dtype
        return y.view(B, T, d).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        C = ctx.C
        _prepare_grads(C)
        B, T, d = g.shape
        g32 = g.reshape(B * T, d).float().contiguous()
        dx = Bk.enc_layer_bwd(C, ctx.S, g32, g32.to(C.cd), None)
        return (None, None, dx.view(B, T, d).to(ctx.xdt)) + (None,) * len(_params(ctx.layer))


def encoder_layer(layer, x):
    C = make_ctx(layer, layer.p)
    return _EncLayerFn.apply(layer, C, x, *_params(layer))


class _DecLayerFn(torch.autograd.Function):
    """Standalone DecoderLayer(x, mask, enc_x): `mask` is the attention mask as the reference passes it to
    the layer (bool/uint8 broadcastable to (B, L, L), >0 = masked), cross-attention K/V from enc_x."""

    @staticmethod
    def forward(ctx, layer, C, x, mask, enc_x, *params):
        B, L, d = x.shape
        Te = enc_x.shape[1]
        x32 = x.reshape(B * L, d).float().contiguous()
        enc_c = _cd_input(C, enc_x)
        ca = layer._cross_attention
        kv = torch.empty(B * Te, 2 * d, dtype=C.cd, device=x32.device)
        K.linear(enc_c, C.W(ca.wkv), kv, bias=ca.bkv.data)
        spec = MaskSpec.from_attention_mask(mask.to(x32.device) if mask is not None else None, B, L, L)
        y, S = Bk.dec_layer_fwd(C, x32, layer, B, L, layer.num_heads, spec, kv, 2 * d, Te)
        ctx.layer, ctx.C, ctx.S, ctx.extra = layer, C, S, (enc_c, kv, x.dtype, enc_x.dtype, Te)
        return y.view(B, L, d).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        C, layer = ctx.C, ctx.layer
        _prepare_grads(C)
        enc_c, kv, xdt, edt, Te = ctx.extra
        B, L, d = g.shape
        g32 = g.reshape(B * L, d).float().contiguous()
        dkv = torch.empty(B * Te, 2 * d, dtype=C.cd, device=g32.device)
        dx = Bk.dec_layer_bwd(C, ctx.S, g32, g32.to(C.cd), dkv, None)
        ca = layer._cross_attention
        denc = torch.empty(B * Te, d, dtype=torch.float32, device=g32.device)
        K.linear_dgrad(dkv, C.W(ca.wkv), denc)
        K.linear_wgrad(dkv, enc_c, C.G(ca.wkv), bias_grad=C.G(ca.bkv))
        return (None, None, dx.view(B, L, d).to(xdt), None, denc.view(B, Te, d).to(edt)) + \
            (None,) * len(_params(layer))


def decoder_layer(layer, x, mask, enc_x):
    C = make_ctx(layer, layer.p)
    return _DecLayerFn.apply(layer, C, x, mask, enc_x, *_params(layer))
