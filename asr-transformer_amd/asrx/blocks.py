"""Forward / backward kernel programs of the Speech-Transformer sublayers.

Every function here issues native kernels only (asrx.kernels -> libasrx.so).  Activations are row-major
token-major matrices [B*T, features]; the residual stream is kept in fp32, GEMM operands in the compute dtype
(bf16 on the training path, fp32 on the parity path).  Forward functions stash what their backward needs in a
plain dict `S`.

Reference call sites (modules/Transformer): pre-LN sublayers model.py:18-25 / 65-75; MHA layers.py:15-40;
FeedForward layers.py:53-58; front-end model.py:168-171 + 41-47; decoder embedding model.py:117.
"""
import bisect
import math

import torch

from . import kernels as K
from .kernels import MaskSpec


class FreshGrads:
    """Weight-gradient regions of the flat fp32 gradient buffer that a training step leaves UNZEROED because their
    only writer is one weight-gradient GEMM (asrx.train.Trainer): the first GEMM that covers such a region exactly
    writes it with beta = 0 (no zero fill before, no read of C inside); any other writer first zeroes the fresh
    regions it overlaps.  Whatever no writer claimed is zeroed by drain()."""

    def __init__(self, store, params):
        self.grad = store.grad
        self.base = store.grad.data_ptr()
        ent = sorted((store.offset(p), p.numel()) for p in params)
        self.offs = [o for o, _ in ent]
        self.live = dict(ent)

    def take(self, gw):
        """True: gw covers only fresh regions, exactly (write with beta 0); they are claimed.  False: the fresh
        regions gw overlaps (if any) are zeroed and claimed (accumulate with beta 1)."""
        if not self.live:
            return False
        a = (gw.data_ptr() - self.base) // 4
        rows, cols = (gw.shape[0], gw.shape[1]) if gw.dim() == 2 else (1, gw.numel())
        ld = gw.stride(0) if gw.dim() == 2 else cols
        b = a + (rows - 1) * ld + cols
        i = bisect.bisect_left(self.offs, a)
        if i > 0 and self.offs[i - 1] + self.live.get(self.offs[i - 1], 0) > a:
            i -= 1
        hit = []
        while i < len(self.offs) and self.offs[i] < b:
            o = self.offs[i]
            if o in self.live:
                hit.append(o)
            i += 1
        if not hit:
            return False
        full = (ld == cols and (gw.dim() < 2 or gw.stride(1) == 1) and hit[0] == a
                and sum(self.live[o] for o in hit) == b - a)
        for o in hit:
            n = self.live.pop(o)
            if not full:
                self.grad[o:o + n].zero_()
        return full

    def drain(self, params=None, store=None):
        """Zero the fresh regions nobody wrote (all, or those of `params` — e.g. before their ranges are handed
        to the gradient all-reduce)."""
        offs = list(self.live) if params is None else [store.offset(p) for p in params if store.offset(p) in self.live]
        for o in offs:
            self.grad[o:o + self.live.pop(o)].zero_()


class Ctx:
    """Per-call configuration shared by the programs."""

    def __init__(self, store, cd, train, p_drop, seeds, attn_impl="fused"):
        self.store = store
        self.cd = cd                    # compute dtype of GEMM operands: torch.bfloat16 | torch.float32
        self.train = train
        self.p = p_drop if train else 0.0
        self.seeds = seeds
        self.attn_impl = attn_impl
        self.wq = None                  # list -> weight gradients are queued and issued grouped (flush_wgrad)
        self.lnq = None                 # list -> LayerNorm dgamma|dbeta partials queued for one grouped reduce
        self.fresh = None               # FreshGrads of a Trainer step (unzeroed weight-gradient regions)
        self.adam = None                # AdamDesc -> the optimizer step fused into the grouped weight gradients
        self.adam_cover = []            # (offset, numel) of the flat-gradient ranges whose AdamW ran fused
        self._gwritten = set()          # data_ptr of every dW / db this step has written so far (fused-AdamW guard)

    def W(self, p):
        return self.store.w16(p) if self.cd == torch.bfloat16 else self.store.w32(p)

    def G(self, p):
        return self.store.g(p)

    def seed(self):
        return self.seeds.next() if self.p > 0 else 0

    def wgrad(self, dy, x, gw, gb=None):
        """dW (+)= dy^T x, db (+)= colsum(dy).  Weight gradients feed nothing but the optimizer, so while a
        queue is open they are deferred and later issued as grouped launches (no split-K)."""
        if self.wq is not None and K.wgrad_groupable(dy, x, gw):
            self.wq.append((dy, x, gw, gb))
        else:
            first = self.fresh is not None and self.fresh.take(gw)
            self._note_writes(gw, gb)
            K.linear_wgrad(dy, x, gw, bias_grad=gb, beta=0.0 if first else 1.0)

    def _note_writes(self, *ts):
        cov = {o for o, _ in self.adam_cover}
        base = self.store.grad.data_ptr()
        for t in ts:
            if t is not None:
                # a gradient whose AdamW already ran fused must never be written again in the step
                assert (t.data_ptr() - base) // 4 not in cov, "asrx: write to a gradient after its fused AdamW"
                self._gwritten.add(t.data_ptr())

    def _adam_safe(self, q0):
        """Fused AdamW is correct only if the grouped launch is the sole and final writer of every dW / db it covers:
        each target appears once in q0 and nothing wrote it before in this step (a second bias contributor, e.g. a
        colsum in a data-gradient epilogue, or an earlier flush).  FreshGrads.take already claimed every dW of q0."""
        seen = set()
        for _, _, gw, gb in q0:
            for t in (gw, gb):
                if t is None:
                    continue
                if t.data_ptr() in seen or t.data_ptr() in self._gwritten:
                    return False
                seen.add(t.data_ptr())
        return True

    def _issue_wgrads(self, q):
        """One grouped launch for the queued weight gradients; with fresh (unzeroed) targets the first writes go
        in a beta = 0 launch ahead of the accumulating one."""
        if self.fresh is None:
            for _, _, gw, gb in q:
                self._note_writes(gw, gb)
            K.linear_wgrad_grouped(q)
            return
        q0, q1 = [], []
        for it in q:
            (q0 if self.fresh.take(it[2]) else q1).append(it)
        # fused AdamW only where every written gradient is final in this launch: first writers (beta 0), no second
        # writer in the step (the Trainer enables it for a single end-of-backward flush only; _adam_safe checks it)
        adam = self.adam if not q1 and self._adam_safe(q0) else None
        for _, _, gw, gb in q0 + q1:
            self._note_writes(gw, gb)
        kname = K.linear_wgrad_grouped(q0, beta=0.0, adam=adam)
        if adam is not None and kname in K.GROUPED_FUSED_KERNELS:
            base = self.store.grad.data_ptr()
            for _, _, gw, gb in q0:
                for t in (gw, gb):
                    if t is not None:
                        self.adam_cover.append(((t.data_ptr() - base) // 4, t.numel()))
        K.linear_wgrad_grouped(q1)

    def defer_wgrad(self):
        if self.cd == torch.bfloat16 and self.wq is None:
            self.wq, self.lnq = [], []
            return True
        return False

    def flush_wgrad(self):
        q, self.wq = self.wq, None
        lq, self.lnq = self.lnq, None
        self._issue_wgrads(q or [])
        K.reduce_rows_grouped(lq or [])


class Seeds:
    def __init__(self, base):
        self.base = base
        self.i = 0

    def next(self):
        self.i += 1
        x = (self.base * 0x9E3779B97F4A7C15 + self.i * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
        return x ^ (x >> 31)


# Fixed choices whose A/B switches were removed in round 5 (measurements in DESIGN §4):
# * the FFN hidden layer's ReLU/dropout mask is kept as bits for the data gradient (not re-read from the bf16 f);
# * the attention keep bits are generated inside the preceding LayerNorm's launch, for the decoder's
#   cross-attention too (round 4);
# * weight gradients are not issued per layer on a side stream (no gain: they compete with the backward chain
#   for the same CUs), nor the keep bits (18.2 vs 17.75 ms/step: the VALU-heavy generator stole the GEMM's CUs).
GATE_BITS = True
LN_DROPGEN = True
LN_DROPGEN_CROSS = True


def _empty(shape, dtype, like):
    return torch.empty(shape, dtype=dtype, device=like.device)


# ------------------------------------------------------------------------------------------------ LayerNorm

def ln_fwd(C, x, ln, out_dtype=None):
    y = _empty(x.shape, out_dtype or C.cd, x)
    mean, rstd = K.layernorm_fwd(x, ln.weight.data, ln.bias.data, y)
    return y, mean, rstd


def ln_grad_buf(C, ln):
    gw, gb = C.G(ln.weight), C.G(ln.bias)
    if gb.data_ptr() == gw.data_ptr() + 4 * gw.numel():
        return C.store.grad[C.store.offset(ln.weight):C.store.offset(ln.weight) + 2 * gw.numel()], None
    tmp = torch.zeros(2 * gw.numel(), device=gw.device, dtype=torch.float32)
    return tmp, (gw, gb)


def ln_bwd(C, x, dy, ln, mean, rstd, dres=None, drop_out=None, drop_seed=0, drop_p=0.0):
    """dx (fp32) = LN^T dy + dres; optional drop_out (compute dtype) = dropout_bwd(dx)."""
    buf, split = ln_grad_buf(C, ln)
    dx = K.layernorm_bwd(x, dy, ln.weight.data, mean, rstd, buf, dres=dres, dx_drop=drop_out, dropout_p=drop_p,
                         seed=drop_seed, defer=C.lnq if split is None else None)
    if split is not None:
        d = split[0].numel()
        K.ewise(K.EW_ADD, split[0], split[0], b=buf[:d])
        K.ewise(K.EW_ADD, split[1], split[1], b=buf[d:])
    return dx


# ------------------------------------------------------------------------------------------------ attention

def attn_prepare(C, B, H, Lq, Lk, dh, device):
    """Draw the attention-dropout seed (the keep bits themselves come from the preceding LayerNorm's launch where
    ln_fwd_attn applies, else from the attention forward's own launch)."""
    return {"seed": C.seed(), "dropmask": None, "event": None}


def attn_fwd(C, q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, prep=None):
    """Fused LDS-tiled kernel on the bf16 path; materialised scores + row softmax otherwise."""
    if prep is None:
        prep = {"seed": C.seed(), "dropmask": None, "event": None}
    seed = prep["seed"]
    S = {"seed": seed, "spec": spec, "dims": (B, H, Lq, Lk, dh), "strides": strides, "scale": scale}
    if C.cd == torch.bfloat16 and C.attn_impl == "fused" and dh in (32, 64):
        dm, ready = prep["dropmask"], prep["event"] is not None or prep.get("ready", False)
        if prep["event"] is not None:
            torch.cuda.current_stream(q.device).wait_event(prep["event"])
        elif not ready:
            dm = K.dropmask_buffer(B, H, Lq, Lk, dh, C.p, q.device)
        S["dropmask"] = dm
        # training: the O rounding residual keeps the backward's delta exact (see include/asrx.h o_lo)
        S["o_lo"] = torch.empty_like(o) if C.train else None
        S["lse"] = K.attention_fwd(q, k, v, o, B, H, Lq, Lk, dh, strides, scale, spec, C.p, seed,
                                   dropmask=dm, dropmask_ready=ready, o_lo=S["o_lo"])
        S["impl"] = "fused"
        return S
    S["impl"] = "unfused"
    (qr, qb), (kr, kb), (vr, vb), (orr, ob) = strides
    ld = (Lk + 7) // 8 * 8
    nbh = B * H
    sc = _empty((nbh, Lq, ld), C.cd, q)
    K.gemm(q, k, sc, Lq, Lk, dh, lda=qr, ldb=kr, ldc=ld, batch=nbh, batch_inner=H, sa=(qb, dh), sb=(kb, dh),
           sc=(H * Lq * ld, Lq * ld))
    p = _empty((nbh, Lq, ld), C.cd, q)
    pd = _empty((nbh, Lq, ld), C.cd, q) if C.p > 0 else None
    K.softmax_fwd(sc, p, pd, nbh, H, Lq, Lk, ld, scale, spec, C.p, seed)
    pv = pd if pd is not None else p
    K.gemm(pv, v, o, Lq, dh, Lk, lda=ld, ldb=vr, ldc=orr, b_trans=True, batch=nbh, batch_inner=H,
           sa=(H * Lq * ld, Lq * ld), sb=(vb, dh), sc=(ob, dh))
    S["p"], S["pd"], S["ld"] = p, pd, ld
    return S


def attn_bwd(C, S, q, k, v, o, do, dq, dk, dv, gstrides):
    B, H, Lq, Lk, dh = S["dims"]
    strides, scale, spec, seed = S["strides"], S["scale"], S["spec"], S["seed"]
    if S["impl"] == "fused":
        K.attention_bwd(q, k, v, o, S["lse"], do, dq, dk, dv, B, H, Lq, Lk, dh, strides, gstrides, scale, spec,
                        C.p, seed, dropmask=S["dropmask"], o_lo=S["o_lo"])
        return
    (qr, qb), (kr, kb), (vr, vb), _ = strides
    (dor, dob), (dqr, dqb), (dkr, dkb), (dvr, dvb) = gstrides
    p, pd, ld = S["p"], S["pd"], S["ld"]
    nbh = B * H
    so = (H * Lq * ld, Lq * ld)
    dpd = _empty((nbh, Lq, ld), C.cd, q)
    K.gemm(do, v, dpd, Lq, Lk, dh, lda=dor, ldb=vr, ldc=ld, batch=nbh, batch_inner=H, sa=(dob, dh), sb=(vb, dh),
           sc=so)
    ds = _empty((nbh, Lq, ld), C.cd, q)
    K.softmax_bwd(p, dpd, ds, nbh, Lq, Lk, ld, scale, C.p, seed)
    pv = pd if pd is not None else p
    # dV = Pd^T dO ; dQ = dS K ; dK = dS^T Q
    K.gemm(pv, do, dv, Lk, dh, Lq, lda=ld, ldb=dor, ldc=dvr, a_trans=True, b_trans=True, batch=nbh, batch_inner=H,
           sa=so, sb=(dob, dh), sc=(dvb, dh))
    K.gemm(ds, k, dq, Lq, dh, Lk, lda=ld, ldb=kr, ldc=dqr, b_trans=True, batch=nbh, batch_inner=H, sa=so,
           sb=(kb, dh), sc=(dqb, dh))
    K.gemm(ds, q, dk, Lk, dh, Lq, lda=ld, ldb=qr, ldc=dkr, a_trans=True, b_trans=True, batch=nbh, batch_inner=H,
           sa=so, sb=(qb, dh), sc=(dkb, dh))


# ------------------------------------------------------------------------------------------------ sublayers

def ln_fwd_attn(C, x, ln, prep, B, H, Lq, Lk, dh, on=True):
    """The sublayer's LayerNorm; where the fused attention will take dropout keep bits, they are generated in the
    same launch (asrx_layernorm_fwd_attn_dropgen) and handed to the attention through prep."""
    d = x.shape[1]
    dm = (K.dropmask_buffer(B, H, Lq, Lk, dh, C.p, x.device)
          if on and LN_DROPGEN and prep["dropmask"] is None and C.cd == torch.bfloat16 and C.attn_impl == "fused"
          and d == 512 and x.dtype == torch.float32 else None)
    if dm is None:
        return ln_fwd(C, x, ln)
    h = _empty(x.shape, C.cd, x)
    mean, rstd = K.layernorm_fwd_dropgen(x, ln.weight.data, ln.bias.data, h, B, H, Lq, Lk, dh, C.p, prep["seed"], dm)
    prep["dropmask"], prep["ready"] = dm, True
    return h, mean, rstd


def self_attn_fwd(C, x, ln, mha, B, T, H, spec):
    """x + Drop(MHA(LN(x))) with fused per-head projections (layers.py:10-12 -> one N=3d GEMM)."""
    M, d = x.shape
    dh = d // H
    prep = attn_prepare(C, B, H, T, T, dh, x.device)
    h, mean, rstd = ln_fwd_attn(C, x, ln, prep, B, H, T, T, dh)
    qkv = _empty((M, 3 * d), C.cd, x)
    K.linear(h, C.W(mha.wqkv), qkv, bias=mha.bqkv.data)
    o = _empty((M, d), C.cd, x)
    st = ((3 * d, T * 3 * d),) * 3 + ((d, T * d),)
    A = attn_fwd(C, qkv, qkv[:, d:], qkv[:, 2 * d:], o, B, H, T, T, dh, st, d ** -0.5, spec, prep)
    y = _empty((M, d), torch.float32, x)
    sd = C.seed()
    K.linear(o, C.W(mha._out_linear.weight), y, bias=mha._out_linear.bias.data, dropout_p=C.p, seed=sd, resid=x,
             ld_resid=d)
    return y, dict(x=x, h=h, mean=mean, rstd=rstd, qkv=qkv, o=o, A=A, sd=sd, ln=ln, mha=mha, H=H, T=T, B=B)


def self_attn_bwd(C, S, dy, dy_c, dx_c_out=None, dx_c_p=0.0, dx_c_seed=0):
    """dy: fp32 grad of the sublayer output; dy_c: dropout_bwd(dy) in the compute dtype (out-proj dY).
    Returns dx (fp32) and fills dx_c_out (compute dtype) = dropout_bwd of dx for the sublayer below."""
    x, h, qkv, o, mha = S["x"], S["h"], S["qkv"], S["o"], S["mha"]
    M, d = x.shape
    T, B = S["T"], S["B"]
    W, G = C.W, C.G
    do = _empty((M, d), C.cd, x)
    K.linear_dgrad(dy_c, W(mha._out_linear.weight), do)
    C.wgrad(dy_c, o, G(mha._out_linear.weight), G(mha._out_linear.bias))
    dqkv = _empty((M, 3 * d), C.cd, x)
    gst = ((d, T * d),) + ((3 * d, T * 3 * d),) * 3
    attn_bwd(C, S["A"], qkv, qkv[:, d:], qkv[:, 2 * d:], o, do, dqkv, dqkv[:, d:], dqkv[:, 2 * d:], gst)
    dh = _empty((M, d), C.cd, x)
    K.linear_dgrad(dqkv, W(mha.wqkv), dh)
    C.wgrad(dqkv, h, G(mha.wqkv), G(mha.bqkv))
    return ln_bwd(C, x, dh, S["ln"], S["mean"], S["rstd"], dres=dy, drop_out=dx_c_out, drop_seed=dx_c_seed,
                  drop_p=dx_c_p)


def cross_attn_fwd(C, x, ln, mha, kv, kv_ld, B, L, Te, H):
    """x + Drop(MHA(LN(x), enc)) — no mask (model.py:71); K/V come from the precomputed all-layer projection."""
    M, d = x.shape
    dh = d // H
    prep = attn_prepare(C, B, H, L, Te, dh, x.device)
    h, mean, rstd = ln_fwd_attn(C, x, ln, prep, B, H, L, Te, dh, on=LN_DROPGEN_CROSS)
    q = _empty((M, d), C.cd, x)
    K.linear(h, C.W(mha.wq), q, bias=mha.bq.data)
    o = _empty((M, d), C.cd, x)
    st = ((d, L * d), (kv_ld, Te * kv_ld), (kv_ld, Te * kv_ld), (d, L * d))
    A = attn_fwd(C, q, kv, kv[:, d:], o, B, H, L, Te, dh, st, d ** -0.5, MaskSpec(), prep)
    y = _empty((M, d), torch.float32, x)
    sd = C.seed()
    K.linear(o, C.W(mha._out_linear.weight), y, bias=mha._out_linear.bias.data, dropout_p=C.p, seed=sd, resid=x,
             ld_resid=d)
    return y, dict(x=x, h=h, mean=mean, rstd=rstd, q=q, o=o, A=A, sd=sd, ln=ln, mha=mha, L=L, Te=Te, kv=kv,
                   kv_ld=kv_ld)


def cross_attn_bwd(C, S, dy, dy_c, dkv, dx_c_out=None, dx_c_p=0.0, dx_c_seed=0):
    x, h, q, o, mha, kv, kv_ld = S["x"], S["h"], S["q"], S["o"], S["mha"], S["kv"], S["kv_ld"]
    M, d = x.shape
    L, Te = S["L"], S["Te"]
    W, G = C.W, C.G
    do = _empty((M, d), C.cd, x)
    K.linear_dgrad(dy_c, W(mha._out_linear.weight), do)
    C.wgrad(dy_c, o, G(mha._out_linear.weight), G(mha._out_linear.bias))
    dq = _empty((M, d), C.cd, x)
    gst = ((d, L * d), (d, L * d), (kv_ld, Te * kv_ld), (kv_ld, Te * kv_ld))
    attn_bwd(C, S["A"], q, kv, kv[:, d:], o, do, dq, dkv, dkv[:, d:], gst)
    dh = _empty((M, d), C.cd, x)
    K.linear_dgrad(dq, W(mha.wq), dh)
    C.wgrad(dq, h, G(mha.wq), G(mha.bq))
    return ln_bwd(C, x, dh, S["ln"], S["mean"], S["rstd"], dres=dy, drop_out=dx_c_out, drop_seed=dx_c_seed,
                  drop_p=dx_c_p)


def ffn_fwd(C, x, ln, ff):
    """x + W2 Drop(ReLU(W1 LN(x) + b1)) + b2 (layers.py:53-58; residual model.py:24,74)."""
    M, d = x.shape
    h, mean, rstd = ln_fwd(C, x, ln)
    nf = ff.squeeze.weight.shape[0]
    f = _empty((M, nf), C.cd, x)
    sf = C.seed()
    # bf16: the epilogue also writes the 1-bit mask f > 0 (ReLU and dropout keep), which the data gradient
    # reads as its gate: M*nf/8 bytes instead of the 2*M*nf of f itself
    fb = None
    if C.train and C.cd == torch.bfloat16 and nf % 32 == 0 and GATE_BITS:   # (only the backward reads them)
        fb = _empty((M, nf // 32), torch.int32, x)
    K.linear(h, C.W(ff.squeeze.weight), f, bias=ff.squeeze.bias.data, relu=True, dropout_p=C.p, seed=sf,
             mask_out=fb, ld_mask=nf // 32)
    y = _empty((M, d), torch.float32, x)
    K.linear(f, C.W(ff.unsqueeze.weight), y, bias=ff.unsqueeze.bias.data, resid=x, ld_resid=d)
    return y, dict(x=x, h=h, mean=mean, rstd=rstd, f=f, fb=fb, ln=ln, ff=ff)


def ffn_bwd(C, S, dy, dy_c, dx_c_out=None, dx_c_p=0.0, dx_c_seed=0):
    x, h, f, ff = S["x"], S["h"], S["f"], S["ff"]
    M, d = x.shape
    nf = f.shape[1]
    W, G = C.W, C.G
    dpre = _empty((M, nf), C.cd, x)
    keep_scale = 1.0 / (1.0 - C.p) if C.p > 0 else 1.0
    # f = Drop(ReLU(pre)) -> dpre = df * [f > 0] / (1-p)   (f > 0 <=> pre > 0 and kept)
    if S.get("fb") is not None:
        K.linear_dgrad(dy_c, W(ff.unsqueeze.weight), dpre, alpha=keep_scale, gate=S["fb"], ld_gate=nf // 32,
                       gate_bits=True)
    else:
        K.linear_dgrad(dy_c, W(ff.unsqueeze.weight), dpre, alpha=keep_scale, gate=f, ld_gate=nf)
    C.wgrad(dy_c, f, G(ff.unsqueeze.weight), G(ff.unsqueeze.bias))
    dh = _empty((M, d), C.cd, x)
    K.linear_dgrad(dpre, W(ff.squeeze.weight), dh)
    C.wgrad(dpre, h, G(ff.squeeze.weight), G(ff.squeeze.bias))
    return ln_bwd(C, x, dh, S["ln"], S["mean"], S["rstd"], dres=dy, drop_out=dx_c_out, drop_seed=dx_c_seed,
                  drop_p=dx_c_p)


# ------------------------------------------------------------------------------------------------ layers

def enc_layer_fwd(C, x, layer, B, T, H):
    """EncoderLayer.forward (model.py:18-25): no attention mask."""
    x1, Sa = self_attn_fwd(C, x, layer._norm1, layer._attention, B, T, H, MaskSpec())
    x2, Sf = ffn_fwd(C, x1, layer._norm2, layer._feedforward)
    return x2, (Sa, Sf)


def enc_layer_bwd(C, S, dy, dy_c, dx_c_out, dx_c_p=0.0, dx_c_seed=0):
    Sa, Sf = S
    d = dy.shape[1]
    dmid_c = _empty(dy.shape, C.cd, dy)
    dmid = ffn_bwd(C, Sf, dy, dy_c, dx_c_out=dmid_c, dx_c_p=C.p, dx_c_seed=Sa["sd"])
    return self_attn_bwd(C, Sa, dmid, dmid_c, dx_c_out=dx_c_out, dx_c_p=dx_c_p, dx_c_seed=dx_c_seed)


def dec_layer_fwd(C, x, layer, B, L, H, spec, kv, kv_ld, Te):
    """DecoderLayer.forward (model.py:65-75)."""
    x1, Sa = self_attn_fwd(C, x, layer._norm1, layer._mask_attention, B, L, H, spec)
    x2, Sc = cross_attn_fwd(C, x1, layer._norm2, layer._cross_attention, kv, kv_ld, B, L, Te, H)
    x3, Sf = ffn_fwd(C, x2, layer._norm3, layer._feedforward)
    return x3, (Sa, Sc, Sf)


def dec_layer_bwd(C, S, dy, dy_c, dkv, dx_c_out, dx_c_p=0.0, dx_c_seed=0):
    Sa, Sc, Sf = S
    d2_c = _empty(dy.shape, C.cd, dy)
    d2 = ffn_bwd(C, Sf, dy, dy_c, dx_c_out=d2_c, dx_c_p=C.p, dx_c_seed=Sc["sd"])
    d1_c = _empty(dy.shape, C.cd, dy)
    d1 = cross_attn_bwd(C, Sc, d2, d2_c, dkv, dx_c_out=d1_c, dx_c_p=C.p, dx_c_seed=Sa["sd"])
    return self_attn_bwd(C, Sa, d1, d1_c, dx_c_out=dx_c_out, dx_c_p=dx_c_p, dx_c_seed=dx_c_seed)


# ------------------------------------------------------------------------------------------------ front-end

def frontend_fwd(C, spectrum, conv1, conv2):
    """input_layer (model.py:168-171) -> (B*T2, F2*64) features, column order f*64 + c (the conv2 GEMM output
    rows are (b, t2, f2), so the reference's view/transpose/contiguous of model.py:43-45 costs nothing)."""
    B, _, F, T = spectrum.shape
    F1, T1 = (F - 3) // 2 + 1, (T - 3) // 2 + 1
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    x = spectrum.contiguous().float()
    y1 = _empty((B, F1, T1, 64), C.cd, x)
    y1m = torch.empty((B, F1, T1, 8), dtype=torch.uint8, device=x.device) if C.cd == torch.bfloat16 else None
    K.conv1_fwd(x, conv1.weight.data.reshape(64, 9).contiguous(), conv1.bias.data, y1, mask=y1m)
    feats = _empty((B * T2, F2 * 64), C.cd, x)
    if C.cd == torch.bfloat16:   # implicit GEMM over y1: no im2col image (forward or backward)
        K.conv2_fwd(y1, C.W(conv2.weight), conv2.bias.data, feats)
        cols = None
    else:
        cols = _empty((B * T2 * F2, 576), C.cd, x)
        K.im2col_conv2(y1, cols)
        K.gemm(cols, C.W(conv2.weight), feats, B * T2 * F2, 64, 576, lda=576, ldb=576, ldc=64,
               bias=conv2.bias.data, relu=True)
    return feats, dict(x=x, y1=y1, y1m=y1m, cols=cols, feats=feats, dims=(B, F, T, F1, T1, F2, T2))


def frontend_bwd(C, S, dfeats_c, conv1, conv2):
    """dfeats_c: gradient of the features (compute dtype, already gated by the conv2 ReLU)."""
    B, F, T, F1, T1, F2, T2 = S["dims"]
    M2 = B * T2 * F2
    dy2 = dfeats_c.view(M2, 64)
    cols = S["cols"]
    G = C.G
    if cols is None:
        gw = G(conv2.weight)
        if C.fresh is not None:
            C.fresh.take(gw)
        K.conv2_wgrad(dy2, S["y1"], gw, G(conv2.bias))
    else:
        C.wgrad(dy2, cols, G(conv2.weight), G(conv2.bias))
    if cols is None and T1 <= K.CONV_BWD_MAXT1:   # conv2 data gradient never materialised
        K.conv_bwd_implicit(dy2, C.W(conv2.weight), S["y1m"], S["x"], G(conv1.weight).view(64, 9), G(conv1.bias))
        return
    dcols = _empty((M2, 576), C.cd, dy2)
    K.linear_dgrad(dy2, C.W(conv2.weight), dcols)
    K.conv1_bwd_fused(dcols, S["y1"], S["x"], G(conv1.weight).view(64, 9), G(conv1.bias))
