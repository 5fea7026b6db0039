"""Native forward / backward programs of the post-LN model family (modules/Transformer/new/), as autograd Functions
over libasrx.so kernels: every GEMM, attention, LayerNorm, embedding and row-wise op goes to the library (no CPU
fallback, no torch arithmetic).  Blocks follow the variant's own module boundaries (new/layers.py:35-64,
new/model.py:9-29,67-91): the residual adds inside MHA / FeedForward are fused into their last GEMM's epilogue, the
post-LN and the non_pad_mask product are one LayerNorm launch plus a row scale.

Activations are row-major [rows, features] with rows = b * T + t; the residual stream is fp32, GEMM operands the
compute dtype (fp32, or bf16 with fp32 accumulation).  Attention heads are full width (head dim = d_model), so the
attention core runs on the materialised-score path (batched GEMMs + the row-softmax kernel), whose masks are the
structured key-validity / causal form.
"""
import torch

from .. import blocks as Bk
from .. import kernels as K
from ..kernels import MaskSpec


def _cd(x, cd):
    """x (any float dtype, contiguous 2-D) in the compute dtype — a native cast when it differs."""
    if x.dtype == cd:
        return x.contiguous()
    out = torch.empty(x.shape, dtype=cd, device=x.device)
    K.cast(x.contiguous(), out)
    return out


def _w(W, cd):
    return _cd(W.detach(), cd)


class Cfg:
    """Per-call configuration: compute dtype, dropout (training only) and the seed stream."""

    def __init__(self, cd, p, training, device):
        self.cd, self.train = cd, training
        self.p = p if training else 0.0
        from ..functions import draw_seed
        self.seeds = Bk.Seeds(draw_seed(device) if training and p > 0 else 0)
        self.ctx = Bk.Ctx(None, cd, training, p, self.seeds, "unfused")

    def seed(self):
        return self.seeds.next() if self.p > 0 else 0


def _wgrad(dy_c, x_c, W, b):
    """(dW, db) of y = x W^T + b with fp32 gradients (fused bias row sums on bf16 operands)."""
    gW = torch.zeros(W.shape, dtype=torch.float32, device=dy_c.device)
    gb = torch.zeros(W.shape[0], dtype=torch.float32, device=dy_c.device) if b is not None else None
    K.linear_wgrad(dy_c, x_c, gW, beta=0.0, bias_grad=gb)
    return gW, gb


class LinearFn(torch.autograd.Function):
    """y = x W^T (+ b) in fp32 (the encoder's lin_in, the classifier)."""

    @staticmethod
    def forward(ctx, x, W, b, cfg):
        xc = _cd(x, cfg.cd)
        y = torch.empty(x.shape[0], W.shape[0], dtype=torch.float32, device=x.device)
        K.linear(xc, _w(W, cfg.cd), y, bias=b.detach() if b is not None else None)
        ctx.save_for_backward(xc, W, b if b is not None else torch.empty(0))
        ctx.cfg, ctx.has_b, ctx.xdt = cfg, b is not None, x.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        xc, W, b = ctx.saved_tensors
        cfg = ctx.cfg
        gc = _cd(g, cfg.cd)
        dx = torch.empty(xc.shape, dtype=torch.float32, device=g.device)
        K.linear_dgrad(gc, _w(W, cfg.cd), dx)
        gW, gb = _wgrad(gc, xc, W, b if ctx.has_b else None)
        return dx if ctx.xdt == torch.float32 else dx.to(ctx.xdt), gW, gb, None


class LNFn(torch.autograd.Function):
    """y = LN(x) * rowmask (post-LN + non_pad_mask, new/model.py:24-25) or LN(x) + table[r % period] (norm_in + pe,
    new/model.py:60); fp32 in / out.  mode: None, ('scale', mask [rows]) or ('add', table [period, d])."""

    @staticmethod
    def forward(ctx, x, gamma, beta, mode, aux):
        x = x.contiguous()
        y = torch.empty_like(x)
        mean, rstd = K.layernorm_fwd(x, gamma.detach(), beta.detach(), y)
        if mode == "scale":
            K.rowwise(K.ROW_SCALE, y, aux, y)
        elif mode == "add":
            K.rowwise(K.ROW_ADD, y, aux, y, period=aux.shape[0])
        ctx.save_for_backward(x, gamma, mean, rstd, aux if mode == "scale" else torch.empty(0))
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, g):
        x, gamma, mean, rstd, m = ctx.saved_tensors
        g = g.contiguous()
        if ctx.mode == "scale":
            gs = torch.empty_like(g)
            K.rowwise(K.ROW_SCALE, g, m, gs)
            g = gs
        d = x.shape[1]
        dgb = torch.zeros(2 * d, dtype=torch.float32, device=x.device)
        dx = K.layernorm_bwd(x, g, gamma.detach(), mean, rstd, dgb)
        return dx, dgb[:d], dgb[d:], None, None


class EmbedFn(torch.autograd.Function):
    """x = dropout(emb(tok) + pe[t]) (new/model.py:120), fp32 [B*L, d]."""

    @staticmethod
    def forward(ctx, table, tok, pe, L, pad_id, cfg):
        tok = tok.reshape(-1).to(torch.int64).contiguous()
        out = torch.empty(tok.numel(), table.shape[1], dtype=torch.float32, device=table.device)
        seed = cfg.seed()
        K.embed_fwd(tok, table.detach(), pe, out, L, cfg.p, seed)
        ctx.save_for_backward(tok)
        ctx.L, ctx.pad, ctx.p, ctx.seed, ctx.shape = L, pad_id, cfg.p, seed, table.shape
        return out

    @staticmethod
    def backward(ctx, g):
        (tok,) = ctx.saved_tensors
        dt = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        K.embed_bwd(tok, g.contiguous(), dt, ctx.L, ctx.pad, ctx.p, ctx.seed)
        return dt, None, None, None, None, None


class MHAResFn(torch.autograd.Function):
    """y = dropout(out(concat_h attn_h(x, kv))) + x (new/layers.py:15-46) for full-width heads: the q / k / v
    projections of all heads in one GEMM (self) or q from x and k / v from kv (cross), scores / softmax / P V on the
    materialised-score path, the out-projection with bias + dropout + the fp32 residual in its epilogue.
    spec: the MaskSpec of the scores (structured key validity / causal)."""

    @staticmethod
    def forward(ctx, x, kv_in, spec, m, cfg, Wq, bq, Wkv, bkv, Wo, bo):
        cd = cfg.cd
        B, Lq, d = x.shape
        Lk = kv_in.shape[1] if kv_in is not None else Lq
        H, hd = m.num_heads, m.num_heads * d
        xf = x.reshape(B * Lq, d).contiguous()
        xc = _cd(xf, cd)
        if kv_in is None:      # Wq / bq: the fused [3 h d, d] q | k | v projection (Wkv, bkv unused)
            qkv = torch.empty(B * Lq, 3 * hd, dtype=cd, device=x.device)
            K.linear(xc, _w(Wq, cd), qkv, bias=bq.detach())
            q, kv, kc = qkv, qkv[:, hd:], None
            st = ((3 * hd, Lq * 3 * hd),) * 3 + ((hd, Lq * hd),)
        else:
            kc = _cd(kv_in.reshape(B * Lk, d), cd)
            q = torch.empty(B * Lq, hd, dtype=cd, device=x.device)
            K.linear(xc, _w(Wq, cd), q, bias=bq.detach())
            kv = torch.empty(B * Lk, 2 * hd, dtype=cd, device=x.device)
            K.linear(kc, _w(Wkv, cd), kv, bias=bkv.detach())
            st = ((hd, Lq * hd), (2 * hd, Lk * 2 * hd), (2 * hd, Lk * 2 * hd), (hd, Lq * hd))
        o = torch.empty(B * Lq, hd, dtype=cd, device=x.device)
        A = Bk.attn_fwd(cfg.ctx, q, kv, kv[:, hd:], o, B, H, Lq, Lk, d, st, d ** -0.5, spec)
        y = torch.empty(B * Lq, d, dtype=torch.float32, device=x.device)
        sd = cfg.seed()
        K.linear(o, _w(Wo, cd), y, bias=bo.detach(), dropout_p=cfg.p, seed=sd, resid=xf, ld_resid=d)
        ctx.cfg, ctx.spec_dims = cfg, (B, Lq, Lk, d, H, hd)
        ctx.S = dict(xc=xc, kc=kc, q=q, kv=kv, o=o, A=A, sd=sd, st=st, self_attn=kv_in is None)
        ctx.save_for_backward(Wq, bq, Wkv, bkv, Wo, bo)
        return y.view(B, Lq, d)

    @staticmethod
    def backward(ctx, g):
        cfg, S = ctx.cfg, ctx.S
        cd = cfg.cd
        Wq, bq, Wkv, bkv, Wo, bo = ctx.saved_tensors
        B, Lq, Lk, d, H, hd = ctx.spec_dims
        dev = g.device
        g2 = g.reshape(B * Lq, d).contiguous().float()
        dy_c = torch.empty(B * Lq, d, dtype=cd, device=dev)
        if cfg.p > 0:      # the out-projection epilogue's keep mask (same seed, element index)
            K.ewise(K.EW_DROPOUT, g2, dy_c, p=cfg.p, seed=S["sd"])
        else:
            K.cast(g2, dy_c)
        do = torch.empty(B * Lq, hd, dtype=cd, device=dev)
        K.linear_dgrad(dy_c, _w(Wo, cd), do)
        gWo, gbo = _wgrad(dy_c, S["o"], Wo, bo)
        q, kv = S["q"], S["kv"]
        dx = torch.empty(B * Lq, d, dtype=torch.float32, device=dev)
        if S["self_attn"]:
            dqkv = torch.empty(B * Lq, 3 * hd, dtype=cd, device=dev)
            gst = ((hd, Lq * hd),) + ((3 * hd, Lq * 3 * hd),) * 3
            Bk.attn_bwd(cfg.ctx, S["A"], q, kv, kv[:, hd:], S["o"], do, dqkv, dqkv[:, hd:], dqkv[:, 2 * hd:], gst)
            K.linear_dgrad(dqkv, _w(Wq, cd), dx)
            gW, gb = _wgrad(dqkv, S["xc"], Wq, bq)
            K.ewise(K.EW_ADD, dx, dx, b=g2)          # + the residual
            return (dx.view(B, Lq, d), None, None, None, None, gW, gb, None, None, gWo, gbo)
        dq = torch.empty(B * Lq, hd, dtype=cd, device=dev)
        dkv = torch.empty(B * Lk, 2 * hd, dtype=cd, device=dev)
        gst = ((hd, Lq * hd), (hd, Lq * hd), (2 * hd, Lk * 2 * hd), (2 * hd, Lk * 2 * hd))
        Bk.attn_bwd(cfg.ctx, S["A"], q, kv, kv[:, hd:], S["o"], do, dq, dkv, dkv[:, hd:], gst)
        K.linear_dgrad(dq, _w(Wq, cd), dx)
        gWq, gbq = _wgrad(dq, S["xc"], Wq, bq)
        K.ewise(K.EW_ADD, dx, dx, b=g2)
        dk_in = torch.empty(B * Lk, d, dtype=torch.float32, device=dev)
        K.linear_dgrad(dkv, _w(Wkv, cd), dk_in)
        gWkv, gbkv = _wgrad(dkv, S["kc"], Wkv, bkv)
        return (dx.view(B, Lq, d), dk_in.view(B, Lk, d), None, None, None, gWq, gbq, gWkv, gbkv, gWo, gbo)


class FFNResFn(torch.autograd.Function):
    """y = x + unsqueeze(dropout(relu(squeeze(x)))) (new/layers.py:59-64): the hidden layer's bias / ReLU /
    dropout in the first GEMM's epilogue, the second GEMM's bias and the fp32 residual in its epilogue; the data
    gradient of the hidden layer gated by its output (f > 0 <=> kept and positive) with the 1/(1-p) scale."""

    @staticmethod
    def forward(ctx, x, cfg, W1, b1, W2, b2):
        cd = cfg.cd
        B, T, d = x.shape
        xf = x.reshape(B * T, d).contiguous()
        xc = _cd(xf, cd)
        f = torch.empty(B * T, W1.shape[0], dtype=cd, device=x.device)
        K.linear(xc, _w(W1, cd), f, bias=b1.detach(), relu=True, dropout_p=cfg.p, seed=cfg.seed())
        y = torch.empty(B * T, d, dtype=torch.float32, device=x.device)
        K.linear(f, _w(W2, cd), y, bias=b2.detach(), resid=xf, ld_resid=d)
        ctx.cfg, ctx.shape = cfg, (B, T, d)
        ctx.save_for_backward(xc, f, W1, b1, W2, b2)
        return y.view(B, T, d)

    @staticmethod
    def backward(ctx, g):
        cfg = ctx.cfg
        cd = cfg.cd
        xc, f, W1, b1, W2, b2 = ctx.saved_tensors
        B, T, d = ctx.shape
        g2 = g.reshape(B * T, d).contiguous().float()
        gc = _cd(g2, cd)
        nf = f.shape[1]
        dpre = torch.empty(B * T, nf, dtype=cd, device=g.device)
        K.linear_dgrad(gc, _w(W2, cd), dpre, alpha=1.0 / (1.0 - cfg.p) if cfg.p > 0 else 1.0, gate=f, ld_gate=nf)
        gW2, gb2 = _wgrad(gc, f, W2, b2)
        dx = torch.empty(B * T, d, dtype=torch.float32, device=g.device)
        K.linear_dgrad(dpre, _w(W1, cd), dx)
        gW1, gb1 = _wgrad(dpre, xc, W1, b1)
        K.ewise(K.EW_ADD, dx, dx, b=g2)
        return dx.view(B, T, d), None, gW1, gb1, gW2, gb2


def valid_spec(valid, causal=False):
    """Structured score mask: key validity (uint8 [B, Lk], 1 = attendable) and / or causality; query rows are never
    masked (the variant masks keys only, new/masking.py:14-29)."""
    if valid is None:
        return MaskSpec(1, causal, None, None, 0) if causal else MaskSpec()
    valid = valid.to(torch.uint8).contiguous()
    return MaskSpec(1, causal, valid, None, valid.stride(0))
