"""Drop-in replacements for modules/Transformer/layers.py (MHAHead/MHA, FeedForward,
TrainablePositionalEncoding) plus LayerNorm — same constructor arguments, same forward signatures, same
state_dict key schema; compute goes to libasrx.so.

Storage differs from the reference where the MI355X layout wants it (documented per class); the
state_dict hooks translate both ways so reference checkpoints load verbatim and saved ones load back into
the reference.
"""
import math

import torch
from torch import nn


class _Lin(nn.Module):
    """Parameter container with nn.Linear's state_dict keys (weight (out,in), bias (out)); no forward —
    the owning block runs the GEMM (fused with its neighbours)."""

    def __init__(self, fin, fout, bias=True):
        super().__init__()
        self.in_features, self.out_features = fin, fout
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.empty(fout)) if bias else None
        a = 1.0 / math.sqrt(fin)
        with torch.no_grad():
            self.weight.uniform_(-a, a)
            if self.bias is not None:
                self.bias.uniform_(-a, a)


class LayerNorm(nn.Module):
    """nn.LayerNorm(d) (eps 1e-5, affine) on the native kernel; keys weight/bias."""

    def __init__(self, normalized_shape, eps=1e-5):
        super().__init__()
        self.d = int(normalized_shape)
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(self.d))
        self.bias = nn.Parameter(torch.zeros(self.d))

    def forward(self, x):
        from .functions import layernorm
        return layernorm(self, x)


class TrainablePositionalEncoding(nn.Module):
    """layers.py:61-73: buffer pe (1, seq_len, d), first half sin / second half cos of p / 10000**(i/d)
    (not trainable despite the name); forward returns pe[:, :x.size(1)]."""

    def __init__(self, seq_len, emb_dim):
        super().__init__()
        pos = torch.arange(0, seq_len).unsqueeze(1).float()
        ang = pos / (10000. ** (torch.arange(0, emb_dim).float() / emb_dim))
        half = emb_dim // 2
        pe = torch.cat([torch.sin(ang[:, :half]), torch.cos(ang[:, half:])], dim=1)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return self.pe[:, :x.size(1)]


class MHA(nn.Module):
    """layers.py:31-40 (+ MHAHead :6-28).  The h per-head q/k/v Linear(d, d/h) are stored FUSED as one
    [3d, d] matrix (rows: q heads | k heads | v heads, head-major) so the projection is a single N=3d MFMA
    GEMM; `cross=True` splits it into wq [d, d] and wkv [2d, d] (the decoder batches the K/V projections of
    all its layers into one GEMM over the encoder output).  state_dict keys stay
    `_heads.{i}._{v,q,k}.{weight,bias}` and `_out_linear.{weight,bias}`.
    forward(x, enc_x=None, attention_mask=None): attention_mask > 0 means masked; scale is emb_dim**-0.5."""

    def __init__(self, num_heads, emb_dim, dropout, cross=False):
        super().__init__()
        assert emb_dim % num_heads == 0
        self.num_heads, self.emb_dim, self.p, self.cross = num_heads, emb_dim, float(dropout), cross
        self._dropout = nn.Dropout(dropout)
        d = emb_dim
        a = 1.0 / math.sqrt(d)
        if cross:
            self.wq = nn.Parameter(torch.empty(d, d).uniform_(-a, a))
            self.bq = nn.Parameter(torch.empty(d).uniform_(-a, a))
            self.wkv = nn.Parameter(torch.empty(2 * d, d).uniform_(-a, a))
            self.bkv = nn.Parameter(torch.empty(2 * d).uniform_(-a, a))
        else:
            self.wqkv = nn.Parameter(torch.empty(3 * d, d).uniform_(-a, a))
            self.bqkv = nn.Parameter(torch.empty(3 * d).uniform_(-a, a))
        self._out_linear = _Lin(d, d)

    # fused row block of projection `w` ('q', 'k', 'v') for head i
    def _rows(self, w, i):
        d, dh = self.emb_dim, self.emb_dim // self.num_heads
        base = {"q": 0, "k": d, "v": 2 * d}[w]
        return slice(base + i * dh, base + (i + 1) * dh)

    def _fused(self):
        if self.cross:
            return torch.cat([self.wq, self.wkv], 0), torch.cat([self.bq, self.bkv], 0)
        return self.wqkv, self.bqkv

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        W, b = self._fused()
        for i in range(self.num_heads):
            for w in ("v", "q", "k"):
                r = self._rows(w, i)
                wt, bt = W[r], b[r]
                if not keep_vars:
                    wt, bt = wt.detach(), bt.detach()
                destination[f"{prefix}_heads.{i}._{w}.weight"] = wt.clone() if not keep_vars else wt
                destination[f"{prefix}_heads.{i}._{w}.bias"] = bt.clone() if not keep_vars else bt

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        d = self.emb_dim
        W = torch.empty(3 * d, d)
        b = torch.empty(3 * d)
        ok = True
        for i in range(self.num_heads):
            for w in ("v", "q", "k"):
                r = self._rows(w, i)
                for name, dst in (("weight", W), ("bias", b)):
                    key = f"{prefix}_heads.{i}._{w}.{name}"
                    if key not in state_dict:
                        missing_keys.append(key)
                        ok = False
                        continue
                    dst[r].copy_(state_dict[key].detach().reshape(dst[r].shape))
        if not ok:
            return
        with torch.no_grad():
            if self.cross:
                self.wq.copy_(W[:d])
                self.bq.copy_(b[:d])
                self.wkv.copy_(W[d:])
                self.bkv.copy_(b[d:])
            else:
                self.wqkv.copy_(W)
                self.bqkv.copy_(b)
        if strict:
            for key in state_dict:
                if key.startswith(prefix) and not key[len(prefix):].startswith(("_heads.", "_out_linear.")):
                    unexpected_keys.append(key)

    def forward(self, x, enc_x=None, attention_mask=None):
        from .functions import mha
        return mha(self, x, enc_x, attention_mask)


class FeedForward(nn.Module):
    """layers.py:43-58: squeeze (d->ff) -> ReLU -> dropout -> unsqueeze (ff->d); keys squeeze.*, unsqueeze.*"""

    def __init__(self, emb_dim, ff_dim, dropout):
        super().__init__()
        self.emb_dim, self.ff_dim, self.p = emb_dim, ff_dim, float(dropout)
        self.squeeze = _Lin(emb_dim, ff_dim)
        self.ReLU = nn.ReLU()
        self.dropout = nn.Dropout(dropout)
        self.unsqueeze = _Lin(ff_dim, emb_dim)

    def forward(self, x):
        from .functions import feed_forward
        return feed_forward(self, x)
