"""Drop-in replacements for modules/Transformer/new/layers.py (MHAHead/MHA with full-width heads, FeedForward with
its residual, the interleaved TrainablePositionalEncoding): same constructor arguments, forward signatures and
state_dict keys; compute goes to libasrx.so (asrx.new.ops).

MHA stores the h heads' q / k / v Linear(d, d) FUSED — one [3 h d, d] matrix for self-attention (rows q heads |
k heads | v heads), wq [h d, d] + wkv [2 h d, d] for cross-attention use — and the state_dict hooks translate to and
from the reference's `heads.{i}.{v,q,k}.{weight,bias}` keys, so reference checkpoints load verbatim.
"""
import math

import torch
from torch import nn

from ..layers import _Lin


class TrainablePositionalEncoding(nn.Module):
    """new/layers.py:67-80: buffer pe (1, seq_len, d) with pe[p, 2i] = sin(p w_i), pe[p, 2i+1] = cos(p w_i),
    w_i = exp(-2i ln(10000) / d); forward returns pe[:, :x.size(1)]."""

    def __init__(self, seq_len, emb_dim):
        super().__init__()
        pe = torch.zeros(seq_len, emb_dim)
        pos = torch.arange(0, seq_len).unsqueeze(1).float()
        w = torch.exp(torch.arange(0, emb_dim, 2).float() * -(math.log(10000.0) / emb_dim))
        pe[:, 0::2] = torch.sin(pos * w)
        pe[:, 1::2] = torch.cos(pos * w)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return self.pe[:, :x.size(1)]


class MHA(nn.Module):
    """new/layers.py:35-46 (+ MHAHead :6-32): h heads each projecting d -> d, concatenated in head order, out (h d ->
    d), dropout, + x.  forward(x, enc_x=None, attention_mask=None) with attention_mask > 0 = masked (any
    shape broadcastable to (B, Lq, Lk)); the model passes its masks in the structured form (asrx.new.model)."""

    def __init__(self, num_heads, emb_dim, dropout):
        super().__init__()
        self.num_heads, self.emb_dim, self.p = num_heads, emb_dim, float(dropout)
        self.dropout = nn.Dropout(dropout)
        d, hd = emb_dim, num_heads * emb_dim
        a = 1.0 / math.sqrt(d)
        self.wqkv = nn.Parameter(torch.empty(3 * hd, d).uniform_(-a, a))
        self.bqkv = nn.Parameter(torch.empty(3 * hd).uniform_(-a, a))
        self.out = _Lin(hd, d)

    def _rows(self, w, i):
        d, hd = self.emb_dim, self.num_heads * self.emb_dim
        base = {"q": 0, "k": hd, "v": 2 * hd}[w]
        return slice(base + i * d, base + (i + 1) * d)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        for i in range(self.num_heads):
            for w in ("v", "q", "k"):
                r = self._rows(w, i)
                wt, bt = self.wqkv[r], self.bqkv[r]
                destination[f"{prefix}heads.{i}.{w}.weight"] = wt if keep_vars else wt.detach().clone()
                destination[f"{prefix}heads.{i}.{w}.bias"] = bt if keep_vars else bt.detach().clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        W, b = torch.empty_like(self.wqkv, device="cpu"), torch.empty_like(self.bqkv, device="cpu")
        ok = True
        for i in range(self.num_heads):
            for w in ("v", "q", "k"):
                r = self._rows(w, i)
                for name, dst in (("weight", W), ("bias", b)):
                    key = f"{prefix}heads.{i}.{w}.{name}"
                    if key not in state_dict:
                        missing_keys.append(key)
                        ok = False
                        continue
                    dst[r].copy_(state_dict[key].detach().reshape(dst[r].shape))
        if ok:
            with torch.no_grad():
                self.wqkv.copy_(W)
                self.bqkv.copy_(b)
        if strict:
            for key in state_dict:
                if key.startswith(prefix) and not key[len(prefix):].startswith(("heads.", "out.")):
                    unexpected_keys.append(key)

    def forward(self, x, enc_x=None, attention_mask=None):
        from .model import mha_forward
        return mha_forward(self, x, enc_x, attention_mask)


class FeedForward(nn.Module):
    """new/layers.py:49-64: x + unsqueeze(dropout(relu(squeeze(x)))); keys squeeze.*, unsqueeze.*"""

    def __init__(self, emb_dim, ff_dim, dropout):
        super().__init__()
        self.emb_dim, self.ff_dim, self.p = emb_dim, ff_dim, float(dropout)
        self.squeeze = _Lin(emb_dim, ff_dim)
        self.ReLU = nn.ReLU()
        self.dropout = nn.Dropout(dropout)
        self.unsqueeze = _Lin(ff_dim, emb_dim)

    def forward(self, x):
        from .model import ffn_forward
        return ffn_forward(self, x)
