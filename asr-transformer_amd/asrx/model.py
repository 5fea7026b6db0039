"""Drop-in replacements for modules/Transformer/model.py: EncoderLayer, Encoder, DecoderLayer, Decoder,
Transformer — same constructor signatures (model.py:9-16, 28-39, 55-63, 78-102, 154-191), same forward /
evaluate signatures, same state_dict keys.  Whole stacks run as explicit native kernel programs
(asrx.blocks) behind one autograd node each; parameters live in one flat buffer (asrx.params).

Extra keyword-only knobs (not in the reference): precision ("bf16" training path | "fp32" parity path),
attention ("fused" LDS-tiled kernel | "unfused" materialised scores + row softmax).
"""
import math
import weakref

import torch
from torch import nn

from .layers import MHA, FeedForward, LayerNorm, TrainablePositionalEncoding, _Lin


def _adopt(root):
    """Point every submodule at `root`, whose flat parameter store they share (weakref: no module cycle)."""
    for m in root.modules():
        if m is not root:
            m.__dict__["_asrx_root"] = weakref.ref(root)


def subsampled(n):
    """model.py:172 / the conv arithmetic of model.py:168-171."""
    return ((n - 3) // 2 + 1 - 3) // 2 + 1


class _LinIn(_Lin):
    """Encoder._lin_in (model.py:32).  Stored with its input columns permuted from the reference's channel-major
    feature order (c*F''+f, model.py:43-45) to (f*64+c): the conv2 GEMM then writes the encoder input directly
    and the reference's transpose+contiguous copy disappears.  state_dict hooks un/permute."""

    def __init__(self, fin, fout, n_freq):
        super().__init__(fin, fout)
        self.n_freq = n_freq      # F''
        self.n_ch = fin // n_freq  # 64

    def _to_ref(self, w):          # phys (d, F*64 + c) -> ref (d, c*F + f)
        d = w.shape[0]
        return w.reshape(d, self.n_freq, self.n_ch).permute(0, 2, 1).reshape(d, -1)

    def _from_ref(self, w):
        d = w.shape[0]
        return w.reshape(d, self.n_ch, self.n_freq).permute(0, 2, 1).reshape(d, -1)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight if keep_vars else self.weight.detach()
        destination[prefix + "weight"] = self._to_ref(w).contiguous()
        destination[prefix + "bias"] = self.bias if keep_vars else self.bias.detach()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        sd = dict(state_dict)
        if prefix + "weight" in sd:
            sd[prefix + "weight"] = self._from_ref(sd[prefix + "weight"])
        super()._load_from_state_dict(sd, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs)


class _Classifier(nn.Module):
    """Decoder._classifier = Linear(d, V, bias=False) (model.py:102).  Rows padded to a multiple of 64 (V=250
    -> 256) so the logits/dlogits rows are 16-byte aligned GEMM operands; padding rows stay zero."""

    def __init__(self, d, V):
        super().__init__()
        self.V = V
        self.Vp = (V + 63) // 64 * 64
        a = 1.0 / math.sqrt(d)
        w = torch.zeros(self.Vp, d)
        w[:V].uniform_(-a, a)
        self.weight = nn.Parameter(w)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight if keep_vars else self.weight.detach()
        destination[prefix + "weight"] = w[:self.V] if keep_vars else w[:self.V].clone()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        key = prefix + "weight"
        if key not in state_dict:
            missing_keys.append(key)
            return
        with torch.no_grad():
            self.weight.zero_()
            self.weight[:self.V].copy_(state_dict[key])


class _Embedding(nn.Module):
    """nn.Embedding(V, d, padding_idx) container (model.py:94): key `weight`; the padding row is zero at init
    and never receives gradient."""

    def __init__(self, V, d, padding_idx):
        super().__init__()
        self.padding_idx = padding_idx
        w = torch.randn(V, d)
        if padding_idx is not None:
            w[padding_idx] = 0
        self.weight = nn.Parameter(w)


class FrontEnd(nn.Sequential):
    """Transformer.input_layer (model.py:168-171) with the reference's child indices (0: conv, 1: relu,
    2: conv, 3: relu).  conv2's weight is kept channels-last (cout, kh, kw, cin) in memory, which is the
    [64][576] operand of the im2col GEMM.  forward returns the reference's logical (B, 64, F'', T'') tensor as
    a permuted view of the (B, T'', F'', 64) buffer the encoder consumes."""

    def __init__(self):
        super().__init__(nn.Conv2d(1, 64, 3, stride=2), nn.ReLU(), nn.Conv2d(64, 64, 3, stride=2), nn.ReLU())
        self[2].weight._asrx_phys = ((64, 3, 3, 64), (0, 3, 1, 2))
        with torch.no_grad():
            self[2].weight.data = self[2].weight.data.contiguous(memory_format=torch.channels_last)

    def forward(self, spectrum):
        from .functions import frontend
        return frontend(self, spectrum)


class EncoderLayer(nn.Module):
    """model.py:9-25"""

    def __init__(self, emb_dim, num_heads, ff_dim, dropout):
        super().__init__()
        self.num_heads, self.p = num_heads, float(dropout)
        self._norm_in = LayerNorm(emb_dim)          # unused by the reference forward (model.py:12)
        self._attention = MHA(num_heads, emb_dim, dropout)
        self._norm1 = LayerNorm(emb_dim)
        self._feedforward = FeedForward(emb_dim, ff_dim, dropout)
        self._norm2 = LayerNorm(emb_dim)
        _adopt(self)

    def forward(self, x):
        from .functions import encoder_layer
        return encoder_layer(self, x)


class Encoder(nn.Module):
    """model.py:28-52"""

    def __init__(self, seq_len, emb_dim, input_dim, num_layers, num_heads, ff_dim, dropout=0.1, n_freq=None):
        super().__init__()
        self.emb_dim, self.num_heads, self.p = emb_dim, num_heads, float(dropout)
        n_freq = n_freq if n_freq is not None else input_dim // 64
        self._lin_in = _LinIn(input_dim, emb_dim, n_freq)
        self._norm_out = LayerNorm(emb_dim)
        self._pe = TrainablePositionalEncoding(seq_len, emb_dim)
        self._layers = nn.ModuleList([EncoderLayer(emb_dim, num_heads, ff_dim, dropout) for _ in range(num_layers)])
        _adopt(self)

    def forward(self, x):
        from .functions import encoder
        return encoder(self, x)


class DecoderLayer(nn.Module):
    """model.py:55-75"""

    def __init__(self, emb_dim, num_heads, ff_dim, dropout):
        super().__init__()
        self.num_heads, self.p = num_heads, float(dropout)
        self._mask_attention = MHA(num_heads, emb_dim, dropout)
        self._norm1 = LayerNorm(emb_dim)
        self._cross_attention = MHA(num_heads, emb_dim, dropout, cross=True)
        self._norm2 = LayerNorm(emb_dim)
        self._feedforward = FeedForward(emb_dim, ff_dim, dropout)
        self._norm3 = LayerNorm(emb_dim)
        _adopt(self)

    def forward(self, x, mask, enc_x):
        from .functions import decoder_layer
        return decoder_layer(self, x, mask, enc_x)


class Decoder(nn.Module):
    """model.py:78-151"""

    def __init__(self, vocab_size, seq_len, emb_dim, num_layers, num_heads, ff_dim, eos_token_id, dropout=0.1,
                 pad_token_id=0):
        super().__init__()
        self._seq_len = seq_len
        self._eos_token_id = eos_token_id
        self.pad_token_id = pad_token_id
        self.vocab_size, self.emb_dim, self.num_heads, self.p = vocab_size, emb_dim, num_heads, float(dropout)
        self._embedding = _Embedding(vocab_size, emb_dim, pad_token_id)
        self._pe = TrainablePositionalEncoding(seq_len, emb_dim)
        self._dropout = nn.Dropout(dropout)
        self._layers = nn.ModuleList([DecoderLayer(emb_dim, num_heads, ff_dim, dropout) for _ in range(num_layers)])
        self._norm_layer = LayerNorm(emb_dim)
        self._classifier = _Classifier(emb_dim, vocab_size)
        _adopt(self)

    def forward(self, x, mask, enc_x):
        from .functions import decoder
        return decoder(self, x, mask, enc_x)

    def evaluate(self, x, enc_x):
        from .functions import decoder_evaluate
        return decoder_evaluate(self, x, enc_x)


class Transformer(nn.Module):
    """model.py:154-206.  forward(spectrum (B,1,F,T), text (B,L) int, mask (B,L)) -> logits (B,L,V)."""

    def __init__(self, vocab_size, input_dim, embedding_dim, decoder_seq_len, encoder_seq_len, encoder_num_layers,
                 decoder_num_layers, num_heads, ff_dim, dropout=0.1, pad_token_id=4, eos_token_id=2, *,
                 precision="bf16", attention="fused"):
        super().__init__()
        self.input_layer = FrontEnd()
        n_freq = subsampled(input_dim)
        fdim = n_freq * 64
        self.input_encoding = _Lin(fdim, embedding_dim)   # built but unused by the reference (model.py:173)
        self.encoder = Encoder(seq_len=encoder_seq_len, input_dim=fdim, emb_dim=embedding_dim,
                               num_layers=encoder_num_layers, num_heads=num_heads, ff_dim=ff_dim, dropout=dropout,
                               n_freq=n_freq)
        self.decoder = Decoder(vocab_size=vocab_size, seq_len=decoder_seq_len, emb_dim=embedding_dim,
                               num_layers=decoder_num_layers, num_heads=num_heads, ff_dim=ff_dim,
                               eos_token_id=eos_token_id, dropout=dropout, pad_token_id=pad_token_id)
        self.precision = precision
        self.attention = attention
        _adopt(self)

    def forward(self, spectrum, text, mask):
        from .functions import transformer
        return transformer(self, spectrum, text, mask)

    def evaluate(self, spectrum, text):
        from .functions import transformer_evaluate
        return transformer_evaluate(self, spectrum, text)
