"""ORACLE — test infrastructure only.

A functional fp32 CPU restatement of the reference's second model family, `modules/Transformer/new/`
(`new/model.py:9-209`, `new/layers.py:6-80`, `new/masking.py:4-29`): post-LN encoder / decoder layers, full-width
attention heads (each head projects d -> d; MHA.out maps h*d -> d and MHA adds its input), the residual inside
FeedForward, length-based key-padding masks and the interleaved sin/cos positional table.  As shipped the variant
imports the main `layers` / `masking` modules and raises; the behaviour restated here is the one it
has with its own `new/layers.py` and `new/masking.py` (how `tests/golden/make_golden_new.py` runs it).

Used ONLY by `tests/` (parity of `asrx.new`) and never by the shipped package.  Pinned by
`tests/test_oracle_golden.py::test_oracle_new_*` against `tests/golden/new_model.npz`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class NewConfig:
    """Constructor arguments of `new/model.py:145-159` `Transformer` (the ones that shape the model)."""
    vocab_size: int = 50
    n_mels: int = 32              # = emb_dim (new/model.py:177)
    enc_seq_len: int = 1          # seconds-like unit: encoder length = ceil(enc_seq_len * sr / n_fft * 2) (:162)
    dec_seq_len: int = 8
    hidden_dim: int = 4           # the unused VGG front-end's width (:163-174)
    n_enc: int = 2
    n_dec: int = 2
    n_heads: int = 2
    ff_dim: int = 64
    dropout: float = 0.0
    sr: int = 16000
    n_fft: int = 1024
    pad_id: int = 4               # nn.Embedding padding_idx (:157,:107)
    eos_id: int = 2               # also the decoder's padding token (:117-118)
    bos_id: int = 1

    @property
    def enc_len(self):
        return math.ceil(self.enc_seq_len * self.sr / self.n_fft * 2)


def pe_interleaved(n: int, d: int) -> torch.Tensor:
    """`TrainablePositionalEncoding` of new/layers.py:67-80: pe[p, 2i] = sin(p w_i), pe[p, 2i+1] = cos(p w_i),
    w_i = exp(-2i ln(10000) / d)."""
    pe = torch.zeros(n, d)
    pos = torch.arange(0, n).unsqueeze(1).float()
    w = torch.exp(torch.arange(0, d, 2).float() * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(pos * w)
    pe[:, 1::2] = torch.cos(pos * w)
    return pe


def _lin(P, key, x):
    return F.linear(x, P[key + ".weight"], P.get(key + ".bias"))


def _ln(P, key, x):
    return F.layer_norm(x, (x.shape[-1],), P[key + ".weight"], P[key + ".bias"], 1e-5)


# Tests only (as oracle/ref_model.py): a callable (site, shape) -> keep mask replacing nn.Dropout's draws; site
# ("attn", head key), ("out", MHA key), ("ffn", FeedForward key) or ("emb", "decoder").  None = torch's dropout.
DROP_MASKS = None


def _drop(x, p, training, site=None):
    """nn.Dropout (new/layers.py:29,46,63; new/model.py:121): x * keep / (1 - p) in training mode."""
    if not (training and p > 0):
        return x
    if DROP_MASKS is not None:
        return x * DROP_MASKS(site, tuple(x.shape)).to(x.dtype) / (1.0 - p)
    return F.dropout(x, p, training)


def head(P, key, x, kv, mask, d, p, training):
    """new/layers.py:15-32: v, q, k projections d -> d; scale d^-0.5; masked_fill(mask > 0, -inf); softmax (NO
    nan_to_num); dropout; @ v."""
    v = _lin(P, key + ".v", kv)
    q = _lin(P, key + ".q", x)
    k = _lin(P, key + ".k", kv)
    s = q.bmm(k.transpose(1, 2)) * (d ** -0.5)
    if mask is not None:
        s = s.masked_fill(mask.gt(0), float("-inf"))
    a = _drop(torch.softmax(s, dim=-1), p, training, ("attn", key))
    return a.bmm(v)


def mha(P, key, x, kv, mask, cfg: NewConfig, training):
    """new/layers.py:44-46: heads concatenated in index order -> out (h*d -> d) -> dropout -> + x."""
    kv = x if kv is None else kv
    hs = torch.cat([head(P, f"{key}.heads.{i}", x, kv, mask, cfg.n_mels, cfg.dropout, training)
                    for i in range(cfg.n_heads)], dim=-1)
    return _drop(_lin(P, key + ".out", hs), cfg.dropout, training, ("out", key)) + x


def ffn(P, key, x, cfg: NewConfig, training):
    """new/layers.py:59-64: x + unsqueeze(dropout(relu(squeeze(x))))."""
    h = _drop(torch.relu(_lin(P, key + ".squeeze", x)), cfg.dropout, training, ("ffn", key))
    return x + _lin(P, key + ".unsqueeze", h)


def valid_rows(lens, T):
    """new/masking.py:4-11 with input_lengths: 1 for t < lens[b], else 0 — (B, T) float."""
    return (torch.arange(T).unsqueeze(0) < lens.reshape(-1, 1)).float()


def encoder(P, spectre, lens, cfg: NewConfig, training=False):
    """new/model.py:51-64: (B, C, F, T) -> (B, T, C*F); key-padding self-attention mask by length (expanded to the
    encoder's seq_len rows, :58 / masking.py:25-29); norm_in(lin_in(x)) + pe; post-LN layers with the rows past
    each length zeroed after every norm (:22-29)."""
    B, C, Fm, T = spectre.shape
    x = spectre.reshape(B, C * Fm, T).transpose(1, 2)
    npm = valid_rows(lens, T)
    mask = npm.lt(1).unsqueeze(1).expand(-1, cfg.enc_len, -1)
    x = _ln(P, "encoder.norm_in", _lin(P, "encoder.lin_in", x)) + pe_interleaved(cfg.enc_len, cfg.n_mels)[:T]
    for l in range(cfg.n_enc):
        k = f"encoder.layers.{l}"
        x = _ln(P, k + ".norm1", mha(P, k + ".attention", x, None, mask, cfg, training)) * npm.unsqueeze(-1)
        x = _ln(P, k + ".norm2", ffn(P, k + ".ff", x, cfg, training)) * npm.unsqueeze(-1)
    return x


def decoder_layer(P, k, x, amask, enc, emask, npm, cfg, training):
    """new/model.py:80-91."""
    x = _ln(P, k + ".norm1", mha(P, k + ".mask_attention", x, None, amask, cfg, training)) * npm
    x = _ln(P, k + ".norm2", mha(P, k + ".attention", x, enc, emask, cfg, training)) * npm
    x = _ln(P, k + ".norm3", ffn(P, k + ".ff", x, cfg, training)) * npm
    return x


def decoder(P, text, enc, enc_lens, cfg: NewConfig, training=False):
    """new/model.py:116-123: rows equal to the EOS id are padding (:117); self-attention mask = causal OR key ==
    EOS (:118, masking.py:14-22); cross-attention mask = encoder key past its length (:119); emb + pe -> dropout ->
    layers -> classifier (no bias, no final norm)."""
    B, L = text.shape
    npm = text.ne(cfg.eos_id).float().unsqueeze(-1)
    causal = torch.triu(torch.ones((L, L), dtype=torch.uint8), diagonal=1).unsqueeze(0).expand(B, -1, -1)
    amask = (causal + text.eq(cfg.eos_id).unsqueeze(1).expand(-1, L, -1)).gt(0)
    emask = valid_rows(enc_lens, enc.shape[1]).lt(1).unsqueeze(1).expand(-1, cfg.dec_seq_len, -1)
    x = F.embedding(text, P["decoder.emb.weight"], padding_idx=cfg.pad_id) + pe_interleaved(cfg.dec_seq_len, cfg.n_mels)[:L]
    x = _drop(x, cfg.dropout, training, ("emb", "decoder"))
    for l in range(cfg.n_dec):
        x = decoder_layer(P, f"decoder.layers.{l}", x, amask, enc, emask, npm, cfg, training)
    return F.linear(x, P["decoder.classifier.weight"])


def forward(P, spectre, lens, text, cfg: NewConfig, training=False):
    """new/model.py:200-204 (batch dict: spectre, spectrogram_len, encoded_text)."""
    return decoder(P, text, encoder(P, spectre, lens, cfg, training), lens, cfg, training)


def evaluate(P, spectre, lens, cfg: NewConfig):
    """new/model.py:206-209 -> Decoder.evaluate (:125-142): batched greedy decode from BOS for seq_len steps,
    causal mask only, no cross mask, no row mask; returns (tokens (B, seq_len + 1) int32, last logits (B, seq_len,
    V), eoses: the last step at which each row predicted EOS, seq_len - 1 if never)."""
    enc = encoder(P, spectre, lens, cfg, False)
    B = enc.shape[0]
    dec_in = torch.full((B, 1), cfg.bos_id, dtype=torch.int32)
    eoses = torch.full((B,), cfg.dec_seq_len - 1)
    pe = pe_interleaved(cfg.dec_seq_len, cfg.n_mels)
    prob = None
    for i in range(cfg.dec_seq_len):
        L = dec_in.shape[1]
        ones = torch.ones(B, L, 1)
        causal = torch.triu(torch.ones((L, L), dtype=torch.uint8), diagonal=1).unsqueeze(0).expand(B, -1, -1)
        prob = F.embedding(dec_in.long(), P["decoder.emb.weight"], padding_idx=cfg.pad_id) + pe[:L]
        for l in range(cfg.n_dec):
            prob = decoder_layer(P, f"decoder.layers.{l}", prob, causal, enc, None, ones, cfg, False)
        prob = F.linear(prob, P["decoder.classifier.weight"])
        nxt = prob[:, -1].argmax(dim=-1)
        for j in range(B):
            if nxt[j] == cfg.eos_id:
                eoses[j] = i
        dec_in = torch.cat([dec_in, nxt.unsqueeze(-1).to(dec_in.dtype)], dim=1)
    return dec_in, prob, eoses


def param_shapes(cfg: NewConfig) -> dict:
    """The reference state_dict schema of new/model.py (buffers `*.pe.pe` excluded)."""
    d, ff, V, hd = cfg.n_mels, cfg.ff_dim, cfg.vocab_size, cfg.hidden_dim
    s = {"vgg.0.weight": (hd, 1, 3, 3), "vgg.0.bias": (hd,), "vgg.2.weight": (hd, hd, 3, 3), "vgg.2.bias": (hd,),
         "vgg.5.weight": (2 * hd, hd, 3, 3), "vgg.5.bias": (2 * hd,), "vgg.7.weight": (2 * hd, 2 * hd, 3, 3),
         "vgg.7.bias": (2 * hd,),
         "encoder.lin_in.weight": (d, d), "encoder.lin_in.bias": (d,),
         "encoder.norm_in.weight": (d,), "encoder.norm_in.bias": (d,)}

    def mha_(key):
        for i in range(cfg.n_heads):
            for w in ("v", "q", "k"):
                s[f"{key}.heads.{i}.{w}.weight"] = (d, d)
                s[f"{key}.heads.{i}.{w}.bias"] = (d,)
        s[f"{key}.out.weight"] = (d, d * cfg.n_heads)
        s[f"{key}.out.bias"] = (d,)

    def ffn_(key):
        s[key + ".squeeze.weight"] = (ff, d); s[key + ".squeeze.bias"] = (ff,)
        s[key + ".unsqueeze.weight"] = (d, ff); s[key + ".unsqueeze.bias"] = (d,)

    def ln_(key):
        s[key + ".weight"] = (d,); s[key + ".bias"] = (d,)

    for l in range(cfg.n_enc):
        k = f"encoder.layers.{l}"
        mha_(k + ".attention"); ln_(k + ".norm1"); ffn_(k + ".ff"); ln_(k + ".norm2")
    s["decoder.emb.weight"] = (V, d)
    for l in range(cfg.n_dec):
        k = f"decoder.layers.{l}"
        mha_(k + ".mask_attention"); ln_(k + ".norm1"); mha_(k + ".attention"); ln_(k + ".norm2")
        ffn_(k + ".ff"); ln_(k + ".norm3")
    s["decoder.classifier.weight"] = (V, d)
    return s


def det_params(cfg: NewConfig, seed: int = 0) -> dict:
    """Deterministic fp32 weights keyed by (seed, state_dict key) — the rule of oracle.ref_model.det_params
    (U(-1/sqrt(fan_in), 1/sqrt(fan_in)), LayerNorm gains 1 + 0.1 U(-1, 1), embedding N(0, 1) with the padding row
    zeroed)."""
    from oracle.ref_model import _key_seed
    out = {}
    for key, shape in param_shapes(cfg).items():
        g = torch.Generator().manual_seed(_key_seed(seed, "new:" + key))
        if key == "decoder.emb.weight":
            t = torch.randn(shape, generator=g)
            t[cfg.pad_id] = 0
        elif ".norm" in key and key.endswith(".weight"):
            t = 1.0 + 0.1 * (2 * torch.rand(shape, generator=g) - 1)
        else:
            fan_in = (shape[1] * (9 if len(shape) == 4 else 1)) if len(shape) > 1 else cfg.n_mels
            a = 1.0 / math.sqrt(fan_in)
            t = (2 * torch.rand(shape, generator=g) - 1) * a
        out[key] = t.float()
    return out


def synthetic_batch(cfg: NewConfig, batch: int, seed: int = 1234):
    """A `new/` batch dict: spectre (B, 1, n_mels, enc_len) ~ N(0, 1), lengths ~ U[enc_len/2, enc_len] (the first
    row full length), encoded_text = BOS, tokens ~ U[5, V), EOS, then EOS padding (the decoder's padding token),
    length dec_seq_len."""
    g = torch.Generator().manual_seed(seed)
    T, L = cfg.enc_len, cfg.dec_seq_len
    spectre = torch.randn((batch, 1, cfg.n_mels, T), generator=g)
    lens = torch.randint(T // 2, T + 1, (batch,), generator=g)
    lens[0] = T
    text = torch.full((batch, L), cfg.eos_id, dtype=torch.long)
    for b in range(batch):
        n = int(torch.randint(max(2, L // 2), L + 1, (1,), generator=g))
        text[b, 0] = cfg.bos_id
        if n > 2:
            text[b, 1:n - 1] = torch.randint(5, cfg.vocab_size, (n - 2,), generator=g)
    return spectre, lens, text


NEW_CONFIGS = {
    "new_micro": NewConfig(),
    # d_model 80 (n_mels) x 4 full-width heads over 2 s of frames (63 encoder positions), as the variant's own
    # training script sizes it (new/train.py feeds 80-bin mel spectrograms)
    "new_small": NewConfig(vocab_size=250, n_mels=80, enc_seq_len=2, dec_seq_len=16, hidden_dim=8, n_enc=2, n_dec=2,
                           n_heads=4, ff_dim=256),
}
