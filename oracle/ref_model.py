"""ORACLE — test infrastructure only.

A functional fp32 CPU restatement of the reference Speech-Transformer forward path
(`/root/reference/modules/Transformer/model.py` + `layers.py`).  It is used ONLY as:
  * the checker in `tests/` (parity of the HIP path),
  * the checker in `__graft_entry__.smoke()`,
  * the `cpu_baseline` leg of `bench.py` (timed on the host cores, kind="port").
Nothing in the shipped path (`asr-transformer_amd/asrx`) imports it.

Parity pinning: the restatement is checked against golden vectors produced by importing the
reference itself in the build container (`tests/golden/make_golden.py`,
`tests/test_oracle_golden.py`).

The restatement is written op-for-op in the reference's structure (per-head Linear loop, 1/sqrt(d_model)
scale, masked_fill(-inf) -> softmax -> nan_to_num) so that its CPU timing represents the reference,
but it is a set of functions over a flat ``{state_dict key: tensor}`` mapping rather than nn.Modules.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class OracleConfig:
    """Constructor arguments of the reference `Transformer` (model.py:155-166)."""
    vocab_size: int = 250
    input_dim: int = 80          # mel bins before the conv front-end
    d_model: int = 128
    dec_len: int = 16            # decoder_seq_len (PE table length, greedy-decode steps)
    enc_len: int = 100           # encoder_seq_len (PE table length, must be >= T')
    n_enc: int = 2
    n_dec: int = 2
    n_heads: int = 4
    ff_dim: int = 512
    dropout: float = 0.1
    pad_id: int = 4
    eos_id: int = 2


def subsampled(n: int) -> int:
    """Length after two unpadded 3x3 stride-2 convs (model.py:168-172)."""
    return ((n - 3) // 2 + 1 - 3) // 2 + 1


def pe_table(n_pos: int, d: int) -> torch.Tensor:
    """Sinusoid table of `TrainablePositionalEncoding` (layers.py:61-70).

    angle[p, i] = p / 10000**(i/d); first half of the features uses sin, second half cos
    (NOT the interleaved textbook layout)."""
    pos = torch.arange(0, n_pos).unsqueeze(1).float()
    angle = pos / (10000. ** (torch.arange(0, d).float() / d))
    tab = torch.zeros(n_pos, d)
    half = d // 2
    tab[:, :half] = torch.sin(angle[:, :half])
    tab[:, half:] = torch.cos(angle[:, half:])
    return tab


def _lin(P, key, x):
    b = P.get(key + ".bias")
    return F.linear(x, P[key + ".weight"], b)


def _ln(P, key, x):
    """nn.LayerNorm(d), eps 1e-5 (model.py:14,16,33,59,61,63,101)."""
    return F.layer_norm(x, (x.shape[-1],), P[key + ".weight"], P[key + ".bias"], 1e-5)


# Tests only: a callable (site, shape) -> keep mask (bool, broadcastable to shape) that replaces torch's dropout
# draws, so a training-mode forward / backward can be compared with the HIP path's own masks (the counter hash of
# csrc/common.h, restated in tests/rng_ref.py).  site: ("attn", head key) for the attention probabilities,
# ("out", MHA key) for the MHA output, ("ffn", FeedForward key) for the hidden layer, ("emb", "decoder") for the
# decoder input.  None = nn.Dropout's own masks (the reference).
DROP_MASKS = None


def _drop(x, p, training, site=None):
    """nn.Dropout (layers.py:27,40,56; model.py:117): x * keep / (1 - p) in training mode."""
    if not (training and p > 0):
        return x
    if DROP_MASKS is not None:
        return x * DROP_MASKS(site, tuple(x.shape)).to(x.dtype) / (1.0 - p)
    return F.dropout(x, p, training)


def attention_head(P, key, x, kv, mask, d_model, p, training):
    """One `MHAHead` (layers.py:15-28): q from x, k/v from kv; scale d_model**-0.5 (NOT d_head);
    masked_fill(mask>0, -inf) -> softmax -> nan_to_num (all-masked rows become 0) -> dropout -> @ v."""
    v = _lin(P, key + "._v", kv)
    k = _lin(P, key + "._k", kv)
    q = _lin(P, key + "._q", x)
    s = torch.bmm(q, k.transpose(1, 2)) * (d_model ** -0.5)
    if mask is not None:
        s = s.masked_fill(mask.gt(0), float("-inf"))
    a = torch.nan_to_num(torch.softmax(s, dim=-1))
    a = _drop(a, p, training, ("attn", key))
    return torch.bmm(a, v)


def multi_head(P, key, x, kv, mask, cfg: OracleConfig, training):
    """`MHA.forward` (layers.py:38-40): heads concatenated in index order -> _out_linear -> dropout."""
    kv = x if kv is None else kv
    outs = [attention_head(P, f"{key}._heads.{i}", x, kv, mask, cfg.d_model, cfg.dropout, training)
            for i in range(cfg.n_heads)]
    y = _lin(P, key + "._out_linear", torch.cat(outs, dim=-1))
    return _drop(y, cfg.dropout, training, ("out", key))


def feed_forward(P, key, x, cfg: OracleConfig, training):
    """`FeedForward.forward` (layers.py:53-58): squeeze -> ReLU -> dropout -> unsqueeze."""
    h = torch.relu(_lin(P, key + ".squeeze", x))
    h = _drop(h, cfg.dropout, training, ("ffn", key))
    return _lin(P, key + ".unsqueeze", h)


def front_end(P, spectrum):
    """`Transformer.input_layer` (model.py:168-171) + the encoder's flatten (model.py:43-45):
    (B,1,F,T) -> conv s2 -> relu -> conv s2 -> relu -> (B, T', 64*F'') with feature = c*F''+f."""
    y = torch.relu(F.conv2d(spectrum, P["input_layer.0.weight"], P["input_layer.0.bias"], stride=2))
    y = torch.relu(F.conv2d(y, P["input_layer.2.weight"], P["input_layer.2.bias"], stride=2))
    b, c, f, t = y.shape
    return y.reshape(b, c * f, t).transpose(1, 2).contiguous()


def encoder(P, feats, cfg: OracleConfig, training=False):
    """`Encoder.forward` (model.py:41-52): _lin_in + PE, pre-LN layers with NO attention mask, _norm_out."""
    pe = pe_table(cfg.enc_len, cfg.d_model)
    x = _lin(P, "encoder._lin_in", feats) + pe[: feats.shape[1]].unsqueeze(0)
    for l in range(cfg.n_enc):
        key = f"encoder._layers.{l}"
        x = multi_head(P, key + "._attention", _ln(P, key + "._norm1", x), None, None, cfg, training) + x
        x = feed_forward(P, key + "._feedforward", _ln(P, key + "._norm2", x), cfg, training) + x
    return _ln(P, "encoder._norm_out", x)


def decoder_mask(mask):
    """Decoder self-attention mask (model.py:108-115): key-pad OR query-pad OR causal; True = masked."""
    bsz, n = mask.shape
    pad = mask.lt(1).unsqueeze(1).expand(-1, n, -1)
    causal = torch.triu(torch.ones((n, n), dtype=torch.uint8), diagonal=1).unsqueeze(0).expand(bsz, -1, -1)
    return torch.logical_or(torch.logical_or(pad, pad.mT), causal)


def decoder_layer(P, key, x, self_mask, enc, cfg: OracleConfig, training):
    """`DecoderLayer.forward` (model.py:65-75): masked self-attn, cross-attn (no mask), FFN; all pre-LN."""
    x = multi_head(P, key + "._mask_attention", _ln(P, key + "._norm1", x), None, self_mask, cfg, training) + x
    x = multi_head(P, key + "._cross_attention", _ln(P, key + "._norm2", x), enc, None, cfg, training) + x
    x = feed_forward(P, key + "._feedforward", _ln(P, key + "._norm3", x), cfg, training) + x
    return x


def decoder(P, text, mask, enc, cfg: OracleConfig, training=False):
    """`Decoder.forward` (model.py:104-123): emb + PE -> dropout -> layers -> _norm_layer -> classifier (no bias)."""
    pe = pe_table(cfg.dec_len, cfg.d_model)
    m = decoder_mask(mask)
    x = F.embedding(text, P["decoder._embedding.weight"], padding_idx=cfg.pad_id) + pe[: text.shape[1]].unsqueeze(0)
    x = _drop(x, cfg.dropout, training, ("emb", "decoder"))
    for l in range(cfg.n_dec):
        x = decoder_layer(P, f"decoder._layers.{l}", x, m, enc, cfg, training)
    x = _ln(P, "decoder._norm_layer", x)
    return F.linear(x, P["decoder._classifier.weight"])


def forward(P, spectrum, text, mask, cfg: OracleConfig, training=False, return_encoder=False):
    """`Transformer.forward` (model.py:194-198)."""
    enc = encoder(P, front_end(P, spectrum), cfg, training)
    logits = decoder(P, text, mask, enc, cfg, training)
    return (logits, enc) if return_encoder else logits


def greedy_decode(P, spectrum, text, cfg: OracleConfig):
    """`Transformer.evaluate` -> `Decoder.evaluate` (model.py:125-151, 201-206), quirks included:
    per-sample loop, full prefix recomputed every step, uint8 causal mask, NO final LayerNorm before the
    classifier, no break on EOS, returns the LAST sample's token row and the list of logits snapshots."""
    enc = encoder(P, front_end(P, spectrum), cfg, False)
    pe = pe_table(cfg.dec_len, cfg.d_model)
    probs = []
    row = None
    for s in range(text.shape[0]):
        row = text[s].unsqueeze(0)
        e = enc[s].unsqueeze(0)
        for i in range(1, cfg.dec_len + 1):
            causal = torch.triu(torch.ones((i, i), dtype=torch.uint8), diagonal=1)
            h = F.embedding(row, P["decoder._embedding.weight"], padding_idx=cfg.pad_id) + pe[: row.shape[1]].unsqueeze(0)
            for l in range(cfg.n_dec):
                h = decoder_layer(P, f"decoder._layers.{l}", h, causal, e, cfg, False)
            logit = F.linear(h, P["decoder._classifier.weight"])
            nxt = logit.argmax(dim=-1)[:, -1].unsqueeze(1)
            row = torch.cat([row, nxt.to(row.dtype)], dim=-1)
            if nxt.item() == cfg.eos_id or i == cfg.dec_len:
                probs.append(logit[:, :-1].squeeze())
    return row, probs


def train_step_grads(P, spectrum, text, mask, cfg: OracleConfig, training=False):
    """Loss and gradients of one teacher-forced step as the build defines it (train.py:22-34 without the
    batch-coupled index_put quirk): inputs text[:, :-1], targets text[:, 1:], mean cross-entropy.
    P values must be leaf tensors with requires_grad."""
    logits = forward(P, spectrum, text[:, :-1], mask[:, :-1], cfg, training)
    loss = F.cross_entropy(logits.transpose(1, 2), text[:, 1:])
    loss.backward()
    return loss.detach(), {k: (v.grad.detach().clone() if v.grad is not None else None) for k, v in P.items()}


# ---------------------------------------------------------------------------------------------
# Deterministic parameters and inputs shared by the fixture generator, the tests and the bench.
# ---------------------------------------------------------------------------------------------

def param_shapes(cfg: OracleConfig) -> dict:
    """The reference state_dict schema; buffers (`_pe.pe`) excluded."""
    d, ff, V = cfg.d_model, cfg.ff_dim, cfg.vocab_size
    dh = d // cfg.n_heads
    fdim = subsampled(cfg.input_dim) * 64
    s = {
        "input_layer.0.weight": (64, 1, 3, 3), "input_layer.0.bias": (64,),
        "input_layer.2.weight": (64, 64, 3, 3), "input_layer.2.bias": (64,),
        "input_encoding.weight": (d, fdim), "input_encoding.bias": (d,),
        "encoder._lin_in.weight": (d, fdim), "encoder._lin_in.bias": (d,),
        "encoder._norm_out.weight": (d,), "encoder._norm_out.bias": (d,),
    }

    def mha(key):
        for i in range(cfg.n_heads):
            for w in ("_v", "_q", "_k"):
                s[f"{key}._heads.{i}.{w}.weight"] = (dh, d)
                s[f"{key}._heads.{i}.{w}.bias"] = (dh,)
        s[f"{key}._out_linear.weight"] = (d, d)
        s[f"{key}._out_linear.bias"] = (d,)

    def ffn(key):
        s[f"{key}.squeeze.weight"] = (ff, d); s[f"{key}.squeeze.bias"] = (ff,)
        s[f"{key}.unsqueeze.weight"] = (d, ff); s[f"{key}.unsqueeze.bias"] = (d,)

    def ln(key):
        s[key + ".weight"] = (d,); s[key + ".bias"] = (d,)

    for l in range(cfg.n_enc):
        k = f"encoder._layers.{l}"
        ln(k + "._norm_in"); mha(k + "._attention"); ln(k + "._norm1"); ffn(k + "._feedforward"); ln(k + "._norm2")
    s["decoder._embedding.weight"] = (V, d)
    for l in range(cfg.n_dec):
        k = f"decoder._layers.{l}"
        mha(k + "._mask_attention"); ln(k + "._norm1"); mha(k + "._cross_attention"); ln(k + "._norm2")
        ffn(k + "._feedforward"); ln(k + "._norm3")
    ln("decoder._norm_layer")
    s["decoder._classifier.weight"] = (V, d)
    return s


def _key_seed(seed: int, key: str) -> int:
    h = 2166136261
    for ch in key.encode():
        h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
    return (seed * 1000003 + h) & 0x7FFFFFFFFFFF


def det_params(cfg: OracleConfig, seed: int = 0) -> dict:
    """Deterministic fp32 weights keyed by (seed, state_dict key): U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for
    weights/biases, 1 + 0.1*U(-1,1) for LayerNorm gains, N(0,1) for the embedding (row pad_id zeroed as
    nn.Embedding(padding_idx) does at init, model.py:94)."""
    out = {}
    for key, shape in param_shapes(cfg).items():
        g = torch.Generator().manual_seed(_key_seed(seed, key))
        if key == "decoder._embedding.weight":
            t = torch.randn(shape, generator=g)
            t[cfg.pad_id] = 0
        elif ("_norm" in key) and key.endswith(".weight"):
            t = 1.0 + 0.1 * (2 * torch.rand(shape, generator=g) - 1)
        else:
            if key.startswith("input_layer"):
                fan_in = 9 * (1 if key.startswith("input_layer.0") else 64)
            elif key.endswith(".bias"):
                fan_in = cfg.d_model
            else:
                fan_in = shape[1]
            a = 1.0 / math.sqrt(fan_in)
            t = (2 * torch.rand(shape, generator=g) - 1) * a
        out[key] = t.float()
    return out


def synthetic_batch(cfg: OracleConfig, batch: int, n_frames: int, text_len: int, seed: int = 1234):
    """Synthetic inputs of the bench contract: spectrum ~ N(0,1) in the reference
    layout (B,1,F,T); text = BOS, tokens ~ U[5,V), EOS at a length ~ U[L/2, L], PAD after;
    mask = (text != PAD) as float."""
    g = torch.Generator().manual_seed(seed)
    spectrum = torch.randn((batch, 1, cfg.input_dim, n_frames), generator=g)
    text = torch.full((batch, text_len), cfg.pad_id, dtype=torch.long)
    lo = max(2, text_len // 2)
    lens = torch.randint(lo, text_len + 1, (batch,), generator=g)
    for b in range(batch):
        n = int(lens[b])
        text[b, 0] = 1
        if n > 2:
            text[b, 1:n - 1] = torch.randint(5, cfg.vocab_size, (n - 2,), generator=g)
        text[b, n - 1] = cfg.eos_id
    mask = (text != cfg.pad_id).float()
    return spectrum, text, mask


# Bench / test configurations of BASELINE.json (L chosen per SURVEY.md §8(d)).
CONFIGS = {
    "micro": dict(cfg=OracleConfig(vocab_size=250, input_dim=80, d_model=64, dec_len=8, enc_len=16, n_enc=1,
                                   n_dec=1, n_heads=4, ff_dim=256), batch=2, frames=60, text_len=8),
    "c1": dict(cfg=OracleConfig(d_model=128, dec_len=16, enc_len=100, n_enc=2, n_dec=2, n_heads=4, ff_dim=512),
               batch=4, frames=100, text_len=16),
    "c2": dict(cfg=OracleConfig(d_model=256, dec_len=32, enc_len=512, n_enc=6, n_dec=6, n_heads=4, ff_dim=1024),
               batch=32, frames=512, text_len=32),
    "c3": dict(cfg=OracleConfig(d_model=512, dec_len=64, enc_len=1000, n_enc=12, n_dec=12, n_heads=8, ff_dim=2048),
               batch=64, frames=1000, text_len=64),
    "c5": dict(cfg=OracleConfig(d_model=512, dec_len=256, enc_len=4000, n_enc=12, n_dec=12, n_heads=8, ff_dim=2048),
               batch=16, frames=4000, text_len=256),
    # d_head = 64 gradient fixtures (tests/golden/make_golden.py): the bf16 training path's resident-K/V attention
    # kernels (T' = 49 <= 256) and the tiled long-sequence kernels (T' = 274 > 256) pinned to the reference
    "g64": dict(cfg=OracleConfig(d_model=128, dec_len=16, enc_len=64, n_enc=1, n_dec=1, n_heads=2, ff_dim=256),
                batch=2, frames=200, text_len=16),
    "g64l": dict(cfg=OracleConfig(d_model=128, dec_len=16, enc_len=300, n_enc=1, n_dec=1, n_heads=2, ff_dim=256),
                 batch=1, frames=1100, text_len=16),
}
