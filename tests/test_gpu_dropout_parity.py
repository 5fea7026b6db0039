"""The training configuration itself — dropout 0.1 — against the oracle: the HIP path draws its dropout decisions
from its counter hash (csrc/common.h), the reference from torch's Philox stream, so the two can only be compared
with the SAME masks.  The seeds the HIP forward draws are recorded (asrx.blocks.Seeds, in the forward's fixed
order), the masks regenerated on the CPU by tests/rng_ref.py (the hash restated in numpy, pinned by
test_host_cpu / test_gpu_kernels) and injected into the oracle's nn.Dropout sites (oracle.ref_model.DROP_MASKS):
logits, loss and every parameter gradient of one training step must then agree — which pins, per dropout site of
the reference (layers.py:27 attention probabilities, :40 MHA output, :56 FFN hidden, model.py:117 decoder input),
that the HIP path drops where the reference drops, scales by 1/(1-p), and regenerates the same masks in the
backward.  Tolerances as tests/test_gpu_model.py / test_gpu_train_parity.py: fp32 logits <= 1e-4, gradients
<= 1e-3 (relative, both norms); bf16 (the bench's fused attention + LayerNorm keep-bit path, d_head 64): logits
within 1.5x the reference's own bf16-autocast error, gradients <= 5e-2 Frobenius / 1.5e-1 max norm or within 1.5x
that path's own error."""
import dataclasses
import os
import re

import numpy as np
import pytest
import torch

import oracle.ref_model as R
from oracle.ref_model import CONFIGS, det_params, synthetic_batch
from tests.rng_ref import attn_keep, elem_keep

pytestmark = pytest.mark.gpu
dev = "cuda"
P_DROP = 0.1


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def relerr(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def site_seeds(seeds, cfg):
    """Map the HIP forward's seed draws to the reference's dropout sites.  Draw order (asrx/functions.py
    encoder_fwd / decoder_fwd, asrx/blocks.py): per encoder layer the self-attention probabilities (attn_prepare),
    its output projection, the FFN hidden layer; then the decoder input embedding; per decoder layer the masked
    self-attention probabilities and output, the cross-attention probabilities and output, the FFN."""
    it = iter(seeds)
    out = {}
    for l in range(cfg.n_enc):
        key = f"encoder._layers.{l}"
        out[("attn", key + "._attention")] = next(it)
        out[("out", key + "._attention")] = next(it)
        out[("ffn", key + "._feedforward")] = next(it)
    out[("emb", "decoder")] = next(it)
    for l in range(cfg.n_dec):
        key = f"decoder._layers.{l}"
        for mha in ("._mask_attention", "._cross_attention"):
            out[("attn", key + mha)] = next(it)
            out[("out", key + mha)] = next(it)
        out[("ffn", key + "._feedforward")] = next(it)
    assert next(it, None) is None, "more seed draws than dropout sites"
    return out


def mask_provider(seeds, cfg, batch, swap=None):
    """DROP_MASKS callable over the recorded seeds (swap: one site whose mask is drawn from a wrong seed)."""
    H = cfg.n_heads

    def masks(site, shape):
        kind, key = site
        if kind == "attn":
            mha, head = re.match(r"(.*)\._?heads\.(\d+)$", key).groups()   # main `._heads.i`, new/ `.heads.i`
            seed = seeds[("attn", mha)] ^ (1 if ("attn", mha) == swap else 0)
            b, lq, lk = shape
            keep = attn_keep(seed, b * H, lq, lk, P_DROP).reshape(b, H, lq, lk)[:, int(head)]
        else:
            seed = seeds[site] ^ (1 if site == swap else 0)
            keep = elem_keep(seed, int(np.prod(shape)), P_DROP).reshape(shape)
        return torch.from_numpy(np.ascontiguousarray(keep))

    return masks


def run_hip(name, precision, batch=None, frames=None):
    """One training-mode forward + backward of the asrx Transformer at dropout 0.1; returns logits, loss, grads
    (reference state_dict keys) and the recorded seeds."""
    import asrx
    import asrx.blocks as Bk
    import asrx.kernels as K
    cfg = CONFIGS[name]["cfg"]
    spec = CONFIGS[name]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=P_DROP, precision=precision)
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    m = m.to(dev).train()
    s, t, k = synthetic_batch(cfg, batch or spec["batch"], frames or spec["frames"], spec["text_len"] + 1, seed=77)
    K.set_seed_offset(0)   # eager: the kernels use the drawn seeds as they are (a Trainer may have left an offset)
    torch.cuda.manual_seed(1234)   # the seed base (functions.draw_seed reads torch's CUDA generator): reproducible
    drawn = []
    nxt = Bk.Seeds.next

    def record(self):
        v = nxt(self)
        drawn.append(v)
        return v

    Bk.Seeds.next = record
    try:
        logits = m(s.to(dev), t[:, :-1].to(dev), k[:, :-1].to(dev))
    finally:
        Bk.Seeds.next = nxt
    loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), t[:, 1:].to(dev))
    loss.backward()
    torch.cuda.synchronize()
    twin = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                            cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0)
    with torch.no_grad():
        for p1, p2 in zip(m.parameters(), twin.parameters()):
            p2.copy_(p1.grad.cpu() if p1.grad is not None else torch.zeros_like(p2))
    return logits.detach().cpu(), float(loss.detach()), twin.state_dict(), drawn, (s, t, k), cfg


def run_oracle(cfg, batch, masks, autocast=False):
    P = {k_: v.double().requires_grad_(True) for k_, v in det_params(cfg, 0).items()}
    s, t, k = batch
    old = R.DROP_MASKS
    R.DROP_MASKS = masks
    try:
        if autocast:   # the reference's bf16 path: torch.autocast over the fp32 oracle, forward and backward
            P = {k_: v.detach().float().requires_grad_(True) for k_, v in P.items()}
            with torch.autocast("cpu", dtype=torch.bfloat16):
                logits = R.forward(P, s.float(), t[:, :-1], k[:, :-1], cfg, True).float()
        else:
            logits = R.forward(P, s.double(), t[:, :-1], k[:, :-1], cfg, True)
        loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), t[:, 1:])
        loss.backward()
        return logits.detach(), float(loss.detach()), {k_: v.grad for k_, v in P.items()}
    finally:
        R.DROP_MASKS = old


def frorel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def check_grads(gsd, ref_grads, tol, max_tol, ref16=None):
    """Every gradient within tol (Frobenius) and max_tol (max norm) of the fp64 oracle, relative; with ref16 (the
    reference's own bf16-autocast gradients) a tensor may exceed them while it stays within 1.5x that path's error
    in both norms (the rule of tests/test_gpu_train_parity.py)."""
    gmax = max(float(g.abs().max()) for g in ref_grads.values() if g is not None)
    worst = []
    for key, ref in ref_grads.items():
        if ref is None:
            continue
        if float(ref.abs().max()) < 1e-6 * gmax:   # mathematically zero (K bias): absolute at the global scale
            assert float((gsd[key].double() - ref).abs().max()) < tol * 1e-2 * gmax, key
            continue
        e, em = frorel(gsd[key], ref), relerr(gsd[key], ref)
        t, mt = tol, max_tol
        if ref16 is not None:
            t, mt = max(t, 1.5 * frorel(ref16[key], ref)), max(mt, 1.5 * relerr(ref16[key], ref))
        worst.append((max(e / t, em / mt), key, e, em))
    worst.sort(reverse=True)
    print("worst gradients (err / allowed, key, frobenius, max):",
          [(round(r, 3), k, f"{e:.2e}", f"{em:.2e}") for r, k, e, em in worst[:3]])
    assert worst[0][0] < 1.0, worst[:3]


def test_dropout_training_step_fp32_matches_oracle_with_same_masks():
    """c1 dims (2+2 layers, d 128, 4 heads: the materialised-score attention with the softmax-kernel dropout),
    dropout 0.1: logits, loss and every gradient of the step against the oracle (fp64) with the HIP path's masks;
    a control with ONE site's mask drawn from a wrong seed must fail the same bound."""
    torch.set_num_threads(max(1, min(32, len(os.sched_getaffinity(0)))))
    logits, loss, gsd, drawn, batch, cfg = run_hip("c1", "fp32")
    seeds = site_seeds(drawn, cfg)
    assert len(set(seeds.values())) == len(seeds)
    ref, ref_loss, ref_grads = run_oracle(cfg, batch, mask_provider(seeds, cfg, batch))
    e = relerr(logits, ref)
    print(f"\nc1 fp32 dropout {P_DROP}: logits rel err {e:.2e}, loss {loss:.6f} vs {ref_loss:.6f}")
    assert e < 1e-4, e
    assert abs(loss - ref_loss) < 1e-4 * abs(ref_loss)
    check_grads(gsd, ref_grads, 1e-3, 1e-3)
    for swap in (("out", "encoder._layers.1._attention"), ("attn", "decoder._layers.0._cross_attention")):
        bad, _, _ = run_oracle(cfg, batch, mask_provider(seeds, cfg, batch, swap=swap))
        assert relerr(logits, bad) > 1e-2, swap   # the comparison sees a single wrong mask


@pytest.mark.parametrize("name,batch,frames", [("g64", None, None), ("c3", 2, 1000)])
def test_dropout_training_step_bf16_matches_oracle_with_same_masks(name, batch, frames):
    """bf16 at d_head 64, dropout 0.1, against the fp64 oracle under the HIP path's masks: g64 (1+1 layers) and the
    bench's own model dims c3 (12+12 layers, d 512, 8 heads, T = 1000 frames; B = 2) — the fused attention with keep
    bits from the preceding LayerNorm's launch, the ws / p4 GEMM epilogues' dropout and the FFN1 1-bit gate: the
    timed configuration's kernels.  Logits within 1.5x the reference's own bf16-autocast error (same masks),
    gradients by the bf16 rule of test_gpu_train_parity.py."""
    torch.set_num_threads(max(1, min(32, len(os.sched_getaffinity(0)))))
    logits, loss, gsd, drawn, data, cfg = run_hip(name, "bf16", batch, frames)
    seeds = site_seeds(drawn, cfg)
    masks = mask_provider(seeds, cfg, data)
    ref, ref_loss, ref_grads = run_oracle(cfg, data, masks)
    ref16, _, grads16 = run_oracle(cfg, data, masks, autocast=True)
    e, e16 = relerr(logits, ref), relerr(ref16, ref)
    print(f"\n{name} bf16 dropout {P_DROP}: logits rel err {e:.2e} (reference bf16 autocast {e16:.2e}), "
          f"loss {loss:.5f} vs {ref_loss:.5f}")
    assert e <= 1.5 * e16, (e, e16)
    assert abs(loss - ref_loss) < 1e-2 * abs(ref_loss)
    check_grads(gsd, ref_grads, 5e-2, 1.5e-1, ref16=grads16)


def test_new_family_dropout_training_step_matches_oracle_with_same_masks():
    """The new/ family (post-LN, full-width heads, asrx.new) at new_small dims, fp32, dropout 0.1: logits, loss and
    every gradient against oracle/ref_model_new.py (fp64) with the HIP path's masks — the same draw order as the
    main family (per encoder layer: attention probabilities, output, FFN; the decoder embedding; per decoder layer:
    masked self-attention, cross-attention, FFN)."""
    import asrx.blocks as Bk
    import asrx.kernels as K
    import asrx.new
    import oracle.ref_model_new as N
    torch.set_num_threads(max(1, min(32, len(os.sched_getaffinity(0)))))
    c = N.NEW_CONFIGS["new_small"]
    m = asrx.new.Transformer(c.vocab_size, c.n_mels, c.enc_seq_len, c.dec_seq_len, c.hidden_dim, c.n_enc, c.n_dec,
                             c.n_heads, c.ff_dim, dev, dropout=P_DROP, sr=c.sr, n_fft=c.n_fft, padding_idx=c.pad_id,
                             eos_token=c.eos_id, bos_token=c.bos_id)
    sd = m.state_dict()
    sd.update(N.det_params(c, 0))
    m.load_state_dict(sd)
    m = m.to(dev).train()
    s, lens, text = N.synthetic_batch(c, 4, seed=31)
    tgt = torch.full_like(text, c.eos_id)
    tgt[:, :-1] = text[:, 1:]
    batch = {"spectre": s.to(dev), "spectrogram_len": lens.to(dev), "encoded_text": text.to(dev)}
    K.set_seed_offset(0)
    torch.cuda.manual_seed(4321)
    drawn, nxt = [], Bk.Seeds.next

    def record(self):
        v = nxt(self)
        drawn.append(v)
        return v

    Bk.Seeds.next = record
    try:
        logits = m(batch)
    finally:
        Bk.Seeds.next = nxt
    loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), tgt.to(dev))
    loss.backward()
    it = iter(drawn)
    seeds = {}
    for l in range(c.n_enc):
        k = f"encoder.layers.{l}"
        seeds[("attn", k + ".attention")], seeds[("out", k + ".attention")] = next(it), next(it)
        seeds[("ffn", k + ".ff")] = next(it)
    seeds[("emb", "decoder")] = next(it)
    for l in range(c.n_dec):
        k = f"decoder.layers.{l}"
        for mha in (".mask_attention", ".attention"):
            seeds[("attn", k + mha)], seeds[("out", k + mha)] = next(it), next(it)
        seeds[("ffn", k + ".ff")] = next(it)
    assert next(it, None) is None
    cfg_like = type("C", (), {"n_heads": c.n_heads})
    masks = mask_provider(seeds, cfg_like, None)
    P = {k: v.double().requires_grad_(True) for k, v in N.det_params(c, 0).items()}
    old = N.DROP_MASKS
    N.DROP_MASKS = masks
    try:   # (the oracle's dropout rate comes from its config: new_small's is the reference constructor's 0.0)
        ref = N.forward(P, s.double(), lens, text, dataclasses.replace(c, dropout=P_DROP), True)
    finally:
        N.DROP_MASKS = old
    ref_loss = torch.nn.functional.cross_entropy(ref.transpose(1, 2), tgt)
    ref_loss.backward()
    e = relerr(logits.detach(), ref.detach())
    print(f"\nnew_small fp32 dropout {P_DROP}: logits rel err {e:.2e}, loss {float(loss.detach()):.6f} vs "
          f"{float(ref_loss.detach()):.6f}")
    assert e < 1e-4, e
    twin = asrx.new.Transformer(c.vocab_size, c.n_mels, c.enc_seq_len, c.dec_seq_len, c.hidden_dim, c.n_enc, c.n_dec,
                                c.n_heads, c.ff_dim, dev, dropout=0.0, sr=c.sr, n_fft=c.n_fft, padding_idx=c.pad_id,
                                eos_token=c.eos_id, bos_token=c.bos_id).to(dev)
    with torch.no_grad():
        for p1, p2 in zip(m.parameters(), twin.parameters()):
            p2.copy_(p1.grad if p1.grad is not None else torch.zeros_like(p2))
    gsd = {k: v.cpu() for k, v in twin.state_dict().items()}
    check_grads(gsd, {k: v.grad for k, v in P.items() if v.grad is not None}, 1e-3, 1e-3)
