"""Pin the oracle (CPU restatement) to golden vectors produced by the reference itself."""
import os

import numpy as np
import pytest
import torch

from oracle.ref_model import (CONFIGS, attention_head, decoder_layer, decoder_mask, det_params, encoder, feed_forward,
                              forward, front_end, greedy_decode, multi_head, pe_table, synthetic_batch,
                              train_step_grads, _ln)


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def rel(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))


def test_pe_table_bitwise(golden_dir):
    g = load(golden_dir, "pe.npz")
    for key in g.files:
        _, n, d = key.split("_")
        np.testing.assert_array_equal(pe_table(int(n), int(d)).numpy(), g[key])


def test_ops_micro(golden_dir):
    g = load(golden_dir, "ops_micro.npz")
    cfg = CONFIGS["micro"]["cfg"]
    P = det_params(cfg)
    x, enc = torch.from_numpy(g["x"]), torch.from_numpy(g["enc"])
    dmask = torch.from_numpy(g["dmask"]).bool()
    ek, dk = "encoder._layers.0", "decoder._layers.0"
    with torch.no_grad():
        assert rel(multi_head(P, ek + "._attention", x, None, None, cfg, False), g["mha_self"]) < 1e-6
        assert rel(multi_head(P, dk + "._mask_attention", x, None, dmask, cfg, False), g["mha_masked"]) < 1e-6
        assert rel(multi_head(P, dk + "._cross_attention", x, enc, None, cfg, False), g["mha_cross"]) < 1e-6
        assert rel(feed_forward(P, ek + "._feedforward", x, cfg, False), g["ffn"]) < 1e-6
        assert rel(_ln(P, ek + "._norm1", x), g["ln"]) < 1e-6
        assert rel(decoder_layer(P, dk, x, dmask, enc, cfg, False), g["dec_layer"]) < 1e-6
        front = front_end(P, torch.from_numpy(g["spec"]))
        ref = torch.from_numpy(g["front"])
        b, c, f, t = ref.shape
        assert rel(front, ref.reshape(b, c * f, t).transpose(1, 2)) < 1e-6


def test_all_masked_row_is_zero(golden_dir):
    """nan_to_num(softmax(all -inf)) == 0 (layers.py:25): sample 2 has only 2 valid tokens, so its query
    rows >= 2 are fully masked and the head output there is exactly 0."""
    g = load(golden_dir, "ops_micro.npz")
    cfg = CONFIGS["micro"]["cfg"]
    P = det_params(cfg)
    x = torch.from_numpy(g["x"])
    dmask = torch.from_numpy(g["dmask"]).bool()
    with torch.no_grad():
        h = attention_head(P, "decoder._layers.0._mask_attention._heads.0", x, x, dmask, cfg.d_model, 0.0, False)
    assert torch.all(h[2, 2:] == 0)
    assert torch.all(torch.isfinite(h))


@pytest.mark.parametrize("name", ["micro", "c1"])
def test_model_forward(golden_dir, name):
    g = load(golden_dir, f"model_{name}.npz")
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    P = det_params(cfg)
    s, t, m = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1234)
    np.testing.assert_array_equal(s.numpy(), g["spectrum"])
    np.testing.assert_array_equal(t.numpy(), g["text"])
    with torch.no_grad():
        logits, enc = forward(P, s, t[:, :-1], m[:, :-1], cfg, False, return_encoder=True)
    assert rel(enc, g["enc"]) < 1e-5
    assert rel(logits, g["logits"]) < 1e-5


@pytest.mark.parametrize("name", ["micro", "c1"])
def test_train_step_grads(golden_dir, name):
    g = load(golden_dir, f"model_{name}.npz")
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    P = {k: v.clone().requires_grad_(True) for k, v in det_params(cfg).items()}
    s, t, m = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1234)
    loss, grads = train_step_grads(P, s, t, m, cfg, training=False)
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    names = list(g["grad_names"])
    for k, n in zip(names, g["grad_norms"]):
        assert grads[k] is not None, k
        assert abs(float(grads[k].norm()) - n) <= 1e-4 * n + 1e-7, k
        if "grad/" + k in g.files:
            assert rel(grads[k], g["grad/" + k]) < 1e-4, k
    # params the reference never touches get no gradient (input_encoding, _norm_in)
    for k in g["nograd_names"]:
        assert grads[k] is None or float(grads[k].abs().max()) == 0.0, k


@pytest.mark.parametrize("name", ["g64", "g64l"])
def test_train_step_grads_dh64(golden_dir, name):
    """d_head = 64 fixtures (the bf16 path's resident / tiled attention kernels): oracle loss, logits and every
    gradient vs the reference's own training step."""
    g = load(golden_dir, f"grads_{name}.npz")
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    P = {k: v.clone().requires_grad_(True) for k, v in det_params(cfg).items()}
    s, t, m = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=4242)
    np.testing.assert_array_equal(s.numpy(), g["spectrum"])
    np.testing.assert_array_equal(t.numpy(), g["text"])
    logits = forward(P, s, t[:, :-1], m[:, :-1], cfg, False)
    assert rel(logits.detach(), g["logits"]) < 1e-5
    loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), t[:, 1:])
    loss.backward()
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    for k, n in zip(g["grad_names"], g["grad_norms"]):
        gk = P[k].grad
        assert abs(float(gk.norm()) - n) <= 1e-4 * n + 1e-7, k
        if "grad/" + k in g.files:
            assert rel(gk, g["grad/" + k]) < 1e-4, k


def test_greedy_decode(golden_dir):
    g = load(golden_dir, "model_c1.npz")
    spec = CONFIGS["c1"]
    cfg = spec["cfg"]
    P = det_params(cfg)
    s = torch.from_numpy(g["spectrum"])
    bos = torch.full((spec["batch"], 1), 1, dtype=torch.int32)
    with torch.no_grad():
        row, probs = greedy_decode(P, s, bos, cfg)
    np.testing.assert_array_equal(row.numpy(), g["greedy_row"])
    assert len(probs) == int(g["greedy_nprobs"])
    assert rel(probs[-1], g["greedy_last_probs"]) < 1e-5


def test_decoder_mask_semantics():
    mask = torch.tensor([[1., 1., 1., 0.], [1., 0., 0., 0.]])
    m = decoder_mask(mask)
    assert m[0, 0].tolist() == [False, True, True, True]
    assert m[0, 3].tolist() == [True, True, True, True]     # query pad -> whole row masked
    assert m[1, 0].tolist() == [False, True, True, True]


# ---- the second model family, modules/Transformer/new/ (tests/golden/make_golden_new.py)

@pytest.mark.parametrize("name", ["new_micro", "new_small"])
def test_oracle_new_forward_grads_evaluate(golden_dir, name):
    """oracle.ref_model_new against the reference's new/ variant run with its own layers / masking: eval logits and
    encoder output, the dropout-0 loss and every parameter gradient (cross-entropy against the left-shifted tokens),
    the unused VGG front-end without gradients, and the greedy evaluate() tokens, EOS steps and last logits."""
    from oracle import ref_model_new as N
    g = load(golden_dir, "new_model.npz")
    cfg = N.NEW_CONFIGS[name]
    p = name + "/"
    s, lens, text = (torch.from_numpy(g[p + k]) for k in ("spectre", "lens", "text"))
    spec, lens2, text2 = N.synthetic_batch(cfg, 3, seed=99)
    assert torch.equal(spec, s) and torch.equal(lens2, lens) and torch.equal(text2, text)
    P = {k: v.clone().requires_grad_(True) for k, v in N.det_params(cfg).items()}
    logits = N.forward(P, s, lens, text, cfg, False)
    assert rel(logits.detach(), g[p + "logits"]) < 1e-5
    with torch.no_grad():
        assert rel(N.encoder(P, s, lens, cfg), g[p + "enc"]) < 1e-5
    tgt = torch.full_like(text, cfg.eos_id)
    tgt[:, :-1] = text[:, 1:]
    loss = torch.nn.functional.cross_entropy(logits.transpose(1, 2), tgt)
    loss.backward()
    assert abs(float(loss.detach()) - float(g[p + "loss"])) < 1e-5 * abs(float(g[p + "loss"]))
    for k in g[p + "grad_names"]:
        assert rel(P[k].grad, g[p + "grad/" + k]) < 1e-4, k
    for k in g[p + "nograd_names"]:
        assert P[k].grad is None, k
    with torch.no_grad():
        toks, last, eoses = N.evaluate(P, s, lens, cfg)
    np.testing.assert_array_equal(toks.numpy(), g[p + "eval_tokens"])
    np.testing.assert_array_equal(eoses.numpy(), g[p + "eval_eoses"])
    assert rel(last, g[p + "eval_last"]) < 1e-5
