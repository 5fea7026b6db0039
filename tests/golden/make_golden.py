"""Generate golden vectors by running the REFERENCE implementation (build container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

Imports `/root/reference/modules/Transformer/{model,layers}.py` read-only, builds the reference
`Transformer` for small configs, loads the deterministic weights of `oracle.det_params` into it and
records inputs/outputs.  The reference never travels to the GPU box: only the .npz data does.
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

from modules.Transformer.layers import TrainablePositionalEncoding  # noqa: E402
from modules.Transformer.model import Transformer  # noqa: E402

from oracle.ref_model import CONFIGS, det_params, synthetic_batch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def build_ref(cfg, dropout=None):
    m = Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                    cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout if dropout is None else dropout,
                    pad_token_id=cfg.pad_id, eos_token_id=cfg.eos_id)
    sd = m.state_dict()
    P = det_params(cfg, seed=0)
    for k, v in P.items():
        assert sd[k].shape == v.shape, (k, sd[k].shape, v.shape)
        sd[k] = v
    m.load_state_dict(sd)
    return m


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def gen_pe():
    out = {}
    for n, d in ((10, 8), (100, 128), (64, 512)):
        out[f"pe_{n}_{d}"] = np32(TrainablePositionalEncoding(n, d).pe[0])
    np.savez_compressed(os.path.join(OUT, "pe.npz"), **out)


def gen_ops():
    """Per-op cases on the micro config's submodules (d=64, h=4)."""
    cfg = CONFIGS["micro"]["cfg"]
    m = build_ref(cfg).eval()
    g = torch.Generator().manual_seed(7)
    B, Lq, Lk, d = 3, 9, 13, cfg.d_model
    x = torch.randn(B, Lq, d, generator=g)
    enc = torch.randn(B, Lk, d, generator=g)
    valid = torch.ones(B, Lq)
    valid[1, 6:] = 0
    valid[2, 2:] = 0
    pad = valid.lt(1).unsqueeze(1).expand(-1, Lq, -1)
    causal = torch.triu(torch.ones((Lq, Lq), dtype=torch.uint8), diagonal=1).unsqueeze(0).expand(B, -1, -1)
    dmask = torch.logical_or(torch.logical_or(pad, pad.mT), causal)
    dl = m.decoder._layers[0]
    el = m.encoder._layers[0]
    with torch.no_grad():
        out = dict(
            x=np32(x), enc=np32(enc), valid=np32(valid), dmask=dmask.numpy().astype(np.uint8),
            mha_self=np32(el._attention(x)),
            mha_masked=np32(dl._mask_attention(x, attention_mask=dmask)),
            mha_cross=np32(dl._cross_attention(x, enc_x=enc)),
            ffn=np32(el._feedforward(x)),
            ln=np32(el._norm1(x)),
            dec_layer=np32(dl(x, dmask, enc)),
            enc_layer=np32(el(x)),
        )
        spec = torch.randn(2, 1, cfg.input_dim, 100, generator=g)
        out["spec"] = np32(spec)
        out["front"] = np32(m.input_layer(spec))
    np.savez_compressed(os.path.join(OUT, "ops_micro.npz"), **out)


def gen_model(name, train_grads_full):
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    spectrum, text, mask = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1234)
    m = build_ref(cfg).eval()
    out = dict(spectrum=np32(spectrum), text=text.numpy().astype(np.int64), mask=np32(mask))
    with torch.no_grad():
        feat = m.input_layer(spectrum)
        enc = m.encoder(feat)
        logits = m(spectrum, text[:, :-1], mask[:, :-1])
    out["enc"] = np32(enc)
    out["logits"] = np32(logits)
    # dropout=0 training step: CE(logits^T, text[:,1:]) as train.py:32, then backward (train.py:34).
    mt = build_ref(cfg, dropout=0.0).train()
    lt = mt(spectrum, text[:, :-1], mask[:, :-1])
    loss = torch.nn.functional.cross_entropy(lt.transpose(1, 2), text[:, 1:])
    loss.backward()
    out["loss"] = np.float32(loss.item())
    names, norms = [], []
    for k, p in mt.named_parameters():
        if p.grad is None:
            continue
        names.append(k)
        norms.append(float(p.grad.norm()))
        if train_grads_full:
            out["grad/" + k] = np32(p.grad)
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array(norms, dtype=np.float64)
    out["nograd_names"] = np.array([k for k, p in mt.named_parameters() if p.grad is None])
    # greedy decode (model.py:201-206) from a BOS column, as eval_epoch builds it (train.py:70)
    with torch.no_grad():
        bos = torch.full((spec["batch"], 1), 1, dtype=torch.int32)
        row, probs = m.evaluate(spectrum, bos)
    out["greedy_row"] = row.numpy().astype(np.int64)
    out["greedy_nprobs"] = np.int64(len(probs))
    if len(probs):
        out["greedy_last_probs"] = np32(probs[-1])
    np.savez_compressed(os.path.join(OUT, f"model_{name}.npz"), **out)


def gen_grads(name, full_filter=None):
    """dropout=0 training step of the reference at a d_head = 64 config (train.py:28-34: forward, CE over
    text[:, 1:], backward): loss, logits, every parameter gradient (full tensors for keys passing
    `full_filter`, norms for all)."""
    spec = CONFIGS[name]
    cfg = spec["cfg"]
    spectrum, text, mask = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=4242)
    out = dict(spectrum=np32(spectrum), text=text.numpy().astype(np.int64), mask=np32(mask))
    mt = build_ref(cfg, dropout=0.0).train()
    lt = mt(spectrum, text[:, :-1], mask[:, :-1])
    loss = torch.nn.functional.cross_entropy(lt.transpose(1, 2), text[:, 1:])
    loss.backward()
    out["logits"] = np32(lt)
    out["loss"] = np.float32(loss.item())
    names, norms = [], []
    for k, p in mt.named_parameters():
        if p.grad is None:
            continue
        names.append(k)
        norms.append(float(p.grad.norm()))
        if full_filter is None or full_filter(k):
            out["grad/" + k] = np32(p.grad)
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array(norms, dtype=np.float64)
    out["nograd_names"] = np.array([k for k, p in mt.named_parameters() if p.grad is None])
    np.savez_compressed(os.path.join(OUT, f"grads_{name}.npz"), **out)


def gen_schema():
    """Reference state_dict key order and shapes (drop-in schema check without the reference present)."""
    import json
    out = {}
    for name in ("micro", "c1", "c3"):
        cfg = CONFIGS[name]["cfg"]
        m = build_ref(cfg) if name != "c3" else Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len,
                                                           cfg.enc_len, cfg.n_enc, cfg.n_dec, cfg.n_heads,
                                                           cfg.ff_dim)
        out[name] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        out[name + "_nparams"] = sum(p.numel() for p in m.parameters())
    with open(os.path.join(OUT, "ref_state_dict_schema.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    torch.manual_seed(0)
    gen_schema()
    gen_pe()
    gen_ops()
    gen_model("micro", train_grads_full=True)
    gen_model("c1", train_grads_full=False)
    gen_grads("g64")
    # long sequence: full tensors for the attention parameters (the tiled kernels' gradients), norms elsewhere
    gen_grads("g64l", lambda k: "_attention" in k or "_norm" in k)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
