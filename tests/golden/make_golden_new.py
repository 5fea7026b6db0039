"""Golden vectors of the reference's second model family, `modules/Transformer/new/` (build container only).

    python tests/golden/make_golden_new.py          # writes tests/golden/new_model.npz

As shipped, `new/model.py:5-6` imports the MAIN `modules.Transformer.layers` / `masking` and raises.
This script runs the variant the way it works — with its OWN `new/layers.py` and `new/masking.py` registered under
the module names `new/model.py` imports (read-only, nothing is written under /root/reference) — builds it for the
`oracle.ref_model_new.NEW_CONFIGS` configurations, loads the deterministic weights of `oracle.ref_model_new.det_params`
and records inputs and outputs: eval logits, a dropout-0 training loss (cross-entropy against the left-shifted
tokens, as new/train.py feeds `true_text`) with every parameter gradient, greedy `evaluate` outputs and the
state_dict schema.  The reference never travels to the GPU box: only the .npz data does.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

_nl = importlib.import_module("modules.Transformer.new.layers")
_nm = importlib.import_module("modules.Transformer.new.masking")
sys.modules["modules.Transformer.layers"] = _nl      # the variant's own modules under the names it imports
sys.modules["modules.Transformer.masking"] = _nm
_model = importlib.import_module("modules.Transformer.new.model")

from oracle.ref_model_new import NEW_CONFIGS, det_params, synthetic_batch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def build_ref(cfg):
    m = _model.Transformer(vocab_size=cfg.vocab_size, n_mels=cfg.n_mels, enc_seq_len=cfg.enc_seq_len,
                           dec_seq_len=cfg.dec_seq_len, hidden_dim=cfg.hidden_dim, enc_num_layers=cfg.n_enc,
                           dec_num_layers=cfg.n_dec, num_heads=cfg.n_heads, ff_dim=cfg.ff_dim, device="cpu",
                           dropout=cfg.dropout, sr=cfg.sr, n_fft=cfg.n_fft, padding_idx=cfg.pad_id,
                           eos_token=cfg.eos_id, bos_token=cfg.bos_id)
    sd = m.state_dict()
    P = det_params(cfg, 0)
    for k, v in P.items():
        assert sd[k].shape == v.shape, (k, sd[k].shape, v.shape)
        sd[k] = v
    m.load_state_dict(sd)
    return m


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def targets(text, eos):
    """new/train.py's `true_text`: the tokens shifted left by one, EOS-filled."""
    t = torch.full_like(text, eos)
    t[:, :-1] = text[:, 1:]
    return t


def main():
    out, schema = {}, {}
    for name, cfg in NEW_CONFIGS.items():
        m = build_ref(cfg)
        schema[name] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        schema[name + "_nparams"] = sum(p.numel() for p in m.parameters())
        spectre, lens, text = synthetic_batch(cfg, 3, seed=99)
        batch = {"spectre": spectre, "spectrogram_len": lens, "encoded_text": text}
        m.eval()
        with torch.no_grad():
            logits = m(batch)
            enc = m.encoder(spectre, lens)
        m.train()      # dropout 0: the training graph, same values
        m.zero_grad()
        lg = m(batch)
        loss = torch.nn.functional.cross_entropy(lg.transpose(1, 2), targets(text, cfg.eos_id))
        loss.backward()
        m.eval()
        with torch.no_grad():
            preds, last, eoses = m.evaluate(batch)
        p = name + "/"
        out[p + "spectre"], out[p + "lens"], out[p + "text"] = np32(spectre), lens.numpy(), text.numpy()
        out[p + "logits"], out[p + "enc"], out[p + "loss"] = np32(logits), np32(enc), np.float32(loss.item())
        names, nograd = [], []
        for k, prm in m.named_parameters():
            if prm.grad is None:
                nograd.append(k)
            else:
                names.append(k)
                out[p + "grad/" + k] = np32(prm.grad)
        out[p + "grad_names"], out[p + "nograd_names"] = np.array(names), np.array(nograd)
        out[p + "eval_tokens"], out[p + "eval_last"], out[p + "eval_eoses"] = \
            preds.numpy(), np32(last), eoses.numpy()
        print(name, "loss", float(loss), "logits", tuple(logits.shape), "tokens", preds[0].tolist())
    np.savez_compressed(os.path.join(OUT, "new_model.npz"), **out)
    with open(os.path.join(OUT, "ref_new_state_dict_schema.json"), "w") as f:
        json.dump(schema, f)


if __name__ == "__main__":
    main()
