"""Host-side (Python) cost of the c3 training step: cProfile over a few steps, top functions by own time.

    python tools/host_profile.py [--steps 3]
"""
import argparse
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import asrx
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch
    spec = CONFIGS["c3"]
    cfg = spec["cfg"]
    torch.manual_seed(0)
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    tr = Trainer(model)
    s, t, m = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1)
    s, t, m = s.cuda(), t.cuda(), m.cuda()
    for _ in range(2):
        tr.step(s, t, m)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        tr.step(s, t, m)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(45)


if __name__ == "__main__":
    main()
