"""Every GEMM launch of one c3 training step (B=64): kernel instantiation and shape, with counts.

    python tools/plan_log.py
"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    import asrx
    from asrx import kernels as K
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch
    spec = CONFIGS["c3"]
    cfg = spec["cfg"]
    torch.manual_seed(0)
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    tr = Trainer(m, graph=False)
    s, t, k = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1)
    s, t, k = s.cuda(), t.cuda(), k.cuda()
    tr.step(s, t, k)
    probe = K.KernelProbe(target="", log=[])
    probe.active = True
    K.PROBE = probe
    tr.step(s, t, k)
    torch.cuda.synchronize()
    K.PROBE = None
    c = collections.Counter(probe.log)
    for (name, mm, n, kk, b, sk), cnt in sorted(c.items(), key=lambda x: (x[0][1], x[0][2], x[0][3])):
        print(f"{cnt:3d} x  M={mm:6d} N={n:6d} K={kk:6d} batch={b} splitk={sk}  {name}")


if __name__ == "__main__":
    main()
