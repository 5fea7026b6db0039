"""Per-parameter gradient error of the bf16 Trainer step vs the oracle in fp32, next to the oracle's own bf16-autocast
error (the reference's bf16 path), sorted by the ratio of the two.

    python tools/grad_diag.py [--config c3] [--batch 2] [--frames 1000] [--top 40]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--attention", default="fused")
    args = ap.parse_args()
    import asrx
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, det_params, synthetic_batch, train_step_grads
    spec = CONFIGS[args.config]
    cfg = spec["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=0.0, precision="bf16", attention=args.attention)
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    m = m.cuda().train()
    s, t, k = synthetic_batch(cfg, args.batch, args.frames, spec["text_len"] + 1, seed=2024)
    tr = Trainer(m, graph=False)
    tr.forward_backward(s.cuda(), t.cuda(), k.cuda())
    tr.forward_backward(s.cuda(), t.cuda(), k.cuda())
    torch.cuda.synchronize()
    twin = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                            cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=0.0)
    with torch.no_grad():
        for p1, p2 in zip(m.parameters(), twin.parameters()):
            p2.copy_(p1.grad.cpu())
    ours = twin.state_dict()
    torch.set_num_threads(max(1, min(32, len(os.sched_getaffinity(0)))))
    P = {kk: v.clone().requires_grad_(True) for kk, v in det_params(cfg, 0).items()}
    _, ref = train_step_grads(P, s, t, k, cfg, training=False)
    P16 = {kk: v.clone().requires_grad_(True) for kk, v in det_params(cfg, 0).items()}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        _, r16 = train_step_grads(P16, s, t, k, cfg, training=False)

    def fro(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))
    rows = []
    for kk, v in ref.items():
        if v is None or float(v.abs().max()) == 0:
            continue
        e, e16 = fro(ours[kk], v), fro(r16[kk], v)
        rows.append((e / max(e16, 1e-12), e, e16, kk))
    rows.sort(reverse=True)
    print(f"{'ratio':>7} {'ours':>9} {'autocast':>9}  param")
    for r, e, e16, kk in rows[:args.top]:
        print(f"{r:7.2f} {e:9.2e} {e16:9.2e}  {kk}")
    import statistics
    print("median ours", statistics.median(r[1] for r in rows), "median autocast", statistics.median(r[2] for r in rows))


if __name__ == "__main__":
    main()
