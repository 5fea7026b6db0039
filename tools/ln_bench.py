"""LayerNorm forward/backward micro-benchmark on the c3 shapes: time per call and achieved HBM GB/s
(algorithmic bytes: every operand read once, every output written once).

    python tools/ln_bench.py [--reps 20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402


def timed(fn, reps):
    """GPU time per call: reps calls captured in a HIP graph and replayed (no host launch gaps)."""
    sys.path.insert(0, REPO)
    from bench import _graph_time_ms
    return _graph_time_ms([fn], launches=reps) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--blocks", default="")
    args = ap.parse_args()
    d = 512
    for rows, name in ((64 * 249, "enc"), (64 * 64, "dec")):
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(rows, d, device="cuda", generator=g)
        gamma = torch.rand(d, device="cuda", generator=g) + 0.5
        beta = torch.randn(d, device="cuda", generator=g)
        y = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
        mean, rstd = K.layernorm_fwd(x, gamma, beta, y)
        for rw in (1, 2, 4):   # rows per wave of the forward (asrx_set_tuning)
            K.set_tuning("ln_rw", rw)
            t = timed(lambda: K.layernorm_fwd(x, gamma, beta, y), args.reps)
            by = rows * d * (4 + 2) + rows * 8
            print(f"ln_fwd {name} rows={rows} rw={rw}: {t*1e6:7.2f} us  {by/t/1e9:7.0f} GB/s", flush=True)
        K.set_tuning("ln_rw", 0)
        dy = torch.randn(rows, d, device="cuda", generator=g).bfloat16()
        dres = torch.randn(rows, d, device="cuda", generator=g)
        dxd = torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)
        dgb = torch.zeros(2 * d, device="cuda")
        for nb in ([int(b) for b in args.blocks.split(",")] if args.blocks else [K.LN_BWD_BLOCKS]):
            K.LN_BWD_BLOCKS = nb
            t = timed(lambda: K.layernorm_bwd(x, dy, gamma, mean, rstd, dgb, dres=dres, dx_drop=dxd,
                                              dropout_p=0.1, seed=3, defer=[]), args.reps)
            by = rows * d * (4 + 2 + 4 + 4 + 2) + rows * 8
            print(f"ln_bwd {name} rows={rows} blocks={nb}: {t*1e6:7.2f} us  {by/t/1e9:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
