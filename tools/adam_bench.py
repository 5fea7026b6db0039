"""The separate AdamW launch (the data-parallel step's optimizer, asrx_adam) alone: HIP-graph replays over the c3
flat buffers' size (half of the 89 M parameters per launch, as the DP step's two calls), 30 B per parameter moved
(p, m, v read + written, g read, bf16 shadow written).

    python tools/adam_bench.py [--n 44484864] [--vars 0,1]   (ASRX_ADAM_VAR: read by A/B builds that carry variants)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402
from bench import _graph_time_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=44484864)
    ap.add_argument("--vars", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    n = args.n
    g = torch.Generator(device="cuda").manual_seed(0)
    p = torch.randn(n, device="cuda", generator=g)
    gr = torch.randn(n, device="cuda", generator=g) * 1e-3
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    for var in args.vars.split(","):
        os.environ["ASRX_ADAM_VAR"] = var
        fn = lambda: K.adam(p, gr, m, v, pb, 1e-4, 0.9, 0.98, 1e-9, 0.01, 10)   # noqa: E731
        fn()
        t = _graph_time_ms([fn], launches=4, rounds=args.rounds) * 1e-3
        print(f"var {var:>2s}  {t * 1e6:8.1f} us  {30 * n / t / 1e12:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
