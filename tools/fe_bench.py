"""Front-end micro-benchmark at the c3 shape (B = 64, 80 x 1000 spectrum): conv1 forward, conv2 forward (implicit
GEMM), conv2 weight gradient (tall-K), conv1 gradients from dy2 (conv_bwd_implicit); time per launch (HIP-graph
replays, warm: one buffer set) and the HBM bytes each moves at least (every operand read once, outputs written once).

    python tools/fe_bench.py [--rounds 5]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--dbg", default="0", help="comma list of asrx_gemm_set_debug flags (diagnostics: garbage results)")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    B, F, T = args.B, 80, 1000
    F1, T1 = (F - 3) // 2 + 1, (T - 3) // 2 + 1
    F2, T2 = (F1 - 3) // 2 + 1, (T1 - 3) // 2 + 1
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, 1, F, T, device="cuda", generator=g)
    w1 = torch.randn(64, 1, 3, 3, device="cuda", generator=g) * 0.3
    b1 = torch.randn(64, device="cuda", generator=g) * 0.1
    y1 = torch.empty(B, F1, T1, 64, device="cuda", dtype=torch.bfloat16)
    m1 = torch.empty(B, F1, T1, 8, device="cuda", dtype=torch.uint8)
    w2 = (torch.randn(64, 576, device="cuda", generator=g) * 0.05).bfloat16()
    b2 = torch.randn(64, device="cuda", generator=g) * 0.1
    y2 = torch.empty(B * T2 * F2, 64, device="cuda", dtype=torch.bfloat16)
    dy2 = (torch.randn(B * T2 * F2, 64, device="cuda", generator=g) * 0.1).bfloat16()
    dw2 = torch.zeros(64, 576, device="cuda")
    db2 = torch.zeros(64, device="cuda")
    dw1 = torch.zeros(64, 9, device="cuda")
    db1 = torch.zeros(64, device="cuda")
    K.conv1_fwd(x, w1, b1, y1, m1)
    rows1, rows2 = B * F1 * T1, B * T2 * F2
    cases = [
        ("conv1_fwd", lambda: K.conv1_fwd(x, w1, b1, y1, m1), x.numel() * 4 + rows1 * 64 * 2 + rows1 * 8),
        ("conv2_fwd", lambda: K.conv2_fwd(y1, w2, b2, y2), rows1 * 64 * 2 + rows2 * 64 * 2),
        ("conv2_wgrad", lambda: K.conv2_wgrad(dy2, y1, dw2, db2), rows1 * 64 * 2 + rows2 * 64 * 2),
        ("conv_bwd_implicit", lambda: K.conv_bwd_implicit(dy2, w2, m1, x, dw1, db1), rows2 * 64 * 2 + rows1 * 8 + x.numel() * 4),
    ]
    for name, fn, byts in cases:
        if args.only and name not in args.only.split(","):
            continue
        for dbg in [int(v) for v in args.dbg.split(",")]:
            K.call("asrx_gemm_set_debug", dbg)
            t = _graph_time_ms([fn], launches=8, rounds=args.rounds) * 1e-3
            K.call("asrx_gemm_set_debug", 0)
            tag = name if dbg == 0 else f"{name}/d{dbg}"
            print(f"{tag:18s} {t * 1e6:8.1f} us   {byts / 1e6:7.1f} MB min   {byts / t / 1e12:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
