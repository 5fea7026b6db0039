"""GEMM micro-benchmark on the c3 training-step shapes (A/B of kernel variants in ONE process, interleaved).

    python tools/gemm_bench.py [--variants glds,reg] [--reps 20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402

M_ENC, M_DEC = 64 * 249, 64 * 64
# (name, M, N, K, kind): fwd = x.W^T ; dgrad = dy.W ; wgrad = dy^T.x
SHAPES = [
    ("enc_qkv_fwd", M_ENC, 1536, 512, "fwd"), ("enc_ffn1_fwd", M_ENC, 2048, 512, "fwd"),
    ("enc_ffn2_fwd", M_ENC, 512, 2048, "fwd"), ("enc_out_fwd", M_ENC, 512, 512, "fwd"),
    ("cross_kv_fwd", M_ENC, 12288, 512, "fwd"), ("dec_ffn1_fwd", M_DEC, 2048, 512, "fwd"),
    ("enc_ffn1_dgrad", M_ENC, 512, 2048, "dgrad"), ("enc_qkv_dgrad", M_ENC, 512, 1536, "dgrad"),
    ("enc_ffn2_dgrad", M_ENC, 2048, 512, "dgrad"), ("cross_kv_dgrad", M_ENC, 512, 12288, "dgrad"),
    ("enc_ffn1_wgrad", M_ENC, 2048, 512, "wgrad"), ("enc_qkv_wgrad", M_ENC, 1536, 512, "wgrad"),
    ("enc_out_wgrad", M_ENC, 512, 512, "wgrad"), ("cross_kv_wgrad", M_ENC, 12288, 512, "wgrad"),
    ("dec_ffn1_wgrad", M_DEC, 2048, 512, "wgrad"),
    ("dec_out_fwd", M_DEC, 512, 512, "fwd"), ("dec_qkv_fwd", M_DEC, 1536, 512, "fwd"),
    ("dec_out_dgrad", M_DEC, 512, 512, "dgrad"), ("dec_ffn1_dgrad", M_DEC, 512, 2048, "dgrad"),
    ("dec_qkv_dgrad", M_DEC, 512, 1536, "dgrad"),
]


def run_shape(M, N, Kd, kind, bufs, variant="auto"):
    x, w, y, dy, wg, bg = bufs
    if variant == "torch":   # hipBLASLt / rocBLAS through torch (reference point only, not used by asrx)
        if kind == "fwd":
            torch.matmul(x, w.t(), out=y)
        elif kind == "dgrad":
            torch.matmul(dy, w, out=y)
        else:
            wg.add_(torch.matmul(dy.t(), x).float())
        return
    if kind == "fwd":
        K.linear(x, w, y)
    elif kind == "dgrad":
        K.linear_dgrad(dy, w, y)
    else:
        K.linear_wgrad(dy, x, wg, bias_grad=bg)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="auto,p3,glds,reg")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated shape names")
    args = ap.parse_args()
    variants = args.variants.split(",")
    results = {}
    for name, M, N, Kd, kind in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        if kind == "fwd":
            x = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
            w = torch.randn(N, Kd, device="cuda", generator=g).bfloat16()
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            bufs = (x, w, y, None, None, None)
        elif kind == "dgrad":       # y[M,N] = dy[M,K] . w[K,N]
            dy = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
            w = torch.randn(Kd, N, device="cuda", generator=g).bfloat16()
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            bufs = (None, w, y, dy, None, None)
        else:                       # wg[N,K] = dy[M,N]^T x[M,K]
            dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
            x = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
            wg = torch.zeros(N, Kd, device="cuda")
            bg = torch.zeros(N, device="cuda")
            bufs = (x, None, None, dy, wg, bg)
        flops = 2.0 * M * N * Kd
        times = {v: [] for v in variants}
        for r in range(args.reps + 2):
            for v in variants:
                kv = v.split("+")          # "ring+ASRX_RING_XCD=0": kernel family plus extra env settings
                os.environ["ASRX_GEMM_KERNEL"] = kv[0]
                for ev in kv[1:]:
                    key, val = ev.split("=")
                    os.environ[key] = val
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run_shape(M, N, Kd, kind, bufs, kv[0])
                for ev in kv[1:]:
                    os.environ.pop(ev.split("=")[0], None)
                e.record()
                e.synchronize()
                if r >= 2:
                    times[v].append(s.elapsed_time(e))
        line = f"{name:18s} M={M:6d} N={N:6d} K={Kd:6d}"
        for v in variants:
            t = sorted(times[v])[len(times[v]) // 2]
            line += f" | {v}: {t*1e3:7.1f}us {flops/t/1e9:6.0f}TF"
            results.setdefault(v, 0.0)
            results[v] += t
        print(line, flush=True)
    print("total(ms):", {v: round(t, 3) for v, t in results.items()})


if __name__ == "__main__":
    main()
