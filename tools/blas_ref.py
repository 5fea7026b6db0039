"""Library ceiling check: the c3 projection / data-gradient / weight-gradient GEMM shapes timed with torch.mm
(hipBLASLt on ROCm, plain C = A.B, no epilogue) beside asrx's own kernels (with the epilogue the step uses
where noted).  Each number: median over rounds of `reps` back-to-back launches, HIP events.

    python tools/blas_ref.py [--reps 20] [--rounds 5]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402

# (name, kind, M, N, K): fwd C[M,N] = X[M,K] W[N,K]^T ; dgrad C[M,K'] = dY[M,N] W[N,K'] ; wgrad C[N,K] = dY^T X
SHAPES = [
    ("qkv fwd", "fwd", 15936, 1536, 512),
    ("ffn1 fwd", "fwd", 15936, 2048, 512),
    ("ffn2 fwd", "fwd", 15936, 512, 2048),
    ("out fwd", "fwd", 15936, 512, 512),
    ("xkv fwd", "fwd", 15936, 12288, 512),
    ("qkv dgrad", "dgrad", 15936, 512, 1536),
    ("ffn1 dgrad", "dgrad", 15936, 512, 2048),
    ("ffn2 dgrad", "dgrad", 15936, 2048, 512),
    ("xkv dgrad", "dgrad", 15936, 512, 12288),
    ("qkv wgrad", "wgrad", 1536, 512, 15936),
    ("ffn1 wgrad", "wgrad", 2048, 512, 15936),
    ("ffn2 wgrad", "wgrad", 512, 2048, 15936),
    ("xkv wgrad", "wgrad", 12288, 512, 15936),
]


def timeit(fn, reps, rounds):
    fn()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps * 1e-3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*s):
        return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()
    for name, kind, M, N, Kd in SHAPES:
        if kind == "fwd":
            x, w = rnd(M, Kd), rnd(N, Kd)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            flops = 2.0 * M * N * Kd
            tb = timeit(lambda: torch.mm(x, w.t(), out=y), args.reps, args.rounds)
            ta = timeit(lambda: K.linear(x, w, y), args.reps, args.rounds)
        elif kind == "dgrad":
            dy, w = rnd(M, N), rnd(N, Kd)
            y = torch.empty(M, Kd, device="cuda", dtype=torch.bfloat16)
            flops = 2.0 * M * N * Kd
            tb = timeit(lambda: torch.mm(dy, w, out=y), args.reps, args.rounds)
            ta = timeit(lambda: K.linear_dgrad(dy, w, y), args.reps, args.rounds)
        else:   # wgrad: C[M=N_out, N=K_in] over the Kd rows
            dy, x = rnd(Kd, M), rnd(Kd, N)
            c32 = torch.zeros(M, N, device="cuda")
            cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            flops = 2.0 * M * N * Kd
            tb = timeit(lambda: torch.mm(dy.t(), x, out=cb), args.reps, args.rounds)
            ta = timeit(lambda: K.linear_wgrad_grouped([(dy, x, c32, None)], beta=0.0), args.reps, args.rounds)
        print(f"{name:11s} M={M:6d} N={N:6d} K={Kd:6d} | hipBLASLt {tb * 1e6:7.1f}us {flops / tb / 1e12:6.0f}TF"
              f" | asrx {ta * 1e6:7.1f}us {flops / ta / 1e12:6.0f}TF", flush=True)


if __name__ == "__main__":
    main()
