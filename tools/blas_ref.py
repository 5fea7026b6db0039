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
    # the step's fused epilogues: FFN1 forward (bias, ReLU, dropout 0.1, 1-bit ReLU mask out) and the FFN2 data
    # gradient gated by those bits (alpha = 1/0.9)
    ("ffn1 fwd epi", "fwdepi", 15936, 2048, 512),
    ("ffn2 dgrad gated", "dgradg", 15936, 512, 2048),
    ("dec ffn1 fwd epi", "fwdepi", 4096, 2048, 512),
    ("dec ffn2 dgrad gated", "dgradg", 4096, 512, 2048),
    ("dec qkv fwd", "fwd", 4096, 1536, 512),
    # the step's plain data gradients (out 512 wide; dgrad kind: y[M, Kd] = dy[M, N] . w[N, Kd])
    ("enc qkv dg512", "dgrad", 15936, 1536, 512),
    ("enc ffn1 dg512", "dgrad", 15936, 2048, 512),
    ("enc out dg512", "dgrad", 15936, 512, 512),
    ("dec ffn1 dg512", "dgrad", 4096, 2048, 512),
    ("dec qkv dg512", "dgrad", 4096, 1536, 512),
    ("dec out dg512", "dgrad", 4096, 512, 512),
    # the FFN2 forward of the step: fp32 residual stream out = x . w^T + bias + resid
    ("ffn2 fwd res", "fwdres", 15936, 512, 2048),
    ("dec ffn2 fwd res", "fwdres", 4096, 512, 2048),
    ("out fwd res", "fwdres", 15936, 512, 512),
    ("lin_in fwd pe", "fwdres", 15936, 512, 1216),
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
    ap.add_argument("--variants", default="p3,p4")
    ap.add_argument("--dbg", default="0", help="comma list of asrx_gemm_set_debug flags to time (diagnostics)")
    ap.add_argument("--only", default="", help="comma list of shape names")
    ap.add_argument("--nobias", action="store_true")
    ap.add_argument("--wgrad", default="ws,p4,p3", help="grouped weight-gradient kinds to time")
    ap.add_argument("--nogrouped", action="store_true")
    ap.add_argument("--noblas", action="store_true")
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*s):
        return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()
    variants = args.variants.split(",")
    dbg = [int(x) for x in args.dbg.split(",")]

    def dbg_runs(res, key, fn, base=0):
        for f in dbg:
            K.call("asrx_gemm_set_debug", f | base)
            res[key + ("" if f == 0 else f"/d{f}")] = timeit(fn, args.reps, args.rounds)
        K.call("asrx_gemm_set_debug", 0)

    def kb(v):   # "p3+16": kernel family p3 with debug flags 16 (diagnostic A/B variants of one family)
        k, _, f = v.partition("+")
        return k, int(f or 0)
    for name, kind, M, N, Kd in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        res = {}
        flops = 2.0 * M * N * Kd
        if kind == "fwd":
            x, w = rnd(M, Kd), rnd(N, Kd)
            bias = torch.randn(N, device="cuda", generator=g)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            if not args.noblas:
                res["hipBLASLt"] = timeit(lambda: torch.mm(x, w.t(), out=y), args.reps, args.rounds)
            for v in variants:
                kk, fb = kb(v)
                dbg_runs(res, v, lambda: K.linear(x, w, y, kernel=kk), fb)
                if not args.nobias:
                    K.call("asrx_gemm_set_debug", fb)
                    res[v + "+bias"] = timeit(lambda: K.linear(x, w, y, bias=bias, kernel=kk), args.reps, args.rounds)
                    K.call("asrx_gemm_set_debug", 0)
        elif kind == "dgrad":
            dy, w = rnd(M, N), rnd(N, Kd)
            y = torch.empty(M, Kd, device="cuda", dtype=torch.bfloat16)
            res["hipBLASLt"] = timeit(lambda: torch.mm(dy, w, out=y), args.reps, args.rounds)
            for v in variants + ["ws"]:
                kk, fb = kb(v)
                dbg_runs(res, v, lambda: K.linear_dgrad(dy, w, y, kernel=kk), fb)
        elif kind == "fwdres":
            x, w = rnd(M, Kd), rnd(N, Kd)
            bias = torch.randn(N, device="cuda", generator=g)
            r = torch.randn(M, N, device="cuda", generator=g)
            y = torch.empty(M, N, device="cuda")
            for v in variants + ["ws", "auto"]:
                kk = None if v == "auto" else kb(v)[0]
                res[v] = timeit(lambda: K.linear(x, w, y, bias=bias, resid=r, ld_resid=N, kernel=kk), args.reps,
                                args.rounds)
        elif kind == "fwdepi":
            x, w = rnd(M, Kd), rnd(N, Kd)
            bias = torch.randn(N, device="cuda", generator=g)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            bits = torch.empty(M, N // 32, device="cuda", dtype=torch.int32)
            for v in variants:
                kk, fb = kb(v)
                dbg_runs(res, v, lambda: K.linear(x, w, y, bias=bias, relu=True, dropout_p=0.1, seed=5,
                                                  mask_out=bits, ld_mask=N // 32, kernel=kk), fb)
                K.call("asrx_gemm_set_debug", fb)
                res[v + ":relu"] = timeit(lambda: K.linear(x, w, y, bias=bias, relu=True, kernel=kk), args.reps,
                                          args.rounds)
                res[v + ":relu+drop"] = timeit(lambda: K.linear(x, w, y, bias=bias, relu=True, dropout_p=0.1, seed=5,
                                                                kernel=kk), args.reps, args.rounds)
                res[v + ":relu+mask"] = timeit(lambda: K.linear(x, w, y, bias=bias, relu=True, mask_out=bits,
                                                                ld_mask=N // 32, kernel=kk), args.reps, args.rounds)
                K.call("asrx_gemm_set_debug", 0)
        elif kind == "dgradg":   # out [M, Kd] = dy [M, N] . w [N, Kd], gated by bits of [M, Kd]
            dy, w = rnd(M, N), rnd(N, Kd)
            y = torch.empty(M, Kd, device="cuda", dtype=torch.bfloat16)
            bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (M, Kd // 32), device="cuda", dtype=torch.int32)
            for v in variants:
                kk, fb = kb(v)
                dbg_runs(res, v, lambda: K.linear_dgrad(dy, w, y, alpha=1 / 0.9, gate=bits, ld_gate=Kd // 32,
                                                        gate_bits=True, kernel=kk), fb)
        else:   # wgrad: C[M=N_out, N=K_in] over the Kd rows
            dy, x = rnd(Kd, M), rnd(Kd, N)
            cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            res["hipBLASLt"] = timeit(lambda: torch.mm(dy.t(), x, out=cb), args.reps, args.rounds)
        line = f"{name:11s} M={M:6d} N={N:6d} K={Kd:6d}"
        for v, t in res.items():
            line += f" | {v} {t * 1e6:7.1f}us {flops / t / 1e12:5.0f}TF"
        print(line, flush=True)
    if args.nogrouped:
        return
    # the step's grouped weight-gradient launch over the 12 encoder layers (distinct buffers per layer)
    rows, d, ff = 15936, 512, 2048
    items = []
    for _ in range(12):
        xs, xf = rnd(rows, d), rnd(rows, ff)
        for (n_out, k_in, x) in ((3 * d, d, xs), (d, d, xs), (ff, d, xs), (d, ff, xf)):
            items.append((rnd(rows, n_out), x, torch.zeros(n_out, k_in, device="cuda"),
                          torch.zeros(n_out, device="cuda")))
    flops = sum(2.0 * rows * it[0].shape[1] * it[1].shape[1] for it in items)
    line = f"grouped wgrad, 12 encoder layers ({flops / 1e12:.3f} TFLOP)"
    for v in args.wgrad.split(","):
        kk, fb = kb(v)
        for f in dbg:
            K.call("asrx_gemm_set_debug", f | fb)
            t = timeit(lambda: K.linear_wgrad_grouped(items, beta=0.0, kind=kk), 3, args.rounds)
            line += f" | {v}{'' if f == 0 else f'/d{f}'} {t * 1e6:8.1f}us {flops / t / 1e12:5.0f}TF"
        K.call("asrx_gemm_set_debug", 0)
    print(line, flush=True)


if __name__ == "__main__":
    main()
