"""GEMM probe: A/B kernel families on a ladder of shapes, variants interleaved in rounds in ONE process.

    python tools/gemm_probe.py [--variant p3,p5] [--rounds 7] [--reps 10] [--shapes fwd:15936x1536x512,...]

A variant is a kernel family (ASRX_GEMM_KERNEL) plus optional env settings: "p5+ASRX_GEMM_DBG=1".
Reports the median over rounds of (time of `reps` back-to-back launches) / reps.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402

DEFAULT = ("fwd:15936x1536x512,fwd:2048x1536x512,fwd:15936x2048x512,fwd:15936x512x2048,fwd:15936x512x512,"
           "dgrad:15936x512x1536,dgrad:15936x2048x512,fwd:15936x12288x512,fwd:4096x4096x4096")


def set_env(v):
    parts = v.split("+")
    os.environ["ASRX_GEMM_KERNEL"] = parts[0]
    for key in ("ASRX_GEMM_DBG", "ASRX_P5_XCD", "ASRX_P3_XCD"):
        os.environ.pop(key, None)
    for ev in parts[1:]:
        key, val = ev.split("=")
        os.environ[key] = val


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="p3,p5")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default=DEFAULT)
    args = ap.parse_args()
    variants = args.variant.split(",")
    for spec in args.shapes.split(","):
        kind, dims = spec.split(":")
        M, N, Kd = (int(x) for x in dims.split("x"))
        g = torch.Generator(device="cuda").manual_seed(0)
        if kind in ("wgrad", "wgradp"):   # C[M,N] (+)= A^T B, A = dy [K][M], B = x [K][N]; wgradp: linear_wgrad plan
            a = (torch.rand(Kd, M, device="cuda", generator=g) * 2 - 1).bfloat16()
            w = (torch.rand(Kd, N, device="cuda", generator=g) * 2 - 1).bfloat16()
            y = torch.zeros(M, N, device="cuda")
        else:
            a = (torch.rand(M, Kd, device="cuda", generator=g) * 2 - 1).bfloat16()
        if kind in ("wgrad", "wgradp"):
            pass
        elif kind in ("fwd", "fwdb", "fwdr") or kind.startswith("fwds"):
            w = (torch.rand(N, Kd, device="cuda", generator=g) * 2 - 1).bfloat16()
        else:
            w = (torch.rand(Kd, N, device="cuda", generator=g) * 2 - 1).bfloat16()
        if kind not in ("wgrad", "wgradp"):
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        bg = torch.zeros(M, device="cuda")

        bias = torch.randn(N, device="cuda", generator=g) if kind in ("fwdb", "fwdr") else None
        if kind == "fwdr":      # out-projection / FFN2 epilogue: bias, dropout, fp32 residual add, fp32 out
            resid = torch.randn(M, N, device="cuda", generator=g)
            yf = torch.empty(M, N, device="cuda")
        if kind == "dgradg":    # FFN2 data gradient gated by the ReLU of the hidden activation
            gate = torch.randn(M, N, device="cuda", generator=g).bfloat16()

        def run():
            if kind.startswith("dgrads"):   # dgradsN: data gradient with split-K N
                K.linear_dgrad(a, w, y, splitk=int(kind[6:]))
            elif kind.startswith("fwds"):   # fwdsN: forward with split-K N
                K.linear(a, w, y, splitk=int(kind[4:]))
            elif kind == "fwdb":
                K.linear(a, w, y, bias=bias)
            elif kind == "fwdr":
                K.linear(a, w, yf, bias=bias, dropout_p=0.1, seed=3, resid=resid, ld_resid=N)
            elif kind == "dgradg":
                K.linear_dgrad(a, w, y, gate=gate, ld_gate=N)
            elif kind == "wgradp":
                K.linear_wgrad(a, w, y, bias_grad=bg)
            elif kind == "wgrad":
                K.gemm(a, w, y, M, N, Kd, lda=M, ldb=N, ldc=N, a_trans=True, b_trans=True, beta=1.0, splitk=1)
            elif kind == "fwd":
                K.linear(a, w, y)
            else:
                K.linear_dgrad(a, w, y)
        times = {v: [] for v in variants}
        for r in range(args.rounds + 1):
            for v in variants:
                set_env(v)
                run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.reps):
                    run()
                e.record()
                e.synchronize()
                if r > 0:
                    times[v].append(s.elapsed_time(e) / args.reps * 1e-3)
        line = f"{kind:5s} M={M:6d} N={N:6d} K={Kd:5d}"
        for v in variants:
            t = sorted(times[v])[len(times[v]) // 2]
            line += f" | {v}: {t*1e6:7.1f}us {2.0*M*N*Kd/t/1e12:5.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
