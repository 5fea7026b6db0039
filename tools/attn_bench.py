"""Attention micro-benchmark on the c3 shapes (B=64, h=8, dh=64): encoder self (249x249), cross (64x249),
decoder self (64x64, causal + padding), forward and backward, dropout 0.1.

    python tools/attn_bench.py [--reps 20] [--only enc,cross,dec] [--variant auto|tiled]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402
from asrx.kernels import MaskSpec  # noqa: E402

B, H, DH = 64, 8, 64
D = H * DH


def case(name, Lq, Lk, causal, kv_width=2 * D, B=B):
    """kv_width: row width of the K/V tensor (2 D = a head's rows 2 KB apart; 12 * 2 D = the model's all-layer cross
    K/V tensor, rows 24 KB apart, this case reading one layer's slice)."""
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B * Lq, D, device="cuda", generator=g).bfloat16()
    kv = torch.randn(B * Lk, kv_width, device="cuda", generator=g).bfloat16()[:, :2 * D]
    o = torch.empty(B * Lq, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B * Lq, D, device="cuda", generator=g).bfloat16()
    dq = torch.empty_like(q)
    if causal:
        valid = torch.ones(B, Lq, device="cuda", dtype=torch.uint8)
        valid[:, Lq - 8:] = 0
        spec = MaskSpec(1, True, valid, valid, valid.stride(0))
    else:
        spec = MaskSpec()
    kw = kv_width
    st = ((D, Lq * D), (kw, Lk * kw), (kw, Lk * kw), (D, Lq * D))
    dkv = torch.empty(B * Lk, kw, device="cuda", dtype=torch.bfloat16)[:, :2 * D]
    gst = ((D, Lq * D), (D, Lq * D), (kw, Lk * kw), (kw, Lk * kw))
    p, seed = 0.1, 77
    dm = K.dropmask_buffer(B, H, Lq, Lk, DH, p, "cuda")
    state = {}

    def fwd():
        state["lse"] = K.attention_fwd(q, kv, kv[:, D:], o, B, H, Lq, Lk, DH, st, D ** -0.5, spec, p, seed,
                                       dropmask=dm)

    def bwd():
        K.attention_bwd(q, kv, kv[:, D:], o, state["lse"], do, dq, dkv, dkv[:, D:], B, H, Lq, Lk, DH, st, gst,
                        D ** -0.5, spec, p, seed, dropmask=dm)

    flops_f = 4.0 * B * H * Lq * Lk * DH
    return name, fwd, bwd, flops_f, 2.5 * flops_f


def timeit(fn, reps):
    """ms per call: reps calls captured in a HIP graph and replayed (no host launch gaps)."""
    sys.path.insert(0, REPO)
    from bench import _graph_time_ms
    return _graph_time_ms([fn], launches=reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="enc,cross,dec")
    ap.add_argument("--variant", default="auto")
    ap.add_argument("--batch", type=int, default=B, help="batch size of the c3 cases (default 64)")
    ap.add_argument("--sweep", action="store_true", help="Lq sweep at Lk=249 (per-chunk vs fixed cost)")
    ap.add_argument("--dbg", action="store_true", help="phase timestamps (a diagnostic build: ASRX_CFLAGS=-DASRX_ATTN_STAMPS)")
    ap.add_argument("--exp", default="", help="comma list of ASRX_ATTN_EXP values for the backward (a diagnostic "
                    "build's timing-only switches, wrong results: 1 no loop barrier, 2 no chunk fetch, 4 no dQ sweep, "
                    "8 no dV/dK MFMAs)")
    ap.add_argument("--exp-fwd", action="store_true", help="--exp sweeps the forward instead (1 no K/V wait, 2 no "
                    "output stores, 4 no v_exp, 8 no PV MFMAs, 16 no QK MFMAs)")
    args = ap.parse_args()
    os.environ["ASRX_ATTN_KERNEL"] = args.variant
    bb = args.batch
    cases = {"enc": ("enc_self", 249, 249, False, 2 * D, bb), "cross": ("cross", 64, 249, False, 2 * D, bb),
             "cross24k": ("cross24k", 64, 249, False, 12 * 2 * D, bb), "dec": ("dec_self", 64, 64, True, 2 * D, bb),
             "c5": ("c5_self", 999, 999, False, 2 * D, 16)}   # c5: B = 16, T' = 999 (the streamed kernels)
    if args.sweep:
        for lq in (32, 64, 128, 192, 249):
            cases[f"s{lq}"] = (f"lq{lq}", lq, 249, False)
        args.only = ",".join(k for k in cases if k.startswith("s"))
    if args.dbg:
        import ctypes
        os.environ["ASRX_ATTN_DBG"] = "1"   # read once, at the library's first attention call
        from asrx._lib import lib
        for key in args.only.split(","):
            name, fwd, bwd, ff, fb = case(*cases[key])
            fwd()
            bwd()
            torch.cuda.synchronize()
            fwd()
            bwd()
            torch.cuda.synchronize()
            nb = bb * H
            buf = (ctypes.c_ulonglong * (128 + 8 * 1024))()
            lib().asrx_attn_debug_read(buf, 128 + 8 * 1024)
            ts = list(buf)
            pc = lambda v: [int(sorted(v)[int(q * (len(v) - 1))]) for q in (0, .1, .5, .9, 1)]   # noqa: E731
            bw = [ts[128 + 4096 + 4 * i:132 + 4096 + 4 * i] for i in range(nb)]
            if bw[0][0]:
                t0b = min(x[0] for x in bw)
                print(name, "bwd per-block (10 ns ticks; pct 0/10/50/90/100): start", pc([x[0] - t0b for x in bw]),
                      " total", pc([x[2] - x[0] for x in bw]), " end", pc([x[2] - t0b for x in bw]),
                      " distinct CUs", len(set(x[3] for x in bw)))
                srt = sorted(bw, key=lambda x: x[0])
                print("   bwd start ticks of blocks 240..272 by start order:", [x[0] - t0b for x in srt[240:272]])
            blk = [ts[128 + 4 * i:132 + 4 * i] for i in range(nb)]
            t00 = min(x[0] for x in blk)
            print(name, "fwd per-block (10 ns ticks; pct 0/10/50/90/100): start", pc([x[0] - t00 for x in blk]),
                  " staged", pc([x[1] - x[0] for x in blk]), " total", pc([x[2] - x[0] for x in blk]),
                  " end", pc([x[2] - t00 for x in blk]), " distinct CUs", len(set(x[3] for x in blk)))
            from collections import Counter
            per = Counter(x[3] for x in blk)
            late = [x for x in blk if x[0] - t00 > 200]
            print("   blocks per CU id:", sorted(Counter(per.values()).items()), " late starters:", len(late),
                  " late per CU count:", sorted(Counter(per[x[3]] for x in late).items()),
                  " late bh ids:", [i for i, x in enumerate(blk) if x[0] - t00 > 200][:24])
            f0 = ts[44]
            if f0:
                print(name, "fwd: staging-issued", ts[45] - f0, " barrier", ts[46] - f0,
                      " tiles", [ts[47 + k] - f0 for k in range(8) if ts[47 + k] >= f0], " end", ts[55] - f0)
            for wv, base in ((0, 0), (4, 64)):
                t0 = ts[base]
                print(name, f"bwd wave {wv}: prologue", ts[base + 1] - t0, "cycles")
                for ch in range(8):
                    a, b, c, d = ts[base + 2 + 4 * ch:base + 6 + 4 * ch]
                    if a == 0 or a < t0:
                        break
                    print(f"  chunk {ch}: fetch-issued {a - t0:7d}  compute {b - a:6d}  publish {d - b:6d}  "
                          f"barrier {c - d:6d}")
        return
    if args.exp:
        for key in args.only.split(","):
            name, fwd, bwd, ff, fb = case(*cases[key])
            fwd()
            for e in args.exp.split(","):
                os.environ["ASRX_ATTN_EXP"] = e
                tb = timeit(fwd if args.exp_fwd else bwd, args.reps)
                print(f"{name:9s} exp {e:>3s} {'fwd' if args.exp_fwd else 'bwd'} {tb*1e3:7.1f}us", flush=True)
            os.environ.pop("ASRX_ATTN_EXP", None)
        return
    for key in args.only.split(","):
        name, fwd, bwd, ff, fb = case(*cases[key])
        fwd()
        tf = timeit(fwd, args.reps)
        tb = timeit(bwd, args.reps)   # includes the delta prologue kernel
        print(f"{name:9s} fwd {tf*1e3:7.1f}us {ff/tf/1e9:6.0f}TF | bwd {tb*1e3:7.1f}us {fb/tb/1e9:6.0f}TF "
              f"(bwd counted as 2.5x fwd FLOPs)", flush=True)


if __name__ == "__main__":
    main()
