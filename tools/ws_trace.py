"""Per-tile timeline (slot of the block -> tile map; the persistent queue kernel or one workgroup per tile) of the grouped weight-gradient launch (gemm_bf16_wsg_kernel) of one eager c3 training step:
which XCD / CU ran each tile, when, and how far apart the tiles of each 32-tile round started and ended (they
share operand panels through their XCD's L2 only while they run together).

    python tools/ws_trace.py
"""
import collections
import ctypes
import os
import sys

os.environ["ASRX_GEMM_DBG"] = "128"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    import asrx
    from asrx._lib import lib
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
    for _ in range(3):
        tr.step(s, t, k)
    torch.cuda.synchronize()
    n = 8192
    buf = (ctypes.c_ulonglong * (4 * n))()
    assert lib().asrx_ws_trace_read(buf, 4 * n) == 0
    rows = []
    for b in range(n):
        t0, t1, w2, w3 = buf[4 * b:4 * b + 4]
        if t0 == 0:
            continue
        rows.append(dict(b=b, t0=t0, t1=t1, xcc=w2 & 15, rs=(w2 >> 7) & 1, cu=(w2 >> 8) & 0xffffff, tile=w2 >> 32, k=w3 & 0xffffffff,
                         g=(w3 >> 32) & 0xffff, wg=w3 >> 48))
    tmin = min(r["t0"] for r in rows)
    tmax = max(r["t1"] for r in rows)
    print(f"blocks traced {len(rows)}, launch span {(tmax - tmin) / 100:.1f} us (10 ns ticks)")
    bad = sum(1 for r in rows if r["xcc"] != r["wg"] % 8)
    print(f"tiles whose XCD != workgroup % 8: {bad}; slots run on another XCD than slot % 8: "
          f"{sum(1 for r in rows if r['xcc'] != r['b'] % 8)}")
    per_x = collections.defaultdict(list)
    for r in rows:
        per_x[r["xcc"]].append(r)
    for x in sorted(per_x):
        rs = sorted(per_x[x], key=lambda r: r["t0"])
        busy = sum(r["t1"] - r["t0"] for r in rs) / 100
        end = (max(r["t1"] for r in rs) - tmin) / 100
        print(f"XCD {x}: {len(rs)} blocks, busy {busy / 32:.1f} us per CU, last end {end:.1f} us")
    # tile durations by reduction length, with / without the fused bias-gradient row sums (loader waves)
    for kk in sorted(set(r["k"] for r in rows)):
        for rs in (0, 1):
            du = sorted((r["t1"] - r["t0"]) / 100 for r in rows if r["k"] == kk and r["rs"] == rs)
            if du:
                print(f"k {kk} row-sum tile {rs}: {len(du)} tiles, duration p10 {du[len(du) // 10]:.1f} "
                      f"p50 {du[len(du) // 2]:.1f} p90 {du[9 * len(du) // 10]:.1f} us")
    # rounds: consecutive 32 blocks of an XCD in block order
    print("per-XCD rounds (32 consecutive blocks of one XCD): group set, k, start spread, end spread, duration p50")
    for x in sorted(per_x):
        rs = sorted(per_x[x], key=lambda r: r["b"])
        for i in range(0, len(rs), 32):
            rd = rs[i:i + 32]
            st = sorted((r["t0"] - tmin) / 100 for r in rd)
            en = sorted((r["t1"] - tmin) / 100 for r in rd)
            du = sorted((r["t1"] - r["t0"]) / 100 for r in rd)
            gs = sorted(set(r["g"] for r in rd))
            ks = sorted(set(r["k"] for r in rd))
            print(f"  x{x} r{i // 32}: groups {gs} k {ks} start {st[0]:7.1f}..{st[-1]:7.1f}  end {en[0]:7.1f}..{en[-1]:7.1f}"
                  f"  dur p50 {du[len(du) // 2]:6.1f} max {du[-1]:6.1f}")


if __name__ == "__main__":
    main()
