"""Per-kernel table of ONE steady-state training step from a rocprofv3 kernel trace: the launches between two
consecutive optimizer launches (adam_kernel, or adam_spans_kernel when AdamW runs fused into the grouped weight
gradients: one per step), so warm-up and setup launches are excluded.

    python tools/step_table.py gpurun_out/prof/run_kernel_trace.csv [--step -1]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-1, help="which adam-to-adam interval (default: the last)")
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, grid size): separates the shapes")
    ap.add_argument("--marker", default="", help="kernel-name substring that starts a step (default: the optimizer "
                    "launches; the data-parallel step runs several)")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    if args.marker:
        adam = [i - 1 for i, r in enumerate(rows) if args.marker in r["Kernel_Name"] and i > 0]
    else:
        adam = [i for i, r in enumerate(rows)
                if "adam_kernel" in r["Kernel_Name"] or "adam_spans_kernel" in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need two optimizer launches (adam_kernel / adam_spans_kernel) in the trace")
    pairs = list(zip(adam[:-1], adam[1:]))
    a, b = pairs[args.step]
    seg = rows[a + 1:b + 1]
    wall = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3
    agg = collections.defaultdict(list)
    for r in seg:
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
        if args.by_grid:
            n = n[:60] + " g" + "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        agg[n[:80]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    busy = sum(sum(v) for v in agg.values())
    print(f"one step: {len(seg)} launches, {wall / 1e3:.3f} ms adam-to-adam, {busy / 1e3:.3f} ms of kernel time "
          f"(trace timestamps include each launch's boundary)")
    print(f"{'us/step':>9s} {'%':>6s} {'calls':>6s} {'avg_us':>8s}  kernel")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v):9.1f} {100 * sum(v) / busy:6.2f} {len(v):6d} {sum(v) / len(v):8.2f}  {n}")


if __name__ == "__main__":
    main()
