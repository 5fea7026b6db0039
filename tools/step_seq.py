"""Ordered launch list of ONE steady training step from a rocprofv3 kernel trace: per launch its start offset from
the step's first launch, duration, the idle gap since the previous launch ended, grid and kernel name.

    python tools/step_seq.py gpurun_out/prof/run_kernel_trace.csv [--marker conv1_fwd] [--step -1]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="conv1_fwd", help="kernel-name substring of a step's first launch")
    ap.add_argument("--step", type=int, default=-2, help="which marker-to-marker interval (default: the second last)")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
    pairs = list(zip(starts[:-1], starts[1:]))
    a, b = pairs[args.step]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for i in range(a, b):
        r = rows[i]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        grid = r.get("Grid_Size_X", r.get("Grid_Size", ""))
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f} {(s - prev_end) / 1e3:6.2f}  g{grid:>8}  {r['Kernel_Name'][:110]}")
        prev_end = e
    span = int(rows[b]["Start_Timestamp"]) - t0
    print(f"# {b - a} launches, span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
