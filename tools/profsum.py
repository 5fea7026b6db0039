"""Summarise a rocprofv3 kernel_stats.csv: per-kernel totals per step (names as asrx_gemm_kernel_name prints).

    python tools/profsum.py run_kernel_stats.csv STEPS [TOP]
"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'ms/step':>8s} {'%':>6s} {'calls/step':>10s} {'avg_us':>9s}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} {float(r['Percentage']):6.2f} "
          f"{float(r['Calls'])/steps:10.1f} {float(r['AverageNs'])/1e3:9.2f}  {short(r['Name'])[:110]}")
print(f"total {tot/1e6/steps:.3f} ms/step (all kernels incl. warmup/setup launches, divided by {steps:g})")
