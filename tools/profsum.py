"""Summarise a rocprofv3 kernel_stats.csv: per-kernel totals per step."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r["Name"].replace("(anonymous namespace)::", "")[:95]
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f}ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step={float(r['Calls'])/steps:7.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {n}")
print(f"total {tot/1e6/steps:.3f} ms/step")
