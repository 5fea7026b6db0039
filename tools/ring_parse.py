"""Median in-kernel time per (shape, variant) from a rocprofv3 kernel trace of tools/gemm_bench.py."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/profg/run_kernel_trace.csv"
nv = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
rows = list(csv.DictReader(open(path)))
seq = [(r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0],
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows if "gemm_bf16" in r["Kernel_Name"]]
for si in range(len(seq) // (nv * reps)):
    blk = seq[si * nv * reps:(si + 1) * nv * reps]
    line = f"shape{si}"
    for v in range(nv):
        ts = sorted(t for i, (n, t) in enumerate(blk) if i % nv == v)
        line += f" | {blk[v][0][10:42]:32s} {ts[len(ts) // 2]:6.1f}"
    print(line)
