#!/bin/bash
# Round-closing measurement, part B: rocprofv3 kernel trace + stats of the graph-mode step and its step tables.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other
step steptab 120 python3 tools/step_table.py gpurun_out/prof/run_kernel_trace.csv --marker conv1_fwd
step steptabg 120 python3 tools/step_table.py gpurun_out/prof/run_kernel_trace.csv --marker conv1_fwd --by-grid
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv
