#!/bin/bash
# round-2 probes: library GEMM ceiling, counter list, kernel stats of the graph-mode step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 40 "gpurun_out/$name.log"; [ "$rc" -lt 124 ] || exit "$rc"; }
for s in "$@"; do
  case "$s" in
    blas) step blas 300 python tools/blas_ref.py ;;
    counters) step counters 120 rocprofv3 -L ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub ;;
    pmcm) step pmcm 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcm -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub && python3 tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv --out gpurun_out/c3_pmc_mfma.json ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
