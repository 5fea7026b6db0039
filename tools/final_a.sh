#!/bin/bash
# Round-closing measurement, part A (fits one gpurun call): PMC passes (traffic + MFMA, copied into profiles/ so
# the bench line reads them), then the full default bench line.  Part B: tools/final_b.sh.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
B="python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other"
step pmcf 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- $B
step pmcw 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- $B
step pmctr 120 python3 tools/pmc_traffic.py gpurun_out/pmcf/run_counter_collection.csv gpurun_out/pmcw/run_counter_collection.csv c3 gpurun_out/c3_pmc_traffic.json
step pmcm 200 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcm -o run --output-format csv -- $B
step pmcmj 120 python3 tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv --out gpurun_out/c3_pmc_mfma.json
cp gpurun_out/c3_pmc_traffic.json gpurun_out/c3_pmc_mfma.json profiles/
step bench 600 python bench.py
cat gpurun_out/bench.log | grep '^{' > gpurun_out/bench_line.json
