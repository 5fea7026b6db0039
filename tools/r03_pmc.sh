#!/bin/bash
# PMC passes of the c3 step (eager steps: one dispatch per kernel launch): HBM traffic (FETCH_SIZE, WRITE_SIZE in
# separate passes) and MFMA counters, summarised into gpurun_out/c3_pmc_{traffic,mfma}.json (bench.py reads the
# copies under profiles/).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
B="python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other"
step pmcf 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- $B
step pmcw 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- $B
step pmctr 120 python3 tools/pmc_traffic.py gpurun_out/pmcf/run_counter_collection.csv gpurun_out/pmcw/run_counter_collection.csv c3 gpurun_out/c3_pmc_traffic.json
step pmcm 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcm -o run --output-format csv -- $B
step pmcmj 120 python3 tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv --out gpurun_out/c3_pmc_mfma.json
rm -rf gpurun_out/pmcf gpurun_out/pmcw gpurun_out/pmcm
