#!/bin/bash
# Round-closing measurement on one box: GPU tests, smoke, PMC passes (traffic + MFMA, copied into profiles/ so the
# bench line reads them), the full default bench line, the rocprofv3 kernel trace of the graph-mode step and its
# step table, and any step A/Bs given as prof_step.sh variants.
# usage: bash tools/final.sh [--no-tests] [VAR=val[,VAR=val] ...]   (variants: see tools/prof_step.sh; default none)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tests=1
if [ "${1:-}" = "--no-tests" ]; then tests=0; shift; fi
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 8 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
B="python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other"
if [ $tests -eq 1 ]; then
  step gputests 900 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
fi
step pmcf 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- $B
step pmcw 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- $B
step pmctr 120 python3 tools/pmc_traffic.py gpurun_out/pmcf/run_counter_collection.csv gpurun_out/pmcw/run_counter_collection.csv c3 gpurun_out/c3_pmc_traffic.json
step pmcm 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcm -o run --output-format csv -- $B
step pmcmj 120 python3 tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv --out gpurun_out/c3_pmc_mfma.json
cp gpurun_out/c3_pmc_traffic.json gpurun_out/c3_pmc_mfma.json profiles/   # (the bench line below reads them)
step bench 900 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other
step steptab 120 python3 tools/step_table.py gpurun_out/prof/run_kernel_trace.csv
if [ $# -gt 0 ]; then bash tools/prof_step.sh fin ASRX_NONE=0 "$@" || exit $?; fi
