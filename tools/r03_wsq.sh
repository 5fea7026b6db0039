#!/bin/bash
# wsgq check: grouped / parity / graph tests, per-tile trace, one-step kernel table, PMC traffic of the step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step wsq_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "grouped or wgrad" tests/test_gpu_train_parity.py tests/test_gpu_graph.py
step wsq_trace 300 python tools/ws_trace.py
step wsq_prof 400 bash tools/prof_step.sh wsq X=1
B="python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other"
step wsq_pmcf 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/wpmcf -o run --output-format csv -- $B
step wsq_pmcw 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wpmcw -o run --output-format csv -- $B
step wsq_pmctr 120 python3 tools/pmc_traffic.py gpurun_out/wpmcf/run_counter_collection.csv gpurun_out/wpmcw/run_counter_collection.csv c3 gpurun_out/wsq_pmc_traffic.json
grep -A3 wsgq gpurun_out/wsq_pmc_traffic.json | head -5
rm -rf gpurun_out/wpmcf gpurun_out/wpmcw
