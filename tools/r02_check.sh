#!/bin/bash
# round-2 GPU check: graph + parity tests, kernel tests, quick bench (stops at the first crash/timeout)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ]; then echo "FATAL: $name rc=$rc"; exit "$rc"; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    graph)  run graph 600 python -u -m pytest tests/test_gpu_graph.py -x -v -s --timeout 300 --timeout-method thread -m gpu ;;
    parity) run parity 900 python -u -m pytest tests/test_gpu_train_parity.py -v -s --timeout 400 --timeout-method thread -m gpu ;;
    kernels) run kernels 900 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu ;;
    gpu)    run gputests 1100 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu ;;
    benchq) run benchq 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    bench)  run bench 900 python bench.py --steps 20 --warmup 5 ;;
    eager)  run eager 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-graph ;;
    prof)   run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
