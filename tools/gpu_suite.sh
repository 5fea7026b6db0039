#!/bin/bash
# GPU-box driver: runs the named steps in order; stops at the first crash/timeout (rc>=124).
# usage: bash tools/gpu_suite.sh step [step ...]
#   kernels | model | smoke | bench | prof | pmc
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
  tail -n 25 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ]; then echo "FATAL: $name rc=$rc — stopping"; exit "$rc"; fi
  return 0
}
# refuse to run with a stale libasrx.so (sources newer than the library)
LIB=asr-transformer_amd/asrx/lib/libasrx.so
for src in asr-transformer_amd/csrc/* include/asrx.h; do
  if [ "$src" -nt "$LIB" ]; then echo "STALE LIBRARY: $src is newer than $LIB"; exit 3; fi
done
for step in "$@"; do
  case "$step" in
    kernels) run kernels 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rf --timeout=400 ;;
    model)   run model 1200 python -m pytest tests/test_gpu_model.py -q -m gpu -rf --timeout=600 ;;
    gpu)     run gputests 1500 python -m pytest tests -q -m gpu -rf --timeout=600 ;;
    smoke)   run smoke 300 python __graft_entry__.py smoke ;;
    bench)   run bench 900 python bench.py --steps 10 --warmup 3 ;;
    benchq)  run benchq 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof)    run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --no-sub --no-other ;;
    pmcf)    run pmcf 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-sub --no-other ;;
    pmcw)    run pmcw 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-sub --no-other ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
