#!/bin/bash
# round-5 baseline on a fresh box: quick bench line + one-step kernel table
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other > gpurun_out/r05_base_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r05_base_bench.log
bash tools/prof_step.sh r05base "ASRX_NONE=0" || exit $?
