#!/bin/bash
# Round-4: the data-parallel path on one GPU (one-rank RCCL group, ASRX_DP_REHEARSE=1: bucketed all-reduce, early
# AdamW on the side stream, the fused optimizer off) — the GPU DP tests and a short bench line, both fp32 and bf16 wire.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_dist 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread
step dp_bench 600 env ASRX_DP_REHEARSE=1 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-sub --no-other
grep '^{"metric"' gpurun_out/dp_bench.log > gpurun_out/r04_dp_rehearsal_bench.json
