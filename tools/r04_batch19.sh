#!/bin/bash
# Round-4 batch 19: non-temporal conv1 output stores — front-end tests, then same-box step A/B against the previous
# library (asrx/lib/libasrx_prev.so, untracked), both orders.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_fe 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "conv or frontend or front"
P=$PWD/asr-transformer_amd/asrx/lib/libasrx_prev.so
bash tools/prof_step.sh b19 ASRX_NONE=0 ASRX_LIB=$P || exit $?
bash tools/prof_step.sh b19b ASRX_LIB=$P ASRX_NONE=0 || exit $?
