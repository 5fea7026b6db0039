#!/bin/bash
# Round-4 batch 17: non-temporal attention output stores (O, its rounding residual, dQ / dK / dV) — attention tests,
# then same-box step A/B against the previous library (asrx/lib/libasrx_prev.so, untracked), both orders.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_attn 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attention"
P=$PWD/asr-transformer_amd/asrx/lib/libasrx_prev.so
bash tools/prof_step.sh b17 ASRX_NONE=0 ASRX_LIB=$P || exit $?
bash tools/prof_step.sh b17b ASRX_LIB=$P ASRX_NONE=0 || exit $?
