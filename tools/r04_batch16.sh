#!/bin/bash
# Round-4 batch 16: non-temporal LayerNorm (d = 512) output stores — LayerNorm tests, then same-box step A/B against
# the previous library (asrx/lib/libasrx_prev.so, HEAD built by hand, untracked), both orders.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_ln 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "layernorm or keep_bits"
P=$PWD/asr-transformer_amd/asrx/lib/libasrx_prev.so
bash tools/prof_step.sh b16 ASRX_NONE=0 ASRX_LIB=$P || exit $?
bash tools/prof_step.sh b16b ASRX_LIB=$P ASRX_NONE=0 || exit $?
