#!/bin/bash
# Round-4 batch 26: LayerNorm rows in flight per wave 2 by default — the GPU tests that touch LayerNorm, then a
# same-box step A/B against ASRX_LN_PF=1.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_ln 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train_parity.py tests/test_gpu_model.py tests/test_gpu_fused_adam.py -x -q --timeout 300 --timeout-method thread
bash tools/prof_step.sh b26 ASRX_NONE=0 ASRX_LN_PF=1 || exit $?
