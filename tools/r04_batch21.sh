#!/bin/bash
# Round-4 batch 21: the 16-byte-load grouped row reduce (LayerNorm dgamma|dbeta partials) — the tests that check
# those gradients, then same-box step A/B against the scalar kernel (ASRX_RG_VEC=0), both orders.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_rg 900 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_kernels.py tests/test_gpu_fused_adam.py -x -q --timeout 300 --timeout-method thread -k "parity or grads or reduce or layernorm or fused_adam or trainer"
bash tools/prof_step.sh b21 ASRX_NONE=0 ASRX_RG_VEC=0 || exit $?
bash tools/prof_step.sh b21b ASRX_RG_VEC=0 ASRX_NONE=0 || exit $?
