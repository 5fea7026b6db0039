#!/bin/bash
# Round-4 batch 11: the cross-attention keep bits inside its LayerNorm launch (default) — GPU tests of the touched
# paths — then same-box step A/B: default, ASRX_LN_DROPGEN_CROSS=0, and the dropout-hash cost diagnostic
# (ASRX_GEMM_DBG=512: GEMM epilogues without the hash; wrong masks, timing only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_lndg 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "keep_bits or dropout"
step t_model 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train_parity.py -x -q --timeout 300 --timeout-method thread
bash tools/prof_step.sh b11 ASRX_NONE=0 ASRX_LN_DROPGEN_CROSS=0 ASRX_GEMM_DBG=512 || exit $?
