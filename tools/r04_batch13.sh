#!/bin/bash
# Round-4 batch 13: the paired bf16 epilogue's row-major store order (p3 / p4 / wsp) — GEMM tests, then same-box
# step A/B against the previous commit's library (asrx/lib/libasrx_prev.so, built from HEAD~ by hand, untracked).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_gemm 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or linear or mask"
step t_par 600 python -u -m pytest tests/test_gpu_train_parity.py -x -q --timeout 300 --timeout-method thread
P=$PWD/asr-transformer_amd/asrx/lib/libasrx_prev.so
bash tools/prof_step.sh b13 ASRX_NONE=0 ASRX_LIB=$P ASRX_NONE=1 ASRX_LIB=$P || exit $?
