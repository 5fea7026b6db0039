#!/bin/bash
# Round-4 batch 15: non-temporal GEMM output stores (ASRX_GEMM_DBG=1024) — the GEMM tests under it, then same-box
# step A/B (twice, alternating).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_nt 600 env ASRX_GEMM_DBG=1024 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused_adam.py -x -q --timeout 120 --timeout-method thread -k "gemm or linear or mask or fused_adam"
bash tools/prof_step.sh b15 ASRX_NONE=0 ASRX_GEMM_DBG=1024 || exit $?
bash tools/prof_step.sh b15b ASRX_GEMM_DBG=1024 ASRX_NONE=0 || exit $?
