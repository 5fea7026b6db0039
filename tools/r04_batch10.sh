#!/bin/bash
# Round-4 batch 10: the Adam epilogue's load look-ahead and the ws register epilogue (ASRX_WSR) — GPU tests of the
# touched paths, then same-box step A/B: default, look-ahead off (ASRX_GEMM_DBG=256), WSR on.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_fadam 400 python -u -m pytest tests/test_gpu_fused_adam.py -x -q --timeout 300 --timeout-method thread
step t_wsr 400 env ASRX_WSR=1 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ws"
step t_wsrpar 600 env ASRX_WSR=1 python -u -m pytest tests/test_gpu_train_parity.py -x -q --timeout 300 --timeout-method thread -k "bench_batch"
bash tools/prof_step.sh b10 ASRX_NONE=0 ASRX_GEMM_DBG=256 ASRX_WSR=1 || exit $?
bash tools/prof_step.sh b10b ASRX_WSR=1 ASRX_NONE=0 || exit $?
