#!/bin/bash
# Round-4 batch 7: the cross-attention backward as two 128-key blocks (ASRX_ATTN_XSPLIT): tests, micro-bench, step A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit "$rc";; esac
  return 0
}
run t_xsplit 400 env ASRX_ATTN_XSPLIT=1 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train_parity.py -x -q \
    --timeout 300 --timeout-method thread -m gpu -k "attention or g64 or bench_batch"
run attn_x0 200 python tools/attn_bench.py --only cross,cross24k
run attn_x1 200 env ASRX_ATTN_XSPLIT=1 python tools/attn_bench.py --only cross,cross24k
bash tools/prof_step.sh b7 ASRX_NONE=0 ASRX_ATTN_XSPLIT=1 || exit $?
