#!/bin/bash
# Round-4 batch 6: dQ partials per key block instead of fp32 atomics (long-key attention backward): attention and
# model tests, the c5 attention micro-bench.
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
run t_attn 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "attention or c5 or g64l or long"
run attn_c5 300 python tools/attn_bench.py --only c5,enc,cross
