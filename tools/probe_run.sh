#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k "gemm" --timeout 120 > gpurun_out/gemmtests.log 2>&1; rc=$?
tail -2 gpurun_out/gemmtests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_model.py tests/test_gpu_dist.py -q -x -m gpu --timeout 300 > gpurun_out/modeltests.log 2>&1; rc=$?
tail -2 gpurun_out/modeltests.log
[ $rc -ne 0 ] && exit $rc
b() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub > gpurun_out/bench_$n.log 2>&1 || { tail -5 gpurun_out/bench_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['achieved'])"
}
b p3 ASRX_WGRAD_KIND=p3
b reg ASRX_WGRAD_KIND=reg
b p3noxcd ASRX_WGRAD_KIND=p3 ASRX_WGRAD_XCD=0
b p5 ASRX_WGRAD_KIND=p5
b p3 ASRX_WGRAD_KIND=p3
