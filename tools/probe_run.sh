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
S="fwdr:15936x512x2048,fwdr:15936x512x512,dgradg:15936x2048x512,fwdb:15936x1536x512"
timeout -k 10 400 python tools/gemm_probe.py --shapes $S --variant p3,p3+ASRX_GEMM_DBG=1 > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])"
