#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k "gemm" --timeout 120 > gpurun_out/gemmtests.log 2>&1; rc=$?
tail -3 gpurun_out/gemmtests.log
[ $rc -ne 0 ] && exit $rc
S="fwd:15936x1536x512,fwd:15936x2048x512,fwd:15936x512x2048,fwd:15936x512x512,dgrad:15936x512x1536,dgrad:15936x2048x512,fwd:15936x12288x512,dgrad:15936x512x12288"
timeout -k 10 400 python tools/gemm_probe.py --shapes $S --variant p3,p3+ASRX_GEMM_DBG=1,p5,p5+ASRX_GEMM_DBG=1,p5m > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
