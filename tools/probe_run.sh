#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=asr-transformer_amd/asrx/lib/libasrx.so
for src in asr-transformer_amd/csrc/* include/asrx.h; do
  if [ "$src" -nt "$LIB" ]; then echo "STALE LIBRARY: $src is newer than $LIB"; exit 3; fi
done
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k "gemm" --timeout 120 > gpurun_out/gemmtests.log 2>&1; rc=$?
tail -2 gpurun_out/gemmtests.log
[ $rc -ne 0 ] && exit $rc
S="fwdb:15936x1536x512,fwdb:15936x2048x512,fwdr:15936x512x2048,dgrad:15936x512x1536,dgradg:15936x2048x512,wgrad:12288x512x15936"
timeout -k 10 400 python tools/gemm_probe.py --shapes $S --variant p3,p3+ASRX_GEMM_DBG=4 > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
