#!/bin/bash
# g4 grouped weight gradients: correctness (grouped + fused AdamW tests), then timing against ws
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "grouped_wgrad and g4" --timeout 120 --timeout-method thread > gpurun_out/r05_g4_t1.log 2>&1; rc=$?; tail -5 gpurun_out/r05_g4_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_adam.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_g4_t2.log 2>&1; rc=$?; tail -5 gpurun_out/r05_g4_t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/blas_ref.py --only none --wgrad ws,g4 --rounds 5 > gpurun_out/r05_g4_bench.log 2>&1; rc=$?; cat gpurun_out/r05_g4_bench.log; exit $rc
