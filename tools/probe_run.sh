#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
L=asr-transformer_amd/asrx/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attention or attn" > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for i in 1 2; do
  for v in libasrx_old.so libasrx.so; do
    echo "== $v"
    ASRX_LIB=$L/$v timeout -k 10 300 python tools/attn_bench.py > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/ab.log
  done
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- python3 tools/gemm_probe.py --variant p3 --shapes fwd:15936x1536x512,dgrad:15936x512x1536 --rounds 1 --reps 3 > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pmc.log | grep -v "^W2026\|^E2026" | tail -3
