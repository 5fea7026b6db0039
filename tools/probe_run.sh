#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "tallk or conv_frontend or wgrad or frontend" > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fe -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-sub > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log
f=$(find gpurun_out/prof_fe -name '*kernel_stats.csv' | head -1)
grep -i "conv1\|tallk\|im2col\|reduce\|gemm_bf16_kernel<64" "$f" | cut -d, -f1-4
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pm.log 2>&1 || { tail -40 gpurun_out/pm.log; exit 1; }
tail -2 gpurun_out/pm.log
