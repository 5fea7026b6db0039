#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "mask or epilogue or gemm_layouts" > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pm.log 2>&1 || { tail -40 gpurun_out/pm.log; exit 1; }
tail -1 gpurun_out/pm.log
for v in 0 1 0 1; do
  ASRX_GATE_BITS=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-sub > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  echo "bits=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe --no-sub > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
python3 tools/profsum.py gpurun_out/prof_q/run_kernel_stats.csv 7 30
