#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "layernorm or ln or embedding or cross" > gpurun_out/pt.log 2>&1 || { tail -40 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python tools/ln_bench.py 2>&1 | grep -v amdgpu.ids
