#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pm.log 2>&1 || { tail -40 gpurun_out/pm.log; exit 1; }
tail -1 gpurun_out/pm.log
