#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=asr-transformer_amd/asrx/lib/libasrx.so
for src in asr-transformer_amd/csrc/* include/asrx.h; do
  if [ "$src" -nt "$LIB" ]; then echo "STALE LIBRARY: $src is newer than $LIB"; exit 3; fi
done
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -x -m gpu -k "attention_fused or c5 or c3" --timeout 300 -rf > gpurun_out/t.log 2>&1; rc=$?
tail -4 gpurun_out/t.log
exit $rc
