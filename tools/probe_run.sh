#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -m gpu -k "layernorm or reduce_rows or colsum" --timeout 120 > gpurun_out/lntests.log 2>&1; rc=$?
tail -3 gpurun_out/lntests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ln_bench.py --blocks 256,512,1024,2048,4096 > gpurun_out/ln.log 2>&1 || { cat gpurun_out/ln.log; exit 1; }
cat gpurun_out/ln.log
for nb in 512 1024 2048; do
  ASRX_LN_BWD_BLOCKS=$nb timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$nb.log 2>&1 || { tail -5 gpurun_out/bench_$nb.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$nb.log').read().strip().splitlines()[-1]); print('$nb', d['ms_per_step'])"
done
