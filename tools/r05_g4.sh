#!/bin/bash
# g4 grouped weight gradients + attention backward VALU cut: correctness, then timing
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
t() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
t r05_g4_t1 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "grouped_wgrad and g4" --timeout 120 --timeout-method thread
t r05_att_t 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention" --timeout 120 --timeout-method thread
t r05_g4_t2 400 python -u -m pytest tests/test_gpu_fused_adam.py -x -q --timeout 200 --timeout-method thread
t r05_g4_bench 300 python tools/blas_ref.py --only none --wgrad ws,g4 --rounds 5
cat gpurun_out/r05_g4_bench.log
t r05_attn_bench 300 python tools/attn_bench.py
cat gpurun_out/r05_attn_bench.log | tail -20
