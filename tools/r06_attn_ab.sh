#!/bin/bash
# Round-6 attention A/B: the attention kernel tests on the new build, then tools/attn_bench.py alternating the base
# library (ab/lib_base.so) and the new one (ABBA), then the backward's phase stamps.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "attention" > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
only=${ATTN_ONLY:-enc,cross,dec,c5}
for v in old new new old; do
  if [ $v = old ]; then lib=$PWD/${ATTN_BASE:-ab/lib_base.so}; else lib=$PWD/asr-transformer_amd/asrx/lib/libasrx.so; fi
  ASRX_LIB=$lib timeout -k 10 300 python tools/attn_bench.py --only $only > gpurun_out/attn_$v.log 2>&1 || exit 1
  echo "== $v"; cat gpurun_out/attn_$v.log
done
timeout -k 10 300 python tools/attn_bench.py --dbg --only enc > gpurun_out/stamps_new.log 2>&1 || exit 1
ASRX_LIB=$PWD/ab/lib_base.so timeout -k 10 300 python tools/attn_bench.py --dbg --only enc > gpurun_out/stamps_old.log 2>&1
grep "bwd wave\|chunk" gpurun_out/stamps_new.log | head -20
