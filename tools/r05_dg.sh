#!/bin/bash
# keep-bit transpose in registers + conv1-gradient two-item lookahead: tests, front-end alone (base vs new), then
# the step A/B against ab/lib_base.so (the previous commit)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "attention or attn or dropout or drop or conv or frontend" > gpurun_out/dg_t.log 2>&1; rc=$?; tail -2 gpurun_out/dg_t.log; [ $rc -eq 0 ] || exit $rc
for lib in ab/lib_base.so asr-transformer_amd/asrx/lib/libasrx.so; do echo "== $lib"; ASRX_LIB=$PWD/$lib timeout -k 10 200 python tools/fe_bench.py --only conv_bwd_implicit > gpurun_out/dg_f.log 2>&1 || exit $?; grep -v amdgpu.ids gpurun_out/dg_f.log; done
bash tools/prof_step.sh dg ASRX_NONE=0 || exit $?
grep "ln_dropgen\|attn_dropgen\|conv_bwd" gpurun_out/stepg_dg_ASRX_NONE_0.txt
bash tools/ab_lib.sh ab/lib_base.so 2 || exit $?
