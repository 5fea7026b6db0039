#!/bin/bash
# epilogue A/B: base library vs this tree's — p4 wide GEMMs alone (blas_ref), then the training step (bench, ABBA)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in ab/lib_base.so asr-transformer_amd/asrx/lib/libasrx.so; do
  echo "== $lib"
  ASRX_LIB=$PWD/$lib timeout -k 10 400 python tools/blas_ref.py --only "ffn1 fwd epi,ffn2 dgrad gated,dec ffn1 fwd epi,dec ffn2 dgrad gated,xkv fwd" --variants p4 --nogrouped --noblas --rounds 5 > gpurun_out/r05_epi.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/r05_epi.log; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_lib.sh ab/lib_base.so 2 || exit $?
