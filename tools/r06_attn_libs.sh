#!/bin/bash
# tools/attn_bench.py on several libraries in rotation (one box): bash tools/r06_attn_libs.sh ONLY lib1.so lib2.so ...
# (the in-tree build is "cur"); two rounds, the order reversed in the second.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
only=$1; shift
libs=("asr-transformer_amd/asrx/lib/libasrx.so" "$@")
for r in 1 2; do
  if [ $r = 2 ]; then libs=($(printf '%s\n' "${libs[@]}" | tac)); fi
  for lib in "${libs[@]}"; do
    ASRX_LIB=$PWD/$lib timeout -k 10 300 python tools/attn_bench.py --only $only > gpurun_out/al.log 2>&1 || exit 1
    echo "== $(basename $lib) r$r"; grep -v amdgpu.ids gpurun_out/al.log
  done
done
