#!/bin/bash
# Step time of several builds of libasrx.so in one box session, round-robin (order reversed every other round).
# usage: bash tools/ab_multi.sh ROUNDS LIB.so... ("cur" = the in-tree build)
set -u
cd "$(dirname "$0")/.."
rounds=$1; shift
libs=("$@")
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  order=("${libs[@]}")
  if [ $((r % 2)) -eq 0 ]; then order=(); for ((i=${#libs[@]}-1; i>=0; i--)); do order+=("${libs[$i]}"); done; fi
  for v in "${order[@]}"; do
    if [ "$v" = cur ]; then lib=$PWD/asr-transformer_amd/asrx/lib/libasrx.so; else lib=$PWD/$v; fi
    tag=$(basename "$v" .so)
    ASRX_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other \
      > gpurun_out/abm_${tag}_$r.log 2>&1 || exit $?
    echo "$tag $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abm_${tag}_$r.log)"
  done
done
