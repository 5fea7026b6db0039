#!/bin/bash
# A/B of two builds of libasrx.so in one box session: bench step time alternating OLD / NEW (ASRX_LIB), in
# ABBA order per pair of rounds (the second run of a back-to-back pair runs on a warmer card, ~0.05 ms slower).
# usage: bash tools/ab_lib.sh OLD.so [rounds] [extra bench args]
set -u
cd "$(dirname "$0")/.."
old=$1; rounds=${2:-2}; shift 2 || true
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  if [ $((r % 2)) -eq 1 ]; then order="old new"; else order="new old"; fi
  for v in $order; do
    if [ "$v" = old ]; then lib=$PWD/$old; else lib=$PWD/asr-transformer_amd/asrx/lib/libasrx.so; fi
    ASRX_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other "$@" \
      > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v$r.log)"
  done
done
