#!/bin/bash
# A/B of module constants in one box session: bench step time alternating A / B in ABBA order.
# usage: bash tools/ab_flags.sh ROUNDS "MOD.NAME=VAL[ MOD.NAME=VAL]" "MOD.NAME=VAL[ ...]" [extra bench args]
set -u
cd "$(dirname "$0")/.."
rounds=$1; fa=$2; fb=$3; shift 3
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  if [ $((r % 2)) -eq 1 ]; then order="a b"; else order="b a"; fi
  for v in $order; do
    if [ "$v" = a ]; then f=$fa; else f=$fb; fi
    timeout -k 10 300 python tools/with_flags.py $f -- bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other "$@" \
      > gpurun_out/abf_$v$r.log 2>&1 || exit $?
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abf_$v$r.log)"
  done
done
