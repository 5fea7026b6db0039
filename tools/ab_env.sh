#!/bin/bash
# Step-time A/B of environment switches in one box session: bench.py alternating over "VAR=value" settings.
# usage: bash tools/ab_env.sh ROUNDS "VAR=a" "VAR=b,VAR2=c" ...   (a setting may join several assignments with commas)
set -u
cd "$(dirname "$0")/.."
rounds=$1; shift
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for kv in "$@"; do
    tag=$(echo "$kv" | tr '=/ ,' '____')
    env $(echo "$kv" | tr "," " ") timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other \
      > "gpurun_out/abenv_${tag}_$r.log" 2>&1 || exit $?
    echo "$kv $r $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/abenv_${tag}_$r.log")"
  done
done
