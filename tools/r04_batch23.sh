#!/bin/bash
# Round-4 batch 23 (measurement): what the bench's kernel probe (the dominant kernel in a graph segment of its own)
# costs the timed step — bench lines with and without it, alternating on one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other > gpurun_out/b23_probe_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other --no-probe > gpurun_out/b23_noprobe_$i.log 2>&1 || exit $?
done
for f in gpurun_out/b23_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
