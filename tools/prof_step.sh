#!/bin/bash
# Per-kernel table of one steady training step under rocprofv3 for each "VAR=value" setting given (same box):
#   bash tools/prof_step.sh TAG "VAR=a" "VAR=b,VAR2=c" ...   -> gpurun_out/step_TAG_<setting>.txt
# (a setting may join several assignments with commas)
set -u
cd "$(dirname "$0")/.."
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "$@"; do
  t=$(echo "$kv" | tr '=/ ,' '____')
  d=gpurun_out/prof_${tag}_$t
  rm -rf "$d"
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 400 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other > "$d.log" 2>&1 || exit $?
  f=$(find "$d" -name "*kernel_trace.csv" | head -1)
  python3 tools/step_table.py "$f" --marker conv1_fwd > "gpurun_out/step_${tag}_$t.txt"
  python3 tools/step_table.py "$f" --marker conv1_fwd --by-grid > "gpurun_out/stepg_${tag}_$t.txt"
  rm -rf "$d"
  echo "== $kv"; head -3 "gpurun_out/step_${tag}_$t.txt" | tail -2
done
