#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=asr-transformer_amd/asrx/lib/libasrx.so
for src in asr-transformer_amd/csrc/* include/asrx.h; do
  if [ "$src" -nt "$LIB" ]; then echo "STALE LIBRARY: $src is newer than $LIB"; exit 3; fi
done
timeout -k 10 900 python -m pytest tests -q -x -m gpu --timeout 300 > gpurun_out/t.log 2>&1; rc=$?
tail -2 gpurun_out/t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"
