#!/bin/bash
# Round-4 batch 24: the cross K/V data gradient on split-K p4 tiles (ASRX_XKV_SPLIT) — accuracy and time alone,
# the model-level parity under it, then same-box step A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step xkv 300 python tools/xkv_check.py
step t_xkv 600 env ASRX_XKV_SPLIT=2 python -u -m pytest tests/test_gpu_train_parity.py -x -q --timeout 300 --timeout-method thread -k "bench_batch"
bash tools/prof_step.sh b24 ASRX_NONE=0 ASRX_XKV_SPLIT=2 ASRX_XKV_SPLIT=3 || exit $?
