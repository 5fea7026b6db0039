#!/bin/bash
# Round-4 batch 14: the streamed attention forward for 128 < Lk <= 256 (ASRX_ATTN_STREAM_FWD=1, opt-in) — the
# attention tests under it, the kernel alone both ways, then same-box step A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step t_sfwd 600 env ASRX_ATTN_STREAM_FWD=1 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attention"
step ab_res 300 python tools/attn_bench.py --only enc
step ab_str 300 env ASRX_ATTN_STREAM_FWD=1 python tools/attn_bench.py --only enc
step t_sfwd_par 600 env ASRX_ATTN_STREAM_FWD=1 python -u -m pytest tests/test_gpu_train_parity.py -x -q --timeout 300 --timeout-method thread
bash tools/prof_step.sh b14 ASRX_NONE=0 ASRX_ATTN_STREAM_FWD=1 || exit $?
