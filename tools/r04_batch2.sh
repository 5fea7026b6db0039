#!/bin/bash
# Round-4 batch 2: attention-backward OPT variants (tests, micro-bench), GEMM compute-stream diagnostics, the new
# model family's tests, step profiles (PRER off / attention OPT).  Each GPU step has its own time limit; a fault /
# abort / time-out ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit "$rc";; esac
  return 0
}
run t_attn7 300 env ASRX_ATTN_BWD_OPT=7 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
    --timeout-method thread -m gpu -k "attention"
run t_new 300 python -u -m pytest tests/test_gpu_new_model.py -x -q --timeout 120 --timeout-method thread -m gpu -s
for o in 0 1 2 4 6 7; do
  run attn_o$o 200 env ASRX_ATTN_BWD_OPT=$o python tools/attn_bench.py --only enc,cross
done
run blas_diag 300 python tools/blas_ref.py --only "qkv dgrad,ffn1 dgrad" --variants ws --dbg 0,8,72 --noblas \
    --wgrad ws
bash tools/prof_step.sh b2 ASRX_NONE=0 ASRX_GEMM_DBG=32 ASRX_ATTN_BWD_OPT=7 || exit $?
