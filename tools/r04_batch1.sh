#!/bin/bash
# Round-4 batch on one box: the new kernels' tests, the new model family's tests, GEMM epilogue microbench, attention
# backward phase stamps, step profiles with / without wse, one bench line.  Each GPU step has its own time limit; a
# fault / abort / time-out ends the script (no further GPU step).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit "$rc";; esac
  return $rc
}
run t_wse 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu \
    -k "wse or relu_mask or zero_spans or wsp or ws_bias_resid or ws_rowadd"
run t_new 300 python -u -m pytest tests/test_gpu_new_model.py -x -q --timeout 120 --timeout-method thread -m gpu -s
run blas_wse 300 python tools/blas_ref.py --only "ffn1 fwd epi,ffn2 dgrad gated,qkv fwd,xkv fwd" --variants p4,wse \
    --dbg 0,1 --nogrouped --noblas
run attn_dbg 200 python tools/attn_bench.py --dbg --only enc,cross
bash tools/prof_step.sh w1 ASRX_WSE=1 ASRX_WSE=0 || exit $?
run bench_w1 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
