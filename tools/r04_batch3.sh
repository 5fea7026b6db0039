#!/bin/bash
# Round-4 batch 3: ws on 8 compute waves (ASRX_WS8) — kernel tests, GEMM micro-bench, step A/B; the new family's
# tests.  Each GPU step has its own time limit; a fault / abort / time-out ends the script.
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
run t_ws8 300 env ASRX_WS8=3 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
    --timeout-method thread -m gpu -k "ws_plain or ws_bias_resid or ws_rowadd or grouped or layouts"
run t_new 300 python -u -m pytest tests/test_gpu_new_model.py -x -q --timeout 120 --timeout-method thread -m gpu -s
run blas_ws8 300 env ASRX_WS8=3 python tools/blas_ref.py --only "enc qkv dg512,enc ffn1 dg512,enc out dg512,dec qkv dg512,dec out dg512,ffn2 fwd res,dec ffn2 fwd res,out fwd res" \
    --variants ws,ws64 --dbg 0,72 --noblas --wgrad ws
run blas_ws4 300 python tools/blas_ref.py --only "enc qkv dg512,enc ffn1 dg512,enc out dg512,dec qkv dg512,dec out dg512,ffn2 fwd res,dec ffn2 fwd res,out fwd res" \
    --variants ws,ws64 --dbg 0,72 --noblas --wgrad ws
bash tools/prof_step.sh b3 ASRX_NONE=0 ASRX_WS8=1 ASRX_WS8=3 || exit $?
run t_par8 600 env ASRX_WS8=3 python -u -m pytest tests/test_gpu_train_parity.py -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "bench_batch"
