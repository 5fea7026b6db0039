#!/bin/bash
# Round-4 batch 8: AdamW fused into the grouped weight-gradient launch — tests, step A/B, bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 8 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit "$rc";; esac
  return $rc
}
timeout -k 10 300 python tools/fadam_diag.py > gpurun_out/fadam_diag.log 2>&1; grep -E "losses|differing" gpurun_out/fadam_diag.log
run t_fadam 500 python -u -m pytest tests/test_gpu_fused_adam.py tests/test_gpu_graph.py tests/test_gpu_train_epoch.py \
    -x -q --timeout 300 --timeout-method thread -m gpu || exit 1
bash tools/prof_step.sh b8 ASRX_NONE=0 ASRX_FUSED_ADAM=0 || exit $?
run bench_b8 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other
run dualmb 300 python tools/dualmb_probe.py --reps 10
