#!/bin/bash
# Round-4 batch 12 (diagnostics, timing only): where the p4 / ws K-loops wait — one step under the profiler with no
# operand loads (ASRX_GEMM_DBG=8), no loads and no epilogue (9), no epilogue (1); and the grouped weight gradients
# on p4 tiles (ASRX_WGRAD_KIND=p4) against ws, both without the fused optimizer.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/prof_step.sh b12 ASRX_NONE=0 ASRX_GEMM_DBG=8 ASRX_GEMM_DBG=9 ASRX_GEMM_DBG=1 \
  ASRX_FUSED_ADAM=0 ASRX_FUSED_ADAM=0,ASRX_WGRAD_KIND=p4 || exit $?
