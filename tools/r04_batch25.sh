#!/bin/bash
# Round-4 batch 25 (configuration only): rows in flight per wave (ASRX_LN_PF) and blocks per CU (ASRX_LN_BPC) of the
# d = 512 LayerNorm kernels, re-measured in the round-4 step.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/prof_step.sh b25 ASRX_NONE=0 ASRX_LN_PF=2 ASRX_LN_BPC=8 ASRX_LN_PF=2,ASRX_LN_BPC=2 || exit $?
