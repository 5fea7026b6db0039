#!/bin/bash
# Round-4 batch 9: fused AdamW step A/B (same box), twice in alternation.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/prof_step.sh b9a ASRX_NONE=0 ASRX_FUSED_ADAM=0 || exit $?
bash tools/prof_step.sh b9b ASRX_NONE=0 ASRX_FUSED_ADAM=0 || exit $?
