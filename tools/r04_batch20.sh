#!/bin/bash
# Round-4 batch 20: fewer LayerNorm-backward blocks (ASRX_LN_BWD_BLOCKS=256: half the dgamma|dbeta partial rows for
# the grouped reduce) — same-box step A/B, both orders.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/prof_step.sh b20 ASRX_NONE=0 ASRX_LN_BWD_BLOCKS=256 || exit $?
bash tools/prof_step.sh b20b ASRX_LN_BWD_BLOCKS=256 ASRX_NONE=0 || exit $?
