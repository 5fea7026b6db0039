#!/bin/bash
# Round-4 batch 22 (configuration only): the grouped weight-gradient tile layout under the fused optimizer —
# default vs whole groups per XCD (ASRX_WGRAD_PACK=0) vs one table order over all XCDs (ASRX_WGRAD_XCD=0).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/prof_step.sh b22 ASRX_NONE=0 ASRX_WGRAD_PACK=0 ASRX_WGRAD_XCD=0 ASRX_NONE=1 || exit $?
