#!/bin/bash
# Round-4 batch 4: MFMA issue-rate probe; the full GPU test suite on the default configuration.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== probe"
timeout -k 10 120 ./tools/mfma_probe > gpurun_out/mfma_probe.log 2>&1; rc=$?
cat gpurun_out/mfma_probe.log; echo "rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
echo "== gpu tests"
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -x \
    > gpurun_out/gputests_b4.log 2>&1; rc=$?
tail -5 gpurun_out/gputests_b4.log; echo "rc=$rc"
exit $rc
