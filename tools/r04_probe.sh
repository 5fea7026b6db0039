#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/mfma_probe > gpurun_out/mfma_probe2.log 2>&1; rc=$?
cat gpurun_out/mfma_probe2.log; exit $rc
