#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python tools/fadam_diag.py > gpurun_out/fadam_diag.log 2>&1; rc=$?
tail -60 gpurun_out/fadam_diag.log; exit $rc
