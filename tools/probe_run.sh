#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
S="wgradp:64x576x302784,dgrad:15936x512x12288,wgradp:256x512x4096"
timeout -k 10 400 python tools/gemm_probe.py --shapes $S --variant auto,p3,reg --rounds 4 --reps 5 > gpurun_out/probe.log 2>&1 || { cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
