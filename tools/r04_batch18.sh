#!/bin/bash
# Round-4 batch 18 (measurement only): per-shape p4 (256x256 tiles, 8 waves) vs ws (256x128, warp-specialised) on
# the long-K data gradients and the FFN2 forward — does the 256x256 tile's lower staging traffic per FLOP show at
# long K?  (tools/blas_ref.py)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/blas_ref.py --only "xkv dgrad,ffn1 dgrad,qkv dgrad,ffn2 fwd,qkv fwd,ffn1 fwd" --variants "p4,ws" --nogrouped --noblas > gpurun_out/blas_p4ws.log 2>&1
rc=$?; cat gpurun_out/blas_p4ws.log; exit $rc
