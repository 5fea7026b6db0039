#!/bin/bash
# diagnostics: g4 decomposition (no loads / no epilogue), attention backward phase stamps
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
t() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -30; [ $rc -eq 0 ] || exit $rc; }
t r05_g4_dbg 300 python tools/blas_ref.py --only none --wgrad ws,g4 --dbg 0,8,1,9 --rounds 3
t r05_attn_dbg 300 python tools/attn_bench.py --dbg --only enc
