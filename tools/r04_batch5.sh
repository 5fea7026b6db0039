#!/bin/bash
# Round-4 batch 5: where the one-round ws GEMMs spend their time (diagnostic flags: 1 no epilogue, 8 no operand
# loads, 64 no ring barriers / loaders idle), step profile with the attention OPT and ws8 off (baseline repeat).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit "$rc";; esac
  return 0
}
run blas_decomp 300 python tools/blas_ref.py --only "enc qkv dg512,enc ffn1 dg512,enc out dg512,dec ffn1 dg512,ffn1 fwd epi,ffn2 dgrad gated" \
    --variants ws,ws64,p4 --dbg 0,1,8,9,72,73 --noblas --nogrouped
