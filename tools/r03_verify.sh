#!/bin/bash
# round-3 re-entry verification on one box: GPU tests, smoke, the default bench line (PMC / trace passes: r03_final.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 8 "gpurun_out/$name.log"; [ "$rc" -eq 0 ] || exit "$rc"; }
step gputests 600 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python bench.py
