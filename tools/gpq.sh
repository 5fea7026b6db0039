#!/bin/bash
# Submit one gpurun command, re-submitting only while gpurun reports that NOTHING ran (exit 3: no box or slot free /
# backing off; or a box lost while being prepared, nothing charged).  A run that started is never repeated.
#   bash tools/gpq.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ "$rc" -eq 3 ] || grep -q "status=transient rc=None charged=0.0s" "$out"; then sleep 60; continue; fi
  echo "rc=$rc" >> "$out"
  exit $rc
done
