#!/bin/bash
# run one gpurun command, retrying only while the pool has no free slot (nothing ran, nothing charged)
# usage: scratch/gpu_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy\|no box or slot free" $out; then sleep 150; continue; fi
  exit $rc
done
exit 3
