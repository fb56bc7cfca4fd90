#!/bin/bash
# (local helper, not run on the GPU box) retry a gpurun call only while the pool reports no box/slot (nothing ran); $1 = log, rest = command
log=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > $log 2>&1
  grep -q "status=transient" $log || break
  sleep 90
done
tail -45 $log | cut -c1-300
