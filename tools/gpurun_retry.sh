#!/bin/bash
# Runs one gpurun call; when the pool has no free box (exit 3) or the lease
# was lost while the box was being prepared (before the command started),
# waits and asks again -- never re-runs a command that ran.
# usage: tools/gpurun_retry.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" $log; then sleep 90; continue; fi
  exit $rc
done
exit 3
