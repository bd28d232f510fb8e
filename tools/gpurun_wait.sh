#!/bin/bash
# Run one gpurun call, re-submitting it only while the pool answers "no box
# or slot free" (exit 3: nothing ran, nothing charged), at most 12 times, 4
# minutes apart.  Any other exit (success, failure, refusal) ends it.
#   tools/gpurun_wait.sh <log> <timeout s> <command>
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  echo "exit $rc" >> $log
  [ $rc -ne 3 ] && exit $rc
  sleep 240
done
exit 3
