#!/bin/bash
# gpurun, retried while the pool has no free box (exit 3: nothing ran, nothing
# charged).  Any other exit code is final.  Usage: tools/gpurun_wait.sh <timeout> <command>
t=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box (try $i), waiting 120 s"
  sleep 120
done
exit 3
