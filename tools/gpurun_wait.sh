#!/bin/bash
# gpurun, retried only while the pool answers "no box / slot free right now" (exit 3: nothing ran,
# nothing charged); any other exit is returned as is.  usage: tools/gpurun_wait.sh LOG TIMEOUT CMD...
log=$1; t=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && { echo "rc=$rc" >> "$log"; exit $rc; }
  sleep 120
done
echo "rc=3 (gave up)" >> "$log"
exit 3
