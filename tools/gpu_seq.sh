#!/bin/bash
# Runs GPU steps in order, each "name|seconds|command" under its own time limit, output in
# gpurun_out/<name>.log.  A step that exits 0 or 1 (pytest: tests failed) lets the next one run;
# anything else (a fault, an abort, a time limit) ends the call there.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -4 "gpurun_out/$name.log" | cut -c1-400
  echo "== $name rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
