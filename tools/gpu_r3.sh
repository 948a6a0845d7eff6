#!/bin/bash
# Round-3 GPU pass: the whole -m gpu suite, the C++ single-PU timing, SQ counters of the search
# kernel.  Each step under its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run single 120 ./hm16.9-nn_fme_amd/host/test_hm_adapter --time-single 300
if [ "${SQ:-1}" = 1 ]; then bash tools/gpu_sq.sh hm16.9-nn_fme_amd/libfme_amd.so; fi
echo "== all done"
