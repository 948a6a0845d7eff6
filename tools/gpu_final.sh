#!/bin/bash
# Final GPU pass of a round: the whole -m gpu suite, the C++ single-call timing, smoke(), then the
# measurement pass (kernel trace, PMC traffic, SQ counters, every BASELINE workload) into
# gpurun_out/$ROUND.  Each step under its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run single 120 ./hm16.9-nn_fme_amd/host/test_hm_adapter --time-single 300
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
bash tools/gpu_profile.sh
