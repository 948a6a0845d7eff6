#!/bin/bash
# Round-5 GPU pass: steps named on the command line, each under its own time limit, the first
# failure ends the call.  Steps: tests, dlab (download-engine A/B), bench, prof (rocprofv3 kernel
# trace of the bench), single.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log" | cut -c1-300; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    newtests) run pytest_new 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    dlab) run dlab 400 python -u tools/download_engine_ab.py 24 ;;
    bench) run bench 400 python -u bench.py --no-pi --no-tz --no-mc ;;
    benchfull) run benchfull 600 python -u bench.py ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
