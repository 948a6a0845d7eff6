#!/bin/bash
# Round-6 second-session GPU pass (main10 integer search / producers, C4 parity leg): steps named on
# the command line, each under its own time limit, the first failure ends the call (no retries).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log" | cut -c1-300; exit $rc; fi
}
B="python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline"
for step in "$@"; do
  case $step in
    t2) run t2 300 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tz.py tests/test_main10_producers.py ;;
    smoke) run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    m10legs) run m10legs 400 python -u bench.py --workload c3_qp22_main10 --steps 10 --warmup 3 --no-mc --parity-seconds 10 --cpu-seconds 6 ;;
    m10unstaged) run m10unstaged 400 env FME_TZ10_UNSTAGED=1 python -u bench.py --workload c3_qp22_main10 --steps 10 --warmup 3 --no-mc --no-pi --parity-seconds 0 --no-cpu-baseline ;;
    c4par) run c4par 400 $B --workload c4 --steps 10 --warmup 2 --parity-seconds 60 ;;
    m10tzprof) run m10tzprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/m10tzprof -o run -- python3 bench.py --workload c3_qp22_main10 --no-pi --no-mc --no-cpu-baseline --parity-seconds 0 --steps 5 ;;
    tzprof) run tzprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tzprof -o run -- python3 bench.py --no-pi --no-mc --no-cpu-baseline --parity-seconds 0 --steps 5 ;;
    bench) run bench 400 python -u bench.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
