#!/bin/bash
# One GPU-box pass: parity tests -> smoke -> bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
[ "${SKIP_TESTS:-0}" = 1 ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${PMC:-1}" = 1 ]; then
  # HBM traffic of the search kernels: FETCH_SIZE and WRITE_SIZE in separate passes
  for c in fetch:FETCH_SIZE write:WRITE_SIZE; do
    run pmc_${c%%:*} 600 rocprofv3 --pmc ${c##*:} --output-format csv -d gpurun_out/pmc_traffic/${c%%:*} -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
  done
  python3 tools/pmc_traffic.py gpurun_out/pmc_traffic gpurun_out/pmc_traffic.json && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
fi
run bench 600 python bench.py --steps "$STEPS" --warmup 3
if [ "${PROFILE:-1}" = 1 ]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pi
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
  cat gpurun_out/kernel_stats.csv | cut -c1-200
fi
echo "== all done"
