#!/bin/bash
# Round-2 GPU pass: new async / dist tests first, then the whole -m gpu suite, smoke, bench, rocprof.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -60 "gpurun_out/$name.log"; exit $rc; fi
}
run pytest_new 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dist.py tests/test_deep_nn.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --no-cpu-baseline
run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pi --no-tz --no-mc
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cut -c1-150 gpurun_out/kernel_stats.csv | head -14
echo "== all done"
