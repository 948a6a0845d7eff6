#!/bin/bash
# A/B of library variants (tools/ab_bench.py: same inputs, one process, results must be
# byte-identical), then the GPU parity tests on the in-tree library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_bench.py "$@" > gpurun_out/ab.log 2>&1; rc=$?; tail -12 gpurun_out/ab.log; [ $rc -eq 0 ] || exit $rc
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== all done"
