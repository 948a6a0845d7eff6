#!/bin/bash
# A/B of search-kernel variants on the GPU box: the unaligned-load probe, the golden parity tests
# of the built library, then tools/ab_bench.py over the variants given as arguments.
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 60 ./tools/probes/unaligned_probe && \
$T 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_t.log 2>&1; rc=$?; tail -3 gpurun_out/ab_t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/ab_t.log | head -20; exit $rc; }
$T 400 python tools/ab_bench.py "$@" > gpurun_out/ab.log 2>&1; rc=$?; tail -20 gpurun_out/ab.log; exit $rc
