#!/bin/bash
# Round-4 A/B of search-kernel variants: each variant's golden parity tests (FME_LIB_PATH), then
# tools/ab_bench.py over all of them in one process (results must be byte-identical).
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
for v in "$@"; do
  FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/$v/libfme_amd.so $T 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden or split or device" > gpurun_out/ab_$(basename $v).log 2>&1
  rc=$?; echo "== $v parity rc=$rc: $(tail -1 gpurun_out/ab_$(basename $v).log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/ab_$(basename $v).log | head -20; exit $rc; }
done
$T 400 python tools/ab_bench.py "$@" --rounds 6 > gpurun_out/ab.log 2>&1; rc=$?; tail -20 gpurun_out/ab.log; exit $rc
