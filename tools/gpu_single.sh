#!/bin/bash
# Single-PU entry points: parity tests (Python + the C++ adapter) and the C++ per-call timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_deep_nn.py tests/test_gpu_sanitize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "single or adapter or nn_pred" > gpurun_out/single_tests.log 2>&1; rc=$?; tail -4 gpurun_out/single_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/single_tests.log; exit $rc; }
$T 120 ./hm16.9-nn_fme_amd/host/test_hm_adapter --time-single 300 | tee gpurun_out/single.log
