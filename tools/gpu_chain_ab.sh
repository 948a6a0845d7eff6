#!/bin/bash
# Producer-chain variants: the P-frame probe (tools/pred_inter_probe.py) per library, each after its
# producer parity tests (tests/test_pred_inter.py, tests/test_pred_inter_b.py -m gpu).
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=$PWD/hm16.9-nn_fme_amd/$v/libfme_amd.so
  FME_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_pred_inter.py tests/test_pred_inter_b.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/chain_ab_$(basename $v).log 2>&1
  rc=$?; echo "== $v parity rc=$rc: $(tail -1 gpurun_out/chain_ab_$(basename $v).log)"
  [ $rc -eq 0 ] || exit $rc
  FME_LIB_PATH=$lib timeout -k 10 200 python tools/pred_inter_probe.py 3 2>&1 | grep pred_inter || exit 1
done
