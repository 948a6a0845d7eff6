#!/bin/bash
# A/B of the single-call server builds (drop-in latency, C++ through fme_hm::FracSearch):
# the in-tree library against each variants/<name>/libfme_amd.so given, interleaved twice.
# usage: tools/ab_single.sh name...   (output: gpurun_out/ab_single.log)
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
exe=hm16.9-nn_fme_amd/host/test_hm_adapter
# the adapter finds the nets next to the library it loaded
for v in "$@"; do ln -sfn ../../weights hm16.9-nn_fme_amd/variants/$v/weights; done
for rep in 1 2; do
  echo "default: $(timeout -k 10 120 $exe --time-single 300 | tail -1)" | tee -a gpurun_out/ab_single.log
  for v in "$@"; do
    echo "$v: $(LD_LIBRARY_PATH=$PWD/hm16.9-nn_fme_amd/variants/$v timeout -k 10 120 $exe --time-single 300 | tail -1)" \
      | tee -a gpurun_out/ab_single.log
  done
done
