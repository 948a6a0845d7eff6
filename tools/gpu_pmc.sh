#!/bin/bash
# PMC passes over a short bench run (each counter group in its own rocprofv3 pass, kernel
# trace + counters only; no sys/runtime tracing).  Output: gpurun_out/pmc/<pass>/...
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${TAG:-pmc}
pass() {  # name, counters...
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run \
      -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/pmc/$name.log; echo "pass $name failed rc=$rc"; exit $rc; fi
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pass b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
pass c FETCH_SIZE
pass d WRITE_SIZE
pass e SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FP32 SQ_INSTS_VALU_FP64 SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
