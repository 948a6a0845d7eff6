#!/bin/bash
# SQ counter passes over a short bench (per-kernel instruction mix, wave cycles, waits).
set -o pipefail
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "== pass $name"
  timeout -k 10 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/sq/$name -o run \
      -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/sq/$name.log; echo "pass $name failed rc=$rc"; exit $rc; fi
}
pass n SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE
pass o SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
if [ "${MEM:-0}" = 1 ]; then
  pass j TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES
  pass j2 TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY
  pass k TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY
  pass l TCC_HIT TCC_MISS TCC_TAG_STALL TCC_REQ
fi
python3 tools/pmc_summary.py gpurun_out/sq > gpurun_out/sq/summary.txt
grep -A 30 "^fme::$" gpurun_out/sq/summary.txt
