#!/bin/bash
# Memory-pipeline PMC passes (TA/TD/TCP/TCC) over a short bench; one counter group per pass.
set -o pipefail
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc3/$name -o run \
      -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc3/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/pmc3/$name.log; echo "pass $name failed rc=$rc"; exit $rc; fi
}
pass j TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES
pass j2 TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY
pass k TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY
pass k2 TCP_TOTAL_CACHE_ACCESSES TCP_CACHE_MISS
pass l TCC_HIT TCC_MISS TCC_TAG_STALL TCC_REQ
pass n SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
pass o SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
python3 tools/pmc_summary.py gpurun_out/pmc3 > gpurun_out/pmc3/summary.txt && grep -A 40 "k_search_small" gpurun_out/pmc3/summary.txt | head -40
