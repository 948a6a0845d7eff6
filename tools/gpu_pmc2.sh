#!/bin/bash
# Stall-diagnosis PMC passes (instruction cache, TLB, LDS, memory levels) over a short bench.
set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc2/$name -o run \
      -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc2/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/pmc2/$name.log; echo "pass $name failed rc=$rc"; exit $rc; fi
}
pass f SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS
pass g TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
pass h SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD
pass i SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py gpurun_out/pmc2 > gpurun_out/pmc2/summary.txt && grep -A 40 "k_search_small" gpurun_out/pmc2/summary.txt | head -40
