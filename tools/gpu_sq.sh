#!/bin/bash
# SQ instruction / wait counters of the search kernel for one or more library variants
# (tools/ab_bench.py, one variant per run), summarised per kernel into gpurun_out/sq_<name>.txt.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  n=$(echo "$v" | tr '/.' '__')
  O=gpurun_out/sq_$n
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SMEM --output-format csv -d $O/n -o run -- python tools/ab_bench.py "$v" --rounds 2 --reps 2 > $O.n.log 2>&1 || { tail -20 $O.n.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/o -o run -- python tools/ab_bench.py "$v" --rounds 2 --reps 2 > $O.o.log 2>&1 || { tail -20 $O.o.log; exit 1; }
  python3 tools/pmc_summary.py $O > gpurun_out/sq_$n.txt
  grep -A17 "k_search_lane" gpurun_out/sq_$n.txt
done
