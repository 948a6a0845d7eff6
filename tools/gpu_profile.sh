#!/bin/bash
# One round's measurement pass on the GPU box (ROUND=r02 ...): kernel trace + stats of the headline
# bench, HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes), SQ instruction / wait counters,
# then one bench line per BASELINE.json workload.  Every step has its own time limit; the first
# failure ends the call.  Results under gpurun_out/$ROUND/ (copied into profiles/ afterwards).
set -o pipefail
R=${ROUND:-r02}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -2 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -30 "$O/$name.log"; exit $rc; fi
}
B="python bench.py --no-cpu-baseline --no-pi --no-tz --no-mc"
P="python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --no-pcie --parity-seconds 0"   # profiled: kernels alone
if [ "${PROF:-1}" = 1 ]; then
  run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $P --steps 10 --warmup 2
  run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch -o run -- $P --steps 2 --warmup 1
  run pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/write -o run -- $P --steps 2 --warmup 1
  python3 tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json > /dev/null
  run sq_n 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq/n -o run -- $P --steps 2 --warmup 1
  run sq_o 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq/o -o run -- $P --steps 2 --warmup 1
  python3 tools/pmc_summary.py $O/sq > $O/sq_summary.txt
  if [ "${M10:-0}" = 1 ]; then   # the main10 search kernel (k_search_lane10): kernel stats and SQ counters
    run trace10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace10 -o run -- $P --workload c3_qp22_main10 --steps 10 --warmup 2
    run sq10_n 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq10/n -o run -- $P --workload c3_qp22_main10 --steps 2 --warmup 1
    run sq10_o 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq10/o -o run -- $P --workload c3_qp22_main10 --steps 2 --warmup 1
    python3 tools/pmc_summary.py $O/sq10 > $O/sq10_summary.txt
  fi
fi
if [ "${WORKLOADS:-1}" = 1 ]; then
  run bench_c1 300 python bench.py --workload c1 --no-pi --no-tz --no-mc --cpu-seconds 12 --cpu-cores -1
  for w in c2 c3_qp27 c3_qp32 c3_qp37 c3_qp22_main10 c4 c5 c5_exact c5_b4x40; do
    run bench_$w 300 $B --workload $w
  done
fi
echo "== all done"
