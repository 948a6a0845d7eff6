#!/bin/bash
# Quick GPU pass: parity tests, bench (no CPU baseline), kernel trace, optional SQ counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cut -c1-150 gpurun_out/kernel_stats.csv | head -12
if [ "${SQ:-0}" = 1 ]; then
  mkdir -p gpurun_out/sq
  run sq_n 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sq/n -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
  run sq_o 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/sq/o -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
  python3 tools/pmc_summary.py gpurun_out/sq > gpurun_out/sq/summary.txt 2>&1 || true
fi
echo "== all done"
