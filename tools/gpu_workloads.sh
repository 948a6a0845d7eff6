#!/bin/bash
# Every BASELINE.json workload through bench.py (no CPU baseline), one JSON line each.
set -o pipefail
mkdir -p gpurun_out/workloads
export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c3_qp22 c3_qp27 c3_qp32 c3_qp37 c4}; do
  echo "== $w"
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-mc \
      > gpurun_out/workloads/$w.log 2>&1 || { tail -20 gpurun_out/workloads/$w.log; exit 1; }
  grep '^{' gpurun_out/workloads/$w.log | cut -c1-220
done
