#!/bin/bash
# Round-4 GPU pass, steps picked by STEPS (space-separated; default "bench trace"):
#   tests  the parity / async / dist / deep-net GPU tests
#   all    the whole -m gpu suite
#   bench  one headline bench line (no side legs)
#   trace  rocprofv3 kernel trace of the headline bench, steady-launch stats (tools/steady_stats.py)
#   sq     SQ instruction / wait counters of the batch kernels (two passes)
#   pmc    FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json
# Output under gpurun_out/$TAG.  Each step under its own time limit; the first failure ends the call.
set -o pipefail
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "$O/$name.log"; exit $rc; fi
}
B="python bench.py --no-cpu-baseline --no-pi --no-tz --no-mc ${BENCH_ARGS:-}"
for s in ${STEPS:-bench trace}; do
  case $s in
    tests) run tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_dist.py \
             tests/test_deep_nn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    all) run all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run bench 300 $B ;;
    trace)
      run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B --steps 20 --warmup 3
      python3 tools/steady_stats.py $O/trace $O/kernel_stats_steady.csv --skip 3 ;;
    sq)
      run sq_n 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq/n -o run -- $B --steps 2 --warmup 1
      run sq_o 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq/o -o run -- $B --steps 2 --warmup 1
      python3 tools/pmc_summary.py $O/sq > $O/sq_summary.txt ;;
    pmc)
      run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch -o run -- $B --steps 2 --warmup 1
      run pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/write -o run -- $B --steps 2 --warmup 1
      python3 tools/pmc_traffic.py $O/pmc $O/pmc_traffic.json > /dev/null ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== all done"
