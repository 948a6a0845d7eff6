set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_bench.py variants/cur variants/v5 --rounds 3 > gpurun_out/ab.log 2>&1; rc=$?; tail -3 gpurun_out/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1; rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/rocprof.log; exit $rc; }
cut -c1-150 gpurun_out/prof/run_kernel_stats.csv | head -12
