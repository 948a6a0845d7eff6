set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py variants/coop variants/lane --rounds 3 > gpurun_out/ab.log 2>&1; rc=$?; tail -4 gpurun_out/ab.log; exit $rc
