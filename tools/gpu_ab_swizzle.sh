set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_bench.py variants/noswz variants/swz --rounds 3 > gpurun_out/ab.log 2>&1 && tail -4 gpurun_out/ab.log &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in noswz swz; do
  FME_LIB_PATH=hm16.9-nn_fme_amd/variants/$v/libfme_amd.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$v/fetch -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || exit 1
  python3 tools/pmc_traffic.py gpurun_out/pmc_$v gpurun_out/pmc_$v.json | grep -A3 search_small
done
