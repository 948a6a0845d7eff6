#!/bin/bash
# Round-5 GPU pass: steps named on the command line, each under its own time limit, the first
# failure ends the call.  Steps: tests, dlab (download-engine A/B), bench, prof (rocprofv3 kernel
# trace of the bench), single.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log" | cut -c1-300; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    newtests) run pytest_new 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    dlab) run dlab 400 python -u tools/download_engine_ab.py 24 ;;
    bench) run bench 400 python -u bench.py --no-pi --no-tz --no-mc ;;
    benchfull) run benchfull 600 python -u bench.py ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pdebug) run pdebug 300 python -u tools/parity_debug.py ;;
    d2h) run d2h 200 ./tools/probes/d2h_kernel_probe ;;
    deepab) run deep_hoist 400 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 && \
            FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/deep_nohoist/libfme_amd.so run deep_nohoist 400 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 ;;
    pbench) run pb3 300 python -u bench.py --no-pi --no-tz --no-mc --cpu-seconds 2 --steps 3 --parity-seconds 4 && \
            run pb20 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20 --parity-seconds 4 && \
            run pb20blit 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20 --parity-seconds 4 --download-engine blit ;;
    occab) run occab 400 python -u tools/ab_bench.py hm16.9-nn_fme_amd hm16.9-nn_fme_amd/variants/s0 hm16.9-nn_fme_amd/variants/w3s0 --rounds 4 ;;
    tzprof) run tzprof 700 bash tools/gpu_tz_prof.sh ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
