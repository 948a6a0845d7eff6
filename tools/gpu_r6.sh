#!/bin/bash
# Round-6 GPU pass: steps named on the command line, each under its own time limit, the first
# failure ends the call (no retries).  Output under gpurun_out/<name>.log.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "== $name FAILED rc=$rc"; tail -40 "gpurun_out/$name.log" | cut -c1-300; exit $rc; fi
}
B="python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline"
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    replaytests) run replaytests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_c4.py tests/test_gpu_main10.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    pipeab) run p_default 200 $B --steps 20 --parity-seconds 10 && \
            run p_2streams 200 $B --steps 20 --parity-seconds 0 --copy-streams 2 && \
            run p_unpacked 200 $B --steps 20 --parity-seconds 0 --no-packed && \
            run p_blit 200 $B --steps 20 --parity-seconds 0 --download-engine blit && \
            run p_c1 200 $B --steps 20 --parity-seconds 5 --workload c1 ;;
    m10) run m10tests 300 python -u -m pytest tests/test_gpu_main10.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread && \
         run m10bench 300 $B --workload c3_qp22_main10 --steps 10 --parity-seconds 10 ;;
    stall) run s_c3 200 $B --steps 20 --parity-seconds 0 && run s_c1 200 $B --steps 20 --parity-seconds 0 --workload c1 ;;
    tztests) run tztests 400 python -u -m pytest tests/test_gpu_tz.py tests/test_ring.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    stamps) run lane_stamps 200 python -u tools/lane_stamps.py 5 ;;
    pkab) run pkab 300 python -u tools/ab_bench.py . variants/pk16 --rounds 4 ;;
    ordab) run ordab 300 python -u tools/ab_bench.py . variants/ord1 variants/ord2 --rounds 4 ;;
    pfab) run pfab 300 python -u tools/ab_bench.py . variants/pf --rounds 5 ;;
    u44ab) run u44ab 300 python -u tools/ab_bench.py . variants/u44 --rounds 4 ;;
    pipe2) run q_c3 200 $B --steps 20 --parity-seconds 10 && run q_c3_ma0 200 $B --steps 20 --parity-seconds 0 --max-ahead 0 && \
           run q_c3_ma2 200 $B --steps 20 --parity-seconds 0 --max-ahead 2 && run q_c3_blit 200 $B --steps 20 --parity-seconds 0 --download-engine blit && \
           run q_c1 200 $B --workload c1 --steps 20 --parity-seconds 5 && run q_c1_blit 200 $B --workload c1 --steps 20 --parity-seconds 0 --download-engine blit ;;
    pipe3) run r_c3 200 $B --steps 20 --parity-seconds 5 && run r_c3_ma0 200 $B --steps 20 --parity-seconds 0 --max-ahead 0 && \
           run r_c3_lazy 200 $B --steps 20 --parity-seconds 0 --lazy-events && \
           run r_c1 200 $B --workload c1 --steps 20 --parity-seconds 5 && run r_c1_ma0 200 $B --workload c1 --steps 20 --parity-seconds 0 --max-ahead 0 ;;
    envab) for e in "NONE=1" "ROC_SIGNAL_POOL_SIZE=4096" "ROC_AQL_QUEUE_SIZE=65536" "AMD_DIRECT_DISPATCH=0" \
                    "HSA_KERNARG_POOL_SIZE=67108864" "GPU_MAX_HW_QUEUES=8" "HSA_ENABLE_SDMA=0" "ROC_CPU_WAIT_FOR_SIGNAL=0" \
                    "DEBUG_CLR_MAX_BATCH_SIZE=100000" "GPU_NUM_MEM_DEPENDENCY=4096"; do
             run "env_${e%%=*}" 200 env "$e" $B --steps 30 --parity-seconds 0 || exit 1
           done ;;
    pipe4) run t_2str 200 $B --steps 30 --parity-seconds 0 --copy-streams 2 && \
           run t_blit 200 $B --steps 30 --parity-seconds 0 --download-engine blit && \
           run t_kern 200 $B --steps 30 --parity-seconds 0 --download-engine kernel && \
           run t_dd0_c1 200 env AMD_DIRECT_DISPATCH=0 $B --workload c1 --steps 30 --parity-seconds 5 && \
           run t_c1 200 $B --workload c1 --steps 30 --parity-seconds 0 ;;
    warm) run w_c3 200 $B --steps 30 --parity-seconds 5 && \
          run w_c3_nowarm 200 $B --steps 30 --parity-seconds 0 --no-warm-engines && \
          run w_c3_ma0 200 $B --steps 30 --parity-seconds 0 --max-ahead 0 && \
          run w_c3_ma8 200 $B --steps 30 --parity-seconds 0 --max-ahead 8 && \
          run w_c1 200 $B --workload c1 --steps 30 --parity-seconds 5 && \
          run w_c3_100 200 $B --steps 100 --parity-seconds 0 ;;
    m10b) run m10tests 400 python -u -m pytest tests/test_gpu_main10.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread && \
          run m10bench 300 $B --workload c3_qp22_main10 --steps 10 --parity-seconds 10 && \
          run m10bench_px 300 env FME_MAIN10_SEARCH=px $B --workload c3_qp22_main10 --steps 10 --parity-seconds 0 ;;
    copytl_rocpd) run copytl_rocpd 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format rocpd -d gpurun_out/copytl_rocpd -o run -- python3 bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 10 ;;
    tl) run tl_c3 200 $B --steps 20 --parity-seconds 0 --timeline gpurun_out/timeline_c3.txt && \
        run tl_c1 200 $B --workload c1 --steps 20 --parity-seconds 0 --timeline gpurun_out/timeline_c1.txt ;;
    mc10) run mc10tests 300 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_main10.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    logwait) run env_logwait 200 env AMD_LOG_LEVEL=4 AMD_LOG_MASK=294 $B --steps 12 --parity-seconds 0 ;;
    tzc) run tz_counts 200 python -u tools/tz_counts.py ;;
    icache) A="python tools/ab_bench.py . --rounds 2 --reps 2"
            run ic_a 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS --output-format csv -d gpurun_out/ic/a -o run -- $A && \
            run ic_b 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/ic/b -o run -- $A && \
            run ic_c 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/ic/c -o run -- $A && \
            python3 tools/pmc_summary.py gpurun_out/ic > gpurun_out/icache.txt ;;
    bench) run bench 400 python -u bench.py --no-pi --no-tz --no-mc ;;
    benchfull) run benchfull 600 python -u bench.py ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    copytl) run copytl 300 env FME_CRASH_TRACE=1 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/copytl -o run -- python3 bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 10 ;;
    copytl_dbg) run copytl_dbg 300 env FME_CRASH_TRACE=1 LD_DEBUG=files rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/copytl -o run -- python3 bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 10 ;;
    copytl_c1) run copytl_c1 300 env FME_CRASH_TRACE=1 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/copytl_c1 -o run -- python3 bench.py --workload c1 --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 --steps 10 ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 --no-pcie ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
