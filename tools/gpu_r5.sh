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
    pdebug) run pdebug 300 python -u tools/parity_debug.py 20 3 8 && run pdebug10 300 python -u tools/parity_debug.py 3 3 10 ;;
    verify) run pm_base 200 python -u tools/parity_debug.py 20 3 8 base && run pm_base10 200 python -u tools/parity_debug.py 6 3 10 base && \
            run pb20 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20 --parity-seconds 10 && \
            run vtests 500 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_main10.py tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_async.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread && \
            run tz_new 200 python -u tools/tz_probe.py gpurun_out/tz_new.npz && \
            run tztests 400 python -u -m pytest tests -m gpu -k "tz or ring or integer or pred_inter" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread && \
            CPU=0 run pprobe 300 python -u tools/pred_inter_probe.py 3 ;;
    dlab2) B="python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 20"
           run d_blit_def 200 $B && run d_blit_imm 200 $B --download immediate && \
           run d_k_def_r0 200 $B --download-engine kernel && \
           run d_k_def_r8 200 $B --download-engine kernel --search-reserve 8 && \
           run d_k_def_r16 200 $B --download-engine kernel --search-reserve 16 && \
           run d_k_def_r32w16 200 $B --download-engine kernel --search-reserve 32 --download-wgs 16 && \
           run d_k_imm_r16 200 $B --download-engine kernel --search-reserve 16 --download immediate && \
           run d_blit_def_r16 200 $B --search-reserve 16 ;;
    dlab3) B="python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 20"
           run e_r16 200 $B --search-reserve 16 && run e_r32 200 $B --search-reserve 32 && run e_r64 200 $B --search-reserve 64 && \
           DEBUG_CLR_LIMIT_BLIT_WG=16 run e_lim16 200 $B && DEBUG_CLR_LIMIT_BLIT_WG=64 run e_lim64 200 $B && \
           DEBUG_CLR_LIMIT_BLIT_WG=16 run e_lim16_r16 200 $B --search-reserve 16 && \
           GPU_BLIT_ENGINE_TYPE=1 run e_bet1 200 $B && GPU_BLIT_ENGINE_TYPE=2 run e_bet2 200 $B ;;
    timeline) run tl 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --steps 10 --search-reserve 16 && \
              bash tools/gpu_r5.sh dlab4 deepsq ;;
    pxab) run m10t 300 python -u -m pytest tests/test_gpu_main10.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread && \
          run px4 300 python -u bench.py --workload c3_qp22_main10 --no-cpu-baseline --parity-seconds 0 --steps 10 && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/px6/libfme_amd.so run px6 300 python -u bench.py --workload c3_qp22_main10 --no-cpu-baseline --parity-seconds 0 --steps 10 && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tz6/libfme_amd.so run tz6 200 python -u tools/tz_probe.py gpurun_out/tz6.npz && \
          run tz5b 200 python -u tools/tz_probe.py gpurun_out/tz5b.npz ;;
    deepsq) run deepsq 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/deepsq -o run -- python3 bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 3 --warmup 1 && \
            python3 tools/pmc_summary.py gpurun_out/deepsq > gpurun_out/deepsq_summary.txt && grep -A9 "deep_tail" gpurun_out/deepsq_summary.txt ;;
    dlab4) B="python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20"
           run s_sdma 200 $B --download-engine sdma --parity-seconds 5 && run s_sdma_r16 200 $B --download-engine sdma --search-reserve 16 --parity-seconds 0 && \
           run s_blit 200 $B --parity-seconds 0 && run s_blit_r16 200 $B --search-reserve 16 --parity-seconds 0 && \
           run s_sdma_imm 200 $B --download-engine sdma --download immediate --parity-seconds 0 ;;
    pxab2) B="python -u bench.py --workload c3_qp22_main10 --no-cpu-baseline --parity-seconds 0 --steps 10"
           run px6d 300 $B && FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/px5/libfme_amd.so run px5 300 $B && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/px8/libfme_amd.so run px8 300 $B && run px6p 300 $B --parity-seconds 10 ;;
    sbab) run sbab 500 python -u tools/ab_bench.py . variants/sb1 variants/sb16 --rounds 4 && \
          P="python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --no-pcie --parity-seconds 0 --steps 2 --warmup 1" && \
          run sb8_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sbpmc/sb8/fetch -o run -- $P && \
          run sb8_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sbpmc/sb8/write -o run -- $P && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/sb1/libfme_amd.so run sb1_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sbpmc/sb1/fetch -o run -- $P && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/sb16/libfme_amd.so run sb16_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sbpmc/sb16/fetch -o run -- $P ;;
    c5w) B="python -u bench.py --no-cpu-baseline --no-pi --no-tz --no-mc"
         run bench_c5 300 $B --workload c5 && run bench_c5_exact 300 $B --workload c5_exact && run bench_c5_b4x40 300 $B --workload c5_b4x40 ;;
    icache) P="python3 bench.py --no-cpu-baseline --no-pi --no-tz --no-mc --no-pcie --parity-seconds 0 --steps 2 --warmup 1"
            run icache 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/icache -o run -- $P && \
            python3 tools/pmc_summary.py gpurun_out/icache > gpurun_out/icache_summary.txt && \
            run icache_tz 200 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/icache_tz -o run -- python3 tools/tz_probe.py gpurun_out/tz_ic.npz && \
            python3 tools/pmc_summary.py gpurun_out/icache_tz > gpurun_out/icache_tz_summary.txt ;;
    tlc1) run tlc1 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tlc1 -o run -- python3 bench.py --workload c1 --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 --steps 10 && \
          python3 tools/timeline.py gpurun_out/tlc1 3 8 > gpurun_out/tlc1_timeline.txt ;;
    tzs) run tzs_tests 400 python -u -m pytest tests -m gpu -k "tz or ring or integer or pred_inter" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread && \
         run tzs_def 200 python -u tools/tz_probe.py gpurun_out/tzs_def.npz && \
         FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzs0/libfme_amd.so run tzs_0 200 python -u tools/tz_probe.py gpurun_out/tzs_0.npz && \
         python3 -c "import numpy as np; a=np.load('gpurun_out/tzs_def.npz'); b=np.load('gpurun_out/tzs_0.npz'); print('identical', all((a[k]==b[k]).all() for k in a.files))" ;;
    warm) run warm 200 python -u -c "import torch; print(torch.__version__, torch.cuda.is_available())" ;;
    tzdbg) FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzs0/libfme_amd.so true && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzdbg/libfme_amd.so run tzg_dbg 60 python -u tools/tz_golden_probe.py tz_far_fen0_sr32 ;;
    tzab3) FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzC/libfme_amd.so run tzC 50 python -u tools/tz_golden_probe.py tz_far_fen0_sr32 && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzB/libfme_amd.so run tzB 50 python -u tools/tz_golden_probe.py tz_far_fen0_sr32 && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzA/libfme_amd.so run tzA 50 python -u tools/tz_golden_probe.py tz_far_fen0_sr32 ;;
    tzs2) run tzs_tests 400 python -u -m pytest tests -m gpu -k "tz or ring or integer or pred_inter" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread && \
          run tzs_def 200 python -u tools/tz_probe.py gpurun_out/tzs_def.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzs0/libfme_amd.so run tzs_0 200 python -u tools/tz_probe.py gpurun_out/tzs_0.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzn8/libfme_amd.so run tzs_n8 200 python -u tools/tz_probe.py gpurun_out/tzs_n8.npz && \
          python3 -c "import numpy as np; a=np.load('gpurun_out/tzs_def.npz'); b=np.load('gpurun_out/tzs_0.npz'); c=np.load('gpurun_out/tzs_n8.npz'); print('identical', all((a[k]==b[k]).all() and (a[k]==c[k]).all() for k in a.files))" && \
          run tzs_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tzs_trace -o run -- python3 tools/tz_probe.py gpurun_out/tzs_t.npz ;;
    tzs3) run tzs_tests 400 python -u -m pytest tests -m gpu -k "tz or ring or integer or pred_inter" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread && \
          run tzs_def 200 python -u tools/tz_probe.py gpurun_out/tzs_def.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzs0/libfme_amd.so run tzs_0 200 python -u tools/tz_probe.py gpurun_out/tzs_0.npz && \
          python3 -c "import numpy as np; a=np.load('gpurun_out/tzs_def.npz'); b=np.load('gpurun_out/tzs_0.npz'); print('identical', all((a[k]==b[k]).all() for k in a.files))" && \
          run tzs_trace 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tzs_trace -o run -- python3 tools/tz_probe.py gpurun_out/tzs_t.npz ;;
    tzs4) run tzs_def 200 python -u tools/tz_probe.py gpurun_out/tzs_def.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzn10/libfme_amd.so run tzs_n10 200 python -u tools/tz_probe.py gpurun_out/tzs_n10.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tzw4/libfme_amd.so run tzs_w4 200 python -u tools/tz_probe.py gpurun_out/tzs_w4.npz && \
          run tzs_def2 200 python -u tools/tz_probe.py gpurun_out/tzs_def2.npz && \
          python3 -c "import numpy as np; a=np.load('gpurun_out/tzs_def.npz'); b=np.load('gpurun_out/tzs_n10.npz'); c=np.load('gpurun_out/tzs_w4.npz'); print('identical', all((a[k]==b[k]).all() and (a[k]==c[k]).all() for k in a.files))" ;;
    bround) run bround_tests 400 python -u -m pytest tests -m gpu -k "pred_inter or tz or ring or integer" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread && \
            CPU=0 run pprobe 300 python -u tools/pred_inter_probe.py 3 ;;
    cagg) run cagg 400 python -u tools/ab_bench.py . variants/cagg --rounds 4 ;;
    tzm) run tzm_def 200 python -u tools/tz_probe.py gpurun_out/tzm_def.npz && \
         FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/m64/libfme_amd.so run tzm_64 200 python -u tools/tz_probe.py gpurun_out/tzm_64.npz && \
         FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/m88/libfme_amd.so run tzm_88 200 python -u tools/tz_probe.py gpurun_out/tzm_88.npz && \
         run tzm_def2 200 python -u tools/tz_probe.py gpurun_out/tzm_def2.npz && \
         python3 -c "import numpy as np; a=np.load('gpurun_out/tzm_def.npz'); b=np.load('gpurun_out/tzm_64.npz'); c=np.load('gpurun_out/tzm_88.npz'); print('identical', all((a[k]==b[k]).all() and (a[k]==c[k]).all() for k in a.files))" ;;
    tzo) run tzo_def 200 python -u tools/tz_probe.py gpurun_out/tzo_def.npz && \
         FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/ord/libfme_amd.so run tzo_ord 200 python -u tools/tz_probe.py gpurun_out/tzo_ord.npz && \
         run tzo_def2 200 python -u tools/tz_probe.py gpurun_out/tzo_def2.npz && \
         FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/ord/libfme_amd.so run tzo_ord2 200 python -u tools/tz_probe.py gpurun_out/tzo_ord2.npz && \
         python3 -c "import numpy as np; a=np.load('gpurun_out/tzo_def.npz'); b=np.load('gpurun_out/tzo_ord.npz'); print('identical', all((a[k]==b[k]).all() for k in a.files))" ;;
    tlc1k) run tlc1k 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlc1k -o run -- python3 bench.py --workload c1 --no-cpu-baseline --no-pi --no-tz --no-mc --parity-seconds 0 --steps 10 && \
           python3 tools/timeline.py gpurun_out/tlc1k 3 8 > gpurun_out/tlc1k_timeline.txt ;;
    bigab) run bigab 400 python -u tools/ab_bench.py . variants/big --rounds 4 && bash tools/gpu_r5.sh bench1 bench2 ;;
    bench1) run bench1 300 python -u bench.py --no-pi --no-tz --no-mc --cpu-seconds 3 --parity-seconds 10 ;;
    bench2) run bench2 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --dist-backend gloo ;;
    pmodes) run pm_base 200 python -u tools/parity_debug.py 20 3 8 base && run pm_base10 200 python -u tools/parity_debug.py 6 3 10 base && \
            run pi_tests 400 python -u -m pytest tests -m gpu -k "pred_inter" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread && \
            run pb20 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20 --parity-seconds 10 && \
            CPU=0 run pprobe 300 python -u tools/pred_inter_probe.py 3 && \
            bash tools/gpu_r5.sh tzab tests ;;
    pprobe) CPU=0 run pprobe 300 python -u tools/pred_inter_probe.py 3 ;;
    m10prof) run m10prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m10prof -o run -- python3 bench.py --workload c3_qp22_main10 --no-cpu-baseline --parity-seconds 0 --steps 5 ;;
    d2h) run d2h 200 ./tools/probes/d2h_kernel_probe ;;
    deepab) run deep_hoist 400 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 && \
            FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/deep_nohoist/libfme_amd.so run deep_nohoist 400 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 ;;
    pbench) run pbA 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --steps 20 --parity-seconds 3 && \
            run pbB 300 python -u bench.py --no-pi --no-tz --no-mc --cpu-seconds 2 --steps 3 --parity-seconds 3 && \
            run pbC 300 python -u bench.py --workload c3_qp22_main10 --no-cpu-baseline --steps 3 --parity-seconds 3 && \
            run pbD 300 python -u bench.py --workload c3_qp22_main10 --cpu-seconds 2 --steps 3 --parity-seconds 3 ;;
    resab) run res_blit 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/res16/libfme_amd.so run res16_k8 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --download-engine kernel --download-wgs 8 && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/res16/libfme_amd.so run res16_k16 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 --download-engine kernel --download-wgs 16 && \
           FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/res16/libfme_amd.so run res16_blit 300 python -u bench.py --no-pi --no-tz --no-mc --no-cpu-baseline --parity-seconds 0 ;;
    occab) run occab 400 python -u tools/ab_bench.py . variants/s0 variants/w3s0 variants/nosj --rounds 4 ;;
    main10) run main10_test 300 python -u -m pytest tests/test_gpu_main10.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread && \
            run main10_bench 400 python -u bench.py --workload c3_qp22_main10 --cpu-seconds 6 --parity-seconds 15 ;;
    deepab2) run deeptests 400 python -u -m pytest tests/test_deep_nn.py tests/test_ring.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread && \
             run deep_mall 300 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 && \
             FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/deep_mall0/libfme_amd.so run deep_mall0 300 python -u bench.py --workload c5 --no-cpu-baseline --parity-seconds 0 --steps 20 ;;
    tzab) run tz_in 200 python -u tools/tz_probe.py gpurun_out/tz_in.npz && \
          FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/tz5/libfme_amd.so run tz_5 200 python -u tools/tz_probe.py gpurun_out/tz_5.npz && \
          run tz_in2 200 python -u tools/tz_probe.py gpurun_out/tz_in2.npz && \
          python3 -c "import numpy as np; a=np.load('gpurun_out/tz_in.npz'); b=np.load('gpurun_out/tz_5.npz'); print('identical', all((a[k]==b[k]).all() for k in a.files))" ;;
    tzprof) run tzprof 700 bash tools/gpu_tz_prof.sh ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
