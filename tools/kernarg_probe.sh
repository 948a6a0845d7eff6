mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-pi --no-tz --no-mc"
summ() { python -c "
import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,1), round(d['ms_per_step'],4), {k:round(v,3) for k,v in d['roofline']['batch_kernel_ms'].items()}, round(d['device_resident']['ms_per_step'],4))" $1; }
timeout -k 10 200 $B > gpurun_out/k0.log 2>&1 && summ gpurun_out/k0.log && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 $B > gpurun_out/k1.log 2>&1 && summ gpurun_out/k1.log && \
timeout -k 10 200 $B > gpurun_out/k2.log 2>&1 && summ gpurun_out/k2.log && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 $B > gpurun_out/k3.log 2>&1 && summ gpurun_out/k3.log
