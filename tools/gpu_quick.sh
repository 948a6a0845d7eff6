#!/bin/bash
# Quick GPU check of the batch path after a change: parity / async / dist / deep-net tests, the
# pipeline probe and one headline bench line (no side legs).
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_dist.py tests/test_deep_nn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 && tail -3 gpurun_out/t.log && \
$T 120 python tools/pipe_probe.py c3_qp22 > gpurun_out/pp.log 2>&1 && \
$T 300 python bench.py --no-cpu-baseline --no-pi --no-tz --no-mc > gpurun_out/b.log 2>&1 && \
grep -v amdgpu.ids gpurun_out/pp.log && python -c "
import json;d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),round(d['ms_per_step'],4),{k:round(v,3) for k,v in d['roofline']['batch_kernel_ms'].items()},round(d['device_resident']['ms_per_step'],4))"
