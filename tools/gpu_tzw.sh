#!/bin/bash
# Integer search A/B: lane-per-unit kernels (FME_TZ_WAVE=0) vs the wave-uniform search (default):
# timing + identical MVs / SADs on the 1080p frame, the TZ / producer GPU tests, the P-frame probe.
set -o pipefail
mkdir -p gpurun_out/tz
export TMPDIR=/tmp
T="timeout -k 10"
FME_TZ_WAVE=0 $T 120 python tools/tz_probe.py gpurun_out/tz/old.npz || exit 1
$T 120 python tools/tz_probe.py gpurun_out/tz/new.npz || exit 1
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/tz/old.npz"); b = np.load("gpurun_out/tz/new.npz")
for k in a.files:
    d = a[k] != b[k]
    print(k, "identical" if not d.any() else f"DIFFERENT in {int(d.sum())} entries, first {np.flatnonzero(d.ravel())[:5]}")
PY
$T 400 python -u -m pytest tests/test_gpu_tz.py tests/test_pred_inter.py tests/test_pred_inter_b.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tz/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/tz/pytest.log; [ $rc -eq 0 ] || exit $rc
FME_TZ_WAVE=0 $T 200 python tools/pred_inter_probe.py 3 || exit 1
$T 200 python tools/pred_inter_probe.py 3
