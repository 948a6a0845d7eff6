#!/bin/bash
# Integer-search variants: timing + identical-result check against the in-tree library.
set -o pipefail
mkdir -p gpurun_out/tz
export TMPDIR=/tmp
timeout -k 10 120 python tools/tz_probe.py gpurun_out/tz/cur.npz || exit 1
for v in "$@"; do
  FME_LIB_PATH=$PWD/hm16.9-nn_fme_amd/variants/$v/libfme_amd.so timeout -k 10 120 python tools/tz_probe.py gpurun_out/tz/$v.npz || exit 1
done
python3 - "$@" <<'PY'
import sys, numpy as np
a = np.load("gpurun_out/tz/cur.npz")
for v in sys.argv[1:]:
    b = np.load(f"gpurun_out/tz/{v}.npz")
    print(v, "identical" if all(np.array_equal(a[k], b[k]) for k in a.files) else "DIFFERENT")
PY
