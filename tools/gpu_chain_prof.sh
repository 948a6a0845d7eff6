#!/bin/bash
# Producer chain profile: kernel trace of one P frame (tools/pred_inter_probe.py), the k_tz_level
# duration distribution and the gaps between consecutive level launches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chain
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python tools/pred_inter_probe.py 3 > $O/pi.log 2>&1 || { tail -20 $O/pi.log; exit 1; }
grep pred_inter $O/pi.log
python3 - <<'PY'
import csv, numpy as np
rows = [r for r in csv.DictReader(open("gpurun_out/chain/run_kernel_trace.csv")) if "k_tz_level" in r["Kernel_Name"]]
s = np.array([int(r["Start_Timestamp"]) for r in rows]); e = np.array([int(r["End_Timestamp"]) for r in rows])
o = np.argsort(s); s, e = s[o], e[o]
d = (e - s) / 1e3; g = (s[1:] - e[:-1]) / 1e3
print("levels", len(d), "sum dur ms", d.sum() / 1e3, "sum gaps ms", g[g < 1000].sum() / 1e3)
print("dur pct 10/50/90/99/max us", np.percentile(d, [10, 50, 90, 99, 100]).round(1))
print("gap pct 10/50/90/99 us", np.percentile(g, [10, 50, 90, 99]).round(1))
grid = np.array([int(r["Grid_Size_X"]) for r in rows])[o]
print("grid (threads) pct 10/50/90/max", np.percentile(grid, [10, 50, 90, 100]))
PY
