#!/bin/bash
# Integer-search profile on the 1080p frame (tools/tz_probe.py): kernel trace + stats, SQ counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tzprof
mkdir -p $O
T="timeout -k 10"
$T 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/tz_probe.py $O/x.npz > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
$T 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SMEM --output-format csv -d $O/sq/n -o run -- python tools/tz_probe.py $O/x.npz > $O/sqn.log 2>&1 || { tail -20 $O/sqn.log; exit 1; }
$T 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq/o -o run -- python tools/tz_probe.py $O/x.npz > $O/sqo.log 2>&1 || { tail -20 $O/sqo.log; exit 1; }
$T 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/sq/c -o run -- python tools/tz_probe.py $O/x.npz > $O/sqc.log 2>&1 || { tail -20 $O/sqc.log; exit 1; }
python3 tools/pmc_summary.py $O/sq > $O/sq_summary.txt
grep -A22 "k_tz_wave" $O/sq_summary.txt | head -60
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/tzprof/trace/run_kernel_trace.csv")))
ks = collections.defaultdict(list)
for r in rows:
    ks[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in ks.items():
    print(k, len(v), [round(x) for x in v[:12]])
PY
$T 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pi -o run -- python tools/pred_inter_probe.py 3 > $O/pi.log 2>&1 || { tail -20 $O/pi.log; exit 1; }
grep pred_inter $O/pi.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/tzprof/pi/run_kernel_stats.csv")):
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
