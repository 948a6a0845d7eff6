#!/usr/bin/env python3
"""Per-kernel duration statistics from a rocprofv3 kernel trace, over steady launches only.

rocprofv3 --stats averages every dispatch of a kernel, the cold first launches of a process
included.  This reads <dir>/**/run_kernel_trace.csv, sorts each kernel's dispatches by start
time, drops the first --skip of them (the bench's warmup steps) and writes the same columns as
rocprofv3's kernel_stats.csv (plus the median) over the rest.

usage: steady_stats.py TRACE_DIR OUT_CSV [--skip N]
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("out_csv")
    ap.add_argument("--skip", type=int, default=3, help="first dispatches of each kernel to drop")
    a = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(p)))
    per = defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = []
    for k, v in per.items():
        v.sort()
        d = [x[1] for x in v[a.skip:]] or [x[1] for x in v]
        out.append((k, len(d), sum(d), sum(d) / len(d), statistics.median(d), min(d), max(d),
                    statistics.pstdev(d) if len(d) > 1 else 0.0, len(v) - len(d)))
    out.sort(key=lambda o: -o[2])
    tot = sum(o[2] for o in out) or 1
    with open(a.out_csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "Percentage", "MinNs", "MaxNs",
                    "StdDev", "SkippedColdCalls"])
        for k, n, s, avg, med, mn, mx, sd, sk in out:
            w.writerow([k, n, s, round(avg, 3), med, round(100.0 * s / tot, 3), mn, mx, round(sd, 3), sk])
    for k, n, s, avg, med, mn, mx, sd, sk in out[:8]:
        print(f"{k.split('(')[0][:60]:60s} n={n:4d} avg={avg / 1e3:9.2f}us med={med / 1e3:9.2f}us "
              f"min={mn / 1e3:9.2f} max={mx / 1e3:9.2f} (skipped {sk})")


if __name__ == "__main__":
    main()
