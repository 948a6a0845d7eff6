#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run of bench.py: the last steps'
kernels and copies in start order with their offsets and durations, and per-step spacing
(k_classify to k_classify).

usage: timeline.py TRACE_DIR [steps_to_show] [first_step]
first_step: index of the first k_classify launch shown (default: the last steps_to_show steps;
bench.py runs the PCIe-inclusive pass before the resident one, so its steps come first)."""
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    first = int(sys.argv[3]) if len(sys.argv) > 3 else None
    ev = []
    for p in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", name[-40:], r.get("Queue_Id", "")))
    for p in glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            kind = r.get("Direction", r.get("Operation", "copy"))
            size = r.get("Size", r.get("Bytes", ""))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", f"{kind} {size}", ""))
    ev.sort()
    cls = [e for e in ev if e[2] == "K" and "k_classify" in e[3]]
    if len(cls) < show + 1:
        print("too few steps", len(cls))
        return
    gaps = [(cls[i + 1][0] - cls[i][0]) / 1e3 for i in range(len(cls) - 1)]
    print("classify-to-classify (us):", [round(g) for g in gaps])
    i0 = len(cls) - show - 1 if first is None else first
    t0 = cls[i0][0]
    t1 = cls[min(i0 + show, len(cls) - 1)][0]
    for s, e, k, name, q in ev:
        if t0 <= s <= t1 or t0 <= e <= t1:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {k} {name} {q}")


if __name__ == "__main__":
    main()
