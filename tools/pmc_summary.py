#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (counter_collection) per kernel: mean value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "?")
            name = row.get("Counter_Name")
            try:
                v = float(row.get("Counter_Value", "nan"))
            except ValueError:
                continue
            acc[k][(row.get("Dispatch_Id"), name)].append(v)
for k, d in acc.items():
    per = defaultdict(list)
    for (disp, name), vals in d.items():
        per[name].append(sum(vals))   # sum over instances (XCDs/SEs) within a dispatch
    short = k.replace("(anonymous namespace)::", "").split("(")[0]
    print(short)
    for name in sorted(per):
        v = per[name]
        print(f"   {name:28s} {sum(v)/len(v):18.1f}   (dispatches {len(v)})")
