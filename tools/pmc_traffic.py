#!/usr/bin/env python3
"""HBM traffic per launch of the search kernels from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; separate passes, MI355X_MICROARCH.md "rocprofv3 PMC slots").

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over the TCC instances here).  gfx950
tallies 128-B read requests at 64 B, so FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM); our
own check: k_classify's FETCH_SIZE x 2 equals the 27.6 MB job array it streams.
Usage: pmc_traffic.py <pmc dir with fetch/ and write/ passes> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(root, counter):
    acc = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = row.get("Kernel_Name", "?").split("(")[0]
                acc[k][row.get("Dispatch_Id")] += float(row["Counter_Value"])
    return {k: sum(d.values()) / len(d) for k, d in acc.items() if d}


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch = per_dispatch(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(root, "write"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("fme::"):
            continue
        f = fetch.get(k, 0.0) * 1024 * 2
        w = write.get(k, 0.0) * 1024
        kernels[k] = {"fetch_bytes": f, "write_bytes": w, "bytes_per_launch": f + w}
    main_ks = [k for k in kernels if k.startswith("fme::k_search_lane")] or ["fme::k_search_small"]
    d = {
        "kernel": "+".join(main_ks),
        "bytes_per_launch": sum(kernels.get(k, {}).get("bytes_per_launch") or 0 for k in main_ks) or None,
        "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, separate passes, "
                  "bench.py --steps 2 --warmup 1 (profiles/pmc_traffic.json)",
        "kernels": kernels,
    }
    with open(out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
