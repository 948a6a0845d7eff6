#!/usr/bin/env python3
"""One integer-search golden case through the library (FME_LIB_PATH selects a variant): prints the
mismatch count against the golden MVs / SADs.  Debugging aid for the TZ kernels.

usage: FME_LIB_PATH=... python tools/tz_golden_probe.py CASE"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    from conftest import load_golden
    from test_gpu_tz import _ctx
    g = load_golden(sys.argv[1])
    print("jobs", len(g["jobs"]), "pictures", [p.shape for p in g["pictures"]], flush=True)
    jobs, sad = _ctx(g).integer_search(g["jobs"], g["ext"])
    bad = (jobs["mv_x"] != g["mv_x"]) | (jobs["mv_y"] != g["mv_y"]) | (sad != g["sad"])
    print(sys.argv[1], "mismatches", int(bad.sum()), "of", len(bad), flush=True)


if __name__ == "__main__":
    main()
