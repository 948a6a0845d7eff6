#!/usr/bin/env python3
"""Where the staged integer search's candidate windows come from (the tzcount diagnostic build:
make -C hm16.9-nn_fme_amd variant NAME=tzcount DEFS=-DFME_TZ_COUNT=1): per unit-shape kernel, the
lane-windows read from the group's LDS tile and from global memory (the fallback when a window
leaves the tile), over one 1080p frame of bench.py's tz-leg jobs.

usage: python tools/tz_counts.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    import torch
    from nnfme import synth
    from nnfme.runtime import FmeContext
    lib_path = os.path.join(ROOT, "hm16.9-nn_fme_amd", "variants", "tzcount", "libfme_amd.so")
    W, H = 1920, 1080
    rng = np.random.default_rng(2024)
    pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs, ext = synth.make_tz_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0, 1, 2, 3])
    ctx = FmeContext(lib_path=lib_path, nn_mode=0, fast_inter_mode=1, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    lib = ctypes.CDLL(lib_path)
    lib.fme_debug_tz_counts.argtypes = [ctypes.c_void_p, ctypes.c_int]
    cnt = np.zeros(6, np.uint64)
    assert lib.fme_debug_tz_counts(cnt.ctypes.data, 1) == 0
    ctx.integer_search(jobs, ext)
    assert lib.fme_debug_tz_counts(cnt.ctypes.data, 0) == 0
    kid = np.where(jobs["w"] % 8 != 0, 0, np.where(jobs["h"] % 8 != 0, 1, 2))
    print(f"# staged integer search, one 1080p frame ({len(jobs)} jobs): lane-windows by source")
    for k, name in enumerate(("4x8 units", "8x4 units", "8x8 units")):
        lds, glob = int(cnt[2 * k]), int(cnt[2 * k + 1])
        n = int((kid == k).sum())
        print(f"  {name}: {n} PUs, LDS tile {lds}, global {glob} ({100.0 * glob / max(lds + glob, 1):.2f} % "
              f"fallback, {glob / max(n, 1):.1f} per PU)")
    ctx.close()


if __name__ == "__main__":
    main()
