#!/usr/bin/env python3
"""Per-phase cycle shares of the search kernels from a FME_STAMPS=1 diagnostic build.
usage: python tools/phase_stamps.py variants/stamps   (run on the GPU box)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))
PHASES = ["descr+stage+transpose", "EMI items", "EMI decision", "planes", "half planes",
          "half SATD", "half argmin", "quarter SATD", "quarter argmin"]


def main():
    import torch
    from nnfme import synth
    from nnfme.abi import RESULT_DTYPE
    from nnfme.runtime import FmeContext
    v = sys.argv[1]
    W, H = 1920, 1080
    rng = np.random.default_rng(1000)
    jobs = synth.make_ctu_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0])
    sizes = sys.argv[2:] if len(sys.argv) > 2 else None
    c = FmeContext(lib_path=os.path.join(ROOT, "hm16.9-nn_fme_amd", v, "libfme_amd.so"), max_jobs=len(jobs))
    for k, t in enumerate((7, 6, 5, 4, 0)):
        c.set_picture(k, synth.synth_luma(W, H, t))
    c.set_lambda(0, synth.LDP_LAMBDA[22][1])
    res = np.zeros(len(jobs), RESULT_DTYPE)
    c.refine(jobs)
    c.debug_phase_cycles(reset=True)
    for _ in range(3):
        c.refine(jobs)
    st = c.debug_phase_cycles(reset=True).astype(np.float64)
    tot = st[:9].sum()
    print(f"workgroups {int(st[15])}, mean cycles per workgroup {tot / st[15]:.0f}")
    for i, n in enumerate(PHASES):
        print(f"  {n:24s} {100 * st[i] / tot:6.1f} %   {st[i] / st[15]:8.0f} cyc/wg")
    sub = ["  prologue: descriptors", "  prologue: fill+barrier", "  prologue: samples (wave0)",
           "  prologue: wait others", "  prologue: transpose"]
    for i, n in enumerate(sub):
        print(f"  {n:28s} {st[9 + i] / st[15]:8.0f} cyc/wg")


if __name__ == "__main__":
    main()
