#!/usr/bin/env python3
"""Where k_search_lane's wave time goes, by phase: the stamp build of the search kernel
(make -C hm16.9-nn_fme_amd variant NAME=stamps DEFS=-DFME_LANE_STAMPS=1) over the 1080p LDP QP22
frame batch of bench.py.  Each lane_unit call stamps s_memtime at its phase boundaries after
waiting for its outstanding loads (so a phase carries the memory latency it exposes); the sums are
wave-cycles per (PU class, phase).  The stamp build's own run time is not the kernel's: only the
shares are read (cdna_hip_programming.md §7, In-kernel stamps).

usage: python tools/lane_stamps.py [reps]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))

PHASES = ("job+key load", "EMI step", "sub-pel window+key", "half-pel stage", "quarter-pel stage", "record stores")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import torch
    from nnfme import synth
    from nnfme.abi import RESULT_DTYPE
    from nnfme.runtime import FmeContext
    lib_path = os.path.join(ROOT, "hm16.9-nn_fme_amd", "variants", "stamps", "libfme_amd.so")
    W, H = 1920, 1080
    jobs = synth.make_ctu_jobs(np.random.default_rng(1000), W, H, 423, 4, [0, 1, 2, 3], [0])
    ctx = FmeContext(lib_path=lib_path, max_jobs=len(jobs))
    for k, t in enumerate((7, 6, 5, 4, 0)):
        ctx.set_picture(k, synth.synth_luma(W, H, t))
    ctx.set_lambda(0, synth.LDP_LAMBDA[22][1])
    lib = ctypes.CDLL(lib_path)
    lib.fme_debug_lane_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    dr = torch.empty(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    ctx.refine_device(dj.data_ptr(), dr.data_ptr(), len(jobs), s.cuda_stream)   # warm-up
    s.synchronize()
    st = np.zeros((24, 8), np.uint64)
    assert lib.fme_debug_lane_stamps(st.ctypes.data, 1) == 0
    for _ in range(reps):
        ctx.nn_reset()
        ctx.refine_device(dj.data_ptr(), dr.data_ptr(), len(jobs), s.cuda_stream)
    s.synchronize()
    assert lib.fme_debug_lane_stamps(st.ctypes.data, 0) == 0
    st = st.astype(np.float64)
    cls_w = (4, 8, 8, 4, 16, 8, 16, 12, 16, 16, 8, 32, 16, 32, 24, 32, 32, 16, 64, 32, 64, 48, 64, 64)
    cls_h = (8, 4, 8, 16, 4, 16, 8, 16, 12, 16, 32, 8, 32, 16, 32, 24, 32, 64, 16, 64, 32, 64, 48, 64)
    tot = st[:, :6].sum()
    print(f"# k_search_lane phase stamps (stamp build, {reps} batches of the 1080p LDP QP22 frame, "
          f"{len(jobs)} jobs): wave-cycles summed over every lane_unit call")
    print("# share of all stamped wave-cycles by phase:")
    for p, name in enumerate(PHASES):
        print(f"  {name:22s} {100.0 * st[:, p].sum() / tot:6.2f} %")
    print("# per class: wave tiles per batch, cycles per tile by phase")
    print("%-8s %8s " % ("class", "tiles") + " ".join("%12s" % n.split()[0] for n in PHASES) + " %10s" % "total")
    for c in range(24):
        n = st[c, 6]
        if n == 0:
            continue
        per = st[c, :6] / n
        print("%-8s %8d " % (f"{cls_w[c]}x{cls_h[c]}", int(n / reps)) + " ".join("%12.0f" % v for v in per)
              + " %10.0f" % per.sum())
    ctx.close()


if __name__ == "__main__":
    main()
