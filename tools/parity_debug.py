"""Debug of the bench's after-run parity leg: every step of a FrameReplay (the bench's 1080p job
stream) against the library's host path with that step's bindings, NN off so that no carried state
enters: a mismatch is a binding (pictures, lambdas, jobs) or ordering problem of the replay.

usage: python tools/parity_debug.py [steps] [warmup] [bit_depth] [mode]
mode: base | nodefer (downloads right after each batch) | noprefetch | serial (synchronize after
every step) | noprof (profiling off)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hm16.9-nn_fme_amd"), ROOT, os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import bench  # noqa: E402
from nnfme import synth  # noqa: E402
from nnfme.abi import MV_FIELDS  # noqa: E402
from nnfme.pipeline import ORG0, REFS, FrameReplay  # noqa: E402
from nnfme.runtime import FmeContext  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    bd = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    mode = sys.argv[4] if len(sys.argv) > 4 else "base"
    wl = bench.WORKLOADS["c3_qp22"]
    jobs = bench.make_frame_jobs(1000, "ctu", wl["calls"], wl["bipred"])
    m = 4000
    pic = (lambda t: synth.synth_luma(1920, 1080, t)) if bd == 8 else \
        (lambda t: synth.synth_luma_hbd(1920, 1080, t, bit_depth=bd))
    pool = np.stack([pic(t) for t in range(8)])
    ctx = FmeContext(device=0, nn_mode=0, qp=22, fast_inter_mode=1, max_jobs=len(jobs), bit_depth=bd)
    lam = lambda f: bench.frame_lambda(wl, f)   # noqa: E731
    rep = FrameReplay(ctx, jobs, pool, lam, warm + steps, device=torch.device("cuda", 0),
                      defer_download=mode != "nodefer")
    rep.prime()
    for s in range(warm):
        rep.issue(s, prefetch=s + 1 < warm)
    rep.drain()
    ctx.set_profiling(mode != "noprof")
    for s in range(warm, warm + steps):
        rep.issue(s, prefetch=mode != "noprefetch")
        if mode == "serial":
            torch.cuda.synchronize()
    rep.finish(first_step=warm)
    torch.cuda.synchronize()
    c2 = FmeContext(device=0, nn_mode=0, qp=22, fast_inter_mode=1, max_jobs=m, bit_depth=bd)
    for k in range(warm + steps):
        f0 = rep.first_frame(k)
        c2.set_picture(ORG0, pool[f0 % 8])
        c2.set_lambda(0, lam(f0))
        for slot in range(REFS):
            c2.set_picture(slot, pool[(f0 - REFS + slot) % 8])
        b = c2.refine_mv(rep.jobs[:m])
        g = rep.results(k)[:m]
        bad = {f: int((b[f] != g[f]).sum()) for f in MV_FIELDS if f != "status"}
        # which frame's bindings do the replay's results match?
        match = None
        if any(bad.values()):
            for d in (-2, -1, 1, 2):
                f1 = f0 + d
                c2.set_picture(ORG0, pool[f1 % 8])
                c2.set_lambda(0, lam(f1))
                for slot in range(REFS):
                    c2.set_picture(slot, pool[(f1 - REFS + slot) % 8])
                b2 = c2.refine_mv(rep.jobs[:m])
                if all(int((b2[f] != g[f]).sum()) == 0 for f in ("mv_x", "mv_y", "cost")):
                    match = d
                    break
            for dl in (-1, 1, 2):   # only the lambda of another frame
                c2.set_picture(ORG0, pool[f0 % 8])
                for slot in range(REFS):
                    c2.set_picture(slot, pool[(f0 - REFS + slot) % 8])
                c2.set_lambda(0, lam(f0 + dl))
                b2 = c2.refine_mv(rep.jobs[:m])
                if all(int((b2[f] != g[f]).sum()) == 0 for f in ("mv_x", "mv_y", "cost")):
                    match = f"lambda{dl:+d}"
                    break
        print(f"[{mode}] step {k}: frame {f0} lambda {lam(f0)} mismatches {bad} matches frame offset {match}", flush=True)


if __name__ == "__main__":
    main()
