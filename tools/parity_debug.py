"""Debug of the bench's after-run parity leg: the replay's results of one step against (A) oracle/_ref
with the parity leg's bindings, (B) the HIP host path with the same bindings, (C) the replay's own
download engines."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hm16.9-nn_fme_amd"), ROOT, os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import bench  # noqa: E402
from nnfme import synth, weights  # noqa: E402
from nnfme.abi import MV_FIELDS  # noqa: E402
from nnfme.pipeline import ORG0, REFS, FrameReplay  # noqa: E402
from nnfme.runtime import FmeContext  # noqa: E402


def main():
    wl = bench.WORKLOADS["c3_qp22"]
    bench.W, bench.H, bench.QP = wl["W"], wl["H"], wl["QP"]
    jobs = bench.make_frame_jobs(1000, "ctu", wl["calls"], wl["bipred"])
    ctx = FmeContext(device=0, nn_mode=1, qp=22, fast_inter_mode=1, max_jobs=len(jobs))
    pool = np.stack([synth.synth_luma(bench.W, bench.H, t) for t in range(8)])
    m = 20000
    for engine in ("blit", "kernel"):
        ctx.nn_reset()
        rep = FrameReplay(ctx, jobs, pool, lambda f: bench.frame_lambda(wl, f), 6, device=torch.device("cuda", 0),
                          download_engine=engine)
        rep.prime()
        for s in range(3):
            rep.issue(s, prefetch=s < 2)
        rep.drain()
        st = ctx.nn_get_state()
        for s in range(3, 6):
            rep.issue(s)
        rep.finish()
        g = rep.results(3)[:m]
        a = bench.parity_leg(rep, wl, None, 3, st, 60.0, max_jobs=m)
        print(engine, "parity leg:", {k: a[k] for k in ("jobs_checked", "mismatches", "per_field", "first_mismatch")},
              flush=True)
        # (B) the host path with the same bindings and state
        c2 = FmeContext(device=0, nn_mode=1, qp=22, fast_inter_mode=1, max_jobs=m)
        f0 = rep.first_frame(3)
        c2.set_picture(ORG0, pool[f0 % 8])
        c2.set_lambda(0, bench.frame_lambda(wl, f0))
        for slot in range(REFS):
            c2.set_picture(slot, pool[(f0 - REFS + slot) % 8])
        c2.nn_set_state(st)
        b = c2.refine_mv(rep.jobs[:m])
        for f in MV_FIELDS:
            d = int((b[f] != g[f]).sum())
            if d:
                print(engine, "host path vs replay: field", f, d, "first", int(np.flatnonzero(b[f] != g[f])[0]))
        print(engine, "host path vs replay checked", flush=True)
        print("job0", rep.jobs[0], "gpu", g[0], "host", b[0])
        del rep


if __name__ == "__main__":
    main()
