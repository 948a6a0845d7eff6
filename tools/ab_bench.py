#!/usr/bin/env python3
"""A/B timing of library variants in ONE process on the same inputs (1080p QP22 frame batch).

usage: python tools/ab_bench.py variants/b40 variants/b20 ... [--rounds 5]
Each variant directory holds a libfme_amd.so.  Rounds interleave the variants; reports the
median / min of the search-kernel time (HIP events) and of the whole batch, and checks that
every variant's results are byte-identical to the first one's.
"""
import argparse
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--jobs", choices=("ctu", "uniform"), default="ctu")
    args = ap.parse_args()
    import torch
    from nnfme import synth
    from nnfme.abi import RESULT_DTYPE
    from nnfme.runtime import FmeContext
    W, H = 1920, 1080
    rng = np.random.default_rng(1000)
    if args.jobs == "uniform":
        jobs = synth.make_jobs(rng, W, H, synth.jobs_per_frame(W, H), 4, [0, 1, 2, 3], [0])
    else:
        jobs = synth.make_ctu_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0])
    pics = [synth.synth_luma(W, H, t) for t in (7, 6, 5, 4, 0)]
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    ctxs, res = [], []
    for v in args.variants:
        path = os.path.join(ROOT, "hm16.9-nn_fme_amd", v, "libfme_amd.so") if not v.endswith(".so") else v
        c = FmeContext(lib_path=path, max_jobs=len(jobs))
        for k, p in enumerate(pics):
            c.set_picture(k, p)
        c.set_lambda(0, synth.LDP_LAMBDA[22][1])
        c.set_profiling(True)
        ctxs.append(c)
        res.append(torch.empty(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev))
    s = torch.cuda.current_stream(dev).cuda_stream
    times = [[] for _ in args.variants]
    for r in range(args.rounds):
        for i, c in enumerate(ctxs):
            for _ in range(args.reps):
                c.nn_reset()
                c.refine_device(dj.data_ptr(), res[i].data_ptr(), len(jobs), s)
                t = c.last_timings()
                if r > 0:
                    times[i].append(t)
    base = res[0].cpu().numpy()
    for i, v in enumerate(args.variants):
        same = bool(np.array_equal(res[i].cpu().numpy(), base))
        srch = [t["search"] for t in times[i]]
        bat = [t["batch"] for t in times[i]]
        nn = [t["nn_tail"] for t in times[i]]
        print(f"{v:28s} search med {statistics.median(srch):7.3f} min {min(srch):7.3f} ms | "
              f"nn {statistics.median(nn):6.3f} | batch med {statistics.median(bat):7.3f} ms "
              f"-> {len(jobs) / statistics.median(bat) / 1e3:8.1f} M PU/s | identical={same}")


if __name__ == "__main__":
    main()
