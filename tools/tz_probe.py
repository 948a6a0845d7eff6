#!/usr/bin/env python3
"""Integer-search timing probe on one 1080p frame of TZ jobs (bench.py's tz leg workload).

usage: FME_LIB_PATH=... python tools/tz_probe.py OUT.npz
Prints the median kernel time (library HIP events) and writes the MVs / SADs so variants can be
compared for identical results."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    import torch
    from nnfme import synth
    from nnfme.runtime import LIB_PATH, FmeContext
    W, H = 1920, 1080
    rng = np.random.default_rng(2024)
    pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs, ext = synth.make_tz_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0, 1, 2, 3])
    dev = torch.device("cuda", 0)
    ctx = FmeContext(nn_mode=0, fast_inter_mode=1, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    src = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    dj = src.clone()
    de = torch.from_numpy(np.ascontiguousarray(ext).view(np.uint8).copy()).to(dev)
    ds = torch.zeros(len(jobs), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.set_profiling(True)
    ms = []
    for _ in range(5):
        dj.copy_(src)
        ctx.integer_search_device(dj.data_ptr(), de.data_ptr(), ds.data_ptr(), len(jobs), s)
        ms.append(ctx.integer_search_last_ms())
    from nnfme.abi import JOB_DTYPE
    out = dj.cpu().numpy().view(JOB_DTYPE)
    np.savez(sys.argv[1], mv_x=out["mv_x"], mv_y=out["mv_y"], sad=ds.cpu().numpy())
    print(f"{os.path.relpath(LIB_PATH, ROOT)}: integer search {np.median(ms[1:]):.3f} ms "
          f"({len(jobs) / np.median(ms[1:]) / 1e3:.1f} M PU/s)", flush=True)


if __name__ == "__main__":
    main()
