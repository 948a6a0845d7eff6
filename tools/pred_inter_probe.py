#!/usr/bin/env python3
"""predInterSearch producer (fme_pred_inter_p) on one 1080p P frame of CTU-quadtree requests
(64 -> 8 CUs, AMP, 4 references, NN on): wall time per frame and requests / jobs per second.

usage: python tools/pred_inter_probe.py [max_depth] [height]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hm16.9-nn_fme_amd"), os.path.join(ROOT, "oracle")]


def main():
    from nnfme import synth
    from nnfme.runtime import FmeContext
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    W, H = 1920, int(sys.argv[2]) if len(sys.argv) > 2 else 1080
    rng = np.random.default_rng(2)
    pics = {i: synth.synth_luma(W, H, t) for i, t in zip(range(5), (7, 6, 5, 4, 0))}
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=depth)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1, max_jobs=4 * len(reqs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    ctx.pred_inter_p(reqs)   # warm-up
    ts = []
    for _ in range(3):
        ctx.pred_inter_reset()
        t0 = time.perf_counter()
        res = ctx.pred_inter_p(reqs)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    nj = int(reqs["num_refs"].astype(np.int64).sum())
    print(f"pred_inter_p {W}x{H} depth {depth}: {len(reqs)} PU requests ({nj} xMotionEstimation jobs) in {t * 1e3:.1f} ms "
          f"-> {len(reqs) / t / 1e6:.2f} M requests/s, {nj / t / 1e6:.2f} M jobs/s; ref_idx histogram "
          f"{np.bincount(res['ref_idx'], minlength=4).tolist()}", flush=True)
    print("pred_inter phases (ms, last frame):",
          {k: round(v, 2) for k, v in ctx.pred_inter_phases().items()}, flush=True)
    # the B slice of bench.py's producer leg: L0 = {t-1, t-2}, L1 = {t+1, t+2}, FEN 1
    ctx.set_picture(5, synth.synth_luma(W, H, 3))
    reqs_b = synth.make_pu_requests_b(np.random.default_rng(3), W, H, org_id=4, l0=[(0, 1), (1, 2)],
                                      l1=[(5, -1), (2, -2)], lambda_id=0, max_depth=depth)
    ctx.pred_inter_b(reqs_b)   # warm-up
    ts = []
    for _ in range(3):
        ctx.pred_inter_reset()
        t0 = time.perf_counter()
        ctx.pred_inter_b(reqs_b)
        ts.append(time.perf_counter() - t0)
    print(f"pred_inter_b {W}x{H} depth {depth}: {len(reqs_b)} PU requests in {np.median(ts) * 1e3:.1f} ms; phases (ms):",
          {k: round(v, 2) for k, v in ctx.pred_inter_phases().items()}, flush=True)
    # CPU: the oracle's sequential restatement on a bounded sample (first CTU rows)
    if os.environ.get("CPU", "1") == "1":
        from oracle import Oracle
        from nnfme import weights
        orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
        orc.load_nn(weights.load_weights(22))
        for k, v in pics.items():
            orc.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
            orc.set_lambda(lid, lam)
        sample = reqs[:20000]
        t0 = time.perf_counter()
        orc.pred_inter_p(sample)
        tc = time.perf_counter() - t0
        print(f"oracle (1 core, sequential): {len(sample)} requests in {tc:.2f} s -> {len(sample) / tc / 1e3:.1f} K requests/s",
              flush=True)


if __name__ == "__main__":
    main()
