"""GPU probe: exact vs MFMA NN engines (nn_mode 2) on one 1080p frame, per net.

Prints class agreement, the exact engine's top-1 minus top-2 margin distribution, and the margins
of the disagreeing jobs, so an MFMA layout bug (large margins) is told apart from rounding (ties).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))

import torch  # noqa: E402

from nnfme import synth, weights  # noqa: E402
from nnfme.runtime import FmeContext  # noqa: E402


def run(pics, jobs, name, engine):
    ctx = FmeContext(nn_mode=2, net=weights.case_net(name), nn_engine=engine, qp=22, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    m = torch.zeros(len(jobs), dtype=torch.float32, device="cuda")
    ctx.set_nn_margin_output(m.data_ptr())
    res = ctx.refine(jobs)
    ctx.set_nn_margin_output(0)
    ctx.close()
    return res, m.cpu().numpy()


def main():
    W, H = 1920, 1080
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    rng = np.random.default_rng(2023)
    pics = {i: synth.synth_luma(W, H, i) for i in range(5)}
    jobs = synth.make_ctu_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [1])[:n]
    for name in ("master", "blowing4x40+rezero", "scr3x40"):
        ex, mex = run(pics, jobs, name, 0)
        mf, mmf = run(pics, jobs, name, 1)
        dis = ex["nn_class"] != mf["nn_class"]
        print(f"{name}: jobs {len(jobs)} agree {1 - dis.mean():.6f} classes {len(np.unique(ex['nn_class']))}")
        print(f"  exact margin pct 1/5/50: {np.percentile(mex, [1, 5, 50])}")
        if dis.any():
            idx = np.flatnonzero(dis)
            print(f"  disagreeing: {len(idx)}; exact margins pct 50/99: {np.percentile(mex[idx], [50, 99])}; "
                  f"mfma margins pct 50: {np.percentile(mmf[idx], 50)}")
            print(f"  first: {idx[:8]} ex {ex['nn_class'][idx[:8]]} mf {mf['nn_class'][idx[:8]]} (i % 64: {idx[:8] % 64})")
            print(f"  disagreement by lane (i % 64) histogram: {np.bincount(idx % 64, minlength=64)}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
