#!/usr/bin/env python3
"""Generate tests/golden/*.npz — TEST INFRASTRUCTURE ONLY (run in the build container).

Expected outputs come from oracle/_ref/libhmref.so: the reference's own TLibCommon sources
(TComInterpolationFilter, TComRdCost, TComPicYuv, TComPrediction scratch planes) compiled
from /root/reference and driven in TEncSearch's order by oracle/ref_harness.cpp.  Every case
is also run through the plain-C oracle (fme_oracle.c); generation aborts on any mismatch.

Each fixture holds inputs and outputs only (data): pictures, lambdas, bi-pred key blocks,
jobs (fme_job records), results (fme_result records) and the configuration.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, os.path.join(ROOT, "hm16.9-nn_fme_amd")]

from oracle import Oracle, Reference  # noqa: E402
from nnfme import synth, weights  # noqa: E402
from nnfme.abi import JOB_BIPRED, JOB_EMI, JOB_LOSSLESS, compare_results  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def edge_jobs(rng, width, height, n):
    """Jobs that hit the corners: search-range edges (< 8 EMI pushes), picture borders with MVs
    pointing outside (edge replication), the largest PUs."""
    sizes = [s for s in synth.ALL_PU_SIZES]
    picks = [sizes[i % len(sizes)] for i in range(n)]
    w = np.array([p[0] for p in picks])
    h = np.array([p[1] for p in picks])
    j = synth.make_jobs(rng, width, height, n, 4, [0, 1, 2], [0, 1, 2, 3], sizes=(w, h))
    for i in range(n):
        kind = i % 6
        if kind == 0:      # TZ best on the left/top range edge
            j["mv_x"][i] = j["lt_x"][i]
            j["mv_y"][i] = j["lt_y"][i]
        elif kind == 1:    # right/bottom edge
            j["mv_x"][i] = j["rb_x"][i]
            j["mv_y"][i] = j["rb_y"][i]
        elif kind == 2:    # PU at the top-left corner, MV far outside
            j["x"][i] = 0
            j["y"][i] = 0
            j["mv_x"][i] = max(int(j["lt_x"][i]), -60)
            j["mv_y"][i] = max(int(j["lt_y"][i]), -60)
        elif kind == 3:    # bottom-right corner
            j["x"][i] = (width - j["w"][i]) // 4 * 4
            j["y"][i] = (height - j["h"][i]) // 4 * 4
        elif kind == 4:    # degenerate range: a single column
            j["lt_x"][i] = j["rb_x"][i] = j["mv_x"][i]
        else:              # lossless CU (SAD in FracDIF)
            j["flags"][i] = JOB_EMI | JOB_LOSSLESS
    # the search range must contain the start point (xTZSearch invariant)
    return j


def build_case(name, seed, width, height, n_jobs, hadme, fen, nn_mode, qp, bipred=0.15, n_edge=96):
    rng = np.random.default_rng(seed)
    pics = {i: synth.synth_luma(width, height, i, seed=seed) for i in range(5)}
    lambdas = np.array(synth.LDP_LAMBDA[qp if qp in synth.LDP_LAMBDA else 22], dtype=np.float64)
    a = synth.make_jobs(rng, width, height, n_jobs, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=bipred)
    b = edge_jobs(rng, width, height, n_edge)
    jobs = np.concatenate([b[:8], a, b[8:]])
    # recompute the bi-pred keys over the final order
    jobs["key_offset"][(jobs["flags"] & JOB_BIPRED) != 0] = -2
    keys = synth.make_bipred_keys(rng, jobs, pics)
    ref = Reference(use_hadamard=hadme, nn_mode=nn_mode, fast_inter_mode=fen)
    orc = Oracle(use_hadamard=hadme, nn_mode=nn_mode, qp=qp, fast_inter_mode=fen)
    wts = weights.load_weights(qp)
    for eng in (ref, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(lambdas):
            eng.set_lambda(lid, float(lam))
        eng.set_keys(keys if keys.size else np.zeros(1, np.int16))
        eng.load_nn(wts)
    r_ref = ref.refine(jobs)
    r_orc = orc.refine(jobs)
    bad, first, counts = compare_results(r_ref, r_orc)
    if bad:
        raise SystemExit(f"{name}: oracle disagrees with _ref on {bad} jobs (first {first}): {counts}")
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(
        path,
        pictures=np.stack([pics[i] for i in range(5)]),
        lambdas=lambdas,
        keys=keys,
        jobs=jobs,
        results=r_ref,
        config=np.array([hadme, fen, nn_mode, qp], dtype=np.int32),
    )
    print(f"{path}: {len(jobs)} jobs, {int((jobs['flags'] & JOB_BIPRED != 0).sum())} bi-pred, "
          f"{int((r_ref['n_emi'] < 8).sum())} with < 8 EMI pushes")


CASES = [
    # name, seed, W, H, jobs, HADME, FEN, nn_mode, QP
    ("ldp_qp22_hadme_fen1_nn", 11, 160, 96, 1200, 1, 1, 1, 22),
    ("sad_fen0_nnoff", 12, 160, 96, 600, 0, 0, 0, 22),
    ("fen3_qp27_nn", 13, 128, 96, 400, 1, 3, 1, 27),
    ("qp32_nn", 14, 128, 96, 400, 1, 1, 1, 32),
    ("qp37_nn", 15, 128, 96, 400, 1, 1, 1, 37),
]


def main():
    os.makedirs(OUT, exist_ok=True)
    for c in CASES:
        build_case(*c)
    return 0


if __name__ == "__main__":
    sys.exit(main())
