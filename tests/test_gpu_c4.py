"""configs[3] at full size through the HIP path: one 2560x1600 random-access QP27 frame batch.

≈1.33 M xMotionEstimation jobs in HM's CTU order (40 x 25 CTUs x 333 calls x 4 references),
20.5 % of them bi-pred iterations whose FracDIF key is TComYuv::removeHighFreq of the other
list's uni-pred prediction (TEncSearch.cpp:4461-4471, TComYuv.cpp:411-455), built on the
device by fme_build_bipred_keys / fme_build_bipred_keys_device (k_bi_key); the RA GOP-8 lambda
(TEncSlice.cpp:246-325).  Checked by size-independent properties, as the 1080p frame of
test_gpu_parity.py is:
  * the stream-ordered key builder gives the same results as the synchronous one;
  * run-to-run determinism and batch-split invariance of the carried NN state;
  * every per-job field against the oracle (keys from synth.bipred_keys, the vectorised
    restatement that oracle/ pins against the reference's removeHighFreq) on 3,000 sampled jobs,
    bi-pred ones included;
  * the NN class of every job against the float32 restatement (nn_host_emulation);
  * the tail's MV from the class.
"""
import numpy as np
import pytest

from nnfme import synth, weights
from nnfme.abi import JOB_BIPRED, compare_results

from test_gpu_parity import _assert_same, nn_host_emulation

pytestmark = pytest.mark.gpu

W, H, QP = 2560, 1600, 27
ORG = 4
LAMBDA = synth.ra_lambda(QP, 1)   # GOP-8 entry 1 (POC 4, depth 1): the Clip3(2, 4, ...) branch


@pytest.fixture(scope="module")
def frame_c4():
    rng = np.random.default_rng(3027)
    pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs = synth.make_ctu_jobs(rng, W, H, 333, ORG, [0, 1, 2, 3], [0], bipred_frac=0.205)
    reqs, key_count = synth.make_bipred_key_reqs(np.random.default_rng(77), jobs, ORG, [0, 1, 2, 3])
    return pics, jobs, reqs, key_count


def _c4_ctx(pics):
    from nnfme.runtime import FmeContext
    ctx = FmeContext(nn_mode=1, qp=QP, fast_inter_mode=1, max_jobs=1400000)
    for k, v in pics.items():
        ctx.set_picture(k, v)
    ctx.set_lambda(0, LAMBDA)
    return ctx


def test_c4_frame_full_size(frame_c4):
    import torch
    from oracle import Oracle
    pics, jobs, reqs, key_count = frame_c4
    n = len(jobs)
    assert n > 1_300_000
    bi = (jobs["flags"] & JOB_BIPRED) != 0
    assert 0.19 < bi.mean() < 0.22

    ctx = _c4_ctx(pics)
    ctx.build_bipred_keys(reqs, key_count)
    a = ctx.refine(jobs)
    assert not np.any(a["status"] & 0x8000), "batch rejected"

    # stream-ordered key building (the frame replay's per-frame path) == the synchronous one
    dev = torch.device("cuda", 0)
    d_reqs = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
    ctx2 = _c4_ctx(pics)
    s = torch.cuda.current_stream(dev)
    ctx2.build_bipred_keys_device(d_reqs.data_ptr(), len(reqs), key_count, s.cuda_stream)
    b = ctx2.refine(jobs)
    _assert_same(b, a, "device-built keys")

    # determinism and batch-split invariance
    ctx.nn_reset()
    _assert_same(ctx.refine(jobs), a, "rerun")
    ctx.nn_reset()
    k = n // 3
    _assert_same(np.concatenate([ctx.refine(jobs[:k]), ctx.refine(jobs[k:])]), a, "split")

    # the oracle on a sample (NN off there: per-job fields are independent of the carried state)
    rng = np.random.default_rng(11)
    sel = np.sort(np.concatenate([rng.choice(np.flatnonzero(bi), 1000, replace=False),
                                  rng.choice(np.flatnonzero(~bi), 2000, replace=False)]))
    keys = synth.bipred_keys(reqs, pics, key_count)
    o = Oracle(nn_mode=0, qp=QP)
    for kk, v in pics.items():
        o.set_picture(kk, v)
    o.set_lambda(0, LAMBDA)
    o.set_keys(keys)
    ro = o.refine(jobs[sel])
    fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi")   # + the pushed emi values
    bad, first, counts = compare_results(a[sel], ro, fields)
    assert bad == 0, f"c4 sample: {bad} mismatches, first {first}: {counts}"

    # NN class of every job (bi-pred jobs repeat the carried state's class) and the tail's MV
    cls = nn_host_emulation(jobs, a, weights.load_weights(QP))
    mism = np.flatnonzero(cls != a["nn_class"])
    assert len(mism) == 0, f"{len(mism)} NN class mismatches, first {mism[:5]}"
    assert np.array_equal(a["mv_x"], 4 * a["mv_int_x"].astype(np.int32) + a["nn_class"] % 7 - 3)
    assert np.array_equal(a["mv_y"], 4 * a["mv_int_y"].astype(np.int32) + a["nn_class"] // 7 - 3)


def test_replay_builds_keys_per_frame():
    """FrameReplay with bi-pred key requests: each step uploads its frames' requests and builds
    their keys on the device from that step's pictures; the replayed results (MV, cost, bits, NN
    class, carried state across frames) equal the oracle run frame after frame with each frame's
    own pictures and keys."""
    import torch
    from nnfme import pipeline
    from nnfme.abi import MV_RESULT_DTYPE
    from nnfme.pipeline import FrameReplay
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    w, h, F, steps = 416, 240, 2, 3
    rng = np.random.default_rng(41)
    base = synth.make_ctu_jobs(rng, w, h, 120, 4, [0, 1, 2, 3], [0], bipred_frac=0.2)
    reqs, kc = synth.make_bipred_key_reqs(np.random.default_rng(42), base, 4, [0, 1, 2, 3])
    pool = np.stack([synth.synth_luma(w, h, t) for t in range(8)])
    lam = lambda f: synth.ra_lambda(QP, f % 8)   # noqa: E731
    ctx = FmeContext(nn_mode=1, qp=QP, fast_inter_mode=1)
    rep = FrameReplay(ctx, base, pool, lam, steps, frames_per_step=F, device=torch.device("cuda", 0),
                      key_reqs=reqs, key_count=kc)
    rep.prime()
    for k in range(steps):
        rep.issue(k)
    rep.finish()
    o = Oracle(nn_mode=1, qp=QP)
    o.load_nn(weights.load_weights(QP))
    for k in range(steps):
        f0 = rep.first_frame(k)
        pics = {pipeline.ORG0 + j: pool[(f0 + j) % 8] for j in range(F)}
        pics.update({s: pool[(f0 - pipeline.REFS + s) % 8] for s in range(F + pipeline.REFS - 1)})
        for kk, v in pics.items():
            o.set_picture(kk, v)
        for j in range(F):
            o.set_lambda(j, lam(f0 + j))
        o.set_keys(synth.bipred_keys(rep.kreqs, pics, kc * F))
        want = o.refine(rep.jobs)
        got = rep.results(k)
        for f in ("mv_x", "mv_y", "cost", "bits", "nn_class"):
            bad = np.flatnonzero(got[f] != want[f])
            assert len(bad) == 0, f"step {k}: {f} differs at {len(bad)} jobs, first {bad[:5]}"
    assert got.dtype == MV_RESULT_DTYPE
