"""GPU parity of the integer motion estimation: fme_integer_search
(xTZSearch for uni-pred jobs, xPatternSearch for bi-pred jobs) against the golden vectors made by
the reference harness (oracle/_ref) and the C restatement (orc_integer_search).  Integer output
(MV, ruiSAD): bit-exact."""
import numpy as np
import pytest

from conftest import golden_bit_depth, load_golden, tz_golden_cases
from nnfme import synth
from nnfme.abi import JOB_BIPRED, TZ_EXT_DTYPE

pytestmark = pytest.mark.gpu


def _ctx(g=None, fen=1, bit_depth=8):
    from nnfme.runtime import FmeContext
    if g is not None:
        fen = int(g["config"][0])
        bit_depth = golden_bit_depth(g)
    ctx = FmeContext(nn_mode=0, fast_inter_mode=fen, bit_depth=bit_depth)
    if g is not None:
        for i, p in enumerate(g["pictures"]):
            ctx.set_picture(i, p)
        for i, lam in enumerate(g["lambdas"]):
            ctx.set_lambda(i, float(lam))
        if g["keys"].size:
            ctx.set_keys(g["keys"])
    return ctx


@pytest.mark.parametrize("case", tz_golden_cases())
def test_tz_golden(case):
    g = load_golden(case)
    jobs, sad = _ctx(g).integer_search(g["jobs"], g["ext"])
    bad = (jobs["mv_x"] != g["mv_x"]) | (jobs["mv_y"] != g["mv_y"]) | (sad != g["sad"])
    assert not bad.any(), f"{case}: {int(bad.sum())} of {len(bad)} jobs differ (first {int(np.flatnonzero(bad)[0])})"
    # only the MV fields change
    for f in ("x", "y", "w", "h", "mvp_x", "mvp_y", "lt_x", "rb_y", "flags", "key_offset"):
        assert np.array_equal(jobs[f], g["jobs"][f])


def test_tz_1080p_sample_matches_oracle():
    """A 1080p frame of integer-search jobs (4 refs, 15 % bi-pred full searches, 2Nx2N starts,
    predictors up to 40 px off so raster searches run) on the GPU; a 2,500-job random sample
    against the C oracle, and run-to-run determinism of the whole frame."""
    from oracle import Oracle
    W, H = 1920, 1080
    rng = np.random.default_rng(17)
    pics = {i: synth.synth_luma(W, H, t) for i, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs, ext = synth.make_tz_jobs(rng, W, H, 60, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=0.15, mvp_noise=160)
    keys = synth.make_bipred_keys_fast(rng, jobs, pics)
    ctx = _ctx()
    orc = Oracle(fast_inter_mode=1)
    for eng in (ctx, orc):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
            eng.set_lambda(lid, lam)
        eng.set_keys(keys)
    got, sad = ctx.integer_search(jobs, ext)
    got2, sad2 = ctx.integer_search(jobs, ext)
    assert np.array_equal(got, got2) and np.array_equal(sad, sad2)
    idx = np.sort(rng.choice(len(jobs), 2500, replace=False))
    exp, esad = orc.integer_search(jobs[idx], ext[idx])
    bad = (got["mv_x"][idx] != exp["mv_x"]) | (got["mv_y"][idx] != exp["mv_y"]) | (sad[idx] != esad)
    assert not bad.any(), f"{int(bad.sum())} of {len(idx)} sampled jobs differ"
    assert ((jobs["flags"][idx] & JOB_BIPRED) != 0).sum() > 100


def test_tz_then_refine_matches_oracle_chain():
    """xMotionEstimation end to end on the GPU: integer search, then the sub-pel path (EMI step,
    FracDIF, NN, tail) on its output, against the oracle chain."""
    from nnfme import weights
    from nnfme.abi import compare_results
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    g = load_golden("tz_ldp_fen1")
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
    orc.load_nn(weights.load_weights(22))
    for eng in (ctx, orc):
        for i, p in enumerate(g["pictures"]):
            eng.set_picture(i, p)
        for i, lam in enumerate(g["lambdas"]):
            eng.set_lambda(i, float(lam))
        eng.set_keys(g["keys"])
    jobs, _ = ctx.integer_search(g["jobs"], g["ext"])
    ojobs, _ = orc.integer_search(g["jobs"], g["ext"])
    bad, first, counts = compare_results(ctx.refine(jobs), orc.refine(ojobs))
    assert bad == 0, f"{bad} jobs differ, first {first}: {counts}"


def test_tz_device_and_timing():
    import torch
    g = load_golden("tz_far_fen0_sr32")
    ctx = _ctx(g)
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(g["jobs"].view(np.uint8).copy()).to(dev)
    de = torch.from_numpy(np.ascontiguousarray(g["ext"]).view(np.uint8).copy()).to(dev)
    ds = torch.zeros(len(g["jobs"]), dtype=torch.int32, device=dev)
    ctx.set_profiling(True)
    ctx.integer_search_device(dj.data_ptr(), de.data_ptr(), ds.data_ptr(), len(g["jobs"]),
                              torch.cuda.current_stream(dev).cuda_stream)
    assert ctx.integer_search_last_ms() > 0
    from nnfme.abi import JOB_DTYPE
    out = dj.cpu().numpy().view(JOB_DTYPE)
    assert np.array_equal(out["mv_x"], g["mv_x"]) and np.array_equal(out["mv_y"], g["mv_y"])
    assert np.array_equal(ds.cpu().numpy().view(np.uint32), g["sad"])
    # invalid job -> rejected, nothing written
    from nnfme.runtime import FmeError
    bad = g["jobs"].copy()
    bad["w"][3] = 6
    with pytest.raises(FmeError):
        ctx.integer_search(bad, g["ext"])
    assert TZ_EXT_DTYPE.itemsize == 12


@pytest.mark.parametrize("case", ["tz_enhanced_fen1", "tz_full_sr8_fen1", "tz10_enhanced_fen1", "tz10_full_sr8_fen3"])
def test_tz2_device_and_mode_flags(case):
    """FastSearch 0 / 3 (fme_tz_ext2) through the device entry point; the same jobs through the
    12-byte records search with zero neighbour predictors, as the oracle does."""
    import torch
    sys_path_oracle()
    from oracle import Oracle
    from nnfme.abi import JOB_DTYPE
    g = load_golden(case)
    ctx = _ctx(g)
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(g["jobs"].view(np.uint8).copy()).to(dev)
    de = torch.from_numpy(np.ascontiguousarray(g["ext"]).view(np.uint8).copy()).to(dev)
    ds = torch.zeros(len(g["jobs"]), dtype=torch.int32, device=dev)
    ctx.integer_search2_device(dj.data_ptr(), de.data_ptr(), ds.data_ptr(), len(g["jobs"]),
                               torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    out = dj.cpu().numpy().view(JOB_DTYPE)
    assert np.array_equal(out["mv_x"], g["mv_x"]) and np.array_equal(out["mv_y"], g["mv_y"])
    assert np.array_equal(ds.cpu().numpy().view(np.uint32), g["sad"])
    base = np.ascontiguousarray(g["ext"]["base"])
    jobs, sad = ctx.integer_search(g["jobs"], base)
    orc = Oracle(fast_inter_mode=int(g["config"][0]), bit_depth=golden_bit_depth(g))
    for i, p in enumerate(g["pictures"]):
        orc.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        orc.set_lambda(i, float(lam))
    orc.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    ref_jobs, ref_sad = orc.integer_search(g["jobs"], base)
    assert np.array_equal(jobs["mv_x"], ref_jobs["mv_x"]) and np.array_equal(jobs["mv_y"], ref_jobs["mv_y"])
    assert np.array_equal(sad, ref_sad)


def sys_path_oracle():
    import os
    import sys
    from conftest import ROOT
    p = os.path.join(ROOT, "oracle")
    if p not in sys.path:
        sys.path.insert(0, p)


def test_tz_staged_uneven_groups():
    """k_tz_staged runs one workgroup of 8 waves per (unit-shape kernel, reference, CTU) group, wave w
    taking the group's PUs w, w + 8, ...: groups of 1, 2, 7, 8, 9, 15, 16, 17 and 40 PUs (waves with
    no PU, with one, with several) all give the oracle's MVs and SADs.  (The static wave-to-PU order
    keeps each wave's PU index wave-uniform by construction: a readfirstlane of the wave index plus
    a constant stride; tz_wave's candidate lists and minima assume a wave-uniform job.)"""
    sys_path_oracle()
    from oracle import Oracle
    W, H = 448, 192   # 7 x 3 CTUs
    rng = np.random.default_rng(77)
    pics = {i: synth.synth_luma(W, H, i, seed=77) for i in range(5)}
    jobs, ext = synth.make_tz_jobs(rng, W, H, 60, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=0.0)
    ctu = (jobs["y"].astype(int) // 64) * 7 + jobs["x"].astype(int) // 64
    kid = np.where(jobs["w"] % 8 != 0, 0, np.where(jobs["h"] % 8 != 0, 1, 2))
    sizes = [1, 2, 7, 8, 9, 15, 16, 17, 40]
    keep = np.zeros(len(jobs), bool)
    for c in range(21):
        for r in range(4):
            for k in range(3):
                idx = np.flatnonzero((ctu == c) & (jobs["ref_id"] == r) & (kid == k))
                want = sizes[(c * 12 + r * 3 + k) % len(sizes)]
                keep[idx[:want]] = True
    jobs, ext = jobs[keep], ext[keep]
    orc = Oracle(fast_inter_mode=1)
    ctx = _ctx(fen=1)
    for eng in (orc, ctx):
        for k, v in pics.items():
            eng.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
            eng.set_lambda(lid, lam)
    ref_jobs, ref_sad = orc.integer_search(jobs, ext)
    got, sad = ctx.integer_search(jobs, ext)
    bad = (got["mv_x"] != ref_jobs["mv_x"]) | (got["mv_y"] != ref_jobs["mv_y"]) | (sad != ref_sad)
    assert not bad.any(), f"{int(bad.sum())} of {len(jobs)} jobs differ"
