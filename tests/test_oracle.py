"""CPU tests of the oracle: pinned against the golden vectors (made by oracle/_ref, the
reference's own compiled primitives) and, where the reference is present, re-checked live."""
import os

import numpy as np
import pytest

from conftest import (golden_bit_depth, tz_golden_cases, mc_golden_cases, mc10_golden_cases, mc_inputs, golden_cases, load_golden,
                      main10_golden_cases)
from nnfme import synth, weights
from nnfme.abi import PARITY_FIELDS, compare_results
from oracle import REF_SO, Oracle, Reference

HAVE_REF = os.path.exists(REF_SO)


def _engine(cls, g):
    hadme, fen, nn_mode, qp = (int(v) for v in g["config"])
    kw = dict(use_hadamard=hadme, nn_mode=nn_mode, fast_inter_mode=fen,
              bit_depth=int(g["bit_depth"][0]) if "bit_depth" in g else 8)
    if cls is Oracle:
        kw["qp"] = qp
    e = cls(**kw)
    for i, p in enumerate(g["pictures"]):
        e.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        e.set_lambda(i, float(lam))
    e.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    e.load_nn(weights.load_weights(qp))
    if "net" in g:
        e.load_nn_net(weights.case_net(str(g["net"])))
    return e


@pytest.mark.parametrize("case", golden_cases())
def test_oracle_matches_golden(case):
    g = load_golden(case)
    res = _engine(Oracle, g).refine(g["jobs"])
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{case}: {bad} mismatching jobs, first {first}: {counts}"


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("case", golden_cases())
def test_reference_harness_matches_golden(case):
    g = load_golden(case)
    res = _engine(Reference, g).refine(g["jobs"])
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{case}: {bad} mismatching jobs, first {first}: {counts}"


@pytest.mark.parametrize("case", main10_golden_cases())
def test_main10_oracle_matches_golden(case):
    """Bit depth 10 (main10): the plain-C restatement's interpolation (headRoom 4: first-stage shift
    2, second-stage shift 10, clip to 1023) and distortions (>> 2, SSE (d * d) >> 4 per sample)
    against _ref's TComInterpolationFilter / TComRdCost run at bitDepth 10."""
    g = load_golden(case)
    assert int(g["bit_depth"][0]) == 10 and g["pictures"].dtype == np.uint16 and g["pictures"].max() > 255
    res = _engine(Oracle, g).refine(g["jobs"])
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{case}: {bad} mismatching jobs, first {first}: {counts}"


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("case", main10_golden_cases())
def test_main10_reference_harness_matches_golden(case):
    g = load_golden(case)
    res = _engine(Reference, g).refine(g["jobs"])
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{case}: {bad} mismatching jobs, first {first}: {counts}"


def test_main10_goldens_cover_every_pu_shape():
    seen, flags = set(), 0
    for case in main10_golden_cases():
        j = load_golden(case)["jobs"]
        seen |= set(zip(j["w"].tolist(), j["h"].tolist()))
        flags |= int(np.bitwise_or.reduce(j["flags"]))
    assert set(synth.ALL_PU_SIZES) <= seen
    assert flags == 0x7


def test_golden_covers_every_pu_shape_and_flag():
    seen, flags = set(), 0
    for case in golden_cases():
        j = load_golden(case)["jobs"]
        seen |= set(zip(j["w"].tolist(), j["h"].tolist()))
        flags |= int(np.bitwise_or.reduce(j["flags"]))
    assert set(synth.ALL_PU_SIZES) <= seen
    assert flags == 0x7


@pytest.mark.parametrize("case", mc_golden_cases())
def test_mc_oracle_matches_golden(case):
    """orc_mc (plain-C restatement) against the reference's motion compensation."""
    g = load_golden(case)
    pics, jobs, (y, cb, cr) = mc_inputs(g)
    Oracle().mc(pics, jobs, y, cb, cr)
    for got, exp, comp in ((y, g["pred_y"], "Y"), (cb, g["pred_cb"], "Cb"), (cr, g["pred_cr"], "Cr")):
        assert np.array_equal(got, exp), f"{case} {comp}: {int((got != exp).sum())} samples differ"


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
@pytest.mark.parametrize("seed,bi,amp", [(31, 0.0, 8), (32, 0.5, 64), (33, 0.8, 600)])
def test_mc_oracle_matches_reference_random(seed, bi, amp):
    """Random frame partitions (every PU shape, bi-pred, identical motion, MVs far outside the
    picture so clipMv bites) through orc_mc and the reference's filters + addAvg."""
    from nnfme import synth
    W, H = 200, 136
    rng = np.random.default_rng(seed)
    pics = {}
    ref = Reference()
    for k in range(4):
        cb, cr = synth.synth_chroma(W, H, k, seed=seed)
        pics[k] = (synth.synth_luma(W, H, k, seed=seed), cb, cr)
        ref.set_picture_yuv(k, *pics[k])
    jobs = synth.make_mc_partition(rng, W, H, [0, 1, 2, 3], bi_frac=bi, mv_amp=amp, identical_frac=0.2)
    outs = []
    for eng in ("orc", "ref"):
        y, cb, cr = np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8)
        if eng == "orc":
            Oracle().mc(pics, jobs, y, cb, cr)
        else:
            ref.mc(jobs, y, cb, cr)
        outs.append((y, cb, cr))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
@pytest.mark.parametrize("case", mc10_golden_cases())
def test_mc10_golden_is_the_reference(case):
    """The main10 MC fixtures are oracle/_ref's output at bitDepth 10 (the reference's own
    TComInterpolationFilter and TComYuv::addAvg): recomputed here, bit for bit."""
    g = load_golden(case)
    assert int(g["bit_depth"][0]) == 10
    pics, jobs, (y, cb, cr) = mc_inputs(g)
    ref = Reference(bit_depth=10)
    for k, p in pics.items():
        ref.set_picture_yuv(k, *p)
    ref.mc(jobs, y, cb, cr)
    for got, exp, comp in ((y, g["pred_y"], "Y"), (cb, g["pred_cb"], "Cb"), (cr, g["pred_cr"], "Cr")):
        assert got.dtype == np.uint16 and np.array_equal(got, exp), f"{case} {comp}"


def test_mc10_goldens_cover_bi_clip_and_range():
    bi = uni = 0
    for case in mc10_golden_cases():
        g = load_golden(case)
        bi += int(((g["jobs"]["flags"] & 3) == 3).sum())
        uni += int(((g["jobs"]["flags"] & 3) != 3).sum())
        assert g["pred_y"].max() > 255 and g["pred_y"].max() <= 1023   # really 10-bit samples
    assert bi > 50 and uni > 50 and len(mc10_golden_cases()) >= 3


def test_mc_golden_covers_cases():
    shapes, flags, clipped = set(), set(), False
    for case in mc_golden_cases():
        g = load_golden(case)
        j = g["jobs"]
        shapes |= set(zip(j["w"].tolist(), j["h"].tolist()))
        flags |= set(j["flags"].tolist())
        W = g["pred_y"].shape[1]
        clipped |= bool(((j["mv"][:, :, 0] >> 2) + j["x"][:, None] > W + 8).any())
    assert len(shapes) >= 20 and flags == {1, 2, 3} and clipped


def _tz_engine(cls, g):
    fen, _ = (int(v) for v in g["config"])
    eng = cls(fast_inter_mode=fen, bit_depth=golden_bit_depth(g))
    for i, p in enumerate(g["pictures"]):
        eng.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        eng.set_lambda(i, float(lam))
    eng.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    return eng


@pytest.mark.parametrize("case", tz_golden_cases())
def test_tz_oracle_matches_golden(case):
    """orc_integer_search (xTZSearch / xPatternSearch restated) against the reference harness's run."""
    g = load_golden(case)
    jobs, sad = _tz_engine(Oracle, g).integer_search(g["jobs"], g["ext"])
    assert np.array_equal(jobs["mv_x"], g["mv_x"]) and np.array_equal(jobs["mv_y"], g["mv_y"])
    assert np.array_equal(sad, g["sad"])


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
@pytest.mark.parametrize("case", tz_golden_cases())
def test_tz_reference_harness_matches_golden(case):
    g = load_golden(case)
    jobs, sad = _tz_engine(Reference, g).integer_search(g["jobs"], g["ext"])
    assert np.array_equal(jobs["mv_x"], g["mv_x"]) and np.array_equal(jobs["mv_y"], g["mv_y"])
    assert np.array_equal(sad, g["sad"])


def test_tz_golden_covers_cases():
    from nnfme.abi import JOB_BIPRED, TZ_ENHANCED, TZ_FULL, TZ_PRED2NX2N
    shapes, bi, pred, far, sr, modes = set(), 0, 0, 0, set(), {0: 0, TZ_FULL: 0, TZ_ENHANCED: 0}
    for case in tz_golden_cases():
        g = load_golden(case)
        j = g["jobs"]
        e = g["ext"]["base"] if g["ext"].dtype.names[0] == "base" else g["ext"]
        shapes |= set(zip(j["w"].tolist(), j["h"].tolist()))
        bi += int(((j["flags"] & JOB_BIPRED) != 0).sum())
        pred += int(((e["flags"] & TZ_PRED2NX2N) != 0).sum())
        far += int((np.abs(g["mv_x"] * 4 - j["mvp_x"]) > 4 * 32).sum())   # raster-search territory
        sr.add(int(g["config"][1]))
        uni = (j["flags"] & JOB_BIPRED) == 0
        for m in modes:
            modes[m] += int((uni & ((e["flags"] & (TZ_FULL | TZ_ENHANCED)) == m)).sum())
    assert len(shapes) >= 18 and bi > 100 and pred > 300 and far > 50 and {32, 64} <= sr
    # FastSearch 1 (diamond), 0 (full) and 3 (enhanced diamond) each on > 100 uni-pred jobs
    assert min(modes.values()) > 100, modes


def test_exp_golomb_bits():
    o = Oracle()
    # TComRdCost::xGetExpGolombNumberOfBits: 0 -> 1, 1 -> 3, -1 -> 3, 2 -> 5 ...
    expect = {0: 1, 1: 3, -1: 3, 2: 5, -2: 5, 3: 5, -3: 5, 4: 7, 255: 17, -255: 17, -256: 19, 256: 19}
    for v, b in expect.items():
        assert o.lib.orc_eg_bits(v) == b, v


def test_cost_is_truncated_double():
    o = Oracle()
    ml = 65536.0 * np.sqrt(20.196)
    for b in range(0, 80):
        assert o.lib.orc_cost(ml, b) == int((ml * b) / 65536.0)


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
def test_prediction_matches_reference_filters():
    rng = np.random.default_rng(3)
    pic = synth.synth_luma(96, 64, 0, seed=21)
    o, r = Oracle(), Reference()
    r.set_picture(0, pic)
    for _ in range(300):
        w, h = synth.ALL_PU_SIZES[int(rng.integers(len(synth.ALL_PU_SIZES)))]
        x, y = int(rng.integers(0, 96 - w + 1)), int(rng.integers(0, 64 - h + 1))
        qx, qy = int(rng.integers(-200, 200)), int(rng.integers(-200, 200))
        np.testing.assert_array_equal(o.pred_block(pic, x, y, w, h, qx, qy), r.pred_block(0, x, y, w, h, qx, qy))


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
def test_satd_matches_reference():
    rng = np.random.default_rng(4)
    o, r = Oracle(), Reference()
    for w, h in synth.ALL_PU_SIZES:
        a = rng.integers(-255, 511, (h, w)).astype(np.int16)
        b = rng.integers(0, 256, (h, w)).astype(np.int16)
        assert o.lib.orc_satd(a.ctypes.data, w, b.ctypes.data, w, w, h) == r.satd(a, b, True)
        assert o.lib.orc_sad(a.ctypes.data, w, b.ctypes.data, w, w, h, 0) == r.satd(a, b, False)


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_nn_class_matches_harness(qp):
    rng = np.random.default_rng(qp)
    o, r = Oracle(qp=qp), Reference()
    wts = weights.load_weights(qp)
    r.load_nn(wts)
    for _ in range(500):
        e = rng.integers(0, 400000, 8).astype(np.uint32)
        c = int(rng.integers(0, 400000))
        h, w = synth.ALL_PU_SIZES[int(rng.integers(len(synth.ALL_PU_SIZES)))][::-1]
        assert o.nn_class(wts, e, c, h, w)[0] == r.nn_class(e, c, h, w)


def test_parity_fields_complete():
    assert {"mv_x", "mv_y", "cost", "frac_cost", "nn_class"} <= set(PARITY_FIELDS)
