"""Bit depth 10 (the main10 configurations, cfg/encoder_lowdelay_P_main10.cfg:58 and
encoder_randomaccess_main10.cfg:60, InternalBitDepth 10) outside the sub-pel batch: the producers'
stages (xGetTemplateCost, TEncSearch.cpp:4397-4436; the bi-pred key of xMotionEstimation(bBi),
4461-4471, TComYuv::removeHighFreq, TComYuv.cpp:411-455) and the P / B predInterSearch loops.

Pinning: the oracle's template cost and bi-pred key at bit depth 10 are checked here against
oracle/_ref, which drives the reference's own TComInterpolationFilter, TComRdCost::getDistPart and
TComYuv::removeHighFreq at bitDepth 10; its integer search against the tz10_* goldens
(tests/test_oracle.py); its sub-pel path against the main10_* goldens.  The producer loops then run
on the GPU against the oracle's (the composition is restated, as at 8 bits: test_pred_inter.py).
Integer outputs: bit-exact."""
import os

import numpy as np
import pytest

from nnfme import abi, synth

W, H = 192, 128


def _pics10(n=5):
    return {i: synth.synth_luma_hbd(W, H, t, bit_depth=10) for i, t in zip(range(n), (7, 6, 5, 4, 0, 3))}


def _setup(eng, pics):
    for k, v in pics.items():
        eng.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        eng.set_lambda(lid, lam)


def _template_requests(rng, n):
    """CUs at every quadtree depth, every PU shape that fits, two candidates per reference, MVs near
    and far (clipMv active) (test_pred_inter._template_requests's stream)."""
    reqs = np.zeros(n, dtype=abi.PU_REQ_DTYPE)
    for i in range(n):
        w, h = synth.ALL_PU_SIZES[int(rng.integers(len(synth.ALL_PU_SIZES)))]
        cu = max(8, 1 << int(np.ceil(np.log2(max(w, h)))))
        cu_x, cu_y = cu * int(rng.integers(0, W // cu)), cu * int(rng.integers(0, H // cu))
        reqs[i]["x"] = cu_x + 4 * int(rng.integers(0, (cu - w) // 4 + 1))
        reqs[i]["y"] = cu_y + 4 * int(rng.integers(0, (cu - h) // 4 + 1))
        reqs[i]["w"], reqs[i]["h"], reqs[i]["cu_x"], reqs[i]["cu_y"] = w, h, cu_x, cu_y
        reqs[i]["depth"] = {64: 0, 32: 1, 16: 2, 8: 3}[cu]
        reqs[i]["org_id"], reqs[i]["num_refs"], reqs[i]["ref_id"] = 4, 4, [0, 1, 2, 3]
        reqs[i]["n_cand"] = [2, 2, 1, 2]
        span = 220 if rng.random() < 0.3 else 40
        reqs[i]["cand"] = rng.integers(-4 * span, 4 * span + 1, (4, 2, 2))
        reqs[i]["lambda_id"] = int(rng.integers(0, 4))
    return reqs


def _reference10(pics):
    from oracle import REF_SO, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    ref = Reference(fast_inter_mode=1, bit_depth=10)
    _setup(ref, pics)
    return ref


def test_main10_oracle_template_cost_matches_reference_harness():
    from oracle import Oracle
    pics = _pics10()
    ref = _reference10(pics)
    orc = Oracle(nn_mode=0, bit_depth=10)
    _setup(orc, pics)
    n = 0
    for q in _template_requests(np.random.default_rng(61), 250):
        for k in range(4):
            for m in range(int(q["n_cand"][k])):
                mx, my = (int(v) for v in q["cand"][k][m])
                want = ref.template_cost(4, int(q["ref_id"][k]), int(q["x"]), int(q["y"]), int(q["w"]), int(q["h"]),
                                         int(q["cu_x"]), int(q["cu_y"]), mx, my, 1, int(q["lambda_id"]))
                assert orc.template_cost(q, k, m) == want, (q, k, m)
                n += 1
    assert n > 1200


def test_main10_oracle_bi_key_matches_reference_harness():
    from oracle import Oracle
    pics = _pics10()
    ref = _reference10(pics)
    orc = Oracle(nn_mode=0, bit_depth=10)
    _setup(orc, pics)
    rng = np.random.default_rng(62)
    seen_over = False
    for (w, h) in synth.ALL_PU_SIZES:
        for t in range(8):
            cu_x, cu_y = 64 * int(rng.integers(0, W // 64)), 64 * int(rng.integers(0, H // 64))
            x = cu_x + 4 * int(rng.integers(0, (64 - w) // 4 + 1))
            y = cu_y + 4 * int(rng.integers(0, (64 - h) // 4 + 1))
            span = 200 if t < 3 else 30
            mvx, mvy = (int(v) for v in rng.integers(-4 * span, 4 * span + 1, 2))
            rid, clip = int(rng.integers(0, 4)), bool(t & 1)
            want = ref.bi_key(4, rid, x, y, w, h, cu_x, cu_y, mvx, mvy, clip)
            got = orc.bi_key(4, rid, x, y, w, h, cu_x, cu_y, mvx, mvy, clip)
            assert np.array_equal(got, want), (w, h, x, y, mvx, mvy, clip)
            if clip:
                assert want.min() >= 0 and want.max() <= 1023
            seen_over |= bool(want.max() > 1023)
    assert seen_over   # unclipped keys leave the 10-bit range (the int16 key path)


# ---- GPU parity (through the C ABI) ---------------------------------------------------------------
@pytest.mark.gpu
def test_main10_gpu_template_costs_match_reference_harness():
    """fme_template_costs on a 10-bit context (k_amvp_sad10) against oracle/_ref at bitDepth 10."""
    from nnfme.runtime import FmeContext
    pics = _pics10()
    ref = _reference10(pics)
    ctx = FmeContext(nn_mode=0, bit_depth=10)
    _setup(ctx, pics)
    reqs = _template_requests(np.random.default_rng(63), 300)
    got = ctx.template_costs(reqs)
    n = 0
    for i, q in enumerate(reqs):
        for k in range(4):
            for m in range(2):
                if m >= int(q["n_cand"][k]):
                    assert got[i, k, m] == 0xFFFFFFFF
                    continue
                mx, my = (int(v) for v in q["cand"][k][m])
                want = ref.template_cost(4, int(q["ref_id"][k]), int(q["x"]), int(q["y"]), int(q["w"]), int(q["h"]),
                                         int(q["cu_x"]), int(q["cu_y"]), mx, my, 1, int(q["lambda_id"]))
                assert got[i, k, m] == want, (i, k, m)
                n += 1
    assert n > 1500


@pytest.mark.gpu
def test_main10_pred_inter_p_matches_oracle():
    """A 10-bit CTU-quadtree P request stream (64 -> 8 CUs, AMP, 4 references, NN on, 5 % lossless)
    on the GPU against the oracle, in two calls (m_integerMv2Nx2N and the NN state cross them)."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics10()
    rng = np.random.default_rng(64)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=3,
                                  lossless_frac=0.05)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1, bit_depth=10)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1, bit_depth=10)
    orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    cut = len(reqs) // 3 + 7
    got = np.concatenate([ctx.pred_inter_p(reqs[:cut]), ctx.pred_inter_p(reqs[cut:])])
    exp = orc.pred_inter_p(reqs)
    for f in abi.PU_RES_DTYPE.names:
        if f == "reserved":
            continue
        bad = got[f] != exp[f]
        if bad.ndim > 1:
            bad = bad.reshape(len(bad), -1).any(axis=1)
        assert not bad.any(), f"{f}: {int(bad.sum())} of {len(bad)} requests differ (first {int(np.flatnonzero(bad)[0])})"
    assert np.array_equal(ctx.nn_get_state(), orc.nn_get_state())
    assert len(np.unique(got["ref_idx"])) > 1


@pytest.mark.gpu
@pytest.mark.parametrize("fen", [1, 0])
def test_main10_pred_inter_b_matches_oracle(fen):
    """A 10-bit B request stream (2 + 2 references, one shared; FEN 1: one bi-pred iteration, FEN 0:
    four) on the GPU against the oracle: the bi-pred keys (k_bi_key10), their integer searches and
    refinements, the uni / bi decision."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics10(6)
    rng = np.random.default_rng(65 + fen)
    reqs = synth.make_pu_requests_b(rng, W, H, org_id=4, l0=[(0, 1), (1, 2)], l1=[(5, -1), (1, 2)], lambda_id=0,
                                    max_depth=3, lossless_frac=0.05)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=fen, bit_depth=10)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=fen, bit_depth=10)
    orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    got = ctx.pred_inter_b(reqs)
    exp = orc.pred_inter_b(reqs)
    for f in abi.PU_RES_B_DTYPE.names:
        if f == "reserved":
            continue
        bad = got[f] != exp[f]
        if bad.ndim > 1:
            bad = bad.reshape(len(bad), -1).any(axis=1)
        assert not bad.any(), f"{f}: {int(bad.sum())} of {len(bad)} requests differ (first {int(np.flatnonzero(bad)[0])})"
    assert np.array_equal(ctx.nn_get_state(), orc.nn_get_state())
    assert set(np.unique(got["inter_dir"])) == {1, 2, 3}
