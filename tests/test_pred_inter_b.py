"""predInterSearch on a B slice (TEncSearch.cpp:3746-4105): fme_pred_inter_b
against the oracle's sequential restatement (orc_pred_inter_b, fme_oracle.c).

What pins what:
  * the pieces: the integer search (orc_integer_search), the sub-pel path (orc_refine) and the AMVP
    template cost are pinned against oracle/_ref elsewhere; the bi-pred key (motionCompensation of
    the other list + TComYuv::removeHighFreq) is pinned here against oracle/_ref, which runs the
    reference's own TComInterpolationFilter and TComYuv::removeHighFreq;
  * the loop: restated from TEncSearch.cpp (which needs Eigen and the whole encoder, SURVEY.md
    §8(c)) in the oracle and, independently, in the GPU runtime's host code (which prices the
    uni-pred tails after the fact and runs bi-pred searches in dependency rounds); the rules the
    loop applies to its outputs are checked a third time here in Python.
Integer outputs: bit-exact."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import ROOT
from nnfme import abi, synth

W, H = 192, 128
L0 = [(0, 1), (1, 2)]            # (picture slot, POC distance) per reference index
L1 = [(5, -1), (1, 2)]           # L1 index 1 is L0 index 1 (getList1IdxToList0Idx = 1)


def _pics():
    return {i: synth.synth_luma(W, H, t) for i, t in zip(range(6), (7, 6, 5, 4, 0, 3))}


def _setup(eng, pics):
    for k, v in pics.items():
        eng.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        eng.set_lambda(lid, lam)


def _reqs(seed, **kw):
    rng = np.random.default_rng(seed)
    return synth.make_pu_requests_b(rng, W, H, org_id=4, l0=L0, l1=L1, lambda_id=0, **kw)


def test_struct_layouts_match_header():
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "fme.h"\nint main(void){printf("%zu %zu %zu %zu %zu %zu '
           '%zu %zu %zu %zu %zu %zu",sizeof(fme_pu_req_b), offsetof(fme_pu_req_b, num_refs),'
           'offsetof(fme_pu_req_b, ref_id), offsetof(fme_pu_req_b, l1_to_l0), offsetof(fme_pu_req_b, cand),'
           'sizeof(fme_pu_res_b), offsetof(fme_pu_res_b, mv), offsetof(fme_pu_res_b, bits),'
           'offsetof(fme_pu_res_b, ref_cost), offsetof(fme_pu_res_b, bi_ref_cost),'
           'offsetof(fme_pu_res_b, bi_ref_mv), offsetof(fme_pu_res_b, ref_mvp_idx));return 0;}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    q, r = abi.PU_REQ_B_DTYPE, abi.PU_RES_B_DTYPE
    assert got == [q.itemsize, q.fields["num_refs"][1], q.fields["ref_id"][1], q.fields["l1_to_l0"][1],
                   q.fields["cand"][1], r.itemsize, r.fields["mv"][1], r.fields["bits"][1], r.fields["ref_cost"][1],
                   r.fields["bi_ref_cost"][1], r.fields["bi_ref_mv"][1], r.fields["ref_mvp_idx"][1]]


def test_request_stream_parts():
    """part_idx counts a CU's PUs (0, 1 for two-PU shapes), cu_w is the CU width, the shared
    reference gets its L0 index."""
    reqs = _reqs(1, max_depth=2)
    assert reqs.dtype == abi.PU_REQ_B_DTYPE
    two = (reqs["part_size"] != abi.PART_2Nx2N) & (reqs["part_size"] != abi.PART_NxN)
    assert set(np.unique(reqs["part_idx"][two])) == {0, 1}
    assert (reqs["part_idx"][reqs["part_size"] == abi.PART_2Nx2N] == 0).all()
    second = np.flatnonzero(two & (reqs["part_idx"] == 1))
    assert (reqs["cu_x"][second] == reqs["cu_x"][second - 1]).all()
    assert (reqs["cu_w"] == 64 >> reqs["depth"].astype(int)).all()
    assert list(reqs["l1_to_l0"][0]) == [-1, 1, -1, -1]


def test_bi_key_matches_reference_harness():
    """The bi-pred search key: the other list's uni-pred luma prediction at a clipMv'd MV and
    removeHighFreq, with and without ClipForBiPredMe, on every PU shape and quarter-pel phase,
    against the reference's own TComInterpolationFilter + TComYuv::removeHighFreq (oracle/_ref)."""
    from oracle import REF_SO, Oracle, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    pics = _pics()
    ref, orc = Reference(fast_inter_mode=1), Oracle(nn_mode=0)
    _setup(orc, pics)
    for k, v in pics.items():
        ref.set_picture(k, v)
    rng = np.random.default_rng(17)
    n = 0
    for (w, h) in synth.ALL_PU_SIZES:
        for t in range(10):
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
                assert want.min() >= 0 and want.max() <= 255
            n += 1
    assert n == 10 * len(synth.ALL_PU_SIZES)


def test_vectorised_bipred_keys_equal_oracle():
    """synth.bipred_keys (what fme_build_bipred_keys computes; the bench's CPU copy of the C4 keys)
    against the oracle's orc_bi_key: every shape, far MVs (clipMv), with and without the clip."""
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(9)
    jobs = synth.make_jobs(rng, W, H, 600, 4, [0, 1, 2, 3], [0], bipred_frac=0.5)
    reqs, kc = synth.make_bipred_key_reqs(rng, jobs, 4, [0, 1, 2, 3], mv_span=300)
    reqs["flags"][::3] = abi.PU_CLIP_BIPRED
    keys = synth.bipred_keys(reqs, pics, kc)
    orc = Oracle(nn_mode=0)
    _setup(orc, pics)
    for q in reqs:
        w, h, o = int(q["w"]), int(q["h"]), int(q["key_offset"])
        want = orc.bi_key(int(q["org_id"]), int(q["ref_id"]), int(q["x"]), int(q["y"]), w, h, int(q["cu_x"]),
                          int(q["cu_y"]), int(q["mv_x"]), int(q["mv_y"]), bool(q["flags"] & abi.PU_CLIP_BIPRED))
        assert np.array_equal(keys[o:o + w * h].reshape(h, w), want), q
    assert len(reqs) > 200


def test_oracle_b_decision_rules():
    """The loop's rules on its own outputs: per-list strict minima, costValidList1 over L1
    references not in L0, the copied L1 reference's MV, isBipredRestriction, the bi-pred list
    (opposite the cheaper uni list), the bi-pred search window around the uni MV, and the final
    uni / bi decision with its MVs and predictors."""
    from nnfme import weights
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(2, max_depth=2)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
    orc.load_nn(weights.load_weights(22))
    _setup(orc, pics)
    res = orc.pred_inter_b(reqs)
    n_bi = 0
    for q, o in zip(reqs, res):
        rc = o["ref_cost"].astype(np.int64)
        c0 = int(rc[0, :2].min())
        assert o["uni_cost"][0] == c0
        valid1 = [k for k in range(2) if q["l1_to_l0"][k] < 0]
        assert o["uni_cost"][1] == min(int(rc[1, k]) for k in valid1)
        assert tuple(o["ref_mv"][1][1]) == tuple(o["ref_mv"][0][1])   # FastMEForGenBLowDelay copy
        restricted = q["cu_w"] == 8 and (q["w"] < 8 or q["h"] < 8)
        if restricted:
            assert o["bi_list"] == 0xFF and o["bi_cost"] == 0xFFFFFFFF and o["inter_dir"] != 3
        else:
            c1_all = int(rc[1, :2].min())
            assert o["bi_list"] == (1 if c0 <= c1_all else 0)
            L = int(o["bi_list"])
            assert o["bi_cost"] == int(o["bi_ref_cost"][:2].min())
            for k in range(2):   # xSetSearchRange(uni MV, 4) then the quarter-pel refinement
                d = np.abs(o["bi_ref_mv"][k].astype(int) - o["ref_mv"][L][k].astype(int))
                assert (d <= 4 * 4 + 2 + 3).all()
        bi = int(o["bi_cost"]) <= c0 and int(o["bi_cost"]) <= int(o["uni_cost"][1])
        if bi:
            n_bi += 1
            assert o["inter_dir"] == 3 and o["cost"] == o["bi_cost"] and o["bits"] == o["bi_bits"]
            L = int(o["bi_list"])
            k = int(o["ref_idx"][L])
            assert tuple(o["mv"][L]) == tuple(o["bi_ref_mv"][k])
            assert o["bi_ref_cost"][k] == o["bi_cost"]
            m = int(o["mvp_idx"][L])
            assert tuple(o["mvp"][L]) == tuple(q["cand"][L][k][m])
        elif c0 <= int(o["uni_cost"][1]):
            assert o["inter_dir"] == 1 and o["cost"] == c0 and tuple(o["mv"][1]) == (0, 0)
            k = int(o["ref_idx"][0])
            assert rc[0, k] == c0 and (rc[0, :k] > c0).all()
            assert tuple(o["mv"][0]) == tuple(o["ref_mv"][0][k])
        else:
            assert o["inter_dir"] == 2 and o["cost"] == o["uni_cost"][1]
            k = int(o["ref_idx"][1])
            assert q["l1_to_l0"][k] < 0 and tuple(o["mv"][1]) == tuple(o["ref_mv"][1][k])
    assert n_bi > 50
    assert set(np.unique(res["inter_dir"])) == {1, 2, 3}


def test_oracle_b_list0_searches_equal_p_slice():
    """Without the NN (nn_mode 0: no carried state), the L0 uni-pred searches of the B loop are the
    P loop's (same AMVP choice, same m_integerMv2Nx2N chain for list 0): equal MVs and AMVP
    indices; only uiMbBits differ, so the costs differ by the re-priced bits alone."""
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(3, max_depth=2)
    p = np.zeros(len(reqs), dtype=abi.PU_REQ_DTYPE)
    for f in ("x", "y", "w", "h", "cu_x", "cu_y", "part_size", "depth", "org_id", "lambda_id", "search_range"):
        p[f] = reqs[f]
    p["flags"] = reqs["flags"] & abi.PU_LOSSLESS
    p["num_refs"] = reqs["num_refs"][:, 0]
    p["ref_id"] = reqs["ref_id"][:, 0]
    p["n_cand"] = reqs["n_cand"][:, 0]
    p["cand"] = reqs["cand"][:, 0]
    ob, op = Oracle(nn_mode=0, fast_inter_mode=1), Oracle(nn_mode=0, fast_inter_mode=1)
    _setup(ob, pics)
    _setup(op, pics)
    rb, rp = ob.pred_inter_b(reqs), op.pred_inter_p(p)
    assert np.array_equal(rb["ref_mv"][:, 0, :2], rp["ref_mv"][:, :2])
    assert np.array_equal(rb["ref_mvp_idx"][:, 0, :2], rp["ref_mvp_idx"][:, :2])


def test_oracle_b_rejects_unsupported():
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(4, max_depth=1)
    orc = Oracle(nn_mode=0, fast_inter_mode=2)
    _setup(orc, pics)
    bad = reqs[:8].copy()
    bad["num_refs"][3] = [1, 0]
    with pytest.raises(RuntimeError):
        orc.pred_inter_b(bad)
    bad = reqs[:8].copy()
    bad["flags"][2] |= 0x10   # no such request flag
    with pytest.raises(RuntimeError):
        orc.pred_inter_b(bad)


def test_oracle_b_fen0_iterations():
    """FEN 0/3 (iNumIter 4, TEncSearch.cpp:3918-4022): iteration 0 searches L0 on the key of the L1
    uni best and always improves on MAX, so a non-restricted PU runs 2..4 iterations, alternating
    lists (the last one searched is (iters - 1) % 2); its bi cost never exceeds the FEN-2 search of
    L0 with the same key when FEN 2 also picks L0 (FEN 0 and 2 share the full-row metric; on a
    CU's first PU uiMbBits does not depend on an earlier decision).  FEN 3 is FEN 0's loop with
    the even-row metric of FEN 1.  With bi chosen, each list's MV is a searched MV of that list (or the uni MV of the
    list never searched)."""
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(5, max_depth=2)
    res = {}
    for fen in (0, 2, 3):
        o = Oracle(nn_mode=0, fast_inter_mode=fen)
        _setup(o, pics)
        res[fen] = o.pred_inter_b(reqs)
    restricted = (reqs["cu_w"] == 8) & ((reqs["w"] < 8) | (reqs["h"] < 8))
    for fen in (0, 3):
        r = res[fen]
        it = r["bi_iters"].astype(int)
        assert (it[restricted] == 0).all() and (r["bi_list"][restricted] == 0xFF).all()
        assert it[~restricted].min() >= 2 and it.max() <= 4
        assert (r["bi_list"][~restricted] == (it[~restricted] - 1) % 2).all()
        assert len(set(it[~restricted])) == 3, np.bincount(it)   # 2, 3 and 4 all occur
    r0, r1 = res[0], res[2]
    first = reqs["part_idx"] == 0
    assert np.array_equal(r0["ref_cost"][first], r1["ref_cost"][first])
    assert np.array_equal(r0["uni_cost"][first], r1["uni_cost"][first])
    same_first = ~restricted & first & (r1["bi_list"] == 0)
    assert same_first.sum() > 20
    assert (r0["bi_cost"][same_first] <= r1["bi_cost"][same_first]).all()
    assert (r0["bi_cost"][~restricted] < 0xFFFFFFFF).all()
    assert (r0["inter_dir"] == 3).sum() > 50


def test_oracle_b_mvd_l1_zero():
    """MvdL1ZeroFlag (lowdelay B, both lists the same pictures; TEncSearch.cpp:3805-3810, 3876-3925):
    list 1 at the AMVP predictor of least template cost over its references (zero MVD), one L0
    iteration; L0 uni-pred and the L1 uni searches as without the flag."""
    from oracle import Oracle
    pics = _pics()
    l = [(0, 1), (1, 2)]
    rng = np.random.default_rng(6)
    reqs = synth.make_pu_requests_b(rng, W, H, org_id=4, l0=l, l1=l, lambda_id=0, max_depth=2, mvd_l1_zero=True)
    plain = reqs.copy()
    plain["flags"] &= np.uint8(0xFF ^ abi.PU_MVD_L1_ZERO)
    o, p = Oracle(nn_mode=0, fast_inter_mode=0), Oracle(nn_mode=0, fast_inter_mode=0)
    _setup(o, pics)
    _setup(p, pics)
    r, rp = o.pred_inter_b(reqs), p.pred_inter_b(plain)
    first = reqs["part_idx"] == 0   # (a second PU's uiMbBits follows its CU's first decision)
    assert np.array_equal(r["ref_cost"][first], rp["ref_cost"][first])
    assert np.array_equal(r["uni_cost"][first], rp["uni_cost"][first])
    restricted = (reqs["cu_w"] == 8) & ((reqs["w"] < 8) | (reqs["h"] < 8))
    assert (r["bi_iters"][~restricted] == 1).all() and (r["bi_list"][~restricted] == 0).all()
    bi = np.flatnonzero(r["inter_dir"] == 3)
    assert len(bi) > 20
    for i in bi:
        assert tuple(r["mv"][i][1]) == tuple(r["mvp"][i][1])   # zero MVD in list 1
        k = int(r["ref_idx"][i][1])
        assert tuple(r["mvp"][i][1]) == tuple(reqs["cand"][i][1][k][int(r["mvp_idx"][i][1])])
    # the template costs decide list 1 (xGetTemplateCost with the candidate's index bits)
    p1 = _as_p(reqs, 1)
    for i in bi[:100]:
        q = reqs[i]
        best, kb, mb = None, 0, 0
        for k in range(int(q["num_refs"][1])):
            c = [o.template_cost(p1[i], k, m) for m in range(int(q["n_cand"][1][k]))]
            m = int(np.argmin(c))
            if best is None or c[m] < best:
                best, kb, mb = c[m], k, m
        assert (int(r["ref_idx"][i][1]), int(r["mvp_idx"][i][1])) == (kb, mb), i


def _as_p(reqs, l):
    """The list-l view of B requests as fme_pu_req (the P-slice request layout)."""
    p = np.zeros(len(reqs), dtype=abi.PU_REQ_DTYPE)
    for f in ("x", "y", "w", "h", "cu_x", "cu_y", "part_size", "depth", "org_id", "lambda_id", "search_range"):
        p[f] = reqs[f]
    p["num_refs"] = reqs["num_refs"][:, l]
    p["ref_id"] = reqs["ref_id"][:, l]
    p["n_cand"] = reqs["n_cand"][:, l]
    p["cand"] = reqs["cand"][:, l]
    return p


# ---- GPU parity (through the C ABI) ---------------------------------------------------------------
def _compare(got, exp):
    for f in abi.PU_RES_B_DTYPE.names:
        if f == "reserved":
            continue
        bad = got[f] != exp[f]
        if bad.ndim > 1:
            bad = bad.reshape(len(bad), -1).any(axis=1)
        assert not bad.any(), f"{f}: {int(bad.sum())} of {len(bad)} requests differ (first {int(np.flatnonzero(bad)[0])})"


@pytest.mark.gpu
def test_pred_inter_b_matches_oracle():
    """A CTU-quadtree B-frame request stream (64 -> 8 CUs, AMP, 2 + 2 references with one shared,
    NN on, 5 % lossless) on the GPU against the oracle, in two calls (the cut falls between the two
    PUs of no CU) so that m_integerMv2Nx2N and the NN state cross calls."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(21, max_depth=3, lossless_frac=0.05)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
    orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    cut = len(reqs) // 3
    while reqs["part_idx"][cut] != 0:
        cut += 1
    got = np.concatenate([ctx.pred_inter_b(reqs[:cut]), ctx.pred_inter_b(reqs[cut:])])
    exp = orc.pred_inter_b(reqs)
    _compare(got, exp)
    assert np.array_equal(ctx.nn_get_state(), orc.nn_get_state())
    assert set(np.unique(got["inter_dir"])) == {1, 2, 3}


@pytest.mark.gpu
def test_device_bipred_keys_drive_refine_like_host_keys():
    """fme_build_bipred_keys (k_bi_key) gives the keys synth.bipred_keys computes: bi-pred refine
    jobs read them and equal the same jobs on host-uploaded keys (and the oracle)."""
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(10)
    jobs = synth.make_jobs(rng, W, H, 800, 4, [0, 1, 2, 3], [0, 1, 2, 3], bipred_frac=0.6)
    reqs, kc = synth.make_bipred_key_reqs(rng, jobs, 4, [0, 1, 2, 3], mv_span=200)
    reqs["flags"][::4] = abi.PU_CLIP_BIPRED
    keys = synth.bipred_keys(reqs, pics, kc)
    dev_ctx, host_ctx = FmeContext(nn_mode=1, qp=22), FmeContext(nn_mode=1, qp=22)
    for c in (dev_ctx, host_ctx):
        _setup(c, pics)
    dev_ctx.build_bipred_keys(reqs, kc)
    host_ctx.set_keys(keys)
    a, b = dev_ctx.refine(jobs), host_ctx.refine(jobs)
    assert a.tobytes() == b.tobytes()
    orc = Oracle(nn_mode=1, qp=22)
    from nnfme import weights
    orc.load_nn(weights.load_weights(22))
    _setup(orc, pics)
    orc.set_keys(keys)
    want = orc.refine(jobs)
    for f in ("mv_x", "mv_y", "cost", "bits", "frac_cost"):
        assert np.array_equal(a[f], want[f]), f
    bad = reqs.copy()
    bad["key_offset"][3] += 2   # not a multiple of 4
    from nnfme.runtime import FmeError
    with pytest.raises(FmeError):
        dev_ctx.build_bipred_keys(bad, kc)


@pytest.mark.gpu
def test_pred_inter_b_clip_no_fast_me_and_rejection():
    """ClipForBiPredMe on, FastMEForGenBLowDelay off (the shared reference searched in L1 too),
    FEN 2, SAD metric, NN off; then the rejected batches."""
    from nnfme.runtime import FmeContext, FmeError
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(22, max_depth=2, fast_me_gen_b=False, clip_bipred=True)[:700]
    ctx = FmeContext(nn_mode=0, use_hadamard=0, fast_inter_mode=2)
    orc = Oracle(nn_mode=0, use_hadamard=0, fast_inter_mode=2)
    _setup(ctx, pics)
    _setup(orc, pics)
    _compare(ctx.pred_inter_b(reqs), orc.pred_inter_b(reqs))
    bad = reqs.copy()
    bad["n_cand"][9][1][0] = 3
    with pytest.raises(FmeError):
        ctx.pred_inter_b(bad)
    second = int(np.flatnonzero(reqs["part_idx"] == 1)[0])
    with pytest.raises(FmeError):   # a second PU without its CU's first PU before it
        ctx.pred_inter_b(reqs[second:])
    bad = reqs.copy()
    bad["flags"][5] |= 0x10   # no such request flag
    with pytest.raises(FmeError):
        ctx.pred_inter_b(bad)
    assert len(ctx.pred_inter_b(reqs[:0])) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("fen,nn", [(0, 1), (3, 0)])
def test_pred_inter_b_fen_iterations_match_oracle(fen, nn):
    """FEN 0 / 3: up to four bi-pred iterations per PU, run by the host in rounds (one fme_refine
    per round), against the oracle's sequential loop; NN on for FEN 0 (the carried state across
    the rounds' repeated uni jobs)."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics()
    reqs = _reqs(23, max_depth=2, lossless_frac=0.03)
    kw = dict(nn_mode=nn, qp=22, fast_inter_mode=fen)
    ctx, orc = FmeContext(**kw), Oracle(**kw)
    if nn:
        orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    got, exp = ctx.pred_inter_b(reqs), orc.pred_inter_b(reqs)
    _compare(got, exp)
    assert set(np.unique(got["bi_iters"])) >= {2, 3, 4}
    if nn:
        assert np.array_equal(ctx.nn_get_state(), orc.nn_get_state())


@pytest.mark.gpu
def test_pred_inter_b_mvd_l1_zero_matches_oracle():
    """MvdL1ZeroFlag on a lowdelay-B stream (both lists the same two pictures, FEN 1, NN on):
    list 1 at its best template-cost predictor, one L0 iteration."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics()
    l = [(0, 1), (1, 2)]
    rng = np.random.default_rng(24)
    reqs = synth.make_pu_requests_b(rng, W, H, org_id=4, l0=l, l1=l, lambda_id=0, max_depth=2, mvd_l1_zero=True)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
    orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    got, exp = ctx.pred_inter_b(reqs), orc.pred_inter_b(reqs)
    _compare(got, exp)
    assert (got["inter_dir"] == 3).sum() > 20
