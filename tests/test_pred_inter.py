"""predInterSearch's P-slice PU / reference loop: fme_pred_inter_p against
the oracle's sequential restatement (orc_pred_inter_p, fme_oracle.c), which composes the pinned
integer search (orc_integer_search) and sub-pel path (orc_refine) with the AMVP template cost
(xGetTemplateCost, TEncSearch.cpp:4397-4436), the bit counts (xGetBlkBits 4286-4333, the
reference-index bits 3792-3800, xGetMvpIdxBits 4258-4284), xCheckBestMVP (4344-4394) and the
reference choice (3845-3853).  The composition itself has no reference fixture (TEncSearch.cpp
needs Eigen): its pieces are pinned, the glue is restated twice (C oracle, host
runtime) and once more here in Python for the AMVP / xCheckBestMVP / reference-choice rules.
Integer outputs: bit-exact."""
import os

import numpy as np
import pytest

from conftest import ROOT
from nnfme import abi, synth

W, H = 192, 128


def _pics():
    return {i: synth.synth_luma(W, H, t) for i, t in zip(range(5), (7, 6, 5, 4, 0))}


def _setup(eng, pics):
    for k, v in pics.items():
        eng.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        eng.set_lambda(lid, lam)


# ---- pure-Python restatements of the small host rules (checked against the oracle) -------------
def mvp_idx_bits(idx, num):
    """xGetMvpIdxBits (TEncSearch.cpp:4258-4284)."""
    if num == 1:
        return 0
    if idx == 0:
        return 1
    return 1 + (idx - 1) + (1 if num - 1 > idx else 0)


def eg_bits(v):
    """TComRdCost::xGetExpGolombNumberOfBits (TComRdCost.cpp:172-185)."""
    t = (-v << 1) + 1 if v <= 0 else v << 1
    n = 1
    while t != 1:
        t >>= 1
        n += 2
    return n


def test_struct_layouts_match_header():
    import subprocess
    import tempfile
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "fme.h"\nint main(void){printf("%zu %zu %zu %zu %zu '
           '%zu %zu %zu %zu %zu",sizeof(fme_pu_req), offsetof(fme_pu_req, ref_id), offsetof(fme_pu_req, cand),'
           'offsetof(fme_pu_req, lambda_id), offsetof(fme_pu_req, flags), sizeof(fme_pu_res),'
           'offsetof(fme_pu_res, bits), offsetof(fme_pu_res, ref_cost), offsetof(fme_pu_res, ref_mv),'
           'offsetof(fme_pu_res, ref_mvp_idx));return 0;}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    q, r = abi.PU_REQ_DTYPE, abi.PU_RES_DTYPE
    assert got == [q.itemsize, q.fields["ref_id"][1], q.fields["cand"][1], q.fields["lambda_id"][1],
                   q.fields["flags"][1], r.itemsize, r.fields["bits"][1], r.fields["ref_cost"][1],
                   r.fields["ref_mv"][1], r.fields["ref_mvp_idx"][1]]
    assert q.itemsize == 64 and r.itemsize == 80


def test_mvp_idx_bits_table():
    """m_auiMVPIdxCost as TEncSearch::init fills it (TEncSearch.cpp:412-425), AMVP_MAX_NUM_CANDS = 2."""
    assert [mvp_idx_bits(i, 2) for i in range(2)] == [1, 1]
    assert mvp_idx_bits(0, 1) == 0
    assert [eg_bits(v) for v in (0, 1, -1, 2, -2, 3, 7, -8)] == [1, 3, 3, 5, 5, 5, 7, 9]


def test_request_stream_shape():
    """The synthetic producer input walks xCompressCU's order: per CU 2Nx2N, 2NxN, Nx2N, the
    four AMP shapes (CUs > 8), then the four sub-CUs."""
    rng = np.random.default_rng(3)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=3)
    assert reqs.dtype == abi.PU_REQ_DTYPE
    ctus = ((W + 63) // 64) * ((H + 63) // 64)
    assert len(reqs) == ctus * (21 * 13 + 64 * 5)
    assert (reqs["x"].astype(int) + reqs["w"] <= W).all() and (reqs["y"].astype(int) + reqs["h"] <= H).all()
    first = reqs[0]
    assert first["part_size"] == abi.PART_2Nx2N and first["depth"] == 0 and first["w"] == 64


def test_oracle_single_ref_one_candidate_is_the_plain_chain():
    """With one reference and one AMVP candidate the producer is xMotionEstimation itself: the
    integer search from the predictor, then the sub-pel path, bits_in = the block bits + 1."""
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(5)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0], lambda_id=1, max_depth=1)
    reqs["n_cand"][:, 0] = 1
    reqs = reqs[(reqs["part_size"] != abi.PART_2Nx2N) & (reqs["depth"] == 0)]   # no writer: reads see (0, 0)
    orc = Oracle(nn_mode=0, fast_inter_mode=1)
    _setup(orc, pics)
    res = orc.pred_inter_p(reqs)
    jobs, ext = synth.pu_requests_to_jobs(reqs, W, H)
    orc2 = Oracle(nn_mode=0, fast_inter_mode=1)
    _setup(orc2, pics)
    ij, _ = orc2.integer_search(jobs, ext)
    r = orc2.refine(ij)
    assert np.array_equal(res["mv_x"], r["mv_x"]) and np.array_equal(res["mv_y"], r["mv_y"])
    assert np.array_equal(res["cost"], r["cost"]) and np.array_equal(res["bits"], r["bits"])
    assert (res["ref_idx"] == 0).all() and (res["mvp_idx"] == 0).all()


def test_oracle_amvp_choice_and_check_best_mvp():
    """The AMVP index is the first candidate with the least template cost (luma prediction at the
    clipMv'd candidate, SAD + bits * mlambda / 65536); xCheckBestMVP then moves it only to a
    candidate with strictly fewer MV bits; the reference is the strict cost minimum."""
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(11)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=1)[:100]
    orc = Oracle(nn_mode=0, fast_inter_mode=1)
    _setup(orc, pics)
    res = orc.pred_inter_p(reqs)
    org = pics[4].astype(np.int64)
    ml = 65536.0 * np.sqrt(synth.LDP_LAMBDA[22][0])
    moved = 0
    for i, q in enumerate(reqs):
        x, y, w, h = int(q["x"]), int(q["y"]), int(q["w"]), int(q["h"])
        best = None
        for k in range(int(q["num_refs"])):
            nc = int(q["n_cand"][k])
            costs = []
            for c in range(nc):
                mx = int(synth._clip_cu_qpel(int(q["cand"][k][c][0]), int(q["cu_x"]), W))
                my = int(synth._clip_cu_qpel(int(q["cand"][k][c][1]), int(q["cu_y"]), H))
                pred = orc.pred_block(pics[int(q["ref_id"][k])], x, y, w, h, mx, my)
                sad = int(np.abs(pred.astype(np.int64) - org[y:y + h, x:x + w]).sum())
                costs.append(int(sad + (mvp_idx_bits(c, 2) * ml) / 65536.0))
            amvp = int(np.argmin(costs))
            mv = (int(res["ref_mv"][i][k][0]), int(res["ref_mv"][i][k][1]))
            bits = [eg_bits(mv[0] - int(q["cand"][k][c][0])) + eg_bits(mv[1] - int(q["cand"][k][c][1])) +
                    mvp_idx_bits(c, 2) for c in range(nc)]
            fin = int(res["ref_mvp_idx"][i][k])
            if fin != amvp:
                assert bits[fin] < bits[amvp] and bits[fin] == min(bits)
                moved += 1
            else:
                assert bits[fin] <= min(bits)
            cost = int(res["ref_cost"][i][k])
            if best is None or cost < best[0]:
                best = (cost, k)
        assert int(res["ref_idx"][i]) == best[1] and int(res["cost"][i]) == best[0]
        k = best[1]
        assert (int(res["mv_x"][i]), int(res["mv_y"][i])) == tuple(int(v) for v in res["ref_mv"][i][k])
        c = int(res["mvp_idx"][i])
        assert (int(res["mvp_x"][i]), int(res["mvp_y"][i])) == tuple(int(v) for v in q["cand"][k][c])
    assert len(np.unique(res["ref_idx"])) > 1


# ---- GPU parity (through the C ABI) ---------------------------------------------------------------
@pytest.mark.gpu
def test_pred_inter_matches_oracle():
    """A CTU-quadtree request stream (64 -> 8 CUs, AMP, 4 references, NN on, 5 % lossless) on the
    GPU against the oracle, in two calls so that m_integerMv2Nx2N and the NN state cross calls."""
    from nnfme import weights
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(21)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1, 2, 3], lambda_id=0, max_depth=3,
                                  lossless_frac=0.05)
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1)
    orc = Oracle(nn_mode=1, qp=22, fast_inter_mode=1)
    orc.load_nn(weights.load_weights(22))
    _setup(ctx, pics)
    _setup(orc, pics)
    cut = len(reqs) // 3 + 7
    got = np.concatenate([ctx.pred_inter_p(reqs[:cut]), ctx.pred_inter_p(reqs[cut:])])
    exp = orc.pred_inter_p(reqs)
    for f in ("mv_x", "mv_y", "mvp_x", "mvp_y", "ref_idx", "mvp_idx", "bits", "cost", "ref_cost", "ref_bits",
              "ref_mv", "ref_mvp_idx"):
        bad = got[f] != exp[f]
        if bad.ndim > 1:
            bad = bad.reshape(len(bad), -1).any(axis=1)
        assert not bad.any(), f"{f}: {int(bad.sum())} of {len(bad)} requests differ (first {int(np.flatnonzero(bad)[0])})"
    assert np.array_equal(ctx.nn_get_state(), orc.nn_get_state())
    assert len(np.unique(got["ref_idx"])) > 1


@pytest.mark.gpu
def test_pred_inter_reset_and_rejection():
    from nnfme.runtime import FmeContext, FmeError
    from oracle import Oracle
    pics = _pics()
    rng = np.random.default_rng(8)
    reqs = synth.make_pu_requests(rng, W, H, org_id=4, ref_ids=[0, 1], lambda_id=2, max_depth=2)[:300]
    ctx = FmeContext(nn_mode=0, fast_inter_mode=0)
    _setup(ctx, pics)
    a = ctx.pred_inter_p(reqs)
    ctx.pred_inter_reset()
    b = ctx.pred_inter_p(reqs)
    assert a.tobytes() == b.tobytes()
    orc = Oracle(nn_mode=0, fast_inter_mode=0)
    _setup(orc, pics)
    assert orc.pred_inter_p(reqs).tobytes() == a.tobytes()
    bad = reqs.copy()
    bad["num_refs"][5] = 0
    with pytest.raises(FmeError):
        ctx.pred_inter_p(bad)
    bad = reqs.copy()
    bad["n_cand"][9][0] = 3
    with pytest.raises(FmeError):
        ctx.pred_inter_p(bad)
    assert len(ctx.pred_inter_p(reqs[:0])) == 0


def test_template_cost_matches_reference_harness():
    """xGetTemplateCost (TEncSearch.cpp:4397-4436) as the producer and oracle compute it (clipMv'd
    luma prediction, SAD, SAD + bits * mlambda / 65536) against the reference's own
    TComInterpolationFilter / TComRdCost::getDistPart / calcRdCost (oracle/_ref), on every PU shape,
    every quarter-pel phase and MVs far enough out for clipMv to act."""
    from oracle import REF_SO, Oracle, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    pics = _pics()
    ref = Reference(fast_inter_mode=1)
    orc = Oracle(nn_mode=0)
    for k, v in pics.items():
        ref.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ref.set_lambda(lid, lam)
    rng = np.random.default_rng(31)
    org = pics[4].astype(np.int64)
    n = 0
    for (w, h) in synth.ALL_PU_SIZES:
        for _ in range(12):
            # a PU inside its (64x64) CU, as getPartIndexAndSize gives it: clipMv keeps the reads
            # inside the padded picture only for such geometry
            cu_x, cu_y = 64 * int(rng.integers(0, W // 64)), 64 * int(rng.integers(0, H // 64))
            x = cu_x + 4 * int(rng.integers(0, (64 - w) // 4 + 1))
            y = cu_y + 4 * int(rng.integers(0, (64 - h) // 4 + 1))
            span = 200 if rng.random() < 0.3 else 40
            mvx, mvy = (int(v) for v in rng.integers(-4 * span, 4 * span + 1, 2))
            lid, bits, rid = int(rng.integers(0, 4)), int(rng.integers(0, 3)), int(rng.integers(0, 4))
            cx = int(synth._clip_cu_qpel(mvx, cu_x, W))
            cy = int(synth._clip_cu_qpel(mvy, cu_y, H))
            pred = orc.pred_block(pics[rid], x, y, w, h, cx, cy)
            sad = int(np.abs(pred.astype(np.int64) - org[y:y + h, x:x + w]).sum())
            ml = 65536.0 * np.sqrt(synth.LDP_LAMBDA[22][lid])
            want = int(sad + (bits * ml) / 65536.0)
            got = ref.template_cost(4, rid, x, y, w, h, cu_x, cu_y, mvx, mvy, bits, lid)
            assert got == want, (w, h, x, y, mvx, mvy, got, want)
            n += 1
    assert n == 12 * len(synth.ALL_PU_SIZES)


def _template_requests(rng, n):
    """Requests whose CU sits at any depth of the quadtree (origins on the 64/32/16/8 grid, so not
    64-aligned below depth 0), every PU shape that fits the CU, two candidates per reference with
    MVs near and far (clipMv active)."""
    reqs = np.zeros(n, dtype=abi.PU_REQ_DTYPE)
    sizes = [s for s in synth.ALL_PU_SIZES]
    for i in range(n):
        w, h = sizes[int(rng.integers(len(sizes)))]
        cu = max(8, 1 << int(np.ceil(np.log2(max(w, h)))))
        cu_x = cu * int(rng.integers(0, W // cu))
        cu_y = cu * int(rng.integers(0, H // cu))
        x = cu_x + 4 * int(rng.integers(0, (cu - w) // 4 + 1))
        y = cu_y + 4 * int(rng.integers(0, (cu - h) // 4 + 1))
        reqs[i]["x"], reqs[i]["y"], reqs[i]["w"], reqs[i]["h"] = x, y, w, h
        reqs[i]["cu_x"], reqs[i]["cu_y"] = cu_x, cu_y
        reqs[i]["depth"] = {64: 0, 32: 1, 16: 2, 8: 3}[cu]
        reqs[i]["org_id"] = 4
        reqs[i]["num_refs"] = 4
        reqs[i]["ref_id"] = [0, 1, 2, 3]
        reqs[i]["n_cand"] = [2, 2, 1, 2]
        span = 220 if rng.random() < 0.3 else 40
        reqs[i]["cand"] = rng.integers(-4 * span, 4 * span + 1, (4, 2, 2))
        reqs[i]["lambda_id"] = int(rng.integers(0, 4))
    return reqs


def test_oracle_template_cost_matches_reference_harness():
    """The oracle's own xGetTemplateCost (the one its predInterSearch loop uses: clipMv +
    mc_pred_blk + SAD + calcRdCost) against oracle/_ref's, which drives the reference's
    TComInterpolationFilter and TComRdCost, per (request, reference, candidate), CUs at every depth."""
    from oracle import REF_SO, Oracle, Reference
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    pics = _pics()
    ref, orc = Reference(fast_inter_mode=1), Oracle(nn_mode=0)
    _setup(orc, pics)
    for k, v in pics.items():
        ref.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ref.set_lambda(lid, lam)
    reqs = _template_requests(np.random.default_rng(44), 300)
    n = 0
    for q in reqs:
        for k in range(4):
            for m in range(int(q["n_cand"][k])):
                mx, my = (int(v) for v in q["cand"][k][m])
                want = ref.template_cost(4, int(q["ref_id"][k]), int(q["x"]), int(q["y"]), int(q["w"]), int(q["h"]),
                                         int(q["cu_x"]), int(q["cu_y"]), mx, my, 1, int(q["lambda_id"]))   # m_auiMVPIdxCost[m][2] = 1
                assert orc.template_cost(q, k, m) == want, (q, k, m)
                n += 1
    assert n > 1500


@pytest.mark.gpu
def test_gpu_template_costs_match_reference_harness():
    """fme_template_costs (the producer's AMVP stage, k_amvp_sad) against oracle/_ref's
    xGetTemplateCost over the reference's own filters and RdCost, CUs at every depth."""
    from oracle import REF_SO, Reference
    from nnfme.runtime import FmeContext
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built")
    pics = _pics()
    ctx = FmeContext(nn_mode=0)
    _setup(ctx, pics)
    ref = Reference(fast_inter_mode=1)
    for k, v in pics.items():
        ref.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ref.set_lambda(lid, lam)
    reqs = _template_requests(np.random.default_rng(45), 400)
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
    assert n > 2000
