"""The backups' own NN input path (BASELINE.json configs[4]).

Backups/4 ("SCR 3 layers") and Backups/15 ("blowing 4 lyrs qp 22") push every xTZSearchHelp
distortion into array_e, end xTZSearch with xTZ8PointSquareSearch (distance 1) and
xTZ8PointSquareSearch2 (distance 2) around the star best, and feed NN_pred C = the least push
before that square and array_e[index_ref .. +7] (Backups/4:659, 4343-4359, 4868-4878, 876-965).
Library: fme_integer_search_ring (FME_TZ_RING) writes those nine inputs per job; fme_refine takes
them for FME_JOB_NN_IN jobs from the rows bound with fme_set_nn_inputs (net flag
FME_NN_IN_TZ_RING).  Goldens: oracle/gen_golden.py build_ring_case (oracle/_ref, the oracle agreeing).

CPU: the oracle and _ref reproduce the goldens.  GPU: the integer search and the exact engine are
bit-exact against them, the MFMA engine within the deep-net tolerance of test_deep_nn.py.
"""
import numpy as np
import pytest

from conftest import load_golden, ring_golden_cases
from nnfme import weights
from nnfme.abi import JOB_BIPRED, JOB_NN_IN, RES_NN_STALE, RES_REJECTED, TZ_RING, compare_results
from oracle import REF_SO, Oracle, Reference
import os

HAVE_REF = os.path.exists(REF_SO)


def _engines(g, which):
    fen = int(g["config"][1])
    net = weights.case_net(str(g["net"]))
    e = Oracle(use_hadamard=1, nn_mode=2, fast_inter_mode=fen) if which == "oracle" else \
        Reference(use_hadamard=1, nn_mode=2, fast_inter_mode=fen)
    for i, p in enumerate(g["pictures"]):
        e.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        e.set_lambda(i, float(lam))
    e.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    e.load_nn_net(net)
    return e


def _check_tz(g, jobs, sad, nn_in, who):
    bad = (jobs["mv_x"] != g["mv_x"]) | (jobs["mv_y"] != g["mv_y"]) | (sad != g["sad"]) | \
        (nn_in != g["nn_in"]).any(axis=1)
    assert not bad.any(), f"{who}: {int(bad.sum())} of {len(bad)} integer searches differ " \
                          f"(first {int(np.flatnonzero(bad)[0])})"


@pytest.mark.parametrize("case", ring_golden_cases())
@pytest.mark.parametrize("which", ["oracle", "ref"])
def test_ring_golden_cpu(case, which):
    if which == "ref" and not HAVE_REF:
        pytest.skip("oracle/_ref not built")
    g = load_golden(case)
    e = _engines(g, which)
    jobs, sad, nn_in = e.integer_search_ring(g["jobs"], g["ext"])
    _check_tz(g, jobs, sad, nn_in, which)
    e.set_nn_inputs(g["nn_in"])
    res = e.refine(g["refine_jobs"])
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{which}: {bad} refinements differ (first {first}): {counts}"


def test_ring_goldens_exercise_the_path():
    """The fixtures cover what the path does differently: the square + ring moves the integer MV,
    C is below every input slot it was compared with, bi-pred jobs take the last uni-pred inputs."""
    moved = total = 0
    for case in ring_golden_cases():
        g = load_golden(case)
        uni = (g["jobs"]["flags"] & JOB_BIPRED) == 0
        assert (g["ext"]["flags"][uni] & TZ_RING).all()
        o = _engines(g, "oracle")
        plain, _ = o.integer_search(g["jobs"], g["ext"])   # the same searches without the ring
        moved += int((((plain["mv_x"] != g["mv_x"]) | (plain["mv_y"] != g["mv_y"])) & uni).sum())
        total += int(uni.sum())
        nn = g["nn_in"][uni]
        assert (nn[:, 8] <= nn[:, :8].max(axis=1)).all()   # C: min over a superset-free prefix
        o.set_nn_inputs(g["nn_in"])
        r = o.refine(g["refine_jobs"])   # (the goldens hold _ref's records, which carry no status bits)
        bi = np.flatnonzero(~uni)
        assert len(bi) > 10 and (r["status"][bi] & RES_NN_STALE).all() and not (r["status"][uni] & RES_NN_STALE).any()
        # a bi-pred job's class is the last uni-pred job's (the backups never run NN for it)
        for i in bi[:50]:
            prev = np.flatnonzero(uni[:i])
            if len(prev):
                assert r["nn_class"][i] == r["nn_class"][prev[-1]]
    assert moved > 20 and total > 1500


def test_ring_flag_combinations_rejected():
    net = weights.case_net("scr3x40")
    o = Oracle(nn_mode=2)
    with pytest.raises(RuntimeError):
        o.load_nn_net(net.with_input_flags(weights.TZ_RING | weights.SLOT_RESET))
    with pytest.raises(RuntimeError):
        o.load_nn_net(weights.load_net("blowing4x40").with_input_flags(weights.TZ_RING))   # carry_hidden


# ---- GPU ----------------------------------------------------------------------------------------
def _gpu_ctx(g, engine=0):
    from nnfme.runtime import FmeContext
    ctx = FmeContext(use_hadamard=1, nn_mode=2, qp=22, fast_inter_mode=int(g["config"][1]),
                     net=weights.case_net(str(g["net"])), nn_engine=engine)
    for i, p in enumerate(g["pictures"]):
        ctx.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        ctx.set_lambda(i, float(lam))
    if g["keys"].size:
        ctx.set_keys(g["keys"])
    return ctx


@pytest.mark.gpu
@pytest.mark.parametrize("case", ring_golden_cases())
def test_gpu_ring_integer_search_golden(case):
    g = load_golden(case)
    ctx = _gpu_ctx(g)
    jobs, sad, nn_in = ctx.integer_search_ring(g["jobs"], g["ext"])
    _check_tz(g, jobs, sad, nn_in, "gpu")
    # without FME_TZ_RING the same searches stop before the square (the master's xTZSearch)
    ext = g["ext"].copy()
    ext["flags"] &= np.uint8(0xFF ^ TZ_RING)
    plain, _, rows = ctx.integer_search_ring(g["jobs"], ext)
    assert not rows.any()
    o = _engines(g, "oracle")
    exp, _ = o.integer_search(g["jobs"], ext)
    assert np.array_equal(plain["mv_x"], exp["mv_x"]) and np.array_equal(plain["mv_y"], exp["mv_y"])


def _refine_nn_in(ctx, g, rows=None, engine_rows=True):
    import torch
    dev = torch.device("cuda", 0)
    d_rows = torch.from_numpy(np.ascontiguousarray(g["nn_in"] if rows is None else rows).view(np.uint8).copy()).to(dev)
    if engine_rows:
        ctx.set_nn_inputs(d_rows.data_ptr(), len(g["nn_in"]))
    try:
        return ctx.refine(g["refine_jobs"])
    finally:
        ctx.set_nn_inputs(None)
        torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ring_golden_cases())
def test_gpu_ring_refine_exact_engine_golden(case):
    g = load_golden(case)
    res = _refine_nn_in(_gpu_ctx(g, engine=0), g)
    bad, first, counts = compare_results(res, g["results"])
    assert bad == 0, f"{case}: {bad} refinements differ (first {first}): {counts}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ring_golden_cases())
def test_gpu_ring_refine_mfma_engine(case):
    """MFMA engine: a k-ordered FMA chain (not bit-exact by construction): every search field equal,
    classes equal on >= 99 % of the jobs (test_deep_nn.py's tolerance)."""
    g = load_golden(case)
    res = _refine_nn_in(_gpu_ctx(g, engine=1), g)
    exp = g["results"]
    for f in ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi", "emi"):
        assert np.array_equal(res[f], exp[f]), f
    agree = (res["nn_class"] == exp["nn_class"]).mean()
    assert agree >= 0.99, agree


@pytest.mark.gpu
def test_gpu_ring_device_path_and_rejection():
    """The frame-replay form: jobs, rows and results in device memory; a batch with FME_JOB_NN_IN
    jobs and no rows bound (or rows short of the batch) is rejected on the device; binding them
    makes the same batch run and equal the golden."""
    import torch
    from nnfme.abi import JOB_DTYPE, RESULT_DTYPE
    g = load_golden(ring_golden_cases()[0])
    ctx = _gpu_ctx(g)
    dev = torch.device("cuda", 0)
    jobs = g["refine_jobs"]
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    d_res = torch.zeros(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_rows = torch.from_numpy(g["nn_in"].view(np.uint8).copy()).to(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.refine_device(d_jobs.data_ptr(), d_res.data_ptr(), len(jobs), s)
    assert ctx.refine_status() > 0
    r = d_res.cpu().numpy().view(RESULT_DTYPE)
    assert (r["status"] & RES_REJECTED).all()
    ctx.set_nn_inputs(d_rows.data_ptr(), len(jobs) - 1)
    ctx.refine_device(d_jobs.data_ptr(), d_res.data_ptr(), len(jobs), s)
    assert ctx.refine_status() > 0
    ctx.set_nn_inputs(d_rows.data_ptr(), len(jobs))
    ctx.nn_reset()
    ctx.refine_device(d_jobs.data_ptr(), d_res.data_ptr(), len(jobs), s)
    assert ctx.refine_status() == 0
    r = d_res.cpu().numpy().view(RESULT_DTYPE)
    bad, first, counts = compare_results(r, g["results"])
    assert bad == 0, counts
    assert (jobs["flags"] & JOB_NN_IN).sum() > 100
    assert JOB_DTYPE.itemsize == 32
