"""Generic (deeper) NN_pred nets, nn_mode 2 — BASELINE.json configs[4].

The nets are the reference's own deeper variants, converted from its in-tree backups by
tools/convert_deep_weights.py: Backups/4 "SCR 3 layers" (9 -> 3 x 40 -> 49, double, sigmoid) and
Backups/15 "blowing 4 lyrs qp 22" (17 -> 4 x 40 -> 49, float, X3/X4 carried across calls).  Neither
backup compiles against the shipped headers (their xTZSearchHelp signature predates TEncSearch.h),
so parity is pinned by two independent restatements agreeing bit for bit (oracle/fme_oracle.c and
oracle/ref_harness.cpp), by the golden fixtures they produce, and by the master net run through the
generic path reproducing nn_mode 1 exactly.  The exact GPU engine must equal them bit for bit; the
MFMA engine (k-ordered FMA chain) is checked for agreement and margin-explained disagreements.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, load_golden
from nnfme import synth, weights
from nnfme.abi import RESULT_DTYPE, compare_results
from oracle import REF_SO, Oracle, Reference

HAVE_REF = os.path.exists(REF_SO)
REF_SRC = "/root/reference/source/Lib/TLibEncoder/Backups"


def _rand_inputs(rng, n):
    for _ in range(n):
        e = rng.integers(0, 250000, 8).astype(np.uint32)
        c = int(rng.integers(0, 120000))
        w, h = synth.ALL_PU_SIZES[int(rng.integers(len(synth.ALL_PU_SIZES)))]
        yield e, c, h, w


def test_net_blobs():
    scr = weights.load_net("scr3x40")
    assert (scr.precision, scr.widths, scr.embedding, scr.out_act, scr.carry_hidden) == \
        (weights.F64, [40, 40, 40], weights.EMB_NONE, weights.OUT_SIGMOID, 0)
    assert scr.params.size == 5956 == weights.param_count(scr)
    blow = weights.load_net("blowing4x40")
    assert (blow.precision, blow.widths, blow.embedding, blow.carry_hidden) == \
        (weights.F32, [40, 40, 40, 40], weights.EMB_SWAP, 0b1100)
    assert blow.params.size == 8060
    m = weights.master_net(22)
    assert m.params.size == 2060 and m.widths == [22, 20]


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources not mounted")
def test_blobs_equal_reference_initialisers():
    import importlib.util
    spec = importlib.util.spec_from_file_location("cdw", os.path.join(ROOT, "tools", "convert_deep_weights.py"))
    cdw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cdw)
    for name, (desc, params, src) in (("scr3x40", cdw.scr_net()), ("blowing4x40", cdw.blowing_net())):
        net = weights.load_net(name)
        assert np.array_equal(net.params, np.array(params)), name
        cdw.check_switch(src, name)


@pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built")
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40", "blowing4x40+rezero", "master"])
def test_oracle_forward_equals_harness(name):
    """Two independent restatements of the backups' forward passes agree on every OUT bit,
    including Backups/15's X3/X4 carried from call to call."""
    net = weights.case_net(name)
    o, r = Oracle(nn_mode=2), Reference(nn_mode=2)
    o.load_nn_net(net)
    r.load_nn_net(net)
    rng = np.random.default_rng(7)
    classes = []
    for e, c, h, w in _rand_inputs(rng, 1500):
        a, la = o.nn_net_forward(e, c, h, w)
        b, lb = r.nn_net_class(e, c, h, w)
        assert a == b and np.array_equal(la, lb)
        classes.append(a)
    assert len(set(classes)) > 10


def test_master_through_generic_path_equals_nn_mode_1():
    """The master net in the generic layout (nn_mode 2) reproduces the shipped nn_mode 1 fixture."""
    a = load_golden("deep_master_qp22")
    b = load_golden("ldp_qp22_hadme_fen1_nn")
    assert np.array_equal(a["jobs"], b["jobs"])
    bad, first, counts = compare_results(a["results"], b["results"])
    assert bad == 0, (first, counts)


def test_master_generic_forward_equals_master_forward():
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.master_net(22))
    wts = weights.load_weights(22)
    rng = np.random.default_rng(3)
    for e, c, h, w in _rand_inputs(rng, 1000):
        assert o.nn_net_forward(e, c, h, w)[0] == o.nn_class(wts, e, c, h, w)[0]


def test_deep_goldens_exercise_the_net():
    for case in ("deep_scr3x40_qp22", "deep_blowing4x40_qp22"):
        g = load_golden(case)
        cls = g["results"]["nn_class"]
        assert len(np.unique(cls)) >= 8, case
        assert str(g["net"]) in ("scr3x40", "blowing4x40+rezero")


def test_carry_hidden_changes_results():
    """Backups/15 as shipped (X3/X4 never re-zeroed) differs from the re-zeroed net: the carry is
    observable, so a fixture of the re-zeroed net would not silently stand in for it."""
    o1, o2 = Oracle(nn_mode=2), Oracle(nn_mode=2)
    o1.load_nn_net(weights.case_net("blowing4x40"))
    o2.load_nn_net(weights.case_net("blowing4x40+rezero"))
    rng = np.random.default_rng(5)
    diff = 0
    for e, c, h, w in _rand_inputs(rng, 400):
        diff += o1.nn_net_forward(e, c, h, w)[0] != o2.nn_net_forward(e, c, h, w)[0]
    assert diff > 0


def _small_frame(seed=9, bi=True):
    """A 416x240 LDP frame's jobs (EMI on) plus, optionally, bi-pred jobs with no EMI step, so the
    per-call slot reset sees jobs that push 0..8 slots."""
    W, H = 416, 240
    rng = np.random.default_rng(seed)
    pics = {i: synth.synth_luma(W, H, i) for i in range(3)}
    jobs = synth.make_ctu_jobs(rng, W, H, 60, 2, [0, 1], [2])
    if bi:
        sel = rng.random(len(jobs)) < 0.15
        jobs["flags"][sel] &= ~np.uint8(1)   # FME_JOB_EMI off: this call pushes nothing
    return pics, jobs


def _oracle_refine(name, pics, jobs):
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.case_net(name))
    for k, v in pics.items():
        o.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        o.set_lambda(lid, lam)
    return o.refine(jobs), o.nn_get_state()


def test_slot_reset_is_observable_and_zeroes_unpushed_slots():
    """FME_NN_IN_SLOT_RESET (the backups' per-call memset of array_e) changes classes, and a job
    that pushed nothing sees e = 0 (checked through the oracle's own forward)."""
    pics, jobs = _small_frame()
    a, _ = _oracle_refine("scr3x40", pics, jobs)
    b, st = _oracle_refine("scr3x40+slotreset", pics, jobs)
    assert (a["nn_class"] != b["nn_class"]).any()
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.case_net("scr3x40+slotreset"))
    e, c, ph, pw = nn_reset_inputs(jobs, b)
    for i in np.random.default_rng(4).choice(len(jobs), 300, replace=False):
        assert o.nn_net_forward(e[i], int(c[i]), int(ph[i]), int(pw[i]))[0] == b["nn_class"][i]
    assert st[11] & 0xFF == 0xFF


def nn_reset_inputs(jobs, res):
    """NN inputs under FME_NN_IN_SLOT_RESET: this job's own pushes, zeros elsewhere; C / PU size
    from the last EMI job (carried, as in the backups)."""
    from test_gpu_parity import nn_host_inputs
    _, c, ph, pw = nn_host_inputs(jobs, res)
    n = len(jobs)
    emi_job = (jobs["flags"] & 1) != 0
    e = np.zeros((n, 8), np.uint32)
    for s in range(8):
        own = emi_job & (res["n_emi"] > s)
        e[own, s] = res["emi"][own, s]
    return e, c, ph, pw


# ---- GPU ----------------------------------------------------------------------------------------
def _ctx(net, engine=0, **kw):
    from nnfme.runtime import FmeContext
    return FmeContext(nn_mode=2, net=weights.case_net(net), nn_engine=engine, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40+rezero", "master"])
def test_gpu_nn_pred_single_matches_oracle(name):
    ctx = _ctx(name)
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.case_net(name))
    rng = np.random.default_rng(11)
    for e, c, h, w in _rand_inputs(rng, 150):
        cls, out4 = ctx.nn_pred_single(e, c, h, w)
        assert cls == o.nn_net_forward(e, c, h, w)[0]
        assert 2 * out4[0] + out4[1] == cls % 7 - 3 and 2 * out4[2] + out4[3] == cls // 7 - 3


@pytest.mark.gpu
def test_gpu_load_nn_net_rejections():
    from nnfme.runtime import FmeError
    ctx = _ctx("scr3x40")
    with pytest.raises(FmeError) as e:
        ctx.load_nn_net(weights.case_net("blowing4x40"))   # carried X3/X4: not a batch engine
    assert e.value.code == -4
    bad = weights.load_net("scr3x40")
    bad.widths = [40, 40, 41]
    with pytest.raises(Exception):
        ctx.load_nn_net(bad)
    with pytest.raises(FmeError):
        ctx.set_nn_engine(7)


@pytest.fixture(scope="module")
def frame_1080p_deep():
    W, H = 1920, 1080
    rng = np.random.default_rng(2023)
    pics = {i: synth.synth_luma(W, H, i) for i in range(5)}
    jobs = synth.make_ctu_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [1])
    return pics, jobs


def _frame_run(pics, jobs, name, engine, margin=False, logits=False):
    """One refine batch on the GPU; with logits=True returns (results, OUT[n][49] as float64)."""
    import torch
    ctx = _ctx(name, engine, qp=22, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    m = lg = None
    if margin:
        m = torch.zeros(len(jobs), dtype=torch.float32, device="cuda")
        ctx.set_nn_margin_output(m.data_ptr(), len(jobs))
    if logits:
        dt = torch.float64 if weights.case_net(name).precision == weights.F64 else torch.float32
        lg = torch.full((len(jobs), 49), float("nan"), dtype=dt, device="cuda")
        ctx.set_nn_logit_output(lg.data_ptr(), len(jobs))
    res = ctx.refine(jobs)
    ctx.set_nn_margin_output(0)
    ctx.set_nn_logit_output(0)
    if logits:
        return res, lg.cpu().numpy().astype(np.float64)
    return res, (m.cpu().numpy() if m is not None else None)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40+rezero"])
def test_gpu_1080p_exact_engine_matches_oracle_forward(frame_1080p_deep, name):
    """Full 1080p frame: the exact engine's class for a 20,000-job sample equals the oracle's
    forward on the same (host-resolved) carried inputs."""
    from test_gpu_parity import nn_host_inputs
    pics, jobs = frame_1080p_deep
    res, _ = _frame_run(pics, jobs, name, 0)
    e, c, ph, pw = nn_host_inputs(jobs, res)
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.case_net(name))
    sel = np.random.default_rng(1).choice(len(jobs), 20000, replace=False)
    bad = [i for i in sel if o.nn_net_forward(e[i], int(c[i]), int(ph[i]), int(pw[i]))[0] != res["nn_class"][i]]
    assert not bad, f"{len(bad)} class mismatches, first {bad[:5]}"
    assert np.array_equal(res["mv_x"], 4 * res["mv_int_x"].astype(np.int32) + res["nn_class"] % 7 - 3)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40+rezero"])
def test_gpu_mfma_engine_agreement(frame_1080p_deep, name):
    """MFMA engine vs exact engine on a 1080p frame: identical search fields, class agreement
    >= 99.5 %, and every disagreement sits on a near-tie of the exact outputs."""
    pics, jobs = frame_1080p_deep
    ex, m_ex = _frame_run(pics, jobs, name, 0, margin=True)
    mf, _ = _frame_run(pics, jobs, name, 1)
    fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi")
    bad, first, counts = compare_results(ex, mf, fields)   # (+ the pushed emi values)
    assert bad == 0, (first, counts)
    dis = ex["nn_class"] != mf["nn_class"]
    agree = 1.0 - dis.mean()
    assert agree >= 0.995, agree
    if dis.any():
        assert np.percentile(m_ex[dis], 99) <= np.percentile(m_ex, 5), "disagreements are not near-ties"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40+rezero"])
def test_gpu_exact_engine_outputs_equal_oracle_bits(frame_1080p_deep, name):
    """Every OUT value before the output activation, for 20,000 jobs of a 1080p frame, equals the
    oracle's forward bit for bit (not just the class); the sigmoid itself uses the device's exp
    (within 1 ulp of glibc's), whose ties the saturation tests below pin."""
    pics, jobs = frame_1080p_deep
    res, lg = _frame_run(pics, jobs, name, 0, logits=True)
    from test_gpu_parity import nn_host_inputs
    e, c, ph, pw = nn_host_inputs(jobs, res)
    o = Oracle(nn_mode=2)
    o.load_nn_net(weights.case_net(name))
    sel = np.random.default_rng(2).choice(len(jobs), 20000, replace=False)
    bad = [i for i in sel if not np.array_equal(o.nn_net_forward_pre(e[i], int(c[i]), int(ph[i]), int(pw[i]))[2], lg[i])]
    assert not bad, f"{len(bad)} jobs with OUT bits differing, first {bad[:5]}"


# k-ordered FMA chain vs separate multiply / add: per output the two differ by rounding only,
# << 1e-9 relative in double and << 1e-3 in float for these 40-wide layers; a stale accumulator
# row (the gfx950 f64 MFMA hazard) reads another job's / tile's value: O(1).
MFMA_TOL = {weights.F64: 1e-9, weights.F32: 1e-3}


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["scr3x40", "blowing4x40+rezero"])
def test_gpu_mfma_outputs_within_rounding_of_exact(frame_1080p_deep, name):
    """Deterministic MFMA check: every one of the 49 outputs of every job of a 1080p frame is
    within FMA rounding of the exact engine's, so no accumulator row can be read stale."""
    pics, jobs = frame_1080p_deep
    _, ex = _frame_run(pics, jobs, name, 0, logits=True)
    _, mf = _frame_run(pics, jobs, name, 1, logits=True)
    assert np.isfinite(ex).all() and np.isfinite(mf).all()
    rel = np.abs(mf - ex) / (1.0 + np.abs(ex))
    tol = MFMA_TOL[weights.case_net(name).precision]
    worst = np.unravel_index(np.argmax(rel), rel.shape)
    print(f"{name}: max relative OUT difference {rel.max():.3e} (job {worst[0]}, output {worst[1]})")
    assert rel.max() <= tol, (rel.max(), worst)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", [0, 1])
def test_gpu_slot_reset_matches_oracle(engine):
    """FME_NN_IN_SLOT_RESET on the GPU equals the oracle: every record field (exact engine; the
    MFMA engine on the search fields and >= 99 % of the classes) and the carried state."""
    pics, jobs = _small_frame()
    ref, st = _oracle_refine("scr3x40+slotreset", pics, jobs)
    ctx = _ctx("scr3x40+slotreset", engine, qp=22, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    res = ctx.refine(jobs)
    if engine == 0:
        bad, first, counts = compare_results(ref, res)
        assert bad == 0, (first, counts)
        assert np.array_equal(ctx.nn_get_state(), st)
    else:
        fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi")
        bad, first, counts = compare_results(ref, res, fields)
        assert bad == 0, (first, counts)
        assert (ref["nn_class"] == res["nn_class"]).mean() >= 0.99


def _saturating_net():
    """scr3x40 with output biases pushed into the sigmoid's saturation: +1e4 on outputs 9, 20, 33
    (sigmoid == 1.0 exactly in double, so the first saturated output wins whatever the
    pre-activations) and
    +36.0..37.6 on 40..48 (1 + exp(-x) rounds at the last bit: exp's ulp decides the tie)."""
    net = weights.load_net("scr3x40")
    p = net.params.copy()
    bout = p.size - 27 - 49
    for k in (9, 20, 33):
        p[bout + k] += 1e4
    for q, k in enumerate(range(40, 49)):
        p[bout + k] += 36.0 + 0.2 * q
    return weights.NnNet(net.precision, net.widths, net.embedding, net.out_act, 0, p)


def test_saturating_net_ties_at_the_first_maximum():
    o = Oracle(nn_mode=2)
    o.load_nn_net(_saturating_net())
    rng = np.random.default_rng(12)
    for e, c, h, w in _rand_inputs(rng, 200):
        cls, out = o.nn_net_forward(e, c, h, w)
        assert out[9] == out[20] == out[33] == 1.0 and cls == int(np.argmax(out)) <= 9


@pytest.mark.gpu
def test_gpu_sigmoid_saturation_and_last_bit_ties():
    """Saturated and last-bit sigmoid outputs: the GPU's class (device exp) equals the oracle's
    (glibc exp), the first maximum, for single calls and a batch whose pre-activation OUT bits
    equal the oracle's."""
    from nnfme.runtime import FmeContext
    net = _saturating_net()
    # outputs 40..48 alone (the +60 block removed): ties decided by the last bit of 1 + exp(-x)
    p = net.params.copy()
    bout = p.size - 27 - 49
    for k in (9, 20, 33):
        p[bout + k] -= 1e4
    near = weights.NnNet(net.precision, net.widths, net.embedding, net.out_act, 0, p)
    for nt in (net, near):
        ctx = FmeContext(nn_mode=2, net=nt, nn_engine=0)
        o = Oracle(nn_mode=2)
        o.load_nn_net(nt)
        rng = np.random.default_rng(13)
        for e, c, h, w in _rand_inputs(rng, 100):
            cls, _ = ctx.nn_pred_single(e, c, h, w)
            ocls, _ = o.nn_net_forward(e, c, h, w)
            assert cls == ocls
    pics, jobs = _small_frame(bi=False)
    for nt in (net, near):
        o = Oracle(nn_mode=2)
        o.load_nn_net(nt)
        for k, v in pics.items():
            o.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
            o.set_lambda(lid, lam)
        ref = o.refine(jobs)
        import torch
        ctx = FmeContext(nn_mode=2, net=nt, nn_engine=0, qp=22, max_jobs=len(jobs))
        for k, v in pics.items():
            ctx.set_picture(k, v)
        for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
            ctx.set_lambda(lid, lam)
        lg = torch.zeros((len(jobs), 49), dtype=torch.float64, device="cuda")
        ctx.set_nn_logit_output(lg.data_ptr(), len(jobs))
        res = ctx.refine(jobs)
        assert np.array_equal(res["nn_class"], ref["nn_class"])
        from test_gpu_parity import nn_host_inputs
        e, c, ph, pw = nn_host_inputs(jobs, res)
        lgh = lg.cpu().numpy()
        for i in range(0, len(jobs), max(1, len(jobs) // 300)):
            assert np.array_equal(o.nn_net_forward_pre(e[i], int(c[i]), int(ph[i]), int(pw[i]))[2], lgh[i]), i
