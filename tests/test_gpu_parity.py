"""GPU parity: the HIP path (through the C-ABI) against the golden vectors and the oracle.

Bit-exact for every field the reference computes (integer and double-derived outputs, and the
NN class under the sequential-k float32 contract).  Full-size (1080p frame) checks use
size-independent properties: run-to-run determinism, batch-split invariance of the carried
NN state, the oracle on a random sample of jobs, and a vectorised float32 NN restatement
over every job.
"""
import os

import numpy as np
import pytest

from conftest import ROOT, golden_cases, load_golden
from nnfme import synth, weights
from nnfme.abi import (JOB_BIPRED, JOB_DTYPE, JOB_EMI, RESULT_DTYPE, compare_results)

pytestmark = pytest.mark.gpu


def _ctx(g, **over):
    from nnfme.runtime import FmeContext
    hadme, fen, nn_mode, qp = (int(v) for v in g["config"])
    kw = dict(use_hadamard=hadme, nn_mode=nn_mode, qp=qp, fast_inter_mode=fen,
              bit_depth=int(g["bit_depth"][0]) if "bit_depth" in g else 8)
    if "net" in g:
        kw["net"] = weights.case_net(str(g["net"]))
    kw.update(over)
    ctx = FmeContext(**kw)
    for i, p in enumerate(g["pictures"]):
        ctx.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        ctx.set_lambda(i, float(lam))
    if g["keys"].size:
        ctx.set_keys(g["keys"])
    return ctx


def _assert_same(res, ref, what):
    bad, first, counts = compare_results(res, ref)
    assert bad == 0, f"{what}: {bad} mismatching jobs, first {first}: {counts}"


@pytest.mark.parametrize("case", golden_cases())
def test_golden(case):
    g = load_golden(case)
    _assert_same(_ctx(g).refine(g["jobs"]), g["results"], case)


@pytest.mark.parametrize("case", golden_cases())
def test_golden_split_batches_carry_nn_state(case):
    g = load_golden(case)
    ctx = _ctx(g)
    j = g["jobs"]
    cuts = [0, 1, 7, 300, len(j) - 5, len(j)]
    parts = [ctx.refine(j[a:b]) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    _assert_same(np.concatenate(parts), g["results"], case + " split")


def test_refine_device_resident():
    import torch
    g = load_golden("ldp_qp22_hadme_fen1_nn")
    ctx = _ctx(g)
    jobs = np.ascontiguousarray(g["jobs"])
    dj = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    dr = torch.zeros(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx.refine_device(dj.data_ptr(), dr.data_ptr(), len(jobs), s.cuda_stream)
    s.synchronize()
    res = dr.cpu().numpy().view(RESULT_DTYPE)
    _assert_same(res, g["results"], "device-resident")


@pytest.mark.parametrize("case", golden_cases())
def test_golden_packed_device(case):
    """The 16-byte upload form (fme_pack_jobs -> fme_refine_packed_device, unpacked on the device)
    gives the golden records; a case outside the packed form is refused at pack time."""
    import torch
    from nnfme.runtime import FmeError, pack_jobs
    g = load_golden(case)
    try:
        pk, kb = pack_jobs(g["jobs"])
    except FmeError as e:
        assert e.code == -4, e
        pytest.skip(f"outside the packed form: {e}")
    ctx = _ctx(g)
    dpk = torch.from_numpy(pk.view(np.uint8).copy()).cuda()
    dkb = torch.from_numpy(kb.view(np.uint8).copy()).cuda()
    n = len(pk)
    dr = torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx.refine_packed_device(dpk.data_ptr(), dkb.data_ptr(), dr.data_ptr(), n, s.cuda_stream)
    s.synchronize()
    _assert_same(dr.cpu().numpy().view(RESULT_DTYPE), g["results"], case + " packed")


def test_nn_reset_restores_initial_state():
    g = load_golden("qp32_nn")
    ctx = _ctx(g)
    a = ctx.refine(g["jobs"])
    ctx.nn_reset()
    b = ctx.refine(g["jobs"])
    _assert_same(a, b, "after reset")


def test_empty_batch():
    g = load_golden("qp37_nn")
    ctx = _ctx(g)
    assert len(ctx.refine(g["jobs"][:0])) == 0


def test_invalid_jobs_rejected():
    from nnfme.runtime import FmeError
    g = load_golden("qp37_nn")
    ctx = _ctx(g)
    for field, value in (("w", 20), ("ref_id", 40), ("key_offset", 10 ** 8)):
        j = g["jobs"][:16].copy()
        j[field][3] = value
        with pytest.raises(FmeError) as e:
            ctx.refine(j)
        assert e.value.code == -1
    j = g["jobs"][:16].copy()
    j["key_offset"][5] = -1
    j["x"][5] = 1000   # PU outside the original picture
    with pytest.raises(FmeError):
        ctx.refine(j)
    # the context still works afterwards
    _assert_same(ctx.refine(g["jobs"][:40]), g["results"][:40], "after rejection")


def _frac_single_check(ctx, g, idx):
    jobs, ref = g["jobs"], g["results"]
    pics = g["pictures"]
    pad = 80
    planes = {}
    for i in idx:
        j, r = jobs[i], ref[i]
        w, h, x, y = int(j["w"]), int(j["h"]), int(j["x"]), int(j["y"])
        rid = int(j["ref_id"])
        if rid not in planes:
            planes[rid] = np.pad(pics[rid].astype(np.int16), pad, mode="edge")
        if int(j["key_offset"]) >= 0:
            key = g["keys"][int(j["key_offset"]):int(j["key_offset"]) + w * h].reshape(h, w)
        else:
            key = pics[int(j["org_id"])][y:y + h, x:x + w]
        ml = 65536.0 * np.sqrt(float(g["lambdas"][int(j["lambda_id"])]))
        half, qtr, cost = ctx.frac_dif_single(key, planes[rid], (y + pad, x + pad),
                                              (int(r["mv_int_x"]), int(r["mv_int_y"])),
                                              (int(j["mvp_x"]), int(j["mvp_y"])), ml,
                                              lossless=bool(j["flags"] & 4))
        assert (half, qtr, cost) == ((int(r["half_x"]), int(r["half_y"])), (int(r["qtr_x"]), int(r["qtr_y"])),
                                     int(r["frac_cost"])), (i, w, h)


def test_frac_dif_single_matches_batch():
    """The TEncSearch-shaped single-PU entry point (the resident server, fme_server.hip) equals the
    batch path's FracDIF fields."""
    g = load_golden("ldp_qp22_hadme_fen1_nn")
    _frac_single_check(_ctx(g), g, range(0, len(g["jobs"]), 37))


@pytest.mark.parametrize("case", golden_cases())
def test_frac_dif_single_every_shape(case):
    """Every PU shape of every golden case (SATD 8x8 / 4x4 tilings, SAD with HADME off and for
    lossless jobs, bi-pred keys outside 0..255), up to 6 jobs per shape."""
    g = load_golden(case)
    jobs = g["jobs"]
    idx = []
    for (w, h) in synth.ALL_PU_SIZES:
        sel = np.flatnonzero((jobs["w"] == w) & (jobs["h"] == h))
        idx += list(sel[:: max(1, len(sel) // 6)][:6])
    lossless = np.flatnonzero(jobs["flags"] & 4)
    idx += list(lossless[:8])
    _frac_single_check(_ctx(g), g, idx)


def test_single_call_server_lifecycle():
    """The server instance idles out and is relaunched by the next call, is stopped by batch work
    and by a weight reload (its LDS copy of the net), and answers the same across all of it."""
    import time
    from oracle import Oracle
    g = load_golden("ldp_qp22_hadme_fen1_nn")
    ctx = _ctx(g)
    idx = list(range(0, 400, 40))
    _frac_single_check(ctx, g, idx)
    time.sleep(0.02)                                     # > the idle limit: the instance has left
    _frac_single_check(ctx, g, idx)
    _assert_same(ctx.refine(g["jobs"][:64]), g["results"][:64], "batch between single calls")
    _frac_single_check(ctx, g, idx)
    o = Oracle()
    e, c = np.arange(1000, 9000, 1000, dtype=np.uint32), 4321
    for qp in (22, 27, 22):                              # the resident copy follows each reload
        ctx.load_nn(weights.load_weights(qp))
        cls, _ = ctx.nn_pred_single(e, c, 16, 8)
        assert cls == o.nn_class(weights.load_weights(qp), e, c, 16, 8)[0]
    t0 = time.perf_counter()
    for _ in range(300):
        ctx.nn_pred_single(e, c, 16, 8)
    per_call = (time.perf_counter() - t0) / 300
    assert per_call < 200e-6, per_call


@pytest.mark.parametrize("qp", [22, 27, 32, 37])
def test_nn_pred_single_matches_oracle(qp):
    from nnfme.runtime import FmeContext
    from oracle import Oracle
    ctx = FmeContext(qp=qp)
    o = Oracle(qp=qp)
    wts = weights.load_weights(qp)
    rng = np.random.default_rng(qp + 100)
    for _ in range(200):
        e = rng.integers(0, 300000, 8).astype(np.uint32)
        c = int(rng.integers(0, 300000))
        w, h = synth.ALL_PU_SIZES[int(rng.integers(len(synth.ALL_PU_SIZES)))]
        cls, out4 = ctx.nn_pred_single(e, c, h, w)
        assert cls == o.nn_class(wts, e, c, h, w)[0]
        assert 2 * out4[0] + out4[1] == cls % 7 - 3 and 2 * out4[2] + out4[3] == cls // 7 - 3


# ---------------------------------------------------------------------------------------
# full-size: one 1080p LDP QP22 frame (≈863 K jobs, 4 reference pictures)
# ---------------------------------------------------------------------------------------
def nn_host_inputs(jobs, res):
    """Vectorised restatement of NN_pred's inputs: the last writer per array_e slot and of C /
    PUHeight / PUWidth, in job order, from a fresh state (unwritten -> 0)."""
    n = len(jobs)
    emi_job = (jobs["flags"] & JOB_EMI) != 0
    idx = np.arange(n)
    npush = res["n_emi"].astype(np.int64)
    src = []
    for s in range(9):
        wr = emi_job & ((npush > s) if s < 8 else True)
        src.append(np.maximum.accumulate(np.where(wr, idx, -1)))
    e = np.zeros((n, 8), np.uint32)
    for s in range(8):
        ok = src[s] >= 0
        e[ok, s] = res["emi"][src[s][ok], s]
    ok = src[8] >= 0
    c = np.zeros(n, np.uint32)
    ph = np.zeros(n, np.int64)
    pw = np.zeros(n, np.int64)
    c[ok] = res["c"][src[8][ok]]
    ph[ok] = jobs["h"][src[8][ok]]
    pw[ok] = jobs["w"][src[8][ok]]
    return e, c, ph, pw


def nn_host_emulation(jobs, res, params, state=None):
    """NN_pred's float32 forward (sequential-k, no FMA: numpy float32 ops round each step) on the
    inputs of nn_host_inputs."""
    n = len(jobs)
    e, c, ph, pw = nn_host_inputs(jobs, res)
    t = weights.unpack(params)
    f32 = np.float32
    rowh = {4: 1, 8: 2, 16: 3, 12: 4, 24: 5, 32: 6, 64: 7}
    roww = {4: 1, 8: 2, 12: 3, 16: 4, 24: 5, 32: 6, 64: 7}
    rh = np.array([rowh.get(int(v), 0) for v in range(65)])[ph]
    rw = np.array([roww.get(int(v), 0) for v in range(65)])[pw]
    inp = [t["embs0"][rh, k] for k in range(4)] + [t["embs1"][rw, k] for k in range(4)]
    raw = [e[:, 0], e[:, 1], e[:, 2], e[:, 3], c, e[:, 4], e[:, 5], e[:, 6], e[:, 7]]
    for k in range(9):
        v = raw[k].astype(f32)
        v = (v - t["mean"][k]) / t["stdev"][k]
        inp.append(v * t["BN_gamma_in"][k])

    def layer(x, Wt, b, g=None, be=None):
        out = []
        for r in range(Wt.shape[0]):
            s = np.zeros(n, f32)
            for k in range(Wt.shape[1]):
                s = s + Wt[r, k] * x[k]
            s = s + b[r]
            if g is not None:
                s = np.where(s < 0, f32(0), s)
                s = s * g[r] + be[r]
            out.append(s)
        return out

    x1 = layer(inp, t["in_h1"], t["b1"], t["BN_gamma_1"], t["BN_beta_1"])
    x2 = layer(x1, t["h1_h2"], t["b2"], t["BN_gamma_2"], t["BN_beta_2"])
    out = np.stack(layer(x2, t["h2_out"], t["bout"]), axis=1)
    return np.argmax(out, axis=1)   # first index of the maximum, like Eigen maxCoeff


@pytest.fixture(scope="module")
def frame_1080p():
    W, H = 1920, 1080
    rng = np.random.default_rng(2022)
    pics = {i: synth.synth_luma(W, H, i) for i in range(5)}
    n = synth.jobs_per_frame(W, H)
    jobs = synth.make_jobs(rng, W, H, n, 4, [0, 1, 2, 3], [1])
    return pics, jobs


def _frame_ctx(pics, nn_mode=1):
    from nnfme.runtime import FmeContext
    ctx = FmeContext(nn_mode=nn_mode, qp=22, max_jobs=900000)
    for k, v in pics.items():
        ctx.set_picture(k, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        ctx.set_lambda(lid, lam)
    return ctx


def test_1080p_frame_full_size_properties(frame_1080p):
    from oracle import Oracle
    pics, jobs = frame_1080p
    ctx = _frame_ctx(pics)
    a = ctx.refine(jobs)
    ctx.nn_reset()
    b = ctx.refine(jobs)
    assert a.tobytes() == b.tobytes(), "not deterministic"
    # batch-split invariance of the carried NN state
    ctx.nn_reset()
    k = len(jobs) // 3
    c = np.concatenate([ctx.refine(jobs[:k]), ctx.refine(jobs[k:])])
    _assert_same(c, a, "1080p split")
    # per-job fields against the oracle on a random sample (NN off: per-job independent)
    rng = np.random.default_rng(9)
    sel = np.sort(rng.choice(len(jobs), 3000, replace=False))
    o = Oracle(nn_mode=0)
    for kk, v in pics.items():
        o.set_picture(kk, v)
    for lid, lam in enumerate(synth.LDP_LAMBDA[22]):
        o.set_lambda(lid, lam)
    ro = o.refine(jobs[sel])
    fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi")
    bad, first, counts = compare_results(a[sel], ro, fields)
    assert bad == 0, f"1080p sample: {bad} mismatches, first {first}: {counts}"
    # NN class of every job against the vectorised float32 restatement
    cls = nn_host_emulation(jobs, a, weights.load_weights(22))
    mism = np.flatnonzero(cls != a["nn_class"])
    assert len(mism) == 0, f"{len(mism)} NN class mismatches, first {mism[:5]}"
    # the tail follows from the class
    assert np.array_equal(a["mv_x"], 4 * a["mv_int_x"].astype(np.int32) + a["nn_class"] % 7 - 3)
    assert np.array_equal(a["mv_y"], 4 * a["mv_int_y"].astype(np.int32) + a["nn_class"] // 7 - 3)


def test_cpp_hm_adapter():
    """The C++ TEncSearch-shaped adapter (include/fme_hm.hpp): CTU-row batcher, single-PU
    xPatternSearchFracDIF and NN_pred, bit-exact against the oracle (tests/cpp)."""
    import subprocess
    exe = os.path.join(ROOT, "hm16.9-nn_fme_amd", "host", "test_hm_adapter")
    assert os.path.exists(exe), "build it with __graft_entry__.build() (make host-test)"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "hm adapter ok" in p.stdout


def test_emi_and_nn_in_flags_together():
    """A job flagged both FME_JOB_EMI and FME_JOB_NN_IN takes its NN inputs from its row and runs no
    EMI step (fme.h), in the lane kernel as in the oracle and the reference harness."""
    import torch
    from oracle import Oracle
    from nnfme.abi import JOB_NN_IN
    g = load_golden("ldp_qp22_hadme_fen1_nn")
    jobs = np.ascontiguousarray(g["jobs"][:400]).copy()
    emi = np.flatnonzero(jobs["flags"] & JOB_EMI)
    assert len(emi) > 50
    jobs["flags"][emi[::3]] |= JOB_NN_IN
    rng = np.random.default_rng(17)
    rows = rng.integers(0, 200000, (len(jobs), 9)).astype(np.uint32)
    ctx = _ctx(g)
    d_rows = torch.from_numpy(rows.view(np.uint8).copy()).cuda()
    ctx.set_nn_inputs(d_rows.data_ptr(), len(jobs))
    try:
        res = ctx.refine(jobs)
    finally:
        ctx.set_nn_inputs(None)
    hadme, fen, nn_mode, qp = (int(v) for v in g["config"])
    o = Oracle(use_hadamard=hadme, nn_mode=nn_mode, qp=qp, fast_inter_mode=fen)
    o.load_nn(weights.load_weights(qp))
    for i, p in enumerate(g["pictures"]):
        o.set_picture(i, p)
    for i, lam in enumerate(g["lambdas"]):
        o.set_lambda(i, float(lam))
    o.set_keys(g["keys"] if g["keys"].size else np.zeros(1, np.int16))
    o.set_nn_inputs(rows)
    want = o.refine(jobs)
    _assert_same(res, want, "EMI | NN_IN")
    both = emi[::3]
    assert np.all(res["n_emi"][both] == 8) and np.array_equal(res["c"][both], rows[both, 8])


def test_1080p_ctu_stream_every_job_against_reference():
    """The job stream the bench times (synth.make_ctu_jobs: HM's CTU order, a smooth motion field,
    the SURVEY §8(d) PU mix; one 1080p LDP QP22 frame, NN on) through the HIP batch path, every job's
    every field - integer MV after EMI, half / quarter offsets, FracDIF cost, C, the EMI pushes, the
    NN class, the final MV, bits and cost - against oracle/_ref (the reference's TLibCommon) run over
    the whole frame in job order from a fresh NN state."""
    from oracle import Reference
    W, H = 1920, 1080
    rng = np.random.default_rng(1000)
    pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs = synth.make_ctu_jobs(rng, W, H, 423, 4, [0, 1, 2, 3], [0])
    assert len(jobs) == 862920
    ctx = _frame_ctx(pics)
    ctx.set_lambda(0, synth.LDP_LAMBDA[22][1])
    a = ctx.refine(jobs)
    ref = Reference(use_hadamard=1, nn_mode=1, fast_inter_mode=1)
    for k, v in pics.items():
        ref.set_picture(k, v)
    ref.set_lambda(0, synth.LDP_LAMBDA[22][1])
    ref.load_nn(weights.load_weights(22))
    want = np.concatenate([ref.refine(jobs[i:i + 50000]) for i in range(0, len(jobs), 50000)])
    fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi",
              "nn_class", "mv_x", "mv_y", "bits", "cost")
    bad, first, counts = compare_results(a, want, fields)
    assert bad == 0, f"1080p CTU stream: {bad} of {len(jobs)} jobs differ, first {first}: {counts}"
