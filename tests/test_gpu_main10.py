"""Bit depth 10 (the main10 configurations: cfg/encoder_lowdelay_P_main10.cfg:58,
encoder_randomaccess_main10.cfg:60, encoder_lowdelay_main10.cfg:56 InternalBitDepth 10) through
the HIP path: 16-bit pictures, the lane-per-unit search kernel on int16 samples
(csrc/fme_lane10.hip), the same NN tail; the single-call FracDIF as a one-job batch.

Bit-exact against the main10 goldens (oracle/_ref's TComInterpolationFilter / TComRdCost at
bitDepth 10, the C oracle agreeing) and, over a whole 416x240 frame in HM's CTU order, every field
of every job against oracle/_ref run live."""
import numpy as np
import pytest

from conftest import load_golden, main10_golden_cases
from nnfme import synth, weights
from nnfme.abi import JOB_DTYPE, MV_FIELDS, MV_RESULT_DTYPE, RESULT_DTYPE, compare_results
from test_gpu_parity import _assert_same, _ctx, _frac_single_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", main10_golden_cases())
def test_main10_golden(case):
    g = load_golden(case)
    assert int(g["bit_depth"][0]) == 10
    _assert_same(_ctx(g).refine(g["jobs"]), g["results"], case)


@pytest.mark.parametrize("case", main10_golden_cases())
def test_main10_golden_split_batches_and_device_path(case):
    """Batches split anywhere carry the NN state; the device-resident compact-record path gives
    the same outputs."""
    import torch
    g = load_golden(case)
    ctx = _ctx(g)
    j = g["jobs"]
    cuts = [0, 1, 9, 250, len(j) - 3, len(j)]
    parts = [ctx.refine(j[a:b]) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    _assert_same(np.concatenate(parts), g["results"], case + " split")
    ctx2 = _ctx(g)
    dj = torch.from_numpy(np.ascontiguousarray(j).view(np.uint8).copy()).cuda()
    out = torch.zeros(len(j) * MV_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx2.refine_mv_device(dj.data_ptr(), out.data_ptr(), len(j), s.cuda_stream)
    assert ctx2.refine_status() == 0
    got = out.cpu().numpy().view(MV_RESULT_DTYPE)
    for f in ("mv_x", "mv_y", "cost", "bits", "nn_class"):
        assert np.array_equal(got[f], g["results"][f]), f


def test_main10_context_limits():
    """12 bits is refused at creation with FME_E_UNSUPPORTED (-4); every entry point runs at 10 bits
    (integer search: test_gpu_tz.py's tz10_* goldens; producers and template costs:
    test_main10_producers.py; motion compensation: test_gpu_mc.py); NN_pred is bit-depth independent."""
    from nnfme.runtime import FmeContext, FmeError
    g = load_golden(main10_golden_cases()[0])
    ctx = _ctx(g)
    with pytest.raises(FmeError) as e:
        FmeContext(bit_depth=12)
    assert e.value.code == -4
    cls, _ = ctx.nn_pred_single(np.arange(1, 9, dtype=np.uint32) * 1000, 777, 8, 8)
    assert 0 <= cls < 49


@pytest.mark.parametrize("case", main10_golden_cases())
def test_main10_frac_dif_single_every_shape(case):
    """xPatternSearchFracDIF's single-PU entry point at bit depth 10 (a one-job batch on a private
    10-bit context): rcMvHalf, rcMvQter and ruiCost equal the main10 goldens' FracDIF fields for
    every PU shape (up to 4 jobs per shape, keyed bi-pred jobs and lossless jobs included), and the
    caller's context is untouched (its batch still matches afterwards)."""
    g = load_golden(case)
    jobs = g["jobs"]
    idx = []
    for (w, h) in synth.ALL_PU_SIZES:
        sel = np.flatnonzero((jobs["w"] == w) & (jobs["h"] == h))
        idx += list(sel[:: max(1, len(sel) // 4)][:4])
    idx += list(np.flatnonzero(jobs["flags"] & 4)[:4])
    idx += list(np.flatnonzero(jobs["key_offset"] >= 0)[:4])
    ctx = _ctx(g)
    _frac_single_check(ctx, g, idx)
    ctx.nn_reset()
    _assert_same(ctx.refine(jobs), g["results"], case + " after single calls")


def test_main10_frame_every_job_against_reference():
    """One 416x240 main10 frame (HM's CTU order, the §8(d) PU mix, 4 references, NN on, FEN 1):
    every field of every job against oracle/_ref run live from a fresh NN state."""
    from oracle import Reference
    from nnfme.runtime import FmeContext
    W, H = 416, 240
    pics = {k: synth.synth_luma_hbd(W, H, t, 10) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs = synth.make_ctu_jobs(np.random.default_rng(10), W, H, 331, 4, [0, 1, 2, 3], [0])
    lam = synth.LDP_LAMBDA[22][1]
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1, max_jobs=len(jobs), bit_depth=10)
    ref = Reference(use_hadamard=1, nn_mode=1, fast_inter_mode=1, bit_depth=10)
    for e in (ctx, ref):
        for k, v in pics.items():
            e.set_picture(k, v)
        e.set_lambda(0, lam)
    ref.load_nn(weights.load_weights(22))
    a = ctx.refine(jobs)
    want = ref.refine(jobs)
    fields = ("mv_int_x", "mv_int_y", "half_x", "half_y", "qtr_x", "qtr_y", "frac_cost", "c", "n_emi",
              "nn_class", "mv_x", "mv_y", "bits", "cost")
    bad, first, counts = compare_results(a, want, fields)
    assert bad == 0, f"main10 frame: {bad} of {len(jobs)} jobs differ, first {first}: {counts}"
    assert JOB_DTYPE.itemsize == 32 and RESULT_DTYPE.itemsize == 64 and MV_FIELDS


def test_main10_frame_replay_against_reference():
    """The bench's replay (FrameReplay: per-step uploads of 16-bit originals and reconstructions,
    pictures bound with the stride in samples, the results downloaded by the library's kernel) at
    bit depth 10, two frames per step over three steps: every step's results equal oracle/_ref run
    frame after frame with that step's pictures, lambdas and the NN state carried across steps."""
    import torch
    from nnfme import pipeline
    from nnfme.pipeline import FrameReplay
    from nnfme.runtime import FmeContext
    from oracle import Reference
    w, h, F, steps = 416, 240, 2, 3
    base = synth.make_ctu_jobs(np.random.default_rng(43), w, h, 200, 4, [0, 1, 2, 3], [0])
    pool = np.stack([synth.synth_luma_hbd(w, h, t, 10) for t in range(8)])
    assert pool.dtype == np.uint16 and int(pool.max()) > 255
    lam = lambda f: synth.LDP_LAMBDA[22][(f + 1) % 4]   # noqa: E731
    ctx = FmeContext(nn_mode=1, qp=22, fast_inter_mode=1, bit_depth=10)
    rep = FrameReplay(ctx, base, pool, lam, steps, frames_per_step=F, device=torch.device("cuda", 0))
    rep.prime()
    for k in range(steps):
        rep.issue(k)
    rep.finish()
    ref = Reference(use_hadamard=1, nn_mode=1, fast_inter_mode=1, bit_depth=10)
    ref.load_nn(weights.load_weights(22))
    for k in range(steps):
        f0 = rep.first_frame(k)
        for j in range(F):
            ref.set_picture(pipeline.ORG0 + j, pool[(f0 + j) % 8])
            ref.set_lambda(j, lam(f0 + j))
        for s in range(F + pipeline.REFS - 1):
            ref.set_picture(s, pool[(f0 - pipeline.REFS + s) % 8])
        want = ref.refine(rep.jobs)
        got = rep.results(k)
        for f in ("mv_x", "mv_y", "cost", "bits", "nn_class"):
            bad = np.flatnonzero(got[f] != want[f])
            assert len(bad) == 0, f"step {k}: {f} differs at {len(bad)} jobs, first {bad[:5]}"
