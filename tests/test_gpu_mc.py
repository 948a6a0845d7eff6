"""GPU parity of motion compensation: the HIP path through the C-ABI
(fme_motion_compensate / fme_motion_compensate_device) against the golden planes made by the
reference's own TComInterpolationFilter + TComYuv::addAvg (oracle/_ref) and against the C
restatement (orc_mc) on a full 1080p frame partition.  Integer output: bit-exact."""
import numpy as np
import pytest

from conftest import load_golden, mc10_golden_cases, mc_golden_cases, mc_inputs
from nnfme import synth
from nnfme.abi import MC_JOB_DTYPE, MC_L0, MC_L1

pytestmark = pytest.mark.gpu


def _ctx(pics):
    from nnfme.runtime import FmeContext
    ctx = FmeContext(nn_mode=0)
    for k, (y, cb, cr) in pics.items():
        ctx.set_picture_yuv(k, y, cb, cr)
    return ctx


def _same(got, exp, what):
    for g, e, comp in zip(got, exp, ("Y", "Cb", "Cr")):
        assert np.array_equal(g, e), f"{what} {comp}: {int((g != e).sum())} samples differ"


@pytest.mark.parametrize("case", mc_golden_cases())
def test_mc_golden(case):
    g = load_golden(case)
    pics, jobs, planes = mc_inputs(g)
    _ctx(pics).motion_compensate(jobs, *planes)
    _same(planes, (g["pred_y"], g["pred_cb"], g["pred_cr"]), case)


@pytest.mark.parametrize("case", mc10_golden_cases())
def test_mc10_golden(case):
    """Bit depth 10 (main10): uint16 planes through fme_motion_compensate against the reference's
    own filters and addAvg at bitDepth 10 (k_mc10)."""
    from nnfme.runtime import FmeContext
    g = load_golden(case)
    pics, jobs, planes = mc_inputs(g)
    ctx = FmeContext(nn_mode=0, bit_depth=10)
    for k, (y, cb, cr) in pics.items():
        ctx.set_picture_yuv(k, y, cb, cr)
    ctx.motion_compensate(jobs, *planes)
    _same(planes, (g["pred_y"], g["pred_cb"], g["pred_cr"]), case)


def test_mc10_device_frame_matches_reference():
    """A 416x240 main10 partition (every PU shape, 40 % bi-pred, MVs up to +-150 quarter-pel so
    clipMv acts at the borders) with device-resident jobs and uint16 planes, against oracle/_ref
    at bitDepth 10 run live."""
    import torch
    from nnfme.runtime import FmeContext
    from oracle import Reference
    W, H = 416, 240
    rng = np.random.default_rng(5)
    pics = {}
    for k in range(3):
        cb, cr = synth.synth_chroma(W, H, k)
        lo = rng.integers(0, 4, size=(2,) + cb.shape, dtype=np.uint16)
        pics[k] = (synth.synth_luma_hbd(W, H, k, bit_depth=10), (cb.astype(np.uint16) << 2) | lo[0],
                   (cr.astype(np.uint16) << 2) | lo[1])
    jobs = synth.make_mc_partition(rng, W, H, [0, 1, 2], bi_frac=0.4, mv_amp=150, identical_frac=0.1)
    ctx = FmeContext(nn_mode=0, bit_depth=10)
    ref = Reference(bit_depth=10)
    for k, p in pics.items():
        ctx.set_picture_yuv(k, *p)
        ref.set_picture_yuv(k, *p)
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    dy = torch.zeros((H, W), dtype=torch.int16, device=dev)
    dcb = torch.zeros((H // 2, W // 2), dtype=torch.int16, device=dev)
    dcr = torch.zeros_like(dcb)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.motion_compensate_device(dj.data_ptr(), len(jobs), dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(), W // 2,
                                 W, H, s)
    assert ctx.mc_invalid_count() == 0
    exp = (np.zeros((H, W), np.uint16), np.zeros((H // 2, W // 2), np.uint16), np.zeros((H // 2, W // 2), np.uint16))
    ref.mc(jobs, *exp)
    got = tuple(t.cpu().numpy().view(np.uint16) for t in (dy, dcb, dcr))
    _same(got, exp, "416x240 main10")


def _frame(W, H, refs, seed):
    pics = {}
    for k in range(refs):
        cb, cr = synth.synth_chroma(W, H, k)
        pics[k] = (synth.synth_luma(W, H, k), cb, cr)
    return pics


def test_mc_device_1080p_matches_oracle():
    """A whole 1080p partition (every PU shape, 30 % bi-pred, 10 % identical motion, MVs up to
    +-96 pel so clipMv acts at the borders), device-resident jobs and planes."""
    import torch
    from oracle import Oracle
    W, H = 1920, 1080
    pics = _frame(W, H, 4, 2)
    rng = np.random.default_rng(77)
    jobs = synth.make_mc_partition(rng, W, H, [0, 1, 2, 3], bi_frac=0.3, mv_amp=96, identical_frac=0.1)
    ctx = _ctx(pics)
    dev = torch.device("cuda", 0)
    dj = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    dy = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    dcb = torch.zeros((H // 2, W // 2), dtype=torch.uint8, device=dev)
    dcr = torch.zeros_like(dcb)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.motion_compensate_device(dj.data_ptr(), len(jobs), dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(), W // 2,
                                 W, H, s)
    assert ctx.mc_invalid_count() == 0
    exp = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
    Oracle().mc(pics, jobs, *exp)
    _same((dy.cpu().numpy(), dcb.cpu().numpy(), dcr.cpu().numpy()), exp, "1080p")
    # run-to-run determinism on the same buffers
    ctx.motion_compensate_device(dj.data_ptr(), len(jobs), dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(), W // 2,
                                 W, H, s)
    _same((dy.cpu().numpy(), dcb.cpu().numpy(), dcr.cpu().numpy()), exp, "1080p rerun")


def test_mc_invalid_jobs():
    from nnfme.runtime import FmeError
    W, H = 128, 64
    pics = _frame(W, H, 2, 5)
    ctx = _ctx(pics)
    jobs = np.zeros(3, MC_JOB_DTYPE)
    jobs["w"], jobs["h"], jobs["flags"] = 16, 16, MC_L0
    jobs["x"] = [0, 16, 32]
    planes = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
    bad = jobs.copy()
    bad["w"][1] = 6                       # not a PU size
    with pytest.raises(FmeError, match="job 1: PU size"):
        ctx.motion_compensate(bad, *planes)
    bad = jobs.copy()
    bad["ref_id"][2, 0] = 7               # no such picture
    with pytest.raises(FmeError, match="job 2"):
        ctx.motion_compensate(bad, *planes)
    bad = jobs.copy()
    bad["flags"][0] = 0                   # no list
    with pytest.raises(FmeError, match="job 0"):
        ctx.motion_compensate(bad, *planes)
    assert not planes[0].any()            # nothing ran
    ctx.set_picture(5, synth.synth_luma(W, H, 3))   # luma only: no motion compensation from it
    bad = jobs.copy()
    bad["flags"][0] = MC_L0 | MC_L1
    bad["ref_id"][0] = (0, 5)
    with pytest.raises(FmeError, match="chroma"):
        ctx.motion_compensate(bad, *planes)
    # device path: invalid jobs are skipped and counted, the rest still predicted
    import torch
    from oracle import Oracle
    dev = torch.device("cuda", 0)
    bad = jobs.copy()
    bad["x"][1] = W - 8                   # outside the picture
    dj = torch.from_numpy(bad.view(np.uint8).copy()).to(dev)
    dy = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    dcb = torch.zeros((H // 2, W // 2), dtype=torch.uint8, device=dev)
    dcr = torch.zeros_like(dcb)
    ctx.motion_compensate_device(dj.data_ptr(), 3, dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(), W // 2, W, H,
                                 torch.cuda.current_stream(dev).cuda_stream)
    assert ctx.mc_invalid_count() == 1
    exp = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
    Oracle().mc({0: pics[0]}, bad[[0, 2]], *exp)
    _same((dy.cpu().numpy(), dcb.cpu().numpy(), dcr.cpu().numpy()), exp, "skip invalid")


def test_mc_empty_and_profiled():
    W, H = 64, 64
    pics = _frame(W, H, 1, 9)
    ctx = _ctx(pics)
    planes = (np.zeros((H, W), np.uint8), np.zeros((H // 2, W // 2), np.uint8), np.zeros((H // 2, W // 2), np.uint8))
    ctx.motion_compensate(np.zeros(0, MC_JOB_DTYPE), *planes)
    ctx.set_profiling(True)
    jobs = synth.make_mc_partition(np.random.default_rng(1), W, H, [0])
    ctx.motion_compensate(jobs, *planes)
    assert ctx.mc_last_ms() > 0.0
