"""The host-synchronisation-free batch path (fme_refine_device with a device-built schedule):
device-side rejection, the compact fme_mv_result output, back-to-back batches on one stream with
stream-ordered NN state operations, and the carried-state copy used by frame sharding.
Every check is against the golden vectors (oracle/_ref outputs) or the synchronous path."""
import numpy as np
import pytest

from conftest import load_golden
from nnfme.abi import JOB_DTYPE, MV_FIELDS, MV_RESULT_DTYPE, RES_REJECTED, RESULT_DTYPE, compare_results
from test_gpu_parity import _assert_same, _ctx

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def _mv_of(res):
    out = np.zeros(len(res), MV_RESULT_DTYPE)
    for f in MV_FIELDS:
        out[f] = res[f]
    return out


def test_device_batch_rejected_without_host_sync():
    """An invalid job makes the device skip the whole batch: fme_refine_device returns at once,
    fme_refine_status() reports the count, every record is marked and the NN state is unchanged."""
    import torch
    g = load_golden("qp37_nn")
    ctx = _ctx(g)
    ctx.refine(g["jobs"][:100])
    before = ctx.nn_get_state()
    jobs = np.ascontiguousarray(g["jobs"][:64]).copy()
    jobs["w"][5] = 20
    jobs["ref_id"][9] = 40
    dj = _dev(jobs)
    dr = torch.zeros(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx.refine_device(dj.data_ptr(), dr.data_ptr(), len(jobs), s.cuda_stream)
    assert ctx.refine_status() == 2
    res = dr.cpu().numpy().view(RESULT_DTYPE)
    assert np.all(res["status"] == RES_REJECTED)
    assert np.array_equal(ctx.nn_get_state(), before)
    # the context goes on exactly as if the rejected batch had never been issued
    _assert_same(ctx.refine(g["jobs"][100:400]), g["results"][100:400], "after a rejected device batch")
    assert ctx.refine_status() == 0


def test_refine_mv_equals_full_records():
    g = load_golden("ldp_qp22_hadme_fen1_nn")
    want = _mv_of(g["results"])
    want["status"] = _ctx(g).refine(g["jobs"])["status"]   # (the fixtures hold no status bits)
    ctx = _ctx(g)
    got = ctx.refine_mv(g["jobs"])
    for f in MV_FIELDS:
        assert np.array_equal(got[f], want[f]), f
    # device form, in two batches: the NN state crosses them as in the full-record path
    import torch
    ctx2 = _ctx(g)
    n = len(g["jobs"])
    k = n // 3
    dj = _dev(g["jobs"])
    out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx2.refine_mv_device(dj.data_ptr(), out.data_ptr(), k, s.cuda_stream)
    ctx2.refine_mv_device(dj.data_ptr() + k * JOB_DTYPE.itemsize, out.data_ptr() + k * 16, n - k, s.cuda_stream)
    got2 = out.cpu().numpy().view(MV_RESULT_DTYPE)
    for f in MV_FIELDS:
        assert np.array_equal(got2[f], want[f]), f


def test_refine_mv_rejects_invalid_batch():
    from nnfme.runtime import FmeError
    g = load_golden("qp32_nn")
    ctx = _ctx(g)
    j = g["jobs"][:16].copy()
    j["key_offset"][3] = 10 ** 8
    with pytest.raises(FmeError) as e:
        ctx.refine_mv(j)
    assert e.value.code == -1
    got = ctx.refine_mv(g["jobs"][:50])
    assert np.array_equal(got["cost"], g["results"]["cost"][:50])


@pytest.mark.parametrize("case", ["ldp_qp22_hadme_fen1_nn", "fen3_qp27_nn", "sad_fen0_nnoff"])
def test_back_to_back_device_batches(case):
    """Many batches issued without any host wait, with a stream-ordered reset and set_state
    between them, equal the synchronous path batch for batch."""
    import torch
    g = load_golden(case)
    jobs = g["jobs"]
    cuts = [0, 3, 40, 41, 300, len(jobs)]
    parts = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    # synchronous reference: the same sequence of batches and state operations
    ref = _ctx(g)
    want = []
    for t, (a, b) in enumerate(parts):
        if t == 2:
            ref.nn_reset()
        if t == 3:
            ref.nn_set_state(np.arange(1, 13, dtype=np.uint32) * 1000)
        want.append(ref.refine(jobs[a:b]))
    ctx = _ctx(g)
    dj = _dev(jobs)
    dr = torch.zeros(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    states = torch.zeros((len(parts), 12), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for t, (a, b) in enumerate(parts):
        if t == 2:
            ctx.nn_reset()
        if t == 3:
            ctx.nn_set_state(np.arange(1, 13, dtype=np.uint32) * 1000)
        ctx.refine_device(dj.data_ptr() + a * JOB_DTYPE.itemsize, dr.data_ptr() + a * RESULT_DTYPE.itemsize,
                          b - a, s.cuda_stream)
        ctx.nn_copy_state_device(states[t].data_ptr(), s.cuda_stream)
    s.synchronize()
    res = dr.cpu().numpy().view(RESULT_DTYPE)
    for t, (a, b) in enumerate(parts):
        _assert_same(res[a:b], want[t], f"{case} batch {t}")
    assert np.array_equal(states[-1].cpu().numpy().view(np.uint32), ref.nn_get_state())


def test_profiled_back_to_back_batches():
    """Profiling records a ring of event sets without synchronising; every batch is counted."""
    import torch
    g = load_golden("qp32_nn")
    ctx = _ctx(g)
    jobs = g["jobs"]
    dj = _dev(jobs)
    dr = torch.zeros(len(jobs) * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx.set_profiling(True)
    ctx.accumulated_timings(reset=True)
    for _ in range(40):   # more batches than event sets in the ring
        ctx.refine_device(dj.data_ptr(), dr.data_ptr(), len(jobs), s.cuda_stream)
    nb, acc = ctx.accumulated_timings(reset=True)
    ctx.set_profiling(False)
    assert nb == 40
    assert acc["batch"] > 0 and acc["search"] > 0


def test_download_device_into_pinned_rows():
    """fme_download_device (the frame replay's results download): device rows land in pinned host
    memory byte for byte for any workgroup count, also at an offset into the pinned buffer; unaligned
    sizes and pageable host memory are refused."""
    import torch
    from nnfme.runtime import FmeError
    g = load_golden("qp32_nn")
    ctx = _ctx(g)
    rng = np.random.default_rng(5)
    n = (1 << 20) + 16 * 37
    src = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).cuda()
    dst = torch.zeros(n + 4096, dtype=torch.uint8).pin_memory()
    s = torch.cuda.current_stream()
    for wgs in (0, 1, 3, 8, 64):
        dst.zero_()
        ctx.download_device(src.data_ptr(), dst.data_ptr(), n, wgs, s.cuda_stream)
        s.synchronize()
        assert torch.equal(dst[:n], src.cpu()), wgs
        assert not dst[n:].any()
    dst.zero_()
    ctx.download_device(src.data_ptr() + 64, dst.data_ptr() + 4096, n - 64, 8, s.cuda_stream)
    s.synchronize()
    assert torch.equal(dst[4096:4096 + n - 64], src[64:].cpu())
    with pytest.raises(FmeError):
        ctx.download_device(src.data_ptr(), dst.data_ptr(), 100, 8, s.cuda_stream)
    pageable = np.zeros(4096, np.uint8)
    with pytest.raises(FmeError):
        ctx.download_device(src.data_ptr(), pageable.ctypes.data, 4096, 8, s.cuda_stream)


def test_device_built_keys_rejection_cycle():
    """fme_build_bipred_keys_device with one invalid request (a key block beyond the buffer): a later
    batch whose jobs read keys is rejected on the device; a batch of uni-pred jobs is not; a clean
    rebuild clears the rejection (fme.h, 'rejected until keys are built again')."""
    import torch
    from nnfme import synth
    from nnfme.abi import BIKEY_REQ_DTYPE, JOB_BIPRED, MV_RESULT_DTYPE
    W, H = 416, 240
    rng = np.random.default_rng(41)
    pics = {k: synth.synth_luma(W, H, t) for k, t in zip(range(5), (7, 6, 5, 4, 0))}
    jobs = synth.make_ctu_jobs(rng, W, H, 64, 4, [0, 1, 2, 3], [0], bipred_frac=0.3)
    reqs, key_count = synth.make_bipred_key_reqs(np.random.default_rng(7), jobs, 4, [0, 1, 2, 3])
    from nnfme.runtime import FmeContext
    ctx = FmeContext(nn_mode=1, qp=22, max_jobs=len(jobs))
    for k, v in pics.items():
        ctx.set_picture(k, v)
    ctx.set_lambda(0, synth.LDP_LAMBDA[22][1])
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    bad = np.array(reqs, dtype=BIKEY_REQ_DTYPE, copy=True)
    bad["key_offset"][len(bad) // 2] = key_count          # block beyond the key buffer
    bi = (jobs["flags"] & JOB_BIPRED) != 0
    assert bi.any() and (~bi).any()
    uni = np.ascontiguousarray(jobs[~bi])

    def run(js):
        dj = torch.from_numpy(np.ascontiguousarray(js).view(np.uint8).copy()).to(dev)
        out = torch.zeros(len(js) * MV_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        ctx.refine_mv_device(dj.data_ptr(), out.data_ptr(), len(js), s.cuda_stream)
        st = ctx.refine_status()
        return st, out.cpu().numpy().view(MV_RESULT_DTYPE)

    d_bad = torch.from_numpy(bad.view(np.uint8).copy()).to(dev)
    ctx.build_bipred_keys_device(d_bad.data_ptr(), len(bad), key_count, s.cuda_stream)
    st, out = run(jobs)
    assert st > 0 and np.all(out["status"] & RES_REJECTED), "key batch not rejected"
    st, out = run(uni)
    assert st == 0 and not np.any(out["status"] & RES_REJECTED), "uni-pred batch rejected"
    d_good = torch.from_numpy(np.ascontiguousarray(reqs).view(np.uint8).copy()).to(dev)
    ctx.build_bipred_keys_device(d_good.data_ptr(), len(reqs), key_count, s.cuda_stream)
    st, out = run(jobs)
    assert st == 0 and not np.any(out["status"] & RES_REJECTED), "rejection not cleared by a clean rebuild"
