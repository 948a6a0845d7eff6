"""Frame pipeline (nnfme.pipeline.FrameReplay) against the batch alone: ms per step of the
pipelined replay (uploads, batch, downloads) and of back-to-back device-resident batches."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from nnfme import pipeline, synth  # noqa: E402
from nnfme.runtime import FmeContext  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3_qp22"
    if os.environ.get("PIPE_EV_TIMING"):   # A/B: the replay's ordering events with timing enabled
        ev = torch.cuda.Event
        torch.cuda.Event = lambda *a, **k: ev(enable_timing=True)
    wl = bench.WORKLOADS[name]
    bench.W, bench.H, bench.QP = wl["W"], wl["H"], wl["QP"]
    jobs = bench.make_frame_jobs(1000, "ctu", wl["calls"], wl["bipred"])
    ctx = FmeContext(device=0, nn_mode=wl["nn"], qp=wl["QP"], max_jobs=len(jobs) * wl["frames"])
    pool = np.stack([synth.synth_luma(wl["W"], wl["H"], t) for t in range(8)])
    steps = 24
    rep = pipeline.FrameReplay(ctx, jobs, pool, lambda f: bench.frame_lambda(wl, f), steps,
                               frames_per_step=wl["frames"], device=torch.device("cuda", 0))
    rep.prime()
    for k in range(4):
        rep.issue(k, prefetch=k < 3)
    rep.finish()
    torch.cuda.synchronize()
    host = []
    t = time.perf_counter()
    for k in range(4, steps):
        h = time.perf_counter()
        rep.issue(k)
        host.append((time.perf_counter() - h) * 1e3)
    rep.finish()
    wall = (time.perf_counter() - t) * 1e3 / (steps - 4)
    print(f"{name}: pipelined {wall:.3f} ms/step ({rep.n / wall / 1e3:.1f} M PU/s); host issue() median "
          f"{np.median(host):.3f} ms, max {max(host):.3f}")
    t = time.perf_counter()
    for k in range(20):
        ctx.refine_mv_device(rep.d_jobs[0].data_ptr(), rep.d_out[0].data_ptr(), rep.n, rep.s_comp.cuda_stream)
    rep.s_comp.synchronize()
    wall = (time.perf_counter() - t) * 1e3 / 20
    print(f"{name}: device-resident {wall:.3f} ms/step ({rep.n / wall / 1e3:.1f} M PU/s)")


if __name__ == "__main__" and not os.environ.get("PROBE_HOST"):
    main()


def host_calls():
    """Host time of every HIP call issue() makes (PROBE_HOST=1): which one blocks."""
    import collections
    wl = bench.WORKLOADS["c3_qp22"]
    bench.W, bench.H, bench.QP = wl["W"], wl["H"], wl["QP"]
    jobs = bench.make_frame_jobs(1000, "ctu", wl["calls"], wl["bipred"])
    ctx = FmeContext(device=0, nn_mode=1, qp=22, max_jobs=len(jobs))
    pool = np.stack([synth.synth_luma(wl["W"], wl["H"], t) for t in range(8)])
    steps = 24
    rec = collections.defaultdict(list)

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            rec[name].append((time.perf_counter() - t) * 1e3)
            return r
        return w
    pipeline._memcpy_async = timed("memcpy_async", pipeline._memcpy_async)
    for m in ("refine_mv_device", "bind_picture_device", "set_lambda"):
        setattr(ctx, m, timed(m, getattr(ctx, m)))
    rep = pipeline.FrameReplay(ctx, jobs, pool, lambda f: bench.frame_lambda(wl, f), steps,
                               device=torch.device("cuda", 0))
    for ev in rep.ev_in + rep.ev_comp + rep.ev_out:
        ev.record = timed("event_record", ev.record)
    rep.s_comp.wait_event = timed("wait_event", rep.s_comp.wait_event)
    rep.prime()
    for k in range(4):
        rep.issue(k, prefetch=k < 3)
    rep.finish()
    rec.clear()
    t = time.perf_counter()
    for k in range(4, steps):
        h = time.perf_counter()
        rep.issue(k)
        rec["issue"].append((time.perf_counter() - h) * 1e3)
    h = time.perf_counter()
    rep.finish()
    rec["finish"].append((time.perf_counter() - h) * 1e3)
    wall = (time.perf_counter() - t) * 1e3 / (steps - 4)
    print(f"host_calls: pipelined {wall:.3f} ms/step")
    for k, v in rec.items():
        v = np.array(v)
        print(f"  {k:22s} n={len(v):4d} sum={v.sum():8.3f} max={v.max():7.3f} median={np.median(v):.3f} ms")


if __name__ == "__main__" and os.environ.get("PROBE_HOST"):
    host_calls()   # a fresh process: the first replay
    host_calls()
