"""A/B of the results download beside the next step's search: the frame replay of
the headline workload with each download engine, the search kernel's HIP-event time per batch (mean,
median, max over the timed steps) and the pipelined ms/step, against device-resident batches.

  python tools/download_engine_ab.py [steps]        (one process, every variant, same inputs)
Variants: blit (hipMemcpyAsync = ROCclr's copy kernel), kernel:W (fme_download_device with W one-wave
workgroups), each deferred (the download starts once the next search runs) or immediate."""
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


def run(ctx, jobs, pool, wl, steps, engine, wgs, defer):
    rep = pipeline.FrameReplay(ctx, jobs, pool, lambda f: bench.frame_lambda(wl, f), steps,
                               device=torch.device("cuda", 0), defer_download=defer,
                               download_engine=engine, download_wgs=wgs)
    rep.prime()
    for k in range(3):
        rep.issue(k, prefetch=k < 2)
    rep.finish()
    torch.cuda.synchronize()
    ctx.set_profiling(True)
    search = []
    t = time.perf_counter()
    for k in range(3, steps):
        rep.issue(k)
    rep.finish()
    wall = (time.perf_counter() - t) * 1e3 / (steps - 3)
    # per-batch search times: re-read the event ring one batch at a time is not exposed; use the
    # accumulated mean and, per batch, fme_last_timings after a synchronised replay of single steps
    nb, acc = ctx.accumulated_timings(reset=True)
    ctx.set_profiling(False)
    rep.check_status(3)
    return wall, acc["search_main"] / max(nb, 1), rep


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    wl = bench.WORKLOADS["c3_qp22"]
    bench.W, bench.H, bench.QP = wl["W"], wl["H"], wl["QP"]
    jobs = bench.make_frame_jobs(1000, "ctu", wl["calls"], wl["bipred"])
    ctx = FmeContext(device=0, nn_mode=1, qp=22, max_jobs=len(jobs))
    pool = np.stack([synth.synth_luma(wl["W"], wl["H"], t) for t in range(8)])
    variants = [("blit", 0, True), ("kernel", 8, True), ("kernel", 4, True), ("kernel", 16, True),
                ("kernel", 32, True), ("kernel", 8, False), ("blit", 0, True), ("kernel", 8, True)]
    ref = None
    for engine, wgs, defer in variants:
        wall, search, rep = run(ctx, jobs, pool, wl, steps, engine, wgs, defer)
        out = rep.results(steps - 1).copy()
        same = "" if ref is None else (" results identical" if np.array_equal(out, ref) else " RESULTS DIFFER")
        ref = out if ref is None else ref
        print(f"{engine}:{wgs} {'deferred' if defer else 'immediate'}: {wall:.3f} ms/step "
              f"({rep.n / wall / 1e3:.1f} M PU/s), search mean {search:.3f} ms{same}", flush=True)
        del rep
    comp = torch.cuda.current_stream()
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_out = torch.empty(len(jobs) * 16, dtype=torch.uint8, device="cuda")
    for k, t in zip(range(5), (7, 6, 5, 4, 0)):
        ctx.set_picture(k, synth.synth_luma(bench.W, bench.H, t))
    ctx.set_lambda(0, bench.frame_lambda(wl, 0))
    for _ in range(3):
        ctx.refine_mv_device(d_jobs.data_ptr(), d_out.data_ptr(), len(jobs), comp.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        ctx.refine_mv_device(d_jobs.data_ptr(), d_out.data_ptr(), len(jobs), comp.cuda_stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3 / 20
    print(f"device-resident: {wall:.3f} ms/step ({len(jobs) / wall / 1e3:.1f} M PU/s)", flush=True)


if __name__ == "__main__":
    main()
