#!/usr/bin/env python3
"""Motion-compensation timing probe: kernel ms (library HIP events) against the number of PUs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    import torch
    from nnfme import synth
    from nnfme.runtime import FmeContext
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    ctx = FmeContext(nn_mode=0)
    for k in range(4):
        cb, cr = synth.synth_chroma(W, H, k)
        ctx.set_picture_yuv(k, synth.synth_luma(W, H, k), cb, cr)
    jobs = synth.make_mc_partition(np.random.default_rng(5), W, H, [0, 1, 2, 3], mv_amp=64)
    dy = torch.zeros((H, W), dtype=torch.uint8, device=dev)
    dcb = torch.zeros((H // 2, W // 2), dtype=torch.uint8, device=dev)
    dcr = torch.zeros_like(dcb)
    s = torch.cuda.current_stream(dev)
    ctx.set_profiling(True)
    t = torch.zeros(16, device=dev)
    for _ in range(50):
        t.add_(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(200):
        t.add_(1)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"calibration: trivial torch kernel {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch", flush=True)
    ctx.set_profiling(False)
    dj = torch.from_numpy(jobs[:1].view(np.uint8).copy()).to(dev)
    e0.record(s)
    for _ in range(200):
        ctx.motion_compensate_device(dj.data_ptr(), 1, dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(), W // 2, W, H,
                                     s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"calibration: 1-PU motion compensation (profiling off) {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per call",
          flush=True)
    ctx.set_profiling(True)
    for n in (1, 16, 256, 1024, 4096, len(jobs)):
        for variant in ("prefix", "zero_mv", "int_mv"):
            jj = jobs[:n].copy()
            if variant == "zero_mv":
                jj["mv"] = 0
            elif variant == "int_mv":
                jj["mv"] &= ~3
            dj = torch.from_numpy(jj.view(np.uint8).copy()).to(dev)
            ms = []
            for r in range(8):
                ctx.motion_compensate_device(dj.data_ptr(), n, dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(),
                                             W // 2, W, H, s.cuda_stream)
                ms.append(ctx.mc_last_ms())
            x = torch.randn(4096, 4096, device=dev)
            for _ in range(20):   # keep the GPU busy (clocks up) right before the timed calls
                x = x @ x
                x = x / x.norm()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for r in range(200):
                ctx.motion_compensate_device(dj.data_ptr(), n, dy.data_ptr(), W, dcb.data_ptr(), dcr.data_ptr(),
                                             W // 2, W, H, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            print(f"n={n:6d} {variant:8s} kernel ms med {np.median(ms[2:]):.4f} | torch-event per call "
                  f"{e0.elapsed_time(e1) / 200:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
