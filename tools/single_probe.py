#!/usr/bin/env python3
"""Drop-in call latency breakdown: host wall time per fme_frac_dif_single / fme_nn_pred_single call
(through ctypes, so a little above the C++ figure) against the server's device service time
(fme_single_last_device_us): the difference is host + PCIe + polling.

usage: python tools/single_probe.py [calls]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hm16.9-nn_fme_amd"))


def main():
    from nnfme import synth, weights
    from nnfme.runtime import FmeContext
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    ctx = FmeContext(nn_mode=1, qp=22)
    ctx.load_nn(weights.load_weights(22))
    W, H, pad = 416, 240, 80
    pic = np.pad(synth.synth_luma(W, H, 1).astype(np.int16), pad, mode="edge")
    org = synth.synth_luma(W, H, 2).astype(np.int16)
    rng = np.random.default_rng(3)
    ml = 65536.0 * np.sqrt(synth.LDP_LAMBDA[22][0])
    for (w, h) in ((8, 8), (16, 16), (64, 64)):
        wall, dev, ph = [], [], []
        for i in range(calls):
            x, y = 4 * int(rng.integers(0, (W - w) // 4)), 4 * int(rng.integers(0, (H - h) // 4))
            key = org[y:y + h, x:x + w]
            mv = tuple(int(v) for v in rng.integers(-8, 9, 2))
            mvp = tuple(int(v) for v in rng.integers(-16, 17, 2))
            t0 = time.perf_counter()
            ctx.frac_dif_single(key, pic, (y + pad, x + pad), mv, mvp, ml)
            wall.append(time.perf_counter() - t0)
            p = ctx.single_last_device_us(phases=True)
            dev.append(p[0])
            ph.append(p[1:])
        m = np.median(np.array(ph[1:]), axis=0)
        print(f"frac_dif {w}x{h}: wall {np.median(wall[1:]) * 1e6:.2f} us, device {np.median(dev[1:]):.2f} us "
              f"(payload {m[0]:.2f}, first stage {m[1]:.2f}, half dist {m[2]:.2f}, quarter dist {m[3]:.2f})", flush=True)
    wall, dev, net = [], [], []
    for i in range(calls):
        e = rng.integers(0, 5000, 8).astype(np.uint32)
        t0 = time.perf_counter()
        ctx.nn_pred_single(e, int(rng.integers(0, 5000)), 8, 8)
        wall.append(time.perf_counter() - t0)
        p = ctx.single_last_device_us(phases=True)
        dev.append(p[0])
        net.append(p[1:3])
    # the NN marks: shader-clock cycles of the net (reported through the 100 MHz wall scale) and
    # its wall time, so their ratio is the shader clock while the server runs
    cyc, nus = np.median(np.array(net[1:]), axis=0)
    print(f"nn_pred: wall {np.median(wall[1:]) * 1e6:.2f} us, device {np.median(dev[1:]):.2f} us, "
          f"net {nus:.2f} us = {cyc * 100:.0f} shader cycles ({cyc * 100 / max(nus, 1e-3):.0f} MHz)", flush=True)


if __name__ == "__main__":
    main()
