"""PCIe copy probe: pinned H2D / D2H rates alone, together, and beside a busy kernel stream;
prints which HSA/HIP copy settings the box has."""
import os
import time

import torch

print({k: v for k, v in os.environ.items() if any(s in k for s in ("SDMA", "HSA", "HIP", "GPU_", "ROC"))})
dev = torch.device("cuda", 0)
n_h2d, n_d2h = 31_700_000, 13_800_000
h_in = torch.empty(n_h2d, dtype=torch.uint8).pin_memory()
d_in = torch.empty(n_h2d, dtype=torch.uint8, device=dev)
d_out = torch.empty(n_d2h, dtype=torch.uint8, device=dev)
h_out = torch.empty(n_d2h, dtype=torch.uint8).pin_memory()
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


for name, fn, nbytes in (("h2d", h2d, n_h2d), ("d2h", d2h, n_d2h), ("both", both, n_h2d + n_d2h)):
    ms = timed(fn)
    print(f"{name}: {ms:.3f} ms, {nbytes / ms / 1e6:.1f} GB/s")
