"""Which engine carries a device-to-host hipMemcpyAsync (run under rocprofv3 --kernel-trace):
a blit kernel (__amd_rocclr_copyBuffer in the trace) or SDMA (no kernel).  Variants, separated by
marker fills of distinct sizes: (a) torch pinned tensor, (b) hipHostRegister'd numpy buffer,
(c) hipHostMalloc'd buffer with hipHostMallocNonCoherent (0x40000000... via flags below)."""
import ctypes
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
N = 13_806_720
dev = torch.device("cuda", 0)
src = torch.empty(N, dtype=torch.uint8, device=dev)
s = torch.cuda.Stream(dev)


def marker(k):
    torch.zeros(1024 * (k + 1), dtype=torch.int32, device=dev).add_(1)
    torch.cuda.synchronize()


def copy(dst_ptr, label):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        rc = hip.hipMemcpyAsync(dst_ptr, src.data_ptr(), N, 2, ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, rc
    s.synchronize()
    dt = (time.perf_counter() - t) / 5
    print(f"{label}: {dt * 1e3:.3f} ms per 13.8 MB copy ({N / dt / 1e9:.1f} GB/s)", flush=True)


a = torch.empty(N, dtype=torch.uint8).pin_memory()
marker(1)
copy(a.data_ptr(), "a torch pinned")
b = np.empty(N, np.uint8)
b[:] = 0
assert hip.hipHostRegister(b.ctypes.data, N, 0) == 0
marker(2)
copy(b.ctypes.data, "b hipHostRegister")
for flags, name in ((0x0, "c hipHostMalloc default"), (0x2, "d hipHostMalloc mapped"), (0x80000000, "e hipHostMalloc non-coherent")):
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), N, flags)
    if rc != 0:
        print(name, "hipHostMalloc rc", rc)
        continue
    ctypes.memset(p, 0, N)
    marker(3 + flags % 7)
    copy(p.value, name)
marker(9)
