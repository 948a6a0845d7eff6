"""Which D2H path (SDMA engine or a blit kernel on the CUs) hipMemcpyAsync takes for host memory
allocated with each hipHostMalloc flag; run under rocprofv3 --kernel-trace --memory-copy-trace."""
import ctypes as C
import sys
import time

hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
P, I, S = C.c_void_p, C.c_int, C.c_size_t
hip.hipHostMalloc.argtypes = [C.POINTER(P), S, C.c_uint]
hip.hipMalloc.argtypes = [C.POINTER(P), S]
hip.hipMemcpyAsync.argtypes = [P, P, S, I, P]
hip.hipStreamCreate.argtypes = [C.POINTER(P)]
hip.hipStreamSynchronize.argtypes = [P]
hip.hipDeviceSynchronize.argtypes = []
n = 13_800_000
flags = {"default": 0x0, "portable": 0x1, "mapped": 0x2, "writecombined": 0x4, "numa_user": 0x20000000,
         "coherent": 0x40000000, "noncoherent": 0x80000000}
d = P()
assert hip.hipMalloc(C.byref(d), n) == 0
st = P()
assert hip.hipStreamCreate(C.byref(st)) == 0
which = sys.argv[1:] or list(flags)
for name in which:
    h = P()
    rc = hip.hipHostMalloc(C.byref(h), n, flags[name])
    if rc:
        print(name, "alloc rc", rc)
        continue
    for kind, args in (("d2h", (h, d, n, 2, st)), ("h2d", (d, h, n, 1, st))):
        hip.hipMemcpyAsync(*args)
        hip.hipStreamSynchronize(st)
        t = time.perf_counter()
        for _ in range(10):
            hip.hipMemcpyAsync(*args)
        hip.hipStreamSynchronize(st)
        ms = (time.perf_counter() - t) / 10 * 1e3
        print(f"{name:14s} {kind}: {ms:.3f} ms {n / ms / 1e6:.1f} GB/s", flush=True)
