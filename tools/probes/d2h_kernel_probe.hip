// Device -> pinned host copy by a kernel: bandwidth by workgroup count, workgroup size and store
// flavour (plain / nt / sc0 sc1), against hipMemcpyAsync's own copy, 13.8 MB (one 1080p frame's
// fme_mv_result rows).  Standalone (nothing else runs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void k_dl(const u32x4* __restrict__ src, u32x4* dst, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = src[i];
    if (MODE == 0) dst[i] = v;
    else if (MODE == 1) __builtin_nontemporal_store(v, dst + i);
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(dst + i), "v"(v) : "memory");
  }
}

int main() {
  const size_t bytes = 13806720;
  const long n16 = bytes / 16;
  void *d, *h;
  if (hipMalloc(&d, bytes) != hipSuccess || hipHostMalloc(&h, bytes, 0) != hipSuccess) return 1;
  (void)hipMemset(d, 1, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timeit = [&](auto&& f) {
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 10; r++) f();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
  };
  float ms = timeit([&] { (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0); });
  printf("hipMemcpyAsync D2H: %.3f ms (%.1f GB/s)\n", ms, bytes / ms / 1e6);
  {   // host -> device, the replay's per-step upload size (jobs + two pictures)
    const size_t ub = 31700000 / 16 * 16;
    void *du, *hu;
    if (hipMalloc(&du, ub) != hipSuccess || hipHostMalloc(&hu, ub, 0) != hipSuccess) return 1;
    memset(hu, 3, ub);
    float mu = timeit([&] { (void)hipMemcpyAsync(du, hu, ub, hipMemcpyHostToDevice, 0); });
    printf("hipMemcpyAsync H2D %.1f MB: %.3f ms (%.1f GB/s)\n", ub / 1e6, mu, ub / mu / 1e6);
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t a0, a1, b0, b1;
    (void)hipEventCreate(&a0); (void)hipEventCreate(&a1); (void)hipEventCreate(&b0); (void)hipEventCreate(&b1);
    for (int mode = 0; mode < 2; mode++) {   // 0: both directions on one stream (serial), 1: two streams
      hipStream_t sd = mode ? s2 : s1;
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(a0, s1);
      (void)hipEventRecord(b0, sd);
      for (int r = 0; r < 10; r++) {
        (void)hipMemcpyAsync(du, hu, ub, hipMemcpyHostToDevice, s1);
        (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sd);
      }
      (void)hipEventRecord(a1, s1);
      (void)hipEventRecord(b1, sd);
      (void)hipDeviceSynchronize();
      float ma = 0, mb = 0;
      (void)hipEventElapsedTime(&ma, a0, a1);
      (void)hipEventElapsedTime(&mb, b0, b1);
      printf("%s H2D %.1f MB + D2H %.1f MB: %.3f / %.3f ms per pair\n", mode ? "two non-blocking streams" : "one stream, serial",
             ub / 1e6, bytes / 1e6, ma / 10, mb / 10);
    }
    (void)hipFree(du);
    (void)hipHostFree(hu);
  }
  const int wgs[] = {8, 16, 32, 64, 128, 256, 512, 1024};
  const int thr[] = {64, 256};
  const char* names[] = {"plain", "nt", "sc0sc1"};
  for (int mode = 0; mode < 3; mode++)
    for (int t : thr)
      for (int g : wgs) {
        float m = timeit([&] {
          if (mode == 0) hipLaunchKernelGGL(k_dl<0>, dim3(g), dim3(t), 0, 0, (const u32x4*)d, (u32x4*)h, n16);
          else if (mode == 1) hipLaunchKernelGGL(k_dl<1>, dim3(g), dim3(t), 0, 0, (const u32x4*)d, (u32x4*)h, n16);
          else hipLaunchKernelGGL(k_dl<2>, dim3(g), dim3(t), 0, 0, (const u32x4*)d, (u32x4*)h, n16);
        });
        printf("kernel %-7s %4d WG x %3d: %.3f ms (%.1f GB/s)\n", names[mode], g, t, m, bytes / m / 1e6);
      }
  return 0;
}
