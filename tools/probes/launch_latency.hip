// Probe: host-observed latency of one kernel round trip on this box (the floor of a synchronous
// single-PU call): empty launch + hipStreamSynchronize, launch + host spin on a flag the kernel
// writes to mapped host memory, and a polling "service" wave answering a mailbox in mapped host
// memory (no launch per request).  Median microseconds over 2,000 calls each.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}
__global__ void k_flag(volatile int* f, int v) {
  if (threadIdx.x == 0) { *f = v; __threadfence_system(); }
}
// mailbox: m[0] = request sequence (host), m[1] = answered sequence (device), m[2] = quit
__global__ void k_service(volatile int* m) {
  if (threadIdx.x != 0) return;
  int last = 0;
  for (long it = 0; it < 200000000L; it++) {   // bounded: exits on quit or after the bound
    const int q = m[2];
    if (q) break;
    const int r = m[0];
    if (r != last) {
      last = r;
      m[1] = r;
      __threadfence_system();
    } else {
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

static double med(std::vector<double>& v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
  using clk = std::chrono::steady_clock;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* hm = nullptr;
  (void)hipHostMalloc((void**)&hm, 4096, hipHostMallocMapped | hipHostMallocCoherent);
  int* dm = nullptr;
  (void)hipHostGetDevicePointer((void**)&dm, hm, 0);
  const int N = 2000;
  std::vector<double> a, b, c;
  for (int i = 0; i < N; i++) {
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
    (void)hipStreamSynchronize(s);
    a.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  for (int i = 0; i < N; i++) {
    volatile int* f = hm;
    auto t0 = clk::now();
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, (volatile int*)dm, i + 1);
    while (*f != i + 1) {}
    b.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  (void)hipStreamSynchronize(s);
  hm[0] = hm[1] = hm[2] = 0;
  hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, s, (volatile int*)dm);
  volatile int* vm = hm;
  for (int i = 0; i < N; i++) {
    auto t0 = clk::now();
    vm[0] = i + 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    long spins = 0;
    while (vm[1] != i + 1 && spins < 100000000L) spins++;
    c.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  vm[2] = 1;
  (void)hipStreamSynchronize(s);
  printf("{\"launch_sync_us\": %.2f, \"launch_flag_us\": %.2f, \"service_mailbox_us\": %.2f}\n", med(a), med(b), med(c));
  return 0;
}
