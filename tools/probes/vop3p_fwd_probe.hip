// Does a packed-math (VOP3P) result need a wait state before the next VALU reads it on gfx950?
// LLVM (ROCm 7.2) inserts `s_nop 0` after every v_pk_* whose result the next instruction reads
// (its dst-sel forwarding hazard check reads VOP3P's op_sel_hi bit as VOP3's dst op_sel).  This
// probe runs dependent v_pk_* chains written in ONE asm block (no wait states between them) on
// random inputs and compares every lane with the host's restatement; any mismatch means the
// hazard is real.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

__global__ void k_chain(const uint32_t* a, const uint32_t* b, uint32_t* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = a[i], y = b[i], d, m, s, t;
  // d = x - y; m = max(d, -d) (pk_abs); s = m + y; t = dot2(s, x) + m - every step reads the previous
  // instruction's result with no wait state in between
  asm volatile(
      "v_pk_sub_i16 %0, %4, %5\n\t"
      "v_pk_sub_i16 %1, 0, %0\n\t"
      "v_pk_max_i16 %1, %0, %1\n\t"
      "v_pk_add_u16 %2, %1, %5\n\t"
      "v_pk_mad_u16 %2, %2, %4, %1\n\t"
      "v_dot2_u32_u16 %3, %2, %1, %1\n\t"
      : "=&v"(d), "=&v"(m), "=&v"(s), "=&v"(t)
      : "v"(x), "v"(y));
  o[i] = t;
}

static inline int16_t lo(uint32_t v) { return (int16_t)(v & 0xFFFF); }
static inline int16_t hi(uint32_t v) { return (int16_t)(v >> 16); }
static inline uint32_t pk(int a, int b) { return ((uint32_t)(uint16_t)a) | ((uint32_t)(uint16_t)b << 16); }

int main() {
  const int n = 1 << 22;
  std::vector<uint32_t> a(n), b(n), o(n), e(n);
  srand(1);
  for (int i = 0; i < n; i++) {
    a[i] = ((uint32_t)rand() << 1) ^ (uint32_t)rand();
    b[i] = ((uint32_t)rand() << 1) ^ (uint32_t)rand();
    const int d0 = (int16_t)(lo(a[i]) - lo(b[i])), d1 = (int16_t)(hi(a[i]) - hi(b[i]));
    const int m0 = d0 > (int16_t)(-d0) ? d0 : (int16_t)(-d0), m1 = d1 > (int16_t)(-d1) ? d1 : (int16_t)(-d1);
    const uint32_t m = pk(m0, m1);
    const uint32_t s = pk((uint16_t)(m0 + (uint16_t)lo(b[i])), (uint16_t)(m1 + (uint16_t)hi(b[i])));
    const uint32_t s2 = pk((uint16_t)((uint16_t)lo(s) * (uint16_t)lo(a[i]) + (uint16_t)m0),
                           (uint16_t)((uint16_t)hi(s) * (uint16_t)hi(a[i]) + (uint16_t)m1));
    e[i] = (uint32_t)(uint16_t)lo(s2) * (uint16_t)lo(m) + (uint32_t)(uint16_t)hi(s2) * (uint16_t)hi(m) + m;
  }
  uint32_t *da, *db, *dout;
  hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
  long bad = 0;
  for (int rep = 0; rep < 20; rep++) {
    hipLaunchKernelGGL(k_chain, dim3(n / 256), dim3(256), 0, 0, da, db, dout, n);
    hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; i++) bad += o[i] != e[i];
  }
  printf("vop3p forwarding probe: %ld mismatches in %d lanes x 20 runs%s\n", bad, n, bad ? " (HAZARD REAL)" : "");
  hipFree(da); hipFree(db); hipFree(dout);
  return bad ? 1 : 0;
}
