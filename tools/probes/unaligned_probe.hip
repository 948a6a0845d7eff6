// Probe: do global_load_dword{,x2,x3,x4} at byte-unaligned addresses return the right bytes on
// gfx950 (unaligned access mode)?  Prints mismatches per width and offset.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u3 __attribute__((ext_vector_type(3), aligned(4)));
typedef __attribute__((address_space(1))) const u4 g4;
typedef __attribute__((address_space(1))) const u3 g3;
__global__ void k(const uint8_t* src, uint32_t* out) {
  const int t = threadIdx.x;               // byte offset t (0..63)
  const u4 a = *(g4*)(src + t);
  const u3 b = *(g3*)(src + 100 + t);
  out[8 * t + 0] = a.x; out[8 * t + 1] = a.y; out[8 * t + 2] = a.z; out[8 * t + 3] = a.w;
  out[8 * t + 4] = b.x; out[8 * t + 5] = b.y; out[8 * t + 6] = b.z; out[8 * t + 7] = 0;
}
int main() {
  uint8_t h[256]; for (int i = 0; i < 256; i++) h[i] = (uint8_t)(i * 7 + 3);
  uint8_t* d; uint32_t* o; uint32_t ho[512];
  hipMalloc(&d, 256); hipMalloc(&o, 2048);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(ho, o, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 64; t++) {
    for (int q = 0; q < 4; q++) { uint32_t e = 0; for (int b = 0; b < 4; b++) e |= (uint32_t)h[t + 4 * q + b] << (8 * b); if (ho[8 * t + q] != e) bad++; }
    for (int q = 0; q < 3; q++) { uint32_t e = 0; for (int b = 0; b < 4; b++) e |= (uint32_t)h[100 + t + 4 * q + b] << (8 * b); if (ho[8 * t + 4 + q] != e) bad++; }
  }
  printf("unaligned probe: %d mismatching dwords of %d\n", bad, 64 * 7);
  return bad != 0;
}
