// Probe: what rocprofv3's FETCH_SIZE reports for the search kernel's access pattern, against a
// known byte count (validate the x2 gfx950 correction for per-lane row loads).
//   k_stream: coalesced 16 B/lane streaming read of B bytes (the guide's calibration case);
//   k_rows:   the lane kernel's pattern - lane i reads 16 rows of 16 unaligned bytes of an 8x8
//             unit's window at its own (x, y) in a 1920x1080 plane, neighbouring lanes' windows
//             adjacent (units of one PU row) so lines are shared; every byte of the plane is read
//             by some lane: distinct bytes = the plane (2.07 MB), requested bytes = 64 x 4 per unit.
// Run under rocprofv3 --pmc FETCH_SIZE; each kernel is launched once on a cold 256 MB eviction
// pass first so the measured launch reads from HBM.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_stream(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
// Lane i reads the 16 rows of 16 bytes of its own 16x16 tile (disjoint tiles covering the plane)
// starting `off` bytes into the tile, as the lane kernel reads a window row (one 16-byte load per
// row, unaligned when off % 16 != 0).  Distinct bytes = the plane.
__global__ void k_rows(const uint8_t* __restrict__ pic, int W, int H, int off, uint32_t* out) {
  const int tiles_x = W / 16, tiles = tiles_x * (H / 16);
  uint32_t acc = 0;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < tiles; t += gridDim.x * blockDim.x) {
    const int x = min((t % tiles_x) * 16 + off, W - 16), y = (t / tiles_x) * 16;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const u32x4u v = *(const u32x4u*)(pic + (size_t)(y + r) * W + x);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int W = 1920, H = 1088;
  const size_t big = 256u << 20, stream_bytes = 64u << 20;
  uint8_t *evict, *pic, *buf;
  uint32_t* out;
  hipMalloc(&evict, big);
  hipMalloc(&pic, (size_t)W * H);
  hipMalloc(&buf, stream_bytes);
  hipMalloc(&out, 4);
  hipMemset(evict, 1, big);
  hipMemset(pic, 2, (size_t)W * H);
  hipMemset(buf, 3, stream_bytes);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const uint4*)evict, big / 16, out);   // evict
    hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const uint4*)buf, stream_bytes / 16, out);
    hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const uint4*)evict, big / 16, out);   // evict
    hipLaunchKernelGGL(k_rows, dim3(32), dim3(256), 0, 0, pic, W, H, 0, out);
    hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0, (const uint4*)evict, big / 16, out);   // evict
    hipLaunchKernelGGL(k_rows, dim3(32), dim3(256), 0, 0, pic, W, H, 3, out);
  }
  hipDeviceSynchronize();
  printf("{\"stream_bytes\": %zu, \"rows_plane_bytes\": %d}\n", stream_bytes, W * H);
  return 0;
}
