// fme_xlane.h — cross-lane helpers of the pixel-per-lane kernels (fme_server.hip, fme_px.hip):
// values of lane ^ m without the LDS pipe, Walsh-Hadamard butterflies and sums across a wave.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fme {
namespace xlane {

// The value of lane ^ m (m a power of two below 64): DPP within a row of 16 lanes,
// v_permlane16/32_swap across rows.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int M>
__device__ __forceinline__ int xor_lane(int v, int lane) {
  if constexpr (M == 1) return dpp_i<0xB1>(v);          // quad_perm [1, 0, 3, 2]
  else if constexpr (M == 2) return dpp_i<0x4E>(v);     // quad_perm [2, 3, 0, 1]
  else if constexpr (M == 4) {                          // row_shl:4 / row_shr:4
    const int up = dpp_i<0x104>(v), dn = dpp_i<0x114>(v);
    return (lane & 4) ? dn : up;
  } else if constexpr (M == 8) return dpp_i<0x128>(v);  // row_ror:8
  else if constexpr (M == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? (int)p[0] : (int)p[1];
  } else {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? (int)p[0] : (int)p[1];
  }
}
// Butterfly stage over lane bit M: (a + b, a - b) with a the lower lane's value.
template <int M>
__device__ __forceinline__ int bfly(int d, int lane) {
  const int p = xor_lane<M>(d, lane);
  return (lane & M) ? p - d : d + p;
}
template <int M>
__device__ __forceinline__ uint32_t xsum(uint32_t a, int lane) { return a + (uint32_t)xor_lane<M>((int)a, lane); }
// sum over all 64 lanes (every lane ends with the total)
__device__ __forceinline__ uint32_t wave_sum(uint32_t a, int lane) {
  return xsum<32>(xsum<16>(xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane), lane), lane);
}

}  // namespace xlane
}  // namespace fme
