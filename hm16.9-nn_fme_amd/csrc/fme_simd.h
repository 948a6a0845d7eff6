// fme_simd.h — per-lane integer helpers shared by the search kernels (fme_search.hip,
// fme_lane.hip): MV cost (TComRdCost), packed int16/int8 arithmetic, byte funnels and
// transposes, HEVC luma taps, and the packed SATD/SAD of 4x4 / 8x8 tiles.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fme {

typedef short v2s __attribute__((ext_vector_type(2)));
typedef unsigned short v2u __attribute__((ext_vector_type(2)));

namespace simd {

// ---- scalar helpers ------------------------------------------------------------------
__device__ __forceinline__ int clamp_i(int v, int lo, int hi) { return min(max(v, lo), hi); }

__device__ __forceinline__ uint32_t eg_bits(int v) {  // TComRdCost.cpp:172-185
  const uint32_t t = v <= 0 ? ((uint32_t)(-v) << 1) + 1u : ((uint32_t)v << 1);
  return 1u + 2u * (31u - (uint32_t)__clz((int)t));
}
__device__ __forceinline__ uint32_t mv_bits(int x, int y, int scale, int px, int py) {
  return eg_bits((x << scale) - px) + eg_bits((y << scale) - py);
}
__device__ __forceinline__ uint32_t mv_cost(double ml, uint32_t bits) {  // TComRdCost.h:165
  return (uint32_t)((ml * (double)bits) / 65536.0);
}

// Candidate tables of xPatternRefinement (TEncSearch.cpp:212-236), 2-bit codes.
__device__ __forceinline__ int dec(uint32_t c) { return c == 1 ? -1 : (c == 2 ? 1 : 0); }
__device__ __forceinline__ int cand_dx(int i) { return dec((0x666u >> (2 * (8 - i))) & 3u); }
__device__ __forceinline__ int half_dy(int i) { return dec((0x605au >> (2 * (8 - i))) & 3u); }
__device__ __forceinline__ int qtr_dy(int i) { return dec((0x650au >> (2 * (8 - i))) & 3u); }

// ---- packed arithmetic -----------------------------------------------------------------
__device__ __forceinline__ uint32_t pk(v2s v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ v2s up(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return pk(up(a) + up(b)); }
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) { return pk(up(a) - up(b)); }
__device__ __forceinline__ uint32_t pk_abs(uint32_t a) {
  const v2s x = up(a);
  return pk(__builtin_elementwise_max(x, -x));
}
__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int acc) {
  return __builtin_amdgcn_sdot2(up(a), up(b), acc, false);
}
__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(v2u, a), __builtin_bit_cast(v2u, b), acc, false);
}
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int acc) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, acc, false);
}
// bytes b0..b3 of `w` -> (b0, b1) and (b2, b3) as packed u16 pairs
__device__ __forceinline__ uint32_t lo_pair(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c010c00u); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c030c02u); }
// 4 bytes starting `sh` bytes into (lo, hi)
__device__ __forceinline__ uint32_t funnel8(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__device__ __forceinline__ uint32_t funnel16(uint32_t hi, uint32_t lo) {
  return __builtin_amdgcn_alignbit(hi, lo, 16u);
}
__device__ __forceinline__ uint32_t lds32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
// Global loads through pointers the compiler cannot classify (e.g. read from an LDS table):
// address space 1 makes them global_load (vmcnt only, in order) instead of flat_load, which
// forces s_waitcnt vmcnt(0) lgkmcnt(0) at every control-flow join.
typedef __attribute__((address_space(1))) const uint32_t gu32c;
typedef __attribute__((address_space(1))) const uint8_t gu8c;
__device__ __forceinline__ uint32_t gld32(const void* p) { return *(gu32c*)(p); }
__device__ __forceinline__ uint32_t gld8(const void* p) { return *(gu8c*)(p); }
__device__ __forceinline__ void sts32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }

// 4x4 byte transpose: r[i] holds row i (byte j = column j); c[j] = column j (byte i = row i).
__device__ __forceinline__ void transpose4x4(const uint32_t (&r)[4], uint32_t (&c)[4]) {
  const uint32_t a = __builtin_amdgcn_perm(r[1], r[0], 0x05010400u);
  const uint32_t b = __builtin_amdgcn_perm(r[1], r[0], 0x07030602u);
  const uint32_t d = __builtin_amdgcn_perm(r[3], r[2], 0x05010400u);
  const uint32_t e = __builtin_amdgcn_perm(r[3], r[2], 0x07030602u);
  c[0] = __builtin_amdgcn_perm(d, a, 0x05040100u);
  c[1] = __builtin_amdgcn_perm(d, a, 0x07060302u);
  c[2] = __builtin_amdgcn_perm(e, b, 0x05040100u);
  c[3] = __builtin_amdgcn_perm(e, b, 0x07060302u);
}

// Four picture bytes at (x, y) .. (x+3, y) with edge replication (TComPicYuv::extendPicBorder
// semantics), branch-free: the 4-byte run xa = clamp(x, 0, W-4) is read with at most two
// aligned dword loads, then v_perm picks byte clamp(x+i, 0, W-1) - xa for lane byte i.
// Needs width >= 4 (HEVC luma width is a multiple of 8).
__device__ __forceinline__ uint32_t pic4(const uint8_t* luma, int stride, int width, int height, int x, int y) {
  const int yc = clamp_i(y, 0, height - 1);
  const int xa = clamp_i(x, 0, width - 4);
  const uintptr_t addr = reinterpret_cast<uintptr_t>(luma + (size_t)yc * stride + xa);
  const uint32_t sh = (uint32_t)(addr & 3);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const uint32_t lo = gld32(q);
  const uint32_t hi = gld32(sh ? q + 1 : q);      // second dword only when the run straddles
  const uint32_t run = funnel8(hi, lo, sh);       // pixels xa .. xa+3
  uint32_t sel = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) sel |= (uint32_t)(clamp_i(x + i, 0, width - 1) - xa) << (8 * i);
  return __builtin_amdgcn_perm(0u, run, sel);
}

// Luma taps as packed int8 quads (t0..t3, t4..t7) and int16 pairs (TComInterpolationFilter.cpp:57-63).
__device__ __forceinline__ uint32_t q8(int a, int b, int c, int d) {
  return (uint32_t)(a & 255) | ((uint32_t)(b & 255) << 8) | ((uint32_t)(c & 255) << 16) | ((uint32_t)(d & 255) << 24);
}
__device__ __forceinline__ uint32_t p16(int a, int b) { return (uint32_t)(a & 0xffff) | ((uint32_t)(b & 0xffff) << 16); }
__device__ __forceinline__ void taps8(int f, uint32_t& lo, uint32_t& hi) {
  if (f == 1) { lo = q8(-1, 4, -10, 58); hi = q8(17, -5, 1, 0); }
  else if (f == 2) { lo = q8(-1, 4, -11, 40); hi = q8(40, -11, 4, -1); }
  else { lo = q8(0, 1, -5, 17); hi = q8(58, -10, 4, -1); }
}
__device__ __forceinline__ void taps16(int f, uint32_t (&c)[4]) {
  if (f == 1) { c[0] = p16(-1, 4); c[1] = p16(-10, 58); c[2] = p16(17, -5); c[3] = p16(1, 0); }
  else if (f == 2) { c[0] = p16(-1, 4); c[1] = p16(-11, 40); c[2] = p16(40, -11); c[3] = p16(4, -1); }
  else { c[0] = p16(0, 1); c[1] = p16(-5, 17); c[2] = p16(58, -10); c[3] = p16(4, -1); }
}

// Second-stage rounding of filter<8,true,false,true> (shift 12, offset 2048 + (8192 << 6)).
__device__ __forceinline__ int round2d(int s) { return clamp_i((s + 526336) >> 12, 0, 255); }
// 1-D from bytes: (sum(c*s) + 32) >> 6 with sum(c*s) = sum(c*s') + 8192.
__device__ __forceinline__ int round1d_s8(int s) { return clamp_i((s + 8224) >> 6, 0, 255); }

// ---- SATD on packed tiles ------------------------------------------------------------------
// X[c][j]: column c, rows (2j, 2j+1) packed.  Returns the xCalcHADs value of the tile.
template <int T>
__device__ __forceinline__ uint32_t satd_packed(uint32_t (&X)[T][T / 2]) {
  // horizontal (across columns) butterflies
#pragma unroll
  for (int d = T / 2; d >= 1; d >>= 1)
#pragma unroll
    for (int c = 0; c < T; c++)
      if ((c & d) == 0)
#pragma unroll
        for (int j = 0; j < T / 2; j++) {
          const uint32_t a = X[c][j], b = X[c + d][j];
          X[c][j] = pk_add(a, b);
          X[c + d][j] = pk_sub(a, b);
        }
  // vertical butterflies between row pairs (distances 4 and 2 rows)
#pragma unroll
  for (int d = T / 4; d >= 1; d >>= 1)
#pragma unroll
    for (int c = 0; c < T; c++)
#pragma unroll
      for (int j = 0; j < T / 2; j++)
        if ((j & d) == 0) {
          const uint32_t a = X[c][j], b = X[c][j + d];
          X[c][j] = pk_add(a, b);
          X[c][j + d] = pk_sub(a, b);
        }
  // last butterfly (rows 2j, 2j+1 in one register): |a+b| + |a-b| = 2 max(|a|, |b|)
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < T; c += 2)
#pragma unroll
    for (int j = 0; j < T / 2; j++) {
      const uint32_t a = pk_abs(X[c][j]), b = pk_abs(X[c + 1][j]);
      const uint32_t los = __builtin_amdgcn_perm(b, a, 0x05040100u);   // (a.lo, b.lo)
      const uint32_t his = __builtin_amdgcn_perm(b, a, 0x07060302u);   // (a.hi, b.hi)
      const v2s m = __builtin_elementwise_max(up(los), up(his));
      s = udot2(pk(m), 0x00010001u, s);
    }
  // 8x8: (2s + 2) >> 2 ; 4x4: (2s + 1) >> 1
  return T == 8 ? (s + 1) >> 1 : s;
}

template <int T>
__device__ __forceinline__ uint32_t sad_packed(const uint32_t (&X)[T][T / 2]) {
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < T; c++)
#pragma unroll
    for (int j = 0; j < T / 2; j++) s = udot2(pk_abs(X[c][j]), 0x00010001u, s);
  return s;
}

}  // namespace simd
}  // namespace fme
