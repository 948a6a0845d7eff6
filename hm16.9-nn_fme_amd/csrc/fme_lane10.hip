// fme_lane10.hip — lane-per-unit EMI + FracDIF search at bit depth 10 (the main10
// configurations, cfg/encoder_lowdelay_P_main10.cfg:58 InternalBitDepth 10), gfx950.
//
// The 8-bit lane kernel's layout (fme_lane.hip): a lane owns one 4x8 or 4x4 unit of a PU, the
// PU's units sit in consecutive lanes of one wave, partial distortions are summed across them with
// DPP / swizzle steps, and every lane of a PU takes the same decisions; the reference window stays
// in VGPRs.  Here a sample is an int16 s' = s - 512 (two per dword) instead of a byte, so:
//   * the 8-tap filters are v_dot2_i32_i16 over sample pairs (five pairs per output, the taps
//     shifted by the per-lane integer offset instead of re-aligning the data);
//   * the first 2-D stage is xExtDIFUpSamplingH/Q's filter<8, isFirst, !isLast> at headRoom 4:
//     h = (sum c s') >> 2 (the -8192 << 2 offset cancels 512 * 64); the second is
//     filter<8, !isFirst, isLast>: s' = clip((sum c h + 512) >> 10, -512, 511), computed with taps
//     x 64 so a pair of outputs is the high halves of two sums; a fraction-0 phase uses the taps
//     {0,0,0,64,0,0,0,0}, which equals HM's copy / 1-D paths after both roundings
//     ((64 (16 s') + 512) >> 10 == s', (64 h + 512) >> 10 == (h + 8) >> 4 == (sum c s' + 32) >> 6);
//   * distortions follow TComRdCost at bitDepth 10 (TypeDef.h:140-143 DISTORTION_PRECISION_ADJUSTMENT):
//     the integer SSE sums (d * d) >> 4 per sample (TComRdCost.cpp:875-1130), SAD and SATD sums are
//     >> 2 over the block (:324, 419-854), the 8x8 / 4x4 tile roundings as at 8 bits;
//   * the packed-int16 Hadamard holds |d| <= 1023 (uni-pred) to its last butterfly (32 * 1023 <
//     32768); bi-pred keys (2 org - pred, unclipped: |d| <= 2046) finish an 8x8 tile's row stages
//     in 32 bits.
// Records are those of the lane kernel: the NN tail (k_nn_tail) completes them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <utility>

#include "fme_device.h"
#include "fme_simd.h"

namespace fme {
namespace {
using namespace simd;

#define FME_AI __attribute__((always_inline))

#ifndef FME_L10_WAVES   // occupancy target (waves per SIMD) that bounds the register allocation
#define FME_L10_WAVES 2
#endif

constexpr int kL10NT = 256;
constexpr int kDsh = 2;      // DISTORTION_PRECISION_ADJUSTMENT(bitDepth - 8)

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// Sum over the L lanes of a PU's group (every lane of the group ends with the total).
template <int L>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
  if (L >= 2) v += dpp<0xB1>(v);
  if (L >= 4) v += dpp<0x4E>(v);
  if (L >= 8) v += dpp<0x141>(v);
  if (L >= 16) v += dpp<0x140>(v);
  if (L >= 32) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
  if (L >= 64) v += (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}
__host__ __device__ __forceinline__ constexpr int pow2_at_least(int v) { return v <= 1 ? 1 : 2 * pow2_at_least((v + 1) / 2); }

template <int R, int N>
__device__ __forceinline__ void launder(uint32_t (&v)[R][N]) {
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int k = 0; k < N; k++) asm volatile("" : "+v"(v[r][k]));
}

__device__ __forceinline__ uint32_t pack2(int a, int b) { return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u); }
__device__ __forceinline__ int sx16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ int hx16(uint32_t v) { return (int)v >> 16; }

// Samples (s, s+1) of a row held as int16 pairs v[0..N) (pair k = samples 2k, 2k+1); s is a
// compile-time constant after unrolling.  Past the row's last sample the high half is 0.
template <int N>
__device__ __forceinline__ uint32_t rpair(const uint32_t (&v)[N], int s) {
  const int q = s >> 1;
  if (!(s & 1)) return v[q];
  if (q + 1 < N) return __builtin_amdgcn_alignbyte(v[q + 1], v[q], 2u);
  return v[q] >> 16;
}

// tap k of fraction f (k outside 0..7 -> 0; TComInterpolationFilter.cpp:57-63)
__host__ __device__ __forceinline__ constexpr int tap(int f, int k) {
  return (k < 0 || k > 7) ? 0
         : f == 0        ? (k == 3 ? 64 : 0)
         : f == 1 ? (k == 0 ? -1 : k == 1 ? 4 : k == 2 ? -10 : k == 3 ? 58 : k == 4 ? 17 : k == 5 ? -5 : k == 6 ? 1 : 0)
         : f == 2 ? (k == 0 ? -1 : k == 1 ? 4 : k == 2 ? -11 : k == 3 ? 40 : k == 4 ? 40 : k == 5 ? -11 : k == 6 ? 4 : -1)
                  : (k == 0 ? 0 : k == 1 ? 1 : k == 2 ? -5 : k == 3 ? 17 : k == 4 ? 58 : k == 5 ? -10 : k == 6 ? 4 : -1);
}
// Five coefficient pairs over ten consecutive samples / rows whose 8-tap window starts `o` (0 or 1)
// into them: pair t = (tap(2t - o), tap(2t + 1 - o)) * scale.
__device__ __forceinline__ void cpairs(int f, int o, int scale, uint32_t (&c)[5]) {
#pragma unroll
  for (int t = 0; t < 5; t++) c[t] = p16(scale * tap(f, 2 * t - o), scale * tap(f, 2 * t + 1 - o));
}

// (s0 >> 16, s1 >> 16) clipped to [-512, 511], packed: second-stage sums with taps x 64 and the
// 512 * 64 offset, i.e. (sum c h + 512) >> 10 of filter<8, !isFirst, isLast> in the s' domain.
__device__ __forceinline__ uint32_t pk_round2(int s0, int s1) {
  const v2s m = up(__builtin_amdgcn_perm((uint32_t)s1, (uint32_t)s0, 0x07060302u));
  return pk(__builtin_elementwise_min(__builtin_elementwise_max(m, v2s{-512, -512}), v2s{511, 511}));
}
// ((h0 + 8) >> 4, (h1 + 8) >> 4) clipped, from the packed first-stage pair (h0, h1): the vertical
// fraction-0 pass of filter<8, !isFirst, isLast> (filterCopy: (h + 8192 + 8) >> 4 in the s domain)
__device__ __forceinline__ uint32_t pk_round1(uint32_t hp) {
  const v2s m = (up(hp) + v2s{8, 8}) >> v2s{4, 4};
  return pk(__builtin_elementwise_min(__builtin_elementwise_max(m, v2s{-512, -512}), v2s{511, 511}));
}

// ---- key: K(x, j) = key' rows (2j, 2j+1) of column x, int16 (key - 512) ----------------------
template <int UW, int UJ>
struct KeySrc {
  uint32_t k[UW][UJ];
  __device__ __forceinline__ uint32_t at(int x, int j) const { return k[x][j]; }
};

// ---- distortion of one unit ------------------------------------------------------------------
struct Metric {
  bool had, wide;   // wide: a bi-pred key (|key - pred| up to 2046): 8x8 row stages in 32 bits
  uint32_t sgn, emask;
};

// One 8x8 SATD tile over a lane pair (the even lane columns 0..3, the odd lane 4..7), as the 8-bit
// kernel's satd8_pair (TComRdCost.cpp:1330-1425, the odd lane forms b - a); returns this lane's sum
// of the last stage's max terms (narrow) or of its absolute outputs (wide, already doubled).
__device__ __forceinline__ uint32_t satd8_pair(uint32_t (&X)[4][4], uint32_t sgn, bool wide) {
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int j = 0; j < 4; j++) X[c][j] = pk(up(dpp<0xB1>(X[c][j])) * up(sgn) + up(X[c][j]));
#pragma unroll
  for (int d = 2; d >= 1; d >>= 1)
#pragma unroll
    for (int c = 0; c < 4; c++)
      if ((c & d) == 0)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t a = X[c][j], b = X[c + d][j];
          X[c][j] = pk_add(a, b);
          X[c + d][j] = pk_sub(a, b);
        }
  if (wide) {   // |values| <= 8 * 2046 here: the three row stages in 32 bits
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      int r[8];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        r[2 * j] = sx16(X[c][j]);
        r[2 * j + 1] = hx16(X[c][j]);
      }
#pragma unroll
      for (int d = 4; d >= 1; d >>= 1)
#pragma unroll
        for (int k = 0; k < 8; k++)
          if ((k & d) == 0) {
            const int a = r[k], b = r[k + d];
            r[k] = a + b;
            r[k + d] = a - b;
          }
#pragma unroll
      for (int k = 0; k < 8; k++) s += (uint32_t)abs(r[k]);
    }
    return s;
  }
#pragma unroll
  for (int d = 2; d >= 1; d >>= 1)
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        if ((j & d) == 0) {
          const uint32_t a = X[c][j], b = X[c][j + d];
          X[c][j] = pk_add(a, b);
          X[c][j + d] = pk_sub(a, b);
        }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < 4; c += 2)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t a = pk_abs(X[c][j]), b = pk_abs(X[c + 1][j]);
      const uint32_t los = __builtin_amdgcn_perm(b, a, 0x05040100u);
      const uint32_t his = __builtin_amdgcn_perm(b, a, 0x07060302u);
      const v2s m = __builtin_elementwise_max(up(los), up(his));
      s = udot2(pk(m), 0x00010001u, s);
    }
  return 2 * s;
}

// X[c][j]: key' - pred', column c, rows (2j, 2j+1).  Sum over the unit's tiles of the rounded
// xCalcHADs (had) or of |d| (SAD), before the block's >> 2; a 4x8 half of an 8x8 tile: the even
// lane returns the tile, the odd lane 0.
template <int UW, int UH, int T>
__device__ __forceinline__ uint32_t unit_dist(uint32_t (&X)[UW][UH / 2], const Metric& m) {
  if constexpr (T == 8 && UW == 4) {
    static_assert(UH == 8, "4x8 half tiles");
    if (m.had) {
      uint32_t s = satd8_pair(X, m.sgn, m.wide);
      s += dpp<0xB1>(s);                 // the tile's total in both lanes
      return ((s + 2) >> 2) & m.emask;
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < UW; c++)
#pragma unroll
      for (int j = 0; j < UH / 2; j++) s = udot2(pk_abs(X[c][j]), 0x00010001u, s);
    return s;
  } else {
    uint32_t s = 0;
#pragma unroll
    for (int ty = 0; ty < UH / T; ty++)
#pragma unroll
      for (int tx = 0; tx < UW / T; tx++) {
        uint32_t Y[T][T / 2];
#pragma unroll
        for (int c = 0; c < T; c++)
#pragma unroll
          for (int j = 0; j < T / 2; j++) Y[c][j] = X[tx * T + c][ty * (T / 2) + j];
        s += m.had ? satd_packed<T>(Y) : sad_packed<T>(Y);
      }
    return s;
  }
}

// Candidate tables (xPatternRefinement, TEncSearch.cpp:212-236)
__host__ __device__ __forceinline__ constexpr int h9_dx(int i) { return (i == 3 || i == 5 || i == 7) ? -1 : ((i == 4 || i == 6 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int h9_dy(int i) { return (i == 1 || i == 5 || i == 6) ? -1 : ((i == 2 || i == 7 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int q9_dx(int i) { return (i == 3 || i == 5 || i == 7) ? -1 : ((i == 4 || i == 6 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int q9_dy(int i) { return (i == 1 || i == 3 || i == 4) ? -1 : ((i == 2 || i == 7 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int q9_index(int dx, int dy) {
  return dy == 0 ? (dx == 0 ? 0 : (dx < 0 ? 5 : 6)) : dy < 0 ? (dx == 0 ? 1 : (dx < 0 ? 3 : 4)) : (dx == 0 ? 2 : (dx < 0 ? 7 : 8));
}
__host__ __device__ __forceinline__ constexpr int emi_dx(int p) { return (p == 1 || p == 4 || p == 6) ? -1 : ((p == 3 || p == 5 || p == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int emi_dy(int p) { return p >= 1 && p <= 3 ? -1 : (p >= 6 ? 1 : 0); }

__shared__ PicDesc g10_pics[FME_MAX_PICTURES];
constexpr int kCostBits = 80;
__shared__ uint32_t g10_cost[FME_MAX_LAMBDAS][kCostBits];
__shared__ uint4 g10_rec[kL10NT / 64][64][4];
__shared__ int32_t g10_rec_jid[kL10NT / 64][64];

__device__ __forceinline__ uint32_t mvc(const uint32_t* ml, uint32_t bits) { return ml[bits]; }
template <int L>
__device__ __forceinline__ void take_half(int i, uint32_t part, uint32_t live, const uint32_t* ml, int mvx, int mvy, int px,
                                          int py, uint32_t& best, int& bi) {
  const uint32_t d = (group_sum<L>(part & live) >> kDsh) + mvc(ml, mv_bits(2 * mvx + h9_dx(i), 2 * mvy + h9_dy(i), 1, px, py));
  if (d < best || (d == best && i < bi)) {
    best = d;
    bi = i;
  }
}
template <int L>
__device__ __forceinline__ void take_qtr(int i, uint32_t part, uint32_t live, const uint32_t* ml, int mvx, int mvy, int hx,
                                         int hy, int px, int py, uint32_t& best, int& bi) {
  const int qx = 2 * hx + q9_dx(i), qy = 2 * hy + q9_dy(i);
  const uint32_t d = (group_sum<L>(part & live) >> kDsh) + mvc(ml, mv_bits(4 * mvx + qx, 4 * mvy + qy, 0, px, py));
  if (d < best || (d == best && i < bi)) {
    best = d;
    bi = i;
  }
}

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4a gu4;
typedef __attribute__((address_space(1))) const u32x3a gu3;
typedef __attribute__((address_space(1))) const u32x2a gu2;
typedef __attribute__((address_space(1))) const uint16_t g_u16;

// N dwords from byte address p, any alignment (gfx950 global memory runs unaligned).
template <int N>
__device__ __forceinline__ void ld_dw(const void* p, uint32_t (&o)[N]) {
  const uint8_t* q = (const uint8_t*)p;
  constexpr int K4 = N / 4 * 4;
#pragma unroll
  for (int k = 0; k < K4; k += 4) {
    const u32x4a v = *(gu4*)(q + 4 * k);
    o[k] = v.x; o[k + 1] = v.y; o[k + 2] = v.z; o[k + 3] = v.w;
  }
  if constexpr (N - K4 == 3) {
    const u32x3a v = *(gu3*)(q + 4 * K4);
    o[K4] = v.x; o[K4 + 1] = v.y; o[K4 + 2] = v.z;
  } else if constexpr (N - K4 == 2) {
    const u32x2a v = *(gu2*)(q + 4 * K4);
    o[K4] = v.x; o[K4 + 1] = v.y;
  } else if constexpr (N - K4 == 1) {
    o[K4] = gld32(q + 4 * K4);
  }
}

// Rows y0 .. y0+R-1, samples x0 .. x0 + 2N - 1 of a 10-bit picture as s' pairs, with the padded
// picture's edge replication (TComPicYuv::extendPicBorder: coordinates clamped).
template <int R, int N>
__device__ __forceinline__ void load_window(const PicDesc& pic, int x0, int y0, uint32_t (&v)[R][N]) {
  asm volatile("" : "+v"(x0), "+v"(y0));
  const uint16_t* luma = reinterpret_cast<const uint16_t*>(pic.luma);
  const bool inside = x0 >= 0 && x0 + 2 * N <= pic.width;
  if (inside) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int yy = clamp_i(y0 + r, 0, pic.height - 1);
      ld_dw<N>(luma + (size_t)yy * pic.stride + x0, v[r]);
      if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const g_u16* row = (g_u16*)(luma + (size_t)clamp_i(y0 + r, 0, pic.height - 1) * pic.stride);
#pragma unroll
      for (int k = 0; k < N; k++) {
        const uint32_t a = row[clamp_i(x0 + 2 * k, 0, pic.width - 1)];
        const uint32_t b = row[clamp_i(x0 + 2 * k + 1, 0, pic.width - 1)];
        v[r][k] = a | (b << 16);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int k = 0; k < N; k++) v[r][k] = pk_sub(v[r][k], 0x02000200u);
}

// ---- one candidate pass: a horizontal quarter offset qx (the first stage of every column, once)
// and NQ vertical offsets qy[m] (a second stage and a distortion each); v = window rows -4..UH+3,
// cols -4..UW+3 as pairs.  QX constant (half stage) or kRuntime (qx per lane: the quarter stage).
constexpr int kRuntime = 99;
template <int UW, int UH, int T, int NC, int C0, int NQ>
__device__ __forceinline__ void second_stages(uint32_t (&HQ)[NC][(UH + 8) / 2], const KeySrc<UW, UH / 2>& K,
                                              const Metric& met, const int (&qy)[NQ], uint32_t (&d)[NQ]);
template <int UW, int UH, int T, int QX, int NQ>
__device__ __forceinline__ void qpass(uint32_t (&v)[UH + 8][(UW + 8) / 2], const KeySrc<UW, UH / 2>& K, const Metric& met,
                                      int qx_rt, const int (&qy)[NQ], uint32_t (&d)[NQ]) {
  constexpr int RV = UH + 8;
  uint32_t HQ[UW][RV / 2];   // first-stage rows (2k, 2k+1) of each column
  if constexpr (QX != kRuntime && (QX & 3) == 0) {   // integer columns: h = 16 s' (filterCopy, isFirst)
    launder(v);
#pragma unroll
    for (int x = 0; x < UW; x++)
#pragma unroll
      for (int r = 0; r < RV; r += 2) {
        const uint32_t a = rpair(v[r], x + 4 + (QX >> 2)), b = rpair(v[r + 1], x + 4 + (QX >> 2));
        HQ[x][r / 2] = pk(up(__builtin_amdgcn_perm(b, a, 0x05040100u)) << v2s{4, 4});
      }
  } else {
    const int qx = QX == kRuntime ? qx_rt : QX;
    const int ix = qx >> 2, fx = qx & 3;
    uint32_t ch[5];
    cpairs(fx, 1 + ix, 1, ch);   // samples x .. x+9 of the window, the 8 taps start 1 + ix into them
#pragma unroll
    for (int x = 0; x < UW; x++) {
      launder(v);
#pragma unroll
      for (int r = 0; r < RV; r += 2) {
        int h0 = 0, h1 = 0;
#pragma unroll
        for (int t = 0; t < 5; t++) {
          h0 = dot2(rpair(v[r], x + 2 * t), ch[t], h0);
          h1 = dot2(rpair(v[r + 1], x + 2 * t), ch[t], h1);
        }
        HQ[x][r / 2] = pack2(h0 >> 2, h1 >> 2);
      }
      __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure)
    }
  }
  second_stages<UW, UH, T, UW, 0, NQ>(HQ, K, met, qy, d);
}

// The NQ vertical offsets qy[m] over first-stage columns C0 .. C0 + UW - 1 of HQ: a second stage
// (filter<8, !isFirst, isLast>), key' - pred' and the unit's distortion each, one at a time.
template <int UW, int UH, int T, int NC, int C0, int NQ>
__device__ __forceinline__ void second_stages(uint32_t (&HQ)[NC][(UH + 8) / 2], const KeySrc<UW, UH / 2>& K,
                                              const Metric& met, const int (&qy)[NQ], uint32_t (&d)[NQ]) {
  constexpr int UJ = UH / 2;
#pragma unroll
  for (int m = 0; m < NQ; m++) {
    launder(HQ);   // no candidate's values shared with (and kept live for) another
    const int iy = qy[m] >> 2, fy = qy[m] & 3;
    uint32_t X[UW][UJ];
    if (fy == 0) {   // (then iy == 0) first-stage rows 4.., (h + 8) >> 4
#pragma unroll
      for (int x = 0; x < UW; x++)
#pragma unroll
        for (int jj = 0; jj < UJ; jj++) X[x][jj] = pk_sub(K.at(x, jj), pk_round1(HQ[C0 + x][jj + 2]));
    } else {
      uint32_t ce[5], co[5];
      cpairs(fy, 1 + iy, 64, ce);
      cpairs(fy, 2 + iy, 64, co);
#pragma unroll
      for (int x = 0; x < UW; x++) {
        int vq[UH];
#pragma unroll
        for (int y = 0; y < UH; y++) {
          const int m0 = (y & 1) ? (y - 1) / 2 : y / 2;
          int acc = 512 * 64;
#pragma unroll
          for (int t = 0; t < 5; t++) acc = dot2(HQ[C0 + x][m0 + t], (y & 1) ? co[t] : ce[t], acc);
          vq[y] = acc;
        }
#pragma unroll
        for (int jj = 0; jj < UJ; jj++) X[x][jj] = pk_sub(K.at(x, jj), pk_round2(vq[2 * jj], vq[2 * jj + 1]));
      }
    }
    d[m] = unit_dist<UW, UH, T>(X, met);
    __builtin_amdgcn_sched_barrier(0);   // one candidate at a time
  }
}

// The six half-pel side candidates (-1, 0/-1/+1) and (+1, 0/-1/+1) from the UW + 1 half columns
// x - 1/2, x = 0 .. UW, that both sides share (xExtDIFUpSamplingH's filteredBlock[*][2] columns):
// side -1 reads columns 0 .. UW-1, side +1 columns 1 .. UW.  d = H9 candidates 3, 5, 7, 4, 6, 8.
template <int UW, int UH, int T>
__device__ __forceinline__ void half_sides(uint32_t (&v)[UH + 8][(UW + 8) / 2], const KeySrc<UW, UH / 2>& K,
                                           const Metric& met, uint32_t (&d)[6]) {
  constexpr int RV = UH + 8;
  uint32_t HQ[UW + 1][RV / 2];
  const uint32_t c0 = p16(-1, 4), c1 = p16(-11, 40), c2 = p16(40, -11), c3 = p16(4, -1);
#pragma unroll
  for (int k = 0; k <= UW; k++) {   // window samples k .. k+7: the half column between cols k-1, k
    launder(v);
#pragma unroll
    for (int r = 0; r < RV; r += 2) {
      int h0 = dot2(rpair(v[r], k), c0, 0), h1 = dot2(rpair(v[r + 1], k), c0, 0);
      h0 = dot2(rpair(v[r], k + 2), c1, h0);
      h1 = dot2(rpair(v[r + 1], k + 2), c1, h1);
      h0 = dot2(rpair(v[r], k + 4), c2, h0);
      h1 = dot2(rpair(v[r + 1], k + 4), c2, h1);
      h0 = dot2(rpair(v[r], k + 6), c3, h0);
      h1 = dot2(rpair(v[r + 1], k + 6), c3, h1);
      HQ[k][r / 2] = pack2(h0 >> 2, h1 >> 2);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const int qy[3] = {0, -2, 2};
  uint32_t dl[3], dr[3];
  second_stages<UW, UH, T, UW + 1, 0, 3>(HQ, K, met, qy, dl);
  second_stages<UW, UH, T, UW + 1, 1, 3>(HQ, K, met, qy, dr);
#pragma unroll
  for (int m = 0; m < 3; m++) {
    d[m] = dl[m];
    d[3 + m] = dr[m];
  }
}

typedef __attribute__((address_space(1))) const fme_job g_job;
typedef __attribute__((address_space(1))) const int32_t g_i32;
typedef __attribute__((address_space(1))) fme_result g_res;
typedef __attribute__((address_space(1))) const int16_t g_i16;
typedef __attribute__((address_space(1))) const uint32_t g_u32;

// One lane: unit (ux, uy) of PU p of class (PW x PH), unit UW x UH; PUs of more than 64 units give a
// lane two (top and bottom half), each candidate pass running once per half.
template <int PW, int PH, int UW, int UH>
__device__ __attribute__((noinline)) void lane_unit10(const BatchArgs& a, const int32_t* __restrict__ perm_, int cls_off,
                                                      int cls_cnt, int wt, int wid) {
  g_i32* const perm = (g_i32*)perm_;
  g_res* const outp = (g_res*)a.res;
  g_i16* const keys = (g_i16*)a.keys;
  const int use_hadamard = a.use_hadamard, fen = a.fen;
  constexpr int T = ((PW % 8) == 0 && (PH % 8) == 0) ? 8 : 4;
  static_assert((T == 8 && UW == 4 && UH == 8) || (T == 4 && UW == 4 && (UH == 4 || UH == 8)), "unit shapes");
  constexpr int UX = PW / UW, UY = PH / UH, NU = UX * UY;
  constexpr int UPL = NU > 64 ? 2 : 1;
  constexpr int UYH = UY / UPL, NUH = UX * UYH;
  constexpr int L = pow2_at_least(NUH);
  static_assert(L <= 64, "a PU's group fits one wave");
  constexpr bool kSadEmi = PW == 12 || PW == 24 || PW == 48;
  constexpr int RV = UH + 8;                   // sub-pel window rows -4 .. UH+3
  constexpr int NV = (UW + 8) / 2;             // cols -4 .. UW+3
  constexpr int UJ = UH / 2;
  constexpr int EW = (UW + 2 + 1) / 2;         // EMI window pairs per row (cols -1 .. UW)
  constexpr int KW = UW / 2;                   // key pairs per row

  const int lane = (int)__lane_id();
  const int gl = wt * 64 + lane;
  int p = gl / L;
  const int u = gl - p * L;
  const bool active = p < cls_cnt;
  if (!active) p = cls_cnt - 1;
  const uint32_t live = u < NUH ? ~0u : 0u;
  const int uu = u < NUH ? u : NUH - 1;
  const int ux = uu % UX, uy = uu / UX;

  const int jid = perm[cls_off + p];
  fme_job j;
  {
    g_job* const src = (g_job*)a.jobs + jid;
    const u32x4a q0 = *(gu4*)src, q1 = *(gu4*)((const __attribute__((address_space(1))) uint8_t*)src + 16);
    uint32_t tmp[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    __builtin_memcpy(&j, tmp, sizeof(j));
  }
  auto ref_pic = [&]() FME_AI -> PicDesc {
    int rid = j.ref_id;
    asm volatile("" : "+v"(rid));
    return g10_pics[rid];
  };
  const uint32_t* const ml = g10_cost[j.lambda_id];
  const bool kbuf = j.key_offset >= 0;
  const Metric met = {use_hadamard && !(j.flags & FME_JOB_LOSSLESS), kbuf, (lane & 1) ? 0xFFFFFFFFu : 0x00010001u,
                      (lane & 1) ? 0u : ~0u};
  const int ox = (int)j.x + ux * UW, oy = (int)j.y + uy * UH;
  constexpr int kHalfRows = UYH * UH;
  const int mvp_x = j.mvp_x, mvp_y = j.mvp_y;

  // key rows of half h as s' pairs: kraw[r][k] = (col 2k, col 2k+1)
  auto load_kraw = [&](int h, uint32_t (&kraw)[UH][KW]) FME_AI {
    int ky = oy + h * kHalfRows;
    asm volatile("" : "+v"(ky));
    if (!kbuf) {
      const PicDesc org = g10_pics[j.org_id];
      const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
#pragma unroll
      for (int r = 0; r < UH; r++) ld_dw<KW>(ol + (size_t)(ky + r) * org.stride + ox, kraw[r]);
    } else {
      g_i16* kb = keys + (size_t)j.key_offset + (size_t)(ky - (int)j.y) * PW + ux * UW;
#pragma unroll
      for (int r = 0; r < UH; r++) ld_dw<KW>((const void*)(kb + r * PW), kraw[r]);
    }
#pragma unroll
    for (int r = 0; r < UH; r++)
#pragma unroll
      for (int k = 0; k < KW; k++) kraw[r][k] = pk_sub(kraw[r][k], 0x02000200u);
  };
  uint32_t kraw0[UH][KW];
  if constexpr (UPL == 1) load_kraw(0, kraw0);

  // ---- 1. EMI square step (TEncSearch.cpp:1324-1377, 1155-1188, 5043-5050) ---------------------
  int mvx = j.mv_x, mvy = j.mv_y;
  int n_emi = 0;
  uint32_t cval = 0, emi[8];
#pragma unroll
  for (int k = 0; k < 8; k++) emi[k] = 0;
  if (j.flags & FME_JOB_NN_IN) {
    g_u32* const row = (g_u32*)(a.nn_in + (size_t)9 * jid);
#pragma unroll
    for (int k = 0; k < 8; k++) emi[k] = row[k];
    cval = row[8];
    n_emi = 8;
  } else if (j.flags & FME_JOB_EMI) {
    uint32_t e9[9];
#pragma unroll
    for (int q = 0; q < 9; q++) e9[q] = 0;
#pragma unroll
    for (int h = 0; h < UPL; h++) {
      uint32_t kraw[UH][KW];
      if constexpr (UPL == 1) {
#pragma unroll
        for (int r = 0; r < UH; r++)
#pragma unroll
          for (int k = 0; k < KW; k++) kraw[r][k] = kraw0[r][k];
      } else {
        load_kraw(h, kraw);
      }
      uint32_t w[UH + 2][EW];   // rows -1 .. UH, cols -1 .. UW
      load_window(ref_pic(), ox + mvx - 1, oy + h * kHalfRows + mvy - 1, w);
#pragma unroll
      for (int pos = 0; pos < 9; pos++) {
        const int dx = emi_dx(pos), dy = emi_dy(pos);
        uint32_t e = 0;
        int sq = 0;       // SSE: sum of d * d
        uint32_t lo = 0;  // SSE: sum of (d * d) mod 16 = ((d & 7)^2) & 15
#pragma unroll
        for (int r = 0; r < UH; r++) {
          if (kSadEmi && (r & 1) && (fen == 1 || fen == 3)) continue;   // FEN: even rows (unit rows start even)
#pragma unroll
          for (int k = 0; k < KW; k++) {
            const uint32_t dd = pk_sub(kraw[r][k], rpair(w[r + 1 + dy], 1 + dx + 2 * k));
            if constexpr (kSadEmi) {
              e = udot2(pk_abs(dd), 0x00010001u, e);
            } else {
              sq = dot2(dd, dd, sq);
              const uint32_t m = dd & 0x00070007u;
              const uint32_t f = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, m) * __builtin_bit_cast(v2u, m)) & 0x000F000Fu;
              lo = udot2(f, 0x00010001u, lo);
            }
          }
        }
        // xGetSSE at bitDepth 10 sums (d * d) >> 4 per sample: (sum d^2 - sum (d^2 mod 16)) / 16, exactly
        if constexpr (!kSadEmi) e = ((uint32_t)sq - lo) >> (2 * kDsh);
        e9[pos] += e;
      }
    }
#pragma unroll
    for (int pos = 0; pos < 9; pos++) {
      uint32_t v = group_sum<L>(e9[pos] & live);
      if constexpr (kSadEmi) v = (v << ((fen == 1 || fen == 3) ? 1 : 0)) >> kDsh;   // xGetSAD12/24/48
      e9[pos] = v;
    }
    const int sx = mvx, sy = mvy;
    uint32_t best = e9[0] + mvc(ml, mv_bits(sx, sy, 2, mvp_x, mvp_y));
    uint32_t best_cost = best - e9[0];
    int bx = sx, by = sy;
    const bool top = sy - 1 >= j.lt_y, bot = sy + 1 <= j.rb_y;
    const bool left = sx - 1 >= j.lt_x, right = sx + 1 <= j.rb_x;
#pragma unroll
    for (int pos = 1; pos <= 8; pos++) {
      const int dx = emi_dx(pos), dy = emi_dy(pos);
      const bool ok = (dy == -1 ? top : (dy == 1 ? bot : true)) && (dx == -1 ? left : (dx == 1 ? right : true));
      if (ok) {
        const uint32_t d = e9[pos];
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (k == n_emi) emi[k] = d;
        n_emi++;
        if (d < best) {
          const uint32_t cst = mvc(ml, mv_bits(sx + dx, sy + dy, 2, mvp_x, mvp_y));
          if (d + cst < best) {
            best = d + cst;
            best_cost = cst;
            bx = sx + dx;
            by = sy + dy;
          }
        }
      }
    }
    cval = best - best_cost;
    mvx = bx;
    mvy = by;
  }
  if (u == 0) {
    g10_rec[wid][lane][1] = make_uint4(0u, 0u, cval, emi[0]);
    g10_rec[wid][lane][2] = make_uint4(emi[1], emi[2], emi[3], emi[4]);
    g10_rec[wid][lane][3] = make_uint4(emi[5], emi[6], emi[7], (uint32_t)n_emi);
    g10_rec_jid[wid][lane] = !active ? -1 : jid;
  }

  // ---- the resident half: window rows -4..UH+3, cols -4..UW+3 around mv_int', key columns --------
  uint32_t v[RV][NV];
  KeySrc<UW, UJ> K;
  auto load_half = [&](int h) FME_AI {
    load_window(ref_pic(), ox + mvx - 4, oy + h * kHalfRows + mvy - 4, v);
    uint32_t kraw[UH][KW];
    if constexpr (UPL == 1) {
#pragma unroll
      for (int r = 0; r < UH; r++)
#pragma unroll
        for (int k = 0; k < KW; k++) kraw[r][k] = kraw0[r][k];
    } else {
      load_kraw(h, kraw);
    }
#pragma unroll
    for (int c = 0; c < UW; c++)
#pragma unroll
      for (int jj = 0; jj < UJ; jj++) {
        const uint32_t hs = (c & 1) ? 0x07060302u : 0x05040100u;
        K.k[c][jj] = __builtin_amdgcn_perm(kraw[2 * jj + 1][c >> 1], kraw[2 * jj][c >> 1], hs);
      }
  };
  load_half(0);
  int cur = 0;
  auto over_halves = [&](auto&& pass, auto& d) FME_AI {
    pass(d);
    if constexpr (UPL == 2) {
      cur ^= 1;
      __builtin_amdgcn_sched_barrier(0);
      launder(v);
      load_half(cur);
      __builtin_amdgcn_sched_barrier(0);
      std::remove_reference_t<decltype(d)> d2;
      pass(d2);
#pragma unroll
      for (int m = 0; m < (int)(sizeof(d) / sizeof(d[0])); m++) d[m] += d2[m];
    }
  };

  // ---- 2. half-pel stage: the integer columns' pass, then the six side candidates -------------
  uint32_t hbest = 0xFFFFFFFFu;
  int hbi = 9;
  {
    const int qy[3] = {0, -2, 2};
    uint32_t d[3];
    over_halves([&](uint32_t (&dd)[3]) FME_AI { qpass<UW, UH, T, 0, 3>(v, K, met, 0, qy, dd); }, d);
    take_half<L>(0, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(1, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(2, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
  }
  {
    uint32_t d[6];
    over_halves([&](uint32_t (&dd)[6]) FME_AI { half_sides<UW, UH, T>(v, K, met, dd); }, d);
    take_half<L>(3, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(5, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(7, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(4, d[3], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(6, d[4], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(8, d[5], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
  }
  const int hx = h9_dx(hbi), hy = h9_dy(hbi);

  // ---- 3. quarter-pel stage: a pass per horizontal offset 2hx - 1, 2hx, 2hx + 1 (Q9 candidate 0 =
  // the half best, its cost already known) -----------------------------------------------------
  uint32_t qbest = hbest;
  int qbi = 0;
  auto qcol = [&](auto k_c) FME_AI {
    constexpr int kk = decltype(k_c)::value;   // dqx = kk - 1
    constexpr int NQ = kk == 1 ? 2 : 3;
    int qy[NQ];
    if constexpr (kk == 1) {
      qy[0] = 2 * hy - 1;
      qy[1] = 2 * hy + 1;
    } else {
      qy[0] = 2 * hy - 1;
      qy[1] = 2 * hy;
      qy[2] = 2 * hy + 1;
    }
    uint32_t d[NQ];
    over_halves([&](uint32_t (&dd)[NQ]) FME_AI { qpass<UW, UH, T, kRuntime, NQ>(v, K, met, 2 * hx + kk - 1, qy, dd); }, d);
    take_qtr<L>(q9_index(kk - 1, -1), d[0], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
    if constexpr (kk == 1) {
      take_qtr<L>(q9_index(0, 1), d[1], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
    } else {
      take_qtr<L>(q9_index(kk - 1, 0), d[1], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
      take_qtr<L>(q9_index(kk - 1, 1), d[2], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
    }
  };
  static_for<0, 3>(qcol);
  const int bq = qbi;

  // ---- the record, bytes 0..15 (mv_int, half, qtr, frac_cost); the tail adds the rest ------------
  typedef __attribute__((address_space(1))) u32x4a gw4;
  const uint32_t r_mv = (uint32_t)(uint16_t)mvx | ((uint32_t)(uint16_t)mvy << 16);
  const uint32_t r_hq = (uint32_t)(uint8_t)hx | ((uint32_t)(uint8_t)hy << 8) | ((uint32_t)(uint8_t)q9_dx(bq) << 16) |
                        ((uint32_t)(uint8_t)q9_dy(bq) << 24);
  if (u == 0) g10_rec[wid][lane][0] = make_uint4(r_mv, 0u, r_hq, qbest);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int NP = 64 / L;
#pragma unroll
  for (int s0 = 0; s0 < (NP * 4 + 63) / 64; s0++) {
    const int r = s0 * 16 + (lane >> 2);
    if (r < NP) {
      const int src = r * L;
      const int rj = g10_rec_jid[wid][src];
      if (rj >= 0) {
        const uint4 q = g10_rec[wid][src][lane & 3];
        u32x4a o;
        o.x = q.x; o.y = q.y; o.z = q.z; o.w = q.w;
        *(gw4*)(reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(outp + rj) + 16 * (lane & 3)) = o;
      }
    }
  }
}

__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7; }

}  // namespace

// The 8-bit lane kernel's classes and unit shapes (fme_lane.hip; k_schedule's tile layout is
// sched_params(), shared): 4x8 units, 4x4 units for 8x4 / 16x4 / 16x12.
#define FME_L10_CLASSES(X)                                                                           \
  X(0, 4, 8, 4, 8) X(3, 4, 16, 4, 8) X(1, 8, 4, 4, 4) X(4, 16, 4, 4, 4) X(2, 8, 8, 4, 8)              \
  X(5, 8, 16, 4, 8) X(6, 16, 8, 4, 8) X(9, 16, 16, 4, 8) X(10, 8, 32, 4, 8) X(11, 32, 8, 4, 8)        \
  X(12, 16, 32, 4, 8) X(13, 32, 16, 4, 8) X(16, 32, 32, 4, 8) X(17, 16, 64, 4, 8) X(18, 64, 16, 4, 8) \
  X(19, 32, 64, 4, 8) X(20, 64, 32, 4, 8) X(23, 64, 64, 4, 8) X(7, 12, 16, 4, 8) X(8, 16, 12, 4, 4)   \
  X(14, 24, 32, 4, 8) X(15, 32, 24, 4, 8) X(21, 48, 64, 4, 8) X(22, 64, 48, 4, 8)

// One persistent kernel for every class, the 8-bit kernel's work order: a workgroup claims four
// consecutive wave tiles per atomic from its XCD's queue (Schedule::xq), then the other XCDs'.
#define FME_CASE10(ID, PW_, PH_, UW_, UH_)                                                 \
  case ID:                                                                                 \
    lane_unit10<PW_, PH_, UW_, UH_>(a, w.perm, sc->class_off[ID], sc->class_cnt[ID], wt, wid); \
    break;
__global__ __launch_bounds__(kL10NT) __attribute__((amdgpu_waves_per_eu(FME_L10_WAVES)))
void k_search_lane10(BatchArgs a, WorkBufs w) {
  constexpr int S = FME_LANE_SUBBANDS;
  const Schedule* __restrict__ sc = w.sched;
  if (sc->invalid) return;   // rejected batch: the tail marks every record
  int32_t* ctr = w.tile_ctr;
  __shared__ int32_t s_xq[8][S][kNumClasses + 1];
  {
    const uint32_t* ps = reinterpret_cast<const uint32_t*>(a.pics);
    uint32_t* pd = reinterpret_cast<uint32_t*>(g10_pics);
    for (int i = threadIdx.x; i < (int)(sizeof(g10_pics) / 4); i += kL10NT) pd[i] = ps[i];
    for (int i = threadIdx.x; i < FME_MAX_LAMBDAS * kCostBits; i += kL10NT)
      g10_cost[i / kCostBits][i % kCostBits] = simd::mv_cost(a.mlambda[i / kCostBits], (uint32_t)(i % kCostBits));
    for (int i = threadIdx.x; i < 8 * S * (kNumClasses + 1); i += kL10NT) (&s_xq[0][0][0])[i] = (&sc->xq[0][0][0])[i];
  }
  const int home = xcc_id(), wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  constexpr int kGroup = kL10NT / 64;
  __shared__ int32_t claim[2];
  int x = home, tried = 0, par = 0;
  if (threadIdx.x == 0) claim[0] = atomicAdd(&ctr[x], 1);
  __syncthreads();
  int t = __builtin_amdgcn_readfirstlane(claim[0]);
  while (true) {
    const int len = s_xq[x][S - 1][kNumClasses];
    if (kGroup * t >= len) {
      if (++tried == 8) break;
      x = (home + tried) & 7;
      par ^= 1;
      if (threadIdx.x == 0) claim[par] = atomicAdd(&ctr[x], 1);
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(claim[par]);
      continue;
    }
    int nxt = 0;
    if (threadIdx.x == 0) nxt = atomicAdd(&ctr[x], 1);
    const int tw = kGroup * t + wid;
    if (tw < len) {
      int q = 0, c = 0;
      while (q < S - 1 && tw >= s_xq[x][q][kNumClasses]) q++;
      while (c < kNumClasses - 1 && tw >= s_xq[x][q][c + 1]) c++;
      const int ci = c;   // queue position -> class
      c = lane_class_at(ci);
      const int nt = sc->prefix[c + 1] - sc->prefix[c];
      const int lo = (int)(((long long)nt * (x * S + q)) / (8 * S));
      const int wt = __builtin_amdgcn_readfirstlane(lo + (tw - s_xq[x][q][ci]));
      switch (c) {
        FME_L10_CLASSES(FME_CASE10)
        default: break;
      }
    }
    par ^= 1;
    if (threadIdx.x == 0) claim[par] = nxt;
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(claim[par]);
  }
}
#undef FME_CASE10

hipError_t launch_search_lane10(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    cus = cu_count(dev);
  }
  if (a.n <= 0) return hipSuccess;
  int max_l = 0, classes = 0;
  for (int c = 0; c < kNumClasses; c++)
    if (lane_lanes_per_pu(c)) {
      max_l = std::max(max_l, lane_lanes_per_pu(c));
      classes++;
    }
  const long long waves = ((long long)a.n * max_l + 63) / 64 + classes;
  const int blocks = (int)std::min<long long>((waves + kL10NT / 64 - 1) / (kL10NT / 64), 4LL * cus);
  hipLaunchKernelGGL(k_search_lane10, dim3(blocks), dim3(kL10NT), 0, s, a, w);
  return hipGetLastError();
}

}  // namespace fme
