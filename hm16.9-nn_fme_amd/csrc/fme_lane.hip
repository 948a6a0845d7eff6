// fme_lane.hip — lane-per-unit EMI + FracDIF search kernel (gfx950).
//
// One lane owns one unit of a PU: the whole PU for 8x4 / 4x8, an 8x4 / 4x8 half for
// 16x4 / 4x16, an 8x8 block for the power-of-two 8x8-tiled shapes (8x8 .. 64x64).  A PU's
// L units sit in L consecutive lanes of one wavefront; SATD / SSE partials are summed over
// those lanes with xor shuffles, so every lane of the group takes the same decisions.  Each
// lane keeps its reference window in VGPRs as (sample - 128) bytes and never touches LDS:
//
//   1. load     window rows -5..UH+4, cols -5..UW+4 around the TZ MV (clamped rows, edge-
//               replicated columns near the picture border), the key block (org bytes, or
//               the job's int16 key block for bi-pred), re-aligned to byte 0.
//   2. EMI      9 integer distortions (SSE = So2 - 2 Sop + Spp with v_dot4_i32_i8 on the
//               s-128 bytes) and the square-step decision (TEncSearch.cpp:1324-1377,
//               1155-1188, 5043-5050), then the window is re-centred on mv_int' in place.
//   3. half     the 9 candidates of xPatternRefinement (TEncSearch.cpp:1591-1645) around
//               mv_int' in three triples that share their filtered columns: {(0,0),(0,-1),
//               (0,1)} from the transposed window, {(-1,0),(-1,-1),(-1,1)} and {(1,0),(1,-1),
//               (1,1)} from the horizontal first stage (xExtDIFUpSamplingH, 6331-6365).
//   4. quarter  the 8 candidates around the half best (xExtDIFUpSamplingQ, 6378-6532) as
//               separable 2-D filters with per-lane taps: a phase with fraction 0 uses the
//               tap set {0,0,0,64,0,0,0,0}, which reproduces HM's copy / 1-D paths exactly
//               ((64 A + 2048) >> 12 == (A + 32) >> 6).
// All predictions are formed in the (p - 128) domain: the rounding offsets absorb the 128
// ((s + 8224) >> 6 - 128 == (s + 32) >> 6 for 1-D, (s + 526336) >> 12 - 128 == (s + 2048)
// >> 12 for 2-D), and key - pred is unchanged.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <utility>

#include "fme_device.h"
#include "fme_simd.h"

#ifndef FME_XCD_SWIZZLE
#define FME_XCD_SWIZZLE 1
#endif
// Candidates per quarter pass (2: column-phase pairs, 1: one candidate per pass — fewer live
// registers, the first-stage column recomputed per candidate) and half-stage vertical pairs
// {(0,-1),(0,1)} and {(s,-1),(s,1)} in one pass (2) or one candidate per pass (1); the 8x4 unit
// shape always uses 1 (lane_unit).  A/B on the 1080p batch (tools/ab_bench.py, one kernel for
// every class, all shapes alike): 1/1 1.185 ms, QPAIR 2 1.146, HPAIR 2 1.091, both 2 1.054 — the
// shared first stages save more issue slots than the extra live key - pred array costs at
// 2 waves/SIMD (FME_LANE_WAVES 3 spills: 1.480 ms).
#ifndef FME_LANE_QPAIR
#define FME_LANE_QPAIR 1
#endif
#ifndef FME_LANE_HPAIR
#define FME_LANE_HPAIR 2
#endif
#ifndef FME_LANE_PAIR84   // 1: the 8x4 unit shape paired too
#define FME_LANE_PAIR84 0
#endif
// Each PU class's search is its own function (noinline): inlined into one switch, the classes'
// hoisted constants and live ranges merged into one allocation that spilled (1,286 VGPRs and
// 2,098 SGPRs at 3 waves/SIMD) although every class alone fits.
#ifndef FME_LANE_UNIT_ATTR
#define FME_LANE_UNIT_ATTR __attribute__((noinline))
#endif
// 1: the half stage's six side candidates from shared half columns and the quarter stage as three
// column-phase passes of all their candidates (fewest first stages; needs 2 waves/SIMD of
// registers); 0: the pair modes above
#ifndef FME_LANE_SHARE
#define FME_LANE_SHARE 1
#endif
// 1: the 2-D passes' second stage with taps scaled by 16, so a pair of outputs is packed by one
// v_perm of the two sums' high halves ((16 s) >> 16 == s >> 12) and clipped as a packed pair
// (v_pk_max_i16 / v_pk_min_i16), and the 1-D horizontal rows of the half stage shifted and clipped
// as the packed pairs the vertical pass already holds: 3 instructions per output pair instead of 5
// (two shifts, two med3, one perm).  0: per-output shift and clamp.  A/B on the 1080p batch
// (tools/ab_bench.py, identical results): search 0.904 -> 0.871 ms, batch 1.087 -> 1.055 ms
// (profiles/r06_ab.log).
#ifndef FME_LANE_PK16
#define FME_LANE_PK16 1
#endif
// occupancy target (waves per SIMD) that bounds the register allocation
#ifndef FME_LANE_WAVES
#define FME_LANE_WAVES 2
#endif

// 1: a diagnostic build (make variant NAME=stamps DEFS=-DFME_LANE_STAMPS=1, tools/lane_stamps.py):
// s_memtime stamps at the phase boundaries of every lane_unit call, summed per (class, phase) into
// a debug buffer of their own (g_lane_stamps, read by fme_debug_lane_stamps); each boundary first
// waits for the wave's outstanding loads, so a phase's share includes the memory latency it
// exposes.  Never the product build: the waits forbid overlaps the real kernel has.
#ifndef FME_LANE_STAMPS
#define FME_LANE_STAMPS 0
#endif

namespace fme {
#if FME_LANE_STAMPS
// [class][phase]: 0 job + key loads, 1 EMI step, 2 sub-pel window + key, 3 half-pel stage,
// 4 quarter-pel stage, 5 record stores, 6 calls (wave tiles), 7 unused
__device__ unsigned long long g_lane_stamps[kNumClasses][8];
#endif
namespace {
using namespace simd;

#define FME_AI __attribute__((always_inline))

#if FME_LANE_STAMPS
__device__ __forceinline__ unsigned long long lane_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define FME_STAMP(k) const unsigned long long stamp_##k = lane_stamp()
#else
#define FME_STAMP(k) (void)0
#endif

constexpr int kLaneNT = 256;

// ---- small helpers -------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// Sum over the L lanes of a PU's group (L a power of two <= 64): every lane of the group ends
// with the total.  Offsets 1, 2 swap within a quad (DPP quad_perm); once each quad / octet
// holds its sum, the half-mirror / mirror partner of a lane (DPP row_half_mirror / row_mirror,
// lane i <-> 7-i / 15-i) lies in the other quad / octet; 16 is a ds_swizzle xor, 32 a
// bpermute.  (A/B on the 1080p batch: -1 % search time against bpermute for every step.)
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

// The first dot product of a chain with an inline-constant accumulator, in the VOP3P encoding:
// the compiler picks v_dot4c / v_dot2c (accumulator tied to the destination) and materialises the
// constant with a v_mov first (≈ 700 movs per lane-class function, 11 % of its VALU).
__device__ __forceinline__ int dot4_k32(uint32_t a, uint32_t b) {
  int d;
  asm("v_dot4_i32_i8 %0, %1, %2, 32" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ int dot2_k0(uint32_t a, uint32_t b) {
  int d;
  asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

// low 16 bits of a and b -> one packed pair (a in the low half)
__device__ __forceinline__ uint32_t pack2(int a, int b) { return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u); }
__device__ __forceinline__ int clamp_s8(int v) { return min(max(v, -128), 127); }

// Bytes (b, b+1) of two dwords (row r0 in src1, row r1 in src0) -> sign-extended int16 pair.
__device__ __forceinline__ uint32_t sext_pair(uint32_t hi_row, uint32_t lo_row, int byte) {
  const uint32_t sel = (uint32_t)byte | 0x0c00u | ((uint32_t)(4 + byte) << 16) | 0x0c000000u;
  const uint32_t z = __builtin_amdgcn_perm(hi_row, lo_row, sel);    // zero-extended s' bytes
  return pk_sub(z ^ 0x00800080u, 0x00800080u);                       // sign extension
}

// Opaque to the optimiser (no instructions): values derived from the window before this point
// are not reused after it, so common subexpressions do not stay live across passes.
template <int R, int N>
__device__ __forceinline__ void launder(uint32_t (&v)[R][N]) {
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int k = 0; k < N; k++) asm volatile("" : "+v"(v[r][k]));
}

// 4 bytes starting at byte b of a row held in dwords v[0..N).  Every caller passes a b that
// is a compile-time constant after unrolling, so the register indices fold.
template <int N>
__device__ __forceinline__ uint32_t rbytes(const uint32_t (&v)[N], int b) {
  const int q = b >> 2, r = b & 3;
  return r == 0 ? v[q] : __builtin_amdgcn_alignbyte(v[q + 1], v[q], (uint32_t)r);
}
// 4 bytes starting at byte b + d, d in {0, 1} per lane (b constant after unrolling)
template <int N>
__device__ __forceinline__ uint32_t rbytes_d(const uint32_t (&v)[N], int b, uint32_t d) {
  const int q = b >> 2, r = b & 3;
  const uint32_t lo = v[q], hi = v[q + 1];
  return r == 3 ? (d ? hi : __builtin_amdgcn_alignbyte(hi, lo, 3u))
                : __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)r + d);
}
// bytes b, b+1 of one dword -> sign-extended int16 pair
__device__ __forceinline__ uint32_t sext_bytes(uint32_t d, int b) {
  const uint32_t sel = (uint32_t)b | 0x0c00u | ((uint32_t)(b + 1) << 16) | 0x0c000000u;
  return pk_sub(__builtin_amdgcn_perm(0u, d, sel) ^ 0x00800080u, 0x00800080u);
}

// 8-tap luma filter taps for fraction f in 0..3 as int8 quads (f = 0: 64 at tap 3).
__device__ __forceinline__ void taps8_any(int f, uint32_t& lo, uint32_t& hi) {
  const uint32_t l1 = q8(-1, 4, -10, 58), h1 = q8(17, -5, 1, 0);
  const uint32_t l2 = q8(-1, 4, -11, 40), h2 = q8(40, -11, 4, -1);
  const uint32_t l3 = q8(0, 1, -5, 17), h3 = q8(58, -10, 4, -1);
  const uint32_t l0 = q8(0, 0, 0, 64), h0 = 0u;
  lo = f == 0 ? l0 : (f == 1 ? l1 : (f == 2 ? l2 : l3));
  hi = f == 0 ? h0 : (f == 1 ? h1 : (f == 2 ? h2 : h3));
}
// tap k of fraction f (k outside 0..7 -> 0)
__device__ __forceinline__ int tap(int f, int k) {
  // rows: f = 0..3, taps 0..7 (TComInterpolationFilter.cpp:57-63)
  const int t0 = k == 3 ? 64 : 0;
  const int t1 = k == 0 ? -1 : k == 1 ? 4 : k == 2 ? -10 : k == 3 ? 58 : k == 4 ? 17 : k == 5 ? -5 : k == 6 ? 1 : 0;
  const int t2 = k == 0 ? -1 : k == 1 ? 4 : k == 2 ? -11 : k == 3 ? 40 : k == 4 ? 40 : k == 5 ? -11 : k == 6 ? 4 : k == 7 ? -1 : 0;
  const int t3 = k == 1 ? 1 : k == 2 ? -5 : k == 3 ? 17 : k == 4 ? 58 : k == 5 ? -10 : k == 6 ? 4 : k == 7 ? -1 : 0;
  if (k < 0 || k > 7) return 0;
  return f == 0 ? t0 : (f == 1 ? t1 : (f == 2 ? t2 : t3));
}
// Coefficient pairs for a vertical 8-tap filter of fraction f whose taps start `o` rows into
// a span of 10 rows read as 5 packed row pairs: pair t = (tap(2t - o), tap(2t + 1 - o)), scaled by
// kVS (FME_LANE_PK16: 16).
constexpr int kVS = FME_LANE_PK16 ? 16 : 1;
__device__ __forceinline__ void vpairs(int f, int o, uint32_t (&c)[5]) {
#pragma unroll
  for (int t = 0; t < 5; t++) c[t] = p16(kVS * tap(f, 2 * t - o), kVS * tap(f, 2 * t + 1 - o));
}
// (s0 >> 12, s1 >> 12) clipped to the s - 128 range, packed, from second-stage sums scaled by kVS.
__device__ __forceinline__ uint32_t pk_round2d(int s0, int s1) {
  if constexpr (FME_LANE_PK16) {
    const v2s m = up(__builtin_amdgcn_perm((uint32_t)s1, (uint32_t)s0, 0x07060302u));   // high halves
    return pk(__builtin_elementwise_min(__builtin_elementwise_max(m, v2s{-128, -128}), v2s{127, 127}));
  } else {
    return pack2(clamp_s8(s0 >> 12), clamp_s8(s1 >> 12));
  }
}
// (h0 >> 6, h1 >> 6) clipped, from the packed pair (h0, h1) of 1-D sums (+32 carried)
__device__ __forceinline__ uint32_t pk_round1d(uint32_t hp) {
  const v2s m = up(hp) >> v2s{6, 6};
  return pk(__builtin_elementwise_min(__builtin_elementwise_max(m, v2s{-128, -128}), v2s{127, 127}));
}

// ---- the key block (key - 128 as packed int16 row pairs): K(x, j) = rows (2j, 2j+1) of column x --
template <int UW, int UJ>
struct KeySrc {
  uint32_t k[UW][UJ];
  __device__ __forceinline__ uint32_t at(int x, int j) const { return k[x][j]; }
  __device__ __forceinline__ void set(int x, int j, uint32_t v) { k[x][j] = v; }
};

// ---- distortion of one unit for one candidate ------------------------------------------------
// How a lane's unit is scored: SATD (had) or SAD, and, for the 4x8 units of an 8x8-tiled PU, the
// lane pair that shares each 8x8 tile (sgn: +1 / -1 per half in the even / odd lane; emask: ~0 in
// the even lane, which reports the tile, 0 in the odd one).
struct Metric {
  bool had;
  uint32_t sgn, emask;
};

// One 8x8 SATD tile split over a lane pair: the even lane holds columns 0..3, the odd lane columns
// 4..7 (X[c][j]: this lane's column c, rows 2j, 2j+1).  xCalcHADs8x8's butterflies
// (TComRdCost.cpp:1330-1425) with the column-distance-4 stage across the pair (DPP quad_perm
// [1,0,3,2]); the odd lane forms b - a instead of a - b, and since every later stage is linear and
// the transform ends in |.|, that sign never shows.  Returns this lane's sum of the last stage's
// max terms (see satd_packed).
__device__ __forceinline__ uint32_t satd8_pair(uint32_t (&X)[4][4], uint32_t sgn) {
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
  return s;
}

// X[c][j]: key - pred, column c, rows (2j, 2j+1) packed.  Sum over the unit's T x T tiles of
// xCalcHADs (had) or SAD; for a unit that is half of an 8x8 tile (UW 4, T 8) the even lane
// returns the tile's value and the odd lane 0.
template <int UW, int UH, int T>
__device__ __forceinline__ uint32_t unit_dist(uint32_t (&X)[UW][UH / 2], const Metric& m) {
  if constexpr (T == 8 && UW == 4) {
    static_assert(UH == 8, "4x8 half tiles");
    if (m.had) {
      uint32_t s = satd8_pair(X, m.sgn);
      s += dpp<0xB1>(s);                 // the tile's total in both lanes
      return ((s + 1) >> 1) & m.emask;   // (2s + 2) >> 2
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
        if (m.had) {
          s += satd_packed<T>(Y);
        } else {
          s += sad_packed<T>(Y);
        }
      }
    return s;
  }
}

// Candidate offsets (xPatternRefinement tables, TEncSearch.cpp:212-236).
__host__ __device__ __forceinline__ constexpr int h9_dx(int i) { return (i == 3 || i == 5 || i == 7) ? -1 : ((i == 4 || i == 6 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int h9_dy(int i) { return (i == 1 || i == 5 || i == 6) ? -1 : ((i == 2 || i == 7 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int q9_dx(int i) { return (i == 3 || i == 5 || i == 7) ? -1 : ((i == 4 || i == 6 || i == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int q9_dy(int i) { return (i == 1 || i == 3 || i == 4) ? -1 : ((i == 2 || i == 7 || i == 8) ? 1 : 0); }
// Q9 index of (dqx, dqy)
__host__ __device__ __forceinline__ constexpr int q9_index(int dx, int dy) {
  return dy == 0 ? (dx == 0 ? 0 : (dx < 0 ? 5 : 6)) : dy < 0 ? (dx == 0 ? 1 : (dx < 0 ? 3 : 4)) : (dx == 0 ? 2 : (dx < 0 ? 7 : 8));
}
// EMI positions: 0 centre, then TL, T, TR, L, R, BL, B, BR (xTZ8PointSquareSearch order)
__host__ __device__ __forceinline__ constexpr int emi_dx(int p) { return (p == 1 || p == 4 || p == 6) ? -1 : ((p == 3 || p == 5 || p == 8) ? 1 : 0); }
__host__ __device__ __forceinline__ constexpr int emi_dy(int p) { return p >= 1 && p <= 3 ? -1 : (p >= 6 ? 1 : 0); }

// =============================================================================================
// Candidate passes of one unit.  v: re-centred window (rows -4..UH+3, cols -4..UW+3, s - 128
// bytes), K: key - 128 as packed column pairs.  Each pass keeps at most two key - pred arrays.
// =============================================================================================
// `live`: ~0 on the lanes of a PU's units, 0 on the idle lanes that pad a group of 6 / 12 / 48
// units (AMP shapes) to a power of two, so they add nothing to the group's sum.
// The MV cost from the workgroup's table: g_cost[lambda][bits] = (UInt)(mlambda * bits / 65536.0)
// (TComRdCost.h:165), computed once per launch by the same double arithmetic.
__device__ __forceinline__ uint32_t mv_cost(const uint32_t* ml, uint32_t bits) { return ml[bits]; }
template <int L>
__device__ __forceinline__ void take_half(int i, uint32_t part, uint32_t live, const uint32_t* ml, int mvx, int mvy, int px,
                                          int py, uint32_t& best, int& bi) {
  const uint32_t d = group_sum<L>(part & live) + mv_cost(ml, mv_bits(2 * mvx + h9_dx(i), 2 * mvy + h9_dy(i), 1, px, py));
  if (d < best || (d == best && i < bi)) {
    best = d;
    bi = i;
  }
}
template <int L>
__device__ __forceinline__ void take_qtr(int i, uint32_t part, uint32_t live, const uint32_t* ml, int mvx, int mvy, int hx,
                                         int hy, int px, int py, uint32_t& best, int& bi) {
  const int qx = 2 * hx + q9_dx(i), qy = 2 * hy + q9_dy(i);
  const uint32_t d = group_sum<L>(part & live) + mv_cost(ml, mv_bits(4 * mvx + qx, 4 * mvy + qy, 0, px, py));
  if (d < best || (d == best && i < bi)) {
    best = d;
    bi = i;
  }
}

// (0,0), (0,-1), (0,1)
template <int UW, int UH, int T, int HPM>
__device__ __forceinline__ void half_center(uint32_t (&v)[UH + 8][UW / 4 + 2], const KeySrc<UW, UH / 2>& K,
                                            const Metric& had, uint32_t (&d)[3]) {
  constexpr int RV = UH + 8, UJ = UH / 2;
  uint32_t c2lo, c2hi;
  taps8(2, c2lo, c2hi);
  {   // (0,0): integer samples, window' rows 4+y, cols 4+x
    uint32_t X[UW][UJ];
#pragma unroll
    for (int x = 0; x < UW; x++)
#pragma unroll
      for (int jj = 0; jj < UJ; jj++)
        X[x][jj] = pk_sub(K.at(x, jj), sext_pair(v[5 + 2 * jj][(x + 4) >> 2], v[4 + 2 * jj][(x + 4) >> 2], (x + 4) & 3));
    d[0] = unit_dist<UW, UH, T>(X, had);
  }
  launder(v);
  // (0,-1), (0,1): vertical half-pel on integer columns (transposed window')
  auto vpass = [&](auto sel_c) FME_AI {   // sel 1: (0,-1) only, 2: (0,1) only, 3: both
    constexpr int sel = decltype(sel_c)::value;
    uint32_t X1[UW][UJ], X2[UW][UJ];
#pragma unroll
    for (int g = 0; g < UW / 4; g++) {
      uint32_t CB[4][RV / 4];   // columns 4g..4g+3 (window' cols 4g+4 ..), 4 rows per dword
#pragma unroll
      for (int q = 0; q < RV / 4; q++) {
        const uint32_t rows[4] = {v[4 * q][g + 1], v[4 * q + 1][g + 1], v[4 * q + 2][g + 1], v[4 * q + 3][g + 1]};
        uint32_t cols[4];
        transpose4x4(rows, cols);
#pragma unroll
        for (int c = 0; c < 4; c++) CB[c][q] = cols[c];
      }
#pragma unroll
      for (int c4 = 0; c4 < 4; c4++) {
        const int x = 4 * g + c4;
        int v1[UH + 1];   // half rows i = 0..UH (between rows i-1, i): taps on window' rows i..i+7
#pragma unroll
        for (int i = (sel == 2 ? 1 : 0); i <= (sel == 1 ? UH - 1 : UH); i++) {
          const int acc = dot4(rbytes(CB[c4], i), c2lo, 32);
          v1[i] = clamp_s8(dot4(rbytes(CB[c4], i + 4), c2hi, acc) >> 6);
        }
#pragma unroll
        for (int jj = 0; jj < UJ; jj++) {
          if (sel & 1) X1[x][jj] = pk_sub(K.at(x, jj), pack2(v1[2 * jj], v1[2 * jj + 1]));
          if (sel & 2) X2[x][jj] = pk_sub(K.at(x, jj), pack2(v1[2 * jj + 1], v1[2 * jj + 2]));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (sel & 1) d[1] = unit_dist<UW, UH, T>(X1, had);
    if (sel & 2) d[2] = unit_dist<UW, UH, T>(X2, had);
  };
  if constexpr (HPM == 2) {
    vpass(std::integral_constant<int, 3>{});
  } else {
    vpass(std::integral_constant<int, 1>{});
    launder(v);
    vpass(std::integral_constant<int, 2>{});
  }
}

// (s,0), (s,-1), (s,1) for s = -1 (SIDE 0: half column x) or +1 (SIDE 1: half column x+1)
template <int UW, int UH, int T, int SIDE, int HPM>
__device__ __forceinline__ void half_side(uint32_t (&v)[UH + 8][UW / 4 + 2], const KeySrc<UW, UH / 2>& K,
                                          const Metric& had, uint32_t (&d)[3]) {
  constexpr int RV = UH + 8, UJ = UH / 2;
  uint32_t c2lo, c2hi;
  taps8(2, c2lo, c2hi);
  launder(v);
  {   // (s,0): horizontal half-pel, half column jc = x + SIDE (window' bytes jc .. jc+7)
    uint32_t X[UW][UJ];
#pragma unroll
    for (int x = 0; x < UW; x++) {
      const int jc = x + SIDE;
      int h1[UH];
#pragma unroll
      for (int y = 0; y < UH; y++)
        h1[y] = clamp_s8(dot4(rbytes(v[y + 4], jc + 4), c2hi, dot4(rbytes(v[y + 4], jc), c2lo, 32)) >> 6);
#pragma unroll
      for (int jj = 0; jj < UJ; jj++) X[x][jj] = pk_sub(K.at(x, jj), pack2(h1[2 * jj], h1[2 * jj + 1]));
    }
    d[0] = unit_dist<UW, UH, T>(X, had);
  }
  launder(v);
  // (s,-1), (s,1): 2-D half-pel (first stage rows -4..UH+3 of half column jc, then vertical)
  auto dpass = [&](auto sel_c) FME_AI {   // sel 1: (s,-1) only, 2: (s,1) only, 3: both
    constexpr int sel = decltype(sel_c)::value;
    const uint32_t c16[4] = {p16(-1, 4), p16(-11, 40), p16(40, -11), p16(4, -1)};
    const uint32_t c16o[5] = {p16(0, -1), p16(4, -11), p16(40, 40), p16(-11, 4), p16(-1, 0)};
    uint32_t XB[UW][UJ], XC[UW][UJ];
#pragma unroll
    for (int x = 0; x < UW; x++) {
      const int jc = x + SIDE;
      launder(v);
      uint32_t HP[RV / 2];
#pragma unroll
      for (int r = 0; r < RV; r += 2) {
        const int h0 = dot4(rbytes(v[r], jc + 4), c2hi, dot4(rbytes(v[r], jc), c2lo, 0));
        const int h1 = dot4(rbytes(v[r + 1], jc + 4), c2hi, dot4(rbytes(v[r + 1], jc), c2lo, 0));
        HP[r / 2] = pack2(h0, h1);
      }
      int v2[UH + 1];
#pragma unroll
      for (int i = (sel == 2 ? 1 : 0); i <= (sel == 1 ? UH - 1 : UH); i++) {
        int acc = 2048;
        if ((i & 1) == 0) {
#pragma unroll
          for (int t = 0; t < 4; t++) acc = dot2(HP[i / 2 + t], c16[t], acc);
        } else {
#pragma unroll
          for (int t = 0; t < 5; t++) acc = dot2(HP[(i - 1) / 2 + t], c16o[t], acc);
        }
        v2[i] = clamp_s8(acc >> 12);
      }
#pragma unroll
      for (int jj = 0; jj < UJ; jj++) {
        if (sel & 1) XB[x][jj] = pk_sub(K.at(x, jj), pack2(v2[2 * jj], v2[2 * jj + 1]));
        if (sel & 2) XC[x][jj] = pk_sub(K.at(x, jj), pack2(v2[2 * jj + 1], v2[2 * jj + 2]));
      }
      __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure)
    }
    if (sel & 1) d[1] = unit_dist<UW, UH, T>(XB, had);
    if (sel & 2) d[2] = unit_dist<UW, UH, T>(XC, had);
  };
  if constexpr (HPM == 2) {
    dpass(std::integral_constant<int, 3>{});
  } else {
    dpass(std::integral_constant<int, 1>{});
    dpass(std::integral_constant<int, 2>{});
  }
}

// All six side candidates from the UW + 1 half-pel columns x - 1/2, x = 0..UW, which both sides
// share (side -1 takes columns 0..UW-1, side +1 columns 1..UW): in H9 numbering d = {3: (-1,0),
// 5: (-1,-1), 7: (-1,1), 4: (1,0), 6: (1,-1), 8: (1,1)} as d[0..5] = 3, 5, 7, 4, 6, 8.  One first
// stage per half column (rows -4..UH+3, xExtDIFUpSamplingH's filteredBlock[0][2] row) gives all
// three vertical phases: the first-stage sums carry +32, so the integer rows' 1-D rounding is
// (s + 32) >> 6 of the same sums, and the vertical half-pel pass, whose taps add to 64, gets its
// 2048 rounding offset from them with a zero accumulator.
template <int UW, int UH, int T>
__device__ __forceinline__ void half_sides(uint32_t (&v)[UH + 8][UW / 4 + 2], const KeySrc<UW, UH / 2>& K,
                                           const Metric& had, uint32_t (&d)[6]) {
  constexpr int RV = UH + 8, UJ = UH / 2;
  uint32_t c2lo, c2hi;
  taps8(2, c2lo, c2hi);
  const uint32_t c16[4] = {p16(-kVS, 4 * kVS), p16(-11 * kVS, 40 * kVS), p16(40 * kVS, -11 * kVS), p16(4 * kVS, -kVS)};
  const uint32_t c16o[5] = {p16(0, -kVS), p16(4 * kVS, -11 * kVS), p16(40 * kVS, 40 * kVS), p16(-11 * kVS, 4 * kVS),
                            p16(-kVS, 0)};
  uint32_t XS[6][UW][UJ];
#pragma unroll
  for (int k = 0; k <= UW; k++) {
    launder(v);
    int hv[RV];
#pragma unroll
    for (int r = 0; r < RV; r++) hv[r] = dot4(rbytes(v[r], k + 4), c2hi, dot4_k32(rbytes(v[r], k), c2lo));
    uint32_t HP[RV / 2];
#pragma unroll
    for (int r = 0; r < RV; r += 2) HP[r / 2] = pack2(hv[r], hv[r + 1]);
    uint32_t X0[UJ], XM[UJ], XP[UJ];   // (s,0), (s,-1), (s,1) of this column
    int v2[UH + 1];   // second-stage sums (FME_LANE_PK16: x 16), rounded below
#pragma unroll
    for (int i = 0; i <= UH; i++) {   // half rows between window rows i+3, i+4
      int acc;
      if ((i & 1) == 0) {
        acc = dot2_k0(HP[i / 2], c16[0]);
#pragma unroll
        for (int t = 1; t < 4; t++) acc = dot2(HP[i / 2 + t], c16[t], acc);
      } else {
        acc = dot2_k0(HP[(i - 1) / 2 + 1], c16o[1]);   // pair 0 is (0, -1): row i-1 only
        acc = dot2(HP[(i - 1) / 2], c16o[0], acc);
#pragma unroll
        for (int t = 2; t < 5; t++) acc = dot2(HP[(i - 1) / 2 + t], c16o[t], acc);
      }
      v2[i] = FME_LANE_PK16 ? acc : clamp_s8(acc >> 12);
    }
#pragma unroll
    for (int jj = 0; jj < UJ; jj++) {
      if constexpr (FME_LANE_PK16) {
        X0[jj] = pk_round1d(HP[2 + jj]);   // rows 4 + 2 jj, 5 + 2 jj of the first stage
        XM[jj] = pk_round2d(v2[2 * jj], v2[2 * jj + 1]);
        XP[jj] = pk_round2d(v2[2 * jj + 1], v2[2 * jj + 2]);
      } else {
        X0[jj] = pack2(clamp_s8(hv[4 + 2 * jj] >> 6), clamp_s8(hv[5 + 2 * jj] >> 6));
        XM[jj] = pack2(v2[2 * jj], v2[2 * jj + 1]);
        XP[jj] = pack2(v2[2 * jj + 1], v2[2 * jj + 2]);
      }
    }
#pragma unroll
    for (int jj = 0; jj < UJ; jj++) {
      if (k < UW) {   // side -1, column k
        XS[0][k][jj] = pk_sub(K.at(k, jj), X0[jj]);
        XS[1][k][jj] = pk_sub(K.at(k, jj), XM[jj]);
        XS[2][k][jj] = pk_sub(K.at(k, jj), XP[jj]);
      }
      if (k > 0) {    // side +1, column k - 1
        XS[3][k - 1][jj] = pk_sub(K.at(k - 1, jj), X0[jj]);
        XS[4][k - 1][jj] = pk_sub(K.at(k - 1, jj), XM[jj]);
        XS[5][k - 1][jj] = pk_sub(K.at(k - 1, jj), XP[jj]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure)
  }
#pragma unroll
  for (int m = 0; m < 6; m++) d[m] = unit_dist<UW, UH, T>(XS[m], had);
}

// Quarter pass over one column phase k (dqx = k - 1) with all its row phases l (dqy = l - 1)
// except the half best (1,1) itself: 3, 2, 3 candidates for k = 0, 1, 2, one first stage each.
// First-stage sums carry +32 (the vertical taps add to 64: the 2048 rounding offset), and a
// fraction-0 phase filters with {0,0,0,64,0,0,0,0}, which equals HM's copy / 1-D paths after
// rounding ((64 A + 2048) >> 12 == (A + 32) >> 6).
template <int UW, int UH, int T, int k>
__device__ __forceinline__ void qtr_col(uint32_t (&v)[UH + 8][UW / 4 + 2], const KeySrc<UW, UH / 2>& K,
                                        const Metric& had, int hx, int hy, uint32_t (&d)[3]) {
  constexpr int RV = UH + 8, UJ = UH / 2;
  constexpr int NP = k == 1 ? 2 : 3;
  const int LS[3] = {0, k == 1 ? 2 : 1, 2};
  const int qx = 2 * hx + (k - 1);
  const int ix = qx >> 2, fx = qx & 3;
  const uint32_t dlt = (uint32_t)(1 + ix);
  uint32_t clo, chi;
  taps8_any(fx, clo, chi);
  uint32_t cpe[NP][5], cpo[NP][5];
#pragma unroll
  for (int m = 0; m < NP; m++) {
    const int qy = 2 * hy + (LS[m] - 1);
    const int iy = qy >> 2, fy = qy & 3;
    vpairs(fy, 1 + iy, cpe[m]);
    vpairs(fy, 2 + iy, cpo[m]);
  }
  uint32_t XQ[NP][UW][UJ];
#pragma unroll
  for (int x = 0; x < UW; x++) {
    launder(v);
    uint32_t HQ[RV / 2];
#pragma unroll
    for (int r = 0; r < RV; r += 2) {
      const int h0 = dot4(rbytes_d(v[r], x + 4, dlt), chi, dot4_k32(rbytes_d(v[r], x, dlt), clo));
      const int h1 = dot4(rbytes_d(v[r + 1], x + 4, dlt), chi, dot4_k32(rbytes_d(v[r + 1], x, dlt), clo));
      HQ[r / 2] = pack2(h0, h1);
    }
#pragma unroll
    for (int m = 0; m < NP; m++) {
      int vq[UH];   // second-stage sums (taps scaled by kVS)
#pragma unroll
      for (int y = 0; y < UH; y++) {
        const int m0 = (y & 1) ? (y - 1) / 2 : y / 2;
        int acc = dot2_k0(HQ[m0], (y & 1) ? cpo[m][0] : cpe[m][0]);
#pragma unroll
        for (int t = 1; t < 5; t++) acc = dot2(HQ[m0 + t], (y & 1) ? cpo[m][t] : cpe[m][t], acc);
        vq[y] = acc;
      }
#pragma unroll
      for (int jj = 0; jj < UJ; jj++) XQ[m][x][jj] = pk_sub(K.at(x, jj), pk_round2d(vq[2 * jj], vq[2 * jj + 1]));
    }
    __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure)
  }
#pragma unroll
  for (int m = 0; m < NP; m++) d[m] = unit_dist<UW, UH, T>(XQ[m], had);
}

// Quarter passes: pass PS covers column phase k = QP_K[PS] (dqx = k-1) and one or two row
// phases l (dqy = l-1); candidate (k1, l1) is the half best.  A phase with fraction 0 filters
// with {0,0,0,64,0,0,0,0}, which equals HM's copy / 1-D paths after rounding.
// QM 2: five passes, (k, l) = (0: 0,1) (0: 2) (1: 0,2) (2: 0,1) (2: 2); QM 1: eight, (k, l) for
// k, l in 0..2 without (1,1).
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_passes() { return QM == 2 ? 5 : 8; }
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_k(int ps) {
  return QM == 2 ? (ps < 2 ? 0 : (ps == 2 ? 1 : 2)) : (ps + (ps >= 4 ? 1 : 0)) / 3;
}
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_l0(int ps) {
  return QM == 2 ? ((ps == 1 || ps == 4) ? 2 : 0) : (ps + (ps >= 4 ? 1 : 0)) % 3;
}
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_l1(int ps) {
  return QM == 2 ? (ps == 0 ? 1 : (ps == 2 ? 2 : (ps == 3 ? 1 : -1))) : -1;
}
// Q9 index of pass ps's first / second candidate
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_idx0(int ps) {
  return q9_index(qp_k<QM>(ps) - 1, qp_l0<QM>(ps) - 1);
}
template <int QM> __host__ __device__ __forceinline__ constexpr int qp_idx1(int ps) {
  return qp_l1<QM>(ps) < 0 ? -1 : q9_index(qp_k<QM>(ps) - 1, qp_l1<QM>(ps) - 1);
}

template <int UW, int UH, int T, int QM, int PS>
__device__ __forceinline__ void qtr_pass(uint32_t (&v)[UH + 8][UW / 4 + 2], const KeySrc<UW, UH / 2>& K,
                                         const Metric& had, int hx, int hy, uint32_t (&d)[2]) {
  constexpr int RV = UH + 8, UJ = UH / 2;
  constexpr int k = qp_k<QM>(PS);
  constexpr int NP = qp_l1<QM>(PS) < 0 ? 1 : 2;
  const int LS[2] = {qp_l0<QM>(PS), qp_l1<QM>(PS) < 0 ? 0 : qp_l1<QM>(PS)};
  const int qx = 2 * hx + (k - 1);
  const int ix = qx >> 2, fx = qx & 3;
  const uint32_t dlt = (uint32_t)(1 + ix);
  uint32_t clo, chi;
  taps8_any(fx, clo, chi);
  uint32_t cpe[NP][5], cpo[NP][5];
#pragma unroll
  for (int m = 0; m < NP; m++) {
    const int qy = 2 * hy + (LS[m] - 1);
    const int iy = qy >> 2, fy = qy & 3;
    vpairs(fy, 1 + iy, cpe[m]);
    vpairs(fy, 2 + iy, cpo[m]);
  }
  uint32_t XQ[NP][UW][UJ];
#pragma unroll
  for (int x = 0; x < UW; x++) {
    launder(v);
    uint32_t HQ[RV / 2];
#pragma unroll
    for (int r = 0; r < RV; r += 2) {
      const int h0 = dot4(rbytes_d(v[r], x + 4, dlt), chi, dot4(rbytes_d(v[r], x, dlt), clo, 0));
      const int h1 = dot4(rbytes_d(v[r + 1], x + 4, dlt), chi, dot4(rbytes_d(v[r + 1], x, dlt), clo, 0));
      HQ[r / 2] = pack2(h0, h1);
    }
#pragma unroll
    for (int m = 0; m < NP; m++) {
      int vq[UH];
#pragma unroll
      for (int y = 0; y < UH; y++) {
        const int m0 = (y & 1) ? (y - 1) / 2 : y / 2;
        int acc = 2048 * kVS;
#pragma unroll
        for (int t = 0; t < 5; t++) acc = dot2(HQ[m0 + t], (y & 1) ? cpo[m][t] : cpe[m][t], acc);
        vq[y] = acc;
      }
#pragma unroll
      for (int jj = 0; jj < UJ; jj++) XQ[m][x][jj] = pk_sub(K.at(x, jj), pk_round2d(vq[2 * jj], vq[2 * jj + 1]));
    }
    __builtin_amdgcn_sched_barrier(0);   // one column at a time (register pressure)
  }
  d[0] = unit_dist<UW, UH, T>(XQ[0], had);
  d[1] = NP > 1 ? unit_dist<UW, UH, T>(XQ[NP - 1], had) : 0u;
}

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4a gu4;
typedef __attribute__((address_space(1))) const u32x3a gu3;
typedef __attribute__((address_space(1))) const u32x2a gu2;

// N dwords from byte address p, any alignment (gfx950 runs global memory in unaligned access
// mode; tools/probes/unaligned_probe.hip checks it on the box).
template <int N>
__device__ __forceinline__ void ld_bytes(const void* p, uint32_t (&o)[N]) {
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

// Rows y0 .. y0+R-1, 4N bytes from column x0 of a picture, as (sample - 128) bytes, with HM's
// padded-picture semantics (TComPicYuv::extendPicBorder): rows and columns clamped to the
// picture.  Away from the left / right edges each row is one unaligned load; near them each dword
// is read at the clamped run xa = clamp(x, 0, W-4) and v_perm picks the replicated bytes.
template <int R, int N>
__device__ __forceinline__ void load_window(const PicDesc& pic, int x0, int y0, uint32_t (&v)[R][N]) {
  // opaque origin: the row / column clamps are not shared across calls (hoisted out of a pass
  // loop they stay live, and spill, for the whole search)
  asm volatile("" : "+v"(x0), "+v"(y0));
  const bool inside = x0 >= 0 && x0 + 4 * N <= pic.width;
  if (inside) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int yy = clamp_i(y0 + r, 0, pic.height - 1);
      ld_bytes<N>(pic.luma + (size_t)yy * pic.stride + x0, v[r]);
      // row addresses four at a time: every load is still in flight before the first use, but
      // the scheduler does not keep R 64-bit addresses live at once
      if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    int xa[N];
    uint32_t sel[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
      xa[k] = clamp_i(x0 + 4 * k, 0, pic.width - 4);
      sel[k] = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) sel[k] |= (uint32_t)(clamp_i(x0 + 4 * k + i, 0, pic.width - 1) - xa[k]) << (8 * i);
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint8_t* row = pic.luma + (size_t)clamp_i(y0 + r, 0, pic.height - 1) * pic.stride;
#pragma unroll
      for (int k = 0; k < N; k++) {
        uint32_t t[1];
        ld_bytes<1>(row + xa[k], t);
        v[r][k] = __builtin_amdgcn_perm(0u, t[0], sel[k]);
      }
      if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int k = 0; k < N; k++) v[r][k] ^= 0x80808080u;
}

// Per-workgroup copies of the batch's picture and lambda tables (k_search_lane fills them once):
// every tile reads its PU's reference / original picture descriptor and motion lambda from LDS
// instead of a dependent global load before its window loads.
__shared__ PicDesc g_pics[FME_MAX_PICTURES];
// MV bits of one candidate: two exp-Golomb lengths of values below 2^18 (int16 MVs and predictors,
// cost scale <= 2), each at most 37.
constexpr int kCostBits = 80;
__shared__ uint32_t g_cost[FME_MAX_LAMBDAS][kCostBits];
// Record staging: each PU's 64-byte fme_result is assembled in LDS by the PU's first lane, then
// the wave writes the tile's records with four lanes per record, so every store instruction writes
// whole 64-byte lines (one lane per record wrote four separate 16-byte pieces: 256 bytes of
// WRITE_SIZE per job).
__shared__ uint4 g_rec[256 / 64][64][4];
__shared__ int32_t g_rec_jid[256 / 64][64];


// Global pointers typed as such (global_load / global_store, not flat).
typedef __attribute__((address_space(1))) const fme_job g_job;
typedef __attribute__((address_space(1))) const int32_t g_i32;
typedef __attribute__((address_space(1))) fme_result g_res;
typedef __attribute__((address_space(1))) const int16_t g_i16;
typedef __attribute__((address_space(1))) const uint8_t g_u8;
typedef __attribute__((address_space(1))) const uint32_t g_u32;


// =============================================================================================
// One lane: unit (ux, uy) of PU p of class (PW x PH), unit UW x UH (4x8, or 8x4 for the shapes
// whose height is not a multiple of 8).  PUs of more than 64 units (48x64, 64x48, 64x64) give a
// lane two units, one in the top and one in the bottom half of the PU: every candidate pass then
// runs once per half, with the other half's window and key re-loaded (L1 / L2 hits).
// =============================================================================================
template <int PW, int PH, int UW, int UH>
// (The signature matters to the register allocation of the call: with the kernel-argument
// reference `a` the callee saves no registers; with the same values as separate scalar arguments
// it saved and restored 114 callee-saved VGPRs per call.)
// (The lane comes from mbcnt and the wave index is an argument: a callee that reads no work-item
// id needs none passed, so the caller keeps no VGPR of it alive, and reloads none, around the call.)
__device__ FME_LANE_UNIT_ATTR void lane_unit(const BatchArgs& a, const fme_job* __restrict__ sjobs_,
                                             const int32_t* __restrict__ perm_, int cls_off, int cls_cnt,
                                             int wt, int wid) {
  g_job* const sjobs = (g_job*)sjobs_;
  g_i32* const perm = (g_i32*)perm_;
  g_res* const outp = (g_res*)a.res;
  g_i16* const keys = (g_i16*)a.keys;
  const int use_hadamard = a.use_hadamard, fen = a.fen;
  constexpr int T = ((PW % 8) == 0 && (PH % 8) == 0) ? 8 : 4;
  static_assert((T == 8 && UW == 4 && UH == 8) || (T == 4 && UW == 4 && UH == 4) || (T == 4 && UW * UH == 32),
                "4x8 units (a lane pair per 8x8 SATD tile) or 4x4 units (one 4x4 tile per lane)");
  constexpr bool k84 = UW == 8 && UH == 4 && !FME_LANE_PAIR84;
  constexpr int kQP = k84 ? 1 : FME_LANE_QPAIR, kHP = k84 ? 1 : FME_LANE_HPAIR;
  static_assert(PW % UW == 0 && PH % UH == 0, "units tile the PU");
  constexpr int UX = PW / UW, UY = PH / UH, NU = UX * UY;
  constexpr int UPL = NU > 64 ? 2 : 1;                // units per lane
  constexpr int UYH = UY / UPL, NUH = UX * UYH;       // unit rows / units per half
  static_assert(UPL == 1 || UY % 2 == 0, "halves of whole unit rows");
  constexpr int L = pow2_at_least(NUH);               // lanes of the PU's group (AMP: 6 -> 8, 24 -> 32, 48 -> 64)
  static_assert(L <= 64, "a PU's group fits one wave");
  static_assert(T == 4 || UX % 2 == 0, "an 8x8 tile's two units sit in lanes 2k, 2k+1");
  // the modified setDistParam's integer metric (TComRdCost.cpp:200-230): SAD for W in {12, 24, 48},
  // with xTZSearchHelp's FEN row subsampling (TEncSearch.cpp:1158-1164); SSE otherwise
  constexpr bool kSadEmi = PW == 12 || PW == 24 || PW == 48;
  constexpr int RV = UH + 8;                  // re-centred window rows (-4 .. UH+3)
  constexpr int NV = UW / 4 + 2;              // re-centred dwords per row (cols -4 .. UW+3)
  constexpr int UJ = UH / 2;                  // packed row pairs per column
  constexpr int EW = (UW + 2 + 3) / 4;        // EMI window dwords per row (cols -1 .. UW)
  constexpr int KW = UW / 2;                  // key dwords per row (bytes: UW / 4 used; int16 pairs: UW / 2)

  const int lane = (int)__lane_id();
  const int gl = wt * 64 + lane;               // wave tile wt: 64 lanes = 64 / L PUs
  int p = gl / L;
  const int u = gl - p * L;
  const bool active = p < cls_cnt;
  if (!active) p = cls_cnt - 1;              // duplicate work, no stores (keeps the group whole)
  const uint32_t live = u < NUH ? ~0u : 0u;  // padding lanes repeat the last unit, summed as 0
  const int uu = u < NUH ? u : NUH - 1;
  const int ux = uu % UX, uy = uu / UX;

  FME_STAMP(0);
  const int jid = perm[cls_off + p];
  fme_job j;
  {   // two 16-byte global loads (a struct copy through an address-space-1 pointer does not compile
      // in the host pass): the class-ordered copy, or (FME_SJOBS 0) the caller's job by its index
    g_job* const src = FME_SJOBS ? sjobs + cls_off + p : (g_job*)a.jobs + jid;
    const u32x4a q0 = *(gu4*)src, q1 = *(gu4*)((g_u8*)src + 16);
    uint32_t tmp[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    __builtin_memcpy(&j, tmp, sizeof(j));
  }
  // The reference's descriptor is read from LDS where a window is loaded (an opaque index keeps
  // the compiler from holding the 40-byte copy in registers, or scratch, across the passes).
  auto ref_pic = [&]() FME_AI -> PicDesc {
    int rid = j.ref_id;
    asm volatile("" : "+v"(rid));
    return g_pics[rid];
  };
  const uint32_t* const ml = g_cost[j.lambda_id];
  const Metric met = {use_hadamard && !(j.flags & FME_JOB_LOSSLESS), (lane & 1) ? 0xFFFFFFFFu : 0x00010001u,
                      (lane & 1) ? 0u : ~0u};
  const bool kbuf = j.key_offset >= 0;
  const int ox = (int)j.x + ux * UW, oy = (int)j.y + uy * UH;   // unit origin (top half)
  constexpr int kHalfRows = UYH * UH;                             // bottom half: oy + kHalfRows
  const int mvp_x = j.mvp_x, mvp_y = j.mvp_y;

  // key rows of half h, row-major: org bytes (s - 128) in kraw[r][0 .. UW/4) (uni-pred), or the
  // job's int16 key pairs (cols 2k, 2k+1) in kraw[r][0 .. UW/2)
  auto load_kraw = [&](int h, uint32_t (&kraw)[UH][KW]) FME_AI {
    int ky = oy + h * kHalfRows;
    asm volatile("" : "+v"(ky));   // not shared across calls (see load_window)
    if (!kbuf) {
      const PicDesc org = g_pics[j.org_id];
#pragma unroll
      for (int r = 0; r < UH; r++) {
        uint32_t t[UW / 4];
        ld_bytes<UW / 4>(org.luma + (size_t)(ky + r) * org.stride + ox, t);
#pragma unroll
        for (int k = 0; k < UW / 4; k++) kraw[r][k] = t[k] ^ 0x80808080u;
#pragma unroll
        for (int k = UW / 4; k < KW; k++) kraw[r][k] = 0;
      }
    } else {
      g_i16* kb = keys + (size_t)j.key_offset + (size_t)(ky - (int)j.y) * PW + ux * UW;
#pragma unroll
      for (int r = 0; r < UH; r++) ld_bytes<KW>((const void*)(kb + r * PW), kraw[r]);
    }
  };

  // one unit per lane: its key rows are loaded once, for the EMI step and the sub-pel passes
  uint32_t kraw0[UH][KW];
  if constexpr (UPL == 1) load_kraw(0, kraw0);
  FME_STAMP(1);

  // ---- 1. EMI square step -----------------------------------------------------------------------
  int mvx = j.mv_x, mvy = j.mv_y;
  int n_emi = 0;
  uint32_t cval = 0, emi[8];
#pragma unroll
  for (int k = 0; k < 8; k++) emi[k] = 0;
  // FME_JOB_NN_IN takes precedence over FME_JOB_EMI (fme.h: NN_IN means no EMI step), as in the
  // oracle (fme_oracle.c orc_refine), the harness and nn_pushes()
  if (j.flags & FME_JOB_NN_IN) {
    // the backups' input path: the integer search's square + ring already moved mv and pushed
    // the inputs (FME_TZ_RING); the job's row holds array_e[index_ref .. +7] and C
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
      // integer samples at rows -1 .. UH, cols -1 .. UW around the TZ MV (s - 128 bytes)
      uint32_t w[UH + 2][EW];
      load_window(ref_pic(), ox + mvx - 1, oy + h * kHalfRows + mvy - 1, w);
      int so2 = 0;   // SSE's sum of squared key samples
#pragma unroll
      for (int r = 0; r < UH; r++)
#pragma unroll
        for (int k = 0; k < UW / 4; k++) so2 = dot4(kraw[r][k], kraw[r][k], so2);
      // one position at a time, every array index a compile-time constant (a computed index
      // sends the accumulators to scratch)
#pragma unroll
      for (int pos = 0; pos < 9; pos++) {
        const int dx = emi_dx(pos), dy = emi_dy(pos);
        uint32_t e = 0;
        if constexpr (kSadEmi) {   // SAD of the (even, with FEN) rows, doubled when subsampled
          const bool sub = fen == 1 || fen == 3;   // and PH > 8: every 12/24/48-wide shape
#pragma unroll
          for (int r = 0; r < UH; r++) {
            if ((r & 1) && sub) continue;   // unit rows start on even PU rows
#pragma unroll
            for (int k = 0; k < UW / 4; k++) {
              const uint32_t pv = rbytes(w[r + 1 + dy], 1 + dx + 4 * k) ^ 0x80808080u;   // samples 0..255
              if (!kbuf) {
                e = __builtin_amdgcn_sad_u8(kraw[r][k] ^ 0x80808080u, pv, e);
              } else {   // int16 key: |key - pred| per sample
                const uint32_t d0 = pk_sub(kraw[r][2 * k], lo_pair(pv)), d1 = pk_sub(kraw[r][2 * k + 1], hi_pair(pv));
                e = udot2(pk_abs(d1), 0x00010001u, udot2(pk_abs(d0), 0x00010001u, e));
              }
            }
          }
        } else if (!kbuf) {   // SSE = So2 - 2 Sop + Spp on the s - 128 bytes
          int sop = 0, spp = 0;
#pragma unroll
          for (int r = 0; r < UH; r++)
#pragma unroll
            for (int k = 0; k < UW / 4; k++) {
              const uint32_t pv = rbytes(w[r + 1 + dy], 1 + dx + 4 * k);
              sop = dot4(kraw[r][k], pv, sop);
              spp = dot4(pv, pv, spp);
            }
          e = (uint32_t)(so2 - 2 * sop + spp);
        } else {   // int16 key: sum of (key - pred)^2
#pragma unroll
          for (int r = 0; r < UH; r++)
#pragma unroll
            for (int k = 0; k < UW / 4; k++) {
              const uint32_t x = rbytes(w[r + 1 + dy], 1 + dx + 4 * k) ^ 0x80808080u;   // samples 0..255
              const uint32_t d0 = pk_sub(kraw[r][2 * k], lo_pair(x)), d1 = pk_sub(kraw[r][2 * k + 1], hi_pair(x));
              e = (uint32_t)dot2(d1, d1, dot2(d0, d0, (int)e));
            }
        }
        e9[pos] += e;
      }
    }
    if constexpr (kSadEmi) {
      if (fen == 1 || fen == 3) {
#pragma unroll
        for (int q = 0; q < 9; q++) e9[q] <<= 1;
      }
    }
#pragma unroll
    for (int pos = 0; pos < 9; pos++) e9[pos] = group_sum<L>(e9[pos] & live);
    // decision (TEncSearch.cpp:1341-1376 visiting order and range checks, 1155-1188 update)
    const int sx = mvx, sy = mvy;
    uint32_t best = e9[0] + mv_cost(ml, mv_bits(sx, sy, 2, mvp_x, mvp_y));
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
        // emi[n_emi++] = d with a static register index
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (k == n_emi) emi[k] = d;
        n_emi++;
        if (d < best) {
          const uint32_t cst = mv_cost(ml, mv_bits(sx + dx, sy + dy, 2, mvp_x, mvp_y));
          const uint32_t dc = d + cst;
          if (dc < best) {
            best = dc;
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
  FME_STAMP(2);
  typedef __attribute__((address_space(1))) u32x4a gw4;
  if (u == 0) {   // bytes 16..63 of the record: cost, bits (NN tail), c, emi[8], n_emi
    g_rec[wid][lane][1] = make_uint4(0u, 0u, cval, emi[0]);
    g_rec[wid][lane][2] = make_uint4(emi[1], emi[2], emi[3], emi[4]);
    g_rec[wid][lane][3] = make_uint4(emi[5], emi[6], emi[7], (uint32_t)n_emi);
    g_rec_jid[wid][lane] = !active ? -1 : jid;   // destination record (call order)
  }


  // ---- the resident half: window rows -4..UH+3, cols -4..UW+3 around mv_int', and the key as
  // signed int16 (key - 128) pairs K[c][j] = (row 2j, row 2j+1) of column c ----------------------
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
        const uint32_t ko = sext_pair(kraw[2 * jj + 1][c >> 2], kraw[2 * jj][c >> 2], c & 3);
        const uint32_t hs = (c & 1) ? 0x07060302u : 0x05040100u;   // 16-bit half c&1 of each row
        const uint32_t kb = pk_sub(__builtin_amdgcn_perm(kraw[2 * jj + 1][c >> 1], kraw[2 * jj][c >> 1], hs), 0x00800080u);
        K.set(c, jj, kbuf ? kb : ko);
      }
  };
  load_half(0);
  FME_STAMP(3);
  int cur = 0;
  // One candidate pass over the PU: the resident half first, then (two units per lane) the other.
  auto over_halves = [&](auto&& pass, auto& d) FME_AI {
    pass(d);
    if constexpr (UPL == 2) {
      cur ^= 1;
      __builtin_amdgcn_sched_barrier(0);   // the other half's loads stay after this pass (one window live)
      launder(v);
      load_half(cur);
      __builtin_amdgcn_sched_barrier(0);
      std::remove_reference_t<decltype(d)> d2;
      pass(d2);
#pragma unroll
      for (int m = 0; m < (int)(sizeof(d) / sizeof(d[0])); m++) d[m] += d2[m];
    }
  };

  // ---- 2. half-pel stage (H9 order: (0,0),(0,-1),(0,1),(-1,0),(1,0),(-1,-1),(1,-1),(-1,1),(1,1)) ---
  // Candidates arrive out of H9 order: keep the first strict minimum in H9 order with an index
  // tie-break (d < best, or d == best at a lower index).
  uint32_t hbest = 0xFFFFFFFFu;
  int hbi = 9;
  {
    uint32_t d[3] = {0u, 0u, 0u};
    over_halves([&](uint32_t (&dd)[3]) FME_AI { half_center<UW, UH, T, kHP>(v, K, met, dd); }, d);
    take_half<L>(0, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(1, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(2, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
  }
  if constexpr (FME_LANE_SHARE) {
    uint32_t d[6];
    over_halves([&](uint32_t (&dd)[6]) FME_AI { half_sides<UW, UH, T>(v, K, met, dd); }, d);
    take_half<L>(3, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(5, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(7, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(4, d[3], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(6, d[4], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(8, d[5], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
  } else {
    uint32_t d[3];
    over_halves([&](uint32_t (&dd)[3]) FME_AI { half_side<UW, UH, T, 0, kHP>(v, K, met, dd); }, d);
    take_half<L>(3, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(5, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(7, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    over_halves([&](uint32_t (&dd)[3]) FME_AI { half_side<UW, UH, T, 1, kHP>(v, K, met, dd); }, d);
    take_half<L>(4, d[0], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(6, d[1], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
    take_half<L>(8, d[2], live, ml, mvx, mvy, mvp_x, mvp_y, hbest, hbi);
  }
  const int hx = h9_dx(hbi), hy = h9_dy(hbi);
  FME_STAMP(4);

  // ---- 3. quarter-pel stage: passes over column phases (Q9 candidate 0 = the half best) -------
  uint32_t qbest = hbest;
  int qbi = 0;
  auto qone = [&](auto ps_c) FME_AI {
    constexpr int ps = decltype(ps_c)::value;
    uint32_t d[2];
    over_halves([&](uint32_t (&dd)[2]) FME_AI { qtr_pass<UW, UH, T, kQP, ps>(v, K, met, hx, hy, dd); }, d);
    take_qtr<L>(qp_idx0<kQP>(ps), d[0], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
    if constexpr (qp_l1<kQP>(ps) >= 0)
      take_qtr<L>(qp_idx1<kQP>(ps), d[1], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
  };
  if constexpr (FME_LANE_SHARE) {
    auto qcol = [&](auto k_c) FME_AI {
      constexpr int kk = decltype(k_c)::value;
      uint32_t d[3];
      over_halves([&](uint32_t (&dd)[3]) FME_AI { qtr_col<UW, UH, T, kk>(v, K, met, hx, hy, dd); }, d);
      take_qtr<L>(q9_index(kk - 1, -1), d[0], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
      take_qtr<L>(q9_index(kk - 1, kk == 1 ? 1 : 0), d[1], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
      if constexpr (kk != 1) take_qtr<L>(q9_index(kk - 1, 1), d[2], live, ml, mvx, mvy, hx, hy, mvp_x, mvp_y, qbest, qbi);
    };
    static_for<0, 3>(qcol);
  } else {
    static_for<0, qp_passes<kQP>()>(qone);
  }
  const int bq = qbi;
  FME_STAMP(5);

  // ---- results: bytes 0..15 (mv_int, mv (NN tail), half, qtr, frac_cost) ------------------------
  const uint32_t r_mv = (uint32_t)(uint16_t)mvx | ((uint32_t)(uint16_t)mvy << 16);
  const uint32_t r_hq = (uint32_t)(uint8_t)hx | ((uint32_t)(uint8_t)hy << 8) | ((uint32_t)(uint8_t)q9_dx(bq) << 16) |
                        ((uint32_t)(uint8_t)q9_dy(bq) << 24);
  if (u == 0) g_rec[wid][lane][0] = make_uint4(r_mv, 0u, r_hq, qbest);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the tile's 64 / L records, four lanes per record (quarter = lane % 4): 16 records per store
  constexpr int NP = 64 / L;
#pragma unroll
  for (int s0 = 0; s0 < (NP * 4 + 63) / 64; s0++) {
    const int r = s0 * 16 + (lane >> 2);   // record of this lane's quarter
    if (r < NP) {
      const int src = r * L;              // the PU's first lane
      const int rj = g_rec_jid[wid][src];
      if (rj >= 0) {
        const uint4 q = g_rec[wid][src][lane & 3];
        u32x4a o;
        o.x = q.x; o.y = q.y; o.z = q.z; o.w = q.w;
        *(gw4*)(reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(outp + rj) + 16 * (lane & 3)) = o;
      }
    }
  }
#if FME_LANE_STAMPS
  FME_STAMP(6);
  if (lane == 0) {   // vector atomics into the debug buffer, one lane per wave
    constexpr int C = []() constexpr {
      for (int c = 0; c < kNumClasses; c++)
        if (kClassW[c] == PW && kClassH[c] == PH) return c;
      return 0;
    }();
    unsigned long long* d = g_lane_stamps[C];
    atomicAdd(d + 0, stamp_1 - stamp_0);
    atomicAdd(d + 1, stamp_2 - stamp_1);
    atomicAdd(d + 2, stamp_3 - stamp_2);
    atomicAdd(d + 3, stamp_4 - stamp_3);
    atomicAdd(d + 4, stamp_5 - stamp_4);
    atomicAdd(d + 5, stamp_6 - stamp_5);
    atomicAdd(d + 6, 1ull);
  }
#endif
}

// The XCD this wave runs on (HW_REG_XCC_ID, gfx940+: bits 3:0).
__device__ __forceinline__ int xcc_id() {
#if FME_XCD_SWIZZLE
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7;
#else
  return 0;
#endif
}

}  // namespace

// (class id, PU W, PU H, unit W, unit H) — fme_device.h class table; one kernel per unit
// shape, since a kernel's register allocation is the maximum over its cases.
// 4x8 units for every shape whose width is a multiple of 4 and height a multiple of 8 (an 8x8
// SATD tile is a lane pair; the 4x4-tiled 4x8 / 4x16 / 12x16 keep their two tiles in the lane),
// 4x4 units (one SATD tile each) for 8x4 / 16x4 / 16x12.  (4x4 units for 4x8-tiled shapes: about
// 18 % more instructions per PU, measured 0.924 -> 0.9xx ms; 8x4 units for the 8x4-like shapes gave
// wrong half / quarter results on ~15 % of their golden jobs and are not used)
#ifndef FME_LANE_4X8_UNITS44   // 4x8 PUs as two 4x4 units (a lane pair) instead of one lane each
#define FME_LANE_4X8_UNITS44 0
#endif
#if FME_LANE_4X8_UNITS44
#define FME_LANE48_CLASSES(X) X(3, 4, 16, 4, 8)
#define FME_LANE84_CLASSES(X) X(0, 4, 8, 4, 4) X(1, 8, 4, 4, 4) X(4, 16, 4, 4, 4)
#else
#define FME_LANE48_CLASSES(X) X(0, 4, 8, 4, 8) X(3, 4, 16, 4, 8)
#define FME_LANE84_CLASSES(X) X(1, 8, 4, 4, 4) X(4, 16, 4, 4, 4)
#endif
#define FME_LANE88_CLASSES(X)                                                                        \
  X(2, 8, 8, 4, 8) X(5, 8, 16, 4, 8) X(6, 16, 8, 4, 8) X(9, 16, 16, 4, 8) X(10, 8, 32, 4, 8)         \
  X(11, 32, 8, 4, 8) X(12, 16, 32, 4, 8) X(13, 32, 16, 4, 8) X(16, 32, 32, 4, 8) X(17, 16, 64, 4, 8) \
  X(18, 64, 16, 4, 8) X(19, 32, 64, 4, 8) X(20, 64, 32, 4, 8) X(23, 64, 64, 4, 8)
// the AMP shapes whose unit count is not a power of two: 12x16 (6 of 8 lanes), 16x12 in 4x4 units
// (12 of 16), 24x32 / 32x24 (24 of 32), 48x64 / 64x48 (two halves of 48 units, 48 of 64 lanes)
#define FME_LANE_AMP_CLASSES(X)                                                                      \
  X(7, 12, 16, 4, 8) X(8, 16, 12, 4, 4) X(14, 24, 32, 4, 8) X(15, 32, 24, 4, 8) X(21, 48, 64, 4, 8)   \
  X(22, 64, 48, 4, 8)
#ifndef FME_LANE_CLASSES   // (a subset may be given on the command line for register-usage probes)
#define FME_LANE_CLASSES(X) \
  FME_LANE48_CLASSES(X) FME_LANE84_CLASSES(X) FME_LANE88_CLASSES(X) FME_LANE_AMP_CLASSES(X)
#endif

// One kernel serves every lane class.  A workgroup claims four consecutive 64-lane wave tiles
// (one per wave; a tile holds 64 / L PUs of one class) per atomic from its XCD's queue
// (Schedule::xq: the XCD's contiguous eighth of every class's tiles = one spatial band of the
// CTU-ordered job stream, so each L2 sees one band, searched strip by strip with every class of a
// strip together, and the four waves of a CU search neighbouring PUs whose reference windows share
// L1 lines), then from the other XCDs' queues.  The next claim is issued before the current tiles
// are searched.  The grid is sized to fill the chip, not to the (device-computed) tile count, so
// the host never waits for the class histogram.
// Measured (1080p frame, tools/ab_bench.py): per-wave claims 1.48 ms, four tiles per workgroup
// 1.21 ms, eight 1.24, sixteen 1.29; without the XCD queues 1.25 (the per-wave claim form was
// kept as a build option until round 5 and removed unused).
#define FME_CASE(ID, PW_, PH_, UW_, UH_)                                                             \
  case ID:                                                                                           \
    lane_unit<PW_, PH_, UW_, UH_>(a, w.sjobs, w.perm, sc->class_off[ID], sc->class_cnt[ID], wt, wid); \
    break;
__global__ __launch_bounds__(kLaneNT) __attribute__((amdgpu_waves_per_eu(FME_LANE_WAVES)))
void k_search_lane(BatchArgs a, WorkBufs w) {
  constexpr int S = FME_LANE_SUBBANDS;
  const Schedule* __restrict__ sc = w.sched;
  int32_t* ctr = w.tile_ctr;
  __shared__ int32_t s_xq[8][S][kNumClasses + 1];
  {   // the batch's tables and the XCD queues, once per workgroup
    const uint32_t* ps = reinterpret_cast<const uint32_t*>(a.pics);
    uint32_t* pd = reinterpret_cast<uint32_t*>(g_pics);
    for (int i = threadIdx.x; i < (int)(sizeof(g_pics) / 4); i += kLaneNT) pd[i] = ps[i];
    for (int i = threadIdx.x; i < FME_MAX_LAMBDAS * kCostBits; i += kLaneNT)
      g_cost[i / kCostBits][i % kCostBits] = simd::mv_cost(a.mlambda[i / kCostBits], (uint32_t)(i % kCostBits));
    for (int i = threadIdx.x; i < 8 * S * (kNumClasses + 1); i += kLaneNT) (&s_xq[0][0][0])[i] = (&sc->xq[0][0][0])[i];
  }
  const int home = xcc_id(), wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  constexpr int kGroup = kLaneNT / 64;   // wave tiles per claim
  __shared__ int32_t claim[2];
  int x = home, tried = 0, par = 0;
  if (threadIdx.x == 0) claim[0] = atomicAdd(&ctr[x], 1);
  __syncthreads();
  int t = __builtin_amdgcn_readfirstlane(claim[0]);
  while (true) {
    const int len = s_xq[x][S - 1][kNumClasses];
    if (kGroup * t >= len) {   // queue drained: the next XCD's
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
      int q = 0, c = 0;   // band x S + q of the queue, class c inside it
      while (q < S - 1 && tw >= s_xq[x][q][kNumClasses]) q++;
      while (c < kNumClasses - 1 && tw >= s_xq[x][q][c + 1]) c++;
      const int ci = c;   // queue position -> class
      c = lane_class_at(ci);
      const int nt = sc->prefix[c + 1] - sc->prefix[c];
      const int lo = (int)(((long long)nt * (x * S + q)) / (8 * S));   // the band's first tile of class c
      // wave-uniform: kept in an SGPR, so no VGPR of it lives (and is spilled) across the call
      const int wt = __builtin_amdgcn_readfirstlane(lo + (tw - s_xq[x][q][ci]));
      switch (c) {
        FME_LANE_CLASSES(FME_CASE)
        default: break;
      }
    }
    par ^= 1;   // claim[par] is rewritten only after every wave has passed the barrier below
    if (threadIdx.x == 0) claim[par] = nxt;
    __syncthreads();
    t = __builtin_amdgcn_readfirstlane(claim[par]);
  }
  (void)wid;
}
#undef FME_CASE

// Lanes per PU of a lane-kernel class, 0 for classes the cooperative kernels serve.
int lane_lanes_per_pu(int cls) {
  switch (cls) {
#define FME_L(ID, PW_, PH_, UW_, UH_) \
  case ID: return pow2_at_least((PW_ / UW_) * (PH_ / UH_) > 64 ? (PW_ / UW_) * (PH_ / UH_) / 2 : (PW_ / UW_) * (PH_ / UH_));
    FME_LANE_CLASSES(FME_L)
#undef FME_L
    default: return 0;
  }
}

// Workgroups of the lane-kernel launch: at most the wave tiles n jobs could need (4 per
// workgroup), at most 4 per CU (the kernel holds 2; spare workgroups find the queues drained
// and exit).
static int lane_grid(int n, int reserve) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    cus = cu_count(dev);
  }
  int max_l = 0, classes = 0;
  for (int c = 0; c < kNumClasses; c++)
    if (lane_lanes_per_pu(c)) {
      max_l = std::max(max_l, lane_lanes_per_pu(c));
      classes++;
    }
  const long long waves = ((long long)n * max_l + 63) / 64 + classes;
  // reserve > 0: exactly the resident workgroups less `reserve` (spare workgroups beyond the
  // resident ones would take the slots left free as soon as they open)
  const long long cap = reserve > 0 ? std::max(1LL, (long long)FME_LANE_WAVES * cus - reserve) : 4LL * cus;
  return (int)std::min<long long>((waves + kLaneNT / 64 - 1) / (kLaneNT / 64), cap);
}

#if FME_LANE_STAMPS
// The diagnostic build's per-(class, phase) cycle sums (kNumClasses x 8 words); reset clears them.
extern "C" int fme_debug_lane_stamps(unsigned long long* out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lane_stamps), sizeof(g_lane_stamps)) != hipSuccess) return -2;
  if (reset) {
    static const unsigned long long zero[kNumClasses][8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lane_stamps), zero, sizeof(zero)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

hipError_t launch_search_lane(const BatchArgs& a, const WorkBufs& w, int reserve, hipStream_t s) {
  const int blocks = lane_grid(a.n, reserve);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_search_lane, dim3(blocks), dim3(kLaneNT), 0, s, a, w);
  return hipGetLastError();
}

}  // namespace fme
