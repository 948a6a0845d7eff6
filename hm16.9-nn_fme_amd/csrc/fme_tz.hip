// fme_tz.hip — integer motion estimation on gfx950.
//
// xMotionEstimation's integer search (TEncSearch.cpp:4504-4527):
//   uni-pred  xPatternSearchFast -> xTZSearch (4737-5036) with the shipped settings: FastSearch 1
//             (diamond, not extended), FastMEAssumingSmootherMV (first search stops 3 rounds after
//             the best), raster step 5, star refinement; up to, not including, the EMI square step
//             (that is the first step of the sub-pel kernels);
//   bi-pred   xPatternSearch (4627-4680): every point of the range in raster order.
// Helpers restated: xTZSearchHelp's normal branch (1078-1188), xTZ8PointDiamondSearch (1379-1589),
// xTZ2PointSearch (1191-1322), xSetSearchRange (4602-4624), TComDataCU::clipMv
// (TComDataCU.cpp:2773-2786), TComMv::divideByPowerOf2 (TComMv.h:122-130).
//
// Mapping: one wave per PU (k_tz_wave; tz_wave below): the PU's units (8x8, 8x4 or 4x8; the group
// of L lanes padded to a power of two) sit in consecutive lanes, and the wave's 64 / L groups
// evaluate the candidates of one reference list (a diamond ring, the raster, ...) together.
// Metric (the NN_FME integer-ME setDistParam, TComRdCost.cpp:200-230): SSE for widths 4..64, SAD
// for 12/24/48 with the FEN even-row subsampling when H > 8; uni-pred keys as (s - 128) bytes
// (SSE = Sk2 - 2 Sks + Sss with v_dot4_i32_i8, SAD with v_sad_u8), bi-pred keys (2 org - pred,
// int16) as packed pairs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "fme_device.h"
#include "fme_simd.h"

// 1: a diagnostic build (make variant NAME=tzcount DEFS=-DFME_TZ_COUNT=1, tools/tz_counts.py) that
// counts, per unit-shape kernel, the candidate windows read from the staged LDS tile and from global
// memory (g_tz_count, read by fme_debug_tz_counts).  Never the product build.
#ifndef FME_TZ_COUNT
#define FME_TZ_COUNT 0
#endif

namespace fme {
#if FME_TZ_COUNT
__device__ unsigned long long g_tz_count[3][2];   // [kernel 4x8 / 8x4 / 8x8 units][LDS tile, global]
#endif
namespace {
using namespace simd;

#ifndef FME_TZ_NT   // threads per workgroup of the bulk search (one wave per PU)
#define FME_TZ_NT 256
#endif
constexpr int kTzNT = FME_TZ_NT;
#define FME_AI __attribute__((always_inline))

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// Sum over the L lanes of a group (L a power of two <= 64, uniform over the workgroup).
__device__ __forceinline__ uint32_t group_sum(uint32_t v, int L) {
  if (L >= 2) v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
  if (L >= 4) v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
  if (L >= 8) v += dpp<0x141>(v);   // row_half_mirror
  if (L >= 16) v += dpp<0x140>(v);  // row_mirror
  if (L >= 32) v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
  if (L >= 64) v += (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}

__device__ __forceinline__ int round4(int v) { return (v + 2) >> 2; }   // divideByPowerOf2(2)

__device__ __forceinline__ void clip_qpel(int& x, int& y, int pw, int ph, int cu_x, int cu_y) {
  x = min((pw + 8 - cu_x - 1) << 2, max((-64 - 8 - cu_x + 1) * 4, x));
  y = min((ph + 8 - cu_y - 1) << 2, max((-64 - 8 - cu_y + 1) * 4, y));
}

struct Range {
  int l, r, t, b;
};


struct Tz {
  // IntTZSearchStruct
  uint32_t best_sad;
  int bx, by, bdist, bround, pnr;
  int ox, oy;           // origin of the running diamond / two-point / square search
  int dist, k, opnr;
  Range R, RR;          // search range, raster range
  int range;            // m_iSearchRange
  bool corners;         // bCheckCornersAtDist1 of the running diamond (FastSearch 3: first search, star)
};

// xTZ8PointSquareSearch (TEncSearch.cpp:1324-1377) at distance 1: point k of (1 2 3 / 4 . 5 / 6 7 8) in
// call order with the reference's range checks (the middle column is only checked vertically).
__device__ __forceinline__ bool square_point(const Tz& s, int k, bool& ok, int& x, int& y) {
  if (k >= 8) return false;
  const int dx = (k == 0 || k == 3 || k == 5) ? -1 : ((k == 1 || k == 6) ? 0 : 1);
  const int dy = k < 3 ? -1 : (k < 5 ? 0 : 1);
  x = s.ox + dx;
  y = s.oy + dy;
  ok = (dy < 0 ? y >= s.R.t : true) && (dy > 0 ? y <= s.R.b : true) && (dx < 0 ? x >= s.R.l : true) &&
       (dx > 0 ? x <= s.R.r : true);
  return true;
}

// Point i of the backups' final pair of squares around (ox, oy): i < 8: xTZ8PointSquareSearch at
// distance 1 (square_point); i = 8..23: xTZ8PointSquareSearch2 at distance 2 (Backups/4:876-965),
// 16 points in its call order with its range checks, which test the x -/+ 1 points of the top and
// bottom rows against the left / right bound of distance 2.
__device__ __forceinline__ void ring_square_point(const Tz& s, int i, bool& ok, int& x, int& y) {
  if (i < 8) {
    square_point(s, i, ok, x, y);
    return;
  }
  // per ring point: dx, dy in -2..2 (stored +2), and which bounds it checks: bit 0 top, 1 bottom,
  // 2 left (x - 2 >= l), 3 right (x + 2 <= r)
  const int k = i - 8;
  // 4-bit fields per point k (dx + 2, dy + 2, checks), packed so a runtime k needs no table in memory
  const uint64_t kDx = 0x4321040404043210ull, kDy = 0x4444433221100000ull, kChk = 0xaa26684848499155ull;
  const int dxk = (int)((kDx >> (4 * k)) & 15), dyk = (int)((kDy >> (4 * k)) & 15);
  x = s.ox + dxk - 2;
  y = s.oy + dyk - 2;
  const int c = (int)((kChk >> (4 * k)) & 15);
  ok = (!(c & 1) || s.oy - 2 >= s.R.t) && (!(c & 2) || s.oy + 2 <= s.R.b) && (!(c & 4) || s.ox - 2 >= s.R.l) &&
       (!(c & 8) || s.ox + 2 <= s.R.r);
}

// Point k of xTZ8PointDiamondSearch(origin, dist) in call order, with the range check the
// reference applies before testing it (the "inside" fast path tests the same points in the same
// order, and every per-point check holds there).  Returns false past the last point.
__device__ __forceinline__ bool diamond_point(const Tz& s, int k, bool& ok, int& x, int& y, int& pnr, int& pd) {
  const int d = s.dist, ox = s.ox, oy = s.oy;
  const Range& R = s.R;
  if (d == 1) {
    if (s.corners) {   // bCheckCornersAtDist1 (TEncSearch.cpp:1404-1451): the square's 8 points, its checks
      pd = 1;
      pnr = k + 1;
      return square_point(s, k, ok, x, y);
    }
    if (k >= 4) return false;
    const int dx = k == 1 ? -1 : (k == 2 ? 1 : 0), dy = k == 0 ? -1 : (k == 3 ? 1 : 0);
    x = ox + dx;
    y = oy + dy;
    pnr = k == 0 ? 2 : (k == 1 ? 4 : (k == 2 ? 5 : 7));
    pd = 1;
    ok = (dy < 0 ? y >= R.t : true) && (dy > 0 ? y <= R.b : true) && (dx < 0 ? x >= R.l : true) &&
         (dx > 0 ? x <= R.r : true);
    return true;
  }
  if (d <= 8) {
    if (k >= 8) return false;
    const int h = d >> 1;
    // 2:(0,-d) 1:(-h,-h) 3:(h,-h) 4:(-d,0) 5:(d,0) 6:(-h,h) 8:(h,h) 7:(0,d)
    const int dx = k == 0 || k == 7 ? 0 : (k == 1 || k == 5 ? -h : (k == 2 || k == 6 ? h : (k == 3 ? -d : d)));
    const int dy = k == 0 ? -d : (k == 7 ? d : (k == 1 || k == 2 ? -h : (k == 5 || k == 6 ? h : 0)));
    const int nr[8] = {2, 1, 3, 4, 5, 6, 8, 7};
    pnr = nr[k];
    pd = (k == 1 || k == 2 || k == 5 || k == 6) ? h : d;
    x = ox + dx;
    y = oy + dy;
    ok = (dy < 0 ? y >= R.t : true) && (dy > 0 ? y <= R.b : true) && (dx < 0 ? x >= R.l : true) &&
         (dx > 0 ? x <= R.r : true);
    return true;
  }
  if (k >= 16) return false;
  pnr = 0;
  pd = d;
  if (k < 4) {
    const int dx = k == 1 ? -d : (k == 2 ? d : 0), dy = k == 0 ? -d : (k == 3 ? d : 0);
    x = ox + dx;
    y = oy + dy;
    ok = (dy < 0 ? y >= R.t : true) && (dy > 0 ? y <= R.b : true) && (dx < 0 ? x >= R.l : true) &&
         (dx > 0 ? x <= R.r : true);
    return true;
  }
  const int idx = 1 + ((k - 4) >> 2), m = (k - 4) & 3, q = (d >> 2) * idx;
  const int yt = oy - d + q, yb = oy + d - q, xl = ox - q, xr = ox + q;
  x = (m & 1) ? xr : xl;
  y = (m & 2) ? yb : yt;
  ok = ((m & 2) ? yb <= R.b : yt >= R.t) && ((m & 1) ? xr <= R.r : xl >= R.l);
  return true;
}

// xTZ2PointSearch: the two neighbours of a distance-1 best the diamond did not test.
__device__ __forceinline__ bool two_point(const Tz& s, int k, bool& ok, int& x, int& y) {
  if (k >= 2 || s.opnr < 1 || s.opnr > 8) return false;
  // per point_nr: (dx0, dy0, dx1, dy1), 2-bit codes 0 -> 0, 1 -> -1, 2 -> +1
  const uint32_t tab[9] = {0u, 0x41u, 0x65u, 0x24u, 0x59u, 0xa6u, 0x81u, 0xa9u, 0x82u};
  const uint32_t c = (tab[s.opnr] >> (4 * k)) & 0xFu;
  const int dx = dec(c & 3u), dy = dec(c >> 2);
  x = s.ox + dx;
  y = s.oy + dy;
  ok = (dx < 0 ? x >= s.R.l : true) && (dx > 0 ? x <= s.R.r : true) && (dy < 0 ? y >= s.R.t : true) &&
       (dy > 0 ? y <= s.R.b : true);
  return true;
}

__device__ __forceinline__ bool diamond_has_more(const Tz& s) {
  bool ok;
  int x, y, pnr, pd;
  for (int j = s.k; diamond_point(s, j, ok, x, y, pnr, pd); j++)
    if (ok) return true;
  return false;
}
__device__ __forceinline__ bool two_point_has_more(const Tz& s) {
  bool ok;
  int x, y;
  for (int j = s.k; two_point(s, j, ok, x, y); j++)
    if (ok) return true;
  return false;
}


// The staged bulk search (k_tz_staged): a workgroup takes the PUs of one (unit-shape kernel,
// reference picture, CTU) group and first copies the reference area their searches read into LDS:
// kTileH rows of kTileWD dwords around the CTU displaced by the first PU's start MV, kTileM samples
// of margin on each side (the search range, 64, plus slack for the other PUs' predictors), with the
// padded-picture semantics of the global loads (rows and columns clamped).  A candidate window that
// lies inside the tile is read from LDS, any other from global memory, so the results do not
// depend on the staging.
#ifndef FME_TZS_MARGIN
#define FME_TZS_MARGIN 72
#endif
constexpr int kTileM = FME_TZS_MARGIN;
constexpr int kTileWD = (64 + 2 * kTileM + 3 + 8 + 3) / 4;   // dwords per row (x0 aligned down to 4)
constexpr int kTileH = 64 + 2 * kTileM;
struct TileRef {
  const uint32_t* lds;   // null: no staged tile
  int x0, y0;            // picture coordinates of tile dword 0 of row 0 (x0 a multiple of 4; 10-bit: of 2)
};
// Bit depth 10: the tile holds sample pairs (twice the bytes per sample), so its margin is smaller
// (two 67 KB tiles per CU); windows outside it are read from global memory as before.
#ifndef FME_TZS_MARGIN10
#define FME_TZS_MARGIN10 56
#endif
constexpr int kTileM10 = FME_TZS_MARGIN10;
constexpr int kTileWD10 = (64 + 2 * kTileM10 + 1 + 10 + 1) / 2;   // dwords (sample pairs) per row (x0 even)
constexpr int kTileH10 = 64 + 2 * kTileM10;

// Reference window of one unit at displacement (bx, by) from its origin: UH rows (FEN: even rows
// only) of ND dwords from the aligned column, and the byte shift s0 of the first sample.
template <int UW, int UH>
__device__ __forceinline__ void load_window(uint32_t (&w)[UH][UW / 4 + 1], uint32_t& s0, const PicDesc& ref, int bx,
                                            int by, bool sub, const TileRef& t) {
  constexpr int ND = UW / 4 + 1;
  const int xa = bx & ~3;
  s0 = (uint32_t)(bx - xa);
  const bool in_tile = t.lds && xa >= t.x0 && xa + 4 * ND <= t.x0 + 4 * kTileWD && by >= t.y0 && by + UH <= t.y0 + kTileH;
#if FME_TZ_COUNT
  if (t.lds) {   // this call's lanes, by where their window comes from (one atomic per wave and kind)
    const uint64_t in = __ballot(in_tile), all = __ballot(1);
    if ((threadIdx.x & 63) == (uint32_t)__builtin_ctzll(all)) {
      constexpr int kid = UW == 4 ? 0 : (UH == 4 ? 1 : 2);
      atomicAdd(&g_tz_count[kid][0], (unsigned long long)__builtin_popcountll(in));
      atomicAdd(&g_tz_count[kid][1], (unsigned long long)__builtin_popcountll(all & ~in));
    }
  }
#endif
  if (in_tile) {
    const uint32_t* p = t.lds + (by - t.y0) * kTileWD + ((xa - t.x0) >> 2);
#pragma unroll
    for (int r = 0; r < UH; r++) {
      if (sub && (r & 1)) continue;
#pragma unroll
      for (int q = 0; q < ND; q++) w[r][q] = p[r * kTileWD + q];
    }
    return;
  }
  const bool inside = xa >= 0 && xa + 4 * ND <= ref.width;
#pragma unroll
  for (int r = 0; r < UH; r++) {
    if (sub && (r & 1)) continue;   // FEN: even rows of the PU (UH is even)
    const uint8_t* row = ref.luma + (size_t)clamp_i(by + r, 0, ref.height - 1) * ref.stride;
    if (inside) {   // one vector load per row (dwordx2 / dwordx3): a third of the L1 tag lookups
      typedef uint32_t vec_t __attribute__((ext_vector_type(ND), aligned(4)));
      const vec_t v = *(__attribute__((address_space(1))) const vec_t*)(row + xa);
#pragma unroll
      for (int q = 0; q < ND; q++) w[r][q] = v[q];
    } else {
#pragma unroll
      for (int q = 0; q < ND; q++) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) v |= gld8(row + clamp_i(xa + 4 * q + k, 0, ref.width - 1)) << (8 * k);
        w[r][q] = v;
      }
    }
  }
}

// One unit's share of the distortion (TComRdCost metric of the integer search) for a window.
template <int UW, int UH, int KW>
__device__ __forceinline__ uint32_t unit_part(const uint32_t (&w)[UH][UW / 4 + 1], uint32_t s0,
                                              const uint32_t (&kk)[UH][KW], int sk2, bool kbuf,
                                              bool sad_metric, bool sub) {
  int sop = 0, spp = 0;
  uint32_t acc = 0;
#pragma unroll
  for (int r = 0; r < UH; r++) {
    if (sub && (r & 1)) continue;
#pragma unroll
    for (int c = 0; c < UW / 4; c++) {
      const uint32_t pv = __builtin_amdgcn_alignbyte(w[r][c + 1], w[r][c], s0);   // reference bytes
      if (!kbuf) {
        if (sad_metric) {
          acc = __builtin_amdgcn_sad_u8(pv, kk[r][c], acc);
        } else {
          const uint32_t ps = pv ^ 0x80808080u;
          sop = dot4(kk[r][c] ^ 0x80808080u, ps, sop);
          spp = dot4(ps, ps, spp);
        }
      } else if constexpr (KW == UW / 2) {
        const uint32_t d0 = pk_sub(kk[r][2 * c], lo_pair(pv));
        const uint32_t d1 = pk_sub(kk[r][2 * c + 1], hi_pair(pv));
        if (sad_metric) {
          acc = udot2(pk_abs(d0), 0x00010001u, udot2(pk_abs(d1), 0x00010001u, acc));
        } else {
          acc = (uint32_t)dot2(d1, d1, dot2(d0, d0, (int)acc));
        }
      }
    }
  }
  uint32_t part = (!kbuf && !sad_metric) ? (uint32_t)(sk2 - 2 * sop + spp) : acc;
  if (sub) part <<= 1;
  return part;
}

// ---- bit depth 10 (the main10 configurations, InternalBitDepth 10) --------------------------------
// uint16 planes (strides in samples).  A unit's window row is UW / 2 + 1 dwords of sample pairs from
// the even column at or left of the candidate; s0 = 1 when the candidate column is odd.
template <int UW, int UH>
__device__ __forceinline__ void load_window10(uint32_t (&w)[UH][UW / 2 + 1], uint32_t& s0, const PicDesc& ref,
                                              int bx, int by, bool sub, const TileRef& t) {
  constexpr int ND = UW / 2 + 1;
  const int xa = bx & ~1;
  s0 = (uint32_t)(bx - xa);
  if (t.lds && xa >= t.x0 && xa + 2 * ND <= t.x0 + 2 * kTileWD10 && by >= t.y0 && by + UH <= t.y0 + kTileH10) {
    const uint32_t* p = t.lds + (by - t.y0) * kTileWD10 + ((xa - t.x0) >> 1);
#pragma unroll
    for (int r = 0; r < UH; r++) {
      if (sub && (r & 1)) continue;
#pragma unroll
      for (int q = 0; q < ND; q++) w[r][q] = p[r * kTileWD10 + q];
    }
    return;
  }
  const uint16_t* luma = reinterpret_cast<const uint16_t*>(ref.luma);
  const bool inside = xa >= 0 && xa + 2 * ND <= ref.width;
#pragma unroll
  for (int r = 0; r < UH; r++) {
    if (sub && (r & 1)) continue;   // FEN: even rows of the PU
    const uint16_t* row = luma + (size_t)clamp_i(by + r, 0, ref.height - 1) * ref.stride;
    if (inside) {   // one vector load per row (dwordx3, or x4 + x1), as the 8-bit windows
      typedef uint32_t vec_t __attribute__((ext_vector_type(ND), aligned(4)));
      const vec_t v = *(__attribute__((address_space(1))) const vec_t*)(row + xa);
#pragma unroll
      for (int q = 0; q < ND; q++) w[r][q] = v[q];
    } else {   // the padded picture: columns clamped (TComPicYuv::extendPicBorder)
      typedef __attribute__((address_space(1))) const uint16_t gu16c;
#pragma unroll
      for (int q = 0; q < ND; q++) {
        const uint32_t a = *(gu16c*)(row + clamp_i(xa + 2 * q, 0, ref.width - 1));
        const uint32_t b = *(gu16c*)(row + clamp_i(xa + 2 * q + 1, 0, ref.width - 1));
        w[r][q] = a | (b << 16);
      }
    }
  }
}

// One unit's share of the bit-depth-10 distortion: SSE sums (d * d) >> 4 per sample
// (xGetSSE, TComRdCost.cpp:875-1130, DISTORTION_PRECISION_ADJUSTMENT(2 (bitDepth - 8))) as
// (sum d^2 - sum (d^2 mod 16)) >> 4, with d^2 mod 16 = ((d & 7)^2) & 15; SAD returns the raw sum
// (<< 1 with FEN subsampling), the block's >> 2 (xGetSAD12/24/48: uiSum >> (bitDepth - 8)) comes
// after the group sum.  kk: the key as sample pairs (org samples, or the bi-pred int16 key).
template <int UW, int UH>
__device__ __forceinline__ uint32_t unit_part10(const uint32_t (&w)[UH][UW / 2 + 1], uint32_t s0,
                                                const uint32_t (&kk)[UH][UW / 2], bool sad_metric, bool sub) {
  int sq = 0;
  uint32_t lo = 0, acc = 0;
#pragma unroll
  for (int r = 0; r < UH; r++) {
    if (sub && (r & 1)) continue;
#pragma unroll
    for (int c = 0; c < UW / 2; c++) {
      const uint32_t pv = s0 ? __builtin_amdgcn_alignbyte(w[r][c + 1], w[r][c], 2u) : w[r][c];
      const uint32_t dd = pk_sub(kk[r][c], pv);
      if (sad_metric) {
        acc = udot2(pk_abs(dd), 0x00010001u, acc);
      } else {
        sq = dot2(dd, dd, sq);
        // d^2 mod 16 by d & 7 (0 1 4 9 0 9 4 1) from a byte table: one v_and_or makes the v_perm
        // selector (byte 0x0C selects zero), the perm gives the pair of residues as u16 halves
        const uint32_t sel = (dd & 0x00070007u) | 0x0C000C00u;
        lo = udot2(__builtin_amdgcn_perm(0x01040900u, 0x09040100u, sel), 0x00010001u, lo);
      }
    }
  }
  if (sad_metric) return sub ? acc << 1 : acc;
  return ((uint32_t)sq - lo) >> 4;
}

// ---- wave-uniform search: one wave per PU ------------------------------------------------------
// The reference's xTZSearch is a short sequence of candidate LISTS whose points do not depend on
// each other: the three start points, the first search's diamond rings (dist 1, 2, 4, ... around
// one origin), the two-point pair, the raster, each star round's rings, the EMI square.  A wave
// owns one PU; its G = 64 / L lane groups evaluate G points of a list at a time (L lanes = the
// PU's units), and xTZSearchHelp's in-order updates become a (cost, call index) minimum: in-order
// strict updates keep the first minimum below the running best.  The first search's stop rule
// (3 rings without a new best) needs per-ring minima, so its rings sit in 16-slot segments and are
// decided one by one as their chunk completes (later rings are not evaluated once it stops).
// Every branch is wave-uniform: no lane idles while another lane's search runs on.
//
// Ring slot 16 r + k = point k of xTZ8PointDiamondSearch(origin, 1 << r) (diamond_point order).
// Minimum over lanes l ^ off for off = L, 2L, .. < lim (lanes of one group hold the same key): DPP
// row permutations up to 8, the swizzle for 16, a bpermute only for 32 (a chain of six 64-bit
// bpermutes cost ~0.3 us per candidate chunk of a lone chain wave).
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_min_from(uint64_t key, int L, int lim) {
  auto mn = [](uint64_t a, uint64_t b) { return b < a ? b : a; };
  if (L <= 1 && 1 < lim) key = mn(key, dpp64<0xB1>(key));    // quad_perm [1,0,3,2]
  if (L <= 2 && 2 < lim) key = mn(key, dpp64<0x4E>(key));    // quad_perm [2,3,0,1]
  if (L <= 4 && 4 < lim) key = mn(key, dpp64<0x141>(key));   // row_half_mirror
  if (L <= 8 && 8 < lim) key = mn(key, dpp64<0x140>(key));   // row_mirror
  if (L <= 16 && 16 < lim) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)key, 0x401F);   // lane ^ 16
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(key >> 32), 0x401F);
    key = mn(key, ((uint64_t)hi << 32) | lo);
  }
  if (L <= 32 && 32 < lim) key = mn(key, (uint64_t)__shfl_xor((unsigned long long)key, 32, 64));
  return key;
}

// NW waves of one workgroup on one PU (the producer's chain levels: few jobs, latency-bound): the
// groups of all waves share each list; wave minima meet in LDS.
template <int NW>
__device__ __forceinline__ uint64_t block_min(uint64_t key) {
  if constexpr (NW == 1) {
    return key;
  } else {
    __shared__ uint64_t s_key[NW];
    if ((threadIdx.x & 63) == 0) s_key[threadIdx.x >> 6] = key;
    __syncthreads();
    uint64_t m = s_key[0];
#pragma unroll
    for (int w = 1; w < NW; w++) m = s_key[w] < m ? s_key[w] : m;
    __syncthreads();
    return m;
  }
}

// KB: -1 any job; 0 the uni-pred form (no job of the launch reads a key block: the key rows are
// UW / 4 dwords of bytes, half the registers of the int16 form)
// BD: the luma bit depth (8, or 10: uint16 planes, the key as sample pairs, no staged tile).
template <int UW, int UH, int NW = 1, int KB = -1, int BD = 8>
__device__ __forceinline__ void tz_wave(const TzArgs& ta, int jid, const fme_job& j, int PW, int PH, int pred_x,
                                        int pred_y, const TileRef& tile = TileRef{nullptr, 0, 0}) {
  const BatchArgs& a = ta.a;
  const int lane = (int)threadIdx.x & 63, wid = NW == 1 ? 0 : (int)threadIdx.x >> 6;
  const int UX = PW / UW, LR = UX * (PH / UH);
  int L = 1;
  while (L < LR) L <<= 1;
  const int G = NW * (64 / L), g = wid * (64 / L) + lane / L, u = lane % L;
  const bool real = u < LR;
  const int uu = real ? u : 0;
  const int ux = uu % UX, uy = uu / UX;
  const fme_tz_ext e = tz_ext_at(ta, jid);
  const PicDesc ref = a.pics[j.ref_id];
  const double ml = a.mlambda[j.lambda_id];
  const bool kbuf = KB != 0 && j.key_offset >= 0;
  const bool sad_metric = PW == 12 || PW == 24 || PW == 48;
  const bool sub = sad_metric && (a.fen == 1 || a.fen == 3) && PH > 8;
  const int ox = (int)j.x + ux * UW, oy = (int)j.y + uy * UH;
  constexpr int ND = UW / 4 + 1;

  constexpr int KW = (KB == 0 && BD == 8) ? UW / 4 : UW / 2;   // key dwords per row
  uint32_t kk[UH][KW];
  int sk2 = 0;
  if (BD != 8 && !kbuf) {   // 10-bit org samples as pairs
    const PicDesc org = a.pics[j.org_id];
    const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
#pragma unroll
    for (int r = 0; r < UH; r++)
#pragma unroll
      for (int c = 0; c < KW; c++) kk[r][c] = gld32(ol + (size_t)(oy + r) * org.stride + ox + 2 * c);
  } else if (!kbuf) {
    const PicDesc org = a.pics[j.org_id];
#pragma unroll
    for (int r = 0; r < UH; r++) {
#pragma unroll
      for (int c = 0; c < UW / 4; c++) {
        const uint32_t v = gld32(org.luma + (size_t)(oy + r) * org.stride + ox + 4 * c);
        kk[r][c] = v;
        sk2 = dot4(v ^ 0x80808080u, v ^ 0x80808080u, sk2);
      }
#pragma unroll
      for (int c = UW / 4; c < KW; c++) kk[r][c] = 0;
    }
  } else if constexpr (KW == UW / 2) {   // bi-pred keys (int16)
    const int16_t* kb = a.keys + (size_t)j.key_offset + (size_t)(uy * UH) * PW + ux * UW;
#pragma unroll
    for (int r = 0; r < UH; r++)
#pragma unroll
      for (int c = 0; c < UW / 2; c++)
        kk[r][c] = (uint32_t)(uint16_t)kb[r * PW + 2 * c] | ((uint32_t)(uint16_t)kb[r * PW + 2 * c + 1] << 16);
  }

  // The backups' input path (FME_TZ_RING, Backups/4 and Backups/15 xTZSearch): every distortion
  // xTZSearchHelp computes is pushed into array_e (Backups/4:659, 677); C = the least of the pushes
  // before the final square (:4343-4348), and the square + ring pushes after it are the NN inputs.
  // The bulk kernel only (one wave per PU: the slots are gathered with in-wave shuffles).
  const bool ring = NW == 1 && ta.nn_in != nullptr && (e.flags & FME_TZ_RING) && !(j.flags & FME_JOB_BIPRED);
  uint32_t cmin = 0xFFFFFFFFu;   // least distortion pushed so far (wave-uniform)

  // distortion + MV cost of this group's candidate (all lanes of the group get it); ~0: not tested.
  // dist: the distortion alone (~0 when not tested).
  auto cost_at = [&](int x, int y, bool v, uint32_t& dist) FME_AI -> uint32_t {
    uint32_t part = 0;
    if (v && real) {
      if constexpr (BD == 8) {
        uint32_t w[UH][ND];
        uint32_t s0;
        load_window<UW, UH>(w, s0, ref, ox + x, oy + y, sub, tile);
        part = unit_part<UW, UH, KW>(w, s0, kk, sk2, kbuf, sad_metric, sub);
      } else {
        uint32_t w[UH][UW / 2 + 1];
        uint32_t s0;
        load_window10<UW, UH>(w, s0, ref, ox + x, oy + y, sub, tile);
        part = unit_part10<UW, UH>(w, s0, kk, sad_metric, sub);
      }
    }
    uint32_t d = group_sum(part, L);
    if (BD != 8 && sad_metric) d >>= BD - 8;   // xGetSAD12/24/48 at bitDepth 10: the block sum >> 2
    dist = v ? d : 0xFFFFFFFFu;
    return v ? d + mv_cost(ml, mv_bits(x, y, 2, j.mvp_x, j.mvp_y)) : 0xFFFFFFFFu;
  };
  // the least tested distortion of a chunk into cmin (ring mode)
  auto push_min = [&](uint32_t dist, int lim) FME_AI {
    if (ring) {
      const uint32_t m = (uint32_t)(wave_min_from((uint64_t)dist << 32, L, lim) >> 32);
      cmin = m < cmin ? m : cmin;
    }
  };

  Tz s;   // the wave-uniform IntTZSearchStruct and ranges (diamond_point / two_point read them)
  s.best_sad = 0xFFFFFFFFu;
  s.bx = s.by = s.bdist = s.bround = s.pnr = 0;
  s.R = Range{j.lt_x, j.rb_x, j.lt_y, j.rb_y};
  s.RR = s.R;
  s.range = e.search_range ? e.search_range : 64;
  s.k = 0; s.dist = 1; s.ox = s.oy = 0; s.opnr = 0;
  // FastSearch 0 (FME_TZ_FULL: xPatternSearch for every job, TEncSearch.cpp:4504-4507) and 3
  // (FME_TZ_ENHANCED: xTZSearch with bExtendedSettings, 4726-4727, 4749-4768)
  // (FME_TZ_RING, the backups' FastSearch 1 path, takes precedence over both)
  const bool full = !ring && (e.flags & FME_TZ_FULL) != 0;
  const bool enh = !full && !ring && (e.flags & FME_TZ_ENHANCED) != 0;
  s.corners = enh;   // bFirstCornersForDiamondDist1, bStarRefinementCornersForDiamondDist1
  auto take = [&](uint32_t cost, int x, int y, int pd, int pnr) FME_AI {   // xTZSearchHelp's update
    if (cost < s.best_sad) {
      s.best_sad = cost;
      s.bx = x; s.by = y; s.bdist = pd; s.pnr = pnr; s.bround = 0;
    }
  };
  // (cost << 32 | call index) minimum of a list of n points, G at a time; pt(i, x, y) -> tested?
  auto list_min = [&](int n, auto&& pt) FME_AI -> uint64_t {
    uint64_t best = ~0ull;
    for (int base = 0; base < n; base += G) {
      const int i = base + g;
      int x = 0, y = 0;
      const bool v = i < n && pt(i, x, y);
      uint32_t dist;
      const uint32_t c = cost_at(x, y, v, dist);
      const uint64_t key = block_min<NW>(wave_min_from(((uint64_t)c << 32) | (uint32_t)i, L, 64));
      best = key < best ? key : best;
      push_min(dist, 64);
    }
    return best;
  };
  auto ring_pt = [&](int slot, int& x, int& y, int& pnr, int& pd) FME_AI -> bool {
    s.dist = 1 << (slot >> 4);
    bool ok;
    return diamond_point(s, slot & 15, ok, x, y, pnr, pd) && ok;
  };
  int nr = 0;
  while ((1 << nr) <= s.range) nr++;   // dist 1, 2, 4, ... <= m_iSearchRange
  // compact ring order: ring sizes c0, 8, 8, 8, 16, 16, 16 (xTZ8PointDiamondSearch; c0 = 4, or 8
  // with the distance-1 corners), point i of the concatenation -> ring slot (call order preserved)
  auto ring_start = [](int r, int c0) FME_AI { return r == 0 ? 0 : (r < 4 ? c0 + 8 * (r - 1) : c0 + 24 + 16 * (r - 4)); };
  auto compact_slot = [](int i, int c0) FME_AI {
    return i < c0 ? i : (i < c0 + 24 ? 16 * (1 + (i - c0) / 8) + ((i - c0) & 7) : 16 * (4 + (i - c0 - 24) / 16) + ((i - c0 - 24) & 15));
  };
  const int c0 = s.corners ? 8 : 4;
  const int nring_pts = ring_start(nr, c0);
  auto two_point_search = [&]() FME_AI {   // xTZ2PointSearch around the best, opnr = its point nr
    s.ox = s.bx; s.oy = s.by; s.opnr = s.pnr;
    const uint64_t k = list_min(2, [&](int i, int& x, int& y) FME_AI {
      bool ok;
      return two_point(s, i, ok, x, y) && ok;
    });
    if ((uint32_t)(k >> 32) < s.best_sad) {
      int x, y;
      bool ok;
      two_point(s, (int)(uint32_t)k, ok, x, y);
      take((uint32_t)(k >> 32), x, y, 2, 0);
    }
  };

  if ((j.flags & FME_JOB_BIPRED) || full) {
    // xPatternSearch: every point of the range in raster order
    const int nx = s.R.r - s.R.l + 1, ny = s.R.b - s.R.t + 1;
    if (nx > 0 && ny > 0) {
      const uint64_t k = list_min(nx * ny, [&](int i, int& x, int& y) FME_AI {
        x = s.R.l + i % nx; y = s.R.t + i / nx;
        return true;
      });
      const int i = (int)(uint32_t)k;
      take((uint32_t)(k >> 32), s.R.l + i % nx, s.R.t + i / nx, 0, 0);
    }
  } else {
    // ---- start points: 0 the AMVP predictor, 1..3 the neighbours' MVs (FastSearch 3,
    // m_acMvPredictors), 4 the zero vector, 5 the 2Nx2N MV; costs together, tests in call order ---
    int mx = j.mvp_x, my = j.mvp_y;
    clip_qpel(mx, my, ref.width, ref.height, e.cu_x, e.cu_y);
    const int sx = round4(mx), sy = round4(my);
    const bool has_pred = (e.flags & FME_TZ_PRED2NX2N) != 0;
    int qx = pred_x * 4, qy = pred_y * 4;
    clip_qpel(qx, qy, ref.width, ref.height, e.cu_x, e.cu_y);
    const int px = round4(qx), py = round4(qy);
    int nbx[3] = {0, 0, 0}, nby[3] = {0, 0, 0};
    if (enh) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        int ax, ay;
        tz_pred_at(ta, jid, k, ax, ay);
        clip_qpel(ax, ay, ref.width, ref.height, e.cu_x, e.cu_y);
        nbx[k] = round4(ax);
        nby[k] = round4(ay);
      }
    }
    {
      constexpr int NS = 6;
      uint32_t cs[NS], ds[NS];
#pragma unroll
      for (int q = 0; q < NS; q++) cs[q] = ds[q] = 0xFFFFFFFFu;
      for (int base = 0; base < NS; base += G) {
        const int i = base + g;
        const int x = i == 0 ? sx : (i == 1 ? nbx[0] : (i == 2 ? nbx[1] : (i == 3 ? nbx[2] : (i == 4 ? 0 : px))));
        const int y = i == 0 ? sy : (i == 1 ? nby[0] : (i == 2 ? nby[1] : (i == 3 ? nby[2] : (i == 4 ? 0 : py))));
        const bool v = i < NS && (i == 0 || i == 4 || (i == 5 && has_pred) || (i <= 3 && enh));
        uint32_t dist;
        const uint32_t c = cost_at(x, y, v, dist);
        if constexpr (NW == 1) {
#pragma unroll
          for (int q = 0; q < NS; q++)
            if (q >= base && q < base + G) {
              cs[q] = __shfl(c, (q - base) * L, 64);
              ds[q] = __shfl(dist, (q - base) * L, 64);
            }
        } else {   // several waves: the costs through LDS
          __shared__ uint32_t s_cs[NS];
          if (i < NS && u == 0) s_cs[i] = c;
          __syncthreads();
#pragma unroll
          for (int q = 0; q < NS; q++)
            if (q >= base && q < base + G) cs[q] = s_cs[q];
          __syncthreads();
          (void)dist;
        }
      }
      take(cs[0], sx, sy, 0, 0);
      cmin = ds[0];
      if (enh) {   // bTestOtherPredictedMV (4787-4805): "only test cMv if not obviously previously tested"
#pragma unroll
        for (int k = 0; k < 3; k++)
          if ((nbx[k] != sx || nby[k] != sy) && (nbx[k] != s.bx && nby[k] != s.by)) take(cs[1 + k], nbx[k], nby[k], 0, 0);
      }
      if ((sx != 0 || sy != 0) && (s.bx != 0 || s.by != 0)) {
        take(cs[4], 0, 0, 0, 0);
        cmin = ds[4] < cmin ? ds[4] : cmin;
      }
      if (has_pred && (sx != px || sy != py) && (px != s.bx || py != s.by)) {
        take(cs[5], px, py, 0, 0);
        cmin = ds[5] < cmin ? ds[5] : cmin;
      }
    }
    if (has_pred) {   // xSetSearchRange(currBest << 2, m_iSearchRange): the raster's range
      int cx = s.bx * 4, cy = s.by * 4;
      clip_qpel(cx, cy, ref.width, ref.height, e.cu_x, e.cu_y);
      int lx = cx - (s.range << 2), ly = cy - (s.range << 2), rx = cx + (s.range << 2), ry = cy + (s.range << 2);
      clip_qpel(lx, ly, ref.width, ref.height, e.cu_x, e.cu_y);
      clip_qpel(rx, ry, ref.width, ref.height, e.cu_x, e.cu_y);
      s.RR = Range{round4(lx), round4(rx), round4(ly), round4(ry)};
    }
    const bool best_zero = s.bx == 0 && s.by == 0;   // bBestCandidateZero (4857)

    // ---- first search: rings around the start, stop 3 rings after the last new best --------------
    if (G <= 16 || NW > 1) {   // ring by ring: one candidate list per ring, later rings skipped after the stop
      s.ox = s.bx; s.oy = s.by;
      for (int r = 0; r < nr; r++) {
        const int r0 = ring_start(r, c0);
        const uint64_t k = list_min(ring_start(r + 1, c0) - r0, [&](int i, int& x, int& y) FME_AI {
          int pnr, pd;
          return ring_pt(compact_slot(r0 + i, c0), x, y, pnr, pd);
        });
        s.bround += 1;
        if ((uint32_t)(k >> 32) < s.best_sad) {
          int xx, yy, pn, pdd;
          ring_pt(compact_slot(r0 + (int)(uint32_t)k, c0), xx, yy, pn, pdd);
          take((uint32_t)(k >> 32), xx, yy, pdd, pn);
        }
        if (s.bround >= 3 || 2 * (1 << r) > s.range) break;
      }
    } else {   // G >= 32: rings in 16-slot segments, several rings per chunk
      s.ox = s.bx; s.oy = s.by;
      const int nslot = 16 * nr, seg = 16 * L < 64 ? 16 * L : 64;
      uint64_t rmin = ~0ull;   // running minimum of the ring being completed (G < 16)
      uint32_t rdmin = 0xFFFFFFFFu;   // its least distortion (ring mode)
      bool stop = false;
      for (int base = 0; base < nslot && !stop; base += G) {
        const int i = base + g;
        int x = 0, y = 0, pnr = 0, pd = 0;
        const bool v = i < nslot && ring_pt(i, x, y, pnr, pd);
        uint32_t dist;
        const uint32_t c = cost_at(x, y, v, dist);
        const uint64_t key = wave_min_from(((uint64_t)c << 32) | (uint32_t)i, L, seg);
        // per-ring least distortion (rings after the stop are evaluated here but not tested by the
        // reference, so they must not reach C)
        const uint32_t dseg = ring ? (uint32_t)(wave_min_from((uint64_t)dist << 32, L, seg) >> 32) : 0u;
        // rings completed by this chunk, in order
        const int r0 = base >> 4, r1 = (base + G) >> 4;   // rings [r0, r1) end inside this chunk
        if (G < 16) {
          rmin = key < rmin ? key : rmin;
          rdmin = dseg < rdmin ? dseg : rdmin;
          if (((base + G) & 15) != 0) continue;
        }
        for (int r = r0; r < r1 && r < nr; r++) {
          uint64_t k = G < 16 ? rmin : (uint64_t)__shfl((unsigned long long)key, ((r * 16 - base) * L) & 63, 64);
          if (ring) {
            const uint32_t dr = G < 16 ? rdmin : (uint32_t)__shfl(dseg, ((r * 16 - base) * L) & 63, 64);
            cmin = dr < cmin ? dr : cmin;
          }
          rmin = ~0ull;
          rdmin = 0xFFFFFFFFu;
          s.bround += 1;
          if ((uint32_t)(k >> 32) < s.best_sad) {
            int xx, yy, pn, pdd;
            ring_pt((int)(uint32_t)k, xx, yy, pn, pdd);
            take((uint32_t)(k >> 32), xx, yy, pdd, pn);
          }
          if (s.bround >= 3 || 2 * (1 << r) > s.range) {
            stop = true;
            break;
          }
        }
      }
    }
    // ---- FastSearch 3: the zero vector's neighbourhood at half the range (bNewZeroNeighbourhoodTest,
    // bTestZeroVectorStart, 4900-4917), diamonds without corners around (0, 0), every ring ------------
    if (enh && !best_zero) {
      int nz = 0;
      while ((1 << nz) <= (s.range >> 1)) nz++;
      s.ox = s.oy = 0;
      s.corners = false;
      const uint64_t k = list_min(ring_start(nz, 4), [&](int i, int& x, int& y) FME_AI {
        int pnr, pd;
        return ring_pt(compact_slot(i, 4), x, y, pnr, pd);
      });
      if ((uint32_t)(k >> 32) < s.best_sad) {
        int xx, yy, pn, pdd;
        ring_pt(compact_slot((int)(uint32_t)k, 4), xx, yy, pn, pdd);
        take((uint32_t)(k >> 32), xx, yy, pdd, pn);
      }
      s.corners = true;
    }
    if (s.bdist == 1) {
      s.bdist = 0;
      two_point_search();
    }
    // ---- raster: step 5 over the re-centred range when the best is far; FastSearch 3's adaptive
    // raster (4926-4951) always runs: step 5, or step 6 over the halved range when the best is near --
    if (enh || s.bdist > 5) {
      int win = 5;
      Range rr = s.RR;
      if (enh && !(s.bdist > 5)) {
        win = 6;
        rr.l /= 2; rr.r /= 2; rr.t /= 2; rr.b /= 2;   // C++ division: towards zero
      }
      s.bdist = win;
      if (rr.l <= rr.r && rr.t <= rr.b) {
        const int nx = (rr.r - rr.l) / win + 1, ny = (rr.b - rr.t) / win + 1;
        const uint64_t k = list_min(nx * ny, [&](int i, int& x, int& y) FME_AI {
          x = rr.l + win * (i % nx); y = rr.t + win * (i / nx);
          return true;
        });
        const int i = (int)(uint32_t)k;
        take((uint32_t)(k >> 32), rr.l + win * (i % nx), rr.t + win * (i / nx), win, 0);
      }
    }
    // ---- star refinement: every ring around the best, until the best stays ----------------------
    for (int guard = 0; guard < 4096 && s.bdist > 0; guard++) {
      s.ox = s.bx; s.oy = s.by; s.bdist = 0; s.pnr = 0;
      const uint64_t k = list_min(nring_pts, [&](int i, int& x, int& y) FME_AI {
        int pnr, pd;
        return ring_pt(compact_slot(i, c0), x, y, pnr, pd);
      });
      if ((uint32_t)(k >> 32) < s.best_sad) {
        int xx, yy, pn, pdd;
        ring_pt(compact_slot((int)(uint32_t)k, c0), xx, yy, pn, pdd);
        take((uint32_t)(k >> 32), xx, yy, pdd, pn);
      }
      if (s.bdist == 1) {
        s.bdist = 0;
        if (s.pnr != 0) two_point_search();
      }
    }
  }
  // ---- the EMI square step (producer: m_integerMv2Nx2N is the post-square MV) ----------------------
  const bool square = ta.emi_mv != nullptr && (j.flags & FME_JOB_EMI) && !(j.flags & FME_JOB_BIPRED);
  const int tx = s.bx, ty = s.by;
  const uint32_t tsad = s.best_sad;
  const uint32_t c_tz = cmin;   // C: the pushes before index_ref
  if (square) {
    s.ox = s.bx; s.oy = s.by;
    const uint64_t k = list_min(8, [&](int i, int& x, int& y) FME_AI {
      bool ok;
      return square_point(s, i, ok, x, y) && ok;
    });
    if ((uint32_t)(k >> 32) < s.best_sad) {
      int x, y;
      bool ok;
      square_point(s, (int)(uint32_t)k, ok, x, y);
      take((uint32_t)(k >> 32), x, y, 1, (int)(uint32_t)k + 1);
    }
  }
  // ---- the backups' tail (FME_TZ_RING): xTZ8PointSquareSearch at distance 1 and
  // xTZ8PointSquareSearch2 at distance 2 around the star best (Backups/4:4868-4878, 818-873,
  // 876-965), every distortion pushed; rcMv moves with their xTZSearchHelp updates ---------------
  uint32_t eslot[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};   // array_e[index_ref + k] (0: never pushed)
  if (ring) {
    s.ox = s.bx; s.oy = s.by;
    // the 24 points in call order; bit i of `okm`: point i passes the reference's range checks
    uint32_t okm = 0;
#pragma unroll
    for (int i = 0; i < 24; i++) {
      bool ok;
      int x, y;
      ring_square_point(s, i, ok, x, y);
      okm |= ok ? (1u << i) : 0u;
    }
    uint64_t best = ~0ull;
    for (int base = 0; base < 24; base += G) {
      const int i = base + g;
      int x = 0, y = 0;
      bool ok = false;
      if (i < 24) ring_square_point(s, i, ok, x, y);
      uint32_t dist;
      const uint32_t c = cost_at(x, y, ok, dist);
      const uint64_t key = wave_min_from(((uint64_t)c << 32) | (uint32_t)i, L, 64);
      best = key < best ? key : best;
      // slot k = the k-th pushed point: its group's distortion
      uint32_t m = okm;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int idx = m ? __builtin_ctz(m) : 32;
        m &= m ? m - 1 : 0u;
        if (idx >= base && idx < base + G) eslot[k] = (uint32_t)__shfl((int)dist, ((idx - base) * L) & 63, 64);
      }
    }
    if ((uint32_t)(best >> 32) < s.best_sad) {
      int x, y;
      bool ok;
      ring_square_point(s, (int)(uint32_t)best, ok, x, y);
      take((uint32_t)(best >> 32), x, y, 0, 0);
    }
  }
  if ((NW == 1 ? lane : (int)threadIdx.x) == 0) {   // one writer per PU (NW = 1: per wave)
    fme_job* out = ta.jobs_out + jid;
    // ring mode: rcMv after the ring (Backups/4:4881-4882); otherwise the TZ best before the square
    const int bx = ring ? s.bx : tx, by = ring ? s.by : ty;
    const uint32_t bsad = ring ? s.best_sad : tsad;
    out->mv_x = (int16_t)bx;
    out->mv_y = (int16_t)by;
    if (ta.sad) ta.sad[jid] = bsad - mv_cost(ml, mv_bits(bx, by, 2, j.mvp_x, j.mvp_y));
    if (ta.emi_mv) {   // the integer MV after the square step (rcMv of xTZSearch, TEncSearch.cpp:5037-5048)
      reinterpret_cast<uint32_t*>(ta.emi_mv)[jid] = (uint32_t)(uint16_t)s.bx | ((uint32_t)(uint16_t)s.by << 16);
    }
    if (ring) {   // U1 V1 U2 H1 H2 U3 V2 U4 = array_e[index_ref .. +7], then C (Backups/4:4343-4359)
      uint32_t* o = ta.nn_in + (size_t)9 * jid;
#pragma unroll
      for (int k = 0; k < 8; k++) o[k] = eslot[k];
      o[8] = c_tz;
    }
  }
}

__constant__ int kTzW[kNumClasses] = {4, 8, 8, 4, 16, 8, 16, 12, 16, 16, 8, 32, 16, 32, 24, 32, 32, 16, 64, 32, 64, 48, 64, 64};
__constant__ int kTzH[kNumClasses] = {8, 4, 8, 16, 4, 16, 8, 16, 12, 16, 32, 8, 32, 16, 32, 24, 32, 64, 16, 64, 32, 64, 48, 64};


// Wave-uniform bulk search: one wave per PU of the kernel's unit shape, PUs in class order (CTU
// order inside a class); blocks dealt to the XCDs in contiguous ranges so each L2 sees one band.
#ifndef FME_TZW_WAVES   // waves per SIMD (1080p frame, tools/tz_probe.py: 4 -> 6.17 ms, 5 -> 5.84 ms)
#define FME_TZW_WAVES 5
#endif
// Work order: block b runs on XCD b % 8 (round-robin dispatch), and XCD x owns the x-th eighth of
// every class of this kernel (a spatial band per L2), largest PU class first: the long searches
// (a 64x64 PU's raster is hundreds of dependent candidate chunks) start at once instead of
// forming the kernel's tail behind the small ones.
__device__ __forceinline__ int tz_kid_of(int c) { return (kTzW[c] % 8) ? 0 : ((kTzH[c] % 8) ? 1 : 2); }
// XCD x's PU list: for each class of kernel kid, largest first, the x-th eighth of the class.
// Entry t of the list -> (class, position in class order), or q = -1 past its end.
__device__ __forceinline__ int tz_entry(const TzSchedule& sc, int kid, int x, int t, int& c) {
  for (c = kNumClasses - 1; c >= 0; c--) {
    if (tz_kid_of(c) != kid) continue;
    const int cnt = sc.class_cnt[c];
    const int lo = (int)(((long long)cnt * x) >> 3), hi = (int)(((long long)cnt * (x + 1)) >> 3);
    if (t < hi - lo) return sc.class_off[c] + lo + t;
    t -= hi - lo;
  }
  return -1;
}

template <int UW, int UH, int KB, int BD = 8>
__global__ __launch_bounds__(kTzNT) __attribute__((amdgpu_waves_per_eu(FME_TZW_WAVES)))
void k_tz_wave(TzArgs ta, TzSchedule sc, int kid) {
  const int x = (int)blockIdx.x & 7;
  const int t = ((int)blockIdx.x >> 3) * (kTzNT / 64) + (int)(threadIdx.x >> 6);
  int c;
  const int q = tz_entry(sc, kid, x, t, c);
  if (q < 0) return;
  const int jid = ta.perm[q];
  const fme_job j = FME_SJOBS ? ta.sjobs[q] : ta.a.jobs[jid];
  tz_wave<UW, UH, 1, KB, BD>(ta, jid, j, kTzW[c], kTzH[c], tz_ext_at(ta, jid).pred2n_x, tz_ext_at(ta, jid).pred2n_y);
}

// ---- staged bulk search: PUs grouped by (kernel, reference picture, CTU), a group's search area
// in LDS (TileRef).  k_tz_pair_count / k_tz_pair_scan / k_tz_pair_scatter build the groups on the
// device from the class bytes; k_tz_staged runs one workgroup per group, which stages the group's
// tile and searches its PUs one wave per PU (claimed from the group in order: the scatter visits
// the class order backwards, so the large PUs tend to come first).
__device__ __forceinline__ int tz_pair_key(const TzPairs& tp, const fme_job& j, int kid) {
  const int cx = min((int)j.x >> 6, tp.cw - 1), cy = min((int)j.y >> 6, tp.ch - 1);
  return kid * tp.np + ((int)j.ref_id * tp.ch + cy) * tp.cw + cx;
}

// Per-wave aggregation of the group atomics: the CTU-ordered stream gives a wave few distinct
// groups (<= 12 in a CTU: 4 references x 3 kernels), so each distinct key costs one atomic per wave
// (one per job serialised on the hot counters: 115 us for a 1080p frame).  Returns this lane's
// position among the wave's lanes with its key; *base gets the atomic's old value (scatter).
__device__ __forceinline__ int wave_agg_add(int32_t* ctr, int key, bool valid, int* base) {
  const int lane = (int)threadIdx.x & 63;
  uint64_t todo = __ballot(valid);
  int rank = 0, b = 0;
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    const int k = __builtin_amdgcn_readlane(key, leader);
    const uint64_t m = __ballot(valid && key == k);
    int old = 0;
    if (lane == leader) old = atomicAdd(&ctr[k], __popcll(m));
    old = __builtin_amdgcn_readlane(old, leader);
    if (valid && key == k) {
      rank = __popcll(m & ((1ull << lane) - 1));
      b = old;
    }
    todo &= ~m;
  }
  if (base) *base = b;
  return rank;
}

__global__ __launch_bounds__(256) void k_tz_pair_count(TzArgs ta, TzPairs tp, const uint8_t* __restrict__ cls, int n) {
  const int i = (int)(blockIdx.x * 256 + threadIdx.x);
  const int c = i < n ? cls[i] : 255;
  const bool valid = c < kNumClasses;
  const int key = valid ? tz_pair_key(tp, ta.a.jobs[i], tz_kid_of(c)) : 0;
  (void)wave_agg_add(tp.cnt, key, valid, nullptr);
}

// One workgroup: exclusive prefix of the 3 np group counts (the cursors), and the list of non-empty
// groups, kernel-major (a prefix of the non-empty flags): kernel kid's groups are
// seg[nseg[3 + kid] ..) and there are nseg[kid] of them.
__global__ __launch_bounds__(1024) void k_tz_pair_scan(TzPairs tp) {
  __shared__ int32_t part[1024], nz[1024], first[3];
  const int tot = 3 * tp.np, per = (tot + 1023) / 1024, t = (int)threadIdx.x;
  const int b = min(tot, t * per), e = min(tot, b + per);
  int sum = 0, nnz = 0;
  for (int k = b; k < e; k++) {
    const int c = tp.cnt[k];
    sum += c;
    nnz += c > 0;
  }
  part[t] = sum;
  nz[t] = nnz;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {   // inclusive scans (Hillis-Steele)
    const int v = t >= d ? part[t - d] : 0, w = t >= d ? nz[t - d] : 0;
    __syncthreads();
    part[t] += v;
    nz[t] += w;
    __syncthreads();
  }
  int run = part[t] - sum, r = nz[t] - nnz;
  for (int k = b; k < e; k++) {
    const int c = tp.cnt[k];
    tp.off[k] = run;
    tp.cursor[k] = run;
    if (k % tp.np == 0) first[k / tp.np] = r;   // the kernel's first group in seg
    if (c > 0) tp.seg[r++] = k;
    run += c;
  }
  __syncthreads();
  if (t < 3) {
    tp.nseg[3 + t] = first[t];
    tp.nseg[t] = (t < 2 ? first[t + 1] : nz[1023]) - first[t];
  }
}

// Jobs into their groups, visiting the class order (perm) from the largest class down.
__global__ __launch_bounds__(256) void k_tz_pair_scatter(TzArgs ta, TzPairs tp, const uint8_t* __restrict__ cls, int n) {
  const int i = (int)(blockIdx.x * 256 + threadIdx.x);
  const int jid = i < n ? ta.perm[n - 1 - i] : 0;
  const int c = i < n ? cls[jid] : 255;
  const bool valid = c < kNumClasses;
  const int key = valid ? tz_pair_key(tp, ta.a.jobs[jid], tz_kid_of(c)) : 0;
  int base;
  const int rank = wave_agg_add(tp.cursor, key, valid, &base);
  if (valid) tp.perm[base + rank] = jid;
}

#ifndef FME_TZS_NT   // threads per workgroup of the staged search (1080p frame, tools/tz_probe.py: 6 waves
#define FME_TZS_NT 512   // 5.69 ms, 8 waves 4.83 ms; two 45.7 KB tiles per CU at 5 waves/SIMD of registers)
#endif
#ifndef FME_TZS_WAVES   // waves per SIMD the staged kernel's registers are sized for
#define FME_TZS_WAVES FME_TZW_WAVES
#endif
// One launch per unit-shape kernel, one workgroup per group (the grid an upper bound): stage the
// group's tile, then search its PUs, one wave per PU.  (The three kernels' searches in one launch,
// behind a switch, spilled 282 VGPRs: the allocation is the maximum over the three.)
template <int UW, int UH, int KB, int BD = 8>
__global__ __launch_bounds__(FME_TZS_NT) __attribute__((amdgpu_waves_per_eu(FME_TZS_WAVES)))
void k_tz_staged(TzArgs ta, TzPairs tp, int kid) {
  constexpr int TH = BD == 8 ? kTileH : kTileH10, TWD = BD == 8 ? kTileWD : kTileWD10;
  constexpr int TM = BD == 8 ? kTileM : kTileM10;
  __shared__ uint32_t tile[TH * TWD];
  if ((int)blockIdx.x >= tp.nseg[kid]) return;
  const int key = tp.seg[tp.nseg[3 + kid] + (int)blockIdx.x];
  const int start = tp.off[key], cnt = tp.cnt[key];
  // the tile: the group's CTU displaced by its first PU's start MV (round4 of the clipped AMVP)
  const int j0 = tp.perm[start];
  const fme_job jb = ta.a.jobs[j0];
  const fme_tz_ext e0 = tz_ext_at(ta, j0);
  const PicDesc ref = ta.a.pics[jb.ref_id];
  int mx = jb.mvp_x, my = jb.mvp_y;
  clip_qpel(mx, my, ref.width, ref.height, e0.cu_x, e0.cu_y);
  const int x0 = (((int)jb.x & ~63) + round4(mx) - TM) & (BD == 8 ? ~3 : ~1);
  const int y0 = ((int)jb.y & ~63) + round4(my) - TM;
  for (int i = (int)threadIdx.x; i < TH * TWD; i += FME_TZS_NT) {
    const int r = i / TWD, q = i - r * TWD;
    uint32_t v;
    if constexpr (BD == 8) {
      const uint8_t* row = ref.luma + (size_t)clamp_i(y0 + r, 0, ref.height - 1) * ref.stride;
      const int x = x0 + 4 * q;
      if (x >= 0 && x + 4 <= ref.width) {
        v = gld32(row + x);
      } else {
        v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) v |= gld8(row + clamp_i(x + k, 0, ref.width - 1)) << (8 * k);
      }
    } else {   // sample pairs of the uint16 plane
      typedef __attribute__((address_space(1))) const uint16_t gu16c;
      const uint16_t* row = reinterpret_cast<const uint16_t*>(ref.luma) + (size_t)clamp_i(y0 + r, 0, ref.height - 1) * ref.stride;
      const int x = x0 + 2 * q;
      if (x >= 0 && x + 2 <= ref.width) {
        v = gld32(row + x);
      } else {
        v = (uint32_t)*(gu16c*)(row + clamp_i(x, 0, ref.width - 1)) |
            ((uint32_t)*(gu16c*)(row + clamp_i(x + 1, 0, ref.width - 1)) << 16);
      }
    }
    tile[i] = v;
  }
  __syncthreads();
  const TileRef tr{tile, x0, y0};
  // wave w takes PUs w, w + NW, ... of the group (largest first).  (Claiming them from an LDS
  // counter with ds_add_rtn instead never finished on the box, round 5.)
  for (int p = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); p < cnt; p += FME_TZS_NT / 64) {
    const int jid = tp.perm[start + p];
    const fme_job j = ta.a.jobs[jid];
    tz_wave<UW, UH, 1, KB, BD>(ta, jid, j, j.w, j.h, tz_ext_at(ta, jid).pred2n_x, tz_ext_at(ta, jid).pred2n_y, tr);
  }
}

// One dependency level of a producer's m_integerMv2Nx2N chain (fme_pred_inter_p/b): one wave per
// job in chain mode.  The host launches the levels back to back on one stream, so a level reads the
// post-EMI MVs of earlier levels from global memory (kernel boundaries order them) and no level
// waits for the host.  ch.psrc[q] >= 0: job q's m_integerMv2Nx2N is job psrc[q]'s result; -1: its
// ext already holds it.
#ifndef FME_TZL_WAVES
#define FME_TZL_WAVES 1   // waves per chain job (A/B: 8 waves 276 ms per P frame, spilling; 1 wave 198 ms)
#endif
template <int BD>
__global__ __launch_bounds__(64 * FME_TZL_WAVES) void k_tz_level(TzArgs ta, TzChain ch, int first) {
  const int q = first + (int)blockIdx.x;
  const int PW = ta.a.jobs[q].w, PH = ta.a.jobs[q].h;   // shapes checked by the host
  const int ps = ch.psrc[q];
  int px = tz_ext_at(ta, q).pred2n_x, py = tz_ext_at(ta, q).pred2n_y;
  if (ps >= 0) {
    const uint32_t mv = reinterpret_cast<const uint32_t*>(ta.emi_mv)[ps];
    px = (int)(int16_t)(mv & 0xFFFFu);
    py = (int)(int16_t)(mv >> 16);
  }
  const int kid = (PW % 8) ? 0 : ((PH % 8) ? 1 : 2);
  const fme_job j = ta.a.jobs[q];
  if (kid == 0) tz_wave<4, 8, FME_TZL_WAVES, -1, BD>(ta, q, j, PW, PH, px, py);
  else if (kid == 1) tz_wave<8, 4, FME_TZL_WAVES, -1, BD>(ta, q, j, PW, PH, px, py);
  else tz_wave<8, 8, FME_TZL_WAVES, -1, BD>(ta, q, j, PW, PH, px, py);
}

}  // namespace

#if FME_TZ_COUNT
extern "C" int fme_debug_tz_counts(unsigned long long* out6, int reset) {
  if (out6 && hipMemcpyFromSymbol(out6, HIP_SYMBOL(g_tz_count), sizeof(g_tz_count)) != hipSuccess) return -2;
  if (reset) {
    static const unsigned long long zero[3][2] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tz_count), zero, sizeof(zero)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

hipError_t launch_tz_levels(const TzArgs& ta, const TzChain& ch, const int32_t* h_lvl_off, int bit_depth, hipStream_t s) {
  for (int lv = 0; lv < ch.nlev; lv++) {
    const int n = h_lvl_off[lv + 1] - h_lvl_off[lv];
    if (n <= 0) continue;
    if (bit_depth > 8) hipLaunchKernelGGL(k_tz_level<10>, dim3(n), dim3(64 * FME_TZL_WAVES), 0, s, ta, ch, h_lvl_off[lv]);
    else hipLaunchKernelGGL(k_tz_level<8>, dim3(n), dim3(64 * FME_TZL_WAVES), 0, s, ta, ch, h_lvl_off[lv]);
  }
  return hipGetLastError();
}

// Unit shape of a class for the integer search: 8 wide / tall where the PU allows, else 4.
int tz_kernel_of(int cls) {
  const int w = kClassW[cls], h = kClassH[cls];
  const int uw = (w % 8) == 0 ? 8 : 4, uh = (h % 8) == 0 ? 8 : 4;
  return uw == 4 ? 0 : (uh == 4 ? 1 : 2);
}
int tz_lanes_per_pu(int cls) {
  const int w = kClassW[cls], h = kClassH[cls];
  const int uw = (w % 8) == 0 ? 8 : 4, uh = (h % 8) == 0 ? 8 : 4;
  const int lr = (w / uw) * (h / uh);
  int l = 1;
  while (l < lr) l <<= 1;
  return l;
}

hipError_t launch_tz_pairs(const TzArgs& ta, const TzPairs& tp, const uint8_t* cls, int n, hipStream_t s) {
  const int nb = (n + 255) / 256;
  hipLaunchKernelGGL(k_tz_pair_count, dim3(nb), dim3(256), 0, s, ta, tp, cls, n);
  hipLaunchKernelGGL(k_tz_pair_scan, dim3(1), dim3(1024), 0, s, tp);
  hipLaunchKernelGGL(k_tz_pair_scatter, dim3(nb), dim3(256), 0, s, ta, tp, cls, n);
  return hipGetLastError();
}

hipError_t launch_tz_staged(const TzArgs& ta, const TzPairs& tp, int kid, bool keyed, int bit_depth, hipStream_t s) {
  const dim3 g(tp.np), b(FME_TZS_NT);
  if (bit_depth > 8) {
    if (kid == 0) hipLaunchKernelGGL((k_tz_staged<4, 8, -1, 10>), g, b, 0, s, ta, tp, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_staged<8, 4, -1, 10>), g, b, 0, s, ta, tp, 1);
    else hipLaunchKernelGGL((k_tz_staged<8, 8, -1, 10>), g, b, 0, s, ta, tp, 2);
  } else if (keyed) {
    if (kid == 0) hipLaunchKernelGGL((k_tz_staged<4, 8, -1>), g, b, 0, s, ta, tp, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_staged<8, 4, -1>), g, b, 0, s, ta, tp, 1);
    else hipLaunchKernelGGL((k_tz_staged<8, 8, -1>), g, b, 0, s, ta, tp, 2);
  } else {
    if (kid == 0) hipLaunchKernelGGL((k_tz_staged<4, 8, 0>), g, b, 0, s, ta, tp, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_staged<8, 4, 0>), g, b, 0, s, ta, tp, 1);
    else hipLaunchKernelGGL((k_tz_staged<8, 8, 0>), g, b, 0, s, ta, tp, 2);
  }
  return hipGetLastError();
}

// Wave-uniform bulk search of kernel kid: sc.prefix in waves (one per PU).
hipError_t launch_tz_wave(const TzArgs& ta, const TzSchedule& sc, int kid, bool keyed, int bit_depth, hipStream_t s) {
  int share = 0;   // the largest per-XCD share of this kernel's PUs (waves)
  for (int x = 0; x < 8; x++) {
    int n = 0;
    for (int c = 0; c < kNumClasses; c++)
      if (tz_kernel_of(c) == kid)
        n += (int)(((long long)sc.class_cnt[c] * (x + 1)) >> 3) - (int)(((long long)sc.class_cnt[c] * x) >> 3);
    share = std::max(share, n);
  }
  if (share <= 0) return hipSuccess;
  const int blocks = 8 * ((share + kTzNT / 64 - 1) / (kTzNT / 64));
  if (bit_depth > 8) {   // one form: the 10-bit key rows are sample pairs either way
    if (kid == 0) hipLaunchKernelGGL((k_tz_wave<4, 8, -1, 10>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_wave<8, 4, -1, 10>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 1);
    else hipLaunchKernelGGL((k_tz_wave<8, 8, -1, 10>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 2);
  } else if (keyed) {
    if (kid == 0) hipLaunchKernelGGL((k_tz_wave<4, 8, -1>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_wave<8, 4, -1>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 1);
    else hipLaunchKernelGGL((k_tz_wave<8, 8, -1>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 2);
  } else {
    if (kid == 0) hipLaunchKernelGGL((k_tz_wave<4, 8, 0>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 0);
    else if (kid == 1) hipLaunchKernelGGL((k_tz_wave<8, 4, 0>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 1);
    else hipLaunchKernelGGL((k_tz_wave<8, 8, 0>), dim3(blocks), dim3(kTzNT), 0, s, ta, sc, 2);
  }
  return hipGetLastError();
}


}  // namespace fme
