// fme_mc.hip — motion compensation of decided MVs (gfx950): luma 8-tap + 4:2:0 chroma 4-tap.
//
// TComPrediction::motionCompensation (TComPrediction.cpp:495-560): a few PUs per workgroup, one
// 4x4 luma unit (+ the co-sited 2x2 Cb and Cr units) per lane, reference windows in VGPRs:
//   * clipMv of each list's MV against the CU origin (TComDataCU.cpp:2773-2786);
//   * xCheckIdenticalMotion (TComPrediction.cpp:476-492): both lists on one picture with one MV
//     -> uni-prediction from L0;
//   * xPredInterBlk (616-668) per component: integer offset mv >> (2 + csx), fraction
//     mv & ((4 << csx) - 1); HM copies at fraction (0,0), filters once at (fx,0) / (0,fy) and
//     twice otherwise (TComInterpolationFilter.cpp:94-154 filterCopy, 172-257 filter<N, isVert,
//     isFirst, isLast>).  Here every case runs the two-stage form with the identity filter
//     (64 at the centre tap) for a zero fraction, which gives the same integers: with
//     S = sum c.s and s' = s - 128 (sum c = 64), stage 1 = S - 8192 = sum c.s'; a zero vertical
//     fraction multiplies it by 64, and (64 (S - 8192) + 2048 + (8192 << 6)) >> 12 = (S + 32)
//     >> 6 (uni), (64 (S - 8192)) >> 6 = S - 8192 (bi); a zero horizontal fraction gives
//     stage 1 = 64 s' = (s << 6) - 8192, filterCopy's isFirst output.  Uni-prediction ends at
//     8 bits, bi-prediction keeps the 14-bit values;
//   * TComYuv::addAvg (TComYuv.cpp:354-415): (p0 + p1 + 16448) >> 7, clipped to 8 bits.
// Samples outside a plane are read with edge replication, which equals HM's padded picture for
// every clipped MV (luma margin 80, chroma margin 40: the clipped reads stay within 75 / 38).
#include <hip/hip_runtime.h>

#include "fme_device.h"
#include "fme_simd.h"

namespace fme {
namespace {

using namespace simd;


// TComInterpolationFilter.cpp:57-75 as int8 quads (luma: taps 0-3, 4-7; chroma: taps 0-3).
// Fraction 0 uses the identity filter (64 at the centre tap): through the two-stage form below
// it reproduces filterCopy and the 1-D filters exactly (module header).
__device__ __forceinline__ void luma_taps(int f, uint32_t& lo, uint32_t& hi) {
  lo = f == 0 ? q8(0, 0, 0, 64) : f == 1 ? q8(-1, 4, -10, 58) : f == 2 ? q8(-1, 4, -11, 40) : q8(0, 1, -5, 17);
  hi = f == 0 ? 0u : f == 1 ? q8(17, -5, 1, 0) : f == 2 ? q8(40, -11, 4, -1) : q8(58, -10, 4, -1);
}
__device__ __forceinline__ uint32_t chroma_taps(int f) {
  switch (f) {
    case 0: return q8(0, 64, 0, 0);
    case 1: return q8(-2, 58, 10, -2);
    case 2: return q8(-4, 54, 16, -2);
    case 3: return q8(-6, 46, 28, -4);
    case 4: return q8(-4, 36, 36, -4);
    case 5: return q8(-4, 28, 46, -6);
    case 6: return q8(-2, 16, 54, -4);
    default: return q8(-2, 10, 58, -2);
  }
}
__device__ __forceinline__ int tap_of(uint32_t lo, uint32_t hi, int k) {   // signed byte k of (lo, hi)
  const uint32_t w = k < 4 ? lo : hi;
  return (int)(int8_t)(w >> (8 * (k & 3)));
}

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4a gu4;
typedef __attribute__((address_space(1))) const u32x3a gu3;

struct Plane {
  const uint8_t* p;
  int stride, w, h;
};

// TComDataCU::clipMv (TComDataCU.cpp:2773-2786), max CU 64 (sps.getMaxCUWidth/Height)
__device__ __forceinline__ void clip_mv(int& mx, int& my, int pic_w, int pic_h, int cu_x, int cu_y) {
  const int hor_max = (pic_w + 8 - cu_x - 1) << 2, hor_min = (-64 - 8 - cu_x + 1) * 4;
  const int ver_max = (pic_h + 8 - cu_y - 1) << 2, ver_min = (-64 - 8 - cu_y + 1) * 4;
  mx = min(hor_max, max(hor_min, mx));
  my = min(ver_max, max(ver_min, my));
}

// Rows of (s - 128) bytes of a window: R rows from plane row y0, ND dwords from byte x0 & ~3
// (edge-replicated), and the byte shift of x0 inside the first dword.
template <int R, int ND>
__device__ __forceinline__ uint32_t load_window(const Plane& pl, int x0, int y0, bool aligned, uint32_t (&w)[R][ND]) {
  const int xa = x0 & ~3;
  const bool inside = aligned && xa >= 0 && xa + 4 * ND <= pl.w && y0 >= 0 && y0 + R <= pl.h;
  if (inside) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint8_t* row = pl.p + (size_t)(y0 + r) * pl.stride + xa;
      if constexpr (ND == 4) {
        const u32x4a v = *(gu4*)row;
        w[r][0] = v.x ^ 0x80808080u; w[r][1] = v.y ^ 0x80808080u;
        w[r][2] = v.z ^ 0x80808080u; w[r][3] = v.w ^ 0x80808080u;
      } else if constexpr (ND == 3) {
        const u32x3a v = *(gu3*)row;
        w[r][0] = v.x ^ 0x80808080u; w[r][1] = v.y ^ 0x80808080u; w[r][2] = v.z ^ 0x80808080u;
      } else {
#pragma unroll
        for (int k = 0; k < ND; k++) w[r][k] = gld32(row + 4 * k) ^ 0x80808080u;
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint8_t* row = pl.p + (size_t)clamp_i(y0 + r, 0, pl.h - 1) * pl.stride;
#pragma unroll
      for (int k = 0; k < ND; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) v |= gld8(row + clamp_i(xa + 4 * k + b, 0, pl.w - 1)) << (8 * b);
        w[r][k] = v ^ 0x80808080u;
      }
    }
  }
  return (uint32_t)(x0 - xa);
}

// One U x U output unit of one list (N taps; U = 4 luma, 2 chroma): its window of R = U + N - 1
// rows of (s - 128) bytes around plane position (bx, by) (integer MV applied).
template <int N, int U>
struct UnitWin {
  static constexpr int R = U + N - 1;                   // window rows and columns
  static constexpr int NA = ((U - 1 + N - 4) >> 2) + 2; // re-aligned dwords the dot4 groups read
  static constexpr int ND = NA + 1;                     // dwords loaded per row (any alignment)
  uint32_t w[R][ND];
  uint32_t s0;
  __device__ __forceinline__ void load(const Plane& pl, bool aligned, int bx, int by) {
    s0 = load_window<R, ND>(pl, bx - (N / 2 - 1), by - (N / 2 - 1), aligned, w);
  }
  // Two stages in the (s - 128) domain, which absorbs filterCopy / filter<N, ., isFirst = true,
  // .>'s -IF_INTERNAL_OFFS: stage 1 = sum c.s - 8192; stage 2 uni (isLast): (sum + 2048 +
  // (8192 << 6)) >> 12 clipped, bi: sum >> 6 (14-bit).
  __device__ __forceinline__ void pred(uint32_t hlo, uint32_t hhi, uint32_t vlo, uint32_t vhi, bool uni,
                                       int (&out)[U][U]) const {
    int t[R][U];
#pragma unroll
    for (int r = 0; r < R; r++) {
      uint32_t a[NA];
#pragma unroll
      for (int k = 0; k < NA; k++) a[k] = __builtin_amdgcn_alignbyte(w[r][k + 1], w[r][k], s0);
#pragma unroll
      for (int c = 0; c < U; c++) {   // bytes c .. c+N-1 of the re-aligned row
        const uint32_t b0 = (c & 3) ? __builtin_amdgcn_alignbyte(a[(c >> 2) + 1], a[c >> 2], (uint32_t)(c & 3)) : a[c >> 2];
        int acc = dot4(b0, hlo, 0);
        if constexpr (N == 8) {
          const int q = c + 4;
          const uint32_t b1 = (q & 3) ? __builtin_amdgcn_alignbyte(a[(q >> 2) + 1], a[q >> 2], (uint32_t)(q & 3)) : a[q >> 2];
          acc = dot4(b1, hhi, acc);
        }
        t[r][c] = acc;
      }
    }
#pragma unroll
    for (int y = 0; y < U; y++)
#pragma unroll
      for (int c = 0; c < U; c++) {
        int sum = 0;
#pragma unroll
        for (int k = 0; k < N; k++) sum += t[y + k][c] * tap_of(vlo, vhi, k);
        out[y][c] = uni ? clamp_i((sum + 2048 + (8192 << 6)) >> 12, 0, 255) : (sum >> 6);
      }
  }
};

__device__ __forceinline__ bool mc_job_valid(const McArgs& a, const fme_mc_job& j) {
  if (j.w < 4 || j.h < 4 || j.w > 64 || j.h > 64 || (j.w & 3) || (j.h & 3)) return false;
  if (!(j.flags & (FME_MC_L0 | FME_MC_L1)) || (j.flags & ~(FME_MC_L0 | FME_MC_L1 | FME_MC_WP))) return false;
  if ((int)j.x + j.w > a.width || (int)j.y + j.h > a.height) return false;
  for (int l = 0; l < 2; l++) {
    if (!(j.flags & (1u << l))) continue;
    if (j.ref_id[l] >= FME_MAX_PICTURES) return false;
    const PicDesc& p = a.pics[j.ref_id[l]];
    if (!p.luma || !p.cb || !p.cr || p.width != a.width || p.height != a.height) return false;
  }
  return true;
}

__device__ __forceinline__ void store_row(uint8_t* d, const int* v, int n, bool aligned) {
  if (n == 4 && aligned) {
    *(uint32_t*)d = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  } else if (n == 2 && aligned) {
    *(uint16_t*)d = (uint16_t)((uint32_t)v[0] | ((uint32_t)v[1] << 8));
  } else {
    for (int i = 0; i < n; i++) d[i] = (uint8_t)v[i];
  }
}

// Per-job state shared by the workgroup (LDS), filled by one thread per job.
struct McJobInfo {
  int units;          // 4x4 luma units, 0 when invalid
  int ux_n;           // units per PU row
  int x, y;           // PU luma origin
  int nl;             // lists predicted (2: bi)
  int lix[2], liy[2], lfx[2], lfy[2];   // luma integer offsets / fractions per list
  int cix[2], ciy[2], cfx[2], cfy[2];   // chroma (eighth-pel) per list
  PicDesc pic[2];
  int wp;                              // FME_MC_WP: weighted prediction of the lists' 14-bit values
  int ww[2][3], wsh[3], woff[3];       // per component: the lists' weights, shift, (summed) offset
};

// getWpScaling (TComWeightPrediction.cpp:247-324) for the PU's lists, per component: bi-pred
// w0 / w1, offset o0 + o1, shift log2Wd + 1 (list 0's denominator); uni-pred w, o, shift log2Wd;
// offsets scaled by 1 << (bitDepth - 8); addWeightBi / addWeightUni then add shiftNum =
// max(2, 14 - bitDepth) (:103, :160).
__device__ __forceinline__ void mc_wp_setup(const McArgs& a, const fme_mc_job& j, const int* lists, int nl,
                                            McJobInfo& in) {
  const int bd = a.bit_depth > 8 ? a.bit_depth : 8;
  const int shift_num = 14 - bd > 2 ? 14 - bd : 2;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const fme_wp_param p0 = a.wp[(lists[0] * FME_MAX_PICTURES + j.ref_id[lists[0]]) * 3 + c];
    in.ww[0][c] = p0.weight;
    if (nl == 2) {
      const fme_wp_param p1 = a.wp[(FME_MAX_PICTURES + j.ref_id[1]) * 3 + c];
      in.ww[1][c] = p1.weight;
      in.woff[c] = (p0.offset + p1.offset) * (1 << (bd - 8));
      in.wsh[c] = p0.log2_denom + 1 + shift_num;
    } else {
      in.ww[1][c] = 0;
      in.woff[c] = p0.offset * (1 << (bd - 8));
      in.wsh[c] = p0.log2_denom + shift_num;
    }
  }
}

// weightBidir / weightUnidir (TComWeightPrediction.cpp:46-56) on the 14-bit values p0, p1 (HM's
// stored intermediates, IF_INTERNAL_OFFS 8192 below the sample scale).  The unit-weight branch of
// addWeightUni (noWeightUnidir with shiftNum) is the same value: w = 1 << d turns
// (w (p + 8192) + 2^(d + n - 1)) >> (d + n) into (p + 8192 + 2^(n - 1)) >> n exactly.
__device__ __forceinline__ int mc_wp_sample(const McJobInfo& in, int c, int p0, int p1, int maxv) {
  const int sh = in.wsh[c], half = 1 << (sh - 1);
  if (in.nl == 2)
    return clamp_i((in.ww[0][c] * (p0 + 8192) + in.ww[1][c] * (p1 + 8192) + half + in.woff[c] * half) >> sh, 0, maxv);
  return clamp_i(((in.ww[0][c] * (p0 + 8192) + half) >> sh) + in.woff[c], 0, maxv);
}

#ifndef FME_MC_JOBS
#define FME_MC_JOBS 8
#endif
constexpr int kMcJobs = FME_MC_JOBS;   // consecutive jobs per workgroup
constexpr int kMcBlock = 256;

// kMcJobs consecutive jobs per workgroup; their 4x4 luma units (each with the co-sited 2x2 Cb and
// Cr units) are dealt to the 256 lanes, so small and large PUs fill the waves alike; a lane
// predicts both lists of its unit in registers and averages them.
__global__ __launch_bounds__(kMcBlock) void k_mc(McArgs a) {
  __shared__ McJobInfo info[kMcJobs];
  __shared__ int first_unit[kMcJobs + 1];
  const int j0 = blockIdx.x * kMcJobs;
  const int t = threadIdx.x;
  if (t < kMcJobs) {
    McJobInfo& in = info[t];
    in.units = 0;
    const int ji = j0 + t;
    if (ji < a.n) {
      const fme_mc_job j = a.jobs[ji];
      if (!mc_job_valid(a, j)) {
        atomicAdd(a.invalid, 1);
      } else {
        int nl = 0, lists[2] = {0, 0};
        if (j.flags & FME_MC_L0) lists[nl++] = 0;
        if (j.flags & FME_MC_L1) lists[nl++] = 1;
        in.wp = (j.flags & FME_MC_WP) ? 1 : 0;
        if (nl == 2 && !in.wp && j.ref_id[0] == j.ref_id[1] && j.mv[0][0] == j.mv[1][0] && j.mv[0][1] == j.mv[1][1])
          nl = 1;   // xCheckIdenticalMotion (not with WPBiPred): same picture, same MV -> xPredInterUni(REF_PIC_LIST_0)
        in.nl = nl;
        if (in.wp) mc_wp_setup(a, j, lists, nl, in);
        for (int k = 0; k < nl; k++) {
          const int l = lists[k];
          const PicDesc p = a.pics[j.ref_id[l]];
          int mx = j.mv[l][0], my = j.mv[l][1];
          clip_mv(mx, my, p.width, p.height, j.cu_x, j.cu_y);
          in.lix[k] = mx >> 2;   // xPredInterBlk: shift 2 + csx, fraction mask (4 << csx) - 1
          in.liy[k] = my >> 2;
          in.lfx[k] = mx & 3;
          in.lfy[k] = my & 3;
          in.cix[k] = mx >> 3;
          in.ciy[k] = my >> 3;
          in.cfx[k] = mx & 7;
          in.cfy[k] = my & 7;
          in.pic[k] = p;
        }
        in.x = j.x;
        in.y = j.y;
        in.ux_n = j.w >> 2;
        in.units = (j.w >> 2) * (j.h >> 2);
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int k = 0; k < kMcJobs; k++) {
      first_unit[k] = acc;
      acc += info[k].units;
    }
    first_unit[kMcJobs] = acc;
  }
  __syncthreads();
  const int total = first_unit[kMcJobs];
  const bool ys_al = ((a.y_stride | (int)(uintptr_t)a.y) & 3) == 0;
  const bool cs_al = ((a.c_stride | (int)(uintptr_t)a.cb | (int)(uintptr_t)a.cr) & 1) == 0;
  for (int g = t; g < total; g += kMcBlock) {
    int q = 0;
#pragma unroll
    for (int k = 1; k < kMcJobs; k++) q += g >= first_unit[k] ? 1 : 0;
    const McJobInfo& in = info[q];
    const int u = g - first_unit[q];
    const int ux = u % in.ux_n, uy = u / in.ux_n;
    const bool wp = in.wp != 0;
    const bool uni = in.nl == 1 && !wp;   // weighted prediction filters to the 14-bit values (bi form)
    {   // luma 4x4
      const int x = in.x + 4 * ux, y = in.y + 4 * uy;
      int acc[4][4], o[4][4], q0[4][4];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k >= in.nl) break;
        const PicDesc& p = in.pic[k];
        UnitWin<8, 4> w;
        w.load(Plane{p.luma, p.stride, p.width, p.height}, ((p.stride | (int)(uintptr_t)p.luma) & 3) == 0,
               x + in.lix[k], y + in.liy[k]);
        uint32_t hlo, hhi, vlo, vhi;
        luma_taps(in.lfx[k], hlo, hhi);
        luma_taps(in.lfy[k], vlo, vhi);
        w.pred(hlo, hhi, vlo, vhi, uni, o);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int c = 0; c < 4; c++) {
            if (k == 0) q0[r][c] = o[r][c];
            acc[r][c] = k == 0 ? o[r][c] : clamp_i((acc[r][c] + o[r][c] + 16448) >> 7, 0, 255);
          }
      }
      if (wp)
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int c = 0; c < 4; c++) acc[r][c] = mc_wp_sample(in, 0, q0[r][c], o[r][c], 255);
#pragma unroll
      for (int r = 0; r < 4; r++) store_row(a.y + (size_t)(y + r) * a.y_stride + x, acc[r], 4, ys_al);
    }
#pragma unroll
    for (int comp = 1; comp <= 2; comp++) {   // chroma 2x2 of Cb and Cr (4:2:0)
      const int x = (in.x >> 1) + 2 * ux, y = (in.y >> 1) + 2 * uy;
      int acc[2][2], o[2][2], q0[2][2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k >= in.nl) break;
        const PicDesc& p = in.pic[k];
        const Plane pl{comp == 1 ? p.cb : p.cr, p.cstride, p.width >> 1, p.height >> 1};
        UnitWin<4, 2> w;
        w.load(pl, ((p.cstride | (int)(uintptr_t)pl.p) & 3) == 0, x + in.cix[k], y + in.ciy[k]);
        w.pred(chroma_taps(in.cfx[k]), 0u, chroma_taps(in.cfy[k]), 0u, uni, o);
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
          for (int c = 0; c < 2; c++) {
            if (k == 0) q0[r][c] = o[r][c];
            acc[r][c] = k == 0 ? o[r][c] : clamp_i((acc[r][c] + o[r][c] + 16448) >> 7, 0, 255);
          }
      }
      if (wp)
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
          for (int c = 0; c < 2; c++) acc[r][c] = mc_wp_sample(in, comp, q0[r][c], o[r][c], 255);
      uint8_t* base = comp == 1 ? a.cb : a.cr;
#pragma unroll
      for (int r = 0; r < 2; r++) store_row(base + (size_t)(y + r) * a.c_stride + x, acc[r], 2, cs_al);
    }
  }
}

// ---- bit depth 10 (the main10 configurations): uint16 planes, int samples -----------------------
// xPredInterBlk at bitDepth 10 (headRoom 4, TComInterpolationFilter.cpp:94-257) in the same
// two-stage form as the 8-bit kernel: with s' = s - 512 the first stage filter<N, ., isFirst,
// !isLast> is h = (sum c s - (8192 << 2)) >> 2 = (sum c s') >> 2 (the identity filter gives
// filterCopy's 16 s'), the second uni (isLast): ((sum c h + 512) >> 10) + 512 clipped to 0..1023,
// bi (!isLast): (sum c h) >> 6, which is HM's 14-bit value for every fraction pair (a zero fraction
// is the identity: (64 h) >> 6 = h, (16 sum c s') >> 6 = (sum c s') >> 2).  TComYuv::addAvg at
// bitDepth 10: (p0 + p1 + 16400) >> 5 clipped (shift 14 + 1 - 10, offset 16 + 2 * 8192).
struct Plane16 {
  const uint16_t* p;
  int stride, w, h;
};
typedef __attribute__((address_space(1))) const uint16_t gu16c;

template <int N, int U>
__device__ __forceinline__ void pred10(const Plane16& pl, int bx, int by, uint32_t hlo, uint32_t hhi, uint32_t vlo,
                                       uint32_t vhi, bool uni, int (&out)[U][U]) {
  constexpr int R = U + N - 1;
  const int x0 = bx - (N / 2 - 1), y0 = by - (N / 2 - 1);
  int h[R][U];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const gu16c* row = (const gu16c*)(pl.p + (size_t)clamp_i(y0 + r, 0, pl.h - 1) * pl.stride);
    int sv[R];
#pragma unroll
    for (int c = 0; c < R; c++) sv[c] = (int)row[clamp_i(x0 + c, 0, pl.w - 1)] - 512;
#pragma unroll
    for (int c = 0; c < U; c++) {
      int acc = 0;
#pragma unroll
      for (int k = 0; k < N; k++) acc += tap_of(hlo, hhi, k) * sv[c + k];
      h[r][c] = acc >> 2;
    }
  }
#pragma unroll
  for (int y = 0; y < U; y++)
#pragma unroll
    for (int c = 0; c < U; c++) {
      int sum = 0;
#pragma unroll
      for (int k = 0; k < N; k++) sum += h[y + k][c] * tap_of(vlo, vhi, k);
      out[y][c] = uni ? clamp_i(((sum + 512) >> 10) + 512, 0, 1023) : (sum >> 6);
    }
}

__global__ __launch_bounds__(kMcBlock) void k_mc10(McArgs a) {
  __shared__ McJobInfo info[kMcJobs];
  __shared__ int first_unit[kMcJobs + 1];
  const int j0 = blockIdx.x * kMcJobs;
  const int t = threadIdx.x;
  if (t < kMcJobs) {   // the job set-up of k_mc
    McJobInfo& in = info[t];
    in.units = 0;
    const int ji = j0 + t;
    if (ji < a.n) {
      const fme_mc_job j = a.jobs[ji];
      if (!mc_job_valid(a, j)) {
        atomicAdd(a.invalid, 1);
      } else {
        int nl = 0, lists[2] = {0, 0};
        if (j.flags & FME_MC_L0) lists[nl++] = 0;
        if (j.flags & FME_MC_L1) lists[nl++] = 1;
        in.wp = (j.flags & FME_MC_WP) ? 1 : 0;
        if (nl == 2 && !in.wp && j.ref_id[0] == j.ref_id[1] && j.mv[0][0] == j.mv[1][0] && j.mv[0][1] == j.mv[1][1]) nl = 1;
        in.nl = nl;
        if (in.wp) mc_wp_setup(a, j, lists, nl, in);
        for (int k = 0; k < nl; k++) {
          const int l = lists[k];
          const PicDesc p = a.pics[j.ref_id[l]];
          int mx = j.mv[l][0], my = j.mv[l][1];
          clip_mv(mx, my, p.width, p.height, j.cu_x, j.cu_y);
          in.lix[k] = mx >> 2;
          in.liy[k] = my >> 2;
          in.lfx[k] = mx & 3;
          in.lfy[k] = my & 3;
          in.cix[k] = mx >> 3;
          in.ciy[k] = my >> 3;
          in.cfx[k] = mx & 7;
          in.cfy[k] = my & 7;
          in.pic[k] = p;
        }
        in.x = j.x;
        in.y = j.y;
        in.ux_n = j.w >> 2;
        in.units = (j.w >> 2) * (j.h >> 2);
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int k = 0; k < kMcJobs; k++) {
      first_unit[k] = acc;
      acc += info[k].units;
    }
    first_unit[kMcJobs] = acc;
  }
  __syncthreads();
  const int total = first_unit[kMcJobs];
  uint16_t* const oy = reinterpret_cast<uint16_t*>(a.y);
  uint16_t* const ocb = reinterpret_cast<uint16_t*>(a.cb);
  uint16_t* const ocr = reinterpret_cast<uint16_t*>(a.cr);
  for (int g = t; g < total; g += kMcBlock) {
    int q = 0;
#pragma unroll
    for (int k = 1; k < kMcJobs; k++) q += g >= first_unit[k] ? 1 : 0;
    const McJobInfo& in = info[q];
    const int u = g - first_unit[q];
    const int ux = u % in.ux_n, uy = u / in.ux_n;
    const bool wp = in.wp != 0;
    const bool uni = in.nl == 1 && !wp;   // weighted prediction filters to the 14-bit values (bi form)
    {   // luma 4x4
      const int x = in.x + 4 * ux, y = in.y + 4 * uy;
      int acc[4][4], o[4][4], q0[4][4];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k >= in.nl) break;
        const PicDesc& p = in.pic[k];
        uint32_t hlo, hhi, vlo, vhi;
        luma_taps(in.lfx[k], hlo, hhi);
        luma_taps(in.lfy[k], vlo, vhi);
        pred10<8, 4>(Plane16{reinterpret_cast<const uint16_t*>(p.luma), p.stride, p.width, p.height}, x + in.lix[k],
                     y + in.liy[k], hlo, hhi, vlo, vhi, uni, o);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int c = 0; c < 4; c++) {
            if (k == 0) q0[r][c] = o[r][c];
            acc[r][c] = k == 0 ? o[r][c] : clamp_i((acc[r][c] + o[r][c] + 16400) >> 5, 0, 1023);
          }
      }
      if (wp)
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
          for (int c = 0; c < 4; c++) acc[r][c] = mc_wp_sample(in, 0, q0[r][c], o[r][c], 1023);
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) oy[(size_t)(y + r) * a.y_stride + x + c] = (uint16_t)acc[r][c];
    }
#pragma unroll
    for (int comp = 1; comp <= 2; comp++) {   // chroma 2x2 of Cb and Cr (4:2:0)
      const int x = (in.x >> 1) + 2 * ux, y = (in.y >> 1) + 2 * uy;
      int acc[2][2], o[2][2], q0[2][2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k >= in.nl) break;
        const PicDesc& p = in.pic[k];
        const Plane16 pl{reinterpret_cast<const uint16_t*>(comp == 1 ? p.cb : p.cr), p.cstride, p.width >> 1,
                         p.height >> 1};
        pred10<4, 2>(pl, x + in.cix[k], y + in.ciy[k], chroma_taps(in.cfx[k]), 0u, chroma_taps(in.cfy[k]), 0u, uni, o);
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
          for (int c = 0; c < 2; c++) {
            if (k == 0) q0[r][c] = o[r][c];
            acc[r][c] = k == 0 ? o[r][c] : clamp_i((acc[r][c] + o[r][c] + 16400) >> 5, 0, 1023);
          }
      }
      if (wp)
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
          for (int c = 0; c < 2; c++) acc[r][c] = mc_wp_sample(in, comp, q0[r][c], o[r][c], 1023);
      uint16_t* base = comp == 1 ? ocb : ocr;
#pragma unroll
      for (int r = 0; r < 2; r++)
#pragma unroll
        for (int c = 0; c < 2; c++) base[(size_t)(y + r) * a.c_stride + x + c] = (uint16_t)acc[r][c];
    }
  }
}

// xGetTemplateCost (TEncSearch.cpp:4397-4436) distortion: clipMv of the candidate, the uni-pred
// luma prediction xPredInterBlk(COMPONENT_Y, ..., bi = false) and getDistPart(DF_SAD) against the
// original (plain SAD at every width: setDistParam(UInt, UInt, DFunc) sets no subsampling,
// TComRdCost.cpp:187-197).  One task per wave: the lanes walk the PU's 4x4 units.
__global__ __launch_bounds__(kMcBlock) void k_amvp_sad(AmvpArgs a) {
  const int task = (int)(blockIdx.x * (kMcBlock / 64) + (threadIdx.x >> 6));
  if (task >= a.n) return;   // wave-uniform
  const int lane = (int)(threadIdx.x & 63);
  const AmvpTask t = a.tasks[task];
  const PicDesc ref = a.pics[t.ref_id], org = a.pics[t.org_id];
  int mx = t.mv_x, my = t.mv_y;
  clip_mv(mx, my, ref.width, ref.height, t.cu_x, t.cu_y);
  uint32_t hlo, hhi, vlo, vhi;
  luma_taps(mx & 3, hlo, hhi);
  luma_taps(my & 3, vlo, vhi);
  const bool al = ((ref.stride | (int)(uintptr_t)ref.luma) & 3) == 0;
  const int uxn = t.w >> 2, units = uxn * (t.h >> 2);
  uint32_t sad = 0;
  for (int u = lane; u < units; u += 64) {
    const int x = t.x + 4 * (u % uxn), y = t.y + 4 * (u / uxn);
    UnitWin<8, 4> w;
    w.load(Plane{ref.luma, ref.stride, ref.width, ref.height}, al, x + (mx >> 2), y + (my >> 2));
    int o[4][4];
    w.pred(hlo, hhi, vlo, vhi, true, o);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint8_t* op = org.luma + (size_t)(y + r) * org.stride + x;
#pragma unroll
      for (int c = 0; c < 4; c++) sad += (uint32_t)abs(o[r][c] - (int)gld8(op + c));
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) sad += (uint32_t)__shfl_xor((int)sad, off, 64);
  if (lane == 0) a.sad[task] = sad;
}

// Device-resident requests (fme_build_bipred_keys_device, a.invalid set): the host checks' equivalent;
// a rejected request is counted once (lane 0) and skipped.
__device__ __forceinline__ bool bi_key_task_ok(const BiKeyArgs& a, const BiKeyTask& t, int lane) {
  if (!a.invalid) return true;
  bool shape = false;
#pragma unroll
  for (int k = 0; k < kNumClasses; k++) shape |= kClassW[k] == t.w && kClassH[k] == t.h;
  bool ok = shape && t.org_id < FME_MAX_PICTURES && t.ref_id < FME_MAX_PICTURES && t.key_off >= 0 &&
            (t.key_off & 3) == 0 && (int64_t)t.key_off + (int64_t)t.w * t.h <= a.n_keys &&
            (t.clip & ~FME_PU_CLIP_BIPRED) == 0;
  if (ok) {
    const PicDesc r = a.pics[t.ref_id], o = a.pics[t.org_id];
    ok = r.luma && o.luma && r.width == o.width && r.height == o.height && t.x + t.w <= o.width &&
         t.y + t.h <= o.height;
  }
  if (!ok && lane == 0) atomicAdd(a.invalid, 1);
  return ok;
}

// xMotionEstimation(bBi) (TEncSearch.cpp:4461-4471): motionCompensation of the other list (luma,
// uni-pred, 8-bit) and TComYuv::removeHighFreq (TComYuv.cpp:411-455) into the key buffer.  One
// task per wave: the lanes walk the PU's 4x4 units.
__global__ __launch_bounds__(kMcBlock) void k_bi_key(BiKeyArgs a) {
  const int task = (int)(blockIdx.x * (kMcBlock / 64) + (threadIdx.x >> 6));
  if (task >= a.n) return;   // wave-uniform
  const int lane = (int)(threadIdx.x & 63);
  const BiKeyTask t = a.tasks[task];
  if (!bi_key_task_ok(a, t, lane)) return;   // wave-uniform
  const PicDesc ref = a.pics[t.ref_id], org = a.pics[t.org_id];
  int mx = t.mv_x, my = t.mv_y;
  clip_mv(mx, my, ref.width, ref.height, t.cu_x, t.cu_y);
  uint32_t hlo, hhi, vlo, vhi;
  luma_taps(mx & 3, hlo, hhi);
  luma_taps(my & 3, vlo, vhi);
  const bool al = ((ref.stride | (int)(uintptr_t)ref.luma) & 3) == 0;
  const int uxn = t.w >> 2, units = uxn * (t.h >> 2);
  for (int u = lane; u < units; u += 64) {
    const int ux = u % uxn, uy = u / uxn;
    const int x = t.x + 4 * ux, y = t.y + 4 * uy;
    UnitWin<8, 4> w;
    w.load(Plane{ref.luma, ref.stride, ref.width, ref.height}, al, x + (mx >> 2), y + (my >> 2));
    int o[4][4];
    w.pred(hlo, hhi, vlo, vhi, true, o);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint8_t* op = org.luma + (size_t)(y + r) * org.stride + x;
      int16_t* kp = a.keys + t.key_off + (size_t)(4 * uy + r) * t.w + 4 * ux;
      int v[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        v[c] = 2 * (int)gld8(op + c) - o[r][c];
        if (t.clip) v[c] = clamp_i(v[c], 0, 255);
      }
      // 4 int16 = 8 bytes; key_off and w are multiples of 4, so the store is 8-byte aligned
      *(uint2*)kp = make_uint2((uint32_t)(uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16),
                               (uint32_t)(uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16));
    }
  }
}

// ---- the producers' luma stages at bit depth 10 (uint16 planes; pred10 is k_mc10's uni-pred luma) --
// xGetTemplateCost's SAD: getDistPart(DF_SAD) at bitDepth 10 sums |d| and shifts the block sum >> 2
// (xGetSAD*: uiSum >> DISTORTION_PRECISION_ADJUSTMENT(bitDepth - 8), TComRdCost.cpp:370-536).
__global__ __launch_bounds__(kMcBlock) void k_amvp_sad10(AmvpArgs a) {
  const int task = (int)(blockIdx.x * (kMcBlock / 64) + (threadIdx.x >> 6));
  if (task >= a.n) return;   // wave-uniform
  const int lane = (int)(threadIdx.x & 63);
  const AmvpTask t = a.tasks[task];
  const PicDesc ref = a.pics[t.ref_id], org = a.pics[t.org_id];
  int mx = t.mv_x, my = t.mv_y;
  clip_mv(mx, my, ref.width, ref.height, t.cu_x, t.cu_y);
  uint32_t hlo, hhi, vlo, vhi;
  luma_taps(mx & 3, hlo, hhi);
  luma_taps(my & 3, vlo, vhi);
  const Plane16 pl{reinterpret_cast<const uint16_t*>(ref.luma), ref.stride, ref.width, ref.height};
  const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
  const int uxn = t.w >> 2, units = uxn * (t.h >> 2);
  uint32_t sad = 0;
  for (int u = lane; u < units; u += 64) {
    const int x = t.x + 4 * (u % uxn), y = t.y + 4 * (u / uxn);
    int o[4][4];
    pred10<8, 4>(pl, x + (mx >> 2), y + (my >> 2), hlo, hhi, vlo, vhi, true, o);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const gu16c* op = (const gu16c*)(ol + (size_t)(y + r) * org.stride + x);
#pragma unroll
      for (int c = 0; c < 4; c++) sad += (uint32_t)abs(o[r][c] - (int)op[c]);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) sad += (uint32_t)__shfl_xor((int)sad, off, 64);
  if (lane == 0) a.sad[task] = sad >> 2;
}

// The bi-pred key at bit depth 10: 2 * org - pred (removeHighFreq), ClipBD to 0..1023 with
// ClipForBiPredMe (TComYuv.cpp:411-455).
__global__ __launch_bounds__(kMcBlock) void k_bi_key10(BiKeyArgs a) {
  const int task = (int)(blockIdx.x * (kMcBlock / 64) + (threadIdx.x >> 6));
  if (task >= a.n) return;   // wave-uniform
  const int lane = (int)(threadIdx.x & 63);
  const BiKeyTask t = a.tasks[task];
  if (!bi_key_task_ok(a, t, lane)) return;   // wave-uniform
  const PicDesc ref = a.pics[t.ref_id], org = a.pics[t.org_id];
  int mx = t.mv_x, my = t.mv_y;
  clip_mv(mx, my, ref.width, ref.height, t.cu_x, t.cu_y);
  uint32_t hlo, hhi, vlo, vhi;
  luma_taps(mx & 3, hlo, hhi);
  luma_taps(my & 3, vlo, vhi);
  const Plane16 pl{reinterpret_cast<const uint16_t*>(ref.luma), ref.stride, ref.width, ref.height};
  const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
  const int uxn = t.w >> 2, units = uxn * (t.h >> 2);
  for (int u = lane; u < units; u += 64) {
    const int ux = u % uxn, uy = u / uxn;
    const int x = t.x + 4 * ux, y = t.y + 4 * uy;
    int o[4][4];
    pred10<8, 4>(pl, x + (mx >> 2), y + (my >> 2), hlo, hhi, vlo, vhi, true, o);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const gu16c* op = (const gu16c*)(ol + (size_t)(y + r) * org.stride + x);
      int16_t* kp = a.keys + t.key_off + (size_t)(4 * uy + r) * t.w + 4 * ux;
      int v[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        v[c] = 2 * (int)op[c] - o[r][c];
        if (t.clip) v[c] = clamp_i(v[c], 0, 1023);
      }
      *(uint2*)kp = make_uint2((uint32_t)(uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16),
                               (uint32_t)(uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16));
    }
  }
}

}  // namespace

hipError_t launch_bi_key(const BiKeyArgs& a, hipStream_t s) {
  const dim3 g((a.n + kMcBlock / 64 - 1) / (kMcBlock / 64));
  if (a.n > 0 && a.bit_depth > 8) hipLaunchKernelGGL(k_bi_key10, g, dim3(kMcBlock), 0, s, a);
  else if (a.n > 0) hipLaunchKernelGGL(k_bi_key, g, dim3(kMcBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_mc(const McArgs& a, hipStream_t s) {
  if (a.n > 0 && a.bit_depth > 8)
    hipLaunchKernelGGL(k_mc10, dim3((a.n + kMcJobs - 1) / kMcJobs), dim3(kMcBlock), 0, s, a);
  else if (a.n > 0)
    hipLaunchKernelGGL(k_mc, dim3((a.n + kMcJobs - 1) / kMcJobs), dim3(kMcBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_amvp_sad(const AmvpArgs& a, hipStream_t s) {
  const dim3 g((a.n + kMcBlock / 64 - 1) / (kMcBlock / 64));
  if (a.n > 0 && a.bit_depth > 8) hipLaunchKernelGGL(k_amvp_sad10, g, dim3(kMcBlock), 0, s, a);
  else if (a.n > 0) hipLaunchKernelGGL(k_amvp_sad, g, dim3(kMcBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace fme
