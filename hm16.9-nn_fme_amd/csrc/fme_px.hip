// fme_px.hip — EMI + FracDIF search for bit depths above 8 (the main10 configurations,
// cfg/encoder_lowdelay_P_main10.cfg:58 InternalBitDepth 10), pixel per lane.
//
// The 8-bit lane kernel (fme_lane.hip) keeps each lane's reference window in VGPRs as s - 128
// bytes and filters with v_dot4_i32_i8; 10-bit samples fit neither.  Here a workgroup takes one
// job at a time and keeps its window, key and first filter stage in LDS as int16; a lane owns a
// pixel (the single-call server's formulation, fme_server.hip, generalised over the bit depth):
//   1. load     window rows -5 .. h+4, cols -5 .. w+4 around the TZ MV (edge-replicated, 16-bit
//               samples) and the key block (original samples, or the job's int16 key block);
//   2. EMI      the 9 integer distortions (SSE with the per-sample (d*d) >> 2 (bd - 8), or SAD12/24/48
//               with the FEN row subsampling, >> (bd - 8)), the square-step decision (TEncSearch.cpp:
//               1324-1377, 1155-1188, 5043-5050), the window re-centred by index;
//   3. planes   xExtDIFUpSamplingH/Q's first stage (filterHor, isFirst, !isLast: shift 6 - headRoom,
//               offset -8192 << shift) of fractional phases 1..3 into LDS, once per job;
//   4. half / quarter  per (candidate, 8x8 tile or four 4x4 tiles) one wave, a lane per pixel: the
//               second stage (filterVer, !isFirst, isLast: shift 6 + headRoom, offset 1 << (shift - 1)
//               + (8192 << 6); filterCopy for fraction 0), key - pred, the Walsh-Hadamard
//               butterflies across lanes (xCalcHADs8x8 / 4x4), every candidate's sum >> (bd - 8)
//               (xGetHADs / xGetSAD, TComRdCost.cpp:1428-1495 with DISTORTION_PRECISION_ADJUSTMENT,
//               TypeDef.h:140-143) plus the MV cost, the first strict minimum in xPatternRefinement's
//               order (TEncSearch.cpp:1591-1645);
//   5. record   the 64-byte fme_result fields the NN tail (k_nn_tail) completes, as the lane kernel
//               writes them.
// Interpolation constants: TComInterpolationFilter.cpp:94-257 (headRoom = max(2, 14 - bitDepth)).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fme_device.h"
#include "fme_xlane.h"

namespace fme {
namespace {
using namespace xlane;

constexpr int kPxNT = 256;
constexpr int kPxWaves = kPxNT / 64;

// tap t (a constant after unrolling) of fraction f, as selects of immediates
__device__ __forceinline__ int px_tap(int f, int t) {
  constexpr int8_t T[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                              {-1, 4, -10, 58, 17, -5, 1, 0},
                              {-1, 4, -11, 40, 40, -11, 4, -1},
                              {0, 1, -5, 17, 58, -10, 4, -1}};
  return f == 0 ? T[0][t] : (f == 1 ? T[1][t] : (f == 2 ? T[2][t] : T[3][t]));
}
// xPatternRefinement's candidate orders (s_acMvRefineH / Q, TEncSearch.cpp:212-236) as 2-bit
// (offset + 1) fields
constexpr int8_t kPxRefH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
constexpr int8_t kPxRefQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};
constexpr uint32_t px_pack(const int8_t (&t)[9][2], int c) {
  uint32_t v = 0;
  for (int k = 0; k < 9; k++) v |= (uint32_t)(t[k][c] + 1) << (2 * k);
  return v;
}
constexpr uint32_t kPxHx = px_pack(kPxRefH, 0), kPxHy = px_pack(kPxRefH, 1);
constexpr uint32_t kPxQx = px_pack(kPxRefQ, 0), kPxQy = px_pack(kPxRefQ, 1);
__device__ __forceinline__ int px_ref(uint32_t packed, int k) { return (int)((packed >> (2 * k)) & 3u) - 1; }

// EMI square positions: 0 centre, then TL, T, TR, L, R, BL, B, BR (xTZ8PointSquareSearch order)
__device__ __forceinline__ constexpr int px_emi_dx(int p) { return (p == 1 || p == 4 || p == 6) ? -1 : ((p == 3 || p == 5 || p == 8) ? 1 : 0); }
__device__ __forceinline__ constexpr int px_emi_dy(int p) { return p >= 1 && p <= 3 ? -1 : (p >= 6 ? 1 : 0); }

__device__ __forceinline__ uint32_t px_eg_bits(int v) {   // TComRdCost.cpp:172-185
  const uint32_t t = v <= 0 ? ((uint32_t)(-v) << 1) + 1u : (uint32_t)v << 1;
  return 2u * (31u - (uint32_t)__clz((int)t)) + 1u;
}
__device__ __forceinline__ uint32_t px_cost(double ml, uint32_t bits) {   // TComRdCost.h:165
  return (uint32_t)((ml * (double)bits) / 65536.0);
}

// Classes 0 .. kPxSmallClasses-1 (fme_device.h kClassW / kClassH: 4x8 .. 16x16) are at most 16
// wide and tall: one wave per job (k_search_px_wave); the larger shapes one workgroup per job.
constexpr int kPxSmallClasses = 10;
constexpr int kPxMaxWin = (64 + 10) * (64 + 10);
constexpr int kPxMaxPlane = (64 + 8) * (64 + 1);
struct PxLds {
  int16_t win[kPxMaxWin];        // rows -5 .. h+4, cols -5 .. w+4 around the TZ MV, stride w + 10
  alignas(16) int16_t key[64 * 64];
  int16_t hp[3][kPxMaxPlane];    // first stage of phases 1..3: rows -4 .. h+3, PU cols -1 .. w-1
  uint32_t e9[9];                // EMI partial sums
  uint32_t cost[2][9];           // per candidate: half, quarter (summed tile transforms)
  uint32_t emi[8];
  int32_t ctl[8];                // ex, ey, n_emi, c, hx, hy, qbest, qk
};

// One (candidate, block group) item: lanes = the group's pixels; quarter-pel offset (ox, oy) from
// the re-centred integer MV (wave-uniform).  Returns the group's summed per-tile transform (8x8:
// (s + 2) >> 2 per tile; 4x4: (s + 1) >> 1 per tile) or SAD, on every lane.
template <int BD, bool SAD, bool B8, class LT>
__device__ __forceinline__ uint32_t px_item(const LT& L, int w, int ws, int ex, int ey, int nb4, int b, int ox,
                                            int oy, int lane) {
  constexpr int HR = 14 - BD < 2 ? 2 : 14 - BD, SH2 = 6 + HR, MAXV = (1 << BD) - 1;
  const int bw8 = w >> 3, bw4 = w >> 2;
  int c, r;
  bool valid = true;
  if constexpr (B8) {
    const int by = b / bw8;
    c = (b - by * bw8) * 8 + (lane & 7);
    r = by * 8 + (lane >> 3);
  } else {
    int blk = b * 4 + (lane >> 4);
    valid = blk < nb4;
    blk = valid ? blk : 0;
    const int by = blk / bw4;
    c = (blk - by * bw4) * 4 + (lane & 3);
    r = by * 4 + ((lane >> 2) & 3);
  }
  const int ix = __builtin_amdgcn_readfirstlane(ox >> 2), fx = __builtin_amdgcn_readfirstlane(ox & 3);
  const int iy = __builtin_amdgcn_readfirstlane(oy >> 2), fy = __builtin_amdgcn_readfirstlane(oy & 3);
  const int x = c + ix, wy0 = r + iy + 4;   // first-stage row of the prediction row (rows -4.. -> 0..)
  int hs[8];
  if (fx == 0) {   // filterCopy, isFirst: (s << headRoom) - 8192
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = ((int)L.win[(wy0 + t - 3 + 1 + ey) * ws + x + 5 + ex] << HR) - 8192;
  } else {
    const int16_t* hp = L.hp[fx - 1] + x + 1;
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = hp[(wy0 + t - 3) * (w + 1)];
  }
  int v;
  if (fy == 0) {   // filterCopy, !isFirst isLast
    v = (hs[3] + 8192 + (1 << (HR - 1))) >> HR;
  } else {
    int s = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) s += px_tap(fy, t) * hs[t];
    v = (s + (1 << (SH2 - 1)) + (8192 << 6)) >> SH2;
  }
  v = min(MAXV, max(0, v));
  int d = valid ? (int)L.key[r * w + c] - v : 0;
  if constexpr (SAD) {
    return wave_sum((uint32_t)abs(d), lane);
  } else if constexpr (B8) {   // xCalcHADs8x8 across the lanes
    d = bfly<32>(bfly<16>(bfly<8>(bfly<4>(bfly<2>(bfly<1>(d, lane), lane), lane), lane), lane), lane);
    return (wave_sum((uint32_t)abs(d), lane) + 2) >> 2;
  } else {                     // four xCalcHADs4x4 per wave
    d = bfly<8>(bfly<4>(bfly<2>(bfly<1>(d, lane), lane), lane), lane);
    uint32_t a = (uint32_t)abs(d);
    a = xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane);
    a = valid ? (a + 1) >> 1 : 0u;
    return xsum<32>(xsum<16>(a, lane), lane);
  }
}

// Two candidates of a 32-pixel PU (8x4 / 4x8: two 4x4 tiles) in one wave: lanes 0..31 score
// candidate offset (ox0, oy0), lanes 32..63 (ox1, oy1), each half a lane per pixel (px_item runs one
// candidate per wave and leaves half the lanes idle for these shapes, 60 % of a frame's PUs).
// Returns the half's summed 4x4 transforms (or SAD) on every lane of the half.
template <int BD, bool SAD, class LT>
__device__ __forceinline__ uint32_t px_item_pair(const LT& L, int w, int ws, int ex, int ey, int ox0, int oy0, int ox1,
                                                 int oy1, int lane) {
  constexpr int HR = 14 - BD < 2 ? 2 : 14 - BD, SH2 = 6 + HR, MAXV = (1 << BD) - 1;
  const int half = lane >> 5, blk = (lane >> 4) & 1;
  const int bw4 = w >> 2;
  const int by = blk / bw4;
  const int c = (blk - by * bw4) * 4 + (lane & 3);
  const int r = by * 4 + ((lane >> 2) & 3);
  const int ox = half ? ox1 : ox0, oy = half ? oy1 : oy0;
  const int ix = ox >> 2, fx = ox & 3, iy = oy >> 2, fy = oy & 3;   // per half
  const int x = c + ix, wy0 = r + iy + 4;
  int hs[8];
  if (fx == 0) {   // filterCopy, isFirst: (s << headRoom) - 8192
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = ((int)L.win[(wy0 + t - 3 + 1 + ey) * ws + x + 5 + ex] << HR) - 8192;
  } else {
    const int16_t* hp = L.hp[fx - 1] + x + 1;
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = hp[(wy0 + t - 3) * (w + 1)];
  }
  int v;
  if (fy == 0) {
    v = (hs[3] + 8192 + (1 << (HR - 1))) >> HR;
  } else {
    int sum = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) sum += px_tap(fy, t) * hs[t];
    v = (sum + (1 << (SH2 - 1)) + (8192 << 6)) >> SH2;
  }
  v = min(MAXV, max(0, v));
  int d = (int)L.key[r * w + c] - v;
  if constexpr (SAD) {
    return xsum<16>(xsum<8>(xsum<4>(xsum<2>(xsum<1>((uint32_t)abs(d), lane), lane), lane), lane), lane);
  } else {   // xCalcHADs4x4 per 16 lanes, the half's two tiles summed
    d = bfly<8>(bfly<4>(bfly<2>(bfly<1>(d, lane), lane), lane), lane);
    uint32_t a = (uint32_t)abs(d);
    a = xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane);
    return xsum<16>((a + 1) >> 1, lane);
  }
}

// One xPatternRefinement stage: every candidate's distortion into L.cost[st] (work items
// (candidate, block group), a contiguous run per wave, one LDS add per candidate touched).
template <int BD, bool SAD, bool B8>
__device__ void px_stage(PxLds& L, int w, int h, int ws, int ex, int ey, int st, int bx0, int by0) {
  const int lane = (int)threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int nb4 = (w >> 2) * (h >> 2);
  const int nb = B8 ? (w >> 3) * (h >> 3) : (nb4 + 3) >> 2;
  const int n_items = 9 * nb, per = (n_items + kPxWaves - 1) / kPxWaves;
  const int i0 = wid * per, i1 = min(n_items, i0 + per);
  uint32_t acc = 0;
  int k = i0 < i1 ? i0 / nb : 0, b = i0 - k * nb;
  int kcur = k;
  for (int item = i0; item < i1; item++, b++) {
    if (b == nb) {
      b = 0;
      k++;
    }
    if (k != kcur) {
      if (lane == 0) atomicAdd(&L.cost[st][kcur], acc);
      acc = 0;
      kcur = k;
    }
    const int ox = bx0 + (st == 0 ? 2 * px_ref(kPxHx, k) : px_ref(kPxQx, k));
    const int oy = by0 + (st == 0 ? 2 * px_ref(kPxHy, k) : px_ref(kPxQy, k));
    acc += px_item<BD, SAD, B8, PxLds>(L, w, ws, ex, ey, nb4, b, ox, oy, lane);
  }
  if (i0 < i1 && lane == 0) atomicAdd(&L.cost[st][kcur], acc);
}

// Wave 0: distortion (>> (bd - 8)) + MV cost of candidate `lane`, the first strict minimum.
template <int BD>
__device__ void px_pick(const PxLds& L, int st, double ml, int mvx, int mvy, int hx, int hy, int px, int py, int& best_k,
                        uint32_t& best) {
  const int lane = (int)threadIdx.x & 63;
  uint32_t tot = 0xFFFFFFFFu;
  if (lane < 9) {
    uint32_t bits;
    if (st == 0)   // cost scale 1 around 2 * mv_int
      bits = px_eg_bits(((2 * mvx + px_ref(kPxHx, lane)) << 1) - px) + px_eg_bits(((2 * mvy + px_ref(kPxHy, lane)) << 1) - py);
    else           // cost scale 0 around 4 * mv_int + 2 * half
      bits = px_eg_bits(4 * mvx + 2 * hx + px_ref(kPxQx, lane) - px) + px_eg_bits(4 * mvy + 2 * hy + px_ref(kPxQy, lane) - py);
    tot = (L.cost[st][lane] >> (BD - 8)) + px_cost(ml, bits);
  }
  int k = lane < 9 ? lane : 64;
  auto step = [&](uint32_t ot, int ok) {
    if (ot < tot || (ot == tot && ok < k)) {
      tot = ot;
      k = ok;
    }
  };
  step((uint32_t)xor_lane<1>((int)tot, lane), xor_lane<1>(k, lane));
  step((uint32_t)xor_lane<2>((int)tot, lane), xor_lane<2>(k, lane));
  step((uint32_t)xor_lane<4>((int)tot, lane), xor_lane<4>(k, lane));
  step((uint32_t)xor_lane<8>((int)tot, lane), xor_lane<8>(k, lane));
  best_k = k;
  best = tot;
}

template <int BD>
__global__ __launch_bounds__(kPxNT) void k_search_px(BatchArgs a, WorkBufs wb) {
  __shared__ PxLds L;
  if (wb.sched->invalid) return;   // rejected batch: the tail marks every record
  constexpr int HR = 14 - BD < 2 ? 2 : 14 - BD, SH1 = 6 - HR, DSH = BD - 8;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  // the PUs wider or taller than 16 (class order from k_scatter; k_search_px_wave takes the rest)
  for (int q = wb.sched->class_off[kPxSmallClasses] + (int)blockIdx.x; q < a.n; q += gridDim.x) {
    const int i = wb.perm[q];
    const fme_job j = a.jobs[i];
    const int w = j.w, h = j.h, ws = w + 10, wh = h + 10;
    // ---- 1. window and key -------------------------------------------------------------------
    {
      const PicDesc ref = a.pics[j.ref_id];
      const uint16_t* rl = reinterpret_cast<const uint16_t*>(ref.luma);
      const int x0 = (int)j.x + j.mv_x - 5, y0 = (int)j.y + j.mv_y - 5;
      // every load of a thread issued before the first store (a load-store loop waits out one
      // memory latency per element); (row, col) stepped by kPxNT elements without divisions
      constexpr int kWinPer = (kPxMaxWin + kPxNT - 1) / kPxNT, kKeyPer = 64 * 64 / kPxNT;
      {
        const int dr = kPxNT / ws, dc = kPxNT - dr * ws;
        int r = tid / ws, cc = tid - r * ws;
        int16_t v[kWinPer];
#pragma unroll
        for (int t = 0; t < kWinPer; t++) {
          if (r < wh) {
            const int yy = min(max(y0 + r, 0), ref.height - 1), xx = min(max(x0 + cc, 0), ref.width - 1);
            v[t] = (int16_t)rl[(size_t)yy * ref.stride + xx];
          }
          cc += dc;
          r += dr + (cc >= ws ? 1 : 0);
          cc -= cc >= ws ? ws : 0;
        }
#pragma unroll
        for (int t = 0; t < kWinPer; t++)
          if (tid + t * kPxNT < ws * wh) L.win[tid + t * kPxNT] = v[t];
      }
      {
        const PicDesc org = a.pics[j.org_id];
        const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
        const int16_t* kb = a.keys + (j.key_offset >= 0 ? j.key_offset : 0);
        const int dr = kPxNT / w, dc = kPxNT - dr * w;
        int r = tid / w, cc = tid - r * w;
        int16_t v[kKeyPer];
#pragma unroll
        for (int t = 0; t < kKeyPer; t++) {
          if (r < h)
            v[t] = j.key_offset >= 0 ? kb[tid + t * kPxNT] : (int16_t)ol[(size_t)(j.y + r) * org.stride + j.x + cc];
          cc += dc;
          r += dr + (cc >= w ? 1 : 0);
          cc -= cc >= w ? w : 0;
        }
#pragma unroll
        for (int t = 0; t < kKeyPer; t++)
          if (tid + t * kPxNT < w * h) L.key[tid + t * kPxNT] = v[t];
      }
      if (tid < 9) L.e9[tid] = 0;
      if (tid < 18) (&L.cost[0][0])[tid] = 0;
    }
    __syncthreads();
    const double ml = a.mlambda[j.lambda_id];
    // ---- 2. EMI square step (or the backups' NN input row) -------------------------------------
    if (j.flags & FME_JOB_NN_IN) {   // takes precedence over FME_JOB_EMI (fme.h)
      if (tid < 9) {
        const uint32_t v = a.nn_in[(size_t)9 * i + tid];
        if (tid < 8) L.emi[tid] = v;
        else L.ctl[3] = (int32_t)v;
      }
      if (tid == 0) {
        L.ctl[0] = L.ctl[1] = 0;
        L.ctl[2] = 8;
      }
    } else if (j.flags & FME_JOB_EMI) {
      // the modified setDistParam's metric (TComRdCost.cpp:200-230): SAD for 12/24/48 wide PUs with
      // xTZSearchHelp's FEN row subsampling (TEncSearch.cpp:1158-1164), SSE otherwise
      const bool sad = w == 12 || w == 24 || w == 48;
      const int sub = (sad && (a.fen == 1 || a.fen == 3) && h > 8) ? 1 : 0;
      uint32_t acc[9];
#pragma unroll
      for (int p = 0; p < 9; p++) acc[p] = 0;
      for (int e = tid; e < w * h; e += kPxNT) {
        const int r = e / w, cc = e - r * w;
        if (sub && (r & 1)) continue;
        const int kv = L.key[e];
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int d = kv - (int)L.win[(r + 5 + px_emi_dy(p)) * ws + cc + 5 + px_emi_dx(p)];
          acc[p] += sad ? (uint32_t)abs(d) : ((uint32_t)(d * d) >> (2 * DSH));
        }
      }
#pragma unroll
      for (int p = 0; p < 9; p++) {
        const uint32_t v = wave_sum(acc[p], lane);
        if (lane == 0) atomicAdd(&L.e9[p], v);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t e9[9];
        for (int p = 0; p < 9; p++) e9[p] = sad ? ((L.e9[p] << sub) >> DSH) : L.e9[p];
        const int sx = j.mv_x, sy = j.mv_y;
        auto cost_at = [&](int x, int y) {   // cost scale 2 (full-pel MV against the quarter-pel predictor)
          return px_cost(ml, px_eg_bits((x << 2) - j.mvp_x) + px_eg_bits((y << 2) - j.mvp_y));
        };
        uint32_t best = e9[0] + cost_at(sx, sy), best_cost = best - e9[0];
        int bx = sx, by = sy, n = 0;
        const bool top = sy - 1 >= j.lt_y, bot = sy + 1 <= j.rb_y, left = sx - 1 >= j.lt_x, right = sx + 1 <= j.rb_x;
        for (int p = 1; p <= 8; p++) {
          const int dx = px_emi_dx(p), dy = px_emi_dy(p);
          const bool ok = (dy == -1 ? top : (dy == 1 ? bot : true)) && (dx == -1 ? left : (dx == 1 ? right : true));
          if (!ok) continue;
          const uint32_t d = e9[p];
          L.emi[n++] = d;
          if (d < best) {
            const uint32_t cst = cost_at(sx + dx, sy + dy);
            if (d + cst < best) {
              best = d + cst;
              best_cost = cst;
              bx = sx + dx;
              by = sy + dy;
            }
          }
        }
        for (int s = n; s < 8; s++) L.emi[s] = 0;
        L.ctl[0] = bx - sx;
        L.ctl[1] = by - sy;
        L.ctl[2] = n;
        L.ctl[3] = (int32_t)(best - best_cost);
      }
    } else if (tid < 8) {
      L.emi[tid] = 0;
      if (tid == 0) L.ctl[0] = L.ctl[1] = L.ctl[2] = L.ctl[3] = 0;
    }
    __syncthreads();
    const int ex = L.ctl[0], ey = L.ctl[1];
    const int mvx = j.mv_x + ex, mvy = j.mv_y + ey;
    // ---- 3. first filter stage of phases 1..3 (xExtDIFUpSamplingH/Q's m_filteredBlockTmp) -------
    {
      const int cols = w + 1, plane = (h + 8) * cols;
      for (int e = tid; e < 3 * plane; e += kPxNT) {
        const int f = e / plane, jj = e - f * plane;
        const int wy = jj / cols, xr = jj - wy * cols;
        const int16_t* row = L.win + (wy + 1 + ey) * ws + xr + 1 + ex;
        int s = 0;
#pragma unroll
        for (int t = 0; t < 8; t++) s += px_tap(f + 1, t) * (int)row[t];
        L.hp[f][jj] = (int16_t)((s - 8192 * (1 << SH1)) >> SH1);
      }
    }
    __syncthreads();
    // ---- 4. half and quarter stages ------------------------------------------------------------
    const bool use_sad = !a.use_hadamard || (j.flags & FME_JOB_LOSSLESS);
    const bool b8 = (w & 7) == 0 && (h & 7) == 0;
    auto stage = [&](int st, int bx0, int by0) {
      if (use_sad)
        px_stage<BD, true, false>(L, w, h, ws, ex, ey, st, bx0, by0);
      else if (b8)
        px_stage<BD, false, true>(L, w, h, ws, ex, ey, st, bx0, by0);
      else
        px_stage<BD, false, false>(L, w, h, ws, ex, ey, st, bx0, by0);
    };
    stage(0, 0, 0);
    __syncthreads();
    if (tid < 64) {
      int k;
      uint32_t best;
      px_pick<BD>(L, 0, ml, mvx, mvy, 0, 0, j.mvp_x, j.mvp_y, k, best);
      if (tid == 0) {
        L.ctl[4] = px_ref(kPxHx, k);
        L.ctl[5] = px_ref(kPxHy, k);
      }
    }
    __syncthreads();
    const int hx = L.ctl[4], hy = L.ctl[5];
    stage(1, 2 * hx, 2 * hy);
    __syncthreads();
    // ---- 5. the record (fme_result bytes 0..63; the tail adds mv, cost, bits, class, status) ----
    if (tid < 64) {
      int k;
      uint32_t best;
      px_pick<BD>(L, 1, ml, mvx, mvy, hx, hy, j.mvp_x, j.mvp_y, k, best);
      if (tid < 4) {
        uint4 q;
        if (tid == 0) {
          q = make_uint4((uint32_t)(uint16_t)mvx | ((uint32_t)(uint16_t)mvy << 16), 0u,
                         (uint32_t)(uint8_t)hx | ((uint32_t)(uint8_t)hy << 8) | ((uint32_t)(uint8_t)px_ref(kPxQx, k) << 16) |
                             ((uint32_t)(uint8_t)px_ref(kPxQy, k) << 24),
                         best);
        } else if (tid == 1) {
          q = make_uint4(0u, 0u, (uint32_t)L.ctl[3], L.emi[0]);
        } else if (tid == 2) {
          q = make_uint4(L.emi[1], L.emi[2], L.emi[3], L.emi[4]);
        } else {
          q = make_uint4(L.emi[5], L.emi[6], L.emi[7], (uint32_t)L.ctl[2]);
        }
        reinterpret_cast<uint4*>(a.res + i)[tid] = q;
      }
    }
    __syncthreads();   // the next job rewrites the LDS
  }
}

// ---- one wave per job: the PUs of at most 16 x 16 -------------------------------------------------
// The same five steps as k_search_px with the wave's own LDS slice and no workgroup barrier: the
// 4x8 / 8x4 / 8x8 majority of a frame's PUs kept a 256-lane workgroup and eight barriers busy per
// job (17 us of workgroup time per job on the 1080p main10 frame).  Sums are wave reductions
// (every lane holds every total), so the EMI decision and the candidate picks run on all lanes.
constexpr int kPxSW = 16;                                   // largest side of the wave kernel's PUs
#ifndef FME_PXW_WAVES   // waves per SIMD of the wave kernel (latency-bound: more waves hide more)
#define FME_PXW_WAVES 6
#endif
struct PxSmall {
  int16_t win[(kPxSW + 10) * (kPxSW + 10)];
  alignas(16) int16_t key[kPxSW * kPxSW];
  int16_t hp[3][(kPxSW + 8) * (kPxSW + 1)];
};
__device__ __forceinline__ void px_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int BD, bool SAD, bool B8>
__device__ __forceinline__ void px_wave_costs(const PxSmall& L, int w, int h, int ws, int ex, int ey, int st, int bx0,
                                              int by0, int lane, uint32_t (&cost)[9]) {
  if constexpr (!B8) {
    if (w * h == 32) {   // 8x4 / 4x8: candidates two at a time, one per half-wave
#pragma unroll
      for (int k = 0; k < 9; k += 2) {
        const int k1 = k + 1 < 9 ? k + 1 : k;
        const int ox0 = bx0 + (st == 0 ? 2 * px_ref(kPxHx, k) : px_ref(kPxQx, k));
        const int oy0 = by0 + (st == 0 ? 2 * px_ref(kPxHy, k) : px_ref(kPxQy, k));
        const int ox1 = bx0 + (st == 0 ? 2 * px_ref(kPxHx, k1) : px_ref(kPxQx, k1));
        const int oy1 = by0 + (st == 0 ? 2 * px_ref(kPxHy, k1) : px_ref(kPxQy, k1));
        const uint32_t sum = px_item_pair<BD, SAD, PxSmall>(L, w, ws, ex, ey, ox0, oy0, ox1, oy1, lane);
        cost[k] = (uint32_t)__builtin_amdgcn_readlane((int)sum, 0);
        if (k + 1 < 9) cost[k + 1] = (uint32_t)__builtin_amdgcn_readlane((int)sum, 32);
      }
      return;
    }
  }
  const int nb4 = (w >> 2) * (h >> 2);
  const int nb = B8 ? (w >> 3) * (h >> 3) : (nb4 + 3) >> 2;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int ox = bx0 + (st == 0 ? 2 * px_ref(kPxHx, k) : px_ref(kPxQx, k));
    const int oy = by0 + (st == 0 ? 2 * px_ref(kPxHy, k) : px_ref(kPxQy, k));
    uint32_t acc = 0;
    for (int b = 0; b < nb; b++) acc += px_item<BD, SAD, B8, PxSmall>(L, w, ws, ex, ey, nb4, b, ox, oy, lane);
    cost[k] = acc;
  }
}

template <int BD>
__global__ __launch_bounds__(kPxNT) __attribute__((amdgpu_waves_per_eu(FME_PXW_WAVES))) void k_search_px_wave(BatchArgs a, WorkBufs wb) {
  __shared__ PxSmall Ls[kPxWaves];
  if (wb.sched->invalid) return;
  constexpr int HR = 14 - BD < 2 ? 2 : 14 - BD, SH1 = 6 - HR, DSH = BD - 8;
  const int lane = (int)threadIdx.x & 63, wid = (int)threadIdx.x >> 6;
  PxSmall& L = Ls[wid];
  const int n_small = wb.sched->class_off[kPxSmallClasses];
  for (int q = (int)blockIdx.x * kPxWaves + wid; q < n_small; q += (int)gridDim.x * kPxWaves) {
    const int i = __builtin_amdgcn_readfirstlane(wb.perm[q]);
    const fme_job j = a.jobs[i];
    const int w = j.w, h = j.h, ws = w + 10, wh = h + 10;
    // ---- 1. window and key (rows of the window per pass: 64 / ws) ----
    {
      const PicDesc ref = a.pics[j.ref_id];
      const uint16_t* rl = reinterpret_cast<const uint16_t*>(ref.luma);
      const int x0 = (int)j.x + j.mv_x - 5, y0 = (int)j.y + j.mv_y - 5;
      // all of a lane's loads issued before its first store (one memory latency per job, not one
      // per row): window rows lr, lr + rpp, ... (at most 13), key rows kr, kr + krp, ... (at most 4)
      const int rpp = 64 / ws, lr = lane / ws, lc = lane - lr * ws;
      const int xx = min(max(x0 + lc, 0), ref.width - 1);
      constexpr int kWinRows = (kPxSW + 10 + 1) / 2;   // ws >= 14 -> rpp <= 4; ws = 26 -> rpp = 2
      int16_t wv[kWinRows];
#pragma unroll
      for (int t = 0; t < kWinRows; t++) {
        const int r = lr + t * rpp;
        if (lr < rpp && r < wh) wv[t] = (int16_t)rl[(size_t)min(max(y0 + r, 0), ref.height - 1) * ref.stride + xx];
      }
      const int kr = lane / w, kc = lane - kr * w, krp = 64 / w;
      const PicDesc org = a.pics[j.org_id];
      const uint16_t* ol = reinterpret_cast<const uint16_t*>(org.luma);
      const int16_t* kb = a.keys + (j.key_offset >= 0 ? j.key_offset : 0);
      int16_t kv4[4];
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int r = kr + t * krp;
        if (kr < krp && r < h)
          kv4[t] = j.key_offset >= 0 ? kb[r * w + kc] : (int16_t)ol[(size_t)(j.y + r) * org.stride + j.x + kc];
      }
#pragma unroll
      for (int t = 0; t < kWinRows; t++) {
        const int r = lr + t * rpp;
        if (lr < rpp && r < wh) L.win[r * ws + lc] = wv[t];
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int r = kr + t * krp;
        if (kr < krp && r < h) L.key[r * w + kc] = kv4[t];
      }
    }
    px_wave_sync();
    const double ml = a.mlambda[j.lambda_id];
    // ---- 2. EMI square step (or the backups' NN input row) ----
    int ex = 0, ey = 0, n_emi = 0;
    uint32_t cval = 0, emi[8];
#pragma unroll
    for (int p = 0; p < 8; p++) emi[p] = 0;
    if (j.flags & FME_JOB_NN_IN) {   // takes precedence over FME_JOB_EMI (fme.h)
      const uint32_t* row = a.nn_in + (size_t)9 * i;
#pragma unroll
      for (int p = 0; p < 8; p++) emi[p] = row[p];
      cval = row[8];
      n_emi = 8;
    } else if (j.flags & FME_JOB_EMI) {
      const bool sad = w == 12 || w == 24 || w == 48;
      const int sub = (sad && (a.fen == 1 || a.fen == 3) && h > 8) ? 1 : 0;
      uint32_t e9[9];
#pragma unroll
      for (int p = 0; p < 9; p++) e9[p] = 0;
      for (int e = lane; e < w * h; e += 64) {
        const int r = e / w, cc = e - r * w;
        if (sub && (r & 1)) continue;
        const int kv = L.key[e];
#pragma unroll
        for (int p = 0; p < 9; p++) {
          const int d = kv - (int)L.win[(r + 5 + px_emi_dy(p)) * ws + cc + 5 + px_emi_dx(p)];
          e9[p] += sad ? (uint32_t)abs(d) : ((uint32_t)(d * d) >> (2 * DSH));
        }
      }
#pragma unroll
      for (int p = 0; p < 9; p++) {
        const uint32_t v = wave_sum(e9[p], lane);
        e9[p] = sad ? ((v << sub) >> DSH) : v;
      }
      const int sx = j.mv_x, sy = j.mv_y;
      auto cost_at = [&](int x, int y) {   // cost scale 2 (full-pel MV against the quarter-pel predictor)
        return px_cost(ml, px_eg_bits((x << 2) - j.mvp_x) + px_eg_bits((y << 2) - j.mvp_y));
      };
      uint32_t best = e9[0] + cost_at(sx, sy), best_cost = best - e9[0];
      int bx = sx, by = sy;
      const bool top = sy - 1 >= j.lt_y, bot = sy + 1 <= j.rb_y, left = sx - 1 >= j.lt_x, right = sx + 1 <= j.rb_x;
#pragma unroll
      for (int p = 1; p <= 8; p++) {
        const int dx = px_emi_dx(p), dy = px_emi_dy(p);
        const bool ok = (dy == -1 ? top : (dy == 1 ? bot : true)) && (dx == -1 ? left : (dx == 1 ? right : true));
        if (!ok) continue;
        const uint32_t d = e9[p];
#pragma unroll
        for (int s = 0; s < 8; s++)   // emi[n_emi++] = d with static register indices
          if (s == n_emi) emi[s] = d;
        n_emi++;
        if (d < best) {
          const uint32_t cst = cost_at(sx + dx, sy + dy);
          if (d + cst < best) {
            best = d + cst;
            best_cost = cst;
            bx = sx + dx;
            by = sy + dy;
          }
        }
      }
      ex = bx - sx;
      ey = by - sy;
      cval = best - best_cost;
    }
    const int mvx = j.mv_x + ex, mvy = j.mv_y + ey;
    // ---- 3. first filter stage of phases 1..3, row by row ----
    {
      const int cols = w + 1, rows = h + 8, rpp = 64 / cols, lr = lane / cols, lc = lane - lr * cols;
      if (lr < rpp)
        for (int f = 0; f < 3; f++)
          for (int wy = lr; wy < rows; wy += rpp) {
            const int16_t* row = L.win + (wy + 1 + ey) * ws + lc + 1 + ex;
            int s = 0;
#pragma unroll
            for (int t = 0; t < 8; t++) s += px_tap(f + 1, t) * (int)row[t];
            L.hp[f][wy * cols + lc] = (int16_t)((s - 8192 * (1 << SH1)) >> SH1);
          }
    }
    px_wave_sync();
    // ---- 4. half and quarter stages, the first strict minimum in xPatternRefinement's order ----
    const bool use_sad = !a.use_hadamard || (j.flags & FME_JOB_LOSSLESS);
    const bool b8 = (w & 7) == 0 && (h & 7) == 0;
    uint32_t cost[9];
    auto stage = [&](int st, int bx0, int by0) {
      if (use_sad)
        px_wave_costs<BD, true, false>(L, w, h, ws, ex, ey, st, bx0, by0, lane, cost);
      else if (b8)
        px_wave_costs<BD, false, true>(L, w, h, ws, ex, ey, st, bx0, by0, lane, cost);
      else
        px_wave_costs<BD, false, false>(L, w, h, ws, ex, ey, st, bx0, by0, lane, cost);
    };
    auto pick = [&](int st, int hx, int hy, uint32_t& best) -> int {
      int bk = 0;
      best = 0xFFFFFFFFu;
#pragma unroll
      for (int k = 0; k < 9; k++) {
        uint32_t bits;
        if (st == 0)   // cost scale 1 around 2 * mv_int
          bits = px_eg_bits(((2 * mvx + px_ref(kPxHx, k)) << 1) - j.mvp_x) +
                 px_eg_bits(((2 * mvy + px_ref(kPxHy, k)) << 1) - j.mvp_y);
        else           // cost scale 0 around 4 * mv_int + 2 * half
          bits = px_eg_bits(4 * mvx + 2 * hx + px_ref(kPxQx, k) - j.mvp_x) +
                 px_eg_bits(4 * mvy + 2 * hy + px_ref(kPxQy, k) - j.mvp_y);
        const uint32_t tot = (cost[k] >> DSH) + px_cost(ml, bits);
        if (tot < best) {
          best = tot;
          bk = k;
        }
      }
      return bk;
    };
    uint32_t hbest, qbest;
    stage(0, 0, 0);
    const int hk = pick(0, 0, 0, hbest);
    const int hx = px_ref(kPxHx, hk), hy = px_ref(kPxHy, hk);
    stage(1, 2 * hx, 2 * hy);
    const int qk = pick(1, hx, hy, qbest);
    (void)hbest;
    // ---- 5. the record (fme_result bytes 0..63; the tail adds mv, cost, bits, class, status) ----
    if (lane < 4) {
      uint4 o;
      if (lane == 0)
        o = make_uint4((uint32_t)(uint16_t)mvx | ((uint32_t)(uint16_t)mvy << 16), 0u,
                       (uint32_t)(uint8_t)hx | ((uint32_t)(uint8_t)hy << 8) | ((uint32_t)(uint8_t)px_ref(kPxQx, qk) << 16) |
                           ((uint32_t)(uint8_t)px_ref(kPxQy, qk) << 24),
                       qbest);
      else if (lane == 1)
        o = make_uint4(0u, 0u, cval, emi[0]);
      else if (lane == 2)
        o = make_uint4(emi[1], emi[2], emi[3], emi[4]);
      else
        o = make_uint4(emi[5], emi[6], emi[7], (uint32_t)n_emi);
      reinterpret_cast<uint4*>(a.res + i)[lane] = o;
    }
    px_wave_sync();   // the next job rewrites this wave's LDS
  }
}

}  // namespace

// Workgroups of the pixel kernel: three fit a CU (47 KB of LDS each), persistent over the jobs.
hipError_t launch_search_px(const BatchArgs& a, const WorkBufs& w, int bit_depth, hipStream_t s, hipStream_t s_big) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    cus = cu_count(dev);
  }
  if (a.n <= 0) return hipSuccess;
  if (bit_depth != 10) return hipErrorInvalidValue;
  // the small PUs, a wave each (17 KB of LDS per workgroup), then the larger ones, a workgroup each
  // (s_big: another stream for the second; side by side they took 11.5 ms per 1080p frame against
  // 10.5 in series, profiles/r06_ab.log, so the batch passes none)
  const int wave_blocks = (int)std::min<long long>((a.n + kPxWaves - 1) / kPxWaves, 8LL * cus);
  hipLaunchKernelGGL(k_search_px_wave<10>, dim3(wave_blocks), dim3(kPxNT), 0, s, a, w);
  const int blocks = (int)std::min<long long>(a.n, 3LL * cus);
  hipLaunchKernelGGL(k_search_px<10>, dim3(blocks), dim3(kPxNT), 0, s_big ? s_big : s, a, w);
  return hipGetLastError();
}

}  // namespace fme
