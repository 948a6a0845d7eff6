// fme_server.hip — the single-call server behind fme_frac_dif_single and fme_nn_pred_single.
//
// TEncSearch calls xPatternSearchFracDIF (TEncSearch.cpp:5232-5269) and NN_pred (85-204) once per
// PU, so the drop-in entry points are latency-bound: a kernel launch plus its completion costs
// more than the work.  Instead one workgroup stays resident while calls keep coming: it polls a
// request word in pinned, device-mapped host memory (SrvBox, fme_device.h), serves the call with
// all 16 of its waves, writes the answer back to host memory and releases a completion word the
// host spins on.  It exits after kSrv idle time without a request, after its lifetime, or when
// the host sets `stop`, and says so in `stopped` (the instance's epoch); the host relaunches it on
// the next call (fme_api.cpp srv_call), so no wave outlives its process by more than the idle
// limit and a batch queued behind it on a shared hardware queue waits at most that long.
//
// FracDIF is restated latency-first: a lane per pixel of an 8x8 block (or of four 4x4 blocks), a
// wave per (candidate, block), the separable filter's first stage for the three fractional phases
// computed once into LDS, SATD butterflies across lanes.  Same arithmetic as the batch kernel and
// the oracle (orc_frac_dif): bit-exact.
#include "fme_device.h"
#include "fme_xlane.h"

namespace fme {
namespace {

constexpr int kSrvThreads = 1024;

// TComInterpolationFilter::m_lumaFilter (TComInterpolationFilter.cpp:57-63): tap t (a constant
// after unrolling) of fraction f, as selects of immediates (no memory load in the filter loops).
__device__ __forceinline__ int luma_tap(int f, int t) {
  constexpr int8_t T[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                              {-1, 4, -10, 58, 17, -5, 1, 0},
                              {-1, 4, -11, 40, 40, -11, 4, -1},
                              {0, 1, -5, 17, 58, -10, 4, -1}};
  return f == 0 ? T[0][t] : (f == 1 ? T[1][t] : (f == 2 ? T[2][t] : T[3][t]));
}
// xPatternRefinement's candidate orders (TEncSearch.cpp:1591-1645 over s_acMvRefineH / Q)
// packed as 2-bit (offset + 1) fields so that candidate k's offset is a shift of an immediate,
// not a constant-memory load in the candidate loop
constexpr int8_t kSrvRefH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
constexpr int8_t kSrvRefQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};
constexpr uint32_t pack_ref(const int8_t (&t)[9][2], int c) {
  uint32_t v = 0;
  for (int k = 0; k < 9; k++) v |= (uint32_t)(t[k][c] + 1) << (2 * k);
  return v;
}
constexpr uint32_t kRefHx = pack_ref(kSrvRefH, 0), kRefHy = pack_ref(kSrvRefH, 1);
constexpr uint32_t kRefQx = pack_ref(kSrvRefQ, 0), kRefQy = pack_ref(kSrvRefQ, 1);
__device__ __forceinline__ int ref_of(uint32_t packed, int k) { return (int)((packed >> (2 * k)) & 3u) - 1; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16 bytes of host memory in one request, past the caches
__device__ __forceinline__ u32x4 load_block(const uint32_t* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// two such blocks, both requests in flight before the wait
__device__ __forceinline__ void load_pair(const uint32_t* p, const uint32_t* q, u32x4& a, u32x4& b) {
  asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\tglobal_load_dwordx4 %1, %3, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=&v"(a), "=&v"(b) : "v"(p), "v"(q) : "memory");
}
__device__ __forceinline__ void store_block(uint32_t* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void sys_store_release(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

using namespace xlane;   // xor_lane, bfly, xsum (fme_xlane.h)

// TComRdCost::xGetExpGolombNumberOfBits (TComRdCost.cpp:172-185): 2 * floor(log2 t) + 1
__device__ __forceinline__ uint32_t eg_bits_d(int v) {
  const uint32_t t = v <= 0 ? ((uint32_t)(-v) << 1) + 1u : (uint32_t)v << 1;
  return 2u * (31u - (uint32_t)__clz((int)t)) + 1u;
}

struct SrvLds {
  float nn[kNnPkFloats];
  alignas(16) int16_t key[64 * 64];
  int16_t hp[3][72 * 65];       // first filter stage, fractional phase 1..3, columns -1 .. w-1
  alignas(16) uint8_t win[72 * 72 + 16];
  uint32_t cost[2][16];           // per candidate: half stage, quarter stage
  int32_t ctl[10];              // stop, seq, kind, w, h, mvp_x, mvp_y, sad, tagged, marks
  uint32_t nn_in[12];
  double ml;
  int32_t sel[2];               // half-stage best (hx, hy)
  uint32_t ans[2];              // the answer (SrvBox::res[1..2])
  uint32_t mark[4];             // FracDIF checkpoints (ticks since the request read): payload in LDS,
                                // first stage, half distortions, quarter distortions
};

// Distortion of block group b of the PU at quarter-pel offset (ox, oy) from the integer MV (wave-
// uniform), lanes = the group's pixels: 8x8 SATD, four 4x4 SATDs or SAD, summed over the wave.
template <bool SAD, bool B8>
__device__ __forceinline__ uint32_t item_dist(const SrvLds& L, int w, int nb4, int b, int ox, int oy, int lane) {
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
  // the candidate's phases are wave-uniform: scalar branches, taps as immediates
  const int ix = __builtin_amdgcn_readfirstlane(ox >> 2), fx = __builtin_amdgcn_readfirstlane(ox & 3);
  const int iy = __builtin_amdgcn_readfirstlane(oy >> 2), fy = __builtin_amdgcn_readfirstlane(oy & 3);
  const int x = c + ix, wy0 = r + iy + 4;
  // first-stage samples at window rows wy0 - 3 .. wy0 + 4: the 14-bit values m_filteredBlockTmp
  // holds (filterHor with isLast false; filterCopy's isFirst branch for fraction 0)
  int hs[8];
  if (fx == 0) {
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = ((int)L.win[(wy0 + t - 3) * (w + 8) + x + 4] << 6) - 8192;
  } else {
    const int16_t* hp = L.hp[fx - 1] + x + 1;
#pragma unroll
    for (int t = 0; t < 8; t++) hs[t] = hp[(wy0 + t - 3) * (w + 1)];
  }
  int v;
  if (fy == 0) {
    v = (hs[3] + 8192 + 32) >> 6;                        // filterCopy, !isFirst isLast
  } else {
    int s = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) s += luma_tap(fy, t) * hs[t];
    v = (s + 2048 + (8192 << 6)) >> 12;                  // filter<8, true, false, true>
  }
  v = min(255, max(0, v));
  int d = valid ? (int)L.key[r * w + c] - v : 0;
  uint32_t add;
  if constexpr (SAD) {
    uint32_t a = (uint32_t)abs(d);
    a = xsum<32>(xsum<16>(xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane), lane), lane);
    add = a;
  } else if constexpr (B8) {   // 8x8 Walsh-Hadamard across the lanes, sum |coef|, (s + 2) >> 2 (xCalcHADs8x8)
    d = bfly<32>(bfly<16>(bfly<8>(bfly<4>(bfly<2>(bfly<1>(d, lane), lane), lane), lane), lane), lane);
    uint32_t a = (uint32_t)abs(d);
    a = xsum<32>(xsum<16>(xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane), lane), lane);
    add = (a + 2) >> 2;
  } else {           // four 4x4 blocks per wave, each (s + 1) >> 1 (xCalcHADs4x4)
    d = bfly<8>(bfly<4>(bfly<2>(bfly<1>(d, lane), lane), lane), lane);
    uint32_t a = (uint32_t)abs(d);
    a = xsum<8>(xsum<4>(xsum<2>(xsum<1>(a, lane), lane), lane), lane);
    a = valid ? (a + 1) >> 1 : 0u;
    add = xsum<32>(xsum<16>(a, lane), lane);   // the four blocks' (rounded) sums
  }
  return add;
}

// The 9 candidates of one xPatternRefinement stage: distortion per candidate into L.cost.
// (ox, oy) of candidate k = base + 2 * ref (half) or base + ref (quarter), quarter-pel offsets from
// the integer MV.  Work item (candidate, block) per wave; lanes are the block's pixels.
// SAD: lossless or HADME off; B8: xGetHADs' 8x8 transform (both dimensions multiples of 8).
template <bool SAD, bool B8>
#ifdef FME_SRV_NOINL
__device__ __noinline__
#else
__device__
#endif
void stage_dist(SrvLds& L, int w, int h, bool half, int bx0, int by0) {
  const int lane = (int)threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  constexpr bool b8 = B8;
  const int nb4 = (w >> 2) * (h >> 2);
  const int nb = b8 ? (w >> 3) * (h >> 3) : (nb4 + 3) >> 2;
  // each wave takes a contiguous run of the (candidate-major) items and adds its partial sums to
  // L.cost once per candidate it touched (a run spans at most two candidates once nb >= 16)
  constexpr int NWV = kSrvThreads / 64;
  const int n_items = 9 * nb, per = (n_items + NWV - 1) / NWV;
  const int i0 = wid * per, i1 = min(n_items, i0 + per);
  uint32_t acc = 0;
  int k = i0 < i1 ? i0 / nb : 0, b = i0 - k * nb;   // (candidate, block) of the run's first item
  int kcur = k;
  for (int item = i0; item < i1; item++, b++) {
    if (b == nb) {
      b = 0;
      k++;
    }
    if (k != kcur) {
      if (lane == 0) atomicAdd(&L.cost[half ? 0 : 1][kcur], acc);
      acc = 0;
      kcur = k;
    }
    const int ox = bx0 + (half ? 2 * ref_of(kRefHx, k) : ref_of(kRefQx, k));
    const int oy = by0 + (half ? 2 * ref_of(kRefHy, k) : ref_of(kRefQy, k));
    acc += item_dist<SAD, B8>(L, w, nb4, b, ox, oy, lane);
  }
  if (i0 < i1 && lane == 0) atomicAdd(&L.cost[half ? 0 : 1][kcur], acc);
}

// Wave 0: distortion + MV cost per candidate (lane k), the first strict minimum in candidate order.
__device__ void stage_pick(const SrvLds& L, bool half, int hx, int hy, int& best_k, uint32_t& best) {
  const int lane = (int)threadIdx.x & 63;
  const int px = L.ctl[5], py = L.ctl[6];
  uint32_t tot = 0xFFFFFFFFu;
  if (lane < 9) {
    // getCostOfVectorWithPredictor at cost scale 1 (half) / 0 (quarter), MV relative to the
    // integer MV (the predictor came shifted by 4 * mv_int)
    const int mx = half ? 2 * ref_of(kRefHx, lane) : 2 * hx + ref_of(kRefQx, lane);
    const int my = half ? 2 * ref_of(kRefHy, lane) : 2 * hy + ref_of(kRefQy, lane);
    const uint32_t bits = eg_bits_d(mx - px) + eg_bits_d(my - py);
    tot = L.cost[half ? 0 : 1][lane] + (uint32_t)((L.ml * (double)bits) / 65536.0);
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

__device__ void serve_frac(SrvLds& L, SrvBox* box, uint64_t t_req) {
  const int tid = (int)threadIdx.x;
  const bool marks = L.ctl[9] != 0;   // checkpoints only when asked for (each is a wall-clock read)
  auto mark = [&](int m) {
    if (marks && tid == 0) L.mark[m] = (uint32_t)(wall_clock64() - t_req);
  };
  const int w = L.ctl[3], h = L.ctl[4];
  const bool sad = L.ctl[7] != 0;
  const int pw = w + 8, ph = h + 8;
  // first filter stage of phases 1..3 over window rows 0 .. h+7, PU columns -1 .. w-1
  const int cols = w + 1, plane = ph * cols, span = (plane + 63) & ~63;
  if (3 * span <= 4 * kSrvThreads) {
    // up to 32x32: one output per work item, each phase's plane starting on a wave boundary (the
    // phase is uniform)
    for (int i = tid; i < 3 * span; i += kSrvThreads) {
      const int f = __builtin_amdgcn_readfirstlane(i) / span, j = i - f * span;
      if (j < plane) {
        const int wy = j / cols, xr = j - wy * cols;
        const uint8_t* row = L.win + wy * pw + xr;   // taps at window columns x + 4 - 3 ...
        int s = 0;
#pragma unroll
        for (int t = 0; t < 8; t++) s += luma_tap(f + 1, t) * (int)row[t];
        L.hp[f][j] = (int16_t)(s - 8192);
      }
    }
  } else {   // thread (xr, rr): column xr - 1 of rows rr, rr + 8, ... of the three phases' planes
    const int xr = tid & 127;
    if (xr < cols)
      for (int R = tid >> 7; R < 3 * ph; R += kSrvThreads >> 7) {
        const int f = R >= 2 * ph ? 2 : (R >= ph ? 1 : 0), wy = R - f * ph;
        const uint8_t* row = L.win + wy * pw + xr;
        int s = 0;
#pragma unroll
        for (int t = 0; t < 8; t++) s += luma_tap(f + 1, t) * (int)row[t];
        L.hp[f][wy * cols + xr] = (int16_t)(s - 8192);
      }
  }
  __syncthreads();
  mark(1);
  // one stage's distortions, specialised on the transform
  auto dist = [&](bool half, int bx0, int by0) {
    if (sad)
      stage_dist<true, false>(L, w, h, half, bx0, by0);
    else if ((w & 7) == 0 && (h & 7) == 0)
      stage_dist<false, true>(L, w, h, half, bx0, by0);
    else
      stage_dist<false, false>(L, w, h, half, bx0, by0);
  };
  dist(true, 0, 0);
  __syncthreads();
  mark(2);
  if (tid < 64) {
    int k;
    uint32_t best;
    stage_pick(L, true, 0, 0, k, best);
    if (tid == 0) {
      L.sel[0] = ref_of(kRefHx, k);
      L.sel[1] = ref_of(kRefHy, k);
    }
  }
  __syncthreads();
  const int hx = L.sel[0], hy = L.sel[1];
  dist(false, 2 * hx, 2 * hy);
  __syncthreads();
  mark(3);
  if (tid < 64) {
    int k;
    uint32_t best;
    stage_pick(L, false, hx, hy, k, best);
    if (tid == 0) {
      L.ans[0] = best;
      L.ans[1] = (uint32_t)(uint8_t)hx | ((uint32_t)(uint8_t)hy << 8) | ((uint32_t)(uint8_t)ref_of(kRefQx, k) << 16) |
                 ((uint32_t)(uint8_t)ref_of(kRefQy, k) << 24);
    }
  }
}

// NN_pred (TEncSearch.cpp:85-134) on the packed layout in LDS, in wave 0 alone: lane r owns row r
// of each layer (22, 20 and 49 rows), every row summed in k order without contraction (the batch
// tail's arithmetic, one row at a time instead of row pairs), and a layer's outputs reach every lane
// as scalars (readlane) instead of through LDS and a workgroup barrier.  Every weight a lane needs is
// read from LDS before the first layer starts, so the dependent chains never wait on LDS, and the
// nine input normalisations (a float division each) run once, one per lane, then broadcast.
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// element (row r, k) of a packed [row pairs][K][2] matrix
__device__ __forceinline__ int pk_at(int base, int K, int r, int k) { return base + ((r >> 1) * K + k) * 2 + (r & 1); }
__device__ __forceinline__ float relu1(float s) { return s < 0.0f ? 0.0f : s; }
__device__ void serve_nn(SrvLds& L, SrvBox* box) {
  const int r = (int)threadIdx.x;
  if (r >= 64) return;
  const float* Q = L.nn;
  const uint32_t* v = L.nn_in;   // copied by the polling lanes with the request
  const int t = emb_row_h((int)v[9]) * 8 + emb_row_w((int)v[10]);
  const int r1 = r < 22 ? r : 21, r2 = r < 20 ? r : 19, r3 = r < 49 ? r : 48;
  float w1[9], w2[22], w3[20];
#pragma unroll
  for (int k = 0; k < 9; k++) w1[k] = Q[pk_at(kNnPkW1, 9, r1, k)];
#pragma unroll
  for (int k = 0; k < 22; k++) w2[k] = Q[pk_at(kNnPkW2, 22, r2, k)];
#pragma unroll
  for (int k = 0; k < 20; k++) w3[k] = Q[pk_at(kNnPkW3, 20, r3, k)];
  const float p1 = Q[kNnPkPfx + t * 22 + r1], b1 = Q[kNnPkB1 + r1], g1 = Q[kNnPkG1 + r1], be1 = Q[kNnPkBE1 + r1];
  const float b2 = Q[kNnPkB2 + r2], g2 = Q[kNnPkG2 + r2], be2 = Q[kNnPkBE2 + r2], bo = Q[kNnPkBout + r3];
  // input k in lane k: raw order e0..e3, C, e4..e7
  float xin;
  {
    const int k = r < 9 ? r : 8;
    const int src = k < 4 ? k : (k == 4 ? 8 : k - 1);
    xin = (float)v[src];
    xin = (xin - Q[kNnPkMean + k]) / Q[kNnPkStd + k];
    xin = xin * Q[kNnPkGin + k];
  }
  float x1 = p1;
#pragma unroll
  for (int k = 0; k < 9; k++) x1 = x1 + w1[k] * lane_f(xin, k);
  x1 = relu1(x1 + b1);
  x1 = x1 * g1 + be1;
  float x2 = 0.0f;
#pragma unroll
  for (int k = 0; k < 22; k++) x2 = x2 + w2[k] * lane_f(x1, k);
  x2 = relu1(x2 + b2);
  x2 = x2 * g2 + be2;
  float x3 = 0.0f;
#pragma unroll
  for (int k = 0; k < 20; k++) x3 = x3 + w3[k] * lane_f(x2, k);
  x3 = x3 + bo;
  // the first maximum over the 49 rows (strict >, rows in order) with the batch rule's NaNs (row 0
  // taken first, then strict >): a NaN row 0 wins, a later NaN never
  float bv = -INFINITY;
  int bi = 64;
  if (r < 49) {
    if (x3 != x3) x3 = r == 0 ? INFINITY : -INFINITY;
    bv = x3;
    bi = r;
  }
  // an xor reduction over the 64 lanes (DPP and permlanes, no LDS pipe), ties to the lower row
  auto step = [&](float ov, int oi) {
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  };
  auto xf = [&](auto m, float x) { return __builtin_bit_cast(float, xor_lane<decltype(m)::value>(__builtin_bit_cast(int, x), r)); };
  step(xf(std::integral_constant<int, 1>{}, bv), xor_lane<1>(bi, r));
  step(xf(std::integral_constant<int, 2>{}, bv), xor_lane<2>(bi, r));
  step(xf(std::integral_constant<int, 4>{}, bv), xor_lane<4>(bi, r));
  step(xf(std::integral_constant<int, 8>{}, bv), xor_lane<8>(bi, r));
  step(xf(std::integral_constant<int, 16>{}, bv), xor_lane<16>(bi, r));
  step(xf(std::integral_constant<int, 32>{}, bv), xor_lane<32>(bi, r));
  if (r == 0) {
    L.ans[0] = (uint32_t)bi;
    L.ans[1] = 0;
  }
}

__global__ __launch_bounds__(kSrvThreads) void k_server(SrvBox* box, const float* nn, uint32_t served, uint32_t epoch,
                                                        uint64_t idle_ticks, uint64_t life_ticks) {
  __shared__ SrvLds L;
  const int tid = (int)threadIdx.x;
  if (nn)
    for (int i = tid; i < kNnPkFloats; i += kSrvThreads) L.nn[i] = nn[i];
  const uint64_t t0 = wall_clock64();
  uint64_t last = t0;
  for (;;) {
    if (tid < 64) {   // wave 0 polls: lane l reads request blocks l and l + 64
      const int lane = tid;
      uint32_t seq = served, stop = 0, shape = 0;
      int need = 0;
      u32x4 hd, hb;
      for (;;) {
        load_pair(box->req[lane], box->req[lane + 64], hd, hb);
        seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)hd.x);
        if (seq != served) {
          shape = (uint32_t)__builtin_amdgcn_readfirstlane((int)hd.y);
          need = 4;   // blocks 1..need must all be this call's
          if ((shape & 3u) == kSrvFrac) {
            const int w = (int)((shape >> 8) & 0xFFu) + 1, h = (int)((shape >> 16) & 0xFFu) + 1;
            need = (shape & kSrvTagged) ? 1 + ((w + 8) * (h + 8) + 2 * w * h + 11) / 12 : 1;
          }
          if (__ballot((lane >= 1 && lane <= need && hd.x != seq) || (lane + 64 <= need && hb.x != seq)) == 0) break;
          // a block still carries an older call's sequence word: poll again, but the stop word and the
          // lifetime still end the instance (the host relaunches, or gives up after its own bound)
        }
        stop = (uint32_t)__builtin_amdgcn_readfirstlane((int)hd.w);   // the host's stop word rides in req[0]
        if (stop) break;
        const uint64_t now = wall_clock64();
        if (now - last > idle_ticks || now - t0 > life_ticks) {
          stop = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) {
        L.ctl[0] = (int32_t)stop;
        L.ctl[1] = (int32_t)seq;
        L.ctl[2] = (int32_t)(shape & 3u);                 // kind
        L.ctl[7] = (shape & kSrvSad) ? 1 : 0;
        L.ctl[8] = (shape & kSrvTagged) ? 1 : 0;
        L.ctl[9] = (shape & kSrvMarks) ? 1 : 0;
        L.ctl[3] = (int32_t)((shape >> 8) & 0xFFu) + 1;   // w
        L.ctl[4] = (int32_t)((shape >> 16) & 0xFFu) + 1;  // h
        L.ctl[5] = (int32_t)(int16_t)(hd.z & 0xFFFFu);    // mvp_x - 4 * mv_int_x
        L.ctl[6] = (int32_t)(int16_t)(hd.z >> 16);
      }
      if (!stop && (shape & 3u) == kSrvNn) {
        if (lane >= 1 && lane < 5) {
          L.nn_in[3 * (lane - 1)] = hd.y;
          L.nn_in[3 * (lane - 1) + 1] = hd.z;
          L.nn_in[3 * (lane - 1) + 2] = hd.w;
        }
      } else if (!stop) {
        if (lane < 32) (&L.cost[0][0])[lane] = 0;
        if (lane == 1) L.ml = __builtin_bit_cast(double, (uint64_t)hd.y | ((uint64_t)hd.z << 32));
        if (shape & kSrvTagged) {   // the payload words of blocks 2..need: window, then key
          const int w = (int)((shape >> 8) & 0xFFu) + 1, h = (int)((shape >> 16) & 0xFFu) + 1;
          const int winw = (w + 8) * (h + 8) / 4, totw = winw + w * h / 2;
          uint32_t* wd = reinterpret_cast<uint32_t*>(L.win);
          uint32_t* kd = reinterpret_cast<uint32_t*>(L.key);
          auto put = [&](int blk, const u32x4& v) {
            if (blk < 2 || blk > need) return;
            const uint32_t x[3] = {v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 3; k++) {
              const int q = 3 * (blk - 2) + k;
              if (q < winw) wd[q] = x[k];
              else if (q < totw) kd[q - winw] = x[k];
            }
          };
          put(lane, hd);
          put(lane + 64, hb);
        }
      }
    }
    __syncthreads();
    if (L.ctl[0]) break;
    const uint64_t t_req = wall_clock64();
    if (L.ctl[2] == kSrvFrac) {
      const int w = L.ctl[3], h = L.ctl[4];
      if (L.ctl[8] == 0) {   // not tagged: the window and key, every thread at once (one round trip)
        // 16-byte system-coherent loads: straight from host memory, no cache to invalidate first,
        // one request per block (the window's last block may read into the padding after it)
        const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(box->win);
        u32x4* wdst = reinterpret_cast<u32x4*>(L.win);
        for (int i = tid; i < ((w + 8) * (h + 8) + 15) >> 4; i += kSrvThreads) wdst[i] = load_block(wsrc + 4 * i);
        const uint32_t* ksrc = reinterpret_cast<const uint32_t*>(box->key);
        u32x4* kdst = reinterpret_cast<u32x4*>(L.key);
        for (int i = tid; i < (w * h) >> 3; i += kSrvThreads) kdst[i] = load_block(ksrc + 4 * i);
        __syncthreads();
      }
      if (L.ctl[9] && tid == 0) L.mark[0] = (uint32_t)(wall_clock64() - t_req);
    }
    const uint32_t seq = (uint32_t)L.ctl[1];
    if (L.ctl[2] == kSrvFrac) {
      serve_frac(L, box, t_req);
    } else if (L.ctl[9]) {   // marks: shader-clock cycles and wall ticks of the net itself
      const uint64_t c0 = clock64(), w0 = wall_clock64();
      serve_nn(L, box);
      if (tid == 0) {
        L.mark[0] = (uint32_t)(clock64() - c0);
        L.mark[1] = (uint32_t)(wall_clock64() - w0);
        L.mark[2] = L.mark[3] = 0;
      }
    } else {
      serve_nn(L, box);
    }
    __syncthreads();
    if (tid == 0) {   // the answer and its sequence word in one 16-byte store, past the caches
      if (L.ctl[9]) {
        const u32x4 m = {L.mark[0], L.mark[1], L.mark[2], L.mark[3]};
        store_block(box->marks, m);
      }
      const u32x4 r = {seq, L.ans[0], L.ans[1], (uint32_t)(wall_clock64() - t_req)};
      store_block(box->res, r);
    }
    served = seq;
    last = wall_clock64();
  }
  if (tid == 0) sys_store_release(&box->stopped, epoch);
}

}  // namespace

hipError_t launch_server(SrvBox* box, const float* nn, uint32_t served, uint32_t epoch, uint64_t idle_ticks,
                         uint64_t life_ticks, hipStream_t s) {
  hipLaunchKernelGGL(k_server, dim3(1), dim3(kSrvThreads), 0, s, box, nn, served, epoch, idle_ticks, life_ticks);
  return hipGetLastError();
}

}  // namespace fme
