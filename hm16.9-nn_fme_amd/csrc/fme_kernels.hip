// fme_kernels.hip — CDNA4 (gfx950) kernels of the fractional-pel motion-estimation path.
//
// One batch of PU jobs runs as:
//   classify   per job: PU-shape class, EMI push count; per block: class histogram and the
//              max of the NN "last writer" indices (first pass of a prefix-max scan).
//   scatter    jobs grouped by class (block-aggregated atomics), giving the search tiles.
//   search     one workgroup = one tile of P same-shape PUs: reference window + key in LDS,
//              EMI square step (TEncSearch.cpp:5037-5050), 14-bit horizontal planes,
//              9 half-pel then 9 quarter-pel SATD candidates (xPatternSearchFracDIF,
//              TEncSearch.cpp:5232-5269), first strict minimum of SATD + MV cost.
//   nn_tail    prefix-max over jobs resolves which earlier job last wrote each array_e slot
//              (the reference's stale global state, TEncSearch.cpp:55-57, 198-201), then
//              NN_pred() (85-204) and the xMotionEstimation tail (4586-4597), one lane per job.
//
// Integer arithmetic follows TComInterpolationFilter (14-bit intermediate, offsets -8192 and
// 526336, shift 12) and TComRdCost (xGetHADs 8x8/4x4, SSE, SAD with FEN row subsampling).
// MV cost uses double like TComRdCost::getCost.  The NN is float32 with no contraction
// (this file is compiled with -ffp-contract=off) and sequential-k sums.
#include <hip/hip_runtime.h>

#include "fme_device.h"

namespace fme {

// ---------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int clamp_i(int v, int lo, int hi) { return min(max(v, lo), hi); }

// TComRdCost::xGetExpGolombNumberOfBits (TComRdCost.cpp:172-185) in closed form.
__device__ __forceinline__ uint32_t eg_bits(int v) {
  const uint32_t t = v <= 0 ? ((uint32_t)(-v) << 1) + 1u : ((uint32_t)v << 1);
  return 1u + 2u * (31u - (uint32_t)__clz((int)t));
}

__device__ __forceinline__ uint32_t mv_bits(int x, int y, int scale, int px, int py) {
  return eg_bits((x << scale) - px) + eg_bits((y << scale) - py);
}

// TComRdCost::getCost (TComRdCost.h:165): (Distortion)((lambda * b) / 65536.0).
__device__ __forceinline__ uint32_t mv_cost(double ml, uint32_t bits) {
  return (uint32_t)((ml * (double)bits) / 65536.0);
}

// HEVC luma taps (TComInterpolationFilter.cpp:57-63), selected without memory traffic.
__device__ __forceinline__ void luma_taps(int f, int (&c)[8]) {
  if (f == 1) {
    c[0] = -1; c[1] = 4; c[2] = -10; c[3] = 58; c[4] = 17; c[5] = -5; c[6] = 1; c[7] = 0;
  } else if (f == 2) {
    c[0] = -1; c[1] = 4; c[2] = -11; c[3] = 40; c[4] = 40; c[5] = -11; c[6] = 4; c[7] = -1;
  } else {
    c[0] = 0; c[1] = 1; c[2] = -5; c[3] = 17; c[4] = 58; c[5] = -10; c[6] = 4; c[7] = -1;
  }
}

// Candidate order of xPatternRefinement (s_acMvRefineH / s_acMvRefineQ, TEncSearch.cpp:212-236).
__device__ __forceinline__ int decode_offset(uint32_t code) { return code == 1 ? -1 : (code == 2 ? 1 : 0); }
// 2-bit code per index (0 -> 0, 1 -> -1, 2 -> +1), index 0 in the top pair of 18 bits.
__device__ __forceinline__ int refine_dx(int half, int i) {
  (void)half;  // x components of H9 and Q9 coincide
  return decode_offset((0x666u >> (2 * (8 - i))) & 3u);
}
__device__ __forceinline__ int refine_dy(int half, int i) {
  return decode_offset(((half ? 0x605au : 0x650au) >> (2 * (8 - i))) & 3u);
}

// ---------------------------------------------------------------------------------------
// Hadamard SATD on a tile held in registers (xCalcHADs8x8 / xCalcHADs4x4,
// TComRdCost.cpp:1234-1425).  Any exact WHT factorisation gives the same |coefficients|.
// ---------------------------------------------------------------------------------------
template <int STEP>
__device__ __forceinline__ void wht8(int* v) {
#pragma unroll
  for (int len = 4; len >= 1; len >>= 1)
#pragma unroll
    for (int i = 0; i < 8; i += 2 * len)
#pragma unroll
      for (int j = i; j < i + len; j++) {
        const int a = v[j * STEP], b = v[(j + len) * STEP];
        v[j * STEP] = a + b;
        v[(j + len) * STEP] = a - b;
      }
}

template <int STEP>
__device__ __forceinline__ void wht4(int* v) {
  const int a0 = v[0] + v[3 * STEP], a3 = v[0] - v[3 * STEP];
  const int a1 = v[STEP] + v[2 * STEP], a2 = v[STEP] - v[2 * STEP];
  v[0] = a0 + a1;
  v[2 * STEP] = a0 - a1;
  v[STEP] = a2 + a3;
  v[3 * STEP] = a3 - a2;
}

template <int T>
__device__ __forceinline__ uint32_t satd_tile(int* d) {
  uint32_t s = 0;
  if constexpr (T == 8) {
#pragma unroll
    for (int r = 0; r < 8; r++) wht8<1>(d + r * 8);
#pragma unroll
    for (int c = 0; c < 8; c++) wht8<8>(d + c);
#pragma unroll
    for (int i = 0; i < 64; i++) s += (uint32_t)abs(d[i]);
    return (s + 2) >> 2;
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++) wht4<1>(d + r * 4);
#pragma unroll
    for (int c = 0; c < 4; c++) wht4<4>(d + c);
#pragma unroll
    for (int i = 0; i < 16; i++) s += (uint32_t)abs(d[i]);
    return (s + 1) >> 1;
  }
}

template <int T>
__device__ __forceinline__ uint32_t sad_tile(const int* d) {
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < T * T; i++) s += (uint32_t)abs(d[i]);
  return s;
}

// ---------------------------------------------------------------------------------------
// Per-class geometry of a search tile.
//   window  rows -5..H+4, cols -5..W+4 around the TZ integer MV (EMI +-1, 8-tap -4..+4)
//   planes  fx = 1,2,3 first-stage outputs, rows -4..H+3, cols -1..W-1 around mv_int'
// ---------------------------------------------------------------------------------------
struct PuInfo {
  int32_t job;
  int32_t flags;
  int32_t x, y;
  int32_t ref;
  int32_t wx0, wy0;       // absolute window origin
  int32_t mvx, mvy;       // integer MV (after EMI)
  int32_t ex, ey;         // mv_int' - mv_tz
  int32_t mvp_x, mvp_y;
  int32_t lt_x, lt_y, rb_x, rb_y;
  int32_t had;
  int32_t hx, hy;
  int32_t key_off;
  int32_t pad0;
  double ml;
  uint32_t acc[9];
  uint32_t pad1[3];
};
static_assert(sizeof(PuInfo) % 16 == 0, "PuInfo must keep 16-byte alignment");

template <int W, int H>
struct Geo {
  static constexpr int WS = W + 10;
  static constexpr int WR = H + 10;
  static constexpr int PS = W + 1;
  static constexpr int PR = H + 8;
  static constexpr int WIN = WR * WS;
  static constexpr int KEY = W * H;
  static constexpr int PLANE = PR * PS;
  static constexpr int ELEMS = WIN + KEY + 3 * PLANE;
  static constexpr int BYTES = ((ELEMS * 2) + 15) & ~15;
  static constexpr int T = ((W % 8) == 0 && (H % 8) == 0) ? 8 : 4;
  static constexpr int TILES = (W / T) * (H / T);
  static constexpr int BUDGET = 40 * 1024;
  static constexpr int P0 = BUDGET / (BYTES + (int)sizeof(PuInfo));
  static constexpr int P = P0 < 1 ? 1 : (P0 > 32 ? 32 : P0);
  static constexpr size_t LDS = (size_t)P * (BYTES + sizeof(PuInfo));
  static constexpr int NCH = (PS + 7) / 8;   // 8-column chunks of a plane row
};

template <int W, int H>
struct TileView {
  using G = Geo<W, H>;
  PuInfo* info;
  int16_t* base;
  __device__ TileView(char* lds) {
    info = reinterpret_cast<PuInfo*>(lds);
    base = reinterpret_cast<int16_t*>(lds + G::P * sizeof(PuInfo));
  }
  __device__ int16_t* win(int p) const { return base + (size_t)p * (G::BYTES / 2); }
  __device__ int16_t* key(int p) const { return win(p) + G::WIN; }
  __device__ int16_t* planes(int p) const { return key(p) + G::KEY; }
};

// First-stage (horizontal) value at plane coordinates (pr, pc) for fraction fx:
// fx == 0 is filterCopy's isFirst branch (x << 6) - 8192 (TComInterpolationFilter.cpp:111-124).
template <int W, int H>
__device__ __forceinline__ int stage1(const int16_t* win, const int16_t* planes, int ex, int ey,
                                      int fx, int pr, int pc) {
  using G = Geo<W, H>;
  if (fx == 0) return ((int)win[(1 + ey + pr) * G::WS + 4 + ex + pc] << 6) - 8192;
  return planes[(fx - 1) * G::PLANE + pr * G::PS + pc];
}

// Distortion of one T x T tile of the PU for the candidate at quarter-pel (qx, qy) relative to
// mv_int' (|qx|,|qy| <= 3).  Prediction = second stage of the HEVC luma filter
// (filterVer<8,true,false,true> / filterCopy !isFirst), computed column by column with the
// first-stage column held in registers.
template <int W, int H>
__device__ uint32_t cand_tile_dist(const int16_t* win, const int16_t* planes, const int16_t* key,
                                   int ex, int ey, int qx, int qy, int tile, int had) {
  using G = Geo<W, H>;
  constexpr int T = G::T;
  constexpr int TX = W / T;
  const int ty = tile / TX, tx = tile % TX;
  const int ix = qx >> 2, fx = qx & 3, iy = qy >> 2, fy = qy & 3;
  int d[T * T];
  int cf[8];
  luma_taps(fy, cf);
#pragma unroll
  for (int c = 0; c < T; c++) {
    const int col = tx * T + c;
    const int pc = col + ix + 1;
    if (fy == 0) {
#pragma unroll
      for (int r = 0; r < T; r++) {
        const int row = ty * T + r;
        const int t = stage1<W, H>(win, planes, ex, ey, fx, row + iy + 4, pc);
        const int p = clamp_i((t + 8192 + 32) >> 6, 0, 255);
        d[r * T + c] = (int)key[row * W + col] - p;
      }
    } else {
      int v[T + 7];
#pragma unroll
      for (int m = 0; m < T + 7; m++) v[m] = stage1<W, H>(win, planes, ex, ey, fx, ty * T + iy + 1 + m, pc);
#pragma unroll
      for (int r = 0; r < T; r++) {
        int s = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) s += cf[k] * v[r + k];
        const int p = clamp_i((s + 2048 + (8192 << 6)) >> 12, 0, 255);
        d[r * T + c] = (int)key[(ty * T + r) * W + col] - p;
      }
    }
  }
  return had ? satd_tile<T>(d) : sad_tile<T>(d);
}

// One tile: P PUs of shape W x H.
template <int W, int H>
__device__ void search_tile(const BatchArgs& a, const int32_t* perm, int first, int count, char* lds) {
  using G = Geo<W, H>;
  TileView<W, H> v(lds);
  const int tid = threadIdx.x;

  // ---- descriptors --------------------------------------------------------------------
  if (tid < G::P) {
    PuInfo& in = v.info[tid];
    if (tid < count) {
      const int jid = perm[first + tid];
      const fme_job j = a.jobs[jid];
      in.job = jid;
      in.flags = j.flags;
      in.x = j.x;
      in.y = j.y;
      in.ref = j.ref_id;
      in.wx0 = (int)j.x + j.mv_x - 5;
      in.wy0 = (int)j.y + j.mv_y - 5;
      in.mvx = j.mv_x;
      in.mvy = j.mv_y;
      in.ex = 0;
      in.ey = 0;
      in.mvp_x = j.mvp_x;
      in.mvp_y = j.mvp_y;
      in.lt_x = j.lt_x;
      in.lt_y = j.lt_y;
      in.rb_x = j.rb_x;
      in.rb_y = j.rb_y;
      in.had = (a.use_hadamard && !(j.flags & FME_JOB_LOSSLESS)) ? 1 : 0;
      in.ml = a.mlambda[j.lambda_id];
      in.key_off = j.key_offset;
      in.hx = in.hy = 0;
      // org picture id travels in key_off's place when the key is the picture itself
      in.pad0 = j.org_id;
    } else {
      in.job = -1;
      in.flags = 0;
    }
#pragma unroll
    for (int k = 0; k < 9; k++) in.acc[k] = 0;
  }
  __syncthreads();

  // ---- stage reference window and key into LDS ---------------------------------------
  for (int e = tid; e < count * G::WIN; e += kBlock) {
    const int p = e / G::WIN, rem = e - p * G::WIN;
    const int r = rem / G::WS, c = rem - r * G::WS;
    const PuInfo& in = v.info[p];
    const PicDesc pd = a.pics[in.ref];
    const int ax = clamp_i(in.wx0 + c, 0, pd.width - 1);
    const int ay = clamp_i(in.wy0 + r, 0, pd.height - 1);
    v.win(p)[rem] = pd.luma[(size_t)ay * pd.stride + ax];
  }
  for (int e = tid; e < count * G::KEY; e += kBlock) {
    const int p = e / G::KEY, rem = e - p * G::KEY;
    const int r = rem / W, c = rem - r * W;
    const PuInfo& in = v.info[p];
    int16_t val;
    if (in.key_off >= 0) {
      val = a.keys[(size_t)in.key_off + rem];
    } else {
      const PicDesc pd = a.pics[in.pad0];
      val = pd.luma[(size_t)(in.y + r) * pd.stride + in.x + c];
    }
    v.key(p)[rem] = val;
  }
  __syncthreads();

  // ---- EMI: integer distortion of the centre and its 8 neighbours ---------------------
  // Metric of the modified setDistParam (TComRdCost.cpp:200-230): SSE for W in
  // {4,8,16,32,64}; SAD for 12/24/48, even rows only when FEN in {1,3} and H > 8.
  constexpr bool kSad = (W == 12 || W == 24 || W == 48);
  const int sub = (kSad && (a.fen == 1 || a.fen == 3) && H > 8) ? 1 : 0;
  for (int e = tid; e < count * 9 * H; e += kBlock) {
    const int p = e / (9 * H), rem = e - p * 9 * H;
    const int pos = rem / H, r = rem - pos * H;
    const PuInfo& in = v.info[p];
    if (!(in.flags & FME_JOB_EMI)) continue;
    if (sub && (r & 1)) continue;
    const int dx = pos == 0 ? 0 : ((pos == 1 || pos == 4 || pos == 6) ? -1 : ((pos == 2 || pos == 7) ? 0 : 1));
    const int dy = pos == 0 ? 0 : (pos <= 3 ? -1 : (pos <= 5 ? 0 : 1));
    const int16_t* kr = v.key(p) + r * W;
    const int16_t* wr = v.win(p) + (5 + dy + r) * G::WS + 5 + dx;
    uint32_t s = 0;
#pragma unroll 8
    for (int c = 0; c < W; c++) {
      const int d = (int)kr[c] - (int)wr[c];
      s += kSad ? (uint32_t)abs(d) : (uint32_t)(d * d);
    }
    atomicAdd(&v.info[p].acc[pos], s);
  }
  __syncthreads();

  // EMI square-step decision (xTZ8PointSquareSearch + xTZSearchHelp, TEncSearch.cpp:1324-1377,
  // 1155-1188): push every visited distortion, update the best on d + cost < bestSad.
  if (tid < count) {
    PuInfo& in = v.info[tid];
    fme_result* r = a.res + in.job;
    uint32_t emi[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int n_emi = 0;
    uint32_t cval = 0;
    if (in.flags & FME_JOB_EMI) {
      uint32_t acc[9];
#pragma unroll
      for (int k = 0; k < 9; k++) acc[k] = in.acc[k] << sub;
      const int sx = in.mvx, sy = in.mvy;
      uint32_t best = acc[0] + mv_cost(in.ml, mv_bits(sx, sy, 2, in.mvp_x, in.mvp_y));
      int bx = sx, by = sy;
      const bool top = sy - 1 >= in.lt_y, bot = sy + 1 <= in.rb_y;
      const bool left = sx - 1 >= in.lt_x, right = sx + 1 <= in.rb_x;
      // pos: 1 TL, 2 T, 3 TR, 4 L, 5 R, 6 BL, 7 B, 8 BR
#pragma unroll
      for (int pos = 1; pos <= 8; pos++) {
        const int dx = (pos == 1 || pos == 4 || pos == 6) ? -1 : ((pos == 2 || pos == 7) ? 0 : 1);
        const int dy = pos <= 3 ? -1 : (pos <= 5 ? 0 : 1);
        const bool ok = (dy == -1 ? top : (dy == 1 ? bot : true)) &&
                        (dx == -1 ? left : (dx == 1 ? right : true));
        if (!ok) continue;
        uint32_t d = acc[pos];
        emi[n_emi++] = d;
        if (d < best) {
          d += mv_cost(in.ml, mv_bits(sx + dx, sy + dy, 2, in.mvp_x, in.mvp_y));
          if (d < best) {
            best = d;
            bx = sx + dx;
            by = sy + dy;
          }
        }
      }
      cval = best - mv_cost(in.ml, mv_bits(bx, by, 2, in.mvp_x, in.mvp_y));
      in.ex = bx - sx;
      in.ey = by - sy;
      in.mvx = bx;
      in.mvy = by;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) r->emi[k] = emi[k];
    r->n_emi = (uint8_t)n_emi;
    r->c = cval;
    r->mv_int_x = (int16_t)in.mvx;
    r->mv_int_y = (int16_t)in.mvy;
#pragma unroll
    for (int k = 0; k < 9; k++) in.acc[k] = 0;
  }
  __syncthreads();

  // ---- first-stage planes fx = 1,2,3 around mv_int' ----------------------------------
  // filter<8,false,true,false>: sum - 8192, stored as int16 (TComInterpolationFilter.cpp:196-252).
  for (int e = tid; e < count * G::PR * G::NCH; e += kBlock) {
    const int p = e / (G::PR * G::NCH), rem = e - p * G::PR * G::NCH;
    const int pr = rem / G::NCH, ch = rem - pr * G::NCH;
    const PuInfo& in = v.info[p];
    const int16_t* wrow = v.win(p) + (1 + in.ey + pr) * G::WS;
    const int c0 = 1 + in.ex + ch * 8;
    int w15[15];
#pragma unroll
    for (int m = 0; m < 15; m++) w15[m] = wrow[min(c0 + m, G::WS - 1)];
    int16_t* pl = v.planes(p) + pr * G::PS + ch * 8;
#pragma unroll
    for (int f = 1; f <= 3; f++) {
      int cf[8];
      luma_taps(f, cf);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (ch * 8 + j < G::PS) {
          int s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += cf[k] * w15[j + k];
          pl[(f - 1) * G::PLANE + j] = (int16_t)(s - 8192);
        }
      }
    }
  }
  __syncthreads();

  // ---- half-pel stage: 9 candidates at 2*H9[i] (cost scale 1) --------------------------
  const int items = count * G::TILES;
  for (int e = tid; e < 9 * items; e += kBlock) {
    const int k = e / items, rem = e - k * items;
    const int p = rem / G::TILES, tile = rem - p * G::TILES;
    const PuInfo& in = v.info[p];
    const uint32_t dd = cand_tile_dist<W, H>(v.win(p), v.planes(p), v.key(p), in.ex, in.ey,
                                             2 * refine_dx(1, k), 2 * refine_dy(1, k), tile, in.had);
    atomicAdd(&v.info[p].acc[k], dd);
  }
  __syncthreads();
  if (tid < count) {
    PuInfo& in = v.info[tid];
    uint32_t best = 0xFFFFFFFFu;
    int bi = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int hx = 2 * in.mvx + refine_dx(1, k), hy = 2 * in.mvy + refine_dy(1, k);
      const uint32_t d = in.acc[k] + mv_cost(in.ml, mv_bits(hx, hy, 1, in.mvp_x, in.mvp_y));
      if (d < best) {
        best = d;
        bi = k;
      }
      in.acc[k] = 0;
    }
    in.hx = refine_dx(1, bi);
    in.hy = refine_dy(1, bi);
  }
  __syncthreads();

  // ---- quarter-pel stage: 9 candidates at 2*half + Q9[i] (cost scale 0) --------------
  for (int e = tid; e < 9 * items; e += kBlock) {
    const int k = e / items, rem = e - k * items;
    const int p = rem / G::TILES, tile = rem - p * G::TILES;
    const PuInfo& in = v.info[p];
    const uint32_t dd = cand_tile_dist<W, H>(v.win(p), v.planes(p), v.key(p), in.ex, in.ey,
                                             2 * in.hx + refine_dx(0, k), 2 * in.hy + refine_dy(0, k),
                                             tile, in.had);
    atomicAdd(&v.info[p].acc[k], dd);
  }
  __syncthreads();
  if (tid < count) {
    PuInfo& in = v.info[tid];
    uint32_t best = 0xFFFFFFFFu;
    int bi = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int qx = 4 * in.mvx + 2 * in.hx + refine_dx(0, k);
      const int qy = 4 * in.mvy + 2 * in.hy + refine_dy(0, k);
      const uint32_t d = in.acc[k] + mv_cost(in.ml, mv_bits(qx, qy, 0, in.mvp_x, in.mvp_y));
      if (d < best) {
        best = d;
        bi = k;
      }
    }
    fme_result* r = a.res + in.job;
    r->half_x = (int8_t)in.hx;
    r->half_y = (int8_t)in.hy;
    r->qtr_x = (int8_t)refine_dx(0, bi);
    r->qtr_y = (int8_t)refine_dy(0, bi);
    r->frac_cost = best;
  }
}

// ---------------------------------------------------------------------------------------
// class table helpers
// ---------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ int class_of(int w, int h) {
  for (int c = 0; c < kNumClasses; c++)
    if (kClassW[c] == w && kClassH[c] == h) return c;
  return 255;
}

// Push count of the EMI square step by geometry alone (TEncSearch.cpp:1341-1376).
__device__ __forceinline__ int emi_pushes(const fme_job& j) {
  const bool top = j.mv_y - 1 >= j.lt_y, bot = j.mv_y + 1 <= j.rb_y;
  const bool left = j.mv_x - 1 >= j.lt_x, right = j.mv_x + 1 <= j.rb_x;
  const int cols = 1 + (left ? 1 : 0) + (right ? 1 : 0);
  return (top ? cols : 0) + (left ? 1 : 0) + (right ? 1 : 0) + (bot ? cols : 0);
}

// ---------------------------------------------------------------------------------------
// classify: class histogram + first pass of the NN writer prefix-max
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_classify(BatchArgs a, WorkBufs w) {
  __shared__ int32_t hist[kNumClasses + 1];
  __shared__ int32_t agg[9];
  const int tid = threadIdx.x;
  if (tid < kNumClasses + 1) hist[tid] = 0;
  if (tid < 9) agg[tid] = -1;
  __syncthreads();
  int mx[9];
#pragma unroll
  for (int f = 0; f < 9; f++) mx[f] = -1;
  const int base = blockIdx.x * kJobsPerScanBlock;
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++) {
    const int i = base + q * kBlock + tid;
    if (i >= a.n) break;
    const fme_job j = a.jobs[i];
    int c = class_of(j.w, j.h);
    // reject what would make the search read undefined memory
    bool ok = j.ref_id < FME_MAX_PICTURES && j.lambda_id < FME_MAX_LAMBDAS &&
              a.pics[j.ref_id].luma != nullptr;
    if (ok) {
      if (j.key_offset >= 0) {
        ok = (int64_t)j.key_offset + (int64_t)j.w * j.h <= a.n_keys;
      } else {
        ok = j.org_id < FME_MAX_PICTURES && a.pics[j.org_id].luma != nullptr &&
             (int)j.x + j.w <= a.pics[j.org_id].width && (int)j.y + j.h <= a.pics[j.org_id].height;
      }
    }
    if (!ok) c = 255;
    w.cls[i] = (uint8_t)c;
    atomicAdd(&hist[c == 255 ? kNumClasses : c], 1);
    if (j.flags & FME_JOB_EMI) {
      const int np = emi_pushes(j);
#pragma unroll
      for (int s = 0; s < 8; s++)
        if (np > s) mx[s] = max(mx[s], i);
      mx[8] = max(mx[8], i);
    }
  }
#pragma unroll
  for (int f = 0; f < 9; f++)
    if (mx[f] >= 0) atomicMax(&agg[f], mx[f]);
  __syncthreads();
  if (tid < kNumClasses + 1 && hist[tid]) atomicAdd(&w.counts[tid], hist[tid]);
  if (tid < 9) w.blk_agg[blockIdx.x * 9 + tid] = agg[tid];
}

__global__ __launch_bounds__(kBlock) void k_scatter(BatchArgs a, WorkBufs w, Schedule sc) {
  __shared__ int32_t cnt[kNumClasses], basep[kNumClasses];
  const int tid = threadIdx.x;
  if (tid < kNumClasses) cnt[tid] = 0;
  __syncthreads();
  const int base = blockIdx.x * kJobsPerScanBlock;
  int rank[kJobsPerScanBlock / kBlock];
  int cls[kJobsPerScanBlock / kBlock];
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++) {
    const int i = base + q * kBlock + tid;
    cls[q] = 255;
    if (i < a.n) {
      cls[q] = w.cls[i];
      if (cls[q] < kNumClasses) rank[q] = atomicAdd(&cnt[cls[q]], 1);
    }
  }
  __syncthreads();
  if (tid < kNumClasses) basep[tid] = cnt[tid] ? atomicAdd(&w.cursor[tid], cnt[tid]) : 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++) {
    const int i = base + q * kBlock + tid;
    if (cls[q] < kNumClasses) w.perm[sc.class_off[cls[q]] + basep[cls[q]] + rank[q]] = i;
  }
}

__global__ __launch_bounds__(kBlock) void k_search(BatchArgs a, WorkBufs w, Schedule sc) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int b = blockIdx.x;
  int c = 0;
  while (c < kNumClasses - 1 && b >= sc.tile_prefix[c + 1]) c++;
  const int t = b - sc.tile_prefix[c];
  switch (c) {
#define FME_CASE(ID, W_, H_)                                                             \
  case ID: {                                                                             \
    constexpr int P = Geo<W_, H_>::P;                                                    \
    const int first = sc.class_off[ID] + t * P;                                          \
    const int count = min(P, sc.class_cnt[ID] - t * P);                                  \
    search_tile<W_, H_>(a, w.perm, first, count, lds);                                   \
  } break;
    FME_CASE(0, 4, 8) FME_CASE(1, 8, 4) FME_CASE(2, 8, 8) FME_CASE(3, 4, 16)
    FME_CASE(4, 16, 4) FME_CASE(5, 8, 16) FME_CASE(6, 16, 8) FME_CASE(7, 12, 16)
    FME_CASE(8, 16, 12) FME_CASE(9, 16, 16) FME_CASE(10, 8, 32) FME_CASE(11, 32, 8)
    FME_CASE(12, 16, 32) FME_CASE(13, 32, 16) FME_CASE(14, 24, 32) FME_CASE(15, 32, 24)
    FME_CASE(16, 32, 32) FME_CASE(17, 16, 64) FME_CASE(18, 64, 16) FME_CASE(19, 32, 64)
    FME_CASE(20, 64, 32) FME_CASE(21, 48, 64) FME_CASE(22, 64, 48) FME_CASE(23, 64, 64)
#undef FME_CASE
    default: break;
  }
}

// Exclusive prefix-max over the per-block aggregates (one workgroup of 1024 lanes).
__global__ __launch_bounds__(1024) void k_scan_blocks(WorkBufs w, int nblk) {
  __shared__ int32_t buf[1024];
  const int tid = threadIdx.x;
  const int per = (nblk + 1023) / 1024;
  for (int f = 0; f < 9; f++) {
    // local inclusive over this thread's consecutive blocks
    int m = -1;
    for (int q = 0; q < per; q++) {
      const int b = tid * per + q;
      if (b < nblk) m = max(m, w.blk_agg[b * 9 + f]);
    }
    buf[tid] = m;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int o = tid >= off ? buf[tid - off] : -1;
      __syncthreads();
      buf[tid] = max(buf[tid], o);
      __syncthreads();
    }
    int run = tid > 0 ? buf[tid - 1] : -1;  // exclusive carry into this thread's first block
    for (int q = 0; q < per; q++) {
      const int b = tid * per + q;
      if (b < nblk) {
        w.blk_prefix[b * 9 + f] = run;
        run = max(run, w.blk_agg[b * 9 + f]);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// NN_pred() + xMotionEstimation tail, one lane per job.
// ---------------------------------------------------------------------------------------
enum {
  P_EMB0 = 0, P_EMB1 = 32, P_W1 = 64, P_W2 = 438, P_W3 = 878, P_B1 = 1858, P_G1 = 1880,
  P_BE1 = 1902, P_B2 = 1924, P_G2 = 1944, P_BE2 = 1964, P_BOUT = 1984, P_GIN = 2033,
  P_MEAN = 2042, P_STD = 2051
};

__device__ __forceinline__ int emb_row_h(int h) {
  return h == 4 ? 1 : h == 8 ? 2 : h == 16 ? 3 : h == 12 ? 4 : h == 24 ? 5 : h == 32 ? 6 : h == 64 ? 7 : 0;
}
__device__ __forceinline__ int emb_row_w(int w) {
  return w == 4 ? 1 : w == 8 ? 2 : w == 12 ? 3 : w == 16 ? 4 : w == 24 ? 5 : w == 32 ? 6 : w == 64 ? 7 : 0;
}

__device__ int nn_forward(const float* __restrict__ P, const uint32_t (&e)[8], uint32_t c, int pu_h,
                          int pu_w) {
  float in[17], x1[22], x2[20];
  const int rh = emb_row_h(pu_h), rw = emb_row_w(pu_w);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    in[k] = P[P_EMB0 + rh * 4 + k];
    in[4 + k] = P[P_EMB1 + rw * 4 + k];
  }
  const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    float v = (float)raw[k];
    v = (v - P[P_MEAN + k]) / P[P_STD + k];
    in[8 + k] = v * P[P_GIN + k];
  }
#pragma unroll
  for (int r = 0; r < 22; r++) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 17; k++) s = s + P[P_W1 + r * 17 + k] * in[k];
    s = s + P[P_B1 + r];
    s = s < 0.0f ? 0.0f : s;
    x1[r] = s * P[P_G1 + r] + P[P_BE1 + r];
  }
#pragma unroll
  for (int r = 0; r < 20; r++) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 22; k++) s = s + P[P_W2 + r * 22 + k] * x1[k];
    s = s + P[P_B2 + r];
    s = s < 0.0f ? 0.0f : s;
    x2[r] = s * P[P_G2 + r] + P[P_BE2 + r];
  }
  int best = 0;
  float bv = 0.0f;
#pragma unroll
  for (int r = 0; r < 49; r++) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 20; k++) s = s + P[P_W3 + r * 20 + k] * x2[k];
    s = s + P[P_BOUT + r];
    if (r == 0 || s > bv) {  // Eigen maxCoeff: first index of the maximum
      bv = s;
      best = r;
    }
  }
  return best;
}

__global__ __launch_bounds__(kBlock) void k_nn_tail(BatchArgs a, WorkBufs w,
                                                    const float* __restrict__ nnp, int state_in) {
  __shared__ int32_t wave_tot[kBlock / 64][9];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int Q = kJobsPerScanBlock / kBlock;   // consecutive jobs per lane
  const int i0 = blockIdx.x * kJobsPerScanBlock + tid * Q;

  // writer indices of this lane's jobs (inclusive running max)
  int run[9];
#pragma unroll
  for (int f = 0; f < 9; f++) run[f] = -1;
  int srcs[Q][9];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int i = i0 + q;
    if (i < a.n) {
      const fme_job j = a.jobs[i];
      if (j.flags & FME_JOB_EMI) {
        const int np = emi_pushes(j);
#pragma unroll
        for (int s = 0; s < 8; s++)
          if (np > s) run[s] = i;
        run[8] = i;
      }
    }
#pragma unroll
    for (int f = 0; f < 9; f++) srcs[q][f] = run[f];
  }
  // exclusive prefix-max of the lane totals across the block
  int excl[9];
#pragma unroll
  for (int f = 0; f < 9; f++) {
    int v = run[f];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(v, off, 64);
      if (lane >= off) v = max(v, o);
    }
    const int ex = __shfl_up(v, 1, 64);
    excl[f] = lane == 0 ? -1 : ex;
    if (lane == 63) wave_tot[wid][f] = v;
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 9; f++) {
    int carry = w.blk_prefix[blockIdx.x * 9 + f];
    for (int u = 0; u < wid; u++) carry = max(carry, wave_tot[u][f]);
    excl[f] = max(excl[f], carry);
  }

  const uint32_t* st_in = w.nn_state + 12 * state_in;
  uint32_t* st_out = w.nn_state + 12 * (state_in ^ 1);
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int i = i0 + q;
    if (i >= a.n) break;
    int src[9];
#pragma unroll
    for (int f = 0; f < 9; f++) src[f] = max(srcs[q][f], excl[f]);
    const fme_job j = a.jobs[i];
    fme_result* r = a.res + i;
    const double ml = a.mlambda[j.lambda_id];
    const int mvx = r->mv_int_x, mvy = r->mv_int_y;
    int offx, offy;
    uint16_t status = 0;
    if (a.nn_mode) {
      uint32_t e[8];
      uint32_t written = st_in[11];
#pragma unroll
      for (int s = 0; s < 8; s++) {
        if (src[s] >= 0) {
          e[s] = a.res[src[s]].emi[s];
          written |= 1u << s;
        } else {
          e[s] = st_in[s];
        }
      }
      uint32_t c, ph, pw;
      if (src[8] >= 0) {
        c = a.res[src[8]].c;
        ph = a.jobs[src[8]].h;
        pw = a.jobs[src[8]].w;
        written |= 0x100u;
      } else {
        c = st_in[8];
        ph = st_in[9];
        pw = st_in[10];
      }
      const int cls = nn_forward(nnp, e, c, (int)ph, (int)pw);
      r->nn_class = (uint8_t)cls;
      if (!(j.flags & FME_JOB_EMI) || r->n_emi < 8) status |= FME_RES_NN_STALE;
      if ((written & 0x1FFu) != 0x1FFu) status |= FME_RES_NN_UNINIT;
      offx = cls % 7 - 3;
      offy = cls / 7 - 3;
      if (i == a.n - 1) {  // carry the global state to the next batch
#pragma unroll
        for (int s = 0; s < 8; s++) st_out[s] = e[s];
        st_out[8] = c;
        st_out[9] = ph;
        st_out[10] = pw;
        st_out[11] = written;
      }
    } else {
      r->nn_class = 255;
      offx = 2 * r->half_x + r->qtr_x;
      offy = 2 * r->half_y + r->qtr_y;
    }
    const int fx = 4 * mvx + offx, fy = 4 * mvy + offy;
    r->mv_x = (int16_t)fx;
    r->mv_y = (int16_t)fy;
    const uint32_t mvb = mv_bits(fx, fy, 0, j.mvp_x, j.mvp_y);
    const uint32_t bits = (uint32_t)j.bits_in + mvb;
    r->bits = bits;
    const double fw = (j.flags & FME_JOB_BIPRED) ? 0.5 : 1.0;
    const double val = floor(fw * ((double)r->frac_cost - (double)mv_cost(ml, mvb))) + (double)mv_cost(ml, bits);
    r->cost = (uint32_t)(int64_t)val;   // gcc/x86-64 (Distortion)(double) semantics
    r->status = status;
  }
}

// NN_pred() on one explicit input (fme_nn_pred_single): e[8], C, PUHeight, PUWidth.
__global__ void k_nn_single(const float* __restrict__ nnp, const uint32_t* in, int32_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t e[8];
#pragma unroll
  for (int s = 0; s < 8; s++) e[s] = in[s];
  out[0] = nn_forward(nnp, e, in[8], (int)in[9], (int)in[10]);
}

hipError_t launch_nn_single(const float* nnp, const uint32_t* in, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_nn_single, dim3(1), dim3(64), 0, s, nnp, in, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// host launch helpers
// ---------------------------------------------------------------------------------------
template <int W, int H>
static int p_of() { return Geo<W, H>::P; }
template <int W, int H>
static size_t lds_of() { return Geo<W, H>::LDS; }

int pus_per_tile(int cls) {
  switch (cls) {
#define FME_P(ID, W_, H_) case ID: return p_of<W_, H_>();
    FME_P(0, 4, 8) FME_P(1, 8, 4) FME_P(2, 8, 8) FME_P(3, 4, 16) FME_P(4, 16, 4) FME_P(5, 8, 16)
    FME_P(6, 16, 8) FME_P(7, 12, 16) FME_P(8, 16, 12) FME_P(9, 16, 16) FME_P(10, 8, 32)
    FME_P(11, 32, 8) FME_P(12, 16, 32) FME_P(13, 32, 16) FME_P(14, 24, 32) FME_P(15, 32, 24)
    FME_P(16, 32, 32) FME_P(17, 16, 64) FME_P(18, 64, 16) FME_P(19, 32, 64) FME_P(20, 64, 32)
    FME_P(21, 48, 64) FME_P(22, 64, 48) FME_P(23, 64, 64)
#undef FME_P
    default: return 1;
  }
}

size_t lds_bytes_for_class(int cls) {
  switch (cls) {
#define FME_L(ID, W_, H_) case ID: return lds_of<W_, H_>();
    FME_L(0, 4, 8) FME_L(1, 8, 4) FME_L(2, 8, 8) FME_L(3, 4, 16) FME_L(4, 16, 4) FME_L(5, 8, 16)
    FME_L(6, 16, 8) FME_L(7, 12, 16) FME_L(8, 16, 12) FME_L(9, 16, 16) FME_L(10, 8, 32)
    FME_L(11, 32, 8) FME_L(12, 16, 32) FME_L(13, 32, 16) FME_L(14, 24, 32) FME_L(15, 32, 24)
    FME_L(16, 32, 32) FME_L(17, 16, 64) FME_L(18, 64, 16) FME_L(19, 32, 64) FME_L(20, 64, 32)
    FME_L(21, 48, 64) FME_L(22, 64, 48) FME_L(23, 64, 64)
#undef FME_L
    default: return 0;
  }
}

static int nblocks(int n) { return (n + kJobsPerScanBlock - 1) / kJobsPerScanBlock; }

hipError_t launch_classify(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  hipLaunchKernelGGL(k_classify, dim3(nblocks(a.n)), dim3(kBlock), 0, s, a, w);
  return hipGetLastError();
}

hipError_t launch_scatter(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter, dim3(nblocks(a.n)), dim3(kBlock), 0, s, a, w, sc);
  return hipGetLastError();
}

hipError_t launch_search(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, size_t lds,
                         hipStream_t s) {
  const int tiles = sc.tile_prefix[kNumClasses];
  if (tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_search, dim3(tiles), dim3(kBlock), lds, s, a, w, sc);
  return hipGetLastError();
}

hipError_t launch_nn_tail(const BatchArgs& a, const WorkBufs& w, const float* nn_params,
                          int state_in, hipStream_t s) {
  const int nb = nblocks(a.n);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, w, nb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_nn_tail, dim3(nb), dim3(kBlock), 0, s, a, w, nn_params, state_in);
  return hipGetLastError();
}

}  // namespace fme
