// fme_search.hip — the EMI + FracDIF search kernels (gfx950).
//
// One workgroup refines a tile of P same-shape PUs end to end in LDS:
//   1. stage    reference window (rows -5..H+4, cols -5..W+4 around the TZ MV) as int8
//               (sample - 128) twice: row-major (horizontal taps) and column-major
//               (vertical taps of integer columns); the key block column-major int16.
//   2. EMI      SSE / (FEN-subsampled) SAD of the 9 integer positions around the TZ best,
//               then the square-step decision (TEncSearch.cpp:1324-1377, 1155-1188, 5043-5050).
//   3. planes   first-stage (horizontal) outputs for fx = 1,2,3 around mv_int' — the
//               m_filteredBlockTmp planes of xExtDIFUpSamplingH/Q — column-major int16.
//               With s' = s - 128 and sum(taps) = 64, sum(c*s) - 8192 == sum(c*s') exactly,
//               so each value is two v_dot4_i32_i8.
//   4. half     the shared half-pel planes (m_filteredBlock [2][2], [2][0], [0][2],
//               TEncSearch.cpp:6331-6365) as 8-bit predictions, then 9 SATD candidates
//               (xPatternRefinement, 1591-1645), argmin at cost scale 1.
//   5. quarter  the 8 remaining quarter-pel candidates computed per tile in registers
//               (v_dot2_i32_i16 on packed row pairs); candidate 0 reuses the half-stage
//               distortion of the same position; argmin at cost scale 0.
// SATD runs on packed int16 (|coefficients| <= 16320 before the last butterfly); the last
// butterfly is folded with |a+b| + |a-b| = 2 max(|a|,|b|).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fme_device.h"
#include "fme_simd.h"

// Timing-only ablation knob (never set in the product build): bit 0 EMI, 1 planes,
// 2 half planes, 3 half SATD, 4 quarter SATD, 5 staging.
#ifndef FME_SKIP
#define FME_SKIP 0
#endif
// Diagnostic build only: per-phase s_memtime deltas of lane 0, summed over workgroups.
#ifndef FME_STAMPS
#define FME_STAMPS 0
#endif
// Tuning knobs: LDS budget per workgroup (KB) of the 256- and 512-lane kernels, and tiles per
// workgroup (> 1 turns on the software-pipelined tile loop).
#ifndef FME_SMALL_BUDGET_KB
#define FME_SMALL_BUDGET_KB 24
#endif
#ifndef FME_LARGE_BUDGET_KB
#define FME_LARGE_BUDGET_KB 76
#endif
#ifndef FME_TILES_PER_BLOCK
#define FME_TILES_PER_BLOCK 1
#endif
// XCD-aware tile order (see xcd_tile below); 0 = tiles in block order.
#ifndef FME_XCD_SWIZZLE
#define FME_XCD_SWIZZLE 1
#endif

namespace fme {

__device__ unsigned long long g_fme_stamps[16];

namespace {
using namespace simd;
// ---- per-class layout ----------------------------------------------------------------------
constexpr int align_up(int v, int a) { return (v + a - 1) / a * a; }

struct PuInfo {
  int32_t job, flags, x, y, ref, org, key_off;
  int32_t wx0, wy0;        // absolute window origin (mv_tz - 5)
  int32_t mvx, mvy;        // integer MV (after EMI)
  int32_t ex, ey;          // mv_int' - mv_tz
  int32_t mvp_x, mvp_y;
  int32_t lt_x, lt_y, rb_x, rb_y;
  int32_t had, hx, hy, sub;
  int32_t pad0;
  double ml;
  uint32_t acc[9];
  uint32_t acc_q[9];
  uint32_t cost_e[9];      // EMI: MV cost of each integer position (cost scale 2)
  uint32_t pad1[3];
};
static_assert(sizeof(PuInfo) % 16 == 0, "PuInfo alignment");

template <int W, int H>
struct Lay {
  static constexpr int T = ((W % 8) == 0 && (H % 8) == 0) ? 8 : 4;
  static constexpr int TX = W / T, TY = H / T, TILES = TX * TY;
  static constexpr int WR = H + 10, WC = W + 10;       // window rows / cols
  static constexpr int RS = align_up(WC, 4) + 8;       // row-major window stride (bytes)
  static constexpr int CSB = align_up(WR, 4) + 8;      // column-major window stride (bytes)
  static constexpr int CS = H + 10;                    // stage-1 plane column stride (int16): odd dwords
  static constexpr int PC = W + 1;                     // plane columns (-1..W-1)
  static constexpr int PR = H + 8;                     // plane rows (-4..H+3)
  static constexpr int QS = align_up(H + 1, 8) + 8;    // half-pred byte planes column stride
  static constexpr int O_WINR = 0;
  static constexpr int O_WINC = align_up(O_WINR + WR * RS, 16);
  static constexpr int O_KEY = align_up(O_WINC + align_up(WC, 4) * CSB, 16);   // transposes write align4(WC) columns
  static constexpr int O_PL = align_up(O_KEY + W * H * 2, 16);
  static constexpr int PLANE_B = PC * CS * 2;
  static constexpr int O_Q22 = align_up(O_PL + 3 * PLANE_B + 32, 16);
  static constexpr int O_Q20 = O_Q22 + PC * QS;
  static constexpr int O_Q02 = O_Q20 + W * QS;
  static constexpr int BYTES = align_up(O_Q02 + PC * QS + 16, 16);
};

// Dynamic LDS of a tile: [PuInfo x 2P][quarter work lists 3 x 8P int32][counts x4][PU regions x P]
template <int W, int H, int NT, int BUDGET>
struct Tile {
  using L = Lay<W, H>;
  static constexpr int PER_PU = L::BYTES + 2 * (int)sizeof(PuInfo) + 3 * 8 * 4;
  static constexpr int FIXED = FME_MAX_PICTURES * (int)sizeof(PicDesc) + FME_MAX_LAMBDAS * 8 + 32;
  static constexpr int P0 = (BUDGET - FIXED) / PER_PU;
  static constexpr int P = P0 < 1 ? 1 : (P0 > 64 ? 64 : P0);
  static constexpr int O_PICS = 2 * P * (int)sizeof(PuInfo);               // PicDesc[64]
  static constexpr int O_ML = O_PICS + FME_MAX_PICTURES * (int)sizeof(PicDesc);   // double[64]
  static constexpr int O_QLIST = O_ML + FME_MAX_LAMBDAS * 8;
  static constexpr int O_QCOUNT = O_QLIST + 3 * 8 * P * 4;
  static constexpr int O_REGION = align_up(O_QCOUNT + 16, 16);
  static constexpr size_t LDS = (size_t)O_REGION + (size_t)P * L::BYTES;
  static_assert(LDS <= 160 * 1024, "tile exceeds the CU's LDS");
};

// ---- column loaders -------------------------------------------------------------------------
// T consecutive bytes of a column starting at byte offset `off` (any alignment) -> T/4 dwords.
template <int T>
__device__ __forceinline__ void load_bytes(const uint8_t* base, int off, uint32_t (&out)[T / 4]) {
  const uint8_t* p = base + (off & ~3);
  const uint32_t sh = (uint32_t)(off & 3);
  uint32_t a[T / 4 + 1];
#pragma unroll
  for (int j = 0; j <= T / 4; j++) a[j] = lds32(p + 4 * j);
#pragma unroll
  for (int j = 0; j < T / 4; j++) out[j] = funnel8(a[j + 1], a[j], sh);
}

// T outputs of the vertical 8-tap filter on an int16 column starting at value index pr0
// (any parity): s[m] = sum_k c[k] * v[pr0 + m + k].
template <int T>
__device__ __forceinline__ void vert_i16(const uint8_t* col, int pr0, const uint32_t (&c)[4], int (&s)[T]) {
  constexpr int N = T / 2 + 4;   // dwords read
  const uint8_t* p = col + 4 * (pr0 >> 1);
  uint32_t a[N + 1];
#pragma unroll
  for (int j = 0; j <= N; j++) a[j] = lds32(p + 4 * j);
  const bool odd = (pr0 & 1) != 0;
  uint32_t e[N], o[N];
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint32_t b = funnel16(a[j + 1], a[j]);
    e[j] = odd ? b : a[j];
    o[j] = odd ? a[j + 1] : b;
  }
#pragma unroll
  for (int m = 0; m < T; m++) {
    const uint32_t* q = (m & 1) ? &o[m >> 1] : &e[m >> 1];
    int acc = dot2(q[0], c[0], 0);
    acc = dot2(q[1], c[1], acc);
    acc = dot2(q[2], c[2], acc);
    s[m] = dot2(q[3], c[3], acc);
  }
}

// T outputs of the vertical 8-tap filter on an int8 (s - 128) byte column starting at byte
// offset off: s[m] = sum_k c[k] * s'[off + m + k].
template <int T>
__device__ __forceinline__ void vert_s8(const uint8_t* base, int off, uint32_t clo, uint32_t chi, int (&s)[T]) {
  constexpr int N = (T + 7 + 3) / 4 + 1;   // dwords covering T+7 bytes from any alignment
  const uint8_t* p = base + (off & ~3);
  const uint32_t sh = (uint32_t)(off & 3);
  uint32_t a[N];
#pragma unroll
  for (int j = 0; j < N; j++) a[j] = lds32(p + 4 * j);
  uint32_t d[T + 4];
#pragma unroll
  for (int m = 0; m < T + 4; m++) {
    const int q = m >> 2, r = m & 3;
    // bytes (sh + m) .. (sh + m + 3)
    const uint32_t x = sh + (uint32_t)r;
    d[m] = x >= 4 ? funnel8(a[q + 2], a[q + 1], x - 4) : funnel8(a[q + 1], a[q], x);
  }
#pragma unroll
  for (int m = 0; m < T; m++) s[m] = dot4(d[m + 4], chi, dot4(d[m], clo, 0));
}

}  // namespace

// =============================================================================================
// The tile loop: one workgroup owns tiles tile0, tile0 + stride, ... of one PU shape.  While
// tile t is searched, tile t+stride's descriptors and reference/key samples are in flight in
// registers (issued after the EMI phase, stored to LDS after the quarter stage).
// =============================================================================================
template <int W, int H, int NT, int BUDGET>
struct Pipe {
  using L = Lay<W, H>;
  static constexpr int P = Tile<W, H, NT, BUDGET>::P;
  static constexpr int G = (L::WC + 3) / 4;                 // 4-sample groups per window row
  static constexpr int NWIN = P * L::WR * G;                 // window loads per tile
  static constexpr int UW = (NWIN + NT - 1) / NT;            // per lane
  static constexpr int NKEY = P * (W / 4) * (H / 4);         // 4x4 key blocks per tile
  static constexpr int UK = (NKEY + NT - 1) / NT;
};

// Fill a descriptor from a (class-sorted) job.
__device__ __forceinline__ void fill_info(PuInfo& in, const fme_job& j, int jid, const BatchArgs& a,
                                          const double* ml) {
  in.job = jid;
  in.flags = j.flags;
  in.x = j.x;
  in.y = j.y;
  in.ref = j.ref_id;
  in.org = j.org_id;
  in.key_off = j.key_offset;
  in.wx0 = (int)j.x + j.mv_x - 5;
  in.wy0 = (int)j.y + j.mv_y - 5;
  in.mvx = j.mv_x;
  in.mvy = j.mv_y;
  in.ex = in.ey = 0;
  in.mvp_x = j.mvp_x;
  in.mvp_y = j.mvp_y;
  in.lt_x = j.lt_x;
  in.lt_y = j.lt_y;
  in.rb_x = j.rb_x;
  in.rb_y = j.rb_y;
  in.had = (a.use_hadamard && !(j.flags & FME_JOB_LOSSLESS)) ? 1 : 0;
  in.hx = in.hy = 0;
  in.ml = ml[j.lambda_id];
#pragma unroll
  for (int k = 0; k < 9; k++) in.acc[k] = in.acc_q[k] = 0;
}

template <int W, int H, int NT, int BUDGET>
__device__ __forceinline__ void search_class(const BatchArgs& a, const fme_job* __restrict__ sjobs,
                                             const int32_t* __restrict__ perm, int cls_off, int cls_cnt,
                                             int tile0, int stride, char* lds) {
  using L = Lay<W, H>;
  using TL = Tile<W, H, NT, BUDGET>;
  using PP = Pipe<W, H, NT, BUDGET>;
  constexpr int T = L::T;
  constexpr int P = TL::P;
  PuInfo* infos = reinterpret_cast<PuInfo*>(lds);                     // [2][P] (double-buffered)
  int32_t* qlist = reinterpret_cast<int32_t*>(lds + TL::O_QLIST);     // [3][8P]
  int32_t* qcount = reinterpret_cast<int32_t*>(lds + TL::O_QCOUNT);   // [3]
  uint8_t* region0 = reinterpret_cast<uint8_t*>(lds + TL::O_REGION);
  PicDesc* lpics = reinterpret_cast<PicDesc*>(lds + TL::O_PICS);
  double* lml = reinterpret_cast<double*>(lds + TL::O_ML);
  auto R = [&](int p) { return region0 + (size_t)p * L::BYTES; };
  const int tid = threadIdx.x;
  const int ntiles = (cls_cnt + P - 1) / P;
  if (tile0 >= ntiles) return;
  // picture and motion-lambda tables in LDS (read per sample / per PU below)
  if (tid < FME_MAX_PICTURES) lpics[tid] = a.pics[tid];
  if (tid < FME_MAX_LAMBDAS) lml[tid] = a.mlambda[tid];
  unsigned long long stamp[11], pst[4];
  if (FME_STAMPS && threadIdx.x == 0) stamp[0] = __builtin_amdgcn_s_memtime();

  // ---- staging helpers ---------------------------------------------------------------------
  uint32_t wreg[PP::UW];
  uint32_t kreg[PP::UK][4];
  auto issue_loads = [&](const PuInfo* inf, int cnt, int tid) {
#pragma unroll
    for (int u = 0; u < PP::UW; u++) {
      const int e = tid + u * NT;
      wreg[u] = 0;
      if (!(FME_SKIP & 32) && e < cnt * L::WR * PP::G) {
        const int p = e / (L::WR * PP::G), rem = e - p * (L::WR * PP::G);
        const int r = rem / PP::G, g = rem - r * PP::G;
        const PicDesc& pd = lpics[inf[p].ref];
        wreg[u] = pic4(pd.luma, pd.stride, pd.width, pd.height, inf[p].wx0 + 4 * g, inf[p].wy0 + r);
      }
    }
#pragma unroll
    for (int u = 0; u < PP::UK; u++) {
      const int e = tid + u * NT;
      if (!(FME_SKIP & 32) && e < cnt * (W / 4) * (H / 4)) {
        const int p = e / ((W / 4) * (H / 4)), rem = e - p * ((W / 4) * (H / 4));
        const int rb = rem / (W / 4), cb = rem - rb * (W / 4);
        const PuInfo& in = inf[p];
        if (in.key_off < 0) {   // bi-pred key blocks (int16) are read at store time
          const PicDesc& pd = lpics[in.org];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint8_t* q = pd.luma + (size_t)(in.y + 4 * rb + i) * pd.stride + in.x + 4 * cb;
            const uintptr_t addr = reinterpret_cast<uintptr_t>(q);
            kreg[u][i] = (addr & 3) == 0 ? gld32(q)
                                         : (gld8(q) | (gld8(q + 1) << 8) | (gld8(q + 2) << 16) | (gld8(q + 3) << 24));
          }
        }
      }
    }
  };
  auto store_loads = [&](const PuInfo* inf, int cnt, int tid) {
#pragma unroll
    for (int u = 0; u < PP::UW; u++) {
      const int e = tid + u * NT;
      if (e < cnt * L::WR * PP::G) {
        const int p = e / (L::WR * PP::G), rem = e - p * (L::WR * PP::G);
        const int r = rem / PP::G, g = rem - r * PP::G;
        sts32(R(p) + L::O_WINR + r * L::RS + 4 * g, wreg[u] ^ 0x80808080u);
      }
    }
#pragma unroll
    for (int u = 0; u < PP::UK; u++) {
      const int e = tid + u * NT;
      if (e < cnt * (W / 4) * (H / 4)) {
        const int p = e / ((W / 4) * (H / 4)), rem = e - p * ((W / 4) * (H / 4));
        const int rb = rem / (W / 4), cb = rem - rb * (W / 4);
        uint8_t* kb = R(p) + L::O_KEY;
        if (inf[p].key_off >= 0) {
          const int16_t* src = a.keys + (size_t)inf[p].key_off + (4 * rb) * W + 4 * cb;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            uint8_t* dst = kb + ((4 * cb + j) * H + 4 * rb) * 2;
            sts32(dst, (uint32_t)(uint16_t)src[j] | ((uint32_t)(uint16_t)src[W + j] << 16));
            sts32(dst + 4, (uint32_t)(uint16_t)src[2 * W + j] | ((uint32_t)(uint16_t)src[3 * W + j] << 16));
          }
        } else {
          uint32_t rows[4] = {kreg[u][0], kreg[u][1], kreg[u][2], kreg[u][3]}, cols[4];
          transpose4x4(rows, cols);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            uint8_t* dst = kb + ((4 * cb + j) * H + 4 * rb) * 2;
            sts32(dst, lo_pair(cols[j]));
            sts32(dst + 4, hi_pair(cols[j]));
          }
        }
      }
    }
  };
  auto transpose_window = [&](int cnt, int tid) {
    constexpr int RG = (L::WR + 3) / 4, CG = (L::WC + 3) / 4;
    const int total = (FME_SKIP & 32) ? 0 : cnt * RG * CG;
    for (int e = tid; e < total; e += NT) {
      const int p = e / (RG * CG), rem = e - p * (RG * CG);
      const int rg = rem / CG, cg = rem - rg * CG;
      uint8_t* base = R(p);
      uint32_t rows[4], cols[4];
#pragma unroll
      for (int i = 0; i < 4; i++) rows[i] = lds32(base + L::O_WINR + (4 * rg + i) * L::RS + 4 * cg);
      transpose4x4(rows, cols);
#pragma unroll
      for (int j = 0; j < 4; j++) sts32(base + L::O_WINC + (4 * cg + j) * L::CSB + 4 * rg, cols[j]);
    }
  };

  // ---- prologue: the first tile ---------------------------------------------------------------
  int cur = 0;
  int t = tile0;
  int count = min(P, cls_cnt - t * P);
  {
    fme_job j0{};
    int id0 = -1;
    if (tid < count) {
      const int k = cls_off + t * P + tid;
      j0 = sjobs[k];
      id0 = perm[k];
    }
    __syncthreads();   // tables visible
    if (FME_STAMPS && threadIdx.x == 0) pst[0] = __builtin_amdgcn_s_memtime();
    if (tid < P) {
      if (tid < count) {
        fill_info(infos[tid], j0, id0, a, lml);
      } else {
        infos[tid].job = -1;
        infos[tid].flags = 0;
      }
    }
  }
  __syncthreads();
  if (FME_STAMPS && threadIdx.x == 0) pst[1] = __builtin_amdgcn_s_memtime();
  issue_loads(infos, count, tid);
  store_loads(infos, count, tid);
  if (FME_STAMPS && threadIdx.x == 0) pst[2] = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (FME_STAMPS && threadIdx.x == 0) pst[3] = __builtin_amdgcn_s_memtime();
  transpose_window(count, tid);
  __syncthreads();
  if (FME_STAMPS && threadIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memtime();

  for (;;) {
    // an opaque copy of the lane id per iteration keeps LICM from hoisting the per-lane index
    // arithmetic of every phase out of the tile loop (and keeping it live in VGPRs)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    PuInfo* info = infos + cur * P;
    PuInfo* info_n = infos + (cur ^ 1) * P;
    const int tn = t + stride;
    const int count_n = (FME_TILES_PER_BLOCK > 1 && tn < ntiles) ? min(P, cls_cnt - tn * P) : 0;
    // next tile's descriptors: issued now, consumed after the EMI phase
    fme_job nj{};
    int nid = -1;
    if (tid < count_n) {
      const int k = cls_off + tn * P + tid;
      nj = sjobs[k];
      nid = perm[k];
    }

    // ---- 2. EMI: integer distortion of centre + 8 neighbours, per key column ----------------
    // Metric of the modified setDistParam (TComRdCost.cpp:200-230): SSE for W in {4,8,16,32,64},
    // SAD for 12/24/48 over even rows only when FEN is 1 or 3 and H > 8 (TEncSearch.cpp:1158-1164).
    constexpr bool kSad = (W == 12 || W == 24 || W == 48);
    const int sub = (kSad && (a.fen == 1 || a.fen == 3) && H > 8) ? 1 : 0;
    for (int e = tid; e < ((FME_SKIP & 1) ? 0 : count * 9 * W); e += NT) {
      const int p = e / (9 * W), rem = e - p * 9 * W;
      const int pos = rem / W, c = rem - pos * W;
      const PuInfo& in = info[p];
      if (!(in.flags & FME_JOB_EMI)) continue;
      const int dx = pos == 0 ? 0 : ((pos == 1 || pos == 4 || pos == 6) ? -1 : ((pos == 2 || pos == 7) ? 0 : 1));
      const int dy = pos == 0 ? 0 : (pos <= 3 ? -1 : (pos <= 5 ? 0 : 1));
      const uint8_t* base = R(p);
      const uint8_t* kc = base + L::O_KEY + c * H * 2;
      const int off = L::O_WINC + (c + 5 + dx) * L::CSB + 5 + dy;
      const uint32_t wsel = sub ? 0x00000001u : 0x00010001u;
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < H / 4; q++) {
        uint32_t w4[1];
        load_bytes<4>(base, off + 4 * q, w4);
        const uint32_t x = w4[0] ^ 0x80808080u;
        const uint32_t d0 = pk_sub(lds32(kc + 8 * q), lo_pair(x));
        const uint32_t d1 = pk_sub(lds32(kc + 8 * q + 4), hi_pair(x));
        if (kSad) {
          s = udot2(pk_abs(d0), wsel, s);
          s = udot2(pk_abs(d1), wsel, s);
        } else {
          s = (uint32_t)dot2(d0, d0, (int)s);
          s = (uint32_t)dot2(d1, d1, (int)s);
        }
      }
      atomicAdd(&info[p].acc[pos], s);
      if (c == 0)
        info[p].cost_e[pos] = mv_cost(in.ml, mv_bits(in.mvx + dx, in.mvy + dy, 2, in.mvp_x, in.mvp_y));
    }
    __syncthreads();
    if (FME_STAMPS && threadIdx.x == 0) stamp[2] = __builtin_amdgcn_s_memtime();
    if (tid < 3) qcount[tid] = 0;
    if (tid < count) {
      PuInfo& in = info[tid];
      fme_result* r = (FME_SKIP & 128) ? reinterpret_cast<fme_result*>(lds + TL::O_QLIST) : a.res + in.job;
      int n_emi = 0;
      uint32_t cval = 0;
      if (in.flags & FME_JOB_EMI) {
        const int sx = in.mvx, sy = in.mvy;
        uint32_t best = (in.acc[0] << sub) + in.cost_e[0];
        int bx = sx, by = sy, bpos = 0;
        const bool top = sy - 1 >= in.lt_y, bot = sy + 1 <= in.rb_y;
        const bool left = sx - 1 >= in.lt_x, right = sx + 1 <= in.rb_x;
#pragma unroll
        for (int pos = 1; pos <= 8; pos++) {
          const int dx = (pos == 1 || pos == 4 || pos == 6) ? -1 : ((pos == 2 || pos == 7) ? 0 : 1);
          const int dy = pos <= 3 ? -1 : (pos <= 5 ? 0 : 1);
          const bool ok = (dy == -1 ? top : (dy == 1 ? bot : true)) && (dx == -1 ? left : (dx == 1 ? right : true));
          if (!ok) continue;
          uint32_t d = in.acc[pos] << sub;
          r->emi[n_emi++] = d;
          if (d < best) {
            d += in.cost_e[pos];
            if (d < best) {
              best = d;
              bx = sx + dx;
              by = sy + dy;
              bpos = pos;
            }
          }
        }
        cval = best - in.cost_e[bpos];
        in.ex = bx - sx;
        in.ey = by - sy;
        in.mvx = bx;
        in.mvy = by;
      }
      for (int k = n_emi; k < 8; k++) r->emi[k] = 0;
      r->n_emi = (uint8_t)n_emi;
      r->c = cval;
      r->mv_int_x = (int16_t)in.mvx;
      r->mv_int_y = (int16_t)in.mvy;
    }
    if (tid < P) {
      if (tid < count_n) {
        fill_info(info_n[tid], nj, nid, a, lml);
      } else {
        info_n[tid].job = -1;
        info_n[tid].flags = 0;
      }
    }
    __syncthreads();
    if (FME_STAMPS && threadIdx.x == 0) stamp[3] = __builtin_amdgcn_s_memtime();
    // next tile's samples: in flight through the rest of this tile
    issue_loads(info_n, count_n, tid);

    // ---- 3. first-stage planes fx = 1,2,3 (column-major int16), 4 columns x 8 rows per item -
    {
      constexpr int NG = (L::PC + 3) / 4, NCH = (L::PR + 7) / 8;
      uint32_t tl[3], th[3];
      taps8(1, tl[0], th[0]);
      taps8(2, tl[1], th[1]);
      taps8(3, tl[2], th[2]);
      for (int e = tid; e < ((FME_SKIP & 2) ? 0 : count * NG * NCH); e += NT) {
        const int p = e / (NG * NCH), rem = e - p * (NG * NCH);
        const int ch = rem / NG, g = rem - ch * NG;
        const PuInfo& in = info[p];
        uint8_t* base = R(p);
#pragma unroll
        for (int rr = 0; rr < 8; rr += 2) {
          uint32_t out[4][3][2];
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const int pr = ch * 8 + rr + h;
            const int row = min(1 + in.ey + pr, L::WR - 1);
            const int off = L::O_WINR + row * L::RS + 1 + in.ex + 4 * g;
            const uint8_t* q = base + (off & ~3);
            const uint32_t sh = (uint32_t)(off & 3);
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; j++) w[j] = lds32(q + 4 * j);
            uint32_t d[8];
#pragma unroll
            for (int m = 0; m < 8; m++) {
              const uint32_t x = sh + (uint32_t)(m & 3);
              const int qd = m >> 2;
              d[m] = x >= 4 ? funnel8(w[qd + 2], w[qd + 1], x - 4) : funnel8(w[qd + 1], w[qd], x);
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
              for (int f = 0; f < 3; f++) out[i][f][h] = (uint32_t)dot4(d[i + 4], th[f], dot4(d[i], tl[f], 0));
          }
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int pc = 4 * g + i;
            if (pc < L::PC && ch * 8 + rr < L::PR) {
#pragma unroll
              for (int f = 0; f < 3; f++) {
                uint8_t* col = base + L::O_PL + f * L::PLANE_B + pc * L::CS * 2;
                sts32(col + (ch * 8 + rr) * 2, (out[i][f][0] & 0xffffu) | (out[i][f][1] << 16));
              }
            }
          }
        }
      }
    }
    __syncthreads();

    if (FME_STAMPS && threadIdx.x == 0) stamp[4] = __builtin_amdgcn_s_memtime();
    // ---- 4a. half-pel prediction planes (8-bit, column-major) --------------------------------
    // Q22 = [2][2]: vertical half over plane fx=2, cols -1..W-1, rows -1..H-1
    // Q20 = [2][0]: vertical half over integer columns (bytes), cols 0..W-1, rows -1..H-1
    // Q02 = [0][2]: plane fx=2 rounded, cols -1..W-1, rows 0..H-1
    {
      constexpr int NCH = (H + 1 + 7) / 8;
      constexpr int NCH2 = (H + 7) / 8;
      constexpr int N22 = L::PC * NCH, N20 = W * NCH, N02 = L::PC * NCH2;
      uint32_t c2[4];
      taps16(2, c2);
      uint32_t c2lo, c2hi;
      taps8(2, c2lo, c2hi);
      for (int e = tid; e < ((FME_SKIP & 4) ? 0 : count * (N22 + N20 + N02)); e += NT) {
        const int p = e / (N22 + N20 + N02);
        int rem = e - p * (N22 + N20 + N02);
        const PuInfo& in = info[p];
        uint8_t* base = R(p);
        int s[8];
        uint8_t* dst;
        if (rem < N22) {
          const int ch = rem / L::PC, col = rem - ch * L::PC;
          vert_i16<8>(base + L::O_PL + 1 * L::PLANE_B + col * L::CS * 2, 8 * ch, c2, s);
#pragma unroll
          for (int m = 0; m < 8; m++) s[m] = round2d(s[m]);
          dst = base + L::O_Q22 + col * L::QS + 8 * ch;
        } else if (rem < N22 + N20) {
          rem -= N22;
          const int ch = rem / W, col = rem - ch * W;
          const int off = L::O_WINC + (col + 5 + in.ex) * L::CSB + (8 * ch - 1) + 2 + in.ey;
          vert_s8<8>(base, off, c2lo, c2hi, s);
#pragma unroll
          for (int m = 0; m < 8; m++) s[m] = round1d_s8(s[m]);
          dst = base + L::O_Q20 + col * L::QS + 8 * ch;
        } else {
          rem -= N22 + N20;
          const int ch = rem / L::PC, col = rem - ch * L::PC;
          const uint8_t* pcol = base + L::O_PL + 1 * L::PLANE_B + col * L::CS * 2 + (8 * ch + 4) * 2;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t v = lds32(pcol + 4 * j);
            s[2 * j] = clamp_i(((int)(int16_t)(v & 0xffffu) + 8224) >> 6, 0, 255);
            s[2 * j + 1] = clamp_i(((int)(int16_t)(v >> 16) + 8224) >> 6, 0, 255);
          }
          dst = base + L::O_Q02 + col * L::QS + 8 * ch;
        }
        sts32(dst, (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24));
        sts32(dst + 4, (uint32_t)s[4] | ((uint32_t)s[5] << 8) | ((uint32_t)s[6] << 16) | ((uint32_t)s[7] << 24));
      }
    }
    __syncthreads();

    if (FME_STAMPS && threadIdx.x == 0) stamp[5] = __builtin_amdgcn_s_memtime();
    // ---- 4b. half-pel SATD: 9 candidates x tiles ------------------------------------------------
    {
      const int items = count * L::TILES;
      for (int e = tid; e < ((FME_SKIP & 8) ? 0 : 9 * items); e += NT) {
        const int k = e / items, rem = e - k * items;
        const int p = rem / L::TILES, tt = rem - p * L::TILES;
        const PuInfo& in = info[p];
        const uint8_t* base = R(p);
        const int ty = tt / L::TX, tx = tt - ty * L::TX;
        const int dx = cand_dx(k), dy = half_dy(k);
        int colbase, cstride, rowoff;
        uint32_t flip = 0;
        if (dx == 0 && dy == 0) {
          colbase = L::O_WINC + (5 + in.ex) * L::CSB;
          cstride = L::CSB;
          rowoff = 5 + in.ey;
          flip = 0x80808080u;
        } else if (dx == 0) {
          colbase = L::O_Q20;
          cstride = L::QS;
          rowoff = dy < 0 ? 0 : 1;
        } else if (dy == 0) {
          colbase = L::O_Q02 + (dx < 0 ? 0 : 1) * L::QS;
          cstride = L::QS;
          rowoff = 0;
        } else {
          colbase = L::O_Q22 + (dx < 0 ? 0 : 1) * L::QS;
          cstride = L::QS;
          rowoff = dy < 0 ? 0 : 1;
        }
        uint32_t X[T][T / 2];
#pragma unroll
        for (int c = 0; c < T; c++) {
          const int col = tx * T + c;
          uint32_t b[T / 4];
          load_bytes<T>(base, colbase + col * cstride + rowoff + ty * T, b);
          const uint8_t* kc = base + L::O_KEY + (col * H + ty * T) * 2;
#pragma unroll
          for (int j = 0; j < T / 4; j++) {
            const uint32_t x = b[j] ^ flip;
            X[c][2 * j] = pk_sub(lds32(kc + 8 * j), lo_pair(x));
            X[c][2 * j + 1] = pk_sub(lds32(kc + 8 * j + 4), hi_pair(x));
          }
        }
        uint32_t dd = in.had ? satd_packed<T>(X) : sad_packed<T>(X);
        if (tt == 0) dd += mv_cost(in.ml, mv_bits(2 * in.mvx + dx, 2 * in.mvy + dy, 1, in.mvp_x, in.mvp_y));
        atomicAdd(&info[p].acc_q[k], dd);
      }
    }
    __syncthreads();

    if (FME_STAMPS && threadIdx.x == 0) stamp[6] = __builtin_amdgcn_s_memtime();
    // ---- 4c. half argmin (cost scale 1; costs already added), quarter work list by code path --
    if (tid < count) {
      PuInfo& in = info[tid];
      uint32_t best = 0xFFFFFFFFu;
      int bi = 0;
#pragma unroll
      for (int k = 0; k < 9; k++) {
        const uint32_t d = in.acc_q[k];
        if (d < best) {
          best = d;
          bi = k;
        }
      }
      in.hx = cand_dx(bi);
      in.hy = half_dy(bi);
      in.acc[0] = in.acc_q[bi];   // quarter candidate 0 == the best half position (same bits, same cost)
#pragma unroll
      for (int k = 1; k < 9; k++) {
        in.acc[k] = 0;
        const int qx = 2 * in.hx + cand_dx(k), qy = 2 * in.hy + qtr_dy(k);
        const int path = (qy & 3) == 0 ? 0 : ((qx & 3) == 0 ? 1 : 2);
        const int slot = atomicAdd(&qcount[path], 1);
        qlist[path * 8 * P + slot] = tid * 16 + k;
      }
    }
    __syncthreads();

    if (FME_STAMPS && threadIdx.x == 0) stamp[7] = __builtin_amdgcn_s_memtime();
    // ---- 5. quarter-pel SATD: 8 candidates x tiles, grouped by path ----------------------------
    {
      const int n0 = qcount[0] * L::TILES, n1 = qcount[1] * L::TILES, n2 = qcount[2] * L::TILES;
      for (int e = tid; e < ((FME_SKIP & 16) ? 0 : n0 + n1 + n2); e += NT) {
        int path, idx;
        if (e < n0) { path = 0; idx = e; }
        else if (e < n0 + n1) { path = 1; idx = e - n0; }
        else { path = 2; idx = e - n0 - n1; }
        const int entry = qlist[path * 8 * P + idx / L::TILES];
        const int tt = idx - (idx / L::TILES) * L::TILES;
        const int p = entry >> 4, k = entry & 15;
        const PuInfo& in = info[p];
        const uint8_t* base = R(p);
        const int ty = tt / L::TX, tx = tt - ty * L::TX;
        const int qx = 2 * in.hx + cand_dx(k), qy = 2 * in.hy + qtr_dy(k);
        const int ix = qx >> 2, fx = qx & 3, iy = qy >> 2, fy = qy & 3;
        uint32_t X[T][T / 2];
        if (path == 0) {
          // fy == 0 (iy == 0): horizontal only, plane fx rounded (filterCopy !isFirst)
#pragma unroll
          for (int c = 0; c < T; c++) {
            const int col = tx * T + c;
            const uint8_t* pcol = base + L::O_PL + (fx - 1) * L::PLANE_B + (col + ix + 1) * L::CS * 2 + (ty * T + 4) * 2;
            const uint8_t* kc = base + L::O_KEY + (col * H + ty * T) * 2;
#pragma unroll
            for (int j = 0; j < T / 2; j++) {
              const v2s t16 = up(lds32(pcol + 4 * j));
              v2s pr = (t16 + (v2s)(8224)) >> (v2s)(6);
              pr = __builtin_elementwise_min(__builtin_elementwise_max(pr, (v2s)(0)), (v2s)(255));
              X[c][j] = pk_sub(lds32(kc + 4 * j), pk(pr));
            }
          }
        } else if (path == 1) {
          // fx == 0: vertical only on the integer column (bytes)
          uint32_t clo, chi;
          taps8(fy, clo, chi);
#pragma unroll
          for (int c = 0; c < T; c++) {
            const int col = tx * T + c;
            const int off = L::O_WINC + (col + 5 + in.ex) * L::CSB + ty * T + iy + 2 + in.ey;
            int s[T];
            vert_s8<T>(base, off, clo, chi, s);
            const uint8_t* kc = base + L::O_KEY + (col * H + ty * T) * 2;
#pragma unroll
            for (int j = 0; j < T / 2; j++) {
              const uint32_t pr = (uint32_t)round1d_s8(s[2 * j]) | ((uint32_t)round1d_s8(s[2 * j + 1]) << 16);
              X[c][j] = pk_sub(lds32(kc + 4 * j), pr);
            }
          }
        } else {
          // 2-D: vertical fy over plane fx
          uint32_t cv[4];
          taps16(fy, cv);
#pragma unroll
          for (int c = 0; c < T; c++) {
            const int col = tx * T + c;
            const uint8_t* pcol = base + L::O_PL + (fx - 1) * L::PLANE_B + (col + ix + 1) * L::CS * 2;
            int s[T];
            vert_i16<T>(pcol, ty * T + iy + 1, cv, s);
            const uint8_t* kc = base + L::O_KEY + (col * H + ty * T) * 2;
#pragma unroll
            for (int j = 0; j < T / 2; j++) {
              const uint32_t pr = (uint32_t)round2d(s[2 * j]) | ((uint32_t)round2d(s[2 * j + 1]) << 16);
              X[c][j] = pk_sub(lds32(kc + 4 * j), pr);
            }
          }
        }
        uint32_t dd = in.had ? satd_packed<T>(X) : sad_packed<T>(X);
        if (tt == 0) dd += mv_cost(in.ml, mv_bits(4 * in.mvx + qx, 4 * in.mvy + qy, 0, in.mvp_x, in.mvp_y));
        atomicAdd(&info[p].acc[k], dd);
      }
    }
    __syncthreads();

    if (FME_STAMPS && threadIdx.x == 0) stamp[8] = __builtin_amdgcn_s_memtime();
    // ---- 6. quarter argmin (cost scale 0) and results ---------------------------------------------
    if (tid < count) {
      PuInfo& in = info[tid];
      uint32_t best = 0xFFFFFFFFu;
      int bi = 0;
#pragma unroll
      for (int k = 0; k < 9; k++) {
        const uint32_t d = in.acc[k];
        if (d < best) {
          best = d;
          bi = k;
        }
      }
      fme_result* r = (FME_SKIP & 128) ? reinterpret_cast<fme_result*>(lds + TL::O_QLIST) : a.res + in.job;
      r->half_x = (int8_t)in.hx;
      r->half_y = (int8_t)in.hy;
      r->qtr_x = (int8_t)cand_dx(bi);
      r->qtr_y = (int8_t)qtr_dy(bi);
      r->frac_cost = best;
    }
    if (FME_STAMPS && threadIdx.x == 0) {
      stamp[9] = __builtin_amdgcn_s_memtime();
      for (int i = 0; i < 9; i++) atomicAdd(&g_fme_stamps[i], stamp[i + 1] - stamp[i]);
      atomicAdd(&g_fme_stamps[9], pst[0] - stamp[0]);    // descriptor loads + table copy
      atomicAdd(&g_fme_stamps[10], pst[1] - pst[0]);     // fill_info + barrier
      atomicAdd(&g_fme_stamps[11], pst[2] - pst[1]);     // sample loads issued .. stored (lane 0's wave)
      atomicAdd(&g_fme_stamps[12], pst[3] - pst[2]);     // waiting for the other waves' samples
      atomicAdd(&g_fme_stamps[13], stamp[1] - pst[3]);   // window transpose + barrier
      atomicAdd(&g_fme_stamps[15], 1ull);
    }
    if (count_n == 0) break;
    // ---- hand over to the next tile ---------------------------------------------------------------
    store_loads(info_n, count_n, tid);
    __syncthreads();
    transpose_window(count_n, tid);
    __syncthreads();
    cur ^= 1;
    t = tn;
    count = count_n;
  }
}

// =============================================================================================
// kernels: small shapes (256 lanes) and large shapes (512 lanes).  Blocks of one launch are
// dealt to classes by sc.prefix (block ranges); a block strides over its class's tiles.
// =============================================================================================
// With the lane-per-unit kernel (fme_lane.hip) these kernels serve only the AMP shapes whose
// lane groups are not a power of two (12x16, 16x12, 24x32, 32x24, 48x64, 64x48 — the
// SAD12/24/48 EMI metric).
#define FME_SMALL_CLASSES(X) X(7, 12, 16) X(8, 16, 12) X(14, 24, 32) X(15, 32, 24)
#define FME_LARGE_CLASSES(X) X(21, 48, 64) X(22, 64, 48)

constexpr int kSmallNT = 256, kSmallBudget = FME_SMALL_BUDGET_KB * 1024;
constexpr int kLargeNT = 512, kLargeBudget = FME_LARGE_BUDGET_KB * 1024;

__device__ __forceinline__ int find_class(const int32_t (&prefix)[kNumClasses + 1], int b) {
  int c = 0;
  while (c < kNumClasses - 1 && b >= prefix[c + 1]) c++;
  return c;
}

// Workgroups are dealt round-robin to the 8 XCDs (each with its own L2), so block r of a
// class runs on XCD (first + r) % 8.  Giving XCD k the k-th contiguous eighth of the class's
// tiles (tiles follow the CTU-ordered job stream) keeps each XCD on one spatial band of the
// pictures instead of all eight XCDs fetching every region.
__device__ __forceinline__ int xcd_tile(int r, int n) {
#if FME_XCD_SWIZZLE
  const int k = r & 7;
  return k * (n >> 3) + min(k, n & 7) + (r >> 3);
#else
  (void)n;
  return r;
#endif
}

// The schedule is device-built (k_schedule), so the grid is a fixed multiple of 8 workgroups
// that strides over the kernel's blocks (block b keeps XCD b % 8, as with one block each).
__global__ __launch_bounds__(kSmallNT) void k_search_small(BatchArgs a, WorkBufs w) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const Schedule* __restrict__ sc = w.sched;
  const int total = sc->prefix[kSearchCoop][kNumClasses];
  for (int b = blockIdx.x; b < total; b += gridDim.x) {
    const int c = find_class(sc->prefix[kSearchCoop], b);
    const int nblk = sc->prefix[kSearchCoop][c + 1] - sc->prefix[kSearchCoop][c];
    const int blk = xcd_tile(b - sc->prefix[kSearchCoop][c], nblk);
    switch (c) {
#define FME_CASE(ID, W_, H_)                                                                        \
  case ID:                                                                                          \
    search_class<W_, H_, kSmallNT, kSmallBudget>(a, w.sjobs, w.perm, sc->class_off[ID],              \
                                                 sc->class_cnt[ID], blk, nblk, lds);                \
    break;
      FME_SMALL_CLASSES(FME_CASE)
#undef FME_CASE
      default: break;
    }
    __syncthreads();   // LDS is reused by the next block's tiles
  }
}

__global__ __launch_bounds__(kLargeNT) void k_search_large(BatchArgs a, WorkBufs w) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const Schedule* __restrict__ sc = w.sched;
  const int total = sc->prefix[kSearchCoopLarge][kNumClasses];
  for (int b = blockIdx.x; b < total; b += gridDim.x) {
    const int c = find_class(sc->prefix[kSearchCoopLarge], b);
    const int nblk = sc->prefix[kSearchCoopLarge][c + 1] - sc->prefix[kSearchCoopLarge][c];
    const int blk = xcd_tile(b - sc->prefix[kSearchCoopLarge][c], nblk);
    switch (c) {
#define FME_CASE(ID, W_, H_)                                                                        \
  case ID:                                                                                          \
    search_class<W_, H_, kLargeNT, kLargeBudget>(a, w.sjobs, w.perm, sc->class_off[ID],              \
                                                 sc->class_cnt[ID], blk, nblk, lds);                \
    break;
      FME_LARGE_CLASSES(FME_CASE)
#undef FME_CASE
      default: break;
    }
    __syncthreads();
  }
}

// ---- host helpers ----------------------------------------------------------------------------
int pus_per_tile(int cls) {
  switch (cls) {
#define FME_PS(ID, W_, H_) case ID: return Tile<W_, H_, kSmallNT, kSmallBudget>::P;
#define FME_PL(ID, W_, H_) case ID: return Tile<W_, H_, kLargeNT, kLargeBudget>::P;
    FME_SMALL_CLASSES(FME_PS)
    FME_LARGE_CLASSES(FME_PL)
#undef FME_PS
#undef FME_PL
    default: return 1;
  }
}

size_t lds_bytes_for_class(int cls) {
  switch (cls) {
#define FME_LS(ID, W_, H_) case ID: return Tile<W_, H_, kSmallNT, kSmallBudget>::LDS;
#define FME_LL(ID, W_, H_) case ID: return Tile<W_, H_, kLargeNT, kLargeBudget>::LDS;
    FME_SMALL_CLASSES(FME_LS)
    FME_LARGE_CLASSES(FME_LL)
#undef FME_LS
#undef FME_LL
    default: return 0;
  }
}

int tiles_per_block() { return FME_TILES_PER_BLOCK; }

hipError_t debug_phase_cycles(unsigned long long* out16, bool reset) {
  hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_fme_stamps), 16 * sizeof(unsigned long long));
  if (e != hipSuccess || !reset) return e;
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fme_stamps), z, sizeof(z));
}

int search_kernel_of(int cls) {
  if (lane_lanes_per_pu(cls) > 0) return kSearchLane;
  return cls >= 19 ? kSearchCoopLarge : kSearchCoop;
}

static size_t lds_max(int kernel) {
  size_t m = 0;
  for (int c = 0; c < kNumClasses; c++)
    if (search_kernel_of(c) == kernel && lds_bytes_for_class(c) > m) m = lds_bytes_for_class(c);
  return m;
}

// Workgroups of a cooperative launch: at most the blocks n jobs could need (the smallest tile of
// the kernel's classes), at most 2 per CU, a multiple of 8 (XCD round robin).
static int coop_grid(int kernel, int n) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    cus = cu_count(dev);
  }
  int min_p = 1 << 30, classes = 0;
  for (int c = 0; c < kNumClasses; c++)
    if (search_kernel_of(c) == kernel) {
      min_p = std::min(min_p, pus_per_tile(c));
      classes++;
    }
  if (!classes) return 0;
  const long long tiles = (long long)n / min_p + classes;
  const long long bound = (tiles + tiles_per_block() - 1) / tiles_per_block() + classes;
  const long long g = std::min<long long>(bound, 2LL * cus);
  return (int)((g + 7) / 8 * 8);
}

hipError_t launch_search_large(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  const int blocks = coop_grid(kSearchCoopLarge, a.n);
  if (blocks <= 0) return hipSuccess;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_search_large),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_search_large, dim3(blocks), dim3(kLargeNT), lds_max(kSearchCoopLarge), s, a, w);
  return hipGetLastError();
}

hipError_t launch_search_small(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  const int blocks = coop_grid(kSearchCoop, a.n);
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_search_small, dim3(blocks), dim3(kSmallNT), lds_max(kSearchCoop), s, a, w);
  return hipGetLastError();
}

}  // namespace fme
