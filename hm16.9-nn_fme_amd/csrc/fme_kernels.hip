// fme_kernels.hip — CDNA4 (gfx950) kernels of the fractional-pel motion-estimation path.
//
// One batch of PU jobs runs as:
//   classify   per job: PU-shape class, EMI push count; per block: class histogram and the
//              max of the NN "last writer" indices (first pass of a prefix-max scan).
//   scatter    jobs grouped by class (block-aggregated atomics), giving the search tiles.
//   search     EMI square step + FracDIF per tile of same-shape PUs (fme_search.hip).
//   nn_tail    prefix-max over jobs resolves which earlier job last wrote each array_e slot
//              (the reference's stale global state, TEncSearch.cpp:55-57, 198-201), then
//              NN_pred() (85-204) and the xMotionEstimation tail (4586-4597), one lane per job.
//
// Integer arithmetic follows TComInterpolationFilter (14-bit intermediate, offsets -8192 and
// 526336, shift 12) and TComRdCost (xGetHADs 8x8/4x4, SSE, SAD with FEN row subsampling).
// MV cost uses double like TComRdCost::getCost.  The NN is float32 with no contraction
// (this file is compiled with -ffp-contract=off) and sequential-k sums.
#include <hip/hip_runtime.h>

#include <algorithm>

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
// class table helpers
// ---------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ int class_of(int w, int h) {
  for (int c = 0; c < kNumClasses; c++)
    if (kClassW[c] == w && kClassH[c] == h) return c;
  return 255;
}

// ---------------------------------------------------------------------------------------
// classify: class histogram + first pass of the NN writer prefix-max
// ---------------------------------------------------------------------------------------
// PU shape -> class: [(w/4 - 1) * 16 + h/4 - 1], 255 = not an HEVC inter PU shape
struct ClassLut {
  uint8_t v[256];
  constexpr ClassLut() : v() {
    for (int i = 0; i < 256; i++) v[i] = 255;
    for (int c = 0; c < kNumClasses; c++) v[((kClassW[c] >> 2) - 1) * 16 + (kClassH[c] >> 2) - 1] = (uint8_t)c;
  }
};
__constant__ ClassLut kClassLut = ClassLut();

// All of a block's loads (its 4 jobs per lane, the class table, the picture descriptors) are
// issued before any of them is used: the kernel is a few dependent memory latencies long.
__global__ __launch_bounds__(kBlock) void k_classify(BatchArgs a, WorkBufs w) {
  constexpr int Q = kJobsPerScanBlock / kBlock;
  __shared__ int32_t hist[kNumClasses + 1];
  __shared__ int32_t agg[9];
  __shared__ uint8_t lut[256];
  __shared__ int32_t pic_w[FME_MAX_PICTURES], pic_h[FME_MAX_PICTURES];  // pic_w -1: slot unset
  const int tid = threadIdx.x;
  const int base = blockIdx.x * kJobsPerScanBlock;
  fme_job jb[Q];
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int i = base + q * kBlock + tid;
    if (i < a.n) jb[q] = a.jobs[i];
  }
  __shared__ int32_t keys_bad, keyed;
  if (tid == 0) {
    keys_bad = a.key_invalid ? *a.key_invalid : 0;
    keyed = 0;
  }
  lut[tid] = kClassLut.v[tid];
  if (tid < FME_MAX_PICTURES) {
    const PicDesc p = a.pics[tid];
    pic_w[tid] = p.luma ? p.width : -1;
    pic_h[tid] = p.height;
  }
  if (tid < kNumClasses + 1) hist[tid] = 0;
  if (tid < 9) agg[tid] = -1;
  __syncthreads();
  int mx[9];
#pragma unroll
  for (int f = 0; f < 9; f++) mx[f] = -1;
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const int i = base + q * kBlock + tid;
    if (i < a.n) {
      const fme_job& j = jb[q];
      int c = ((j.w | j.h) & 3) == 0 && j.w >= 4 && j.w <= 64 && j.h >= 4 && j.h <= 64
                  ? lut[((j.w >> 2) - 1) * 16 + (j.h >> 2) - 1] : 255;
      // reject what would make the search read undefined memory
      bool ok = j.ref_id < FME_MAX_PICTURES && j.lambda_id < FME_MAX_LAMBDAS && pic_w[j.ref_id] >= 0;
      if (ok) {
        if (j.key_offset >= 0) {
          ok = (int64_t)j.key_offset + (int64_t)j.w * j.h <= a.n_keys && keys_bad == 0;
        } else {
          ok = j.org_id < FME_MAX_PICTURES && pic_w[j.org_id] >= 0 &&
               (int)j.x + j.w <= pic_w[j.org_id] && (int)j.y + j.h <= pic_h[j.org_id];
        }
      }
      // FME_JOB_NN_IN: its input row must be bound (fme_set_nn_inputs)
      if ((j.flags & FME_JOB_NN_IN) && (!a.nn_in || i >= a.nn_in_cap)) ok = false;
      if (!ok) c = 255;
      w.cls[i] = (uint8_t)c;
      atomicAdd(&hist[c == 255 ? kNumClasses : c], 1);
      if (j.key_offset >= 0) atomicAdd(&keyed, 1);
      if (nn_writes_c(j)) {
        const int np = nn_pushes(j);
#pragma unroll
        for (int s = 0; s < 8; s++)
          if (np > s) mx[s] = max(mx[s], i);
        mx[8] = max(mx[8], i);
      }
    }
  }
#pragma unroll
  for (int f = 0; f < 9; f++)
    if (mx[f] >= 0) atomicMax(&agg[f], mx[f]);
  __syncthreads();
  if (tid < kNumClasses + 1 && hist[tid]) atomicAdd(&w.counts[tid], hist[tid]);
  if (tid == 0 && keyed) atomicAdd(&w.counts[kKeyedWord], keyed);
  if (tid < 9) w.blk_agg[blockIdx.x * 9 + tid] = agg[tid];
}

// ---------------------------------------------------------------------------------------
// schedule: the class histogram -> class offsets, each search kernel's block ranges and the
// lane kernels' per-XCD tile queues, all on the device (one wave, one lane per class), so a
// batch needs no host round trip between classify and search.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_excl_scan(int v) {
  int s = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(s, off, 64);
    if ((int)threadIdx.x >= off) s += o;
  }
  return s - v;
}

__global__ __launch_bounds__(64) void k_schedule(WorkBufs w, SchedParams p) {
  const int c = threadIdx.x;
  Schedule* sc = w.sched;
  const int inv = w.counts[kNumClasses];
  const int cnt = (c < kNumClasses && inv == 0) ? w.counts[c] : 0;
  const int nb = cnt > 0 ? (int)(((long long)cnt * p.lanes[c] + 63) / 64) : 0;   // 64-lane wave tiles
  const int off = wave_excl_scan(cnt);
  if (c < kNumClasses) {
    sc->class_off[c] = off;
    sc->class_cnt[c] = cnt;
  }
  {
    const int ex = wave_excl_scan(nb);
    if (c <= kNumClasses) sc->prefix[c] = ex;     // [kNumClasses] = the total
  }
  // per-XCD queues of bands (Schedule::xq): band B of class c = its tiles [nb B / 8S, nb (B+1) / 8S)
  constexpr int S = FME_LANE_SUBBANDS;
  auto band_lo = [&](int B) { return (int)(((long long)nb * B) / (8 * S)); };
#pragma unroll 1
  for (int x = 0; x < 8; x++) {
    int run = 0;
#pragma unroll 1
    for (int q = 0; q < S; q++) {
      const int B = x * S + q;
      const int mine_c = c < kNumClasses ? band_lo(B + 1) - band_lo(B) : 0;   // class c's band tiles
      const int mine = __shfl(mine_c, c < kNumClasses ? lane_class_at(c) : c);  // position c's
      const int ex = run + wave_excl_scan(mine);
      if (c <= kNumClasses) sc->xq[x][q][c] = ex;
      run = __shfl(ex, kNumClasses);
    }
  }
  if (c == 0) sc->invalid = inv;
}

__global__ __launch_bounds__(kBlock) void k_scatter(BatchArgs a, WorkBufs w) {
  __shared__ int32_t cnt[kNumClasses], basep[kNumClasses];
  const Schedule* __restrict__ sc = w.sched;
  if (sc->invalid) return;   // rejected batch: nothing downstream reads the grouping
  const int tid = threadIdx.x;
  if (tid < kNumClasses) cnt[tid] = 0;
  __syncthreads();
  const int base = blockIdx.x * kJobsPerScanBlock;
  int rank[kJobsPerScanBlock / kBlock];
  int cls[kJobsPerScanBlock / kBlock];
  fme_job jb[kJobsPerScanBlock / kBlock];   // loaded up front, beside the class bytes
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++) {
    const int i = base + q * kBlock + tid;
    cls[q] = 255;
    if (i < a.n) {
      cls[q] = w.cls[i];
      if (FME_SJOBS) jb[q] = a.jobs[i];
    }
  }
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++)
    if (cls[q] < kNumClasses) rank[q] = atomicAdd(&cnt[cls[q]], 1);
  __syncthreads();
  if (tid < kNumClasses) basep[tid] = cnt[tid] ? atomicAdd(&w.cursor[tid], cnt[tid]) : 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kJobsPerScanBlock / kBlock; q++) {
    const int i = base + q * kBlock + tid;
    if (cls[q] < kNumClasses) {
      const int dst = sc->class_off[cls[q]] + basep[cls[q]] + rank[q];
      w.perm[dst] = i;
      if (FME_SJOBS) w.sjobs[dst] = jb[q];
    }
  }
  // Exclusive prefix-max of the NN-writer aggregates over the blocks before this one: k_nn_tail's
  // carry-in of the stale-state scan.  It depends on k_classify only, so it is computed here,
  // before the search, instead of by a serial pass between the search and the tail.
  __shared__ int32_t red[kBlock / 64][9];
  int m[9];
#pragma unroll
  for (int f = 0; f < 9; f++) m[f] = -1;
  for (int b = tid; b < (int)blockIdx.x; b += kBlock) {
#pragma unroll
    for (int f = 0; f < 9; f++) m[f] = max(m[f], w.blk_agg[b * 9 + f]);
  }
#pragma unroll
  for (int f = 0; f < 9; f++) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m[f] = max(m[f], __shfl_xor(m[f], off));
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int f = 0; f < 9; f++) red[tid >> 6][f] = m[f];
  }
  __syncthreads();
  if (tid < 9) {
    int r = red[0][tid];
#pragma unroll
    for (int q = 1; q < kBlock / 64; q++) r = max(r, red[q][tid]);
    w.blk_prefix[blockIdx.x * 9 + tid] = r;
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


// Device layout of the net for the tail (built once per weight load by nn_pack, fme_device.h
// kNnPk*): rows paired for packed f32 math (row r in .x, row r+1 in .y, so both halves run
// the reference's sequential k order), and the 8 embedding terms of layer 1 folded into a
// per-PU-shape prefix: the partial sums after k = 0..7 depend only on (PUHeight, PUWidth).
void nn_pack(const float* P, float* Q) {
  for (int i = 0; i < kNnPkFloats; i++) Q[i] = 0.0f;
  for (int rh = 0; rh < 8; rh++)
    for (int rw = 0; rw < 8; rw++)
      for (int r = 0; r < 22; r++) {
        float s = 0.0f;   // TEncSearch.cpp:120 row r, terms k = 0..7 (embeddings), in order
        for (int k = 0; k < 4; k++) s = s + P[P_W1 + r * 17 + k] * P[P_EMB0 + rh * 4 + k];
        for (int k = 0; k < 4; k++) s = s + P[P_W1 + r * 17 + 4 + k] * P[P_EMB1 + rw * 4 + k];
        Q[kNnPkPfx + (rh * 8 + rw) * 22 + r] = s;
      }
  for (int r = 0; r < 22; r++)
    for (int k = 0; k < 9; k++) Q[kNnPkW1 + ((r / 2) * 9 + k) * 2 + (r & 1)] = P[P_W1 + r * 17 + 8 + k];
  for (int r = 0; r < 20; r++)
    for (int k = 0; k < 22; k++) Q[kNnPkW2 + ((r / 2) * 22 + k) * 2 + (r & 1)] = P[P_W2 + r * 22 + k];
  for (int r = 0; r < 49; r++)
    for (int k = 0; k < 20; k++) Q[kNnPkW3 + ((r / 2) * 20 + k) * 2 + (r & 1)] = P[P_W3 + r * 20 + k];
  for (int r = 0; r < 22; r++) {
    Q[kNnPkB1 + r] = P[P_B1 + r];
    Q[kNnPkG1 + r] = P[P_G1 + r];
    Q[kNnPkBE1 + r] = P[P_BE1 + r];
  }
  for (int r = 0; r < 20; r++) {
    Q[kNnPkB2 + r] = P[P_B2 + r];
    Q[kNnPkG2 + r] = P[P_G2 + r];
    Q[kNnPkBE2 + r] = P[P_BE2 + r];
  }
  for (int r = 0; r < 49; r++) Q[kNnPkBout + r] = P[P_BOUT + r];
  for (int k = 0; k < 9; k++) {
    Q[kNnPkGin + k] = P[P_GIN + k];
    Q[kNnPkMean + k] = P[P_MEAN + k];
    Q[kNnPkStd + k] = P[P_STD + k];
  }
}


// NN_pred() (TEncSearch.cpp:85-134) on the packed layout: float32, every dot product summed in
// k order without contraction (the sequential-k contract), BN as x*g + b.  The
// weights are wave-uniform, so they stream through the scalar cache into SGPR operands.
__device__ __forceinline__ int nn_forward(const float* __restrict__ Q, const uint32_t (&e)[8], uint32_t c, int pu_h,
                                          int pu_w) {
  const int t = emb_row_h(pu_h) * 8 + emb_row_w(pu_w);
  float in[9];
  const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    float v = (float)raw[k];
    v = (v - Q[kNnPkMean + k]) / Q[kNnPkStd + k];
    in[k] = v * Q[kNnPkGin + k];
  }
  const float* pfx = Q + kNnPkPfx + t * 22;
  f2 x1[11];
#pragma unroll
  for (int rp = 0; rp < 11; rp++) {
    f2 s = {pfx[2 * rp], pfx[2 * rp + 1]};
#pragma unroll
    for (int k = 0; k < 9; k++) s = s + ld2(Q, kNnPkW1 + (rp * 9 + k) * 2) * (f2){in[k], in[k]};
    s = relu2(s + ld2(Q, kNnPkB1 + 2 * rp));
    x1[rp] = s * ld2(Q, kNnPkG1 + 2 * rp) + ld2(Q, kNnPkBE1 + 2 * rp);
  }
  f2 x2[10];
#pragma unroll
  for (int rp = 0; rp < 10; rp++) {
    f2 s = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 22; k++) {
      const float xk = (k & 1) ? x1[k / 2].y : x1[k / 2].x;
      s = s + ld2(Q, kNnPkW2 + (rp * 22 + k) * 2) * (f2){xk, xk};
    }
    s = relu2(s + ld2(Q, kNnPkB2 + 2 * rp));
    x2[rp] = s * ld2(Q, kNnPkG2 + 2 * rp) + ld2(Q, kNnPkBE2 + 2 * rp);
  }
  int best = 0;
  float bv = 0.0f;
#pragma unroll 1   // the weights of one row pair per iteration (scalar loads, few SGPRs)
  for (int rp = 0; rp < 25; rp++) {
    f2 s = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 20; k++) {
      const float xk = (k & 1) ? x2[k / 2].y : x2[k / 2].x;
      s = s + ld2(Q, kNnPkW3 + (rp * 20 + k) * 2) * (f2){xk, xk};
    }
    s = s + ld2(Q, kNnPkBout + 2 * rp);
    // Eigen maxCoeff: first index of the maximum (strict >), rows in order
    if (rp == 0 || s.x > bv) {
      bv = s.x;
      best = 2 * rp;
    }
    if (rp < 24 && s.y > bv) {
      bv = s.y;
      best = 2 * rp + 1;
    }
  }
  return best;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NN_pred() on the inputs job i sees + the xMotionEstimation tail (TEncSearch.cpp:4583-4597):
// src = the last writer of each carried field (writer_scan), r0..r3 = the job's 64-byte record.
__device__ __forceinline__ void tail_job(const BatchArgs& a, const WorkBufs& w, const float* __restrict__ nnp_g,
                                         int state_in, int i, const fme_job& j, const int (&src)[9], u32x4 r0,
                                         u32x4 r1, u32x4 r2, u32x4 r3) {
  const uint32_t* st_in = w.nn_state + 12 * state_in;
  uint32_t* st_out = w.nn_state + 12 * (state_in ^ 1);
  fme_result* r = a.res + i;
  const fme_result* sr = search_rec(a, w, i);
  const double ml = a.mlambda[j.lambda_id];
  const int mvx = (int16_t)(r0.x & 0xFFFF), mvy = (int16_t)(r0.x >> 16);
  const uint32_t own_emi[8] = {r1.w, r2.x, r2.y, r2.z, r2.w, r3.x, r3.y, r3.z};
  const uint32_t own_c = r1.z, own_n_emi = r3.w & 0xFF, frac_cost = r0.w;
  int offx, offy, cls = 255;
  uint16_t status = 0;
  if (a.nn_mode) {
    uint32_t e[8];
    uint32_t written = st_in[11];
#pragma unroll
    for (int s = 0; s < 8; s++) {
      if (src[s] == i) {
        e[s] = own_emi[s];
        written |= 1u << s;
      } else if (src[s] >= 0) {
        e[s] = search_rec(a, w, src[s])->emi[s];
        written |= 1u << s;
      } else {
        e[s] = st_in[s];
      }
    }
    uint32_t c, ph, pw;
    if (src[8] == i) {
      c = own_c;
      ph = j.h;
      pw = j.w;
      written |= 0x100u;
    } else if (src[8] >= 0) {
      c = search_rec(a, w, src[8])->c;
      ph = a.jobs[src[8]].h;
      pw = a.jobs[src[8]].w;
      written |= 0x100u;
    } else {
      c = st_in[8];
      ph = st_in[9];
      pw = st_in[10];
    }
    cls = nn_forward(nnp_g, e, c, (int)ph, (int)pw);
    if (!nn_writes_c(j) || own_n_emi < 8) status |= FME_RES_NN_STALE;
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
    const int8_t hx = (int8_t)(r0.z & 0xFF), hy = (int8_t)((r0.z >> 8) & 0xFF);
    const int8_t qx = (int8_t)((r0.z >> 16) & 0xFF), qy = (int8_t)(r0.z >> 24);
    offx = 2 * hx + qx;
    offy = 2 * hy + qy;
  }
  const int fx = 4 * mvx + offx, fy = 4 * mvy + offy;
  const uint32_t mvb = mv_bits(fx, fy, 0, j.mvp_x, j.mvp_y);
  const uint32_t bits = (uint32_t)j.bits_in + mvb;
  const double fw = (j.flags & FME_JOB_BIPRED) ? 0.5 : 1.0;
  const double val = floor(fw * ((double)frac_cost - (double)mv_cost(ml, mvb))) + (double)mv_cost(ml, bits);
  // gcc/x86-64 (Distortion)(double) semantics for the cost
  store_outputs(r, sr, w.mv_out, i, fx, fy, (uint32_t)(int64_t)val, bits, (uint8_t)cls, status);
}

// One lane per job; a block scans one 1024-job block (kJobsPerScanBlock, the granularity of
// k_scatter's carry-in) in rounds of kTailNT jobs, the carry passed from round to round.
// A/B on the 1080p batch (tools/ab_bench.py, identical results): 1024 lanes at 4 waves/SIMD
// 0.112 ms, 512 lanes x 2 rounds at 6 waves/SIMD 0.108, 256 x 4 at 6 0.121, at 5 0.119: the tail
// is bound by its own issue (≈ 3,100 instructions per wave, 1,640 of them packed f32 multiply /
// add in the reference's k order), not by latency; kept at one round.
constexpr int kTailNT = kJobsPerScanBlock;
static_assert(kJobsPerScanBlock % kTailNT == 0, "rounds tile the scan block");

__global__ __launch_bounds__(kTailNT)
void k_nn_tail(BatchArgs a, WorkBufs w, const float* __restrict__ nnp_g, int state_in) {
  __shared__ int32_t wave_tot[kTailNT / 64][9];
  const int tid = threadIdx.x;
  if (w.sched->invalid) {
    for (int rnd = 0; rnd < kJobsPerScanBlock / kTailNT; rnd++) {
      const int i = blockIdx.x * kJobsPerScanBlock + rnd * kTailNT + tid;
      if (i < a.n) reject_job(a, w, i, state_in);
    }
    return;
  }
  int carry[9];
#pragma unroll
  for (int f = 0; f < 9; f++) carry[f] = w.blk_prefix[blockIdx.x * 9 + f];
  for (int rnd = 0; rnd < kJobsPerScanBlock / kTailNT; rnd++) {
    const int base = blockIdx.x * kJobsPerScanBlock + rnd * kTailNT;
    if (base >= a.n) break;   // block-uniform
    const int i = base + tid;
    const bool valid = i < a.n;
    fme_job j{};
    // the job and its 64-byte record, issued before the scan's barrier (the NN inputs are
    // usually the job's own pushes)
    u32x4 r0{}, r1{}, r2{}, r3{};
    if (valid) {
      j = a.jobs[i];
      const u32x4* rb = reinterpret_cast<const u32x4*>(search_rec(a, w, i));
      r0 = rb[0];
      r1 = rb[1];
      r2 = rb[2];
      r3 = rb[3];
    }
    // writer indices of this job (slots it pushes, C / PU size)
    int run[9];
    {
      const bool wr = valid && nn_writes_c(j);
      const int np = wr ? nn_pushes(j) : 0;
#pragma unroll
      for (int s = 0; s < 8; s++) run[s] = (np > s) ? i : -1;
      run[8] = wr ? i : -1;
    }
    int src[9], tot[9];
    writer_scan<kTailNT / 64>(run, carry, base, wave_tot, src, tot);
#pragma unroll
    for (int f = 0; f < 9; f++) carry[f] = tot[f];
    if (valid) tail_job(a, w, nnp_g, state_in, i, j, src, r0, r1, r2, r3);
    if (kJobsPerScanBlock / kTailNT > 1) __syncthreads();   // wave_tot is rewritten next round
  }
}


// ---------------------------------------------------------------------------------------
// host launch helpers
// ---------------------------------------------------------------------------------------
static int nblocks(int n) { return (n + kJobsPerScanBlock - 1) / kJobsPerScanBlock; }

hipError_t launch_classify(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  hipLaunchKernelGGL(k_classify, dim3(nblocks(a.n)), dim3(kBlock), 0, s, a, w);
  return hipGetLastError();
}

// fme_nn_reset_state / fme_nn_set_state, applied in stream order: the 12 words travel as a
// kernel argument, so the host copy is free as soon as the launch returns.
struct State12 {
  uint32_t v[12];
};
__global__ void k_put_state(uint32_t* dst, State12 st) {
  if (threadIdx.x < 12) dst[threadIdx.x] = st.v[threadIdx.x];
}

// The picture / lambda tables of a batch from a pinned, device-mapped host slot (fme_api.cpp
// sync_tables: a ring of slots, each reused only once its launch has run), instead of a 3.5 KB
// kernel argument at the edge of the argument segment.
__global__ __launch_bounds__(256) void k_put_tables(PicDesc* __restrict__ pics, double* __restrict__ ml,
                                                    const TablesSlot* __restrict__ t) {
  const int i = threadIdx.x;
  if (i < FME_MAX_PICTURES) pics[i] = t->pics[i];
  if (i < FME_MAX_LAMBDAS) ml[i] = t->ml[i];
}

hipError_t launch_put_tables(PicDesc* d_pics, double* d_ml, const TablesSlot* t_dev, hipStream_t s) {
  hipLaunchKernelGGL(k_put_tables, dim3(1), dim3(256), 0, s, d_pics, d_ml, t_dev);
  return hipGetLastError();
}

hipError_t launch_put_state(uint32_t* dst, const uint32_t* v12, hipStream_t s) {
  State12 st;
  for (int k = 0; k < 12; k++) st.v[k] = v12[k];
  hipLaunchKernelGGL(k_put_state, dim3(1), dim3(64), 0, s, dst, st);
  return hipGetLastError();
}

hipError_t launch_schedule(const WorkBufs& w, const SchedParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_schedule, dim3(1), dim3(64), 0, s, w, p);
  return hipGetLastError();
}

hipError_t launch_scatter(const BatchArgs& a, const WorkBufs& w, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter, dim3(nblocks(a.n)), dim3(kBlock), 0, s, a, w);
  return hipGetLastError();
}

SchedParams sched_params() {
  SchedParams p{};
  for (int c = 0; c < kNumClasses; c++) p.lanes[c] = lane_lanes_per_pu(c);
  return p;
}

int cu_count(int device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) v = 256;
  return v;
}

// ---------------------------------------------------------------------------------------
// results download: device rows -> pinned host memory, few workgroups.  Each lane keeps four
// 16-byte loads in flight, then stores them non-temporally: the rows go to the PCIe write path
// without allocating in L2.  tools/probes/d2h_kernel_probe.hip (profiles/r05_ab.log): PCIe write
// bound at ~54 GB/s from 8 workgroups of 256 lanes with nt stores (0.264 ms per 13.8 MB), where
// system-scope sc0 sc1 stores need 64 workgroups and one-wave groups 128.
// ---------------------------------------------------------------------------------------
constexpr int kDlThreads = 256;
__device__ __forceinline__ void dl_store(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, p); }
__global__ __launch_bounds__(kDlThreads) void k_download(const u32x4* __restrict__ src, u32x4* dst, long n16) {
  const long stride = (long)gridDim.x * kDlThreads;
  long i = (long)blockIdx.x * kDlThreads + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dl_store(dst + i, a);
    dl_store(dst + i + stride, b);
    dl_store(dst + i + 2 * stride, c);
    dl_store(dst + i + 3 * stride, d);
  }
  for (; i < n16; i += stride) dl_store(dst + i, src[i]);
}

__global__ __launch_bounds__(kBlock) void k_gather_jobs(const fme_job* __restrict__ src,
                                                       const fme_tz_ext* __restrict__ src_ext,
                                                       const int32_t* __restrict__ idx, fme_job* __restrict__ dst,
                                                       fme_tz_ext* __restrict__ dst_ext, int n) {
  const int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= n) return;
  const int u = idx[q];
  dst[q] = src[u];
  if (dst_ext) dst_ext[q] = src_ext[u];
}

hipError_t launch_gather_jobs(const fme_job* src, const fme_tz_ext* src_ext, const int32_t* idx, fme_job* dst,
                              fme_tz_ext* dst_ext, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_jobs, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, src, src_ext, idx, dst,
                     dst_ext, n);
  return hipGetLastError();
}

hipError_t launch_download(const void* src, void* dst, size_t n16, int wgs, hipStream_t s) {
  const long need = (long)((n16 + kDlThreads - 1) / kDlThreads);
  const int g = (int)std::min<long>(wgs, std::max<long>(need, 1));
  hipLaunchKernelGGL(k_download, dim3(g), dim3(kDlThreads), 0, s, static_cast<const u32x4*>(src),
                     static_cast<u32x4*>(dst), (long)n16);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// packed jobs (fme_job_packed, include/fme.h) -> fme_job.  Lane i unpacks job i; a wave is 64
// consecutive jobs, whose keyed blocks follow key_base[wave] densely in job order, so each lane's
// key offset is the base plus the exclusive sum of w*h over the wave's earlier keyed jobs.  The
// range words are the canonical mv -/+ range bit, which gives the EMI step's four tests
// (xTZ8PointSquareSearch, TEncSearch.cpp:1341-1376) the packed answers.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_unpack_jobs(const fme_job_packed* __restrict__ src,
                                                       const int32_t* __restrict__ key_base,
                                                       fme_job* __restrict__ dst, int n) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  fme_job_packed p{};
  if (i < n) p = src[i];
  const uint32_t pu = p.pu, ctl = p.ctl;
  const int w = (int)(((pu >> 22) & 15u) + 1u) * 4, h = (int)(((pu >> 26) & 15u) + 1u) * 4;
  const bool keyed = i < n && ((ctl >> 21) & 1u);
  const int lane = (int)(threadIdx.x & 63);
  int s = keyed ? w * h : 0;   // inclusive scan over the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(s, off, 64);
    if (lane >= off) s += o;
  }
  if (i >= n) return;
  const int base = key_base[i >> 6];
  fme_job j;
  j.x = (uint16_t)((pu & 2047u) * 4u);
  j.y = (uint16_t)(((pu >> 11) & 2047u) * 4u);
  j.w = (uint8_t)w;
  j.h = (uint8_t)h;
  j.org_id = (uint8_t)(ctl & 63u);
  j.ref_id = (uint8_t)((ctl >> 6) & 63u);
  j.lambda_id = (uint8_t)((ctl >> 12) & 31u);
  j.flags = (uint8_t)((ctl >> 17) & 15u);
  const uint32_t rg = (ctl >> 22) & 15u;
  j.bits_in = (uint16_t)(ctl >> 26);
  j.mv_x = p.mv_x;
  j.mv_y = p.mv_y;
  j.mvp_x = p.mvp_x;
  j.mvp_y = p.mvp_y;
  j.lt_x = (int16_t)(p.mv_x - ((rg & FME_PK_RANGE_LEFT) ? 1 : 0));
  j.rb_x = (int16_t)(p.mv_x + ((rg & FME_PK_RANGE_RIGHT) ? 1 : 0));
  j.lt_y = (int16_t)(p.mv_y - ((rg & FME_PK_RANGE_TOP) ? 1 : 0));
  j.rb_y = (int16_t)(p.mv_y + ((rg & FME_PK_RANGE_BOTTOM) ? 1 : 0));
  j.key_offset = keyed ? base + s - w * h : -1;
  dst[i] = j;
}

hipError_t launch_unpack_jobs(const fme_job_packed* src, const int32_t* key_base, fme_job* dst, int n,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_jobs, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, src, key_base, dst, n);
  return hipGetLastError();
}

hipError_t launch_nn_tail(const BatchArgs& a, const WorkBufs& w, const float* nn_params,
                          int state_in, hipStream_t s) {
  const int nb = nblocks(a.n);
  hipLaunchKernelGGL(k_nn_tail, dim3(nb), dim3(kTailNT), 0, s, a, w, nn_params, state_in);
  return hipGetLastError();
}

}  // namespace fme
