// fme_nn_deep.hip — generic (deeper) NN_pred nets + the xMotionEstimation tail (nn_mode 2).
//
// BASELINE.json configs[4] runs a deeper NN_pred on 1080p.  The nets are the reference's own
// deeper variants (include/fme.h fme_nn_net):
//   Backups/4 "SCR 3 layers": 9 -> 40 -> 40 -> 40 -> 49, double, sigmoid output
//     (TEncSearch - SCR 3 layers - no normalization.cpp:4427-4486);
//   Backups/15 "blowing 4 lyrs qp 22": 17 -> 4 x 40 -> 49, float (… 4 lyrs qp 22.cpp:4954-5052);
//   the master net 17 -> 22 -> 20 -> 49 (TEncSearch.cpp:85-134) through the same code.
// Hidden layers are zero-padded to 40 units (a padded unit is relu(0 + 0) * 0 + 0 = 0 and adds
// +0 to every later sum, so the padding changes no result bit).
//
// One block = one 1024-job scan block (kJobsPerScanBlock) in 4 rounds of 256 jobs, so the stale
// array_e / C / PU-size state resolves exactly as in k_nn_tail: a prefix-max of "last writer"
// job indices (carry-in from k_scatter's blk_prefix, then round by round).  Per job:
//   ENGINE EXACT: one lane per job; every dot product in k order with a separate rounding per
//     product and per add (this file is compiled with -ffp-contract=off), weights as wave-uniform
//     scalar loads (SGPR operands), activations in VGPRs.  Bit-exact to the reference's loops.
//   ENGINE MFMA: each wave stages its 64 jobs' activations in LDS and runs every layer as a
//     [64 jobs] x [K] x [48 units] GEMM on v_mfma_f32_16x16x4_f32 (float nets) or
//     v_mfma_f64_16x16x4_f64 (double nets): 4 x 3 output tiles, K / 4 MFMAs each.  The MFMA result
//     is a k-ordered FMA chain (one rounding per step), so a class can differ from the exact
//     engine on a near-tie; fme_set_nn_margin_output reports top-1 minus top-2 to measure that.
// Then argmax (first maximum, std::max_element), class -> (cls%7-3, cls/7-3), and the cost tail
// (TEncSearch.cpp:4586-4597) exactly as k_nn_tail.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "fme_device.h"
#include "fme_simd.h"

namespace fme {

using simd::mv_bits;
using simd::mv_cost;

namespace {

constexpr int kRound = 256;                       // jobs per round = threads per block
constexpr int kRounds = kJobsPerScanBlock / kRound;
constexpr int kHW = FME_NN_MAX_WIDTH;             // hidden width (padded)
constexpr int kHP = 48;                           // hidden rows padded to 3 MFMA tiles
constexpr int kOP = 64;                           // output rows padded to 4 MFMA tiles
constexpr int kAS = 65;                           // LDS activation row stride (elements)
#ifndef FME_DEEP_MALL
#define FME_DEEP_MALL 1
#endif
#ifndef FME_DEEP_BHOIST
#define FME_DEEP_BHOIST 1
#endif


// Embedding rows: W (and Backups/15's H) 4,8,12,16,24,32,64 -> 1..7; the master's H swaps 12/16.
__device__ __forceinline__ int row_w(int v) {
  return v == 4 ? 1 : v == 8 ? 2 : v == 12 ? 3 : v == 16 ? 4 : v == 24 ? 5 : v == 32 ? 6 : v == 64 ? 7 : 0;
}
__device__ __forceinline__ int row_h_master(int v) {
  return v == 4 ? 1 : v == 8 ? 2 : v == 16 ? 3 : v == 12 ? 4 : v == 24 ? 5 : v == 32 ? 6 : v == 64 ? 7 : 0;
}

template <typename T>
__device__ __forceinline__ T relu(T x) { return x > (T)0 ? x : (T)0; }   // Backups/4:292-295

__device__ __forceinline__ float nn_exp(float x) { return expf(x); }
__device__ __forceinline__ double nn_exp(double x) { return exp(x); }

}  // namespace

// Packed device layout (elements of T), built by nn_deep_pack: fixed offsets for a given
// (n_hidden, embedding) so the exact engine's weight reads are compile-time scalar loads.
template <int NH, bool EMB>
struct DeepLayout {
  static constexpr int K0 = EMB ? 17 : 9;                  // real layer-1 fan-in
  static constexpr int KP0 = EMB ? 20 : 12;                // padded to a multiple of 4 (MFMA K)
  static constexpr int kEmb0 = 0, kEmb1 = 32;
  static constexpr int kGin = 64, kMean = 80, kStd = 96;  // 9 each (16-element slots)
  static constexpr int kp(int l) { return l == 0 ? KP0 : kHW; }
  static constexpr int w(int l) { return l == 0 ? 112 : w(l - 1) + kHP * kp(l - 1) + 3 * kHP; }
  static constexpr int b(int l) { return w(l) + kHP * kp(l); }
  static constexpr int g(int l) { return b(l) + kHP; }
  static constexpr int be(int l) { return g(l) + kHP; }
  static constexpr int kWout = w(NH);
  static constexpr int kBout = kWout + kOP * kHW;
  static constexpr int kTotal = kBout + kOP;
};


struct DeepArgs {
  const void* P;          // packed parameters (float or double)
  float* margin;          // [n] or null
  void* logits;           // [n][49] of T (OUT before the output activation) or null
  int32_t emb_mode;       // FME_NN_EMB_MASTER / FME_NN_EMB_SWAP (EMB kernels)
  int32_t out_act;        // FME_NN_OUT_*
  uint32_t in_flags;      // FME_NN_IN_*
};

// ---- exact engine: one lane per job ----------------------------------------------------------
// One layer, fully unrolled (compile-time fan-in / rows): y[i] = act(sum_k W[i][k] * x[k] + b[i]).
template <typename T, int K, int KP, int ROWS, bool HIDDEN>
__device__ __forceinline__ void layer_exact(const T* __restrict__ W, const T* __restrict__ b, const T* __restrict__ g,
                                            const T* __restrict__ be, const T* x, T* y) {
#pragma unroll
  for (int i = 0; i < ROWS; i++) {
    T s = (T)0;
#pragma unroll
    for (int k = 0; k < K; k++) s = s + W[i * KP + k] * x[k];
    s = s + b[i];
    y[i] = HIDDEN ? relu(s) * g[i] + be[i] : s;
  }
}

template <typename T, int NH, bool EMB, int L>
struct HiddenChain {   // layers L..NH-1 from x (in registers), result in x
  static __device__ __forceinline__ void run(const T* __restrict__ P, T (&x)[kHW]) {
    using D = DeepLayout<NH, EMB>;
    T y[kHW];
    layer_exact<T, kHW, kHW, kHW, true>(P + D::w(L), P + D::b(L), P + D::g(L), P + D::be(L), x, y);
#pragma unroll
    for (int i = 0; i < kHW; i++) x[i] = y[i];
    HiddenChain<T, NH, EMB, L + 1>::run(P, x);
  }
};
template <typename T, int NH, bool EMB>
struct HiddenChain<T, NH, EMB, NH> {
  static __device__ __forceinline__ void run(const T* __restrict__, T (&)[kHW]) {}
};

template <typename T, int NH, bool EMB>
__device__ __forceinline__ void forward_exact(const T* __restrict__ P, const T (&in)[17], T (&out)[49]) {
  using D = DeepLayout<NH, EMB>;
  T x[kHW];
  layer_exact<T, D::K0, D::KP0, kHW, true>(P + D::w(0), P + D::b(0), P + D::g(0), P + D::be(0), in, x);
  HiddenChain<T, NH, EMB, 1>::run(P, x);
  layer_exact<T, kHW, kHW, 49, false>(P + D::kWout, P + D::kBout, nullptr, nullptr, x, out);
}

// ---- MFMA engine: one wave = 64 jobs, activations in LDS [64][kAS] ------------------------------
template <typename T>
struct Mfma;
template <>
struct Mfma<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // C/D map of the f32 16x16 forms: col = lane & 15, row = 4 * (lane >> 4) + r
  static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};
template <>
struct Mfma<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // f64 16x16x4: col = lane & 15, row = (lane >> 4) + 4 * r
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

// act[0..63][0..K) (this wave's rows) -> act[0..63][0..NP) = epilogue(act * W^T).  Rows of one
// 16-job tile are read only while that tile is computed, so the tile is overwritten in place.
template <typename T, int K, int NP, bool HIDDEN>
__device__ __forceinline__ void layer_mfma(T* act, const T* __restrict__ W, const T* __restrict__ b,
                                           const T* __restrict__ g, const T* __restrict__ be, int lane) {
  using M = Mfma<T>;
  constexpr int NT = NP / 16;
  const int c16 = lane & 15, k4 = lane >> 4;
  // HOIST: the layer's B fragments (B[k][unit] = W[unit][k]) loaded once per wave, all in flight
  // before the first MFMA and reused by the four 16-job tiles, instead of a load per (tile, k-step,
  // unit tile) that kept each MFMA behind a global-load latency.  The double nets run at one wave
  // per SIMD anyway (33 KB of LDS activations per wave); the float ones would lose their second
  // wave to the registers (FME_DEEP_BHOIST: 1 double only, 2 both, 0 neither).
  constexpr bool HOIST = FME_DEEP_BHOIST >= 2 || (FME_DEEP_BHOIST == 1 && sizeof(T) == 8);
  T bw[HOIST ? K / 4 : 1][NT];
  if constexpr (HOIST) {
#pragma unroll
    for (int kk = 0; kk < K / 4; kk++)
#pragma unroll
      for (int nt = 0; nt < NT; nt++) bw[kk][nt] = W[(nt * 16 + c16) * K + kk * 4 + k4];
  }
  // ALL (FME_DEEP_MALL): the four 16-job tiles' accumulators in flight together, k outermost, so
  // 4 * NT independent MFMA chains hide the f64 MFMA latency at one wave per SIMD (the tile-by-tile
  // order had NT = 3 or 4 chains); each accumulator still sums k in the same order (same bits).
  constexpr int MG = FME_DEEP_MALL ? 4 : 1;   // tiles per pass
#pragma unroll
  for (int m0 = 0; m0 < 4; m0 += MG) {
    typename M::acc_t acc[MG][NT];
#pragma unroll
    for (int mi = 0; mi < MG; mi++)
#pragma unroll
      for (int nt = 0; nt < NT; nt++) acc[mi][nt] = typename M::acc_t{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < K / 4; kk++) {
#pragma unroll
      for (int mi = 0; mi < MG; mi++) {
        const T a = act[((m0 + mi) * 16 + c16) * kAS + kk * 4 + k4];   // A[job][k]
#pragma unroll
        for (int nt = 0; nt < NT; nt++) {
          const T b = HOIST ? bw[HOIST ? kk : 0][nt] : W[(nt * 16 + c16) * K + kk * 4 + k4];
          acc[mi][nt] = M::mma(a, b, acc[mi][nt]);
        }
      }
    }
    if constexpr (sizeof(T) == 8) {
      // v_mfma_f64_16x16x4_f64 on gfx950 writes its upper accumulator registers (rows 8..15 of
      // the tile) later than the compiler's hazard model pads for: measured on the box, those
      // rows were read stale in every tile but the last (tools/deep_probe.py).  Pad explicitly:
      // the accumulators are operands of the pad, so no read of them is placed before it.
#pragma unroll
      for (int mi = 0; mi < MG; mi++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(acc[mi][nt]));
    }
#pragma unroll
    for (int nt = 0; nt < NT; nt++) {
      const int col = nt * 16 + c16;
      T bb = b[col], gg = (T)0, bbe = (T)0;
      if (HIDDEN) {
        gg = g[col];
        bbe = be[col];
      }
#pragma unroll
      for (int mi = 0; mi < MG; mi++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          T s = acc[mi][nt][r] + bb;
          if (HIDDEN) s = relu(s) * gg + bbe;
          act[((m0 + mi) * 16 + M::row(lane, r)) * kAS + col] = s;
        }
    }
  }
}

template <typename T, int NH, bool EMB, int L>
struct MfmaChain {   // hidden layers L..NH-1, in place in this wave's LDS rows
  static __device__ __forceinline__ void run(const T* __restrict__ P, T* act, int lane) {
    using D = DeepLayout<NH, EMB>;
    layer_mfma<T, kHW, kHP, true>(act, P + D::w(L), P + D::b(L), P + D::g(L), P + D::be(L), lane);
    MfmaChain<T, NH, EMB, L + 1>::run(P, act, lane);
  }
};
template <typename T, int NH, bool EMB>
struct MfmaChain<T, NH, EMB, NH> {
  static __device__ __forceinline__ void run(const T* __restrict__, T*, int) {}
};

template <typename T, int NH, bool EMB>
__device__ __forceinline__ void forward_mfma(const T* __restrict__ P, T* act, int lane) {
  using D = DeepLayout<NH, EMB>;
  layer_mfma<T, D::KP0, kHP, true>(act, P + D::w(0), P + D::b(0), P + D::g(0), P + D::be(0), lane);
  MfmaChain<T, NH, EMB, 1>::run(P, act, lane);
  layer_mfma<T, kHW, kOP, false>(act, P + D::kWout, P + D::kBout, nullptr, nullptr, lane);
}


// x = ((T)raw - mean) / stdev * gamma_in for raw = e0..e3, C, e4..e7, after the two embedding rows
// (TEncSearch.cpp:88-113, Backups/4:4427-4441, Backups/15:4966-5005).
template <typename T, bool EMB>
__device__ __forceinline__ void nn_inputs(const T* __restrict__ P, int emb_mode, const uint32_t (&e)[8], uint32_t c,
                                          uint32_t ph, uint32_t pw, T (&in)[17]) {
  using D = DeepLayout<1, EMB>;   // the embedding / normalisation offsets do not depend on NH
  int k0 = 0;
  if (EMB) {
    const int rh = emb_mode == FME_NN_EMB_SWAP ? row_w((int)ph) : row_h_master((int)ph);
    const int rw = row_w((int)pw);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      in[k] = P[D::kEmb0 + rh * 4 + k];
      in[4 + k] = P[D::kEmb1 + rw * 4 + k];
    }
    k0 = 8;
  }
  const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const T v = ((T)raw[k] - P[D::kMean + k]) / P[D::kStd + k];
    in[k0 + k] = v * P[D::kGin + k];
  }
#pragma unroll
  for (int k = k0 + 9; k < 17; k++) in[k] = (T)0;
}

// Output activation, first maximum (std::max_element) and the top-1 minus top-2 margin.
template <typename T>
__device__ __forceinline__ int nn_argmax(T (&out)[49], int out_act, float* margin) {
  if (out_act == FME_NN_OUT_SIGMOID) {
#pragma unroll
    for (int o = 0; o < 49; o++) out[o] = (T)1 / ((T)1 + nn_exp(-out[o]));
  }
  int cls = 0;
  T best = out[0];
#pragma unroll
  for (int o = 1; o < 49; o++) {
    if (best < out[o]) {
      best = out[o];
      cls = o;
    }
  }
  if (margin) {
    T second = cls == 0 ? out[1] : out[0];
#pragma unroll
    for (int o = 1; o < 49; o++)
      if (o != cls && second < out[o]) second = out[o];
    *margin = (float)(best - second);
  }
  return cls;
}

template <typename T, int NH, bool EMB, bool MFMA>
__global__ __launch_bounds__(kRound) void k_nn_deep_tail(BatchArgs a, WorkBufs w, DeepArgs d, int state_in) {
  using L = DeepLayout<NH, EMB>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  __shared__ int32_t wave_tot[kRound / 64][9];
  const T* __restrict__ P = static_cast<const T*>(d.P);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  T* act = reinterpret_cast<T*>(smem_raw) + (MFMA ? wid * 64 * kAS : 0);
  const uint32_t* st_in = w.nn_state + 12 * state_in;
  uint32_t* st_out = w.nn_state + 12 * (state_in ^ 1);
  if (w.sched->invalid) {
    for (int rnd = 0; rnd < kRounds; rnd++) {
      const int i = blockIdx.x * kJobsPerScanBlock + rnd * kRound + tid;
      if (i < a.n) reject_job(a, w, i, state_in);
    }
    return;
  }

  int carry[9];
#pragma unroll
  for (int f = 0; f < 9; f++) carry[f] = w.blk_prefix[blockIdx.x * 9 + f];

  for (int rnd = 0; rnd < kRounds; rnd++) {
    const int i = blockIdx.x * kJobsPerScanBlock + rnd * kRound + tid;
    const bool valid = i < a.n;
    if (!__syncthreads_or(valid)) break;
    fme_job j{};
    if (valid) j = a.jobs[i];
    // writer indices of this job, prefix-max over the round (carry from earlier rounds/blocks)
    int run[9];
    const bool wr = valid && nn_writes_c(j);
    {
      const int np = wr ? nn_pushes(j) : 0;
#pragma unroll
      for (int s = 0; s < 8; s++) run[s] = (np > s) ? i : -1;
      run[8] = wr ? i : -1;
    }
    // FME_NN_IN_SLOT_RESET: the backups memset array_e on every call, so only this call's own
    // pushes are non-zero (Backups/4:4421-4422, Backups/15:4961-4962) and only C / PU size carry.
    // A round whose every job writes them (the backups' input path: every uni-pred job) needs no
    // scan at all: each job is its own last writer, and the carry is the round's last job.
    const bool reset = (d.in_flags & FME_NN_IN_SLOT_RESET) != 0;
    int src[9];
    if (reset && __syncthreads_and(!valid || wr)) {
#pragma unroll
      for (int f = 0; f < 9; f++) src[f] = run[f];
      carry[8] = min(a.n, blockIdx.x * kJobsPerScanBlock + (rnd + 1) * kRound) - 1;
    } else {
      int tot[9];
      writer_scan<kRound / 64>(run, carry, blockIdx.x * kJobsPerScanBlock + rnd * kRound, wave_tot, src, tot);
#pragma unroll
      for (int f = 0; f < 9; f++) carry[f] = tot[f];
      __syncthreads();   // wave_tot is rewritten next round
    }

    // the NN_pred() inputs this job sees (TEncSearch.cpp:88-113 / Backups/15:4944-5000)
    uint32_t e[8];
    uint32_t written = st_in[11];
#pragma unroll
    for (int s = 0; s < 8; s++) {
      if (reset) {
        e[s] = (valid && src[s] == i) ? search_rec(a, w, i)->emi[s] : 0u;
        written |= 1u << s;
      } else if (src[s] >= 0) {
        e[s] = valid ? search_rec(a, w, src[s])->emi[s] : 0u;
        written |= 1u << s;
      } else {
        e[s] = st_in[s];
      }
    }
    uint32_t c = st_in[8], ph = st_in[9], pw = st_in[10];
    if (src[8] >= 0 && valid) {
      c = search_rec(a, w, src[8])->c;
      ph = a.jobs[src[8]].h;
      pw = a.jobs[src[8]].w;
      written |= 0x100u;
    }
    T in[17];
    nn_inputs<T, EMB>(P, d.emb_mode, e, c, ph, pw, in);
    T out[49];
    if (MFMA) {
#pragma unroll
      for (int k = 0; k < L::KP0; k++) act[lane * kAS + k] = k < L::K0 ? in[k] : (T)0;
      forward_mfma<T, NH, EMB>(P, act, lane);
#pragma unroll
      for (int o = 0; o < 49; o++) out[o] = act[lane * kAS + o];
    } else {
      forward_exact<T, NH, EMB>(P, in, out);
    }
    if (!valid) continue;
    if (d.logits) {
      T* lg = static_cast<T*>(d.logits) + (size_t)i * 49;
#pragma unroll
      for (int o = 0; o < 49; o++) lg[o] = out[o];
    }
    const int cls = nn_argmax(out, d.out_act, d.margin ? d.margin + i : nullptr);

    fme_result* r = a.res + i;
    const fme_result* sr = search_rec(a, w, i);
    uint16_t status = 0;
    if (!nn_writes_c(j) || sr->n_emi < 8) status |= FME_RES_NN_STALE;
    if ((written & 0x1FFu) != 0x1FFu) status |= FME_RES_NN_UNINIT;
    if (i == a.n - 1) {
#pragma unroll
      for (int s = 0; s < 8; s++) st_out[s] = e[s];
      st_out[8] = c;
      st_out[9] = ph;
      st_out[10] = pw;
      st_out[11] = written;
    }
    const int fx = 4 * sr->mv_int_x + cls % 7 - 3, fy = 4 * sr->mv_int_y + cls / 7 - 3;
    const double ml = a.mlambda[j.lambda_id];
    const uint32_t mvb = mv_bits(fx, fy, 0, j.mvp_x, j.mvp_y);
    const uint32_t bits = (uint32_t)j.bits_in + mvb;
    const double fw = (j.flags & FME_JOB_BIPRED) ? 0.5 : 1.0;
    const double val = floor(fw * ((double)sr->frac_cost - (double)mv_cost(ml, mvb))) + (double)mv_cost(ml, bits);
    // gcc/x86-64 (Distortion)(double) semantics for the cost
    store_outputs(r, sr, w.mv_out, i, fx, fy, (uint32_t)(int64_t)val, bits, (uint8_t)cls, status);
  }
}

// NN_pred() of the generic net on one explicit input (fme_nn_pred_single, nn_mode 2):
// in11 = array_e slots[8], C, PUHeight, PUWidth.
// The exact engine's arithmetic with the rows of each layer spread over the wave (lane i owns row i;
// every row still sums k = 0.. in order with separate roundings), activations through LDS, then
// the first maximum by a (value, row) reduction: one dependent chain per layer per call.
template <typename T, int NH, bool EMB>
__global__ __launch_bounds__(64) void k_nn_deep_single(DeepArgs d, NnIn11 in11, int32_t* out, uint32_t* flag,
                                                       uint32_t seq) {
  using D = DeepLayout<NH, EMB>;
  __shared__ T s_x[2][kHW];
  const T* __restrict__ P = static_cast<const T*>(d.P);
  const int i = (int)threadIdx.x;
  uint32_t e[8];
#pragma unroll
  for (int q = 0; q < 8; q++) e[q] = in11.v[q];
  T in[17];
  nn_inputs<T, EMB>(P, d.emb_mode, e, in11.v[8], in11.v[9], in11.v[10], in);
  if (i < kHW) {
    T s = (T)0;
#pragma unroll
    for (int k = 0; k < D::K0; k++) s = s + P[D::w(0) + i * D::KP0 + k] * in[k];
    s = s + P[D::b(0) + i];
    s_x[0][i] = relu(s) * P[D::g(0) + i] + P[D::be(0) + i];
  }
  __syncthreads();
#pragma unroll
  for (int l = 1; l < NH; l++) {
    if (i < kHW) {
      T s = (T)0;
#pragma unroll
      for (int k = 0; k < kHW; k++) s = s + P[D::w(l) + i * kHW + k] * s_x[(l - 1) & 1][k];
      s = s + P[D::b(l) + i];
      s_x[l & 1][i] = relu(s) * P[D::g(l) + i] + P[D::be(l) + i];
    }
    __syncthreads();
  }
  T bv = (T)0;
  int bi = 64;
  if (i < 49) {
    T s = (T)0;
#pragma unroll
    for (int k = 0; k < kHW; k++) s = s + P[D::kWout + i * kHW + k] * s_x[(NH - 1) & 1][k];
    s = s + P[D::kBout + i];
    if (d.out_act == FME_NN_OUT_SIGMOID) s = (T)1 / ((T)1 + nn_exp(-s));
    // the serial rule's NaNs (cls = 0, then `best < out[o]`): a NaN row 0 wins, a later NaN never
    if (s != s) s = i == 0 ? (T)INFINITY : (T)-INFINITY;
    bv = s;
    bi = i;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (oi < 64 && (bi == 64 || ov > bv || (ov == bv && oi < bi))) {
      bv = ov;
      bi = oi;
    }
  }
  if (i == 0) {
    out[0] = bi;
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
template <int NH, bool EMB, typename T>
static void pack_into(const fme_nn_net& n, const double* p, T* Q) {
  using L = DeepLayout<NH, EMB>;
  for (int i = 0; i < L::kTotal; i++) Q[i] = (T)0;
  const double* s = p;
  if (EMB) {
    for (int i = 0; i < 64; i++) Q[i] = (T)s[i];
    s += 64;
  }
  int fan = L::K0;
  for (int l = 0; l < NH; l++) {
    const int wd = n.width[l], kp = L::kp(l);
    for (int i = 0; i < wd; i++)
      for (int k = 0; k < fan; k++) Q[L::w(l) + i * kp + k] = (T)s[i * fan + k];
    s += wd * fan;
    for (int i = 0; i < wd; i++) Q[L::b(l) + i] = (T)s[i];
    s += wd;
    for (int i = 0; i < wd; i++) Q[L::g(l) + i] = (T)s[i];
    s += wd;
    for (int i = 0; i < wd; i++) Q[L::be(l) + i] = (T)s[i];
    s += wd;
    fan = wd;
  }
  for (int i = 0; i < 49; i++)
    for (int k = 0; k < fan; k++) Q[L::kWout + i * kHW + k] = (T)s[i * fan + k];
  s += 49 * fan;
  for (int i = 0; i < 49; i++) Q[L::kBout + i] = (T)s[i];
  s += 49;
  for (int k = 0; k < 9; k++) {
    Q[L::kGin + k] = (T)s[k];
    Q[L::kMean + k] = (T)s[9 + k];
    Q[L::kStd + k] = (T)s[18 + k];
  }
}

// This file is compiled once per (precision, engine) with -DFME_DEEP_T=float|double
// -DFME_DEEP_MFMA=0|1 (the kernels, 8 per object, so the four objects build in parallel) and
// once without FME_DEEP_T (the host side: packing and dispatch).
#ifdef FME_DEEP_T
#define FME_CAT2(a, b, c) a##b##c
#define FME_CAT(a, b, c) FME_CAT2(a, b, c)
#define FME_DEEP_SUFFIX FME_CAT(FME_DEEP_T, _, FME_DEEP_MFMA)

template <int NH, bool EMB>
static hipError_t launch_one(const BatchArgs& a, const WorkBufs& w, const DeepArgs& d, int state_in, hipStream_t s) {
  using T = FME_DEEP_T;
  const int nb = (a.n + kJobsPerScanBlock - 1) / kJobsPerScanBlock;
  const size_t lds = FME_DEEP_MFMA ? sizeof(T) * (kRound / 64) * 64 * kAS : 0;
  hipLaunchKernelGGL((k_nn_deep_tail<T, NH, EMB, FME_DEEP_MFMA != 0>), dim3(nb), dim3(kRound), lds, s, a, w, d,
                     state_in);
  return hipGetLastError();
}

hipError_t FME_CAT(launch_deep_, FME_DEEP_SUFFIX, )(int nh, bool emb, const BatchArgs& a, const WorkBufs& w,
                                                    const DeepArgs& d, int state_in, hipStream_t s) {
  switch (nh * 2 + (emb ? 1 : 0)) {
    case 2: return launch_one<1, false>(a, w, d, state_in, s);
    case 3: return launch_one<1, true>(a, w, d, state_in, s);
    case 4: return launch_one<2, false>(a, w, d, state_in, s);
    case 5: return launch_one<2, true>(a, w, d, state_in, s);
    case 6: return launch_one<3, false>(a, w, d, state_in, s);
    case 7: return launch_one<3, true>(a, w, d, state_in, s);
    case 8: return launch_one<4, false>(a, w, d, state_in, s);
    case 9: return launch_one<4, true>(a, w, d, state_in, s);
    default: return hipErrorInvalidValue;
  }
}

#if !FME_DEEP_MFMA
template <int NH, bool EMB>
static hipError_t single_one(const DeepArgs& d, const NnIn11& in11, int32_t* out, uint32_t* flag, uint32_t seq,
                             hipStream_t s) {
  hipLaunchKernelGGL((k_nn_deep_single<FME_DEEP_T, NH, EMB>), dim3(1), dim3(64), 0, s, d, in11, out, flag, seq);
  return hipGetLastError();
}
hipError_t FME_CAT(single_deep_, FME_DEEP_T, )(int nh, bool emb, const DeepArgs& d, const NnIn11& in11,
                                               int32_t* out, uint32_t* flag, uint32_t seq, hipStream_t s) {
  switch (nh * 2 + (emb ? 1 : 0)) {
    case 2: return single_one<1, false>(d, in11, out, flag, seq, s);
    case 3: return single_one<1, true>(d, in11, out, flag, seq, s);
    case 4: return single_one<2, false>(d, in11, out, flag, seq, s);
    case 5: return single_one<2, true>(d, in11, out, flag, seq, s);
    case 6: return single_one<3, false>(d, in11, out, flag, seq, s);
    case 7: return single_one<3, true>(d, in11, out, flag, seq, s);
    case 8: return single_one<4, false>(d, in11, out, flag, seq, s);
    case 9: return single_one<4, true>(d, in11, out, flag, seq, s);
    default: return hipErrorInvalidValue;
  }
}
#endif

#else   // host side

hipError_t launch_deep_float_0(int, bool, const BatchArgs&, const WorkBufs&, const DeepArgs&, int, hipStream_t);
hipError_t launch_deep_float_1(int, bool, const BatchArgs&, const WorkBufs&, const DeepArgs&, int, hipStream_t);
hipError_t launch_deep_double_0(int, bool, const BatchArgs&, const WorkBufs&, const DeepArgs&, int, hipStream_t);
hipError_t launch_deep_double_1(int, bool, const BatchArgs&, const WorkBufs&, const DeepArgs&, int, hipStream_t);
hipError_t single_deep_float(int, bool, const DeepArgs&, const NnIn11&, int32_t*, uint32_t*, uint32_t, hipStream_t);
hipError_t single_deep_double(int, bool, const DeepArgs&, const NnIn11&, int32_t*, uint32_t*, uint32_t, hipStream_t);

static bool deep_supported(const fme_nn_net& n) {
  if (n.n_hidden < 1 || n.n_hidden > FME_NN_MAX_HIDDEN) return false;
  for (int l = 0; l < n.n_hidden; l++)
    if (n.width[l] < 1 || n.width[l] > kHW) return false;
  return n.precision == FME_NN_F32 || n.precision == FME_NN_F64;
}

size_t nn_deep_packed_bytes(const fme_nn_net& n) {
  if (!deep_supported(n)) return 0;
  const size_t el = n.precision == FME_NN_F64 ? sizeof(double) : sizeof(float);
  switch (n.n_hidden * 2 + (n.embedding ? 1 : 0)) {
    case 2: return el * DeepLayout<1, false>::kTotal;
    case 3: return el * DeepLayout<1, true>::kTotal;
    case 4: return el * DeepLayout<2, false>::kTotal;
    case 5: return el * DeepLayout<2, true>::kTotal;
    case 6: return el * DeepLayout<3, false>::kTotal;
    case 7: return el * DeepLayout<3, true>::kTotal;
    case 8: return el * DeepLayout<4, false>::kTotal;
    default: return el * DeepLayout<4, true>::kTotal;
  }
}

template <typename T>
static void pack_t(const fme_nn_net& n, const double* p, T* q) {
  switch (n.n_hidden * 2 + (n.embedding ? 1 : 0)) {
    case 2: return pack_into<1, false, T>(n, p, q);
    case 3: return pack_into<1, true, T>(n, p, q);
    case 4: return pack_into<2, false, T>(n, p, q);
    case 5: return pack_into<2, true, T>(n, p, q);
    case 6: return pack_into<3, false, T>(n, p, q);
    case 7: return pack_into<3, true, T>(n, p, q);
    case 8: return pack_into<4, false, T>(n, p, q);
    default: return pack_into<4, true, T>(n, p, q);
  }
}

void nn_deep_pack(const fme_nn_net& n, const double* params, void* out) {
  if (n.precision == FME_NN_F64)
    pack_t<double>(n, params, static_cast<double*>(out));
  else
    pack_t<float>(n, params, static_cast<float*>(out));
}

hipError_t launch_nn_deep_tail(const fme_nn_net& n, const void* packed, float* margin, void* logits, const BatchArgs& a,
                               const WorkBufs& w, int state_in, int engine, hipStream_t s) {
  if (!deep_supported(n)) return hipErrorInvalidValue;
  const DeepArgs d{packed, margin, logits, n.embedding, n.out_act, n.input_flags};
  const bool emb = n.embedding != FME_NN_EMB_NONE, mfma = engine == FME_NN_ENGINE_MFMA;
  if (n.precision == FME_NN_F64)
    return (mfma ? launch_deep_double_1 : launch_deep_double_0)(n.n_hidden, emb, a, w, d, state_in, s);
  return (mfma ? launch_deep_float_1 : launch_deep_float_0)(n.n_hidden, emb, a, w, d, state_in, s);
}

hipError_t launch_nn_deep_single(const fme_nn_net& n, const void* packed, const NnIn11& in11, int32_t* out,
                                 uint32_t* flag, uint32_t seq, hipStream_t s) {
  if (!deep_supported(n)) return hipErrorInvalidValue;
  const DeepArgs d{packed, nullptr, nullptr, n.embedding, n.out_act, n.input_flags};
  const bool emb = n.embedding != FME_NN_EMB_NONE;
  return n.precision == FME_NN_F64 ? single_deep_double(n.n_hidden, emb, d, in11, out, flag, seq, s)
                                   : single_deep_float(n.n_hidden, emb, d, in11, out, flag, seq, s);
}
#endif

}  // namespace fme
