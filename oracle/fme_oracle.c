/*
 * fme_oracle.c — TEST INFRASTRUCTURE ONLY (see fme_oracle.h).
 *
 * Plain-C restatement of the reference path.  It does not build the m_filteredBlock planes
 * the reference builds (TEncSearch.cpp:6331-6532); it evaluates each candidate as the luma
 * prediction at its quarter-pel MV with the same two-stage 14-bit arithmetic
 * (TComInterpolationFilter.cpp:94-257), which the _ref harness shows equal to the plane
 * walk for every candidate.  Compile with -ffp-contract=off (the NN is float32, no FMA).
 */
#include "fme_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* HEVC luma taps, TComInterpolationFilter.cpp:57-63. */
static const int kLuma[4][8] = {
  {0, 0, 0, 64, 0, 0, 0, 0},
  {-1, 4, -10, 58, 17, -5, 1, 0},
  {-1, 4, -11, 40, 40, -11, 4, -1},
  {0, 1, -5, 17, 58, -10, 4, -1},
};

/* s_acMvRefineH / s_acMvRefineQ, TEncSearch.cpp:212-236 (x, y). */
static const int kRefineH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0},
                                   {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
static const int kRefineQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1},
                                   {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* TComRdCost::xGetExpGolombNumberOfBits, TComRdCost.cpp:172-185. */
uint32_t orc_eg_bits(int v) {
  uint32_t t = (v <= 0) ? ((uint32_t)(-v) << 1) + 1u : (uint32_t)v << 1;
  uint32_t len = 1;
  while (t != 1) {
    t >>= 1;
    len += 2;
  }
  return len;
}

/* TComRdCost::getCost / getCostOfVectorWithPredictor, TComRdCost.h:165-170. */
uint32_t orc_cost(double mlambda, uint32_t bits) {
  return (uint32_t)((mlambda * (double)bits) / 65536.0);
}

/* getBitsOfVectorWithPredictor, TComRdCost.h:171-174. */
static inline uint32_t mv_bits(int x, int y, int scale, int px, int py) {
  return orc_eg_bits(x * (1 << scale) - px) + orc_eg_bits(y * (1 << scale) - py);   /* x << scale (UB for x < 0 in C) */
}

/* Edge-replicated sample (TComPicYuv::extendPicBorder, TComPicYuv.cpp:229-276). */
static inline int ref_px(const orc_picture* p, int x, int y) {
  x = clampi(x, 0, p->width - 1);
  y = clampi(y, 0, p->height - 1);
  return p->luma16 ? p->luma16[(size_t)y * p->stride + x] : p->luma[(size_t)y * p->stride + x];
}
static inline int pic_bd(const orc_picture* p) { return p->bd > 8 ? p->bd : 8; }
static inline int pic_set(const orc_picture* p) { return p->luma != NULL || p->luma16 != NULL; }
/* headRoom = max(2, IF_INTERNAL_PREC - bitDepth): filterCopy's shift and the filters' headroom
 * (TComInterpolationFilter.cpp:113, 129, 201) - 6 at 8 bits, 4 at 10 */
static inline int if_headroom(int bd) { return 14 - bd < 2 ? 2 : 14 - bd; }

/* First (horizontal) stage output at integer row y: the 14-bit value the reference stores
 * in m_filteredBlockTmp[fx] (filterHor with isLast=false: filterCopy isFirst branch for
 * fx==0, TComInterpolationFilter.cpp:111-124, (s << headRoom) - 8192; filter<8,false,true,false>
 * otherwise, :196-252 with shift 6 - headRoom and offset -8192 << shift: shift 0 at 8 bits, 2 at
 * 10).  Stored as Pel (int16). */
static inline int hor_stage(const orc_picture* p, int x, int y, int fx) {
  const int hr = if_headroom(pic_bd(p));
  if (fx == 0) return (ref_px(p, x, y) << hr) - 8192;
  const int sh = 6 - hr;
  int s = 0;
  for (int k = 0; k < 8; k++) s += kLuma[fx][k] * ref_px(p, x + k - 3, y);
  return (int)(int16_t)((s - 8192 * (1 << sh)) >> sh);
}

/* Second (vertical, isLast) stage: filterCopy !isFirst branch for fy==0
 * (TComInterpolationFilter.cpp:126-150: (v + 8192 + (1 << (headRoom-1))) >> headRoom) and
 * filter<8,true,false,true> otherwise (shift 6 + headRoom, offset (1 << (shift-1)) + (8192 << 6):
 * 12 / 2048 at 8 bits, 10 / 512 at 10), clipped to [0, (1 << bitDepth) - 1]. */
int orc_pred_sample(const orc_picture* p, int x, int y, int fx, int fy) {
  const int bd = pic_bd(p), hr = if_headroom(bd);
  int v;
  if (fy == 0) {
    v = (hor_stage(p, x, y, fx) + 8192 + (1 << (hr - 1))) >> hr;
  } else {
    const int sh = 6 + hr;
    int s = 0;
    for (int k = 0; k < 8; k++) s += kLuma[fy][k] * hor_stage(p, x, y + k - 3, fx);
    v = (s + (1 << (sh - 1)) + (8192 << 6)) >> sh;
  }
  return clampi(v, 0, (1 << bd) - 1);
}

/* Prediction block of a PU at (x0,y0) displaced by quarter-pel (qx,qy). */
void orc_pred_block(const orc_picture* p, int x0, int y0, int w, int h, int qx, int qy,
                    int16_t* out) {
  const int ix = qx >> 2, iy = qy >> 2, fx = qx & 3, fy = qy & 3;
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++)
      out[r * w + c] = (int16_t)orc_pred_sample(p, x0 + ix + c, y0 + iy + r, fx, fy);
}

/* xCalcHADs4x4, TComRdCost.cpp:1234-1328: unnormalised 4x4 WHT of the difference,
 * sum of magnitudes, (s+1)>>1. */
static uint32_t had4x4(const int16_t* o, int os, const int16_t* c, int cs) {
  int d[16], m[16];
  for (int r = 0; r < 4; r++)
    for (int k = 0; k < 4; k++) d[r * 4 + k] = o[r * os + k] - c[r * cs + k];
  /* columns: butterfly over rows (0,3),(1,2) then pairs */
  for (int k = 0; k < 4; k++) {
    int a0 = d[k] + d[12 + k], a3 = d[k] - d[12 + k];
    int a1 = d[4 + k] + d[8 + k], a2 = d[4 + k] - d[8 + k];
    m[k] = a0 + a1;
    m[8 + k] = a0 - a1;
    m[4 + k] = a2 + a3;
    m[12 + k] = a3 - a2;
  }
  uint32_t s = 0;
  for (int r = 0; r < 4; r++) {
    int* q = &m[r * 4];
    int b0 = q[0] + q[3], b3 = q[0] - q[3], b1 = q[1] + q[2], b2 = q[1] - q[2];
    s += (uint32_t)abs(b0 + b1) + (uint32_t)abs(b0 - b1) + (uint32_t)abs(b2 + b3) +
         (uint32_t)abs(b3 - b2);
  }
  return (s + 1) >> 1;
}

/* xCalcHADs8x8, TComRdCost.cpp:1330-1425: any exact 8-point WHT factorisation gives the
 * same multiset of |coefficients|; (s+2)>>2. */
static void wht8(int* v, int step) {
  for (int len = 4; len >= 1; len >>= 1)
    for (int i = 0; i < 8; i += 2 * len)
      for (int j = i; j < i + len; j++) {
        int a = v[j * step], b = v[(j + len) * step];
        v[j * step] = a + b;
        v[(j + len) * step] = a - b;
      }
}

static uint32_t had8x8(const int16_t* o, int os, const int16_t* c, int cs) {
  int d[64];
  for (int r = 0; r < 8; r++)
    for (int k = 0; k < 8; k++) d[r * 8 + k] = o[r * os + k] - c[r * cs + k];
  for (int r = 0; r < 8; r++) wht8(&d[r * 8], 1);
  for (int k = 0; k < 8; k++) wht8(&d[k], 8);
  uint32_t s = 0;
  for (int i = 0; i < 64; i++) s += (uint32_t)abs(d[i]);
  return (s + 2) >> 2;
}

/* xGetHADs tiling, TComRdCost.cpp:1428-1495 (8x8 when both dims are multiples of 8). */
uint32_t orc_satd(const int16_t* org, int os, const int16_t* cur, int cs, int w, int h) {
  uint32_t s = 0;
  if ((w % 8) == 0 && (h % 8) == 0) {
    for (int y = 0; y < h; y += 8)
      for (int x = 0; x < w; x += 8) s += had8x8(org + y * os + x, os, cur + y * cs + x, cs);
  } else {
    for (int y = 0; y < h; y += 4)
      for (int x = 0; x < w; x += 4) s += had4x4(org + y * os + x, os, cur + y * cs + x, cs);
  }
  return s;
}

/* xGetSAD4..64/12/24/48 with row subsampling (iSubShift), TComRdCost.cpp:370-860. */
uint32_t orc_sad(const int16_t* org, int os, const int16_t* cur, int cs, int w, int h,
                 int sub_shift) {
  uint32_t s = 0;
  const int step = 1 << sub_shift;
  for (int y = 0; y < h; y += step)
    for (int x = 0; x < w; x++) s += (uint32_t)abs(org[y * os + x] - cur[y * cs + x]);
  return s << sub_shift;
}

/* xGetSSE4..64, TComRdCost.cpp:860-1205 (bit depth 8: no shift). */
uint32_t orc_sse(const int16_t* org, int os, const int16_t* cur, int cs, int w, int h) {
  uint32_t s = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int d = org[y * os + x] - cur[y * cs + x];
      s += (uint32_t)(d * d);
    }
  return s;
}

/* Integer-ME metric selected by the modified setDistParam (TComRdCost.cpp:200-230):
 * SSE for W in {4,8,16,32,64}; SAD for 12/24/48 with the FEN even-row subsampling of
 * xTZSearchHelp (TEncSearch.cpp:1158-1164).  Above 8 bits DISTORTION_PRECISION_ADJUSTMENT
 * (TypeDef.h:140-143, FULL_NBIT 0) drops bits: SAD >> (bd - 8) over the block (TComRdCost.cpp:
 * 370-536), SSE (d * d) >> 2 (bd - 8) per sample (:875-1130). */
static uint32_t int_dist(const int16_t* key, int ks, const int16_t* cur, int cs, int w, int h,
                         int fen, int bd) {
  if (w == 12 || w == 24 || w == 48) {
    int sub = ((fen == 1 || fen == 3) && h > 8) ? 1 : 0;
    return orc_sad(key, ks, cur, cs, w, h, sub) >> (bd - 8);
  }
  if (bd == 8) return orc_sse(key, ks, cur, cs, w, h);
  uint32_t s = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int d = key[y * ks + x] - cur[y * cs + x];
      s += (uint32_t)(d * d) >> (2 * (bd - 8));
    }
  return s;
}

/* xPatternSearchFracDIF (TEncSearch.cpp:5232-5269) with xPatternRefinement (1591-1645):
 * half stage at cost scale 1 around 2*mv_int, quarter stage at cost scale 0 around
 * 4*mv_int + 2*half; first strict minimum of distortion + MV cost in each stage. */
void orc_frac_dif(const orc_picture* p, const int16_t* key, int ks, int x0, int y0, int w, int h,
                  int mv_x, int mv_y, int mvp_x, int mvp_y, double mlambda, int use_hadamard,
                  int8_t half[2], int8_t qtr[2], uint32_t* cost) {
  int16_t* pred = (int16_t*)malloc(sizeof(int16_t) * (size_t)w * h);
  const int dsh = pic_bd(p) - 8;   /* xGetHADs / xGetSAD: uiSum >> (bitDepth - 8) */
  uint32_t best = 0xFFFFFFFFu;
  int bi = 0;
  for (int i = 0; i < 9; i++) {
    const int dx = kRefineH[i][0], dy = kRefineH[i][1];
    orc_pred_block(p, x0, y0, w, h, 4 * mv_x + 2 * dx, 4 * mv_y + 2 * dy, pred);
    uint32_t d = (use_hadamard ? orc_satd(key, ks, pred, w, w, h) : orc_sad(key, ks, pred, w, w, h, 0)) >> dsh;
    d += orc_cost(mlambda, mv_bits(2 * mv_x + dx, 2 * mv_y + dy, 1, mvp_x, mvp_y));
    if (d < best) {
      best = d;
      bi = i;
    }
  }
  const int hx = kRefineH[bi][0], hy = kRefineH[bi][1];
  best = 0xFFFFFFFFu;
  int qi = 0;
  for (int i = 0; i < 9; i++) {
    const int dx = kRefineQ[i][0], dy = kRefineQ[i][1];
    const int qx = 4 * mv_x + 2 * hx + dx, qy = 4 * mv_y + 2 * hy + dy;
    orc_pred_block(p, x0, y0, w, h, qx, qy, pred);
    uint32_t d = (use_hadamard ? orc_satd(key, ks, pred, w, w, h) : orc_sad(key, ks, pred, w, w, h, 0)) >> dsh;
    d += orc_cost(mlambda, mv_bits(qx, qy, 0, mvp_x, mvp_y));
    if (d < best) {
      best = d;
      qi = i;
    }
  }
  free(pred);
  half[0] = (int8_t)hx;
  half[1] = (int8_t)hy;
  qtr[0] = (int8_t)kRefineQ[qi][0];
  qtr[1] = (int8_t)kRefineQ[qi][1];
  *cost = best;
}

/* Visit order and range checks of xTZ8PointSquareSearch (TEncSearch.cpp:1324-1377):
 * TL,T,TR (row above in range), L, R, BL,B,BR (row below in range). */
static int square_points(int sx, int sy, int lt_x, int lt_y, int rb_x, int rb_y, int pts[8][2]) {
  int n = 0;
  const int top = sy - 1, bot = sy + 1, left = sx - 1, right = sx + 1;
  if (top >= lt_y) {
    if (left >= lt_x) { pts[n][0] = left; pts[n][1] = top; n++; }
    pts[n][0] = sx; pts[n][1] = top; n++;
    if (right <= rb_x) { pts[n][0] = right; pts[n][1] = top; n++; }
  }
  if (left >= lt_x) { pts[n][0] = left; pts[n][1] = sy; n++; }
  if (right <= rb_x) { pts[n][0] = right; pts[n][1] = sy; n++; }
  if (bot <= rb_y) {
    if (left >= lt_x) { pts[n][0] = left; pts[n][1] = bot; n++; }
    pts[n][0] = sx; pts[n][1] = bot; n++;
    if (right <= rb_x) { pts[n][0] = right; pts[n][1] = bot; n++; }
  }
  return n;
}

int orc_emi_push_count(int sx, int sy, int lt_x, int lt_y, int rb_x, int rb_y) {
  int pts[8][2];
  return square_points(sx, sy, lt_x, lt_y, rb_x, rb_y, pts);
}

/* EMI step: xTZ8PointSquareSearch(save=true) at the TZ best (TEncSearch.cpp:5043) with
 * xTZSearchHelp's normal branch (1155-1188): push the distortion, compare d, then d+cost,
 * against the running best; C = bestSad - cost(best) (5049-5050).  The incoming bestSad is
 * the TZ best's distortion + cost at cost scale 2, recomputed here. */
int orc_emi(const orc_picture* p, const int16_t* key, int ks, int x0, int y0, int w, int h,
            int sx, int sy, int mvp_x, int mvp_y, int lt_x, int lt_y, int rb_x, int rb_y,
            double mlambda, int fen, uint32_t emi[8], int* best_x, int* best_y, uint32_t* c) {
  int16_t* cur = (int16_t*)malloc(sizeof(int16_t) * (size_t)w * h);
  orc_pred_block(p, x0, y0, w, h, 4 * sx, 4 * sy, cur);
  uint32_t best_sad = int_dist(key, ks, cur, w, w, h, fen, pic_bd(p)) +
                      orc_cost(mlambda, mv_bits(sx, sy, 2, mvp_x, mvp_y));
  int bx = sx, by = sy;
  int pts[8][2];
  const int n = square_points(sx, sy, lt_x, lt_y, rb_x, rb_y, pts);
  for (int i = 0; i < n; i++) {
    orc_pred_block(p, x0, y0, w, h, 4 * pts[i][0], 4 * pts[i][1], cur);
    uint32_t d = int_dist(key, ks, cur, w, w, h, fen, pic_bd(p));
    emi[i] = d;
    if (d < best_sad) {
      d += orc_cost(mlambda, mv_bits(pts[i][0], pts[i][1], 2, mvp_x, mvp_y));
      if (d < best_sad) {
        best_sad = d;
        bx = pts[i][0];
        by = pts[i][1];
      }
    }
  }
  free(cur);
  *best_x = bx;
  *best_y = by;
  *c = best_sad - orc_cost(mlambda, mv_bits(bx, by, 2, mvp_x, mvp_y));
  return n;
}

/* ---- NN_pred(), TEncSearch.cpp:85-204 ------------------------------------------------ */
enum {
  P_EMB0 = 0, P_EMB1 = 32, P_W1 = 64, P_W2 = 438, P_W3 = 878, P_B1 = 1858, P_G1 = 1880,
  P_BE1 = 1902, P_B2 = 1924, P_G2 = 1944, P_BE2 = 1964, P_BOUT = 1984, P_GIN = 2033,
  P_MEAN = 2042, P_STD = 2051
};

/* Embedding rows by PUHeight (TEncSearch.cpp:93-102) and PUWidth (104-113). */
static int emb_row_h(int h) {
  switch (h) {
    case 4: return 1; case 8: return 2; case 16: return 3; case 12: return 4;
    case 24: return 5; case 32: return 6; case 64: return 7; default: return 0;
  }
}
static int emb_row_w(int w) {
  switch (w) {
    case 4: return 1; case 8: return 2; case 12: return 3; case 16: return 4;
    case 24: return 5; case 32: return 6; case 64: return 7; default: return 0;
  }
}

int orc_nn_forward(const float* P, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                   float* logits) {
  float in[17], x1[22], x2[20], out[49];
  const int rh = emb_row_h(pu_h), rw = emb_row_w(pu_w);
  for (int k = 0; k < 4; k++) {
    in[k] = P[P_EMB0 + rh * 4 + k];
    in[4 + k] = P[P_EMB1 + rw * 4 + k];
  }
  /* IN_errors << e0,e1,e2,e3,C,e4,e5,e6,e7 ; (x - mean) / stdev ; * BN_gamma_in */
  const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};
  for (int k = 0; k < 9; k++) {
    float v = (float)raw[k];
    v = (v - P[P_MEAN + k]) / P[P_STD + k];
    in[8 + k] = v * P[P_GIN + k];
  }
  for (int r = 0; r < 22; r++) {
    float s = 0.0f;
    for (int k = 0; k < 17; k++) s = s + P[P_W1 + r * 17 + k] * in[k];
    s = s + P[P_B1 + r];
    s = (s < 0.0f) ? 0.0f : s;
    x1[r] = s * P[P_G1 + r] + P[P_BE1 + r];
  }
  for (int r = 0; r < 20; r++) {
    float s = 0.0f;
    for (int k = 0; k < 22; k++) s = s + P[P_W2 + r * 22 + k] * x1[k];
    s = s + P[P_B2 + r];
    s = (s < 0.0f) ? 0.0f : s;
    x2[r] = s * P[P_G2 + r] + P[P_BE2 + r];
  }
  for (int r = 0; r < 49; r++) {
    float s = 0.0f;
    for (int k = 0; k < 20; k++) s = s + P[P_W3 + r * 20 + k] * x2[k];
    out[r] = s + P[P_BOUT + r];
  }
  int best = 0; /* Eigen maxCoeff: first index of the maximum */
  for (int r = 1; r < 49; r++)
    if (out[r] > out[best]) best = r;
  if (logits) memcpy(logits, out, sizeof(out));
  return best;
}

/* ---- generic nets (nn_mode 2) -------------------------------------------------------------
 * The reference's deeper nets, restated literally:
 *   Backups/4 "SCR 3 layers" (double): IN[k] = (U - mean) / stdev (:4427-4435), IN_norm = IN *
 *     BN_gamma_in (:4439-4441), X_l[i] += w * x for j in order from the memset 0 (:4445-4470),
 *     += b, relu * gamma + beta, OUT[i] += w * X3[j], += bout, sigmoid (:4472-4480),
 *     std::max_element (:4486);
 *   Backups/15 "blowing 4 lyrs qp 22" (float): the same per layer (:5007-5045) with embeddings
 *     (:4979-5000), no sigmoid, and X3 / X4 left out of the per-call memset (:4957-4961), so they
 *     start from the previous call's values.
 * relu is `x > 0 ? x : 0` (Backups/4:292-295, Backups/15:80-83). */
int orc_nn_param_count(const fme_nn_net* d) {
  if (!d || d->n_hidden < 1 || d->n_hidden > FME_NN_MAX_HIDDEN) return FME_E_INVALID;
  if (d->precision != FME_NN_F32 && d->precision != FME_NN_F64) return FME_E_INVALID;
  if (d->embedding < FME_NN_EMB_NONE || d->embedding > FME_NN_EMB_SWAP) return FME_E_INVALID;
  if (d->out_act != FME_NN_OUT_LINEAR && d->out_act != FME_NN_OUT_SIGMOID) return FME_E_INVALID;
  if (d->carry_hidden >> d->n_hidden) return FME_E_INVALID;
  if (d->input_flags & ~(FME_NN_IN_SLOT_RESET | FME_NN_IN_TZ_RING)) return FME_E_INVALID;
  if ((d->input_flags & FME_NN_IN_TZ_RING) && ((d->input_flags & FME_NN_IN_SLOT_RESET) || d->carry_hidden))
    return FME_E_INVALID;
  int n = d->embedding ? 64 : 0, in = d->embedding ? 17 : 9;
  for (int l = 0; l < d->n_hidden; l++) {
    const int w = d->width[l];
    if (w < 1 || w > FME_NN_MAX_WIDTH) return FME_E_INVALID;
    n += w * in + 3 * w;
    in = w;
  }
  return n + 49 * in + 49 + 27;
}

int orc_load_nn_net(orc_ctx* ctx, const fme_nn_net* d, const double* params, int count) {
  const int n = orc_nn_param_count(d);
  if (n < 0 || n != count || n > ORC_NN_NET_MAX_PARAMS) return FME_E_INVALID;
  ctx->net.d = *d;
  ctx->net.count = n;
  for (int i = 0; i < n; i++) {
    ctx->net.pd[i] = params[i];
    ctx->net.pf[i] = (float)params[i];
  }
  memset(ctx->net.carry_d, 0, sizeof(ctx->net.carry_d));
  memset(ctx->net.carry_f, 0, sizeof(ctx->net.carry_f));
  ctx->net.loaded = 1;
  return 0;
}

#define ORC_RELU(x) ((x) > 0 ? (x) : 0)
#define ORC_DEEP_FORWARD(NAME, T, EXPF)                                                          \
  static int NAME(const fme_nn_net* d, const T* P, T carry[][FME_NN_MAX_WIDTH], const uint32_t e[8], \
                  uint32_t c, int pu_h, int pu_w, double* logits, double* pre) {                  \
    T in[17], xa[FME_NN_MAX_WIDTH], xb[FME_NN_MAX_WIDTH], out[49];                                \
    const T* p = P;                                                                               \
    int nin = 0;                                                                                  \
    if (d->embedding) {                                                                           \
      const int rh = d->embedding == FME_NN_EMB_SWAP ? emb_row_w(pu_h) : emb_row_h(pu_h);         \
      const int rw = emb_row_w(pu_w);                                                             \
      for (int k = 0; k < 4; k++) {                                                               \
        in[k] = p[rh * 4 + k];                                                                    \
        in[4 + k] = p[32 + rw * 4 + k];                                                           \
      }                                                                                           \
      p += 64;                                                                                    \
      nin = 8;                                                                                    \
    }                                                                                             \
    const T* tail = P + orc_nn_param_count(d) - 27;                                               \
    const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};                  \
    for (int k = 0; k < 9; k++) {                                                                 \
      T v = (T)raw[k];                                                                            \
      v = (v - tail[9 + k]) / tail[18 + k];                                                       \
      in[nin + k] = v * tail[k];                                                                  \
    }                                                                                             \
    nin += 9;                                                                                     \
    const T* x = in;                                                                              \
    T* y = xa;                                                                                    \
    for (int l = 0; l < d->n_hidden; l++) {                                                       \
      const int w = d->width[l];                                                                  \
      const T *W = p, *b = p + w * nin, *g = b + w, *be = g + w;                                  \
      const int carried = (d->carry_hidden >> l) & 1;                                             \
      for (int i = 0; i < w; i++) {                                                               \
        T s = carried ? carry[l][i] : (T)0;                                                       \
        for (int k = 0; k < nin; k++) s = s + W[i * nin + k] * x[k];                              \
        s = s + b[i];                                                                             \
        s = ORC_RELU(s) * g[i] + be[i];                                                           \
        y[i] = s;                                                                                 \
        if (carried) carry[l][i] = s;                                                             \
      }                                                                                           \
      p = be + w;                                                                                 \
      x = y;                                                                                      \
      y = (y == xa) ? xb : xa;                                                                    \
      nin = w;                                                                                    \
    }                                                                                             \
    for (int i = 0; i < 49; i++) {                                                                \
      T s = 0;                                                                                    \
      for (int k = 0; k < nin; k++) s = s + p[i * nin + k] * x[k];                                \
      s = s + p[49 * nin + i];                                                                    \
      if (pre) pre[i] = (double)s;                                                                \
      if (d->out_act == FME_NN_OUT_SIGMOID) s = (T)1 / ((T)1 + EXPF(-s));                         \
      out[i] = s;                                                                                 \
    }                                                                                             \
    int best = 0;                                                                                 \
    for (int i = 1; i < 49; i++)                                                                  \
      if (out[best] < out[i]) best = i;                                                           \
    if (logits)                                                                                   \
      for (int i = 0; i < 49; i++) logits[i] = (double)out[i];                                    \
    return best;                                                                                  \
  }
ORC_DEEP_FORWARD(deep_forward_f32, float, expf)
ORC_DEEP_FORWARD(deep_forward_f64, double, exp)

int orc_nn_net_forward_pre(orc_ctx* ctx, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                           double* logits, double* pre) {
  if (!ctx->net.loaded) return FME_E_STATE;
  if (ctx->net.d.precision == FME_NN_F64)
    return deep_forward_f64(&ctx->net.d, ctx->net.pd, ctx->net.carry_d, e, c, pu_h, pu_w, logits, pre);
  return deep_forward_f32(&ctx->net.d, ctx->net.pf, ctx->net.carry_f, e, c, pu_h, pu_w, logits, pre);
}
int orc_nn_net_forward(orc_ctx* ctx, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                       double* logits) {
  return orc_nn_net_forward_pre(ctx, e, c, pu_h, pu_w, logits, NULL);
}

/* ---- context -------------------------------------------------------------------------- */
size_t orc_ctx_size(void) { return sizeof(orc_ctx); }

void orc_init(orc_ctx* ctx, const fme_config* cfg) {
  memset(ctx, 0, sizeof(*ctx));
  ctx->cfg = *cfg;
}
void orc_set_picture(orc_ctx* ctx, int id, const uint8_t* luma, int stride, int w, int h) {
  ctx->pics[id].luma = luma;
  ctx->pics[id].luma16 = NULL;
  ctx->pics[id].bd = 8;
  ctx->pics[id].stride = stride;
  ctx->pics[id].width = w;
  ctx->pics[id].height = h;
}
void orc_set_picture16(orc_ctx* ctx, int id, const uint16_t* luma, int stride, int w, int h) {
  ctx->pics[id].luma = NULL;
  ctx->pics[id].luma16 = luma;
  ctx->pics[id].bd = ctx->cfg.bit_depth;
  ctx->pics[id].stride = stride;
  ctx->pics[id].width = w;
  ctx->pics[id].height = h;
}
/* TComRdCost::setLambda + selectMotionLambda(true, 0, false), TComRdCost.cpp:104-110. */
void orc_set_lambda(orc_ctx* ctx, int id, double lambda) {
  const double sq = sqrt(lambda);
  ctx->mlambda[id] = 65536.0 * sq + 0;
}
void orc_set_motion_lambda(orc_ctx* ctx, int id, double ml) { ctx->mlambda[id] = ml; }
void orc_set_nn_inputs(orc_ctx* ctx, const uint32_t* rows, int n) {
  ctx->nn_in = rows;
  ctx->nn_in_n = rows ? n : 0;
}
void orc_set_keys(orc_ctx* ctx, const int16_t* keys, size_t n) {
  ctx->keys = keys;
  ctx->n_keys = n;
}
void orc_load_nn(orc_ctx* ctx, const float* params) {
  memcpy(ctx->nn, params, sizeof(ctx->nn));
  ctx->nn_loaded = 1;
}
void orc_nn_reset(orc_ctx* ctx) {
  memset(&ctx->nn_state, 0, sizeof(ctx->nn_state));
  memset(ctx->net.carry_d, 0, sizeof(ctx->net.carry_d));
  memset(ctx->net.carry_f, 0, sizeof(ctx->net.carry_f));
}
/* 12-word layout of fme_nn_get_state: slots[8], C, PUHeight, PUWidth, written mask. */
void orc_nn_get_state(const orc_ctx* ctx, uint32_t out[12]) {
  memcpy(out, ctx->nn_state.slot, 8 * sizeof(uint32_t));
  out[8] = ctx->nn_state.c;
  out[9] = ctx->nn_state.pu_h;
  out[10] = ctx->nn_state.pu_w;
  out[11] = ctx->nn_state.written;
}
void orc_nn_set_state(orc_ctx* ctx, const uint32_t in[12]) {
  memcpy(ctx->nn_state.slot, in, 8 * sizeof(uint32_t));
  ctx->nn_state.c = in[8];
  ctx->nn_state.pu_h = in[9];
  ctx->nn_state.pu_w = in[10];
  ctx->nn_state.written = in[11];
}

static int valid_size(int w, int h) {
  if (w < 4 || h < 4 || w > 64 || h > 64 || (w & 3) || (h & 3)) return 0;
  return 1;
}

/* xMotionEstimation sub-pel part for each job in order (TEncSearch.cpp:4529-4597). */
int orc_refine(orc_ctx* ctx, const fme_job* jobs, fme_result* res, int n) {
  if (ctx->cfg.nn_mode == 2 && !ctx->net.loaded) return FME_E_STATE;
  int16_t* key = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  for (int i = 0; i < n; i++) {
    const fme_job* j = &jobs[i];
    fme_result* r = &res[i];
    memset(r, 0, sizeof(*r));
    if (!valid_size(j->w, j->h) || j->org_id >= FME_MAX_PICTURES ||
        j->ref_id >= FME_MAX_PICTURES || j->lambda_id >= FME_MAX_LAMBDAS) {
      free(key);
      return FME_E_INVALID;
    }
    const orc_picture* ref = &ctx->pics[j->ref_id];
    const orc_picture* org = &ctx->pics[j->org_id];
    if (!ref->luma && !ref->luma16) { free(key); return FME_E_STATE; }
    const int w = j->w, h = j->h;
    if (j->key_offset >= 0) {
      if ((size_t)j->key_offset + (size_t)w * h > ctx->n_keys) { free(key); return FME_E_INVALID; }
      memcpy(key, ctx->keys + j->key_offset, sizeof(int16_t) * w * h);
    } else {
      if (!org->luma && !org->luma16) { free(key); return FME_E_STATE; }
      for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) key[y * w + x] = (int16_t)ref_px(org, j->x + x, j->y + y);
    }
    const double ml = ctx->mlambda[j->lambda_id];
    int mvx = j->mv_x, mvy = j->mv_y;
    uint32_t c = 0;
    int n_emi = 0;
    if (j->flags & FME_JOB_NN_IN) {
      /* the backups' input path: the row the integer search wrote (FME_TZ_RING), array_e's
       * slots after the per-call memset (Backups/4:4343-4359, 4421-4422) */
      if (!ctx->nn_in || i >= ctx->nn_in_n) { free(key); return FME_E_INVALID; }
      const uint32_t* row = ctx->nn_in + (size_t)9 * i;
      n_emi = 8;
      for (int s = 0; s < 8; s++) r->emi[s] = row[s];
      c = row[8];
      for (int s = 0; s < 8; s++) ctx->nn_state.slot[s] = r->emi[s];
      ctx->nn_state.c = c;
      ctx->nn_state.pu_h = (uint32_t)h;
      ctx->nn_state.pu_w = (uint32_t)w;
      ctx->nn_state.written |= 0x1FFu;
    } else if (j->flags & FME_JOB_EMI) {
      n_emi = orc_emi(ref, key, w, j->x, j->y, w, h, j->mv_x, j->mv_y, j->mvp_x, j->mvp_y,
                      j->lt_x, j->lt_y, j->rb_x, j->rb_y, ml, ctx->cfg.fast_inter_mode, r->emi,
                      &mvx, &mvy, &c);
      /* array_e: clear() then push_back -> slots 0..n-1 overwritten, the rest stale. */
      for (int s = 0; s < n_emi; s++) ctx->nn_state.slot[s] = r->emi[s];
      ctx->nn_state.c = c;
      ctx->nn_state.pu_h = (uint32_t)h;
      ctx->nn_state.pu_w = (uint32_t)w;
      ctx->nn_state.written |= ((1u << n_emi) - 1u) | 0x100u;
    }
    r->n_emi = (uint8_t)n_emi;
    r->c = c;
    r->mv_int_x = (int16_t)mvx;
    r->mv_int_y = (int16_t)mvy;
    const int lossless = (j->flags & FME_JOB_LOSSLESS) != 0;
    orc_frac_dif(ref, key, w, j->x, j->y, w, h, mvx, mvy, j->mvp_x, j->mvp_y, ml,
                 ctx->cfg.use_hadamard && !lossless, &r->half_x, &r->qtr_x, &r->frac_cost);
    int offx, offy;
    if (ctx->cfg.nn_mode) {
      const orc_nn_state* st = &ctx->nn_state;
      /* FME_NN_IN_SLOT_RESET: memset(array_e) on every NN_pred call (Backups/4:4421-4422,
       * Backups/15:4961-4962), so only this call's own pushes are non-zero. */
      uint32_t e[8];
      const int reset = ctx->cfg.nn_mode == 2 && (ctx->net.d.input_flags & FME_NN_IN_SLOT_RESET);
      for (int s = 0; s < 8; s++) e[s] = !reset ? st->slot[s] : (s < n_emi ? r->emi[s] : 0u);
      if (reset) {   /* the cleared array is the state the next call starts from */
        for (int s = 0; s < 8; s++) ctx->nn_state.slot[s] = e[s];
        ctx->nn_state.written |= 0xFFu;
      }
      int cls = ctx->cfg.nn_mode == 2
                    ? orc_nn_net_forward(ctx, e, st->c, (int)st->pu_h, (int)st->pu_w, NULL)
                    : orc_nn_forward(ctx->nn, st->slot, st->c, (int)st->pu_h, (int)st->pu_w, NULL);
      r->nn_class = (uint8_t)cls;
      if (n_emi < 8 || !(j->flags & (FME_JOB_EMI | FME_JOB_NN_IN))) r->status |= FME_RES_NN_STALE;
      if ((st->written & 0x1FFu) != 0x1FFu) r->status |= FME_RES_NN_UNINIT;
      /* class -> (MVX_HALF<<1)+MVX_QRTER, (MVY_HALF<<1)+MVY_QRTER: (cls%7-3, cls/7-3),
       * the switch of TEncSearch.cpp:136-193. */
      offx = cls % 7 - 3;
      offy = cls / 7 - 3;
    } else {
      r->nn_class = 255;
      offx = 2 * r->half_x + r->qtr_x;
      offy = 2 * r->half_y + r->qtr_y;
    }
    const int fmvx = 4 * mvx + offx, fmvy = 4 * mvy + offy;
    r->mv_x = (int16_t)fmvx;
    r->mv_y = (int16_t)fmvy;
    const uint32_t mvb = mv_bits(fmvx, fmvy, 0, j->mvp_x, j->mvp_y);
    const uint32_t bits = (uint32_t)j->bits_in + mvb;
    r->bits = bits;
    const double fw = (j->flags & FME_JOB_BIPRED) ? 0.5 : 1.0;
    const double v = floor(fw * ((double)r->frac_cost - (double)orc_cost(ml, mvb))) +
                     (double)orc_cost(ml, bits);
    /* (Distortion)(double): gcc/x86-64 converts through a signed 64-bit integer. */
    r->cost = (uint32_t)(int64_t)v;
  }
  free(key);
  return FME_OK;
}

/* =====================================================================================
 * Motion compensation of decided MVs: luma 8-tap + 4:2:0 chroma 4-tap.
 * ===================================================================================== */

/* m_chromaFilter, TComInterpolationFilter.cpp:65-75 (eighth-pel, 4 taps). */
static const int kChroma[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2},
                                  {-6, 46, 28, -4}, {-4, 36, 36, -4}, {-4, 28, 46, -6},
                                  {-2, 16, 54, -4}, {-2, 10, 58, -2}};

/* A block of `Pel` samples with its stride: the reference planes are staged into a padded
 * window (edge replication = TComPicYuv::extendPicBorder) so the filters below can walk raw
 * pointers the way TComInterpolationFilter does. */
typedef struct orc_win {
  int16_t* p;     /* sample (0,0) of the block */
  int stride;
} orc_win;

/* TComInterpolationFilter::filterCopy (TComInterpolationFilter.cpp:94-154), bit depth 8:
 * isFirst == isLast -> copy; isFirst -> (x << 6) - 8192; else ((x + 8192 + 32) >> 6) clipped. */
static void mc_copy(const int16_t* src, int ss, int16_t* dst, int ds, int w, int h, int first, int last) {
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int v = src[r * ss + c];
      if (first == last) {
      } else if (first) {
        v = (v << 6) - 8192;
      } else {
        v = clampi((v + 8192 + 32) >> 6, 0, 255);
      }
      dst[r * ds + c] = (int16_t)v;
    }
}

/* filter<N, isVertical, isFirst, isLast> (TComInterpolationFilter.cpp:172-257), bit depth 8:
 * headRoom 6; isLast: shift 6 (+6 when !isFirst), offset 1 << (shift-1) (+ 8192 << 6 when
 * !isFirst), clip; else shift 6 - 6 (isFirst) or 6, offset -8192 (isFirst) or 0. */
static void mc_filter(int ntaps, const int* coef, int vert, int first, int last, const int16_t* src, int ss,
                      int16_t* dst, int ds, int w, int h) {
  const int cstride = vert ? ss : 1;
  const int16_t* s0 = src - (ntaps / 2 - 1) * cstride;
  int shift = 6, offset;
  if (last) {
    shift += first ? 0 : 6;
    offset = 1 << (shift - 1);
    offset += first ? 0 : 8192 << 6;
  } else {
    shift -= first ? 6 : 0;
    offset = first ? -8192 * (1 << shift) : 0;   /* -8192 << shift (UB in C) */
  }
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int sum = 0;
      for (int k = 0; k < ntaps; k++) sum += s0[r * ss + c + k * cstride] * coef[k];
      int v = (sum + offset) >> shift;
      if (last) v = clampi(v, 0, 255);
      dst[r * ds + c] = (int16_t)v;
    }
}

/* TComDataCU::clipMv (TComDataCU.cpp:2773-2786), max CU 64. */
static void mc_clip_mv(int* mx, int* my, int pic_w, int pic_h, int cu_x, int cu_y) {
  const int hor_max = (pic_w + 8 - cu_x - 1) << 2, hor_min = (-64 - 8 - cu_x + 1) * 4;
  const int ver_max = (pic_h + 8 - cu_y - 1) << 2, ver_min = (-64 - 8 - cu_y + 1) * 4;
  *mx = *mx < hor_min ? hor_min : (*mx > hor_max ? hor_max : *mx);
  *my = *my < ver_min ? ver_min : (*my > ver_max ? ver_max : *my);
}

/* xPredInterBlk (TComPrediction.cpp:616-668) for one component: W x H at (x0,y0) of a plane
 * (pw x ph), MV in units of 1 << shift samples; bi keeps 14-bit output. */
static void mc_pred_blk(const uint8_t* plane, int stride, int pw, int ph, int chroma, int x0, int y0, int w, int h,
                        int mx, int my, int bi, int16_t* dst, int ds) {
  const int ntaps = chroma ? 4 : 8, sh = chroma ? 3 : 2;
  const int ix = mx >> sh, iy = my >> sh, fx = mx & ((1 << sh) - 1), fy = my & ((1 << sh) - 1);
  /* padded window: rows -ntaps/2+1 .. h+ntaps/2, cols likewise, around the displaced block */
  const int pad = ntaps / 2, ww = w + 2 * pad, wh = h + 2 * pad;
  int16_t* win = (int16_t*)malloc(sizeof(int16_t) * ww * wh);
  int16_t* tmp = (int16_t*)malloc(sizeof(int16_t) * w * (h + ntaps));
  for (int r = 0; r < wh; r++)
    for (int c = 0; c < ww; c++) {
      const int yy = clampi(y0 + iy + r - pad, 0, ph - 1), xx = clampi(x0 + ix + c - pad, 0, pw - 1);
      win[r * ww + c] = plane[(size_t)yy * stride + xx];
    }
  const int16_t* ref = win + pad * ww + pad;
  int ch[8], cv[8];
  for (int k = 0; k < ntaps; k++) {
    ch[k] = chroma ? kChroma[fx][k] : kLuma[fx][k];
    cv[k] = chroma ? kChroma[fy][k] : kLuma[fy][k];
  }
  if (fy == 0) {         /* filterHor(frac = fx, isLast = !bi); fx == 0 -> filterCopy */
    if (fx == 0) mc_copy(ref, ww, dst, ds, w, h, 1, !bi);
    else mc_filter(ntaps, ch, 0, 1, !bi, ref, ww, dst, ds, w, h);
  } else if (fx == 0) {  /* filterVer(frac = fy, isFirst = true, isLast = !bi) */
    mc_filter(ntaps, cv, 1, 1, !bi, ref, ww, dst, ds, w, h);
  } else {               /* filterHor over h + ntaps - 1 rows, then filterVer(isFirst = false) */
    mc_filter(ntaps, ch, 0, 1, 0, ref - (ntaps / 2 - 1) * ww, ww, tmp, w, w, h + ntaps - 1);
    mc_filter(ntaps, cv, 1, 0, !bi, tmp + (ntaps / 2 - 1) * w, w, dst, ds, w, h);
  }
  free(win);
  free(tmp);
}

/* Explicit weighted prediction (TComWeightPrediction.cpp), restated: getWpScaling (247-324) from
 * wp[list][picture][component] = {iWeight, iOffset (8-bit units), uiLog2WeightDenom}, then
 * weightBidir / weightUnidir / noWeightUnidir (46-66) as addWeightBi / addWeightUni pick them
 * (78-245) on the lists' 14-bit values, 8-bit output (shiftNum 6, IF_INTERNAL_OFFS 8192). */
static int wp_sample(const int (*wp)[FME_MAX_PICTURES][3][3], const fme_mc_job* j, const int* lists, int nl,
                     int comp, int p0, int p1) {
  const int shift_num = 6;   /* max(2, IF_INTERNAL_PREC - 8) */
  const int* a = wp[lists[0]][j->ref_id[lists[0]]][comp];
  if (nl == 2) {
    const int* b = wp[1][j->ref_id[1]][comp];
    const int offset = a[1] + b[1];                     /* o0 + o1, offsetScalingFactor 1 */
    const int shift = a[2] + 1 + shift_num, round = 1 << (shift - 1);
    return clampi((a[0] * (p0 + 8192) + b[0] * (p1 + 8192) + round + offset * (1 << (shift - 1))) >> shift, 0, 255);
  }
  if (a[0] != (1 << a[2])) {                            /* weightUnidir */
    const int shift = a[2] + shift_num, round = shift > 0 ? 1 << (shift - 1) : 0;
    return clampi(((a[0] * (p0 + 8192) + round) >> shift) + a[1], 0, 255);
  }
  /* noWeightUnidir / noWeightOffsetUnidir: shiftNum alone */
  return clampi((((p0 + 8192) + (1 << (shift_num - 1))) >> shift_num) + a[1], 0, 255);
}

static int mc_run_jobs(const orc_yuv* pics, const fme_mc_job* jobs, int n, uint8_t* y, int ys, uint8_t* cb,
                       uint8_t* cr, int cs, int width, int height, const int (*wp)[FME_MAX_PICTURES][3][3]) {
  for (int i = 0; i < n; i++) {
    const fme_mc_job* j = &jobs[i];
    const int wpf = wp && (j->flags & FME_MC_WP);
    if (j->w < 4 || j->h < 4 || j->w > 64 || j->h > 64 || (j->w & 3) || (j->h & 3)) return -1 - i;
    if (!(j->flags & 3u) || (j->flags & ~(wp ? 7u : 3u))) return -1 - i;
    if (j->x + j->w > width || j->y + j->h > height) return -1 - i;
    for (int l = 0; l < 2; l++)
      if ((j->flags & (1u << l)) &&
          (j->ref_id[l] >= FME_MAX_PICTURES || !pics[j->ref_id[l]].y || pics[j->ref_id[l]].width != width ||
           pics[j->ref_id[l]].height != height))
        return -1 - i;
    int lists[2], nl = 0;
    if (j->flags & FME_MC_L0) lists[nl++] = 0;
    if (j->flags & FME_MC_L1) lists[nl++] = 1;
    /* xCheckIdenticalMotion (TComPrediction.cpp:476-492; not with WPBiPred) */
    if (nl == 2 && !wpf && j->ref_id[0] == j->ref_id[1] && j->mv[0][0] == j->mv[1][0] && j->mv[0][1] == j->mv[1][1])
      nl = 1;
    for (int comp = 0; comp < 3; comp++) {
      const int c = comp ? 1 : 0;
      const int w = j->w >> c, h = j->h >> c, x0 = j->x >> c, y0 = j->y >> c;
      int16_t pred[2][64 * 64];
      for (int k = 0; k < nl; k++) {
        const orc_yuv* p = &pics[j->ref_id[lists[k]]];
        int mx = j->mv[lists[k]][0], my = j->mv[lists[k]][1];
        mc_clip_mv(&mx, &my, p->width, p->height, j->cu_x, j->cu_y);
        const uint8_t* plane = comp == 0 ? p->y : (comp == 1 ? p->cb : p->cr);
        mc_pred_blk(plane, comp ? p->c_stride : p->y_stride, p->width >> c, p->height >> c, c, x0, y0, w, h, mx, my,
                    nl == 2 || wpf, pred[k], w);
      }
      uint8_t* out = comp == 0 ? y : (comp == 1 ? cb : cr);
      const int os = comp ? cs : ys;
      for (int r = 0; r < h; r++)
        for (int q = 0; q < w; q++) {
          int v = pred[0][r * w + q];
          /* TComYuv::addAvg (TComYuv.cpp:354-415): shiftNum 7, offset 64 + 2 * 8192 */
          if (wpf) v = wp_sample(wp, j, lists, nl, comp, pred[0][r * w + q], nl == 2 ? pred[1][r * w + q] : 0);
          else if (nl == 2) v = clampi((pred[0][r * w + q] + pred[1][r * w + q] + 16448) >> 7, 0, 255);
          out[(size_t)(y0 + r) * os + x0 + q] = (uint8_t)v;
        }
    }
  }
  return 0;
}

int orc_mc(const orc_yuv* pics, const fme_mc_job* jobs, int n, uint8_t* y, int ys, uint8_t* cb, uint8_t* cr,
           int cs, int width, int height) {
  return mc_run_jobs(pics, jobs, n, y, ys, cb, cr, cs, width, height, NULL);
}

/* orc_mc with FME_MC_WP jobs weighted by wp9 = [2][FME_MAX_PICTURES][3 components][3] ints. */
int orc_mc_wp(const orc_yuv* pics, const fme_mc_job* jobs, int n, const int* wp9, uint8_t* y, int ys, uint8_t* cb,
              uint8_t* cr, int cs, int width, int height) {
  return mc_run_jobs(pics, jobs, n, y, ys, cb, cr, cs, width, height, (const int (*)[FME_MAX_PICTURES][3][3])wp9);
}

/* =====================================================================================
 * Integer motion estimation: xTZSearch with the shipped settings and
 * xPatternSearch for bi-pred jobs (TEncSearch.cpp:4627-5036, helpers 1078-1589).
 * ===================================================================================== */

/* TComMv::divideByPowerOf2(2) with ME_ENABLE_ROUNDING_OF_MVS (TComMv.h:122-130). */
static int mv_round4(int v) { return (v + 2) >> 2; }

/* TComDataCU::clipMv (TComDataCU.cpp:2773-2786), quarter-pel, max CU 64. */
static void tz_clip(int* x, int* y, int pw, int ph, int cu_x, int cu_y) {
  const int hmax = (pw + 8 - cu_x - 1) << 2, hmin = (-64 - 8 - cu_x + 1) * 4;
  const int vmax = (ph + 8 - cu_y - 1) << 2, vmin = (-64 - 8 - cu_y + 1) * 4;
  *x = *x < hmin ? hmin : (*x > hmax ? hmax : *x);
  *y = *y < vmin ? vmin : (*y > vmax ? vmax : *y);
}

/* IntTZSearchStruct (TEncSearch.h) and the state xTZSearchHelp reads. */
typedef struct tz_state {
  const orc_picture* ref;
  const int16_t* key;
  int x0, y0, w, h, fen, mvp_x, mvp_y;
  double ml;
  int16_t* cur;
  uint32_t best_sad;
  int best_x, best_y, best_dist, best_round, point_nr;
  /* the backups' array_e (FME_TZ_RING): pushes before index_ref feed C (their minimum), the first
   * eight after it are the NN inputs */
  int ring, after, npush;
  uint32_t cmin, e[8];
} tz_state;

/* Work counters of the integer searches (bench.py's k_tz roofline): points tested and the samples
 * their distortions read (FEN-subsampled rows counted once). */
static uint64_t g_tz_points, g_tz_samples;
void orc_tz_counters(uint64_t out[2], int reset) {
  out[0] = g_tz_points;
  out[1] = g_tz_samples;
  if (reset) g_tz_points = g_tz_samples = 0;
}
static void tz_count(int w, int h, int fen) {
  const int sub = (w == 12 || w == 24 || w == 48) && (fen == 1 || fen == 3) && h > 8;
  g_tz_points++;
  g_tz_samples += (uint64_t)w * (uint64_t)(sub ? h / 2 : h);
}

/* xTZSearchHelp normal branch (TEncSearch.cpp:1155-1188, save = false). */
static void tz_help(tz_state* s, int x, int y, int point_nr, int dist) {
  tz_count(s->w, s->h, s->fen);
  orc_pred_block(s->ref, s->x0, s->y0, s->w, s->h, 4 * x, 4 * y, s->cur);
  uint32_t d = int_dist(s->key, s->w, s->cur, s->w, s->w, s->h, s->fen, pic_bd(s->ref));
  if (s->ring) { /* array_e[counter_i] = uiSad (Backups/4:659) */
    if (!s->after) s->cmin = d < s->cmin ? d : s->cmin;
    else if (s->npush < 8) s->e[s->npush++] = d;
  }
  if (d < s->best_sad) {
    d += orc_cost(s->ml, mv_bits(x, y, 2, s->mvp_x, s->mvp_y));
    if (d < s->best_sad) {
      s->best_sad = d;
      s->best_x = x;
      s->best_y = y;
      s->best_dist = dist;
      s->best_round = 0;
      s->point_nr = point_nr;
    }
  }
}

typedef struct tz_range { int l, r, t, b; } tz_range;

/* xTZ8PointDiamondSearch (TEncSearch.cpp:1379-1589); corners: bCheckCornersAtDist1 (1402-1451). */
static void tz_diamond(tz_state* s, const tz_range* R, int sx, int sy, int dist, int corners) {
  const int top = sy - dist, bot = sy + dist, left = sx - dist, right = sx + dist;
  s->best_round += 1;
  if (dist == 1) {
    if (top >= R->t) {
      if (corners && left >= R->l) tz_help(s, left, top, 1, dist);
      tz_help(s, sx, top, 2, dist);
      if (corners && right <= R->r) tz_help(s, right, top, 3, dist);
    }
    if (left >= R->l) tz_help(s, left, sy, 4, dist);
    if (right <= R->r) tz_help(s, right, sy, 5, dist);
    if (bot <= R->b) {
      if (corners && left >= R->l) tz_help(s, left, bot, 6, dist);
      tz_help(s, sx, bot, 7, dist);
      if (corners && right <= R->r) tz_help(s, right, bot, 8, dist);
    }
  } else if (dist <= 8) {
    const int t2 = sy - (dist >> 1), b2 = sy + (dist >> 1), l2 = sx - (dist >> 1), r2 = sx + (dist >> 1);
    if (top >= R->t && left >= R->l && right <= R->r && bot <= R->b) {
      tz_help(s, sx, top, 2, dist);
      tz_help(s, l2, t2, 1, dist >> 1);
      tz_help(s, r2, t2, 3, dist >> 1);
      tz_help(s, left, sy, 4, dist);
      tz_help(s, right, sy, 5, dist);
      tz_help(s, l2, b2, 6, dist >> 1);
      tz_help(s, r2, b2, 8, dist >> 1);
      tz_help(s, sx, bot, 7, dist);
    } else {
      if (top >= R->t) tz_help(s, sx, top, 2, dist);
      if (t2 >= R->t) {
        if (l2 >= R->l) tz_help(s, l2, t2, 1, dist >> 1);
        if (r2 <= R->r) tz_help(s, r2, t2, 3, dist >> 1);
      }
      if (left >= R->l) tz_help(s, left, sy, 4, dist);
      if (right <= R->r) tz_help(s, right, sy, 5, dist);
      if (b2 <= R->b) {
        if (l2 >= R->l) tz_help(s, l2, b2, 6, dist >> 1);
        if (r2 <= R->r) tz_help(s, r2, b2, 8, dist >> 1);
      }
      if (bot <= R->b) tz_help(s, sx, bot, 7, dist);
    }
  } else {
    const int q = dist >> 2;
    if (top >= R->t && left >= R->l && right <= R->r && bot <= R->b) {
      tz_help(s, sx, top, 0, dist);
      tz_help(s, left, sy, 0, dist);
      tz_help(s, right, sy, 0, dist);
      tz_help(s, sx, bot, 0, dist);
      for (int k = 1; k < 4; k++) {
        const int yt = top + q * k, yb = bot - q * k, xl = sx - q * k, xr = sx + q * k;
        tz_help(s, xl, yt, 0, dist);
        tz_help(s, xr, yt, 0, dist);
        tz_help(s, xl, yb, 0, dist);
        tz_help(s, xr, yb, 0, dist);
      }
    } else {
      if (top >= R->t) tz_help(s, sx, top, 0, dist);
      if (left >= R->l) tz_help(s, left, sy, 0, dist);
      if (right <= R->r) tz_help(s, right, sy, 0, dist);
      if (bot <= R->b) tz_help(s, sx, bot, 0, dist);
      for (int k = 1; k < 4; k++) {
        const int yt = top + q * k, yb = bot - q * k, xl = sx - q * k, xr = sx + q * k;
        if (yt >= R->t) {
          if (xl >= R->l) tz_help(s, xl, yt, 0, dist);
          if (xr <= R->r) tz_help(s, xr, yt, 0, dist);
        }
        if (yb <= R->b) {
          if (xl >= R->l) tz_help(s, xl, yb, 0, dist);
          if (xr <= R->r) tz_help(s, xr, yb, 0, dist);
        }
      }
    }
  }
}

/* xTZ2PointSearch (TEncSearch.cpp:1191-1322): the 2 untested neighbours of a distance-1 best. */
static void tz_two_point(tz_state* s, const tz_range* R) {
  const int sx = s->best_x, sy = s->best_y;
  switch (s->point_nr) {
    case 1:
      if (sx - 1 >= R->l) tz_help(s, sx - 1, sy, 0, 2);
      if (sy - 1 >= R->t) tz_help(s, sx, sy - 1, 0, 2);
      break;
    case 2:
      if (sy - 1 >= R->t) {
        if (sx - 1 >= R->l) tz_help(s, sx - 1, sy - 1, 0, 2);
        if (sx + 1 <= R->r) tz_help(s, sx + 1, sy - 1, 0, 2);
      }
      break;
    case 3:
      if (sy - 1 >= R->t) tz_help(s, sx, sy - 1, 0, 2);
      if (sx + 1 <= R->r) tz_help(s, sx + 1, sy, 0, 2);
      break;
    case 4:
      if (sx - 1 >= R->l) {
        if (sy + 1 <= R->b) tz_help(s, sx - 1, sy + 1, 0, 2);
        if (sy - 1 >= R->t) tz_help(s, sx - 1, sy - 1, 0, 2);
      }
      break;
    case 5:
      if (sx + 1 <= R->r) {
        if (sy - 1 >= R->t) tz_help(s, sx + 1, sy - 1, 0, 2);
        if (sy + 1 <= R->b) tz_help(s, sx + 1, sy + 1, 0, 2);
      }
      break;
    case 6:
      if (sx - 1 >= R->l) tz_help(s, sx - 1, sy, 0, 2);
      if (sy + 1 <= R->b) tz_help(s, sx, sy + 1, 0, 2);
      break;
    case 7:
      if (sy + 1 <= R->b) {
        if (sx - 1 >= R->l) tz_help(s, sx - 1, sy + 1, 0, 2);
        if (sx + 1 <= R->r) tz_help(s, sx + 1, sy + 1, 0, 2);
      }
      break;
    case 8:
      if (sx + 1 <= R->r) tz_help(s, sx + 1, sy, 0, 2);
      if (sy + 1 <= R->b) tz_help(s, sx, sy + 1, 0, 2);
      break;
    default:   /* assert(false) in the reference: unreachable with distance-1 bests */
      break;
  }
}

/* xTZSearch (TEncSearch.cpp:4737-5036) up to the EMI square step; e->flags FME_TZ_ENHANCED:
 * bExtendedSettings = true (FastSearch 3, 4726-4727) with the neighbour predictors preds[3]
 * (m_acMvPredictors, TEncSearch.cpp:4708-4713, quarter-pel; NULL = zero). */
static void tz_search(tz_state* s, const fme_job* j, const fme_tz_ext* e, const int16_t (*preds)[2], int pw, int ph) {
  const int ext = (e->flags & FME_TZ_ENHANCED) && !(e->flags & FME_TZ_FULL) && !s->ring;
  const int range = e->search_range ? e->search_range : 64;
  int sx = j->mvp_x, sy = j->mvp_y;
  tz_clip(&sx, &sy, pw, ph, e->cu_x, e->cu_y);
  sx = mv_round4(sx);
  sy = mv_round4(sy);
  s->best_sad = 0xFFFFFFFFu;
  tz_help(s, sx, sy, 0, 0);
  if (ext) {   /* bTestOtherPredictedMV (4787-4805): "only test cMv if not obviously previously tested" */
    for (int k = 0; k < 3; k++) {
      int px = preds ? preds[k][0] : 0, py = preds ? preds[k][1] : 0;
      tz_clip(&px, &py, pw, ph, e->cu_x, e->cu_y);
      px = mv_round4(px);
      py = mv_round4(py);
      if ((px != sx || py != sy) && (px != s->best_x && py != s->best_y)) tz_help(s, px, py, 0, 0);
    }
  }
  if ((sx != 0 || sy != 0) && (s->best_x != 0 || s->best_y != 0)) tz_help(s, 0, 0, 0, 0);
  const tz_range R = {j->lt_x, j->rb_x, j->lt_y, j->rb_y};
  tz_range raster = R;
  if (e->flags & FME_TZ_PRED2NX2N) {
    int px = e->pred2n_x * 4, py = e->pred2n_y * 4;
    tz_clip(&px, &py, pw, ph, e->cu_x, e->cu_y);
    px = mv_round4(px);
    py = mv_round4(py);
    if ((sx != px || sy != py) && (px != s->best_x || py != s->best_y)) tz_help(s, px, py, 0, 0);
    /* xSetSearchRange(currBest << 2, m_iSearchRange) for the raster search (4602-4624) */
    int cx = s->best_x * 4, cy = s->best_y * 4;
    tz_clip(&cx, &cy, pw, ph, e->cu_x, e->cu_y);
    int lx = cx - (range << 2), ly = cy - (range << 2), rx = cx + (range << 2), ry = cy + (range << 2);
    tz_clip(&lx, &ly, pw, ph, e->cu_x, e->cu_y);
    tz_clip(&rx, &ry, pw, ph, e->cu_x, e->cu_y);
    raster.l = mv_round4(lx);
    raster.t = mv_round4(ly);
    raster.r = mv_round4(rx);
    raster.b = mv_round4(ry);
  }
  const int best_zero = s->best_x == 0 && s->best_y == 0;   /* bBestCandidateZero (4857) */
  const int startx = s->best_x, starty = s->best_y;
  for (int d = 1; d <= range; d *= 2) {   /* first search, stops 3 rounds after the best */
    tz_diamond(s, &R, startx, starty, d, ext);
    if (s->best_round >= 3) break;
  }
  if (ext && !best_zero) {   /* bNewZeroNeighbourhoodTest (4900-4917): half the range around zero */
    for (int d = 1; d <= (range >> 1); d *= 2) tz_diamond(s, &R, 0, 0, d, 0);
  }
  if (s->best_dist == 1) {
    s->best_dist = 0;
    tz_two_point(s, &R);
  }
  if (ext) {   /* bUseAdaptiveRaster (4926-4951): step 5, or 6 over the halved range when near */
    int win = 5;
    tz_range rr = raster;
    if (!(s->best_dist > 5)) {
      win = 6;
      rr.l /= 2; rr.r /= 2; rr.t /= 2; rr.b /= 2;   /* C++ division: towards zero */
    }
    s->best_dist = win;
    for (int y = rr.t; y <= rr.b; y += win)
      for (int x = rr.l; x <= rr.r; x += win) tz_help(s, x, y, 0, win);
  } else if (s->best_dist > 5) {   /* raster search, iRaster = 5 */
    s->best_dist = 5;
    for (int y = raster.t; y <= raster.b; y += 5)
      for (int x = raster.l; x <= raster.r; x += 5) tz_help(s, x, y, 0, 5);
  }
  while (s->best_dist > 0) {   /* star refinement (corners at distance 1 when extended) */
    const int bx = s->best_x, by = s->best_y;
    s->best_dist = 0;
    s->point_nr = 0;
    for (int d = 1; d < range + 1; d *= 2) tz_diamond(s, &R, bx, by, d, ext);
    if (s->best_dist == 1) {
      s->best_dist = 0;
      if (s->point_nr != 0) tz_two_point(s, &R);
    }
  }
  if (s->ring) {
    /* the backups' tail (Backups/4:4868-4878): index_ref = counter_i, then xTZ8PointSquareSearch at
     * distance 1 and xTZ8PointSquareSearch2 at distance 2, both around the star best */
    s->after = 1;
    const int sx = s->best_x, sy = s->best_y;
    int pts[8][2];
    const int np = square_points(sx, sy, R.l, R.t, R.r, R.b, pts);   /* TEncSearch.cpp:1324-1377 */
    for (int i = 0; i < np; i++) tz_help(s, pts[i][0], pts[i][1], 0, 1);
    /* xTZ8PointSquareSearch2 (Backups/4:876-965): the x -/+ 1 points of the top and bottom rows
     * are checked against the left / right bound of distance 2 */
    const int top = sy - 2, bot = sy + 2, left = sx - 2, right = sx + 2;
    const int okt = top >= R.t, okb = bot <= R.b, okl = left >= R.l, okr = right <= R.r;
    if (okt) {
      if (okl) tz_help(s, left, top, 9, 2);
      if (okl) tz_help(s, sx - 1, top, 10, 2);
      tz_help(s, sx, top, 11, 2);
      if (okr) tz_help(s, sx + 1, top, 12, 2);
      if (okr) tz_help(s, right, top, 13, 2);
    }
    if (okl) tz_help(s, left, sy - 1, 14, 2);
    if (okr) tz_help(s, right, sy - 1, 15, 2);
    if (okl) tz_help(s, left, sy, 16, 2);
    if (okr) tz_help(s, right, sy, 17, 2);
    if (okl) tz_help(s, left, sy + 1, 18, 2);
    if (okr) tz_help(s, right, sy + 1, 19, 2);
    if (okb) {
      if (okl) tz_help(s, left, bot, 20, 2);
      if (okl) tz_help(s, sx - 1, bot, 21, 2);
      tz_help(s, sx, bot, 22, 2);
      if (okr) tz_help(s, sx + 1, bot, 23, 2);
      if (okr) tz_help(s, right, bot, 24, 2);
    }
  }
}

/* ext records of `stride` bytes (fme_tz_ext, or fme_tz_ext2 with the predictors after it) */
static int tz_run_jobs(orc_ctx* ctx, fme_job* jobs, const void* ext0, size_t stride, uint32_t* sad, uint32_t* nn_in,
                       int n);

int orc_integer_search(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n) {
  return tz_run_jobs(ctx, jobs, ext, sizeof(fme_tz_ext), sad, NULL, n);
}

int orc_integer_search2(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext2* ext, uint32_t* sad, int n) {
  return tz_run_jobs(ctx, jobs, ext, sizeof(fme_tz_ext2), sad, NULL, n);
}

int orc_integer_search_ring(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, uint32_t* nn_in,
                            int n) {
  return tz_run_jobs(ctx, jobs, ext, sizeof(fme_tz_ext), sad, nn_in, n);
}

static int tz_run_jobs(orc_ctx* ctx, fme_job* jobs, const void* ext0, size_t stride, uint32_t* sad, uint32_t* nn_in,
                       int n) {
  int16_t* key = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  int16_t* cur = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  for (int i = 0; i < n; i++) {
    fme_job* j = &jobs[i];
    if (!valid_size(j->w, j->h) || j->ref_id >= FME_MAX_PICTURES || j->org_id >= FME_MAX_PICTURES ||
        j->lambda_id >= FME_MAX_LAMBDAS) {
      free(key); free(cur);
      return FME_E_INVALID;
    }
    const orc_picture* ref = &ctx->pics[j->ref_id];
    const orc_picture* org = &ctx->pics[j->org_id];
    if (!ref->luma && !ref->luma16) { free(key); free(cur); return FME_E_STATE; }
    const int w = j->w, h = j->h;
    if (j->key_offset >= 0) {
      if ((size_t)j->key_offset + (size_t)w * h > ctx->n_keys) { free(key); free(cur); return FME_E_INVALID; }
      memcpy(key, ctx->keys + j->key_offset, sizeof(int16_t) * w * h);
    } else {
      if (!org->luma && !org->luma16) { free(key); free(cur); return FME_E_STATE; }
      for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) key[y * w + x] = (int16_t)ref_px(org, j->x + x, j->y + y);
    }
    tz_state s;
    memset(&s, 0, sizeof(s));
    s.ref = ref; s.key = key; s.x0 = j->x; s.y0 = j->y; s.w = w; s.h = h;
    s.fen = ctx->cfg.fast_inter_mode; s.mvp_x = j->mvp_x; s.mvp_y = j->mvp_y;
    s.ml = ctx->mlambda[j->lambda_id]; s.cur = cur;
    const fme_tz_ext* e = (const fme_tz_ext*)((const char*)ext0 + stride * (size_t)i);
    const int16_t (*preds)[2] = stride >= sizeof(fme_tz_ext2) ? ((const fme_tz_ext2*)e)->preds : NULL;
    s.ring = nn_in != NULL && (e->flags & FME_TZ_RING) && !(j->flags & FME_JOB_BIPRED);
    s.cmin = 0xFFFFFFFFu;
    if ((j->flags & FME_JOB_BIPRED) || ((e->flags & FME_TZ_FULL) && !s.ring)) {
      /* xPatternSearch (TEncSearch.cpp:4627-4680): raster order, strict minimum (bi-pred jobs, and
       * every job at FastSearch 0, 4504-4507) */
      s.best_sad = 0xFFFFFFFFu;
      for (int y = j->lt_y; y <= j->rb_y; y++)
        for (int x = j->lt_x; x <= j->rb_x; x++) {
          tz_count(w, h, s.fen);
          orc_pred_block(ref, j->x, j->y, w, h, 4 * x, 4 * y, cur);
          const uint32_t d = int_dist(key, w, cur, w, w, h, s.fen, pic_bd(ref)) + orc_cost(s.ml, mv_bits(x, y, 2, s.mvp_x, s.mvp_y));
          if (d < s.best_sad) { s.best_sad = d; s.best_x = x; s.best_y = y; }
        }
    } else {
      tz_search(&s, j, e, preds, ref->width, ref->height);
    }
    j->mv_x = (int16_t)s.best_x;
    j->mv_y = (int16_t)s.best_y;
    if (sad) sad[i] = s.best_sad - orc_cost(s.ml, mv_bits(s.best_x, s.best_y, 2, s.mvp_x, s.mvp_y));
    if (s.ring) { /* U1 V1 U2 H1 H2 U3 V2 U4, C (Backups/4:4343-4359); unpushed slots read 0 */
      for (int k = 0; k < 8; k++) nn_in[(size_t)9 * i + k] = k < s.npush ? s.e[k] : 0u;
      nn_in[(size_t)9 * i + 8] = s.cmin;
    }
  }
  free(key);
  free(cur);
  return FME_OK;
}

/* =====================================================================================
 * predInterSearch's P-slice PU / reference loop, sequential.
 * ===================================================================================== */

/* xGetMvpIdxBits (TEncSearch.cpp:4258-4284) = m_auiMVPIdxCost[idx][num] (412-425). */
static uint32_t pi_mvp_idx_bits(int idx, int num) {
  if (num == 1) return 0;
  uint32_t len = 1;
  if (idx == 0) return len;
  len += (uint32_t)(idx - 1);
  if (num - 1 > idx) len++;
  return len;
}

/* xGetBlkBits (TEncSearch.cpp:4286-4333) for a P slice: uiBlkBit[0]. */
static uint32_t pi_blk_bits(int part_size) {
  if (part_size == FME_PART_2Nx2N || part_size == FME_PART_NxN) return 1;
  return 3;   /* 2NxN, 2NxnU, 2NxnD, Nx2N, nLx2N, nRx2N */
}

/* xGetTemplateCost (TEncSearch.cpp:4397-4436): clipMv, xPredInterBlk(COMPONENT_Y, bi = false),
 * getDistPart(DF_SAD) (plain SAD, TComRdCost.cpp:187-197, 327-349), calcRdCost(bits, SAD, DF_SAD)
 * (TComRdCost.cpp:57-102, COST_STANDARD_LOSSY: SAD + bits * lambdaMotionSAD / 65536). */
typedef struct pi_pu {   /* the geometry and slots every xMotionEstimation of one PU shares */
  int x, y, w, h, cu_x, cu_y, org_id, lambda_id, lossless;
} pi_pu;

/* motionCompensation's luma part for one list (xPredInterUni, bi = false); above 8 bits the
 * generic quarter-pel predictor at the picture's bit depth (orc_pred_block). */
static void pi_pred_uni(const orc_ctx* ctx, const pi_pu* g, int ref_id, int mx, int my, int16_t* pred) {
  const orc_picture* ref = &ctx->pics[ref_id];
  mc_clip_mv(&mx, &my, ref->width, ref->height, g->cu_x, g->cu_y);
  if (pic_bd(ref) > 8) {
    orc_pred_block(ref, g->x, g->y, g->w, g->h, mx, my, pred);
    return;
  }
  mc_pred_blk(ref->luma, ref->stride, ref->width, ref->height, 0, g->x, g->y, g->w, g->h, mx, my, 0, pred, g->w);
}

static uint32_t pi_tmpl(const orc_ctx* ctx, const pi_pu* g, int ref_id, int mx, int my, int m, int16_t* pred) {
  const orc_picture* org = &ctx->pics[g->org_id];
  pi_pred_uni(ctx, g, ref_id, mx, my, pred);
  uint32_t sad = 0;
  for (int y = 0; y < g->h; y++)
    for (int x = 0; x < g->w; x++) {
      const int d = pred[y * g->w + x] - ref_px(org, g->x + x, g->y + y);
      sad += (uint32_t)(d < 0 ? -d : d);
    }
  sad >>= pic_bd(org) - 8;   /* xGetSAD*: uiSum >> DISTORTION_PRECISION_ADJUSTMENT(bitDepth - 8) */
  const double ml = ctx->mlambda[g->lambda_id];
  return (uint32_t)((double)sad + ((double)pi_mvp_idx_bits(m, 2) * ml) / 65536.0);
}

static pi_pu pi_pu_of(const fme_pu_req* q) {
  pi_pu g = {q->x, q->y, q->w, q->h, q->cu_x, q->cu_y, q->org_id, q->lambda_id, (q->flags & FME_PU_LOSSLESS) != 0};
  return g;
}

/* xGetTemplateCost of AMVP candidate m of reference k of one request (exported for the tests). */
uint32_t orc_template_cost(const orc_ctx* ctx, const fme_pu_req* q, int k, int m) {
  int16_t pred[64 * 64];
  const pi_pu g = pi_pu_of(q);
  return pi_tmpl(ctx, &g, q->ref_id[k], q->cand[k][m][0], q->cand[k][m][1], m, pred);
}

/* xEstimateMvPredAMVP (4186-4256): with two candidates the first with the least template cost.
 * dist_bip (may be null): *puiDistBiP, the chosen candidate's template cost; with one candidate it
 * is computed only when one_cand_dist is set (MvdL1ZeroFlag and list 1, 4214-4217). */
static int pi_amvp2(const orc_ctx* ctx, const pi_pu* g, int ref_id, int n_cand, const int16_t cand[2][2],
                    int16_t* pred, uint32_t* dist_bip, int one_cand_dist) {
  int idx = 0;
  if (n_cand > 1) {
    uint32_t best = 0xFFFFFFFFu;
    for (int m = 0; m < n_cand; m++) {
      const uint32_t c = pi_tmpl(ctx, g, ref_id, cand[m][0], cand[m][1], m, pred);
      if (best > c) {
        best = c;
        idx = m;
        if (dist_bip) *dist_bip = c;
      }
    }
  } else if (one_cand_dist && dist_bip) {
    *dist_bip = pi_tmpl(ctx, g, ref_id, cand[0][0], cand[0][1], 0, pred);
  }
  return idx;
}
static int pi_amvp(const orc_ctx* ctx, const pi_pu* g, int ref_id, int n_cand, const int16_t cand[2][2],
                   int16_t* pred) {
  return pi_amvp2(ctx, g, ref_id, n_cand, cand, pred, NULL, 0);
}

/* The reference-index bits of uiBitsTemp (3792-3800). */
static uint32_t pi_ref_bits(int k, int num_refs) {
  if (num_refs <= 1) return 0;
  return (uint32_t)k + 1u - (k == num_refs - 1 ? 1u : 0u);
}

/* xMotionEstimation (4439-4599) on one (PU, reference): xSetSearchRange around the predictor (uni)
 * or around the start MV bc (bi), the integer search (xTZSearch with the EMI step and the
 * m_integerMv2Nx2N start pred2n, or xPatternSearch on the bi key), FracDIF, NN_pred, the tail. */
static int pi_me(orc_ctx* ctx, const pi_pu* g, int ref_id, int mvp_x, int mvp_y, uint32_t bits, int range,
                 const int16_t* pred2n, const int16_t* bikey, int bc_x, int bc_y, fme_result* r) {
  const orc_picture* org = &ctx->pics[g->org_id];
  fme_job j;
  memset(&j, 0, sizeof(j));
  j.x = (uint16_t)g->x; j.y = (uint16_t)g->y; j.w = (uint8_t)g->w; j.h = (uint8_t)g->h;
  j.org_id = (uint8_t)g->org_id; j.ref_id = (uint8_t)ref_id;
  j.mvp_x = (int16_t)mvp_x; j.mvp_y = (int16_t)mvp_y;
  int cx = bikey ? bc_x : mvp_x, cy = bikey ? bc_y : mvp_y;
  tz_clip(&cx, &cy, org->width, org->height, g->cu_x, g->cu_y);
  int lx = cx - (range << 2), ly = cy - (range << 2), rx = cx + (range << 2), ry = cy + (range << 2);
  tz_clip(&lx, &ly, org->width, org->height, g->cu_x, g->cu_y);
  tz_clip(&rx, &ry, org->width, org->height, g->cu_x, g->cu_y);
  j.lt_x = (int16_t)mv_round4(lx); j.lt_y = (int16_t)mv_round4(ly);
  j.rb_x = (int16_t)mv_round4(rx); j.rb_y = (int16_t)mv_round4(ry);
  j.flags = (uint8_t)((bikey ? FME_JOB_BIPRED : FME_JOB_EMI) | (g->lossless ? FME_JOB_LOSSLESS : 0u));
  j.lambda_id = (uint8_t)g->lambda_id;
  j.bits_in = (uint16_t)bits;
  j.key_offset = bikey ? 0 : -1;
  fme_tz_ext e;
  memset(&e, 0, sizeof(e));
  e.cu_x = (uint16_t)g->cu_x; e.cu_y = (uint16_t)g->cu_y;
  e.search_range = (uint8_t)range;
  if (pred2n) {   /* pIntegerMv2Nx2NPred (4511-4515) */
    e.flags = FME_TZ_PRED2NX2N;
    e.pred2n_x = pred2n[0];
    e.pred2n_y = pred2n[1];
  }
  const int16_t* keys = ctx->keys;
  const size_t n_keys = ctx->n_keys;
  if (bikey) {   /* m_cYuvPredTemp as this job's key block */
    ctx->keys = bikey;
    ctx->n_keys = (size_t)g->w * g->h;
  }
  int rc = orc_integer_search(ctx, &j, &e, NULL, 1);
  if (!rc) rc = orc_refine(ctx, &j, r, 1);
  ctx->keys = keys;
  ctx->n_keys = n_keys;
  return rc;
}

/* xCheckBestMVP (4344-4394), cost scale 0: move to a candidate with strictly fewer MV bits. */
static void pi_check_best_mvp(double ml, const int16_t cand[2][2], int n_cand, int mx, int my, int* idx,
                              uint32_t* bits, uint32_t* cost) {
  if (n_cand < 2) return;
  const int org_bits = (int)(mv_bits(mx, my, 0, cand[*idx][0], cand[*idx][1]) + pi_mvp_idx_bits(*idx, 2));
  int best_bits = org_bits, best_idx = *idx;
  for (int m = 0; m < n_cand; m++) {
    if (m == *idx) continue;
    const int b = (int)(mv_bits(mx, my, 0, cand[m][0], cand[m][1]) + pi_mvp_idx_bits(m, 2));
    if (b < best_bits) {
      best_bits = b;
      best_idx = m;
    }
  }
  if (best_idx != *idx) {
    *idx = best_idx;
    const uint32_t org_total = *bits;
    *bits = org_total - (uint32_t)org_bits + (uint32_t)best_bits;
    *cost = (*cost - orc_cost(ml, org_total)) + orc_cost(ml, *bits);
  }
}

void orc_pred_inter_reset(orc_ctx* ctx) { memset(ctx->int_mv_2n, 0, sizeof(ctx->int_mv_2n)); }

int orc_pred_inter_p(orc_ctx* ctx, const fme_pu_req* reqs, fme_pu_res* res, int n) {
  int16_t* pred = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  for (int i = 0; i < n; i++) {
    const fme_pu_req* q = &reqs[i];
    fme_pu_res* o = &res[i];
    memset(o, 0, sizeof(*o));
    if (q->num_refs < 1 || q->num_refs > FME_MAX_REFS || q->org_id >= FME_MAX_PICTURES ||
        !pic_set(&ctx->pics[q->org_id]) || q->lambda_id >= FME_MAX_LAMBDAS) {
      free(pred);
      return FME_E_INVALID;
    }
    const double ml = ctx->mlambda[q->lambda_id];
    const int range = q->search_range ? q->search_range : 64;
    uint32_t best_cost = 0xFFFFFFFFu;   /* uiCost[0] = max */
    for (int k = 0; k < q->num_refs; k++) {
      if (q->ref_id[k] >= FME_MAX_PICTURES || !pic_set(&ctx->pics[q->ref_id[k]]) || q->n_cand[k] < 1 || q->n_cand[k] > 2) {
        free(pred);
        return FME_E_INVALID;
      }
      /* uiBitsTemp = uiMbBits[0] + reference-index bits (3792-3800) */
      uint32_t bits = pi_blk_bits(q->part_size) + pi_ref_bits(k, q->num_refs);
      const pi_pu g = pi_pu_of(q);
      int idx = pi_amvp(ctx, &g, q->ref_id[k], q->n_cand[k], q->cand[k], pred);
      bits += pi_mvp_idx_bits(idx, 2);   /* m_auiMVPIdxCost[idx][AMVP_MAX_NUM_CANDS] (3812) */
      /* xMotionEstimation (4439-4599): xSetSearchRange, xTZSearch (+ EMI), FracDIF, NN, tail */
      const int reads2n = !(q->part_size == FME_PART_2Nx2N && q->depth == 0);
      fme_result r;
      const int rc = pi_me(ctx, &g, q->ref_id[k], q->cand[k][idx][0], q->cand[k][idx][1], bits, range,
                           reads2n ? ctx->int_mv_2n[0][k] : NULL, NULL, 0, 0, &r);
      if (rc) {
        free(pred);
        return rc;
      }
      if (q->part_size == FME_PART_2Nx2N) {   /* m_integerMv2Nx2N = rcMv after the TZ search (4523-4526) */
        ctx->int_mv_2n[0][k][0] = r.mv_int_x;
        ctx->int_mv_2n[0][k][1] = r.mv_int_y;
      }
      uint32_t rbits = r.bits, rcost = r.cost;
      pi_check_best_mvp(ml, q->cand[k], q->n_cand[k], r.mv_x, r.mv_y, &idx, &rbits, &rcost);
      o->ref_cost[k] = rcost;
      o->ref_bits[k] = rbits;
      o->ref_mv[k][0] = r.mv_x;
      o->ref_mv[k][1] = r.mv_y;
      o->ref_mvp_idx[k] = (uint8_t)idx;
      if (rcost < best_cost) {   /* 3845-3853 */
        best_cost = rcost;
        o->cost = rcost;
        o->bits = rbits;
        o->mv_x = r.mv_x;
        o->mv_y = r.mv_y;
        o->ref_idx = (uint8_t)k;
        o->mvp_idx = (uint8_t)idx;
        o->mvp_x = q->cand[k][idx][0];
        o->mvp_y = q->cand[k][idx][1];
      }
    }
  }
  free(pred);
  return FME_OK;
}

/* =====================================================================================
 * predInterSearch for B slices, sequential: TEncSearch.cpp:3746-4105 —
 * FEN 1/2 (one bi-pred iteration over the list opposite the cheaper uni list), FEN 0/3 (up to four
 * alternating iterations, each on the key of the other list's current best), and MvdL1ZeroFlag
 * (FME_PU_MVD_L1_ZERO, lowdelay B: list 1 fixed at its best AMVP predictor, one L0 iteration).
 * ===================================================================================== */

/* xGetBlkBits (TEncSearch.cpp:4286-4333) for a B slice: uiBlkBit[0..2]. */
static void pi_blk_bits_b(int part_size, int part_idx, int last_mode, uint32_t out[3]) {
  static const uint32_t hor[2][3][3] = {{{0, 0, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {7, 5, 7}, {6, 6, 6}}};
  static const uint32_t ver[2][3][3] = {{{0, 2, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {5, 5, 7}, {6, 6, 6}}};
  if (part_size == FME_PART_2Nx2N || part_size == FME_PART_NxN) {
    out[0] = 3; out[1] = 3; out[2] = 5;
  } else {
    const int hz = part_size == FME_PART_2NxN || part_size == FME_PART_2NxnU || part_size == FME_PART_2NxnD;
    const uint32_t* t = hz ? hor[part_idx][last_mode] : ver[part_idx][last_mode];
    out[0] = t[0]; out[1] = t[1]; out[2] = t[2];
  }
}

/* xMotionEstimation(bBi)'s key (TEncSearch.cpp:4461-4471): the other list's uni-pred luma
 * prediction (motionCompensation) at (mvx, mvy), key = 2 * org - pred (removeHighFreq, TComYuv.cpp
 * :411-455), clipped to the bit depth with ClipForBiPredMe.  key: w*h. */
void orc_bi_key(const orc_ctx* ctx, int org_id, int ref_id, int x, int y, int w, int h, int cu_x, int cu_y,
                int mvx, int mvy, int clip, int16_t* key) {
  int16_t pred[64 * 64];
  const pi_pu g = {x, y, w, h, cu_x, cu_y, org_id, 0, 0};
  pi_pred_uni(ctx, &g, ref_id, mvx, mvy, pred);
  const orc_picture* org = &ctx->pics[org_id];
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int v = 2 * ref_px(org, x + c, y + r) - pred[r * w + c];
      if (clip) v = clampi(v, 0, (1 << pic_bd(org)) - 1);   /* ClipBD */
      key[r * w + c] = (int16_t)v;
    }
}

/* TComDataCU::getNumPartitions for the part_idx check. */
static int pi_num_parts(int part_size) {
  return part_size == FME_PART_2Nx2N ? 1 : (part_size == FME_PART_NxN ? 4 : 2);
}

int orc_pred_inter_b(orc_ctx* ctx, const fme_pu_req_b* reqs, fme_pu_res_b* res, int n) {
  const int fen = ctx->cfg.fast_inter_mode;
  if (fen < 0 || fen > 3) return FME_E_INVALID;
  int16_t* pred = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  int16_t* key = (int16_t*)malloc(sizeof(int16_t) * 64 * 64);
  int last_mode = 0;   /* uiLastMode: 0 L0, 1 L1, 2 bi (predInterSearch local, per CU) */
  int rc = FME_OK;
  for (int i = 0; i < n && !rc; i++) {
    const fme_pu_req_b* q = &reqs[i];
    fme_pu_res_b* o = &res[i];
    memset(o, 0, sizeof(*o));
    if (q->org_id >= FME_MAX_PICTURES || !pic_set(&ctx->pics[q->org_id]) || q->lambda_id >= FME_MAX_LAMBDAS ||
        q->part_size > FME_PART_nRx2N || q->part_idx >= pi_num_parts(q->part_size) ||
        (q->flags & ~(FME_PU_LOSSLESS | FME_PU_FAST_ME_GEN_B | FME_PU_CLIP_BIPRED | FME_PU_MVD_L1_ZERO))) {
      rc = FME_E_INVALID;
      break;
    }
    for (int l = 0; l < 2 && !rc; l++) {
      if (q->num_refs[l] < 1 || q->num_refs[l] > FME_MAX_REFS) rc = FME_E_INVALID;
      for (int k = 0; k < q->num_refs[l] && !rc; k++)
        if (q->ref_id[l][k] >= FME_MAX_PICTURES || !pic_set(&ctx->pics[q->ref_id[l][k]]) || q->n_cand[l][k] < 1 ||
            q->n_cand[l][k] > 2 || (l == 1 && q->l1_to_l0[k] >= q->num_refs[0]))
          rc = FME_E_INVALID;
    }
    if (!rc && q->part_size != FME_PART_2Nx2N && q->part_size != FME_PART_NxN && q->part_idx == 1 &&
        (i == 0 || reqs[i - 1].part_idx != 0 || reqs[i - 1].part_size != q->part_size ||
         reqs[i - 1].cu_x != q->cu_x || reqs[i - 1].cu_y != q->cu_y))
      rc = FME_E_INVALID;   /* uiLastMode comes from the CU's first PU, the request before */
    if (rc) break;
    if (q->part_idx == 0) last_mode = 0;
    const pi_pu g = {q->x, q->y, q->w, q->h, q->cu_x, q->cu_y, q->org_id, q->lambda_id, (q->flags & FME_PU_LOSSLESS) != 0};
    const double ml = ctx->mlambda[q->lambda_id];
    const int range = q->search_range ? q->search_range : 64;
    const int brange = q->bipred_range ? q->bipred_range : 4;
    uint32_t mb[3];
    pi_blk_bits_b(q->part_size, q->part_idx, last_mode, mb);
    uint32_t cost[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, bits[2] = {0, 0};
    int16_t mv[2][2] = {{0, 0}, {0, 0}};
    int ridx[2] = {0, 0};
    uint32_t cost_l0[FME_MAX_REFS], bits_l0[FME_MAX_REFS];
    int16_t mvt[2][FME_MAX_REFS][2];
    int mvpi[2][FME_MAX_REFS];
    uint32_t cost_v1 = 0xFFFFFFFFu, bits_v1 = 0xFFFFFFFFu;   /* costValidList1 / bitsValidList1 */
    int16_t mv_v1[2] = {0, 0};
    int ridx_v1 = 0;
    const int reads2n = !(q->part_size == FME_PART_2Nx2N && q->depth == 0);
    const int mvdl1z = (q->flags & FME_PU_MVD_L1_ZERO) != 0;
    uint32_t best_bip_dist = 0xFFFFFFFFu, bip_dist = 0xFFFFFFFFu;   /* bestBiPDist, biPDistTemp */
    int best_bip_mvp = 0, best_bip_ref = 0;                          /* bestBiPMvpL1, bestBiPRefIdxL1 */
    /* uni-directional prediction (3786-3865) */
    for (int l = 0; l < 2 && !rc; l++)
      for (int k = 0; k < q->num_refs[l] && !rc; k++) {
        uint32_t b = mb[l] + pi_ref_bits(k, q->num_refs[l]);
        int idx = pi_amvp2(ctx, &g, q->ref_id[l][k], q->n_cand[l][k], q->cand[l][k], pred, &bip_dist,
                           mvdl1z && l == 1);
        if (mvdl1z && l == 1 && bip_dist < best_bip_dist) {   /* 3805-3810 */
          best_bip_dist = bip_dist;
          best_bip_mvp = idx;
          best_bip_ref = k;
        }
        b += pi_mvp_idx_bits(idx, 2);
        uint32_t c;
        if ((q->flags & FME_PU_FAST_ME_GEN_B) && l == 1 && q->l1_to_l0[k] >= 0) {
          /* 3814-3827: L0's result, its bit-rate part re-priced with L1's predictor */
          const int k0 = q->l1_to_l0[k];
          mvt[1][k][0] = mvt[0][k0][0];
          mvt[1][k][1] = mvt[0][k0][1];
          c = cost_l0[k0] - orc_cost(ml, bits_l0[k0]);
          b += mv_bits(mvt[1][k][0], mvt[1][k][1], 0, q->cand[1][k][idx][0], q->cand[1][k][idx][1]);
          c += orc_cost(ml, b);
        } else {
          fme_result r;
          rc = pi_me(ctx, &g, q->ref_id[l][k], q->cand[l][k][idx][0], q->cand[l][k][idx][1], b, range,
                     reads2n ? ctx->int_mv_2n[l][k] : NULL, NULL, 0, 0, &r);
          if (rc) break;
          if (q->part_size == FME_PART_2Nx2N) {
            ctx->int_mv_2n[l][k][0] = r.mv_int_x;
            ctx->int_mv_2n[l][k][1] = r.mv_int_y;
          }
          mvt[l][k][0] = r.mv_x;
          mvt[l][k][1] = r.mv_y;
          b = r.bits;
          c = r.cost;
        }
        pi_check_best_mvp(ml, q->cand[l][k], q->n_cand[l][k], mvt[l][k][0], mvt[l][k][1], &idx, &b, &c);
        mvpi[l][k] = idx;
        o->ref_cost[l][k] = c;
        o->ref_mv[l][k][0] = mvt[l][k][0];
        o->ref_mv[l][k][1] = mvt[l][k][1];
        o->ref_mvp_idx[l][k] = (uint8_t)idx;
        if (l == 0) {
          cost_l0[k] = c;
          bits_l0[k] = b;
        }
        if (c < cost[l]) {
          cost[l] = c;
          bits[l] = b;
          mv[l][0] = mvt[l][k][0];
          mv[l][1] = mvt[l][k][1];
          ridx[l] = k;
        }
        if (l == 1 && c < cost_v1 && q->l1_to_l0[k] < 0) {
          cost_v1 = c;
          bits_v1 = b;
          mv_v1[0] = mvt[1][k][0];
          mv_v1[1] = mvt[1][k][1];
          ridx_v1 = k;
        }
      }
    if (rc) break;
    /* bi-predictive motion estimation (3868-4022) */
    uint32_t cost_bi = 0xFFFFFFFFu, bits_bi = 0;
    int16_t mv_bi[2][2] = {{mv[0][0], mv[0][1]}, {mv[1][0], mv[1][1]}};
    int ridx_bi[2] = {ridx[0], ridx[1]};
    int mvpi_bi[2][FME_MAX_REFS];
    memcpy(mvpi_bi, mvpi, sizeof(mvpi));
    o->bi_list = 0xFF;
    o->bi_cost = 0xFFFFFFFFu;
    o->bi_iters = 0;
    const int restricted = q->cu_w == 8 && (q->w < 8 || q->h < 8);   /* isBipredRestriction */
    if (!restricted) {
      uint32_t mot[2];
      /* m_acYuvPred[l]: the (reference, MV) each list's stored prediction was made with */
      int ps_ref[2] = {ridx[0], ridx[1]};
      int16_t ps_mv[2][2] = {{mv[0][0], mv[0][1]}, {mv[1][0], mv[1][1]}};
      if (mvdl1z) {   /* 3876-3909: list 1 at its best template-cost AMVP predictor, MVD zero */
        const int kb = best_bip_ref;
        mvpi_bi[1][kb] = best_bip_mvp;
        mv_bi[1][0] = q->cand[1][kb][best_bip_mvp][0];
        mv_bi[1][1] = q->cand[1][kb][best_bip_mvp][1];
        ridx_bi[1] = kb;
        ps_ref[1] = kb;
        ps_mv[1][0] = mv_bi[1][0];
        ps_mv[1][1] = mv_bi[1][1];
        mot[0] = bits[0] - mb[0];
        mot[1] = mb[1] + pi_ref_bits(kb, q->num_refs[1]) + pi_mvp_idx_bits(mvpi_bi[1][kb], 2);
        bits_bi = mb[2] + mot[0] + mot[1];
        mvt[1][kb][0] = mv_bi[1][0];
        mvt[1][kb][1] = mv_bi[1][1];
      } else {
        mot[0] = bits[0] - mb[0];
        mot[1] = bits[1] - mb[1];
        bits_bi = mb[2] + mot[0] + mot[1];
      }
      /* 4 iterations; FASTINTERSEARCH_MODE1/2 or MvdL1ZeroFlag: one (3919-3925) */
      const int niter = (fen == 1 || fen == 2 || mvdl1z) ? 1 : 4;
      for (int it = 0; it < niter && !rc; it++) {
        int L = it % 2;
        if (fen == 1 || fen == 2) L = cost[0] <= cost[1] ? 1 : 0;   /* 3931-3941 */
        else if (it == 0) L = 0;
        if (it == 0 && !mvdl1z) {   /* motionCompensation of the other list at its uni best (3946-3952) */
          ps_ref[1 - L] = ridx[1 - L];
          ps_mv[1 - L][0] = mv[1 - L][0];
          ps_mv[1 - L][1] = mv[1 - L][1];
        }
        if (mvdl1z) L = 0;   /* 3956-3960 */
        /* xMotionEstimation(bBi)'s key: removeHighFreq of the other list's stored prediction */
        orc_bi_key(ctx, q->org_id, q->ref_id[1 - L][ps_ref[1 - L]], q->x, q->y, q->w, q->h, q->cu_x, q->cu_y,
                   ps_mv[1 - L][0], ps_mv[1 - L][1], (q->flags & FME_PU_CLIP_BIPRED) != 0, key);
        o->bi_list = (uint8_t)L;
        o->bi_iters = (uint8_t)(it + 1);
        memset(o->bi_ref_cost, 0, sizeof(o->bi_ref_cost));
        memset(o->bi_ref_mv, 0, sizeof(o->bi_ref_mv));
        int changed = 0;
        for (int k = 0; k < q->num_refs[L]; k++) {
          uint32_t b = mb[2] + mot[1 - L] + pi_ref_bits(k, q->num_refs[L]) + pi_mvp_idx_bits(mvpi_bi[L][k], 2);
          const int16_t* p = q->cand[L][k][mvpi_bi[L][k]];
          fme_result r;
          /* ±BipredSearchRange around cMvTemp[L][k], the last ME result of (L, k) (4486-4490) */
          rc = pi_me(ctx, &g, q->ref_id[L][k], p[0], p[1], b, brange, NULL, key, mvt[L][k][0], mvt[L][k][1], &r);
          if (rc) break;
          mvt[L][k][0] = r.mv_x;
          mvt[L][k][1] = r.mv_y;
          uint32_t c = r.cost;
          b = r.bits;
          int idx = mvpi_bi[L][k];
          pi_check_best_mvp(ml, q->cand[L][k], q->n_cand[L][k], r.mv_x, r.mv_y, &idx, &b, &c);
          mvpi_bi[L][k] = idx;
          o->bi_ref_cost[k] = c;
          o->bi_ref_mv[k][0] = r.mv_x;
          o->bi_ref_mv[k][1] = r.mv_y;
          if (c < cost_bi) {   /* 3985-4005 */
            changed = 1;
            mv_bi[L][0] = r.mv_x;
            mv_bi[L][1] = r.mv_y;
            ridx_bi[L] = k;
            cost_bi = c;
            mot[L] = b - mb[2] - mot[1 - L];
            bits_bi = b;
            if (niter != 1) {   /* set motion + motionCompensation of list L */
              ps_ref[L] = k;
              ps_mv[L][0] = r.mv_x;
              ps_mv[L][1] = r.mv_y;
            }
          }
        }
        if (rc) break;
        if (!changed) {   /* 4008-4021 */
          if (cost_bi <= cost[0] && cost_bi <= cost[1]) {
            int i0 = mvpi_bi[0][ridx_bi[0]];
            pi_check_best_mvp(ml, q->cand[0][ridx_bi[0]], q->n_cand[0][ridx_bi[0]], mv_bi[0][0], mv_bi[0][1], &i0,
                              &bits_bi, &cost_bi);
            mvpi_bi[0][ridx_bi[0]] = i0;
            if (!mvdl1z) {
              int i1 = mvpi_bi[1][ridx_bi[1]];
              pi_check_best_mvp(ml, q->cand[1][ridx_bi[1]], q->n_cand[1][ridx_bi[1]], mv_bi[1][0], mv_bi[1][1],
                                &i1, &bits_bi, &cost_bi);
              mvpi_bi[1][ridx_bi[1]] = i1;
            }
          }
          break;
        }
      }
      if (rc) break;
    }
    o->bi_cost = cost_bi;
    o->bi_bits = restricted ? 0 : bits_bi;
    o->uni_cost[0] = cost[0];
    o->uni_bits[0] = bits[0];
    o->uni_cost[1] = cost_v1;
    o->uni_bits[1] = bits_v1;
    /* decision (4041-4105) */
    if (cost_bi <= cost[0] && cost_bi <= cost_v1) {
      last_mode = 2;
      o->inter_dir = 3;
      o->bits = bits_bi;
      o->cost = cost_bi;
      for (int l = 0; l < 2; l++) {
        o->ref_idx[l] = (uint8_t)ridx_bi[l];
        o->mvp_idx[l] = (uint8_t)mvpi_bi[l][ridx_bi[l]];
        o->mv[l][0] = mv_bi[l][0];
        o->mv[l][1] = mv_bi[l][1];
        o->mvp[l][0] = q->cand[l][ridx_bi[l]][mvpi_bi[l][ridx_bi[l]]][0];
        o->mvp[l][1] = q->cand[l][ridx_bi[l]][mvpi_bi[l][ridx_bi[l]]][1];
      }
    } else if (cost[0] <= cost_v1) {
      last_mode = 0;
      o->inter_dir = 1;
      o->bits = bits[0];
      o->cost = cost[0];
      o->ref_idx[0] = (uint8_t)ridx[0];
      o->mvp_idx[0] = (uint8_t)mvpi[0][ridx[0]];
      o->mv[0][0] = mv[0][0];
      o->mv[0][1] = mv[0][1];
      o->mvp[0][0] = q->cand[0][ridx[0]][mvpi[0][ridx[0]]][0];
      o->mvp[0][1] = q->cand[0][ridx[0]][mvpi[0][ridx[0]]][1];
    } else {
      last_mode = 1;
      o->inter_dir = 2;
      o->bits = bits_v1;
      o->cost = cost_v1;
      o->ref_idx[1] = (uint8_t)ridx_v1;
      o->mvp_idx[1] = (uint8_t)mvpi[1][ridx_v1];
      o->mv[1][0] = mv_v1[0];
      o->mv[1][1] = mv_v1[1];
      o->mvp[1][0] = q->cand[1][ridx_v1][mvpi[1][ridx_v1]][0];
      o->mvp[1][1] = q->cand[1][ridx_v1][mvpi[1][ridx_v1]][1];
    }
  }
  free(pred);
  free(key);
  return rc;
}
