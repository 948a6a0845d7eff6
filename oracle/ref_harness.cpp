// ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own compiled TLibCommon classes (built from /root/reference by
// oracle/Makefile into oracle/_ref/libhmref.so; nothing is copied into this repository):
//   TComInterpolationFilter::filterHor/filterVer   (TComInterpolationFilter.cpp:341-394)
//   TComRdCost::setDistParam + DistFunc             (TComRdCost.cpp:200-275, 335-1495)
//   TComRdCost cost/lambda helpers                  (TComRdCost.cpp:104-117, .h:159-174)
//   TComPicYuv padding (createWithoutCUInfo + extendPicBorder, TComPicYuv.cpp:81-117, 229-276)
//   TComPrediction::initTempBuff scratch planes     (TComPrediction.cpp:126-145)
//
// TEncSearch.cpp itself needs Eigen 3.3.7 (TEncSearch.cpp:39), which is absent here, so its
// orchestration is restated below in the same plane-walk order the encoder uses:
//   xExtDIFUpSamplingH (TEncSearch.cpp:6331-6365), xExtDIFUpSamplingQ (6378-6532),
//   xPatternRefinement (1591-1645), xPatternSearchFracDIF (5232-5269),
//   xTZ8PointSquareSearch(save) + xTZSearchHelp normal branch (1324-1377, 1155-1188),
//   xMotionEstimation tail (4529-4597).  NN_pred() (85-204) is restated as a scalar loop.
// The restated pieces are independent of oracle/fme_oracle.c, which evaluates each candidate
// as a direct quarter-pel prediction instead of walking the planes.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "TLibCommon/TComPattern.h"
#include "TLibCommon/TComPicYuv.h"
#include "TLibCommon/TComPrediction.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComWeightPrediction.h"
#include "TLibCommon/TComYuv.h"

#include "../include/fme.h"

namespace {

const int kH9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
const int kQ9[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

// A TComPrediction subclass gives access to m_filteredBlock / m_filteredBlockTmp / m_if,
// exactly as TEncSearch (a TComPrediction subclass) uses them.
class RefSearch : public TComPrediction {
 public:
  TComRdCost rd;
  DistParam dp;
  bool hadme = true;
  int fen = 0;
  int bd = 8;   // the sequence's luma bit depth (m_cDistParam.bitDepth, TEncSearch.cpp:1090, 1630)

  RefSearch() {
    initTempBuff(CHROMA_400);
    rd.init();
  }

  void setLambda(double lambda) {
    BitDepths bds;
    bds.recon[CHANNEL_TYPE_LUMA] = bd;
    bds.recon[CHANNEL_TYPE_CHROMA] = bd;
    rd.setLambda(lambda, bds);
    rd.selectMotionLambda(true, 0, false);
  }

  // --- half-pel planes around the integer position (xExtDIFUpSamplingH) -------------
  void upH(Pel* roi, int stride, int w, int h) {
    const int ts = m_filteredBlockTmp[0].getStride(COMPONENT_Y);
    const int ds = m_filteredBlock[0][0].getStride(COMPONENT_Y);
    Pel* src = roi - 4 * stride - 1;  // half filter size rows up, one column left
    m_if.filterHor(COMPONENT_Y, src, stride, m_filteredBlockTmp[0].getAddr(COMPONENT_Y), ts, w + 1, h + 8, 0, false, CHROMA_400, bd);
    m_if.filterHor(COMPONENT_Y, src, stride, m_filteredBlockTmp[2].getAddr(COMPONENT_Y), ts, w + 1, h + 8, 2, false, CHROMA_400, bd);
    Pel* t0 = m_filteredBlockTmp[0].getAddr(COMPONENT_Y);
    Pel* t2 = m_filteredBlockTmp[2].getAddr(COMPONENT_Y);
    m_if.filterVer(COMPONENT_Y, t0 + 4 * ts + 1, ts, m_filteredBlock[0][0].getAddr(COMPONENT_Y), ds, w, h, 0, false, true, CHROMA_400, bd);
    m_if.filterVer(COMPONENT_Y, t0 + 3 * ts + 1, ts, m_filteredBlock[2][0].getAddr(COMPONENT_Y), ds, w, h + 1, 2, false, true, CHROMA_400, bd);
    m_if.filterVer(COMPONENT_Y, t2 + 4 * ts, ts, m_filteredBlock[0][2].getAddr(COMPONENT_Y), ds, w + 1, h, 0, false, true, CHROMA_400, bd);
    m_if.filterVer(COMPONENT_Y, t2 + 3 * ts, ts, m_filteredBlock[2][2].getAddr(COMPONENT_Y), ds, w + 1, h + 1, 2, false, true, CHROMA_400, bd);
  }

  // --- quarter-pel planes around the best half position (xExtDIFUpSamplingQ) ---------
  void upQ(Pel* roi, int stride, int w, int h, int hx, int hy) {
    const int ts = m_filteredBlockTmp[0].getStride(COMPONENT_Y);
    const int ds = m_filteredBlock[0][0].getStride(COMPONENT_Y);
    const int extH = (hy == 0) ? h + 8 : h + 7;
    Pel* base = roi - 4 * stride - 1;
    Pel* s1 = base + (hy > 0 ? stride : 0) + (hx >= 0 ? 1 : 0);
    Pel* s3 = base + (hy > 0 ? stride : 0) + (hx > 0 ? 1 : 0);
    Pel* t0 = m_filteredBlockTmp[0].getAddr(COMPONENT_Y);
    Pel* t1 = m_filteredBlockTmp[1].getAddr(COMPONENT_Y);
    Pel* t2 = m_filteredBlockTmp[2].getAddr(COMPONENT_Y);
    Pel* t3 = m_filteredBlockTmp[3].getAddr(COMPONENT_Y);
    m_if.filterHor(COMPONENT_Y, s1, stride, t1, ts, w, extH, 1, false, CHROMA_400, bd);
    m_if.filterHor(COMPONENT_Y, s3, stride, t3, ts, w, extH, 3, false, CHROMA_400, bd);
    auto ver = [&](Pel* src, int fy, int dy, int dx) {
      m_if.filterVer(COMPONENT_Y, src, ts, m_filteredBlock[dy][dx].getAddr(COMPONENT_Y), ds, w, h, fy, false, true, CHROMA_400, bd);
    };
    const int rowTop = 3 * ts;      // (halfFilterSize - 1) rows
    const int rowZero = hy == 0 ? ts : 0;
    ver(t1 + rowTop + rowZero, 1, 1, 1);
    ver(t1 + rowTop, 3, 3, 1);
    if (hy != 0) {
      ver(t1 + rowTop, 2, 2, 1);
      ver(t3 + rowTop, 2, 2, 3);
    } else {
      ver(t1 + 4 * ts, 0, 0, 1);
      ver(t3 + 4 * ts, 0, 0, 3);
    }
    if (hx != 0) {
      Pel* a = t2 + rowTop + (hx > 0 ? 1 : 0) + (hy >= 0 ? ts : 0);
      ver(a, 1, 1, 2);
      Pel* b = t2 + rowTop + (hx > 0 ? 1 : 0) + (hy > 0 ? ts : 0);
      ver(b, 3, 3, 2);
    } else {
      ver(t0 + rowTop + 1 + (hy >= 0 ? ts : 0), 1, 1, 0);
      ver(t0 + rowTop + 1 + (hy > 0 ? ts : 0), 3, 3, 0);
    }
    ver(t3 + rowTop + rowZero, 1, 1, 3);
    ver(t3 + rowTop, 3, 3, 3);
  }

  // --- 9-candidate refinement (xPatternRefinement) -----------------------------------
  Distortion refine(TComPattern* key, int baseX, int baseY, int frac, int& mvx, int& mvy, bool allowHad) {
    const int rs = m_filteredBlock[0][0].getStride(COMPONENT_Y);
    rd.setDistParam(key, m_filteredBlock[0][0].getAddr(COMPONENT_Y), rs, 1, dp, hadme && allowHad);
    const int (*tab)[2] = frac == 2 ? kH9 : kQ9;
    Distortion best = std::numeric_limits<Distortion>::max();
    int bi = 0;
    for (int i = 0; i < 9; i++) {
      const int hv = (tab[i][0] + baseX) * frac, vv = (tab[i][1] + baseY) * frac;
      Pel* p = m_filteredBlock[vv & 3][hv & 3].getAddr(COMPONENT_Y);
      if (hv == 2 && (vv & 1) == 0) p += 1;
      if ((hv & 1) == 0 && vv == 2) p += rs;
      dp.pCur = p;
      dp.bitDepth = bd;
      Distortion d = dp.DistFunc(&dp);
      d += rd.getCostOfVectorWithPredictor(tab[i][0] + mvx, tab[i][1] + mvy);
      if (d < best) {
        best = d;
        bi = i;
        dp.m_maximumDistortionForEarlyExit = d;
      }
    }
    mvx = tab[bi][0];
    mvy = tab[bi][1];
    return best;
  }

  // --- xPatternSearchFracDIF (cost scale 1 on entry, as xMotionEstimation sets) ------
  Distortion fracDif(bool lossless, TComPattern* key, Pel* refY, int stride, int ix, int iy, int& hx, int& hy, int& qx, int& qy) {
    Pel* roi = refY + ix + iy * stride;
    const int w = key->getROIYWidth(), h = key->getROIYHeight();
    rd.setCostScale(1);
    upH(roi, stride, w, h);
    int mx = ix * 2, my = iy * 2;
    Distortion cost = refine(key, 0, 0, 2, mx, my, !lossless);
    hx = mx;
    hy = my;
    rd.setCostScale(0);
    upQ(roi, stride, w, h, hx, hy);
    int qmx = (ix * 2 + hx) * 2, qmy = (iy * 2 + hy) * 2;
    cost = refine(key, hx * 2, hy * 2, 1, qmx, qmy, !lossless);
    qx = qmx;
    qy = qmy;
    return cost;
  }

  // --- xTZSearchHelp normal branch with save=true -----------------------------------
  struct Best {
    Distortion sad;
    int x, y;
  };
  Distortion intDist(TComPattern* key, Pel* refY, int stride, int x, int y) {
    rd.setDistParam(key, refY + y * stride + x, stride, dp);
    dp.bitDepth = bd;
    if ((fen == 1 || fen == 3) && dp.iRows > 8) dp.iSubShift = 1;
    return dp.DistFunc(&dp);
  }
  void help(TComPattern* key, Pel* refY, int stride, Best& b, int x, int y, std::vector<uint32_t>& pushed) {
    Distortion d = intDist(key, refY, stride, x, y);
    pushed.push_back(d);
    if (d < b.sad) {
      d += rd.getCostOfVectorWithPredictor(x, y);
      if (d < b.sad) {
        b.sad = d;
        b.x = x;
        b.y = y;
      }
    }
  }
};

struct Pic {
  TComPicYuv yuv;
  bool set = false;
  TComPicYuv yuv420;    // 4:2:0 picture with its 80 / 40-sample margins (motion compensation)
  bool set420 = false;
};

// A generic NN_pred net (nn_mode 2) restated in the style of the reference's backups: global-like
// activation arrays X[l][40], memset per call except the carried layers (Backups/15:4957-4961),
// `X[i] += w * x` in j order, `+= b`, relu * gamma + beta, OUT += w * X, += bout, [sigmoid],
// std::max_element (Backups/4:4437-4486, Backups/15:4954-5052).  Independent of fme_oracle.c's
// forward (which walks a parameter pointer); both take the parameters in fme_load_nn_net order.
struct DeepNet {
  fme_nn_net d{};
  std::vector<double> p;
  double Xd[FME_NN_MAX_HIDDEN][FME_NN_MAX_WIDTH] = {};
  float Xf[FME_NN_MAX_HIDDEN][FME_NN_MAX_WIDTH] = {};

  template <typename T>
  int run(T X[][FME_NN_MAX_WIDTH], const uint32_t* e, uint32_t C, int H, int W, double* logits) {
    auto rowMaster = [](int v) { switch (v) { case 4: return 1; case 8: return 2; case 16: return 3; case 12: return 4; case 24: return 5; case 32: return 6; case 64: return 7; default: return 0; } };
    auto rowW = [](int v) { switch (v) { case 4: return 1; case 8: return 2; case 12: return 3; case 16: return 4; case 24: return 5; case 32: return 6; case 64: return 7; default: return 0; } };
    const bool emb = d.embedding != FME_NN_EMB_NONE;
    // offsets of every tensor
    size_t o = emb ? 64 : 0;
    size_t wOff[FME_NN_MAX_HIDDEN], bOff[FME_NN_MAX_HIDDEN], gOff[FME_NN_MAX_HIDDEN], beOff[FME_NN_MAX_HIDDEN];
    int nin = emb ? 17 : 9;
    int fan[FME_NN_MAX_HIDDEN + 1];
    for (int l = 0; l < d.n_hidden; l++) {
      fan[l] = nin;
      wOff[l] = o; o += (size_t)d.width[l] * nin;
      bOff[l] = o; o += d.width[l];
      gOff[l] = o; o += d.width[l];
      beOff[l] = o; o += d.width[l];
      nin = d.width[l];
    }
    fan[d.n_hidden] = nin;
    const size_t outW = o, outB = o + 49 * (size_t)nin, gin = outB + 49, mean = gin + 9, sd = mean + 9;
    auto P = [&](size_t i) { return (T)p[i]; };
    T IN[17] = {};
    const uint32_t errs[9] = {e[0], e[1], e[2], e[3], C, e[4], e[5], e[6], e[7]};
    const int base = emb ? 8 : 0;
    for (int i = 0; i < 9; i++) {
      T v = (T)errs[i];
      IN[base + i] = (v - P(mean + i)) / P(sd + i);
    }
    if (emb) {
      const int rh = d.embedding == FME_NN_EMB_SWAP ? rowW(H) : rowMaster(H);
      for (int k = 0; k < 4; k++) {
        IN[k] = P(rh * 4 + k);
        IN[4 + k] = P(32 + rowW(W) * 4 + k);
      }
    }
    for (int i = 0; i < 9; i++) IN[base + i] = IN[base + i] * P(gin + i);
    for (int l = 0; l < d.n_hidden; l++)
      if (!((d.carry_hidden >> l) & 1)) std::memset(X[l], 0, sizeof(X[l]));
    for (int l = 0; l < d.n_hidden; l++) {
      const T* src = l == 0 ? IN : X[l - 1];
      for (int i = 0; i < d.width[l]; i++) {
        for (int j = 0; j < fan[l]; j++) {
          volatile T prod = P(wOff[l] + (size_t)i * fan[l] + j) * src[j];
          X[l][i] += prod;
        }
        X[l][i] += P(bOff[l] + i);
        const T r = X[l][i] > 0 ? X[l][i] : (T)0;
        volatile T m = r * P(gOff[l] + i);
        X[l][i] = m + P(beOff[l] + i);
      }
    }
    T OUT[49] = {};
    const T* last = X[d.n_hidden - 1];
    for (int i = 0; i < 49; i++) {
      for (int j = 0; j < nin; j++) {
        volatile T prod = P(outW + (size_t)i * nin + j) * last[j];
        OUT[i] += prod;
      }
      OUT[i] += P(outB + i);
      if (d.out_act == FME_NN_OUT_SIGMOID) OUT[i] = (T)1 / ((T)1 + std::exp(-OUT[i]));
    }
    if (logits)
      for (int i = 0; i < 49; i++) logits[i] = (double)OUT[i];
    return (int)std::distance(OUT, std::max_element(OUT, OUT + 49));
  }
  int forward(const uint32_t* e, uint32_t C, int H, int W, double* logits) {
    return d.precision == FME_NN_F64 ? run<double>(Xd, e, C, H, W, logits) : run<float>(Xf, e, C, H, W, logits);
  }
  void reset() {
    std::memset(Xd, 0, sizeof(Xd));
    std::memset(Xf, 0, sizeof(Xf));
  }
};

struct RefCtx {
  RefSearch s;
  DeepNet net;
  Pic pics[FME_MAX_PICTURES];
  double lambda[FME_MAX_LAMBDAS] = {0};
  std::vector<int16_t> keys;
  std::vector<float> nn;
  int nn_mode = 1;
  // NN_pred global state (TEncSearch.cpp:55-57): array_e storage, C, PUHeight, PUWidth.
  uint32_t slot[8] = {0};
  uint32_t C = 0, puh = 0, puw = 0;
  std::vector<uint32_t> nn_in;   // FME_JOB_NN_IN rows (ref_set_nn_inputs), 9 per job
  // explicit WP parameters per [list][picture][component]: iWeight, iOffset, uiLog2WeightDenom
  int wp[2][FME_MAX_PICTURES][3][3];
  RefCtx() {
    for (auto& l : wp)
      for (auto& p : l)
        for (auto& c : p) { c[0] = 1; c[1] = 0; c[2] = 0; }
  }
};

int nnClass(const float* P, const uint32_t* e, uint32_t c, int H, int W) {
  // Scalar NN_pred(): sequential-k float32 sums, no FMA (TEncSearch.cpp:88-134).
  auto eh = [](int v) { switch (v) { case 4: return 1; case 8: return 2; case 16: return 3; case 12: return 4; case 24: return 5; case 32: return 6; case 64: return 7; default: return 0; } };
  auto ew = [](int v) { switch (v) { case 4: return 1; case 8: return 2; case 12: return 3; case 16: return 4; case 24: return 5; case 32: return 6; case 64: return 7; default: return 0; } };
  const float *emb0 = P, *emb1 = P + 32, *w1 = P + 64, *w2 = P + 438, *w3 = P + 878;
  const float *b1 = P + 1858, *g1 = P + 1880, *be1 = P + 1902, *b2 = P + 1924, *g2 = P + 1944;
  const float *be2 = P + 1964, *bo = P + 1984, *gin = P + 2033, *mean = P + 2042, *sd = P + 2051;
  float in[17], x1[22], x2[20];
  for (int k = 0; k < 4; k++) {
    in[k] = emb0[eh(H) * 4 + k];
    in[4 + k] = emb1[ew(W) * 4 + k];
  }
  const uint32_t raw[9] = {e[0], e[1], e[2], e[3], c, e[4], e[5], e[6], e[7]};
  for (int k = 0; k < 9; k++) {
    volatile float t = ((float)raw[k] - mean[k]) / sd[k];
    in[8 + k] = t * gin[k];
  }
  for (int r = 0; r < 22; r++) {
    volatile float s = 0.f;
    for (int k = 0; k < 17; k++) { volatile float p = w1[r * 17 + k] * in[k]; s = s + p; }
    float v = s + b1[r];
    v = v < 0.f ? 0.f : v;
    volatile float m = v * g1[r];
    x1[r] = m + be1[r];
  }
  for (int r = 0; r < 20; r++) {
    volatile float s = 0.f;
    for (int k = 0; k < 22; k++) { volatile float p = w2[r * 22 + k] * x1[k]; s = s + p; }
    float v = s + b2[r];
    v = v < 0.f ? 0.f : v;
    volatile float m = v * g2[r];
    x2[r] = m + be2[r];
  }
  int best = 0;
  float bv = 0.f;
  for (int r = 0; r < 49; r++) {
    volatile float s = 0.f;
    for (int k = 0; k < 20; k++) { volatile float p = w3[r * 20 + k] * x2[k]; s = s + p; }
    float o = s + bo[r];
    if (r == 0 || o > bv) { bv = o; best = r; }
  }
  return best;
}

}  // namespace

extern "C" {

void* ref_create(int use_hadamard, int fen, int nn_mode) {
  initROM();
  RefCtx* c = new RefCtx();
  c->s.hadme = use_hadamard != 0;
  c->s.fen = fen;
  c->nn_mode = nn_mode;
  return c;
}

void ref_destroy(void* h) { delete static_cast<RefCtx*>(h); }

int ref_set_picture(void* h, int id, const uint8_t* luma, int stride, int w, int hgt) {
  RefCtx* c = static_cast<RefCtx*>(h);
  Pic& p = c->pics[id];
  p.yuv.createWithoutCUInfo(w, hgt, CHROMA_400, true, 64, 64);  // 80-sample margin
  Pel* dst = p.yuv.getAddr(COMPONENT_Y);
  const int ds = p.yuv.getStride(COMPONENT_Y);
  for (int y = 0; y < hgt; y++)
    for (int x = 0; x < w; x++) dst[y * ds + x] = luma[(size_t)y * stride + x];
  p.yuv.extendPicBorder();
  p.set = true;
  return 0;
}

// main10: the luma bit depth of the sub-pel path (ref_refine) and 16-bit sample planes
void ref_set_bit_depth(void* h, int bd) { static_cast<RefCtx*>(h)->s.bd = bd; }

int ref_set_picture16(void* h, int id, const uint16_t* luma, int stride, int w, int hgt) {
  RefCtx* c = static_cast<RefCtx*>(h);
  Pic& p = c->pics[id];
  p.yuv.createWithoutCUInfo(w, hgt, CHROMA_400, true, 64, 64);  // 80-sample margin
  Pel* dst = p.yuv.getAddr(COMPONENT_Y);
  const int ds = p.yuv.getStride(COMPONENT_Y);
  for (int y = 0; y < hgt; y++)
    for (int x = 0; x < w; x++) dst[y * ds + x] = (Pel)luma[(size_t)y * stride + x];
  p.yuv.extendPicBorder();
  p.set = true;
  return 0;
}

void ref_set_lambda(void* h, int id, double lambda) { static_cast<RefCtx*>(h)->lambda[id] = lambda; }

void ref_set_keys(void* h, const int16_t* k, size_t n) {
  RefCtx* c = static_cast<RefCtx*>(h);
  c->keys.assign(k, k + n);
}

void ref_load_nn(void* h, const float* p) {
  RefCtx* c = static_cast<RefCtx*>(h);
  c->nn.assign(p, p + FME_NN_PARAMS);
}

void ref_set_nn_inputs(void* h, const uint32_t* rows, int n) {
  RefCtx* c = static_cast<RefCtx*>(h);
  if (rows) c->nn_in.assign(rows, rows + (size_t)9 * n);
  else c->nn_in.clear();
}

void ref_nn_reset(void* h) {
  RefCtx* c = static_cast<RefCtx*>(h);
  std::memset(c->slot, 0, sizeof(c->slot));
  c->C = c->puh = c->puw = 0;
  c->net.reset();
}

// NN_pred()'s carried globals from a 12-word state (fme_nn_get_state layout: array_e slots 0..7, C,
// PUHeight, PUWidth, written mask): the state a run of jobs in the middle of a stream starts from.
void ref_nn_set_state(void* h, const uint32_t* st) {
  RefCtx* c = static_cast<RefCtx*>(h);
  for (int k = 0; k < 8; k++) c->slot[k] = st[k];
  c->C = st[8];
  c->puh = st[9];
  c->puw = st[10];
}

void ref_load_nn_net(void* h, const fme_nn_net* d, const double* p, int count) {
  RefCtx* c = static_cast<RefCtx*>(h);
  c->net.d = *d;
  c->net.p.assign(p, p + count);
  c->net.reset();
}

// One NN_pred() call of the generic net on explicit inputs (updates carried layers).
int ref_nn_net_class(void* h, const uint32_t* e, uint32_t cc, int H, int W, double* logits) {
  return static_cast<RefCtx*>(h)->net.forward(e, cc, H, W, logits);
}

int ref_nn_class(void* h, const uint32_t* e, uint32_t cc, int H, int W) {
  return nnClass(static_cast<RefCtx*>(h)->nn.data(), e, cc, H, W);
}

// Interpolate one PU at quarter-pel (qx,qy) through the reference filter classes
// (TComPrediction::xPredInterBlk order, TComPrediction.cpp:643-683).
int ref_pred_block(void* h, int id, int x0, int y0, int w, int hgt, int qx, int qy, int16_t* out) {
  RefCtx* c = static_cast<RefCtx*>(h);
  if (id < 0 || id >= FME_MAX_PICTURES || !c->pics[id].set || w < 1 || w > 64 || hgt < 1 || hgt > 64)
    return FME_E_STATE;
  TComPicYuv& pic = c->pics[id].yuv;
  const int stride = pic.getStride(COMPONENT_Y);
  Pel* src = pic.getAddr(COMPONENT_Y) + (y0 + (qy >> 2)) * stride + x0 + (qx >> 2);
  const int fx = qx & 3, fy = qy & 3;
  TComInterpolationFilter f;
  std::vector<Pel> dst(w * hgt), tmp(w * (hgt + 7));
  if (fy == 0) {
    f.filterHor(COMPONENT_Y, src, stride, dst.data(), w, w, hgt, fx, true, CHROMA_400, c->s.bd);
  } else if (fx == 0) {
    f.filterVer(COMPONENT_Y, src, stride, dst.data(), w, w, hgt, fy, true, true, CHROMA_400, c->s.bd);
  } else {
    f.filterHor(COMPONENT_Y, src - 3 * stride, stride, tmp.data(), w, w, hgt + 7, fx, false, CHROMA_400, c->s.bd);
    f.filterVer(COMPONENT_Y, tmp.data() + 3 * w, w, dst.data(), w, w, hgt, fy, false, true, CHROMA_400, c->s.bd);
  }
  for (int i = 0; i < w * hgt; i++) out[i] = dst[i];
  return 0;
}

// Distortions through the reference DistParam dispatch.
uint32_t ref_satd(void* h, const int16_t* org, int os, const int16_t* cur, int cs, int w, int hgt, int hadamard) {
  RefCtx* c = static_cast<RefCtx*>(h);
  DistParam d;
  c->s.rd.setDistParam(d, 8, org, os, cur, cs, w, hgt, hadamard != 0);
  return d.DistFunc(&d);
}

// The whole sub-pel part of xMotionEstimation for each job in order.
int ref_refine(void* h, const fme_job* jobs, fme_result* res, int n) {
  RefCtx* c = static_cast<RefCtx*>(h);
  RefSearch& s = c->s;
  std::vector<Pel> keybuf(64 * 64);
  std::vector<uint32_t> pushed;
  for (int i = 0; i < n; i++) {
    const fme_job& j = jobs[i];
    fme_result& r = res[i];
    std::memset(&r, 0, sizeof(r));
    if (!c->pics[j.ref_id].set) return FME_E_STATE;
    TComPicYuv& ref = c->pics[j.ref_id].yuv;
    const int rs = ref.getStride(COMPONENT_Y);
    Pel* refY = ref.getAddr(COMPONENT_Y) + j.y * rs + j.x;
    const int w = j.w, hh = j.h;
    if (j.key_offset >= 0) {
      for (int k = 0; k < w * hh; k++) keybuf[k] = c->keys[j.key_offset + k];
    } else {
      TComPicYuv& org = c->pics[j.org_id].yuv;
      const int os = org.getStride(COMPONENT_Y);
      const Pel* o = org.getAddr(COMPONENT_Y) + j.y * os + j.x;
      for (int y = 0; y < hh; y++)
        for (int x = 0; x < w; x++) keybuf[y * w + x] = o[y * os + x];
    }
    TComPattern key;
    key.initPattern(keybuf.data(), w, hh, w, s.bd);
    s.setLambda(c->lambda[j.lambda_id]);
    TComMv pred(j.mvp_x, j.mvp_y);
    s.rd.setPredictor(pred);

    int ix = j.mv_x, iy = j.mv_y;
    uint32_t C = 0;
    int npush = 0;
    if (j.flags & FME_JOB_NN_IN) {   // the backups' inputs, as xPatternSearchFast read them
      if ((size_t)9 * (i + 1) > c->nn_in.size()) return FME_E_INVALID;
      const uint32_t* row = c->nn_in.data() + (size_t)9 * i;
      npush = 8;
      for (int k = 0; k < 8; k++) {
        r.emi[k] = row[k];
        c->slot[k] = row[k];
      }
      C = row[8];
      c->C = C;
      c->puh = hh;
      c->puw = w;
    } else if (j.flags & FME_JOB_EMI) {
      s.rd.setCostScale(2);
      RefSearch::Best b;
      b.x = j.mv_x;
      b.y = j.mv_y;
      b.sad = s.intDist(&key, refY, rs, b.x, b.y) + s.rd.getCostOfVectorWithPredictor(b.x, b.y);
      pushed.clear();
      const int sx = b.x, sy = b.y;
      if (sy - 1 >= j.lt_y) {
        if (sx - 1 >= j.lt_x) s.help(&key, refY, rs, b, sx - 1, sy - 1, pushed);
        s.help(&key, refY, rs, b, sx, sy - 1, pushed);
        if (sx + 1 <= j.rb_x) s.help(&key, refY, rs, b, sx + 1, sy - 1, pushed);
      }
      if (sx - 1 >= j.lt_x) s.help(&key, refY, rs, b, sx - 1, sy, pushed);
      if (sx + 1 <= j.rb_x) s.help(&key, refY, rs, b, sx + 1, sy, pushed);
      if (sy + 1 <= j.rb_y) {
        if (sx - 1 >= j.lt_x) s.help(&key, refY, rs, b, sx - 1, sy + 1, pushed);
        s.help(&key, refY, rs, b, sx, sy + 1, pushed);
        if (sx + 1 <= j.rb_x) s.help(&key, refY, rs, b, sx + 1, sy + 1, pushed);
      }
      C = b.sad - s.rd.getCostOfVectorWithPredictor(b.x, b.y);
      ix = b.x;
      iy = b.y;
      npush = (int)pushed.size();
      for (int k = 0; k < npush; k++) {
        r.emi[k] = pushed[k];
        c->slot[k] = pushed[k];
      }
      c->C = C;
      c->puh = hh;
      c->puw = w;
    }
    r.n_emi = (uint8_t)npush;
    r.c = C;
    r.mv_int_x = (int16_t)ix;
    r.mv_int_y = (int16_t)iy;
    int hx, hy, qx, qy;
    const bool lossless = (j.flags & FME_JOB_LOSSLESS) != 0;
    Distortion fc = s.fracDif(lossless, &key, refY, rs, ix, iy, hx, hy, qx, qy);
    r.half_x = (int8_t)hx; r.half_y = (int8_t)hy; r.qtr_x = (int8_t)qx; r.qtr_y = (int8_t)qy;
    r.frac_cost = fc;
    s.rd.setCostScale(0);
    int ox, oy;
    if (c->nn_mode) {
      int cls = c->nn_mode == 2 ? c->net.forward(c->slot, c->C, (int)c->puh, (int)c->puw, nullptr)
                                : nnClass(c->nn.data(), c->slot, c->C, (int)c->puh, (int)c->puw);
      r.nn_class = (uint8_t)cls;
      ox = cls % 7 - 3;
      oy = cls / 7 - 3;
    } else {
      r.nn_class = 255;
      ox = 2 * hx + qx;
      oy = 2 * hy + qy;
    }
    const int mx = 4 * ix + ox, my = 4 * iy + oy;
    r.mv_x = (int16_t)mx;
    r.mv_y = (int16_t)my;
    const UInt mvb = s.rd.getBitsOfVectorWithPredictor(mx, my);
    const UInt bits = (UInt)j.bits_in + mvb;
    r.bits = bits;
    const double fw = (j.flags & FME_JOB_BIPRED) ? 0.5 : 1.0;
    r.cost = (Distortion)(std::floor(fw * ((double)fc - (double)s.rd.getCost(mvb))) + (double)s.rd.getCost(bits));
  }
  return 0;
}

// ---- motion compensation ---------------------------------------------------------------------
// 4:2:0 picture for motion compensation: TComPicYuv with margins + extendPicBorder.
extern "C++" {
template <typename S>
static int set_picture_yuv(void* h, int id, const S* y, int ys, const S* cb, const S* cr, int cs, int w, int hgt) {
  RefCtx* c = static_cast<RefCtx*>(h);
  Pic& p = c->pics[id];
  p.yuv420.destroy();
  p.yuv420.createWithoutCUInfo(w, hgt, CHROMA_420, true, 64, 64);
  for (int comp = 0; comp < 3; comp++) {
    const ComponentID id_ = ComponentID(comp);
    Pel* dst = p.yuv420.getAddr(id_);
    const int ds = p.yuv420.getStride(id_);
    const S* src = comp == 0 ? y : (comp == 1 ? cb : cr);
    const int ss = comp ? cs : ys, pw = comp ? w / 2 : w, ph = comp ? hgt / 2 : hgt;
    for (int yy = 0; yy < ph; yy++)
      for (int xx = 0; xx < pw; xx++) dst[yy * ds + xx] = src[(size_t)yy * ss + xx];
  }
  p.yuv420.extendPicBorder();
  p.set420 = true;
  return 0;
}
}  // extern "C++"
int ref_set_picture_yuv(void* h, int id, const uint8_t* y, int ys, const uint8_t* cb, const uint8_t* cr, int cs,
                        int w, int hgt) {
  return set_picture_yuv(h, id, y, ys, cb, cr, cs, w, hgt);
}
// 10-bit planes (strides in samples): the main10 configurations (ref_set_bit_depth first)
int ref_set_picture_yuv16(void* h, int id, const uint16_t* y, int ys, const uint16_t* cb, const uint16_t* cr, int cs,
                          int w, int hgt) {
  return set_picture_yuv(h, id, y, ys, cb, cr, cs, w, hgt);
}

// TComPrediction::motionCompensation per job (TComPrediction.cpp:495-560).  TComDataCU /
// TComPic are not built here, so the CU-level steps are restated: clipMv (TComDataCU.cpp
// :2773-2786), xCheckIdenticalMotion (TComPrediction.cpp:476-492) and xPredInterBlk's
// offset / fraction / filter order (616-668) over the reference's TComInterpolationFilter
// (filterHor / filterVer with the component id and CHROMA_420, TComInterpolationFilter.cpp
// :341-394) on the padded TComPicYuv; bi-prediction averages with TComYuv::addAvg.
extern "C++" {
template <typename S>
static int mc_run(void* h, const fme_mc_job* jobs, int n, S* y, int ys, S* cb, S* cr, int cs, int width, int height,
                  int depth) {
  RefCtx* c = static_cast<RefCtx*>(h);
  TComInterpolationFilter f;
  BitDepths bd;
  bd.recon[CHANNEL_TYPE_LUMA] = depth;
  bd.recon[CHANNEL_TYPE_CHROMA] = depth;
  for (int i = 0; i < n; i++) {
    const fme_mc_job& j = jobs[i];
    int lists[2], nl = 0;
    if (j.flags & FME_MC_L0) lists[nl++] = 0;
    if (j.flags & FME_MC_L1) lists[nl++] = 1;
    for (int k = 0; k < nl; k++)
      if (!c->pics[j.ref_id[lists[k]]].set420) return -1 - i;
    const bool wpf = (j.flags & FME_MC_WP) != 0;   // PPS UseWP (P) / WPBiPred (B)
    // xCheckIdenticalMotion (TComPrediction.cpp:476-492) collapses only without WPBiPred
    if (nl == 2 && !wpf && j.ref_id[0] == j.ref_id[1] && j.mv[0][0] == j.mv[1][0] && j.mv[0][1] == j.mv[1][1]) nl = 1;
    const bool bi = nl == 2;
    const bool inter = bi || wpf;   // the lists' 14-bit values (xPredInterUni(..., bi = true))
    TComYuv pred[2], out;
    for (int k = 0; k < 2; k++) pred[k].create(j.w, j.h, CHROMA_420);
    out.create(j.w, j.h, CHROMA_420);
    for (int k = 0; k < nl; k++) {
      TComPicYuv& ref = c->pics[j.ref_id[lists[k]]].yuv420;
      int mx = j.mv[lists[k]][0], my = j.mv[lists[k]][1];
      {   // clipMv
        const int hmax = (width + 8 - j.cu_x - 1) << 2, hmin = (-64 - 8 - j.cu_x + 1) * 4;
        const int vmax = (height + 8 - j.cu_y - 1) << 2, vmin = (-64 - 8 - j.cu_y + 1) * 4;
        mx = std::min(hmax, std::max(hmin, mx));
        my = std::min(vmax, std::max(vmin, my));
      }
      TComYuv& dstYuv = inter ? pred[k] : out;
      for (int comp = 0; comp < 3; comp++) {
        const ComponentID cid = ComponentID(comp);
        const int csx = comp ? 1 : 0;
        const int shH = 2 + csx, shV = 2 + csx;
        const int rs = ref.getStride(cid);
        Pel* src = ref.getAddr(cid) + ((j.y >> csx) + (my >> shV)) * rs + (j.x >> csx) + (mx >> shH);
        Pel* dst = dstYuv.getAddr(cid);
        const int dstS = dstYuv.getStride(cid);
        const int xf = mx & ((1 << shH) - 1), yf = my & ((1 << shV) - 1);
        const int cw = j.w >> csx, ch = j.h >> csx;
        if (yf == 0) {
          f.filterHor(cid, src, rs, dst, dstS, cw, ch, xf, !inter, CHROMA_420, depth);
        } else if (xf == 0) {
          f.filterVer(cid, src, rs, dst, dstS, cw, ch, yf, true, !inter, CHROMA_420, depth);
        } else {
          const int nt = comp ? NTAPS_CHROMA : NTAPS_LUMA;
          std::vector<Pel> tmp((size_t)cw * (ch + nt - 1));
          f.filterHor(cid, src - ((nt >> 1) - 1) * rs, rs, tmp.data(), cw, cw, ch + nt - 1, xf, false, CHROMA_420, depth);
          f.filterVer(cid, tmp.data() + ((nt >> 1) - 1) * cw, cw, dst, dstS, cw, ch, yf, false, !inter, CHROMA_420, depth);
        }
      }
    }
    if (wpf) {
      // getWpScaling (TComWeightPrediction.cpp:247-324) restated (TComDataCU / TComSlice are not
      // built here), then the reference's own addWeightBi / addWeightUni
      WPScalingParam w0[3], w1[3];
      const int scale = 1 << (depth - 8);   // high-precision offsets off
      for (int comp = 0; comp < 3; comp++) {
        for (int k = 0; k < nl; k++) {
          const int* q = c->wp[lists[k]][j.ref_id[lists[k]]][comp];
          WPScalingParam& w = (k == 0 ? w0 : w1)[comp];
          w.bPresentFlag = true;
          w.iWeight = q[0];
          w.iOffset = q[1];
          w.uiLog2WeightDenom = (UInt)q[2];
          w.w = q[0];
        }
        if (bi) {
          w0[comp].o = w0[comp].iOffset * scale;
          w1[comp].o = w1[comp].iOffset * scale;
          w0[comp].offset = w0[comp].o + w1[comp].o;
          w0[comp].shift = (Int)w0[comp].uiLog2WeightDenom + 1;
          w0[comp].round = 1 << w0[comp].uiLog2WeightDenom;
          w1[comp].offset = w0[comp].offset;
          w1[comp].shift = w0[comp].shift;
          w1[comp].round = w0[comp].round;
        } else {
          w0[comp].offset = w0[comp].iOffset * scale;
          w0[comp].shift = (Int)w0[comp].uiLog2WeightDenom;
          w0[comp].round = w0[comp].uiLog2WeightDenom >= 1 ? (1 << (w0[comp].uiLog2WeightDenom - 1)) : 0;
        }
      }
      TComWeightPrediction wpr;
      if (bi) wpr.addWeightBi(&pred[0], &pred[1], bd, 0, j.w, j.h, w0, w1, &out);
      else wpr.addWeightUni(&pred[0], bd, 0, j.w, j.h, w0, &out);
    } else if (bi) {
      out.addAvg(&pred[0], &pred[1], 0, j.w, j.h, bd);
    }
    for (int comp = 0; comp < 3; comp++) {
      const ComponentID cid = ComponentID(comp);
      const int csx = comp ? 1 : 0;
      const Pel* o = out.getAddr(cid);
      const int os = out.getStride(cid);
      S* d = comp == 0 ? y : (comp == 1 ? cb : cr);
      const int dsd = comp ? cs : ys;
      for (int r = 0; r < (j.h >> csx); r++)
        for (int q = 0; q < (j.w >> csx); q++)
          d[(size_t)((j.y >> csx) + r) * dsd + (j.x >> csx) + q] = (S)o[r * os + q];
    }
    for (int k = 0; k < 2; k++) pred[k].destroy();
    out.destroy();
  }
  return 0;
}
}  // extern "C++"
// Explicit weighted-prediction parameters of (list, picture) for FME_MC_WP jobs: per component
// {iWeight, iOffset, uiLog2WeightDenom} (fme_set_wp).
void ref_set_wp(void* h, int list, int id, const int* p9) {
  RefCtx* c = static_cast<RefCtx*>(h);
  for (int comp = 0; comp < 3; comp++)
    for (int k = 0; k < 3; k++) c->wp[list][id][comp][k] = p9[3 * comp + k];
}
int ref_mc(void* h, const fme_mc_job* jobs, int n, uint8_t* y, int ys, uint8_t* cb, uint8_t* cr, int cs, int width,
           int height) {
  return mc_run(h, jobs, n, y, ys, cb, cr, cs, width, height, 8);
}
// 10-bit planes (strides in samples) at the context's bit depth (ref_set_bit_depth): xPredInterBlk and
// addAvg at bitDepth 10 (TComInterpolationFilter.cpp:94-257 headroom 4, TComYuv.cpp:354-415 shift 5)
int ref_mc16(void* h, const fme_mc_job* jobs, int n, uint16_t* y, int ys, uint16_t* cb, uint16_t* cr, int cs,
             int width, int height) {
  return mc_run(h, jobs, n, y, ys, cb, cr, cs, width, height, static_cast<RefCtx*>(h)->s.bd);
}

// xGetTemplateCost (TEncSearch.cpp:4397-4436) over the reference's own pieces: clipMv, xPredInterBlk's
// luma filter order (uni-prediction, isLast) on the padded TComPicYuv, TComRdCost::getDistPart(DF_SAD)
// (TComRdCost.cpp:327-349) and calcRdCost(bits, SAD, DF_SAD) (57-102) with the slot's lambda; at the
// context's luma bit depth (ref_set_bit_depth: main10 filters with headroom 4, SAD >> 2).
uint32_t ref_template_cost(void* h, int org_id, int ref_id, int x, int y, int w, int hgt, int cu_x, int cu_y,
                           int mvx, int mvy, int bits, int lambda_id) {
  RefCtx* c = static_cast<RefCtx*>(h);
  if (org_id < 0 || org_id >= FME_MAX_PICTURES || ref_id < 0 || ref_id >= FME_MAX_PICTURES ||
      !c->pics[org_id].set || !c->pics[ref_id].set || lambda_id < 0 || lambda_id >= FME_MAX_LAMBDAS)
    return 0xFFFFFFFFu;   // the Python wrapper raises on this sentinel
  TComPicYuv& ref = c->pics[ref_id].yuv;
  TComPicYuv& org = c->pics[org_id].yuv;
  const int W = ref.getWidth(COMPONENT_Y), H = ref.getHeight(COMPONENT_Y);
  {   // TComDataCU::clipMv (TComDataCU.cpp:2773-2786)
    const int hmax = (W + 8 - cu_x - 1) << 2, hmin = (-64 - 8 - cu_x + 1) * 4;
    const int vmax = (H + 8 - cu_y - 1) << 2, vmin = (-64 - 8 - cu_y + 1) * 4;
    mvx = std::min(hmax, std::max(hmin, mvx));
    mvy = std::min(vmax, std::max(vmin, mvy));
  }
  TComInterpolationFilter f;
  const int rs = ref.getStride(COMPONENT_Y);
  Pel* src = ref.getAddr(COMPONENT_Y) + (y + (mvy >> 2)) * rs + x + (mvx >> 2);
  std::vector<Pel> dst((size_t)w * hgt);
  const int xf = mvx & 3, yf = mvy & 3;
  if (yf == 0) {
    f.filterHor(COMPONENT_Y, src, rs, dst.data(), w, w, hgt, xf, true, CHROMA_400, c->s.bd);
  } else if (xf == 0) {
    f.filterVer(COMPONENT_Y, src, rs, dst.data(), w, w, hgt, yf, true, true, CHROMA_400, c->s.bd);
  } else {
    std::vector<Pel> tmp((size_t)w * (hgt + NTAPS_LUMA - 1));
    f.filterHor(COMPONENT_Y, src - ((NTAPS_LUMA >> 1) - 1) * rs, rs, tmp.data(), w, w, hgt + NTAPS_LUMA - 1, xf, false,
                CHROMA_400, c->s.bd);
    f.filterVer(COMPONENT_Y, tmp.data() + ((NTAPS_LUMA >> 1) - 1) * w, w, dst.data(), w, w, hgt, yf, false, true,
                CHROMA_400, c->s.bd);
  }
  const int os = org.getStride(COMPONENT_Y);
  const Pel* o = org.getAddr(COMPONENT_Y) + y * os + x;
  c->s.setLambda(c->lambda[lambda_id]);
  const Distortion sad = c->s.rd.getDistPart(c->s.bd, dst.data(), w, o, os, w, hgt, COMPONENT_Y, DF_SAD);
  return (UInt)c->s.rd.calcRdCost(bits, sad, DF_SAD);
}

// The bi-pred search key of xMotionEstimation(bBi) (TEncSearch.cpp:4461-4471): the other list's
// uni-pred luma prediction (motionCompensation: clipMv, xPredInterBlk's filter order, isLast) in a
// TComYuv, the original copied into m_cYuvPredTemp, then the reference's own
// TComYuv::removeHighFreq (TComYuv.cpp:411-455) with or without ClipForBiPredMe.  key: w*h.
int ref_bi_key(void* h, int org_id, int ref_id, int x, int y, int w, int hgt, int cu_x, int cu_y, int mvx, int mvy,
               int clip, int16_t* key) {
  RefCtx* c = static_cast<RefCtx*>(h);
  if (org_id < 0 || org_id >= FME_MAX_PICTURES || ref_id < 0 || ref_id >= FME_MAX_PICTURES ||
      !c->pics[org_id].set || !c->pics[ref_id].set)
    return -1;
  TComPicYuv& ref = c->pics[ref_id].yuv;
  TComPicYuv& org = c->pics[org_id].yuv;
  const int W = ref.getWidth(COMPONENT_Y), H = ref.getHeight(COMPONENT_Y);
  {   // TComDataCU::clipMv
    const int hmax = (W + 8 - cu_x - 1) << 2, hmin = (-64 - 8 - cu_x + 1) * 4;
    const int vmax = (H + 8 - cu_y - 1) << 2, vmin = (-64 - 8 - cu_y + 1) * 4;
    mvx = std::min(hmax, std::max(hmin, mvx));
    mvy = std::min(vmax, std::max(vmin, mvy));
  }
  TComYuv other, temp;
  other.create(w, hgt, CHROMA_400);
  temp.create(w, hgt, CHROMA_400);
  TComInterpolationFilter f;
  const int rs = ref.getStride(COMPONENT_Y);
  Pel* src = ref.getAddr(COMPONENT_Y) + (y + (mvy >> 2)) * rs + x + (mvx >> 2);
  Pel* dst = other.getAddr(COMPONENT_Y);
  const int ds = other.getStride(COMPONENT_Y);
  const int xf = mvx & 3, yf = mvy & 3;
  if (yf == 0) {
    f.filterHor(COMPONENT_Y, src, rs, dst, ds, w, hgt, xf, true, CHROMA_400, c->s.bd);
  } else if (xf == 0) {
    f.filterVer(COMPONENT_Y, src, rs, dst, ds, w, hgt, yf, true, true, CHROMA_400, c->s.bd);
  } else {
    std::vector<Pel> tmp((size_t)w * (hgt + NTAPS_LUMA - 1));
    f.filterHor(COMPONENT_Y, src - ((NTAPS_LUMA >> 1) - 1) * rs, rs, tmp.data(), w, w, hgt + NTAPS_LUMA - 1, xf, false,
                CHROMA_400, c->s.bd);
    f.filterVer(COMPONENT_Y, tmp.data() + ((NTAPS_LUMA >> 1) - 1) * w, w, dst, ds, w, hgt, yf, false, true, CHROMA_400,
                c->s.bd);
  }
  const int os = org.getStride(COMPONENT_Y), ts = temp.getStride(COMPONENT_Y);
  const Pel* o = org.getAddr(COMPONENT_Y) + y * os + x;
  Pel* t = temp.getAddr(COMPONENT_Y);
  for (int r = 0; r < hgt; r++)
    for (int q = 0; q < w; q++) t[r * ts + q] = o[r * os + q];
  const Int bd[MAX_NUM_CHANNEL_TYPE] = {c->s.bd, c->s.bd};
  temp.removeHighFreq(&other, 0, w, hgt, bd, clip != 0);
  for (int r = 0; r < hgt; r++)
    for (int q = 0; q < w; q++) key[r * w + q] = (int16_t)t[r * ts + q];
  other.destroy();
  temp.destroy();
  return 0;
}

}  // extern "C"

// ---- integer motion estimation ----------------------------------------
// xTZSearch (TEncSearch.cpp:4737-5036, FastSearch = 1 diamond, bExtendedSettings = false,
// FastMEAssumingSmootherMV = true) and xPatternSearch (4627-4680) restated over the reference's
// TComRdCost distortion (setDistParam + DistFunc, the same dispatch as the EMI step) and TComMv
// (divideByPowerOf2).  TEncSearch.cpp itself is unbuildable here (Eigen), TComDataCU is not
// built, so clipMv (TComDataCU.cpp:2773-2786) is restated.
namespace {
struct TzStruct {   // IntTZSearchStruct
  Distortion uiBestSad;
  int iBestX, iBestY;
  unsigned uiBestDistance, uiBestRound;
  int ucPointNr;
};
struct Tz {
  RefSearch& s;
  TComPattern* key;
  Pel* refY;
  int stride;
  int lt_x, lt_y, rb_x, rb_y;
  std::vector<long>* array_e;   // the backups' every-point pushes (Backups/4:659), or null
  void clipMv(TComMv& mv, int pw, int ph, int cux, int cuy) {
    const int hmax = (pw + 8 - cux - 1) << 2, hmin = (-64 - 8 - cux + 1) << 2;
    const int vmax = (ph + 8 - cuy - 1) << 2, vmin = (-64 - 8 - cuy + 1) << 2;
    mv.setHor(std::min(hmax, std::max(hmin, mv.getHor())));
    mv.setVer(std::min(vmax, std::max(vmin, mv.getVer())));
  }
  void help(TzStruct& t, int x, int y, int pnr, unsigned dist) {   // xTZSearchHelp, normal branch
    Distortion d = s.intDist(key, refY, stride, x, y);
    if (array_e) array_e->push_back((long)d);   // array_e[counter_i] = uiSad; counter_i++
    if (d < t.uiBestSad) {
      d += s.rd.getCostOfVectorWithPredictor(x, y);
      if (d < t.uiBestSad) {
        t.uiBestSad = d;
        t.iBestX = x;
        t.iBestY = y;
        t.uiBestDistance = dist;
        t.uiBestRound = 0;
        t.ucPointNr = pnr;
      }
    }
  }
  // xTZ8PointDiamondSearch (TEncSearch.cpp:1379-1589), bCheckCornersAtDist1 = corners
  void diamond(TzStruct& t, int sx, int sy, int iDist, bool corners = false) {
    const int iTop = sy - iDist, iBottom = sy + iDist, iLeft = sx - iDist, iRight = sx + iDist;
    t.uiBestRound += 1;
    if (iDist == 1) {
      if (iTop >= lt_y) {
        if (corners) {
          if (iLeft >= lt_x) help(t, iLeft, iTop, 1, iDist);
          help(t, sx, iTop, 2, iDist);
          if (iRight <= rb_x) help(t, iRight, iTop, 3, iDist);
        } else {
          help(t, sx, iTop, 2, iDist);
        }
      }
      if (iLeft >= lt_x) help(t, iLeft, sy, 4, iDist);
      if (iRight <= rb_x) help(t, iRight, sy, 5, iDist);
      if (iBottom <= rb_y) {
        if (corners) {
          if (iLeft >= lt_x) help(t, iLeft, iBottom, 6, iDist);
          help(t, sx, iBottom, 7, iDist);
          if (iRight <= rb_x) help(t, iRight, iBottom, 8, iDist);
        } else {
          help(t, sx, iBottom, 7, iDist);
        }
      }
      return;
    }
    if (iDist <= 8) {
      const int iTop_2 = sy - (iDist >> 1), iBottom_2 = sy + (iDist >> 1);
      const int iLeft_2 = sx - (iDist >> 1), iRight_2 = sx + (iDist >> 1);
      if (iTop >= lt_y && iLeft >= lt_x && iRight <= rb_x && iBottom <= rb_y) {
        help(t, sx, iTop, 2, iDist);
        help(t, iLeft_2, iTop_2, 1, iDist >> 1);
        help(t, iRight_2, iTop_2, 3, iDist >> 1);
        help(t, iLeft, sy, 4, iDist);
        help(t, iRight, sy, 5, iDist);
        help(t, iLeft_2, iBottom_2, 6, iDist >> 1);
        help(t, iRight_2, iBottom_2, 8, iDist >> 1);
        help(t, sx, iBottom, 7, iDist);
      } else {
        if (iTop >= lt_y) help(t, sx, iTop, 2, iDist);
        if (iTop_2 >= lt_y) {
          if (iLeft_2 >= lt_x) help(t, iLeft_2, iTop_2, 1, iDist >> 1);
          if (iRight_2 <= rb_x) help(t, iRight_2, iTop_2, 3, iDist >> 1);
        }
        if (iLeft >= lt_x) help(t, iLeft, sy, 4, iDist);
        if (iRight <= rb_x) help(t, iRight, sy, 5, iDist);
        if (iBottom_2 <= rb_y) {
          if (iLeft_2 >= lt_x) help(t, iLeft_2, iBottom_2, 6, iDist >> 1);
          if (iRight_2 <= rb_x) help(t, iRight_2, iBottom_2, 8, iDist >> 1);
        }
        if (iBottom <= rb_y) help(t, sx, iBottom, 7, iDist);
      }
      return;
    }
    if (iTop >= lt_y && iLeft >= lt_x && iRight <= rb_x && iBottom <= rb_y) {
      help(t, sx, iTop, 0, iDist);
      help(t, iLeft, sy, 0, iDist);
      help(t, iRight, sy, 0, iDist);
      help(t, sx, iBottom, 0, iDist);
      for (int index = 1; index < 4; index++) {
        const int iPosYT = iTop + ((iDist >> 2) * index), iPosYB = iBottom - ((iDist >> 2) * index);
        const int iPosXL = sx - ((iDist >> 2) * index), iPosXR = sx + ((iDist >> 2) * index);
        help(t, iPosXL, iPosYT, 0, iDist);
        help(t, iPosXR, iPosYT, 0, iDist);
        help(t, iPosXL, iPosYB, 0, iDist);
        help(t, iPosXR, iPosYB, 0, iDist);
      }
    } else {
      if (iTop >= lt_y) help(t, sx, iTop, 0, iDist);
      if (iLeft >= lt_x) help(t, iLeft, sy, 0, iDist);
      if (iRight <= rb_x) help(t, iRight, sy, 0, iDist);
      if (iBottom <= rb_y) help(t, sx, iBottom, 0, iDist);
      for (int index = 1; index < 4; index++) {
        const int iPosYT = iTop + ((iDist >> 2) * index), iPosYB = iBottom - ((iDist >> 2) * index);
        const int iPosXL = sx - ((iDist >> 2) * index), iPosXR = sx + ((iDist >> 2) * index);
        if (iPosYT >= lt_y) {
          if (iPosXL >= lt_x) help(t, iPosXL, iPosYT, 0, iDist);
          if (iPosXR <= rb_x) help(t, iPosXR, iPosYT, 0, iDist);
        }
        if (iPosYB <= rb_y) {
          if (iPosXL >= lt_x) help(t, iPosXL, iPosYB, 0, iDist);
          if (iPosXR <= rb_x) help(t, iPosXR, iPosYB, 0, iDist);
        }
      }
    }
  }
  // xTZ8PointSquareSearch (TEncSearch.cpp:1324-1377 = Backups/4:818-873)
  void square(TzStruct& t, int sx, int sy, int iDist) {
    const int iTop = sy - iDist, iBottom = sy + iDist, iLeft = sx - iDist, iRight = sx + iDist;
    t.uiBestRound += 1;
    if (iTop >= lt_y) {
      if (iLeft >= lt_x) help(t, iLeft, iTop, 1, iDist);
      help(t, sx, iTop, 2, iDist);
      if (iRight <= rb_x) help(t, iRight, iTop, 3, iDist);
    }
    if (iLeft >= lt_x) help(t, iLeft, sy, 4, iDist);
    if (iRight <= rb_x) help(t, iRight, sy, 5, iDist);
    if (iBottom <= rb_y) {
      if (iLeft >= lt_x) help(t, iLeft, iBottom, 6, iDist);
      help(t, sx, iBottom, 7, iDist);
      if (iRight <= rb_x) help(t, iRight, iBottom, 8, iDist);
    }
  }
  // xTZ8PointSquareSearch2 (Backups/4:876-965): 16 points at distance iDist, in its call order
  // and with its checks (the x -/+ 1 points of the top / bottom rows test iLeft / iRight)
  void square2(TzStruct& t, int sx, int sy, int iDist) {
    const int iTop = sy - iDist, iBottom = sy + iDist, iLeft = sx - iDist, iRight = sx + iDist;
    t.uiBestRound += 1;
    if (iTop >= lt_y) {
      if (iLeft >= lt_x) help(t, iLeft, iTop, 9, iDist);
      if (iLeft >= lt_x) help(t, sx - 1, iTop, 10, iDist);
      help(t, sx, iTop, 11, iDist);
      if (iRight <= rb_x) help(t, sx + 1, iTop, 12, iDist);
      if (iRight <= rb_x) help(t, iRight, iTop, 13, iDist);
    }
    if (iLeft >= lt_x) help(t, iLeft, sy - 1, 14, iDist);
    if (iRight <= rb_x) help(t, iRight, sy - 1, 15, iDist);
    if (iLeft >= lt_x) help(t, iLeft, sy, 16, iDist);
    if (iRight <= rb_x) help(t, iRight, sy, 17, iDist);
    if (iLeft >= lt_x) help(t, iLeft, sy + 1, 18, iDist);
    if (iRight <= rb_x) help(t, iRight, sy + 1, 19, iDist);
    if (iBottom <= rb_y) {
      if (iLeft >= lt_x) help(t, iLeft, iBottom, 20, iDist);
      if (iLeft >= lt_x) help(t, sx - 1, iBottom, 21, iDist);
      help(t, sx, iBottom, 22, iDist);
      if (iRight <= rb_x) help(t, sx + 1, iBottom, 23, iDist);
      if (iRight <= rb_x) help(t, iRight, iBottom, 24, iDist);
    }
  }
  void twoPoint(TzStruct& t) {   // xTZ2PointSearch: the two neighbours not yet tested
    const int sx = t.iBestX, sy = t.iBestY;
    static const int kPts[9][2][2] = {{{0, 0}, {0, 0}},   {{-1, 0}, {0, -1}}, {{-1, -1}, {1, -1}},
                                      {{0, -1}, {1, 0}},  {{-1, 1}, {-1, -1}}, {{1, -1}, {1, 1}},
                                      {{-1, 0}, {0, 1}},  {{-1, 1}, {1, 1}},   {{1, 0}, {0, 1}}};
    // the reference switches on ucPointNr once, at entry (TEncSearch.cpp:1203): the first point's
    // xTZSearchHelp may set it to 0 before the second is tested
    const int pnr = t.ucPointNr;
    if (pnr < 1 || pnr > 8) return;
    for (int k = 0; k < 2; k++) {
      const int dx = kPts[pnr][k][0], dy = kPts[pnr][k][1];
      const int x = sx + dx, y = sy + dy;
      if (dx < 0 && x < lt_x) continue;
      if (dx > 0 && x > rb_x) continue;
      if (dy < 0 && y < lt_y) continue;
      if (dy > 0 && y > rb_y) continue;
      help(t, x, y, 0, 2);
    }
  }
};
}  // namespace

static int ref_tz_run(void* h, fme_job* jobs, const void* ext0, size_t stride, uint32_t* sad, uint32_t* nn_in,
                      int n);
extern "C" int ref_integer_search_ring(void* h, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad,
                                       uint32_t* nn_in, int n) {
  return ref_tz_run(h, jobs, ext, sizeof(fme_tz_ext), sad, nn_in, n);
}
extern "C" int ref_integer_search(void* h, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n) {
  return ref_tz_run(h, jobs, ext, sizeof(fme_tz_ext), sad, nullptr, n);
}
// FastSearch 0 (FME_TZ_FULL: xPatternSearch, TEncSearch.cpp:4504-4507) and 3 (FME_TZ_ENHANCED:
// xTZSearch with bExtendedSettings, 4726-4727) with the neighbour predictors of fme_tz_ext2
extern "C" int ref_integer_search2(void* h, fme_job* jobs, const fme_tz_ext2* ext, uint32_t* sad, int n) {
  return ref_tz_run(h, jobs, ext, sizeof(fme_tz_ext2), sad, nullptr, n);
}

// nn_in != null: FME_TZ_RING jobs run the backups' xTZSearch tail (Backups/4:4868-4878) and get the
// inputs xPatternSearchFast builds from array_e (:4343-4359).
static int ref_tz_run(void* h, fme_job* jobs, const void* ext0, size_t stride, uint32_t* sad, uint32_t* nn_in,
                      int n) {
  RefCtx* c = static_cast<RefCtx*>(h);
  RefSearch& s = c->s;
  std::vector<Pel> keybuf(64 * 64);
  for (int i = 0; i < n; i++) {
    fme_job& j = jobs[i];
    if (!c->pics[j.ref_id].set) return FME_E_STATE;
    TComPicYuv& ref = c->pics[j.ref_id].yuv;
    const int rs = ref.getStride(COMPONENT_Y);
    Pel* refY = ref.getAddr(COMPONENT_Y) + j.y * rs + j.x;
    const int w = j.w, hh = j.h;
    if (j.key_offset >= 0) {
      for (int k = 0; k < w * hh; k++) keybuf[k] = c->keys[j.key_offset + k];
    } else {
      TComPicYuv& org = c->pics[j.org_id].yuv;
      const int os = org.getStride(COMPONENT_Y);
      const Pel* o = org.getAddr(COMPONENT_Y) + j.y * os + j.x;
      for (int y = 0; y < hh; y++)
        for (int x = 0; x < w; x++) keybuf[y * w + x] = o[y * os + x];
    }
    TComPattern key;
    key.initPattern(keybuf.data(), w, hh, w, s.bd);
    s.setLambda(c->lambda[j.lambda_id]);
    TComMv pred(j.mvp_x, j.mvp_y);
    s.rd.setPredictor(pred);
    s.rd.setCostScale(2);
    std::vector<long> array_e;   // counter_i = 0 at the call's start (the previous call's memset)
    const fme_tz_ext& e = *reinterpret_cast<const fme_tz_ext*>(static_cast<const char*>(ext0) + stride * (size_t)i);
    const int16_t(*preds)[2] = stride >= sizeof(fme_tz_ext2) ? reinterpret_cast<const fme_tz_ext2*>(&e)->preds : nullptr;
    const bool ring = nn_in && (e.flags & FME_TZ_RING) && !(j.flags & FME_JOB_BIPRED);
    Tz tz{s, &key, refY, rs, j.lt_x, j.lt_y, j.rb_x, j.rb_y, ring ? &array_e : nullptr};
    TzStruct t{std::numeric_limits<Distortion>::max(), 0, 0, 0, 0, 0};
    const int pw = ref.getWidth(COMPONENT_Y), ph = ref.getHeight(COMPONENT_Y);
    // (FME_TZ_RING, the backups' FastSearch 1 path, takes precedence over FastSearch 0 / 3)
    if ((j.flags & FME_JOB_BIPRED) || ((e.flags & FME_TZ_FULL) && !ring)) {   // xPatternSearch (bi-pred; FastSearch 0)
      for (int y = j.lt_y; y <= j.rb_y; y++)
        for (int x = j.lt_x; x <= j.rb_x; x++) {
          Distortion d = s.intDist(&key, refY, rs, x, y) + s.rd.getCostOfVectorWithPredictor(x, y);
          if (d < t.uiBestSad) { t.uiBestSad = d; t.iBestX = x; t.iBestY = y; }
        }
    } else {
      const bool bExt = (e.flags & FME_TZ_ENHANCED) && !(e.flags & FME_TZ_FULL) && !ring;   // bExtendedSettings (TEncSearch.cpp:4749-4768)
      const int uiSearchRange = e.search_range ? e.search_range : 64;
      TComMv rcMv(j.mvp_x, j.mvp_y);
      tz.clipMv(rcMv, pw, ph, e.cu_x, e.cu_y);
      rcMv.divideByPowerOf2(2);
      tz.help(t, rcMv.getHor(), rcMv.getVer(), 0, 0);
      if (bExt) {   // bTestOtherPredictedMV (4787-4805)
        for (int index = 0; index < 3; index++) {
          TComMv cMv(preds ? preds[index][0] : 0, preds ? preds[index][1] : 0);
          tz.clipMv(cMv, pw, ph, e.cu_x, e.cu_y);
          cMv.divideByPowerOf2(2);
          if (cMv != rcMv && (cMv.getHor() != t.iBestX && cMv.getVer() != t.iBestY)) tz.help(t, cMv.getHor(), cMv.getVer(), 0, 0);
        }
      }
      if ((rcMv.getHor() != 0 || rcMv.getVer() != 0) && (0 != t.iBestX || 0 != t.iBestY)) tz.help(t, 0, 0, 0, 0);
      int rL = j.lt_x, rR = j.rb_x, rT = j.lt_y, rB = j.rb_y;
      if (e.flags & FME_TZ_PRED2NX2N) {
        TComMv p(e.pred2n_x, e.pred2n_y);
        p <<= 2;
        tz.clipMv(p, pw, ph, e.cu_x, e.cu_y);
        p.divideByPowerOf2(2);
        if ((rcMv != p) && (p.getHor() != t.iBestX || p.getVer() != t.iBestY)) tz.help(t, p.getHor(), p.getVer(), 0, 0);
        TComMv cur(t.iBestX, t.iBestY);   // xSetSearchRange(currBestMv << 2, m_iSearchRange)
        cur <<= 2;
        TComMv tmp = cur;
        tz.clipMv(tmp, pw, ph, e.cu_x, e.cu_y);
        TComMv lt(tmp.getHor() - (uiSearchRange << 2), tmp.getVer() - (uiSearchRange << 2));
        TComMv rb(tmp.getHor() + (uiSearchRange << 2), tmp.getVer() + (uiSearchRange << 2));
        tz.clipMv(lt, pw, ph, e.cu_x, e.cu_y);
        tz.clipMv(rb, pw, ph, e.cu_x, e.cu_y);
        lt.divideByPowerOf2(2);
        rb.divideByPowerOf2(2);
        rL = lt.getHor(); rR = rb.getHor(); rT = lt.getVer(); rB = rb.getVer();
      }
      const bool bBestCandidateZero = t.iBestX == 0 && t.iBestY == 0;   // 4857
      int iStartX = t.iBestX, iStartY = t.iBestY;
      for (int iDist = 1; iDist <= uiSearchRange; iDist *= 2) {
        tz.diamond(t, iStartX, iStartY, iDist, bExt);   // bFirstCornersForDiamondDist1
        if (t.uiBestRound >= 3) break;
      }
      if (bExt && !bBestCandidateZero)   // bNewZeroNeighbourhoodTest, bTestZeroVectorStart (4900-4917)
        for (int iDist = 1; iDist <= (uiSearchRange >> 1); iDist *= 2) tz.diamond(t, 0, 0, iDist, false);
      if (t.uiBestDistance == 1) {
        t.uiBestDistance = 0;
        tz.twoPoint(t);
      }
      if (bExt) {   // bUseAdaptiveRaster (4926-4951)
        int iWindowSize = 5;
        int L = rL, R = rR, T = rT, B = rB;
        if (!((int)t.uiBestDistance > 5)) {
          iWindowSize++;
          L /= 2; R /= 2; T /= 2; B /= 2;
        }
        t.uiBestDistance = iWindowSize;
        for (iStartY = T; iStartY <= B; iStartY += iWindowSize)
          for (iStartX = L; iStartX <= R; iStartX += iWindowSize) tz.help(t, iStartX, iStartY, 0, iWindowSize);
      } else if ((int)t.uiBestDistance > 5) {
        t.uiBestDistance = 5;
        for (iStartY = rT; iStartY <= rB; iStartY += 5)
          for (iStartX = rL; iStartX <= rR; iStartX += 5) tz.help(t, iStartX, iStartY, 0, 5);
      }
      while (t.uiBestDistance > 0) {
        iStartX = t.iBestX;
        iStartY = t.iBestY;
        t.uiBestDistance = 0;
        t.ucPointNr = 0;
        for (int iDist = 1; iDist < uiSearchRange + 1; iDist *= 2) tz.diamond(t, iStartX, iStartY, iDist, bExt);
        if (t.uiBestDistance == 1) {
          t.uiBestDistance = 0;
          if (t.ucPointNr != 0) tz.twoPoint(t);
        }
      }
      if (ring) {   // Backups/4:4868-4878, then xPatternSearchFast's reads (4343-4359)
        iStartX = t.iBestX;
        iStartY = t.iBestY;
        const size_t index_ref = array_e.size();
        tz.square(t, iStartX, iStartY, 1);
        tz.square2(t, iStartX, iStartY, 2);
        long C = array_e[0];
        for (size_t k = 1; k <= index_ref - 1; k++)
          if (array_e[k] < C) C = array_e[k];
        for (int k = 0; k < 8; k++)
          nn_in[(size_t)9 * i + k] = index_ref + k < array_e.size() ? (uint32_t)array_e[index_ref + k] : 0u;
        nn_in[(size_t)9 * i + 8] = (uint32_t)C;
      }
    }
    j.mv_x = (int16_t)t.iBestX;
    j.mv_y = (int16_t)t.iBestY;
    if (sad) sad[i] = t.uiBestSad - s.rd.getCostOfVectorWithPredictor(t.iBestX, t.iBestY);
  }
  return 0;
}
