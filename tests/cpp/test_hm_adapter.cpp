// test_hm_adapter.cpp — GPU test of the C++ TEncSearch-shaped adapter (include/fme_hm.hpp).
//
// Drives fme_hm::CtuRowBatcher the way an encoder would (jobs of one CTU row queued, the row
// submitted, the next row filled while it runs) over a synthetic 416x240 P-frame with 4
// references, uni- and bi-pred jobs, and checks every result bit-exactly against the CPU
// oracle (oracle/fme_oracle.c, test infrastructure) run over the same job sequence.  Also
// checks the single-PU xPatternSearchFracDIF / NN_pred entry points and the error path.
// Exit status 0 = all equal.  Run by tests/test_gpu_parity.py::test_cpp_hm_adapter.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <vector>

#include "../../include/fme_hm.hpp"
#include "../../oracle/fme_oracle.h"

namespace {

const int W = 416, H = 240, CTU = 64, PAD = 80;
const double kLambda[4] = {7.340, 20.196, 14.797, 20.196};   // LDP QP22
const int kSizes[][2] = {{8, 4}, {4, 8}, {8, 8}, {16, 8}, {8, 16}, {16, 16}, {32, 16}, {16, 32},
                         {32, 32}, {64, 32}, {32, 64}, {64, 64}, {4, 16}, {12, 16}, {16, 4},
                         {16, 12}, {8, 32}, {24, 32}, {32, 8}, {32, 24}, {64, 16}, {48, 64}};
const int kNumSizes = sizeof(kSizes) / sizeof(kSizes[0]);

int failures = 0;
#define EXPECT(cond, ...)                 \
  do {                                    \
    if (!(cond)) {                        \
      if (failures < 20) {                \
        fprintf(stderr, "FAIL: " __VA_ARGS__); \
        fprintf(stderr, "\n");            \
      }                                   \
      failures++;                         \
    }                                     \
  } while (0)

std::vector<int16_t> make_picture(int t, uint32_t seed) {
  std::mt19937 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  double a[8], fx[8], fy[8], ph[8];
  for (int i = 0; i < 8; i++) {
    a[i] = 10 + 30 * U(rng);
    fx[i] = 0.01 + 0.19 * U(rng);
    fy[i] = 0.01 + 0.19 * U(rng);
    ph[i] = 6.2831853 * U(rng);
  }
  std::normal_distribution<double> N(0.0, 2.0);
  std::vector<int16_t> p((size_t)W * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      double v = 128;
      for (int i = 0; i < 8; i++) v += a[i] * std::sin(fx[i] * (x + 0.37 * t) + fy[i] * (y + 0.21 * t) + ph[i]) / 3;
      v += N(rng);
      p[(size_t)y * W + x] = (int16_t)std::min(255.0, std::max(0.0, std::round(v)));
    }
  return p;
}

int clip_qpel(int v, int pos, int pic) {   // TComDataCU::clipMv (TComDataCU.cpp:2778-2785)
  const int vmax = (pic + 8 - pos - 1) * 4, vmin = (-64 - 8 - pos + 1) * 4;   // (HM shifts; UB on negatives here)
  return std::min(vmax, std::max(vmin, v));
}
int div4_round(int v) { return (v + 2) >> 2; }   // TComMv::divideByPowerOf2 with rounding

void check_rc(int rc) {
  if (rc != FME_OK) throw fme_hm::Error(rc, fme_last_error());
}

bool same(const fme_result& a, const fme_result& b) {
  return a.mv_int_x == b.mv_int_x && a.mv_int_y == b.mv_int_y && a.mv_x == b.mv_x && a.mv_y == b.mv_y &&
         a.half_x == b.half_x && a.half_y == b.half_y && a.qtr_x == b.qtr_x && a.qtr_y == b.qtr_y &&
         a.frac_cost == b.frac_cost && a.cost == b.cost && a.bits == b.bits && a.c == b.c &&
         a.n_emi == b.n_emi && !memcmp(a.emi, b.emi, sizeof(a.emi)) && a.nn_class == b.nn_class &&
         a.status == b.status;
}

}  // namespace

static int run() {
  using namespace fme_hm;
  std::vector<std::vector<int16_t>> pics;
  for (int i = 0; i < 5; i++) pics.push_back(make_picture(i == 4 ? 0 : 4 - i, 7 + i));

  SearchConfig cfg;
  cfg.qp = 22;
  cfg.maxJobs = 4096;
  FracSearch search(cfg);
  for (int i = 0; i < 5; i++) search.setPicture(i, pics[i].data(), W, W, H);
  for (int l = 0; l < 4; l++) search.setLambdaSlot(l, kLambda[l]);

  // oracle context over the same inputs
  fme_config oc{8, 1, 1, 22, 1, 0};
  std::unique_ptr<orc_ctx> orc(new orc_ctx());
  orc_init(orc.get(), &oc);
  std::vector<std::vector<uint8_t>> pics8(5);
  for (int i = 0; i < 5; i++) {
    pics8[i].assign(pics[i].begin(), pics[i].end());
    orc_set_picture(orc.get(), i, pics8[i].data(), W, W, H);
  }
  for (int l = 0; l < 4; l++) orc_set_lambda(orc.get(), l, kLambda[l]);
  const std::vector<float> wts = loadWeights("", 22);
  orc_load_nn(orc.get(), wts.data());

  // ---- batch path: one row of CTUs at a time ------------------------------------------------
  std::mt19937 rng(1234);
  auto R = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
  CtuRowBatcher batcher(search, 2);
  std::vector<CtuRowBatcher::Ticket> tickets;
  std::vector<std::vector<fme_job>> row_jobs;
  std::vector<std::vector<int16_t>> row_keys;
  const int rows = (H + CTU - 1) / CTU, cols = (W + CTU - 1) / CTU;
  for (int ry = 0; ry < rows; ry++) {
    std::vector<fme_job> jobs;
    std::vector<int16_t> keys;   // oracle copy of the row's key blocks
    for (int cx = 0; cx < cols; cx++) {
      for (int k = 0; k < 60; k++) {
        const int* s = kSizes[R(0, kNumSizes - 1)];
        const int w = s[0], h = s[1];
        const int x0 = cx * CTU, y0 = ry * CTU;
        const int x = std::min(W - w, x0 + 4 * R(0, (CTU - w) / 4)), y = std::min(H - h, y0 + 4 * R(0, (CTU - h) / 4));
        fme_job j{};
        j.x = (uint16_t)(x & ~3);
        j.y = (uint16_t)(y & ~3);
        j.w = (uint8_t)w;
        j.h = (uint8_t)h;
        j.org_id = 4;
        j.ref_id = (uint8_t)R(0, 3);
        j.lambda_id = (uint8_t)R(0, 3);
        j.mvp_x = (int16_t)R(-256, 256);
        j.mvp_y = (int16_t)R(-256, 256);
        const int cpx = clip_qpel(j.mvp_x, j.x, W), cpy = clip_qpel(j.mvp_y, j.y, H);
        j.lt_x = (int16_t)div4_round(clip_qpel(cpx - (64 << 2), j.x, W));
        j.rb_x = (int16_t)div4_round(clip_qpel(cpx + (64 << 2), j.x, W));
        j.lt_y = (int16_t)div4_round(clip_qpel(cpy - (64 << 2), j.y, H));
        j.rb_y = (int16_t)div4_round(clip_qpel(cpy + (64 << 2), j.y, H));
        j.mv_x = (int16_t)std::min<int>(j.rb_x, std::max<int>(j.lt_x, R(-64, 64)));
        j.mv_y = (int16_t)std::min<int>(j.rb_y, std::max<int>(j.lt_y, R(-64, 64)));
        j.bits_in = (uint16_t)R(1, 6);
        j.flags = FME_JOB_EMI;
        j.key_offset = -1;
        if (R(0, 9) == 0) {
          // bi-pred: key = 2*org - pred_other, unclipped (TComYuv::removeHighFreq)
          std::vector<int16_t> key((size_t)w * h);
          const std::vector<int16_t>& org = pics[4];
          const std::vector<int16_t>& oth = pics[R(0, 3)];
          const int ox = std::min(W - w, std::max(0, j.x + R(-3, 3))), oy = std::min(H - h, std::max(0, j.y + R(-3, 3)));
          for (int yy = 0; yy < h; yy++)
            for (int xx = 0; xx < w; xx++)
              key[(size_t)yy * w + xx] = (int16_t)(2 * org[(size_t)(j.y + yy) * W + j.x + xx] - oth[(size_t)(oy + yy) * W + ox + xx]);
          batcher.addBiPred(j, key.data(), w);
          j.flags = FME_JOB_BIPRED;
          j.key_offset = (int32_t)keys.size();
          keys.insert(keys.end(), key.begin(), key.end());
        } else {
          batcher.add(j);
        }
        jobs.push_back(j);
      }
    }
    tickets.push_back(batcher.submit());   // row ry runs while row ry+1 is built
    row_jobs.push_back(jobs);
    row_keys.push_back(keys);
  }
  int total = 0;
  for (int ry = 0; ry < rows; ry++) {
    const std::vector<fme_result> got = batcher.wait(tickets[ry]);
    std::vector<fme_result> want(row_jobs[ry].size());
    orc_set_keys(orc.get(), row_keys[ry].data(), row_keys[ry].size());
    EXPECT(orc_refine(orc.get(), row_jobs[ry].data(), want.data(), (int)want.size()) == 0, "oracle row %d", ry);
    EXPECT(got.size() == want.size(), "row %d size", ry);
    for (size_t i = 0; i < got.size() && i < want.size(); i++)
      EXPECT(same(got[i], want[i]), "row %d job %zu (%dx%d): mv %d,%d vs %d,%d cost %u vs %u", ry, i,
             row_jobs[ry][i].w, row_jobs[ry][i].h, got[i].mv_x, got[i].mv_y, want[i].mv_x, want[i].mv_y,
             got[i].cost, want[i].cost);
    total += (int)got.size();
  }

  // ---- error path: an unsupported PU shape rejects the row, the context stays usable --------
  {
    fme_job bad = row_jobs[0][0];
    bad.w = 6;
    batcher.add(bad);
    const CtuRowBatcher::Ticket t = batcher.submit();
    bool threw = false;
    try {
      batcher.wait(t);
    } catch (const Error& e) {
      threw = e.code() == FME_E_INVALID;
    }
    EXPECT(threw, "invalid row did not throw FME_E_INVALID");
    fme_job ok = row_jobs[0][1];
    if (ok.flags & FME_JOB_BIPRED) ok = row_jobs[0][2];
    batcher.add(ok);
    EXPECT(batcher.wait(batcher.submit()).size() == 1, "row after the error");
  }

  // ---- single-PU entry points ---------------------------------------------------------------
  const int PW = W + 2 * PAD;
  std::vector<std::vector<int16_t>> padded(4, std::vector<int16_t>((size_t)PW * (H + 2 * PAD)));
  for (int r = 0; r < 4; r++)
    for (int y = -PAD; y < H + PAD; y++)
      for (int x = -PAD; x < W + PAD; x++)
        padded[r][(size_t)(y + PAD) * PW + x + PAD] =
            pics[r][(size_t)std::min(H - 1, std::max(0, y)) * W + std::min(W - 1, std::max(0, x))];
  int singles = 0;
  for (size_t i = 0; i < row_jobs[1].size(); i += 7) {
    const fme_job& j = row_jobs[1][i];
    if (j.flags & FME_JOB_BIPRED) continue;
    std::vector<int16_t> key((size_t)j.w * j.h);
    for (int yy = 0; yy < j.h; yy++)
      for (int xx = 0; xx < j.w; xx++) key[(size_t)yy * j.w + xx] = pics[4][(size_t)(j.y + yy) * W + j.x + xx];
    search.setLambda(kLambda[j.lambda_id]);
    search.setPredictor(Mv(j.mvp_x, j.mvp_y));
    Mv mvInt(j.mv_x, j.mv_y), mh, mq;
    Distortion cost = 0;
    const int16_t* refY = padded[j.ref_id].data() + (size_t)(j.y + PAD) * PW + j.x + PAD;
    search.xPatternSearchFracDIF(false, key.data(), j.w, j.w, j.h, refY, PW, &mvInt, mh, mq, cost);
    orc_picture p{pics8[j.ref_id].data(), W, W, H};
    int8_t oh[2], oq[2];
    uint32_t ocost = 0;
    orc_frac_dif(&p, key.data(), j.w, j.x, j.y, j.w, j.h, j.mv_x, j.mv_y, j.mvp_x, j.mvp_y,
                 65536.0 * std::sqrt(kLambda[j.lambda_id]), 1, oh, oq, &ocost);
    EXPECT(mh.hor == oh[0] && mh.ver == oh[1] && mq.hor == oq[0] && mq.ver == oq[1] && cost == ocost,
           "xPatternSearchFracDIF job %zu: (%d,%d)(%d,%d) %u vs (%d,%d)(%d,%d) %u", i, mh.hor, mh.ver,
           mq.hor, mq.ver, cost, oh[0], oh[1], oq[0], oq[1], ocost);
    singles++;
  }
  for (int k = 0; k < 100; k++) {
    uint32_t e[8];
    for (uint32_t& v : e) v = (uint32_t)R(0, 200000);
    const uint32_t C = (uint32_t)R(0, 200000);
    const int* s = kSizes[R(0, kNumSizes - 1)];
    int xh, xq, yh, yq;
    const int cls = search.NN_pred(e, C, s[1], s[0], xh, xq, yh, yq);
    EXPECT(cls == orc_nn_forward(wts.data(), e, C, s[1], s[0], nullptr), "NN_pred %d", k);
    EXPECT(2 * xh + xq == cls % 7 - 3 && 2 * yh + yq == cls / 7 - 3, "NN_pred offsets %d", k);
  }

  // ---- MotionCompensator: one CTU-quadtree partition of the frame, uni + bi, against orc_mc --------
  int mc_pus = 0;
  {
    fme_hm::MotionCompensator mc(search);
    std::vector<std::vector<int16_t>> cbs, crs;
    orc_yuv yuv[FME_MAX_PICTURES] = {};
    std::vector<std::vector<uint8_t>> y8(3), cb8(3), cr8(3);
    for (int i = 0; i < 3; i++) {
      std::vector<int16_t> cb((size_t)(W / 2) * (H / 2)), cr(cb.size());
      for (int y = 0; y < H / 2; y++)
        for (int x = 0; x < W / 2; x++) {   // chroma: subsampled luma of another frame, flipped
          cb[(size_t)y * (W / 2) + x] = pics[(i + 1) % 5][(size_t)(2 * y) * W + 2 * x];
          cr[(size_t)y * (W / 2) + x] = (int16_t)(255 - pics[(i + 2) % 5][(size_t)(2 * y + 1) * W + 2 * x + 1]);
        }
      mc.setPictureYuv(10 + i, pics[i].data(), W, cb.data(), cr.data(), W / 2, W, H);
      y8[i].assign(pics[i].begin(), pics[i].end());
      cb8[i].assign(cb.begin(), cb.end());
      cr8[i].assign(cr.begin(), cr.end());
      yuv[10 + i] = orc_yuv{y8[i].data(), cb8[i].data(), cr8[i].data(), W, W / 2, W, H};
    }
    std::vector<fme_mc_job> jobs;
    std::mt19937 rng(99);
    for (int cy = 0; cy < H; cy += 16)   // 16x16 CUs: 2Nx2N, 2NxN or Nx2N
      for (int cx = 0; cx < W; cx += 16) {
        const int mode = (int)(rng() % 3);
        const int parts = mode == 0 ? 1 : 2;
        for (int p = 0; p < parts; p++) {
          const int pw = mode == 2 ? 8 : 16, ph = mode == 1 ? 8 : 16;
          const int px = cx + (mode == 2 ? 8 * p : 0), py = cy + (mode == 1 ? 8 * p : 0);
          const bool bi = rng() % 3 == 0;
          fme_hm::Mv m0((int)(rng() % 257) - 128, (int)(rng() % 257) - 128), m1((int)(rng() % 257) - 128, (int)(rng() % 257) - 128);
          const int r0 = 10 + (int)(rng() % 3), r1 = 10 + (int)(rng() % 3);
          mc.add(px, py, pw, ph, cx, cy, r0, m0, bi ? r1 : -1, m1);
          fme_mc_job j = {};
          j.x = (uint16_t)px; j.y = (uint16_t)py; j.w = (uint8_t)pw; j.h = (uint8_t)ph;
          j.cu_x = (uint16_t)cx; j.cu_y = (uint16_t)cy;
          j.flags = FME_MC_L0 | (bi ? FME_MC_L1 : 0);
          j.ref_id[0] = (uint8_t)r0; j.ref_id[1] = (uint8_t)(bi ? r1 : 0);
          j.mv[0][0] = (int16_t)m0.hor; j.mv[0][1] = (int16_t)m0.ver;
          if (bi) { j.mv[1][0] = (int16_t)m1.hor; j.mv[1][1] = (int16_t)m1.ver; }
          jobs.push_back(j);
        }
      }
    mc_pus = (int)jobs.size();
    std::vector<uint8_t> gy((size_t)W * H), gcb((size_t)W * H / 4), gcr(gcb.size());
    std::vector<uint8_t> oy(gy.size()), ocb(gcb.size()), ocr(gcb.size());
    mc.run(gy.data(), W, gcb.data(), gcr.data(), W / 2, W, H);
    EXPECT(mc.pending() == 0, "MotionCompensator queue not cleared");
    EXPECT(orc_mc(yuv, jobs.data(), (int)jobs.size(), oy.data(), W, ocb.data(), ocr.data(), W / 2, W, H) == 0,
           "orc_mc rejected the jobs");
    EXPECT(gy == oy, "MotionCompensator luma differs from orc_mc");
    EXPECT(gcb == ocb && gcr == ocr, "MotionCompensator chroma differs from orc_mc");

    // the same PUs with explicit weighted prediction (setWp + weighted add) against orc_mc_wp
    static int wp9[2][FME_MAX_PICTURES][3][3];
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < FME_MAX_PICTURES; i++)
        for (int c = 0; c < 3; c++) { wp9[l][i][c][0] = 1; wp9[l][i][c][1] = 0; wp9[l][i][c][2] = 0; }
    for (int l = 0; l < 2; l++)
      for (int i = 10; i < 13; i++) {
        int w[3], o[3], d[3];
        for (int c = 0; c < 3; c++) {
          d[c] = c ? 5 : 3;
          w[c] = (1 << d[c]) + (int)(rng() % 31) - 15;
          o[c] = (int)(rng() % 101) - 50;
          wp9[l][i][c][0] = w[c]; wp9[l][i][c][1] = o[c]; wp9[l][i][c][2] = d[c];
        }
        mc.setWp(l, i, w, o, d);
      }
    for (fme_mc_job& j : jobs) {
      j.flags |= FME_MC_WP;
      mc.add(j.x, j.y, j.w, j.h, j.cu_x, j.cu_y, j.ref_id[0], fme_hm::Mv(j.mv[0][0], j.mv[0][1]),
             (j.flags & FME_MC_L1) ? j.ref_id[1] : -1, fme_hm::Mv(j.mv[1][0], j.mv[1][1]), true);
    }
    mc.run(gy.data(), W, gcb.data(), gcr.data(), W / 2, W, H);
    EXPECT(orc_mc_wp(yuv, jobs.data(), (int)jobs.size(), &wp9[0][0][0][0], oy.data(), W, ocb.data(), ocr.data(), W / 2,
                     W, H) == 0, "orc_mc_wp rejected the jobs");
    EXPECT(gy == oy, "MotionCompensator weighted luma differs from orc_mc_wp");
    EXPECT(gcb == ocb && gcr == ocr, "MotionCompensator weighted chroma differs from orc_mc_wp");
  }

  // ---- InterSearchP: predInterSearch's P-slice PU / reference loop ----------
  int pi_reqs = 0;
  {
    InterSearchP inter(search);
    inter.reset();
    orc_pred_inter_reset(orc.get());
    check_rc(fme_nn_reset_state(search.ctx()));
    orc_nn_reset(orc.get());
    std::mt19937 rq(7);
    auto Q = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rq); };
    std::vector<fme_pu_req> reqs;
    auto add_cu = [&](int x0, int y0, int s, int depth) {
      const int parts[3][2][4] = {{{0, 0, s, s}, {-1, 0, 0, 0}},
                                  {{0, 0, s, s / 2}, {0, s / 2, s, s / 2}},
                                  {{0, 0, s / 2, s}, {s / 2, 0, s / 2, s}}};
      for (int ps = 0; ps < 3; ps++)
        for (int p = 0; p < 2; p++) {
          if (parts[ps][p][0] < 0) continue;
          fme_pu_req q = {};
          q.x = (uint16_t)(x0 + parts[ps][p][0]); q.y = (uint16_t)(y0 + parts[ps][p][1]);
          q.w = (uint8_t)parts[ps][p][2]; q.h = (uint8_t)parts[ps][p][3];
          q.cu_x = (uint16_t)x0; q.cu_y = (uint16_t)y0;
          q.part_size = (uint8_t)ps;   // FME_PART_2Nx2N, _2NxN, _Nx2N
          q.depth = (uint8_t)depth;
          q.org_id = 4; q.num_refs = 4; q.lambda_id = 0; q.search_range = 64;
          for (int k = 0; k < 4; k++) {
            q.ref_id[k] = (uint8_t)k;
            q.n_cand[k] = (uint8_t)(Q(0, 9) == 0 ? 1 : 2);
            for (int m = 0; m < 2; m++) {
              q.cand[k][m][0] = (int16_t)(4 * (k + 1) * 3 + Q(-24, 24));
              q.cand[k][m][1] = (int16_t)(-4 * (k + 1) * 2 + Q(-24, 24));
            }
          }
          reqs.push_back(q);
          inter.add(q);
        }
    };
    for (int cy = 0; cy + CTU <= H; cy += CTU)
      for (int cx = 0; cx + CTU <= W; cx += CTU) {
        add_cu(cx, cy, 64, 0);
        for (int k = 0; k < 4; k++) add_cu(cx + 32 * (k & 1), cy + 32 * (k >> 1), 32, 1);
      }
    pi_reqs = (int)reqs.size();
    EXPECT(inter.pending() == pi_reqs, "InterSearchP queue size");
    const std::vector<fme_pu_res> got = inter.run();
    std::vector<fme_pu_res> want(reqs.size());
    EXPECT(orc_pred_inter_p(orc.get(), reqs.data(), want.data(), (int)reqs.size()) == 0, "orc_pred_inter_p failed");
    int bad = 0;
    for (size_t i = 0; i < reqs.size(); i++) bad += memcmp(&got[i], &want[i], sizeof(fme_pu_res)) != 0;
    EXPECT(bad == 0, "InterSearchP: %d of %d requests differ from orc_pred_inter_p", bad, pi_reqs);
    EXPECT(inter.pending() == 0, "InterSearchP queue not cleared");
  }

  if (failures) {
    fprintf(stderr, "hm adapter: %d failure(s)\n", failures);
    return 1;
  }
  printf("hm adapter ok: %d PU motion compensations (Y/Cb/Cr) bit-exact\n", mc_pus);
  printf("hm adapter ok: %d predInterSearch PU requests (4 refs) bit-exact\n", pi_reqs);
  printf("hm adapter ok: %d jobs in %d CTU rows, %d single-PU FracDIF calls, 100 NN_pred calls bit-exact\n",
         total, rows, singles);
  return 0;
}

// --time-single: wall time per synchronous single-PU call from C++ (xPatternSearchFracDIF at
// 8x8 / 16x16 / 64x64 and NN_pred), as an HM encoder in drop-in mode would make them; one JSON
// line on stdout (bench.py's drop_in_single_pu leg).
int time_single(int calls) {
  using namespace fme_hm;
  using clk = std::chrono::steady_clock;
  SearchConfig cfg;
  cfg.qp = 22;
  FracSearch search(cfg);
  const int PW = W + 2 * PAD;
  const std::vector<int16_t> pic = make_picture(1, 11), org = make_picture(0, 12);
  std::vector<int16_t> padded((size_t)PW * (H + 2 * PAD));
  for (int y = -PAD; y < H + PAD; y++)
    for (int x = -PAD; x < W + PAD; x++)
      padded[(size_t)(y + PAD) * PW + x + PAD] =
          pic[(size_t)std::min(H - 1, std::max(0, y)) * W + std::min(W - 1, std::max(0, x))];
  std::mt19937 rng(5);
  auto R = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
  search.setLambda(kLambda[0]);
  printf("{");
  const int shapes[3][2] = {{8, 8}, {16, 16}, {64, 64}};
  for (const auto& sh : shapes) {
    const int w = sh[0], h = sh[1];
    std::vector<double> ts;
    for (int i = 0; i < calls; i++) {
      const int x = 4 * R(0, (W - w) / 4), y = 4 * R(0, (H - h) / 4);
      Mv mvInt(R(-8, 8), R(-8, 8)), mh, mq;
      search.setPredictor(Mv(R(-16, 16), R(-16, 16)));
      Distortion cost = 0;
      const int16_t* key = org.data() + (size_t)y * W + x;
      const int16_t* refY = padded.data() + (size_t)(y + PAD) * PW + x + PAD;
      const auto t0 = clk::now();
      search.xPatternSearchFracDIF(false, key, W, w, h, refY, PW, &mvInt, mh, mq, cost);
      ts.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    std::sort(ts.begin() + 1, ts.end());
    printf("\"frac_dif_%dx%d_us\": %.2f, ", w, h, ts[1 + (ts.size() - 1) / 2]);
  }
  std::vector<double> ts;
  for (int i = 0; i < calls; i++) {
    uint32_t e[8];
    for (uint32_t& v : e) v = (uint32_t)R(0, 5000);
    int xh, xq, yh, yq;
    const auto t0 = clk::now();
    search.NN_pred(e, (uint32_t)R(0, 5000), 8, 8, xh, xq, yh, yq);
    ts.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  std::sort(ts.begin() + 1, ts.end());
  printf("\"nn_pred_us\": %.2f, \"calls\": %d}\n", ts[1 + (ts.size() - 1) / 2], calls);
  return 0;
}

int main(int argc, char** argv) {
  try {
    if (argc > 1 && !strcmp(argv[1], "--time-single")) return time_single(argc > 2 ? atoi(argv[2]) : 300);
    return run();
  } catch (const fme_hm::Error& e) {
    fprintf(stderr, "hm adapter: error %d: %s\n", e.code(), e.what());
    return 2;
  }
}
