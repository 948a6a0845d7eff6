// fme_hm.cpp — the TEncSearch-shaped C++ adapter and CTU-row batcher (include/fme_hm.hpp).
// Pure host code over the C-ABI; every computation runs in libfme_amd.so's HIP kernels.
#include "fme_hm.hpp"

#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace fme_hm {

namespace {

void check(int rc, const char* what) {
  if (rc != FME_OK) throw Error(rc, std::string(what) + ": " + fme_last_error());
}

// Directory of the loaded libfme_amd.so (its weights/ directory sits beside it).
std::string library_dir() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&fme_create), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    const size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s);
  }
  return ".";
}

int weight_set(int qp) { return (qp == 27 || qp == 32 || qp == 37) ? qp : 22; }  // TEncSearch.cpp:472/625/775/925

}  // namespace

std::vector<float> loadWeights(const std::string& dir_in, int qp) {
  std::string dir = dir_in;
  if (dir.empty()) {
    const char* e = getenv("FME_WEIGHTS_DIR");
    dir = e ? std::string(e) : library_dir() + "/weights";
  }
  const std::string path = dir + "/nn2_qp" + std::to_string(weight_set(qp)) + ".bin";
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw Error(FME_E_INVALID, "cannot open " + path);
  std::vector<double> d(FME_NN_PARAMS + 1);
  const size_t got = fread(d.data(), sizeof(double), d.size(), f);
  fclose(f);
  if (got != (size_t)FME_NN_PARAMS) throw Error(FME_E_INVALID, path + ": wrong parameter count");
  // the reference's initialisers are double literals assigned to float arrays
  std::vector<float> w(FME_NN_PARAMS);
  for (int i = 0; i < FME_NN_PARAMS; i++) w[i] = (float)d[i];
  return w;
}

// ---- FracSearch --------------------------------------------------------------------------

FracSearch::FracSearch(const SearchConfig& cfg) : cfg_(cfg) {
  fme_config c{};
  c.bit_depth = 8;
  c.use_hadamard = cfg.useHadamardME ? 1 : 0;
  c.nn_mode = cfg.nnMode;
  c.qp = cfg.qp;
  c.fast_inter_mode = cfg.fastInterMode;
  c.max_jobs = cfg.maxJobs;
  check(fme_create(cfg.device, &c, &ctx_), "fme_create");
  if (cfg.nnMode) {
    const std::vector<float> w = loadWeights(cfg.weightsDir, cfg.qp);
    check(fme_load_nn_weights(ctx_, w.data(), (int)w.size()), "fme_load_nn_weights");
  }
}

FracSearch::~FracSearch() {
  if (ctx_) fme_destroy(ctx_);
}

void FracSearch::setLambda(double lambda) { mlambda_ = 65536.0 * std::sqrt(lambda); }  // TComRdCost.cpp:104-117

void FracSearch::setPredictor(const Mv& mvp) { mvp_ = mvp; }

void FracSearch::xPatternSearchFracDIF(bool lossless, const Pel* key, int keyStride, int width,
                                       int height, const Pel* refY, int refStride,
                                       const Mv* mvInt, Mv& mvHalf, Mv& mvQter,
                                       Distortion& cost) {
  int16_t h[2], q[2];
  uint32_t c = 0;
  std::lock_guard<std::mutex> lk(mu_);
  check(fme_frac_dif_single(ctx_, lossless ? 1 : 0, key, keyStride, width, height, refY, refStride,
                            mvInt->hor, mvInt->ver, mvp_.hor, mvp_.ver, mlambda_, h, q, &c),
        "xPatternSearchFracDIF");
  mvHalf = Mv(h[0], h[1]);
  mvQter = Mv(q[0], q[1]);
  cost = c;
}

int FracSearch::NN_pred(const uint32_t arrayE[8], uint32_t C, int puHeight, int puWidth,
                        int& mvxHalf, int& mvxQrter, int& mvyHalf, int& mvyQrter) {
  int cls = 0;
  int16_t out4[4];
  std::lock_guard<std::mutex> lk(mu_);
  check(fme_nn_pred_single(ctx_, arrayE, C, puHeight, puWidth, &cls, out4), "NN_pred");
  mvxHalf = out4[0];
  mvxQrter = out4[1];
  mvyHalf = out4[2];
  mvyQrter = out4[3];
  return cls;
}

void FracSearch::setPicture(int id, const Pel* plane, int stride, int width, int height) {
  std::lock_guard<std::mutex> lk(mu_);
  stage_.resize((size_t)width * height);
  for (int y = 0; y < height; y++) {
    const Pel* s = plane + (ptrdiff_t)y * stride;
    uint8_t* d = stage_.data() + (size_t)y * width;
    for (int x = 0; x < width; x++) {
      const int v = s[x];
      if (v < 0 || v > 255) throw Error(FME_E_UNSUPPORTED, "setPicture: sample outside 8-bit range");
      d[x] = (uint8_t)v;
    }
  }
  check(fme_set_picture(ctx_, id, stage_.data(), width, width, height, nullptr), "fme_set_picture");
}

void FracSearch::setPicture8(int id, const uint8_t* plane, int stride, int width, int height) {
  std::lock_guard<std::mutex> lk(mu_);
  check(fme_set_picture(ctx_, id, plane, stride, width, height, nullptr), "fme_set_picture");
}

void FracSearch::setLambdaSlot(int lambdaId, double lambda) {
  std::lock_guard<std::mutex> lk(mu_);
  check(fme_set_lambda(ctx_, lambdaId, lambda), "fme_set_lambda");
}

// ---- MotionCompensator ---------------------------------------------------------------------

void MotionCompensator::setPictureYuv(int id, const Pel* y, int ys, const Pel* cb, const Pel* cr, int cs, int width,
                                      int height) {
  const int cw = width / 2, ch = height / 2;
  stage_.resize((size_t)width * height + 2 * (size_t)cw * ch);
  auto to8 = [&](const Pel* src, int stride, int w, int h, uint8_t* dst) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        const int v = src[(ptrdiff_t)r * stride + c];
        if (v < 0 || v > 255) throw Error(FME_E_UNSUPPORTED, "setPictureYuv: sample outside 8-bit range");
        dst[(size_t)r * w + c] = (uint8_t)v;
      }
  };
  uint8_t* dy = stage_.data();
  uint8_t* dcb = dy + (size_t)width * height;
  uint8_t* dcr = dcb + (size_t)cw * ch;
  to8(y, ys, width, height, dy);
  to8(cb, cs, cw, ch, dcb);
  to8(cr, cs, cw, ch, dcr);
  setPictureYuv8(id, dy, width, dcb, dcr, cw, width, height);
}

void MotionCompensator::setPictureYuv8(int id, const uint8_t* y, int ys, const uint8_t* cb, const uint8_t* cr, int cs,
                                       int width, int height) {
  std::lock_guard<std::mutex> lk(search_.mutex());
  check(fme_set_picture(search_.ctx(), id, y, ys, width, height, nullptr), "fme_set_picture");
  check(fme_set_picture_chroma(search_.ctx(), id, cb, cr, cs, nullptr), "fme_set_picture_chroma");
}

void MotionCompensator::setWp(int list, int id, const int weight[3], const int offset[3], const int log2Denom[3]) {
  fme_wp_param p[3];
  for (int c = 0; c < 3; c++) p[c] = fme_wp_param{(int16_t)weight[c], (int16_t)offset[c], (uint8_t)log2Denom[c], {0, 0, 0}};
  std::lock_guard<std::mutex> lk(search_.mutex());
  check(fme_set_wp(search_.ctx(), list, id, p), "fme_set_wp");
}

void MotionCompensator::add(int x, int y, int w, int h, int cuX, int cuY, int refIdL0, const Mv& mvL0, int refIdL1,
                            const Mv& mvL1, bool weighted) {
  fme_mc_job j = {};
  if (weighted) j.flags |= FME_MC_WP;
  j.x = (uint16_t)x;
  j.y = (uint16_t)y;
  j.w = (uint8_t)w;
  j.h = (uint8_t)h;
  j.cu_x = (uint16_t)cuX;
  j.cu_y = (uint16_t)cuY;
  if (refIdL0 >= 0) {
    j.flags |= FME_MC_L0;
    j.ref_id[0] = (uint8_t)refIdL0;
    j.mv[0][0] = (int16_t)mvL0.hor;
    j.mv[0][1] = (int16_t)mvL0.ver;
  }
  if (refIdL1 >= 0) {
    j.flags |= FME_MC_L1;
    j.ref_id[1] = (uint8_t)refIdL1;
    j.mv[1][0] = (int16_t)mvL1.hor;
    j.mv[1][1] = (int16_t)mvL1.ver;
  }
  jobs_.push_back(j);
}

void MotionCompensator::run(uint8_t* y, int ys, uint8_t* cb, uint8_t* cr, int cs, int width, int height) {
  std::lock_guard<std::mutex> lk(search_.mutex());
  check(fme_motion_compensate(search_.ctx(), jobs_.data(), (int)jobs_.size(), y, ys, cb, cr, cs, width, height,
                              nullptr),
        "fme_motion_compensate");
  jobs_.clear();
}

// ---- InterSearchP -------------------------------------------------------------------------

int InterSearchP::add(const fme_pu_req& req) {
  reqs_.push_back(req);
  return (int)reqs_.size() - 1;
}

std::vector<fme_pu_res> InterSearchP::run() {
  std::vector<fme_pu_res> res(reqs_.size());
  std::lock_guard<std::mutex> lk(search_.mutex());
  if (!reqs_.empty())
    check(fme_pred_inter_p(search_.ctx(), reqs_.data(), res.data(), (int)reqs_.size(), nullptr), "fme_pred_inter_p");
  reqs_.clear();
  return res;
}

void InterSearchP::reset() {
  std::lock_guard<std::mutex> lk(search_.mutex());
  check(fme_pred_inter_reset(search_.ctx()), "fme_pred_inter_reset");
}

// ---- InterSearchB -------------------------------------------------------------------------

int InterSearchB::add(const fme_pu_req_b& req) {
  reqs_.push_back(req);
  return (int)reqs_.size() - 1;
}

std::vector<fme_pu_res_b> InterSearchB::run() {
  std::vector<fme_pu_res_b> res(reqs_.size());
  std::lock_guard<std::mutex> lk(search_.mutex());
  if (!reqs_.empty())
    check(fme_pred_inter_b(search_.ctx(), reqs_.data(), res.data(), (int)reqs_.size(), nullptr), "fme_pred_inter_b");
  reqs_.clear();
  return res;
}

void InterSearchB::reset() {
  std::lock_guard<std::mutex> lk(search_.mutex());
  check(fme_pred_inter_reset(search_.ctx()), "fme_pred_inter_reset");
}

// ---- CtuRowBatcher -----------------------------------------------------------------------

CtuRowBatcher::CtuRowBatcher(FracSearch& search, int maxRowsInFlight)
    : search_(search), maxInFlight_(maxRowsInFlight < 1 ? 1 : maxRowsInFlight) {
  thread_ = std::thread(&CtuRowBatcher::worker, this);
}

CtuRowBatcher::~CtuRowBatcher() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  thread_.join();
}

int CtuRowBatcher::add(const fme_job& job) {
  fme_job j = job;
  j.flags &= (uint8_t)~FME_JOB_BIPRED;
  j.key_offset = -1;
  cur_.jobs.push_back(j);
  return (int)cur_.jobs.size() - 1;
}

int CtuRowBatcher::addBiPred(fme_job job, const int16_t* key, int keyStride) {
  job.flags |= FME_JOB_BIPRED;
  job.flags &= (uint8_t)~FME_JOB_EMI;   // bi-pred calls have no TZ/EMI step (A.7-bis)
  job.key_offset = (int32_t)cur_.keys.size();
  for (int y = 0; y < job.h; y++)
    cur_.keys.insert(cur_.keys.end(), key + (ptrdiff_t)y * keyStride, key + (ptrdiff_t)y * keyStride + job.w);
  cur_.jobs.push_back(job);
  return (int)cur_.jobs.size() - 1;
}

CtuRowBatcher::Ticket CtuRowBatcher::submit() {
  std::unique_ptr<Row> r(new Row());
  std::swap(r->jobs, cur_.jobs);
  std::swap(r->keys, cur_.keys);
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return inFlight_ < maxInFlight_; });   // bounded double buffering
  r->ticket = next_++;
  const Ticket t = r->ticket;
  inFlight_++;
  queue_.push_back(std::move(r));
  lk.unlock();
  cv_.notify_all();
  return t;
}

std::vector<fme_result> CtuRowBatcher::wait(Ticket t) {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    for (auto it = done_.begin(); it != done_.end(); ++it) {
      if ((*it)->ticket != t) continue;
      std::unique_ptr<Row> r = std::move(*it);
      done_.erase(it);
      lk.unlock();
      if (r->rc) throw Error(r->rc, r->err);
      return std::move(r->results);
    }
    bool known = running_ == t;
    for (auto& q : queue_) known |= q->ticket == t;
    if (!known) throw Error(FME_E_INVALID, "CtuRowBatcher::wait: unknown or already collected ticket");
    cv_.wait(lk);
  }
}

void CtuRowBatcher::drain() {
  if (!cur_.jobs.empty()) submit();
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return queue_.empty() && inFlight_ == 0; });
}

void CtuRowBatcher::worker() {
  for (;;) {
    std::unique_ptr<Row> r;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
      if (queue_.empty()) return;   // stop requested and nothing left
      r = std::move(queue_.front());
      queue_.pop_front();
      running_ = r->ticket;
    }
    r->results.resize(r->jobs.size());
    {
      // rows run in submission order on the one context: the NN state carries across rows
      std::lock_guard<std::mutex> ctx_lock(search_.mutex());
      fme_ctx* c = search_.ctx();
      int rc = FME_OK;
      if (!r->keys.empty()) rc = fme_set_keys(c, r->keys.data(), r->keys.size(), nullptr);
      if (rc == FME_OK && !r->jobs.empty())
        rc = fme_refine(c, r->jobs.data(), r->results.data(), (int)r->jobs.size(), nullptr);
      if (rc != FME_OK) {
        r->rc = rc;
        r->err = fme_last_error();
      }
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      r->done = true;
      running_ = 0;
      inFlight_--;
      done_.push_back(std::move(r));
    }
    cv_.notify_all();
  }
}

}  // namespace fme_hm
