// fme_api.cpp — host runtime behind the C-ABI of include/fme.h.
//
// A context owns one device's copies of the pictures, the motion-lambda table, the bi-pred key
// blocks, the NN weights, the NN_pred carried state (array_e slots, C, PUHeight, PUWidth,
// TEncSearch.cpp:55-57) and the per-batch work buffers.  A batch is
//   classify -> [one 100-byte D2H: class histogram] -> scatter -> search -> scan -> nn_tail
// on the caller's stream.  Errors are returned as FME_E_* codes; the text is kept per thread.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "fme_device.h"

using namespace fme;

namespace {

thread_local std::string g_last_error = "";

// counts buffer: 25 class counts (+ invalid), 24 scatter cursors, 8 lane tile-queue heads; zeroed per
// batch by one
// hipMemsetAsync, padded to 64 words (256 B) so the runtime issues one fill kernel, not two
constexpr int kCountWords = 64;
static_assert(2 * kNumClasses + 1 + 8 <= kCountWords, "counter block");

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(_e == hipErrorOutOfMemory ? FME_E_NOMEM : FME_E_DEVICE, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(_e), __FILE__, __LINE__);                        \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host memory, grown on demand: the producers' transfer buffers (full-rate DMA, and no page
// faults on the buffers of the next call).
template <typename T>
struct HostBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n + n / 4, 1);   // headroom: fewer regrowths
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// f(lo, hi) over [0, n) in up to 8 host threads (the producers' per-request loops; the caller's
// thread takes the first slice).
template <typename F>
void par_for(int n, F&& f) {
  const unsigned hc = std::thread::hardware_concurrency();
  const int nt = n < 32768 ? 1 : (int)std::min<unsigned>(8u, hc ? hc : 1u);
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)nt - 1);
  for (int t = 1; t < nt; t++)
    th.emplace_back([&f, n, nt, t] { f((int)((long long)n * t / nt), (int)((long long)n * (t + 1) / nt)); });
  f(0, (int)((long long)n / nt));
  for (auto& x : th) x.join();
}

}  // namespace

// The deeper nets' single NN_pred call (k_nn_deep_single): class and completion word.
struct SingleStage {
  int32_t nn_out[4];
  uint32_t flag;                // completion word (call sequence number)
};

struct fme_ctx {
  int device = 0;
  fme_config cfg{};
  PicDesc pics[FME_MAX_PICTURES]{};
  bool pic_owned[FME_MAX_PICTURES]{};
  size_t pic_bytes[FME_MAX_PICTURES]{};
  double mlambda[FME_MAX_LAMBDAS]{};
  bool lambda_set[FME_MAX_LAMBDAS]{};
  bool tables_dirty = true;

  DevBuf<PicDesc> d_pics;
  DevBuf<double> d_mlambda;
  // the tables' upload ring (sync_tables): pinned, device-mapped slots, each guarded by the event of
  // the launch that reads it
  static constexpr int kTabSlots = 16;
  TablesSlot* h_tab = nullptr;
  TablesSlot* h_tab_dev = nullptr;
  hipEvent_t tab_ev[kTabSlots] = {};
  bool tab_used[kTabSlots] = {};
  int tab_next = 0;
  DevBuf<int16_t> d_keys;
  size_t n_keys = 0;
  DevBuf<float> d_nn;         // packed layout (nn_pack, kNnPkFloats)
  bool nn_loaded = false;
  // nn_mode 2: a generic net (fme_load_nn_net), packed by nn_deep_pack
  fme_nn_net net{};
  DevBuf<uint8_t> d_net;
  bool net_loaded = false;
  int nn_engine = FME_NN_ENGINE_EXACT;
  float* nn_margin = nullptr;  // caller-owned device array (fme_set_nn_margin_output)
  int nn_margin_cap = 0;       // its length
  void* nn_logits = nullptr;   // caller-owned device array (fme_set_nn_logit_output), 49 per job
  int nn_logits_cap = 0;       // its length in jobs
  const uint32_t* nn_in = nullptr;   // caller-owned NN input rows of FME_JOB_NN_IN jobs (fme_set_nn_inputs)
  int nn_in_cap = 0;                 // its length in rows

  DevBuf<fme_job> d_jobs;      // staging for fme_refine (host arrays)
  DevBuf<fme_result> d_res;
  DevBuf<fme_mv_result> d_mv;   // staging for fme_refine_mv
  DevBuf<fme_job> d_pk_jobs;    // fme_refine*_packed_device: the unpacked batch
  DevBuf<uint8_t> cls;
  DevBuf<int32_t> perm;
  DevBuf<fme_job> sjobs;
  DevBuf<int32_t> counts;      // 25 counts, 24 cursors, 24 tile-queue heads: one memset
  DevBuf<int32_t> blk_agg;
  DevBuf<int32_t> blk_prefix;
  DevBuf<uint32_t> nn_state;   // 2 x 12 words
  int state_cur = 0;
  bool state_pending = false;   // reset / set_state not yet applied (next batch, stream order)
  uint32_t pending_state[12] = {};
  DevBuf<Schedule> d_sched;     // built by k_schedule each batch
  SchedParams sched_p{};
  int32_t* h_counts = nullptr; // pinned

  // motion compensation: owned chroma planes (cb then cr, one allocation per slot), staging
  uint8_t* chroma_owned[FME_MAX_PICTURES]{};
  size_t chroma_bytes[FME_MAX_PICTURES]{};
  DevBuf<fme_mc_job> d_mc_jobs;
  DevBuf<uint8_t> d_mc_planes;
  DevBuf<int32_t> d_mc_invalid;
  // weighted prediction (fme_set_wp): [list][picture][Y, Cb, Cr], uploaded before a launch when changed
  fme_wp_param h_wp[2][FME_MAX_PICTURES][3] = {};
  bool wp_init = false, wp_dirty = true;
  DevBuf<fme_wp_param> d_mc_wp;
  hipEvent_t ev_mc[2] = {nullptr, nullptr};
  bool mc_timed = false;
  // integer search: staging for the host entry point, timing events
  DevBuf<fme_tz_ext> d_tz_ext;
  DevBuf<uint32_t> d_tz_sad;
  DevBuf<uint32_t> d_tz_nn_in;   // staging of fme_integer_search_ring's NN input rows
  hipEvent_t ev_tz[2] = {nullptr, nullptr};
  bool tz_timed = false;
  // phase wall times of the last producer call (fme_pred_inter_phases)
  double pi_ms[FME_PI_PHASES] = {};
  // predInterSearch producer: m_integerMv2Nx2N[REF_PIC_LIST_0][k] (TEncSearch.h:118), AMVP staging
  int16_t int_mv_2n[2][FME_MAX_REFS][2] = {};   // m_integerMv2Nx2N[list][ref]
  DevBuf<AmvpTask> d_amvp;
  DevBuf<int16_t> d_tz_emi;   // [n][2] post-EMI integer MVs (producer levels)
  DevBuf<uint32_t> d_amvp_sad;
  DevBuf<BiKeyTask> d_bikey;
  DevBuf<int32_t> d_key_invalid;  // invalid requests of the last fme_build_bipred_keys_device
  DevBuf<int32_t> d_ch_i32;     // k_tz_level: psrc
  DevBuf<int32_t> d_tzp;        // staged integer search: 8 words (nseg), then cnt / cursor / off / seg (TzPairs)
  DevBuf<int32_t> d_tzp_perm;   // [n] jobs grouped by (kernel, reference, CTU)
  // fme_pred_inter_p scratch, kept across calls: pinned transfer buffers, host arrays, the
  // level-ordered device copies of the jobs
  HostBuf<AmvpTask> h_pi_tasks;
  HostBuf<uint32_t> h_pi_tsad;
  HostBuf<fme_job> h_pi_jobs;
  HostBuf<fme_tz_ext> h_pi_ext;
  HostBuf<int32_t> h_pi_idx;      // [2 nj]: level order, then its inverse
  HostBuf<int32_t> h_pi_psrc;
  HostBuf<fme_mv_result> h_pi_mv;
  HostBuf<fme_result> h_pi_last;  // the full records of the last 2Nx2N request
  HostBuf<fme_result> h_pi_ures;  // fme_pred_inter_b: the uni-pred jobs' records
  HostBuf<fme_job> h_pi_seq;      // fme_pred_inter_b: one round's jobs in call order
  HostBuf<fme_mv_result> h_pi_rs; // fme_pred_inter_b: their results
  HostBuf<uint32_t> h_pi_rows;    // fme_pred_inter_b: the bi jobs' NN input rows
  std::vector<int> pi_base, pi_task, pi_level, pi_src, pi_lvl, pi_start, pi_byarea;
  std::vector<int32_t> pi_off, pi_fill;
  std::vector<uint8_t> pi_amvp_idx;
  DevBuf<fme_job> d_pi_jobs;      // level order
  DevBuf<fme_tz_ext> d_pi_ext;
  DevBuf<int32_t> d_pi_idx;

  // The deeper nets' single NN_pred: inputs in the kernel argument, class and completion word in
  // pinned, device-mapped host memory.
  struct SingleStage* stage = nullptr;
  uint8_t* stage_dev = nullptr;
  hipStream_t single_stream = nullptr;
  uint32_t single_seq = 0;
  // The single-call server (fme_server.hip) behind fme_frac_dif_single and the master net's
  // fme_nn_pred_single: its mailbox in pinned, device-mapped host memory, its own stream.
  SrvBox* box = nullptr;
  SrvBox* box_dev = nullptr;
  hipStream_t srv_stream = nullptr;
  bool srv_running = false;
  bool srv_orphan = false;      // a wait on the instance timed out: it may still run on srv_stream
  // the streams this context's batches were issued on (note_stream): a buffer that a queued launch
  // may still read is regrown only after those streams have drained, not the whole device
  static constexpr int kMaxStreams = 8;
  hipStream_t used_streams[kMaxStreams] = {};
  int n_used_streams = 0;
  bool used_overflow = false;   // more streams than tracked: fall back to a device synchronisation
  uint32_t srv_epoch = 0;       // of the instance launched last
  uint32_t srv_done = 0;        // sequence number of the last completed call
  uint32_t srv_nn_gen = 0;      // weight generation the running instance copied to LDS
  uint32_t nn_gen = 0;          // bumped by fme_load_nn_weights
  uint64_t srv_khz = 100000;    // wall-clock rate (s_memrealtime)
  bool srv_marks = false;       // the server records its phase checkpoints (fme_single_last_device_us)

  // Profiling: a ring of event sets, one per profiled batch, read once the batch has finished
  // (harvest_events), so profiling a run of batches adds no synchronisation.  Per set: 0 start,
  // 1 classify end, 2 schedule end = scatter begin, 3 scatter end, 4 main search end, 5 search
  // end, 6 batch end.
  static constexpr int kEv = 9;
  static constexpr int kEvSets = 32;
  bool profiling = false;
  bool events_made = false;
  hipEvent_t ev[kEvSets][kEv] = {};
  long long ev_head = 0;        // sets recorded
  long long ev_tail = 0;        // sets harvested
  bool timed = false;
  hipEvent_t ev_done = nullptr; // end of the last batch (fme_refine_status)
  hipEvent_t ev_search = nullptr; // caller's event, recorded before each search launch (fme_set_search_event)
  int search_reserve = 0;         // resident search workgroups left free (fme_set_search_reserve)
  fme_ctx* single10 = nullptr;    // bit depth 10: the private one-job context of fme_frac_dif_single
  hipStream_t single10_stream = nullptr;
  bool main10_px = false;         // bit depth 10: the pixel kernel instead of the lane kernel
                                  // (environment FME_MAIN10_SEARCH=px, an A/B switch)
  bool batch_issued = false;
  float last_ms[FME_NUM_TIMINGS] = {};
  double acc_ms[FME_NUM_TIMINGS] = {};
  int acc_batches = 0;

  // auxiliary streams of the integer search (created on first use)
  hipStream_t aux = nullptr;
  hipStream_t aux2 = nullptr;
  hipEvent_t ev_join2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

namespace fme {
size_t nn_deep_packed_bytes(const fme_nn_net& n);
void nn_deep_pack(const fme_nn_net& n, const double* params, void* out);
hipError_t launch_nn_deep_tail(const fme_nn_net& n, const void* packed, float* margin, void* logits, const BatchArgs& a,
                               const WorkBufs& w, int state_in, int engine, hipStream_t s);
hipError_t launch_nn_deep_single(const fme_nn_net& n, const void* packed, const NnIn11& in11, int32_t* out,
                                 uint32_t* flag, uint32_t seq, hipStream_t s);
}

extern "C" {

int fme_abi_version(void) { return FME_ABI_VERSION; }

const char* fme_last_error(void) { return g_last_error.c_str(); }

int fme_create(int device, const fme_config* cfg, fme_ctx** out_ctx) {
  if (!cfg || !out_ctx) return fail(FME_E_INVALID, "fme_create: null argument");
  *out_ctx = nullptr;
  if (cfg->bit_depth != 8 && cfg->bit_depth != 10)
    return fail(FME_E_UNSUPPORTED, "fme_create: bit_depth %d (8, or 10 for the main10 configurations)", cfg->bit_depth);
  if (cfg->nn_mode < 0 || cfg->nn_mode > 2) return fail(FME_E_INVALID, "fme_create: nn_mode %d", cfg->nn_mode);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(FME_E_INVALID, "fme_create: device %d of %d", device, ndev);
  HIP_TRY(hipSetDevice(device));
  std::unique_ptr<fme_ctx> c(new fme_ctx());
  c->device = device;
  c->cfg = *cfg;
  HIP_TRY(c->d_pics.reserve(FME_MAX_PICTURES));
  HIP_TRY(c->d_mlambda.reserve(FME_MAX_LAMBDAS));
  HIP_TRY(c->d_nn.reserve(kNnPkFloats));
  HIP_TRY(c->counts.reserve(kCountWords));
  HIP_TRY(c->d_sched.reserve(1));
  c->sched_p = sched_params();
  {
    const char* m10 = std::getenv("FME_MAIN10_SEARCH");
    c->main10_px = m10 && std::strcmp(m10, "px") == 0;
  }
  HIP_TRY(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  HIP_TRY(c->nn_state.reserve(24));
  HIP_TRY(hipMemset(c->nn_state.p, 0, 24 * sizeof(uint32_t)));
  HIP_TRY(c->d_key_invalid.reserve(1));
  HIP_TRY(hipMemset(c->d_key_invalid.p, 0, sizeof(int32_t)));
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_counts), kCountWords * sizeof(int32_t), hipHostMallocDefault));
  if (cfg->max_jobs > 0) {
    const size_t n = (size_t)cfg->max_jobs;
    const size_t nb = (n + kJobsPerScanBlock - 1) / kJobsPerScanBlock;
    HIP_TRY(c->cls.reserve(n));
    HIP_TRY(c->perm.reserve(n));
    if (FME_SJOBS) HIP_TRY(c->sjobs.reserve(n));
    HIP_TRY(c->blk_agg.reserve(nb * 9));
    HIP_TRY(c->blk_prefix.reserve(nb * 9));
  }
  *out_ctx = c.release();
  return FME_OK;
}

}  // extern "C"
static int srv_stop(fme_ctx* c);
// Grows the bi-pred key buffer to n elements.  Growing frees the old buffer, which batches queued on
// any stream (the caller's, the integer search's auxiliary streams, another caller stream) may still
// read: every stream of the device is drained first, and only when the buffer really grows.
// Remember a stream this context issued work on (reads of its buffers may be queued there).
static void note_stream(fme_ctx* c, hipStream_t s) {
  for (int i = 0; i < c->n_used_streams; i++)
    if (c->used_streams[i] == s) return;
  if (c->n_used_streams < fme_ctx::kMaxStreams) c->used_streams[c->n_used_streams++] = s;
  else c->used_overflow = true;
}
// Wait for every launch of this context (its tracked streams; the device only if it used more),
// leaving other contexts' work alone.
static int drain_ctx(fme_ctx* c) {
  if (c->used_overflow) {
    HIP_TRY(hipDeviceSynchronize());
  } else {
    for (int i = 0; i < c->n_used_streams; i++) HIP_TRY(hipStreamSynchronize(c->used_streams[i]));
  }
  return FME_OK;
}
static int grow_keys(fme_ctx* c, size_t n) {
  if (n <= c->d_keys.cap) return FME_OK;
  int rc = drain_ctx(c);   // no queued launch of this context still reads the old key buffer
  if (rc) return rc;
  HIP_TRY(c->d_keys.reserve(n));
  return FME_OK;
}
extern "C" {
int fme_destroy(fme_ctx* c) {
  if (!c) return FME_OK;
  (void)hipSetDevice(c->device);
  (void)srv_stop(c);
  if (c->single10) (void)fme_destroy(c->single10);
  if (c->single10_stream) (void)hipStreamDestroy(c->single10_stream);
  (void)hipDeviceSynchronize();
  for (int i = 0; i < FME_MAX_PICTURES; i++)
    if (c->pic_owned[i] && c->pics[i].luma) (void)hipFree(const_cast<uint8_t*>(c->pics[i].luma));
  for (int i = 0; i < FME_MAX_PICTURES; i++)
    if (c->chroma_owned[i]) (void)hipFree(c->chroma_owned[i]);
  c->d_mc_jobs.release(); c->d_mc_planes.release(); c->d_mc_invalid.release(); c->d_mc_wp.release();
  c->d_tz_ext.release(); c->d_tz_sad.release(); c->d_tz_nn_in.release();
  c->d_amvp.release(); c->d_amvp_sad.release(); c->d_bikey.release(); c->d_key_invalid.release(); c->d_ch_i32.release(); c->d_tz_emi.release();
  c->h_pi_tasks.release(); c->h_pi_tsad.release(); c->h_pi_jobs.release(); c->h_pi_ext.release();
  c->h_pi_idx.release(); c->h_pi_psrc.release(); c->h_pi_mv.release(); c->h_pi_last.release();
  c->h_pi_ures.release(); c->h_pi_seq.release(); c->h_pi_rs.release(); c->h_pi_rows.release();
  c->d_pi_jobs.release(); c->d_pi_ext.release(); c->d_pi_idx.release();
  for (auto& e : c->ev_tz)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ev_mc)
    if (e) (void)hipEventDestroy(e);
  c->d_pics.release(); c->d_mlambda.release(); c->d_keys.release(); c->d_nn.release(); c->d_net.release();
  c->d_jobs.release(); c->d_res.release(); c->d_mv.release(); c->d_pk_jobs.release(); c->cls.release(); c->perm.release(); c->sjobs.release();
  c->counts.release(); c->blk_agg.release(); c->blk_prefix.release(); c->nn_state.release();
  c->d_sched.release();
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->stage) (void)hipHostFree(c->stage);
  if (c->single_stream) (void)hipStreamDestroy(c->single_stream);
  if (c->box) (void)hipHostFree(c->box);
  if (c->srv_stream) (void)hipStreamDestroy(c->srv_stream);
  if (c->h_counts) (void)hipHostFree(c->h_counts);
  if (c->h_tab) (void)hipHostFree(c->h_tab);
  for (auto& e : c->tab_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& set : c->ev)
    for (auto& e : set)
      if (e) (void)hipEventDestroy(e);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join2) (void)hipEventDestroy(c->ev_join2);
  if (c->aux2) (void)hipStreamDestroy(c->aux2);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  delete c;
  return FME_OK;
}

// A new luma plane with other dimensions invalidates the slot's chroma planes.
static void keep_chroma(fme_ctx* c, int id, int width, int height) {
  const PicDesc& o = c->pics[id];
  if (o.luma && o.width == width && o.height == height) return;
  if (c->chroma_owned[id]) (void)hipFree(c->chroma_owned[id]);
  c->chroma_owned[id] = nullptr;
  c->chroma_bytes[id] = 0;
  c->pics[id].cb = c->pics[id].cr = nullptr;
  c->pics[id].cstride = 0;
}

int fme_set_picture(fme_ctx* c, int id, const uint8_t* luma, int stride, int width, int height, void* stream) {
  if (!c || !luma) return fail(FME_E_INVALID, "fme_set_picture: null argument");
  if (id < 0 || id >= FME_MAX_PICTURES) return fail(FME_E_INVALID, "fme_set_picture: id %d", id);
  if (width <= 0 || height <= 0 || stride < width || width > 65535 || height > 65535)
    return fail(FME_E_INVALID, "fme_set_picture: %dx%d stride %d", width, height, stride);
  HIP_TRY(hipSetDevice(c->device));
  const size_t bps = c->cfg.bit_depth > 8 ? 2 : 1;   // bytes per sample (10-bit: uint16 samples)
  const size_t bytes = (size_t)width * height * bps;
  uint8_t* dst = c->pic_owned[id] ? const_cast<uint8_t*>(c->pics[id].luma) : nullptr;
  if (!dst || c->pic_bytes[id] < bytes) {
    if (dst) HIP_TRY(hipFree(dst));
    dst = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dst), bytes));
    c->pic_bytes[id] = bytes;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(hipMemcpy2DAsync(dst, width * bps, luma, stride * bps, width * bps, height, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));  // the caller may free its host plane on return
  keep_chroma(c, id, width, height);
  c->pics[id] = PicDesc{dst, width, width, height, c->pics[id].cb, c->pics[id].cr, c->pics[id].cstride, 0};
  c->pic_owned[id] = true;
  c->tables_dirty = true;
  return FME_OK;
}

int fme_bind_picture_device(fme_ctx* c, int id, const uint8_t* d_luma, int stride, int width, int height) {
  if (!c || !d_luma) return fail(FME_E_INVALID, "fme_bind_picture_device: null argument");
  if (id < 0 || id >= FME_MAX_PICTURES) return fail(FME_E_INVALID, "fme_bind_picture_device: id %d", id);
  if (width <= 0 || height <= 0 || stride < width) return fail(FME_E_INVALID, "fme_bind_picture_device: geometry");
  HIP_TRY(hipSetDevice(c->device));
  if (c->pic_owned[id] && c->pics[id].luma) HIP_TRY(hipFree(const_cast<uint8_t*>(c->pics[id].luma)));
  c->pic_owned[id] = false;
  c->pic_bytes[id] = 0;
  keep_chroma(c, id, width, height);
  c->pics[id] = PicDesc{d_luma, stride, width, height, c->pics[id].cb, c->pics[id].cr, c->pics[id].cstride, 0};
  c->tables_dirty = true;
  return FME_OK;
}

int fme_set_picture_chroma(fme_ctx* c, int id, const uint8_t* cb, const uint8_t* cr, int stride, void* stream) {
  if (!c || !cb || !cr) return fail(FME_E_INVALID, "fme_set_picture_chroma: null argument");
  if (id < 0 || id >= FME_MAX_PICTURES) return fail(FME_E_INVALID, "fme_set_picture_chroma: id %d", id);
  if (!c->pics[id].luma) return fail(FME_E_STATE, "fme_set_picture_chroma: picture %d has no luma plane", id);
  const int cw = c->pics[id].width >> 1, ch = c->pics[id].height >> 1;
  if (stride < cw) return fail(FME_E_INVALID, "fme_set_picture_chroma: stride %d < %d", stride, cw);
  HIP_TRY(hipSetDevice(c->device));
  const size_t bps = c->cfg.bit_depth > 8 ? 2 : 1;   // bytes per sample (10-bit: uint16 planes)
  const size_t bytes = 2 * (size_t)cw * ch * bps;
  if (!c->chroma_owned[id] || c->chroma_bytes[id] < bytes) {
    if (c->chroma_owned[id]) HIP_TRY(hipFree(c->chroma_owned[id]));
    c->chroma_owned[id] = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->chroma_owned[id]), bytes));
    c->chroma_bytes[id] = bytes;
  }
  uint8_t* dcb = c->chroma_owned[id];
  uint8_t* dcr = dcb + (size_t)cw * ch * bps;
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(hipMemcpy2DAsync(dcb, cw * bps, cb, stride * bps, cw * bps, ch, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpy2DAsync(dcr, cw * bps, cr, stride * bps, cw * bps, ch, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  c->pics[id].cb = dcb;
  c->pics[id].cr = dcr;
  c->pics[id].cstride = cw;
  c->tables_dirty = true;
  return FME_OK;
}

int fme_bind_picture_chroma_device(fme_ctx* c, int id, const uint8_t* d_cb, const uint8_t* d_cr, int stride) {
  if (!c || !d_cb || !d_cr) return fail(FME_E_INVALID, "fme_bind_picture_chroma_device: null argument");
  if (id < 0 || id >= FME_MAX_PICTURES) return fail(FME_E_INVALID, "fme_bind_picture_chroma_device: id %d", id);
  if (!c->pics[id].luma) return fail(FME_E_STATE, "fme_bind_picture_chroma_device: picture %d has no luma plane", id);
  if (stride < (c->pics[id].width >> 1)) return fail(FME_E_INVALID, "fme_bind_picture_chroma_device: stride %d", stride);
  HIP_TRY(hipSetDevice(c->device));
  if (c->chroma_owned[id]) HIP_TRY(hipFree(c->chroma_owned[id]));
  c->chroma_owned[id] = nullptr;
  c->chroma_bytes[id] = 0;
  c->pics[id].cb = d_cb;
  c->pics[id].cr = d_cr;
  c->pics[id].cstride = stride;
  c->tables_dirty = true;
  return FME_OK;
}

int fme_set_lambda(fme_ctx* c, int id, double lambda) {
  if (!c || id < 0 || id >= FME_MAX_LAMBDAS || !(lambda >= 0.0)) return fail(FME_E_INVALID, "fme_set_lambda: bad argument");
  // TComRdCost::setLambda: m_dLambdaMotionSAD[0] = 65536.0 * sqrt(lambda); selectMotionLambda
  // (true, 0, false) adds iAdd = 0 (TComRdCost.cpp:104-110, TComRdCost.h:159).
  const double sq = std::sqrt(lambda);
  c->mlambda[id] = 65536.0 * sq + 0;
  c->lambda_set[id] = true;
  c->tables_dirty = true;
  return FME_OK;
}

int fme_set_motion_lambda(fme_ctx* c, int id, double ml) {
  if (!c || id < 0 || id >= FME_MAX_LAMBDAS || !(ml >= 0.0)) return fail(FME_E_INVALID, "fme_set_motion_lambda: bad argument");
  c->mlambda[id] = ml;
  c->lambda_set[id] = true;
  c->tables_dirty = true;
  return FME_OK;
}

int fme_set_keys(fme_ctx* c, const int16_t* keys, size_t count, void* stream) {
  if (!c || (!keys && count)) return fail(FME_E_INVALID, "fme_set_keys: null argument");
  HIP_TRY(hipSetDevice(c->device));
  // the upload and the memset below are GPU work: a resident single-call server could hold them up
  // on a hardware queue its stream shares (sync_tables does the same for batches)
  int rc = srv_stop(c);
  if (rc) return rc;
  rc = grow_keys(c, count);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (count) HIP_TRY(hipMemcpyAsync(c->d_keys.p, keys, count * sizeof(int16_t), hipMemcpyHostToDevice, s));
  // fresh host keys: a rejection left by an earlier device build no longer applies (fme.h: rejected
  // "until keys are built again"), in stream order with the upload
  HIP_TRY(hipMemsetAsync(c->d_key_invalid.p, 0, sizeof(int32_t), s));
  HIP_TRY(hipStreamSynchronize(s));
  c->n_keys = count;
  return FME_OK;
}

int fme_load_nn_weights(fme_ctx* c, const float* params, int count) {
  if (!c || !params) return fail(FME_E_INVALID, "fme_load_nn_weights: null argument");
  if (count != FME_NN_PARAMS) return fail(FME_E_INVALID, "fme_load_nn_weights: %d params, expected %d", count, FME_NN_PARAMS);
  HIP_TRY(hipSetDevice(c->device));
  std::vector<float> packed(kNnPkFloats);
  nn_pack(params, packed.data());
  HIP_TRY(hipMemcpy(c->d_nn.p, packed.data(), kNnPkFloats * sizeof(float), hipMemcpyHostToDevice));
  c->nn_loaded = true;
  c->nn_gen++;   // a running server instance holds the old weights in LDS: it is restarted
  return FME_OK;
}

int fme_nn_param_count(const fme_nn_net* n) {
  if (!n) return fail(FME_E_INVALID, "fme_nn_param_count: null descriptor");
  if (n->n_hidden < 1 || n->n_hidden > FME_NN_MAX_HIDDEN)
    return fail(FME_E_INVALID, "fme_nn_param_count: n_hidden %d", n->n_hidden);
  if (n->precision != FME_NN_F32 && n->precision != FME_NN_F64)
    return fail(FME_E_INVALID, "fme_nn_param_count: precision %d", n->precision);
  if (n->embedding < FME_NN_EMB_NONE || n->embedding > FME_NN_EMB_SWAP)
    return fail(FME_E_INVALID, "fme_nn_param_count: embedding %d", n->embedding);
  if (n->out_act != FME_NN_OUT_LINEAR && n->out_act != FME_NN_OUT_SIGMOID)
    return fail(FME_E_INVALID, "fme_nn_param_count: out_act %d", n->out_act);
  if (n->carry_hidden >> n->n_hidden) return fail(FME_E_INVALID, "fme_nn_param_count: carry_hidden 0x%x", n->carry_hidden);
  if (n->input_flags & ~(FME_NN_IN_SLOT_RESET | FME_NN_IN_TZ_RING))
    return fail(FME_E_INVALID, "fme_nn_param_count: input_flags 0x%x", n->input_flags);
  if ((n->input_flags & FME_NN_IN_TZ_RING) && ((n->input_flags & FME_NN_IN_SLOT_RESET) || n->carry_hidden))
    return fail(FME_E_INVALID, "fme_nn_param_count: FME_NN_IN_TZ_RING with FME_NN_IN_SLOT_RESET or carry_hidden");
  int count = n->embedding ? 64 : 0, fan = n->embedding ? 17 : 9;
  for (int l = 0; l < n->n_hidden; l++) {
    const int w = n->width[l];
    if (w < 1 || w > FME_NN_MAX_WIDTH) return fail(FME_E_INVALID, "fme_nn_param_count: width[%d] = %d", l, w);
    count += w * fan + 3 * w;
    fan = w;
  }
  return count + 49 * fan + 49 + 27;
}

int fme_load_nn_net(fme_ctx* c, const fme_nn_net* n, const double* params, int count) {
  if (!c || !n || !params) return fail(FME_E_INVALID, "fme_load_nn_net: null argument");
  const int need = fme_nn_param_count(n);
  if (need < 0) return need;
  if (count != need) return fail(FME_E_INVALID, "fme_load_nn_net: %d params, the descriptor needs %d", count, need);
  if (n->carry_hidden)
    return fail(FME_E_UNSUPPORTED, "fme_load_nn_net: carry_hidden 0x%x (hidden layers carried across calls) is not "
                "supported by the batch engines", n->carry_hidden);
  HIP_TRY(hipSetDevice(c->device));
  const size_t bytes = nn_deep_packed_bytes(*n);
  if (!bytes) return fail(FME_E_UNSUPPORTED, "fme_load_nn_net: no kernel for this net");
  std::vector<unsigned char> packed(bytes);
  nn_deep_pack(*n, params, packed.data());
  {   // a batch of this context in flight may still read the previous net
    const int rc = drain_ctx(c);
    if (rc) return rc;
  }
  HIP_TRY(c->d_net.reserve(bytes));
  HIP_TRY(hipMemcpy(c->d_net.p, packed.data(), bytes, hipMemcpyHostToDevice));
  c->net = *n;
  c->net_loaded = true;
  return FME_OK;
}

int fme_set_nn_engine(fme_ctx* c, int engine) {
  if (!c || (engine != FME_NN_ENGINE_EXACT && engine != FME_NN_ENGINE_MFMA))
    return fail(FME_E_INVALID, "fme_set_nn_engine: bad argument");
  c->nn_engine = engine;
  return FME_OK;
}

int fme_set_nn_logit_output(fme_ctx* c, void* d_logits, int capacity) {
  if (!c) return fail(FME_E_INVALID, "fme_set_nn_logit_output: null ctx");
  if (d_logits && capacity <= 0) return fail(FME_E_INVALID, "fme_set_nn_logit_output: capacity %d", capacity);
  c->nn_logits = capacity > 0 ? d_logits : nullptr;
  c->nn_logits_cap = d_logits ? capacity : 0;
  return FME_OK;
}

int fme_set_nn_inputs(fme_ctx* c, const uint32_t* d_rows, int capacity) {
  if (!c) return fail(FME_E_INVALID, "fme_set_nn_inputs: null ctx");
  if (d_rows && capacity <= 0) return fail(FME_E_INVALID, "fme_set_nn_inputs: capacity %d", capacity);
  c->nn_in = capacity > 0 ? d_rows : nullptr;
  c->nn_in_cap = d_rows ? capacity : 0;
  return FME_OK;
}

int fme_set_nn_margin_output(fme_ctx* c, float* d_margin, int capacity) {
  if (!c) return fail(FME_E_INVALID, "fme_set_nn_margin_output: null ctx");
  if (d_margin && capacity <= 0) return fail(FME_E_INVALID, "fme_set_nn_margin_output: capacity %d", capacity);
  c->nn_margin = capacity > 0 ? d_margin : nullptr;
  c->nn_margin_cap = d_margin ? capacity : 0;
  return FME_OK;
}

int fme_nn_reset_state(fme_ctx* c) {
  if (!c) return fail(FME_E_INVALID, "fme_nn_reset_state: null ctx");
  for (uint32_t& v : c->pending_state) v = 0;
  c->state_pending = true;
  return FME_OK;
}

int fme_nn_get_state(fme_ctx* c, uint32_t* out12) {
  if (!c || !out12) return fail(FME_E_INVALID, "fme_nn_get_state: null argument");
  if (c->state_pending) {
    std::memcpy(out12, c->pending_state, sizeof(c->pending_state));
    return FME_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  {
    const int rc = drain_ctx(c);   // this context's streams only
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpy(out12, c->nn_state.p + 12 * c->state_cur, 12 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return FME_OK;
}

int fme_nn_set_state(fme_ctx* c, const uint32_t* in12) {
  if (!c || !in12) return fail(FME_E_INVALID, "fme_nn_set_state: null argument");
  std::memcpy(c->pending_state, in12, sizeof(c->pending_state));
  c->state_pending = true;
  return FME_OK;
}

int fme_nn_copy_state_device(fme_ctx* c, uint32_t* d_out12, void* stream) {
  if (!c || !d_out12) return fail(FME_E_INVALID, "fme_nn_copy_state_device: null argument");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (c->state_pending)
    HIP_TRY(launch_put_state(d_out12, c->pending_state, s));
  else
    HIP_TRY(hipMemcpyAsync(d_out12, c->nn_state.p + 12 * c->state_cur, 12 * sizeof(uint32_t),
                           hipMemcpyDeviceToDevice, s));
  return FME_OK;
}

static int ensure_work(fme_ctx* c, int n) {
  const size_t nb = ((size_t)n + kJobsPerScanBlock - 1) / kJobsPerScanBlock;
  HIP_TRY(c->cls.reserve(n));
  HIP_TRY(c->perm.reserve(n));
  if (FME_SJOBS) HIP_TRY(c->sjobs.reserve(n));
  HIP_TRY(c->blk_agg.reserve(nb * 9));
  HIP_TRY(c->blk_prefix.reserve(nb * 9));
  return FME_OK;
}

static WorkBufs work_bufs(fme_ctx* c) {
  WorkBufs w{};
  w.cls = c->cls.p;
  w.perm = c->perm.p;
  w.sjobs = c->sjobs.p;
  w.counts = c->counts.p;
  w.cursor = c->counts.p + kNumClasses + 1;
  w.tile_ctr = c->counts.p + 2 * kNumClasses + 1;
  w.blk_agg = c->blk_agg.p;
  w.blk_prefix = c->blk_prefix.p;
  w.nn_state = c->nn_state.p;
  w.sched = c->d_sched.p;
  w.mv_out = nullptr;
  return w;
}

// The picture / lambda tables go to the device in stream order as the argument of a one-block
// kernel: rebinding pictures for the next frame never waits for the batch in flight, and the
// batch stream holds no copy-engine transfer (which would queue behind bulk uploads).
static int sync_tables(fme_ctx* c, hipStream_t s) {
  note_stream(c, s);   // every batch entry point passes here with its stream
  // a resident server could hold up this work on a hardware queue its stream shares: stop it
  // (a few microseconds; the next single call relaunches it)
  int rc = srv_stop(c);
  if (rc) return rc;
  if (!c->tables_dirty) return FME_OK;
  if (!c->h_tab) {
    void* p = nullptr;
    HIP_TRY(hipHostMalloc(&p, fme_ctx::kTabSlots * sizeof(TablesSlot), hipHostMallocMapped));
    c->h_tab = static_cast<TablesSlot*>(p);
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, p, 0));
    c->h_tab_dev = static_cast<TablesSlot*>(d);
    for (auto& e : c->tab_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const int k = c->tab_next;
  c->tab_next = (k + 1) % fme_ctx::kTabSlots;
  if (c->tab_used[k]) HIP_TRY(hipEventSynchronize(c->tab_ev[k]));   // its last launch has run
  std::memcpy(c->h_tab[k].pics, c->pics, sizeof(c->pics));
  std::memcpy(c->h_tab[k].ml, c->mlambda, sizeof(c->mlambda));
  HIP_TRY(launch_put_tables(c->d_pics.p, c->d_mlambda.p, c->h_tab_dev + k, s));
  HIP_TRY(hipEventRecord(c->tab_ev[k], s));
  c->tab_used[k] = true;
  c->tables_dirty = false;
  return FME_OK;
}

// Applies a reset / set of the NN state requested since the last batch, in stream order.
static int apply_pending_state(fme_ctx* c, hipStream_t s) {
  if (!c->state_pending) return FME_OK;
  HIP_TRY(launch_put_state(c->nn_state.p + 12 * c->state_cur, c->pending_state, s));
  c->state_pending = false;
  return FME_OK;
}

// Profiling: a ring of event sets; a set is read once its batch has finished (polled at the next
// batch, waited for only when the ring is full or the caller asks for the timings).
static int harvest_events(fme_ctx* c, bool wait_all) {
  while (c->ev_tail != c->ev_head) {
    const int b = c->ev_tail % fme_ctx::kEvSets;
    hipEvent_t* e = c->ev[b];
    if (wait_all) {
      HIP_TRY(hipEventSynchronize(e[6]));
    } else {
      const hipError_t q = hipEventQuery(e[6]);
      if (q == hipErrorNotReady) break;
      HIP_TRY(q);
    }
    float* ms = c->last_ms;
    HIP_TRY(hipEventElapsedTime(&ms[0], e[0], e[1]));
    HIP_TRY(hipEventElapsedTime(&ms[1], e[2], e[3]));
    HIP_TRY(hipEventElapsedTime(&ms[2], e[3], e[5]));
    HIP_TRY(hipEventElapsedTime(&ms[3], e[5], e[6]));
    HIP_TRY(hipEventElapsedTime(&ms[4], e[0], e[6]));
    HIP_TRY(hipEventElapsedTime(&ms[5], e[3], e[4]));
    ms[6] = 0.f;   // no auxiliary search kernel any more (every shape runs in the lane kernel)
    for (int i = 0; i < FME_NUM_TIMINGS; i++) c->acc_ms[i] += ms[i];
    c->acc_batches++;
    c->timed = true;
    c->ev_tail++;
  }
  return FME_OK;
}

// One batch: classify -> schedule (device) -> scatter -> search (lane kernels on three streams,
// cooperative AMP kernels beside them) -> NN + tail, all enqueued without waiting for the device.
// Device validation covers what the host cannot see for device-resident jobs: a job with an
// unknown PU shape, an unset picture / lambda slot or a key block outside the key buffer makes
// k_schedule mark the batch rejected; every later kernel then skips its work.
static int refine_batch(fme_ctx* c, const fme_job* d_jobs, fme_result* d_res, fme_mv_result* d_mv, int n,
                        hipStream_t s) {
  if (c->cfg.nn_mode == 1 && !c->nn_loaded) return fail(FME_E_STATE, "fme_refine_device: nn_mode set but no weights loaded");
  if (c->cfg.nn_mode == 2 && !c->net_loaded) return fail(FME_E_STATE, "fme_refine_device: nn_mode 2 but no net loaded");
  if (c->cfg.nn_mode == 2 && c->nn_margin && n > c->nn_margin_cap)
    return fail(FME_E_INVALID, "fme_refine: %d jobs but the margin output holds %d", n, c->nn_margin_cap);
  if (c->cfg.nn_mode == 2 && c->nn_logits && n > c->nn_logits_cap)
    return fail(FME_E_INVALID, "fme_refine: %d jobs but the logit output holds %d", n, c->nn_logits_cap);
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_work(c, n);
  if (rc) return rc;
  rc = sync_tables(c, s);
  if (rc) return rc;
  rc = apply_pending_state(c, s);
  if (rc) return rc;

  BatchArgs a{};
  a.jobs = d_jobs;
  a.res = d_res;
  a.keys = c->d_keys.p;
  a.n_keys = (int64_t)c->n_keys;
  a.key_invalid = c->d_key_invalid.p;
  a.mlambda = c->d_mlambda.p;
  a.pics = c->d_pics.p;
  a.n = n;
  a.use_hadamard = c->cfg.use_hadamard ? 1 : 0;
  a.fen = c->cfg.fast_inter_mode;
  a.nn_mode = c->cfg.nn_mode ? 1 : 0;
  a.nn_in = c->nn_in;
  a.nn_in_cap = c->nn_in_cap;
  WorkBufs w = work_bufs(c);
  w.mv_out = d_mv;

  const bool prof = c->profiling;
  hipEvent_t* ev = nullptr;
  int eb = 0;
  if (prof) {
    rc = harvest_events(c, false);
    if (rc) return rc;
    if (c->ev_head - c->ev_tail == fme_ctx::kEvSets) {   // ring full: wait for the oldest set
      HIP_TRY(hipEventSynchronize(c->ev[c->ev_tail % fme_ctx::kEvSets][6]));
      rc = harvest_events(c, false);
      if (rc) return rc;
    }
    eb = c->ev_head % fme_ctx::kEvSets;
    ev = c->ev[eb];
    HIP_TRY(hipEventRecord(ev[0], s));
  }
  HIP_TRY(hipMemsetAsync(c->counts.p, 0, kCountWords * sizeof(int32_t), s));
  HIP_TRY(launch_classify(a, w, s));
  if (prof) HIP_TRY(hipEventRecord(ev[1], s));
  HIP_TRY(launch_schedule(w, c->sched_p, s));
  if (prof) HIP_TRY(hipEventRecord(ev[2], s));
  HIP_TRY(launch_scatter(a, w, s));
  if (prof) HIP_TRY(hipEventRecord(ev[3], s));
  if (c->ev_search) HIP_TRY(hipEventRecord(c->ev_search, s));
  // the lane kernel: every PU shape, one launch on the batch stream (8-bit); the pixel kernel at
  // bit depth 10 (fme_px.hip)
  if (c->cfg.bit_depth > 8) {
    // the small- and large-PU pixel kernels one after the other: side by side on two streams they
    // took 11.5 ms per 1080p frame against 10.5 in series (profiles/r06_ab.log: their LDS and
    // wave slots compete)
    if (c->main10_px)
      HIP_TRY(launch_search_px(a, w, c->cfg.bit_depth, s, nullptr));
    else
      HIP_TRY(launch_search_lane10(a, w, s));
  } else {
    HIP_TRY(launch_search_lane(a, w, c->search_reserve, s));
  }
  if (prof) HIP_TRY(hipEventRecord(ev[4], s));
  if (prof) HIP_TRY(hipEventRecord(ev[5], s));
  HIP_TRY(c->cfg.nn_mode == 2
              ? launch_nn_deep_tail(c->net, c->d_net.p, c->nn_margin, c->nn_logits, a, w, c->state_cur, c->nn_engine, s)
              : launch_nn_tail(a, w, c->d_nn.p, c->state_cur, s));
  if (prof) {
    HIP_TRY(hipEventRecord(ev[6], s));
    c->ev_head++;
  }
  HIP_TRY(hipEventRecord(c->ev_done, s));
  c->batch_issued = true;
  if (a.nn_mode) c->state_cur ^= 1;
  return FME_OK;
}

int fme_refine_device(fme_ctx* c, const fme_job* d_jobs, fme_result* d_res, int n, void* stream) {
  if (!c || (n > 0 && (!d_jobs || !d_res))) return fail(FME_E_INVALID, "fme_refine_device: null argument");
  if (n < 0) return fail(FME_E_INVALID, "fme_refine_device: n = %d", n);
  if (n == 0) return FME_OK;
  return refine_batch(c, d_jobs, d_res, nullptr, n, static_cast<hipStream_t>(stream));
}

int fme_refine_mv_device(fme_ctx* c, const fme_job* d_jobs, fme_mv_result* d_out, int n, void* stream) {
  if (!c || (n > 0 && (!d_jobs || !d_out))) return fail(FME_E_INVALID, "fme_refine_mv_device: null argument");
  if (n < 0) return fail(FME_E_INVALID, "fme_refine_mv_device: n = %d", n);
  if (n == 0) return FME_OK;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(c->d_res.reserve(n));   // full records: context scratch
  return refine_batch(c, d_jobs, c->d_res.p, d_out, n, static_cast<hipStream_t>(stream));
}

// ---- packed jobs (include/fme.h fme_job_packed) -----------------------------------------------
int fme_pack_jobs(const fme_job* jobs, int n, fme_job_packed* out, int32_t* key_base) {
  if (n < 0 || (n > 0 && (!jobs || !out || !key_base))) return fail(FME_E_INVALID, "fme_pack_jobs: bad argument");
  const int waves = (n + FME_PACK_WAVE - 1) / FME_PACK_WAVE;
  for (int wv = 0; wv < waves; wv++) {
    int64_t next = -1;   // where the wave's next keyed block must start (-1: no keyed job yet)
    key_base[wv] = -1;
    const int e = std::min(n, (wv + 1) * FME_PACK_WAVE);
    for (int i = wv * FME_PACK_WAVE; i < e; i++) {
      const fme_job& j = jobs[i];
      const char* why = nullptr;
      if ((j.x & 3) || (j.y & 3) || (j.w & 3) || (j.h & 3) || j.w < 4 || j.w > 64 || j.h < 4 || j.h > 64)
        why = "PU off the 4x4 grid or not 4..64";
      else if (j.x >= 8192 || j.y >= 8192) why = "x or y >= 8192";
      else if (j.org_id >= 64 || j.ref_id >= 64 || j.lambda_id >= 32) why = "slot id >= 64 or lambda_id >= 32";
      else if (j.flags & ~15u) why = "unknown flags";
      else if (j.bits_in >= 64) why = "bits_in >= 64";
      else if (j.mv_x <= -32767 || j.mv_x >= 32766 || j.mv_y <= -32767 || j.mv_y >= 32766) why = "int16-extreme mv";
      else if (j.key_offset >= 0) {
        if (next < 0) key_base[wv] = j.key_offset;
        else if ((int64_t)j.key_offset != next) why = "key block not dense in job order within its wave";
        next = (int64_t)j.key_offset + (int64_t)j.w * j.h;
      }
      if (why) return fail(FME_E_UNSUPPORTED, "fme_pack_jobs: job %d: %s (use fme_job)", i, why);
      uint32_t rg = 0;
      if (j.mv_y - 1 >= j.lt_y) rg |= FME_PK_RANGE_TOP;
      if (j.mv_y + 1 <= j.rb_y) rg |= FME_PK_RANGE_BOTTOM;
      if (j.mv_x - 1 >= j.lt_x) rg |= FME_PK_RANGE_LEFT;
      if (j.mv_x + 1 <= j.rb_x) rg |= FME_PK_RANGE_RIGHT;
      fme_job_packed p;
      p.pu = (uint32_t)(j.x >> 2) | ((uint32_t)(j.y >> 2) << 11) | ((uint32_t)((j.w >> 2) - 1) << 22) |
             ((uint32_t)((j.h >> 2) - 1) << 26);
      p.ctl = (uint32_t)j.org_id | ((uint32_t)j.ref_id << 6) | ((uint32_t)j.lambda_id << 12) |
              ((uint32_t)j.flags << 17) | ((uint32_t)(j.key_offset >= 0) << 21) | (rg << 22) |
              ((uint32_t)j.bits_in << 26);
      p.mv_x = j.mv_x;
      p.mv_y = j.mv_y;
      p.mvp_x = j.mvp_x;
      p.mvp_y = j.mvp_y;
      out[i] = p;
    }
  }
  return FME_OK;
}

int fme_unpack_jobs(const fme_job_packed* packed, const int32_t* key_base, int n, fme_job* out) {
  if (n < 0 || (n > 0 && (!packed || !key_base || !out))) return fail(FME_E_INVALID, "fme_unpack_jobs: bad argument");
  int64_t next = 0;
  for (int i = 0; i < n; i++) {
    const fme_job_packed& p = packed[i];
    if (i % FME_PACK_WAVE == 0) next = key_base[i / FME_PACK_WAVE];
    fme_job j;
    j.x = (uint16_t)((p.pu & 2047u) * 4u);
    j.y = (uint16_t)(((p.pu >> 11) & 2047u) * 4u);
    j.w = (uint8_t)((((p.pu >> 22) & 15u) + 1u) * 4u);
    j.h = (uint8_t)((((p.pu >> 26) & 15u) + 1u) * 4u);
    j.org_id = (uint8_t)(p.ctl & 63u);
    j.ref_id = (uint8_t)((p.ctl >> 6) & 63u);
    j.lambda_id = (uint8_t)((p.ctl >> 12) & 31u);
    j.flags = (uint8_t)((p.ctl >> 17) & 15u);
    const uint32_t rg = (p.ctl >> 22) & 15u;
    j.bits_in = (uint16_t)(p.ctl >> 26);
    j.mv_x = p.mv_x;
    j.mv_y = p.mv_y;
    j.mvp_x = p.mvp_x;
    j.mvp_y = p.mvp_y;
    j.lt_x = (int16_t)(p.mv_x - ((rg & FME_PK_RANGE_LEFT) ? 1 : 0));
    j.rb_x = (int16_t)(p.mv_x + ((rg & FME_PK_RANGE_RIGHT) ? 1 : 0));
    j.lt_y = (int16_t)(p.mv_y - ((rg & FME_PK_RANGE_TOP) ? 1 : 0));
    j.rb_y = (int16_t)(p.mv_y + ((rg & FME_PK_RANGE_BOTTOM) ? 1 : 0));
    if ((p.ctl >> 21) & 1u) {
      j.key_offset = (int32_t)next;
      next += (int64_t)j.w * j.h;
    } else {
      j.key_offset = -1;
    }
    out[i] = j;
  }
  return FME_OK;
}

static int refine_packed(fme_ctx* c, const fme_job_packed* d_jobs, const int32_t* d_key_base, fme_result* d_res,
                         fme_mv_result* d_mv, int n, void* stream, const char* fn) {
  if (!c || (n > 0 && (!d_jobs || !d_key_base || !(d_res || d_mv)))) return fail(FME_E_INVALID, "%s: null argument", fn);
  if (n < 0) return fail(FME_E_INVALID, "%s: n = %d", fn, n);
  if (n == 0) return FME_OK;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(c->d_pk_jobs.reserve(n));
  if (!d_res) {
    HIP_TRY(c->d_res.reserve(n));   // full records: context scratch
    d_res = c->d_res.p;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(launch_unpack_jobs(d_jobs, d_key_base, c->d_pk_jobs.p, n, s));
  return refine_batch(c, c->d_pk_jobs.p, d_res, d_mv, n, s);
}

int fme_refine_packed_device(fme_ctx* c, const fme_job_packed* d_jobs, const int32_t* d_key_base, fme_result* d_res,
                             int n, void* stream) {
  if (c && n > 0 && !d_res) return fail(FME_E_INVALID, "fme_refine_packed_device: null argument");
  return refine_packed(c, d_jobs, d_key_base, d_res, nullptr, n, stream, "fme_refine_packed_device");
}

int fme_refine_mv_packed_device(fme_ctx* c, const fme_job_packed* d_jobs, const int32_t* d_key_base,
                                fme_mv_result* d_out, int n, void* stream) {
  if (c && n > 0 && !d_out) return fail(FME_E_INVALID, "fme_refine_mv_packed_device: null argument");
  return refine_packed(c, d_jobs, d_key_base, nullptr, d_out, n, stream, "fme_refine_mv_packed_device");
}

int fme_set_search_event(fme_ctx* c, void* event) {
  if (!c) return fail(FME_E_INVALID, "fme_set_search_event: null ctx");
  c->ev_search = static_cast<hipEvent_t>(event);
  return FME_OK;
}

int fme_set_search_reserve(fme_ctx* c, int workgroups) {
  if (!c || workgroups < 0 || workgroups > 4096) return fail(FME_E_INVALID, "fme_set_search_reserve: bad argument");
  c->search_reserve = workgroups;
  return FME_OK;
}

int fme_download_device(fme_ctx* c, const void* d_src, void* h_dst, size_t bytes, int workgroups, void* stream) {
  if (!c || (bytes && (!d_src || !h_dst))) return fail(FME_E_INVALID, "fme_download_device: null argument");
  if ((bytes & 15) || (reinterpret_cast<uintptr_t>(d_src) & 15) || (reinterpret_cast<uintptr_t>(h_dst) & 15))
    return fail(FME_E_INVALID, "fme_download_device: pointers and size must be 16-byte multiples");
  if (workgroups < 0 || workgroups > 1024) return fail(FME_E_INVALID, "fme_download_device: %d workgroups", workgroups);
  if (!bytes) return FME_OK;
  HIP_TRY(hipSetDevice(c->device));
  void* dst = nullptr;   // the device's address of the pinned host rows
  if (hipHostGetDevicePointer(&dst, h_dst, 0) != hipSuccess || !dst) {
    (void)hipGetLastError();
    return fail(FME_E_INVALID, "fme_download_device: h_dst is not pinned host memory");
  }
  HIP_TRY(launch_download(d_src, dst, bytes / 16, workgroups ? workgroups : 8, static_cast<hipStream_t>(stream)));
  return FME_OK;
}

// ---- copy-engine warm-up (fme_warm_copy_engines) ---------------------------------------------
// ROCclr submits each hipMemcpyAsync between host and device memory to one SDMA engine of the
// device; when a stream's previous engine is still busy it asks the HSA runtime for a free one
// (hsa_amd_memory_copy_engine_status), and the HSA runtime creates an engine's queue at its first
// use.  That creation blocked the submitting host thread for 5.6-7.5 ms each time a pipelined copy
// landed on an engine not used before (gpurun_out/r06a/env_logwait.log: "Query copy engine status
// ... free_engine_mask 0xfffe" -> copy_engine=0x2 -> a 6.7 ms host gap), and the device drained
// meanwhile.  Here every engine gets one small copy in each direction up front, through the HSA
// runtime HIP already initialised (its symbols resolved from the loaded library, no link
// dependency).
namespace {
struct HsaCopyApi {
  hsa_status_t (*iterate_agents)(hsa_status_t (*)(hsa_agent_t, void*), void*);
  hsa_status_t (*agent_get_info)(hsa_agent_t, hsa_agent_info_t, void*);
  hsa_status_t (*signal_create)(hsa_signal_value_t, uint32_t, const hsa_agent_t*, hsa_signal_t*);
  hsa_status_t (*signal_destroy)(hsa_signal_t);
  hsa_signal_value_t (*signal_wait)(hsa_signal_t, hsa_signal_condition_t, hsa_signal_value_t, uint64_t,
                                    hsa_wait_state_t);
  hsa_status_t (*copy_on_engine)(void*, hsa_agent_t, const void*, hsa_agent_t, size_t, uint32_t,
                                 const hsa_signal_t*, hsa_signal_t, hsa_amd_sdma_engine_id_t, bool);
};
bool hsa_copy_api(HsaCopyApi& a) {
  void* h = dlopen("libhsa-runtime64.so.1", RTLD_LAZY | RTLD_NOLOAD);
  if (!h) h = dlopen("libhsa-runtime64.so.1", RTLD_LAZY);
  if (!h) return false;
  a.iterate_agents = reinterpret_cast<decltype(a.iterate_agents)>(dlsym(h, "hsa_iterate_agents"));
  a.agent_get_info = reinterpret_cast<decltype(a.agent_get_info)>(dlsym(h, "hsa_agent_get_info"));
  a.signal_create = reinterpret_cast<decltype(a.signal_create)>(dlsym(h, "hsa_signal_create"));
  a.signal_destroy = reinterpret_cast<decltype(a.signal_destroy)>(dlsym(h, "hsa_signal_destroy"));
  a.signal_wait = reinterpret_cast<decltype(a.signal_wait)>(dlsym(h, "hsa_signal_wait_scacquire"));
  a.copy_on_engine = reinterpret_cast<decltype(a.copy_on_engine)>(dlsym(h, "hsa_amd_memory_async_copy_on_engine"));
  return a.iterate_agents && a.agent_get_info && a.signal_create && a.signal_destroy && a.signal_wait &&
         a.copy_on_engine;
}
struct AgentPick {
  const HsaCopyApi* api;
  uint32_t bdf, domain;
  bool have_gpu = false, have_cpu = false;
  hsa_agent_t gpu{}, cpu{};
};
hsa_status_t pick_agent(hsa_agent_t ag, void* data) {
  AgentPick* p = static_cast<AgentPick*>(data);
  hsa_device_type_t t;
  if (p->api->agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !p->have_cpu) {
    p->cpu = ag;
    p->have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !p->have_gpu) {
    uint32_t bdf = 0, dom = 0;
    p->api->agent_get_info(ag, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
    p->api->agent_get_info(ag, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
    if (bdf == p->bdf && dom == p->domain) {
      p->gpu = ag;
      p->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}
}  // namespace

int fme_warm_copy_engines(fme_ctx* c, int* engines) {
  if (!c) return fail(FME_E_INVALID, "fme_warm_copy_engines: null ctx");
  if (engines) *engines = 0;
  HIP_TRY(hipSetDevice(c->device));
  HsaCopyApi api{};
  if (!hsa_copy_api(api)) return fail(FME_E_DEVICE, "fme_warm_copy_engines: HSA runtime symbols not found");
  int bus = 0, dev = 0, dom = 0;
  HIP_TRY(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device));
  HIP_TRY(hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, c->device));
  HIP_TRY(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->device));
  AgentPick pk{&api, (uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom};
  api.iterate_agents(pick_agent, &pk);
  if (!pk.have_gpu || !pk.have_cpu) return fail(FME_E_DEVICE, "fme_warm_copy_engines: HSA agents not found");
  uint32_t n_sdma = 0, n_xgmi = 0;
  api.agent_get_info(pk.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_SDMA_ENG), &n_sdma);
  api.agent_get_info(pk.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_SDMA_XGMI_ENG), &n_xgmi);
  const int n_eng = std::min(16, (int)(n_sdma + n_xgmi));
  constexpr size_t kBytes = 4096;
  void* d = nullptr;
  void* h = nullptr;
  HIP_TRY(hipMalloc(&d, kBytes));
  if (hipHostMalloc(&h, kBytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipFree(d);
    return fail(FME_E_NOMEM, "fme_warm_copy_engines: host buffer");
  }
  std::memset(h, 0, kBytes);
  int warmed = 0;
  for (int e = 0; e < n_eng; e++) {
    bool ok = true;
    for (int dir = 0; dir < 2 && ok; dir++) {   // host -> device, device -> host
      hsa_signal_t sig;
      if (api.signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) {
        ok = false;
        break;
      }
      const auto eid = static_cast<hsa_amd_sdma_engine_id_t>(1u << e);
      const hsa_status_t st = dir == 0 ? api.copy_on_engine(d, pk.gpu, h, pk.cpu, kBytes, 0, nullptr, sig, eid, true)
                                       : api.copy_on_engine(h, pk.cpu, d, pk.gpu, kBytes, 0, nullptr, sig, eid, true);
      if (st == HSA_STATUS_SUCCESS)
        api.signal_wait(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
      else
        ok = false;
      api.signal_destroy(sig);
    }
    warmed += ok ? 1 : 0;
  }
  (void)hipHostFree(h);
  (void)hipFree(d);
  if (engines) *engines = warmed;
  return FME_OK;
}

int fme_refine_status(fme_ctx* c) {
  if (!c) return fail(FME_E_INVALID, "fme_refine_status: null ctx");
  if (!c->batch_issued) return 0;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->ev_done));
  int32_t v = 0;
  HIP_TRY(hipMemcpy(&v, &c->d_sched.p->invalid, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

// ---- integer motion estimation (xTZSearch / xPatternSearch) -----------------------------------
// classify (validation + class histogram, one host sync) -> scatter (jobs grouped by PU shape)
// -> one search launch per unit shape (fme_tz.hip) writing mv_x / mv_y (and ruiSAD) in place.
}  // extern "C"

// d_emi (may be null): also run the EMI square step of uni-pred EMI jobs and write the resulting
// integer MV there (the producer's m_integerMv2Nx2N), leaving jobs' mv_x / mv_y at the TZ best.
// d_nn_in (may be null): FME_TZ_RING jobs run the backups' square + ring and write their NN inputs.
static int tz_run(fme_ctx* c, fme_job* d_jobs, const fme_tz_ext* d_ext, uint32_t* d_sad, int n, void* stream,
                  int16_t* d_emi, uint32_t* d_nn_in = nullptr, int ext_stride = (int)sizeof(fme_tz_ext)) {
  if (!c || (n > 0 && (!d_jobs || !d_ext))) return fail(FME_E_INVALID, "fme_integer_search_device: null argument");
  if (n < 0) return fail(FME_E_INVALID, "fme_integer_search_device: n = %d", n);
  if (n == 0) return FME_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = ensure_work(c, n);
  if (rc) return rc;
  rc = sync_tables(c, s);
  if (rc) return rc;
  BatchArgs a{};
  a.jobs = d_jobs;
  a.keys = c->d_keys.p;
  a.n_keys = (int64_t)c->n_keys;
  a.key_invalid = c->d_key_invalid.p;
  a.mlambda = c->d_mlambda.p;
  a.pics = c->d_pics.p;
  a.n = n;
  a.use_hadamard = c->cfg.use_hadamard ? 1 : 0;
  a.fen = c->cfg.fast_inter_mode;
  a.nn_in = c->nn_in;   // FME_JOB_NN_IN jobs (the B producer's bi rounds) pass k_classify with their rows
  a.nn_in_cap = c->nn_in_cap;
  WorkBufs w = work_bufs(c);
  if (c->profiling) {
    if (!c->ev_tz[0]) {
      HIP_TRY(hipEventCreate(&c->ev_tz[0]));
      HIP_TRY(hipEventCreate(&c->ev_tz[1]));
    }
  }
  HIP_TRY(hipMemsetAsync(c->counts.p, 0, kCountWords * sizeof(int32_t), s));
  HIP_TRY(launch_classify(a, w, s));
  HIP_TRY(launch_schedule(w, c->sched_p, s));   // class offsets for the scatter
  HIP_TRY(hipMemcpyAsync(c->h_counts, c->counts.p, kCountWords * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->h_counts[kNumClasses] > 0)
    return fail(FME_E_INVALID, "fme_integer_search_device: %d job(s) with an unsupported PU size or unset picture/lambda/key",
                c->h_counts[kNumClasses]);
  const bool keyed = c->h_counts[kKeyedWord] > 0;
  TzSchedule sc{};
  int off = 0, nb[3] = {0, 0, 0};
  for (int k = 0; k < kNumClasses; k++) {
    const int cnt = c->h_counts[k];
    sc.class_off[k] = off;
    sc.class_cnt[k] = cnt;
    for (int q = 0; q < 3; q++) sc.prefix[q][k] = nb[q];
    nb[tz_kernel_of(k)] += cnt;
    off += cnt;
  }
  for (int q = 0; q < 3; q++) sc.prefix[q][kNumClasses] = nb[q];
  HIP_TRY(launch_scatter(a, w, s));
  TzArgs ta{};
  ta.a = a;
  ta.sjobs = c->sjobs.p;
  ta.perm = c->perm.p;
  ta.jobs_out = d_jobs;
  ta.ext = d_ext;
  ta.ext_stride = ext_stride;
  ta.sad = d_sad;
  ta.emi_mv = d_emi;
  ta.nn_in = d_nn_in;
  if (c->profiling) HIP_TRY(hipEventRecord(c->ev_tz[0], s));
  // the three unit-shape kernels are latency-bound and independent: 4x8 and 8x4 units on the two
  // auxiliary streams, 8x8 units on the caller's stream, joined before returning
  // the integer search's own auxiliary streams (the refinement batch uses none)
  if (!c->aux) HIP_TRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
  if (!c->aux2) HIP_TRY(hipStreamCreateWithFlags(&c->aux2, hipStreamNonBlocking));
  if (!c->ev_fork) HIP_TRY(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
  if (!c->ev_join) HIP_TRY(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
  if (!c->ev_join2) HIP_TRY(hipEventCreateWithFlags(&c->ev_join2, hipEventDisableTiming));
  // the staged form (FME_TZ_STAGE): PUs grouped by (kernel, reference, CTU) on the device, each
  // group's search area read into LDS once (fme_tz.hip k_tz_staged)
  int cw = 0, ch = 0, npic = 0;   // CTU grid of the largest bound picture; reference ids < npic
  for (int i = 0; i < FME_MAX_PICTURES; i++)
    if (c->pics[i].luma) {
      cw = std::max(cw, (c->pics[i].width + 63) / 64);
      ch = std::max(ch, (c->pics[i].height + 63) / 64);
      npic = i + 1;
    }
  const long long np = (long long)npic * cw * ch;
  const bool stage = c->cfg.bit_depth == 8 || std::getenv("FME_TZ10_UNSTAGED") == nullptr;   // (A/B switch)
  if (FME_TZ_STAGE && stage && np > 0 && np <= (1LL << 20)) {
    const size_t words = 8 + 12 * (size_t)np;
    if (c->d_tzp.cap < words || c->d_tzp_perm.cap < (size_t)n) {
      rc = drain_ctx(c);   // no launch of an earlier call still reads the old buffers
      if (rc) return rc;
      HIP_TRY(c->d_tzp.reserve(words));
      HIP_TRY(c->d_tzp_perm.reserve(n));
    }
    TzPairs tp{};
    int32_t* b = c->d_tzp.p;
    tp.nseg = b;
    tp.cnt = b + 8;
    tp.cursor = tp.cnt + 3 * np;
    tp.off = tp.cursor + 3 * np;
    tp.seg = tp.off + 3 * np;
    tp.perm = c->d_tzp_perm.p;
    tp.np = (int32_t)np;
    tp.cw = cw;
    tp.ch = ch;
    HIP_TRY(hipMemsetAsync(b, 0, (8 + 3 * (size_t)np) * sizeof(int32_t), s));
    HIP_TRY(launch_tz_pairs(ta, tp, w.cls, n, s));
    HIP_TRY(hipEventRecord(c->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
    HIP_TRY(hipStreamWaitEvent(c->aux2, c->ev_fork, 0));
    HIP_TRY(launch_tz_staged(ta, tp, 0, keyed, c->cfg.bit_depth, c->aux));
    HIP_TRY(launch_tz_staged(ta, tp, 1, keyed, c->cfg.bit_depth, c->aux2));
    HIP_TRY(launch_tz_staged(ta, tp, 2, keyed, c->cfg.bit_depth, s));
  } else {
    HIP_TRY(hipEventRecord(c->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(c->aux, c->ev_fork, 0));
    HIP_TRY(hipStreamWaitEvent(c->aux2, c->ev_fork, 0));
    HIP_TRY(launch_tz_wave(ta, sc, 0, keyed, c->cfg.bit_depth, c->aux));
    HIP_TRY(launch_tz_wave(ta, sc, 1, keyed, c->cfg.bit_depth, c->aux2));
    HIP_TRY(launch_tz_wave(ta, sc, 2, keyed, c->cfg.bit_depth, s));
  }
  HIP_TRY(hipEventRecord(c->ev_join, c->aux));
  HIP_TRY(hipEventRecord(c->ev_join2, c->aux2));
  HIP_TRY(hipStreamWaitEvent(s, c->ev_join, 0));
  HIP_TRY(hipStreamWaitEvent(s, c->ev_join2, 0));
  if (c->profiling) HIP_TRY(hipEventRecord(c->ev_tz[1], s));
  c->tz_timed = c->profiling;
  return FME_OK;
}

static int tz_run_host(fme_ctx* c, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n, void* stream,
                       int16_t* emi, uint32_t* nn_in = nullptr, int ext_stride = (int)sizeof(fme_tz_ext)) {
  if (!c || (n > 0 && (!jobs || !ext))) return fail(FME_E_INVALID, "fme_integer_search: null argument");
  if (n <= 0) return n == 0 ? FME_OK : fail(FME_E_INVALID, "fme_integer_search: n = %d", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(c->d_jobs.reserve(n));
  HIP_TRY(c->d_tz_ext.reserve(((size_t)n * ext_stride + sizeof(fme_tz_ext) - 1) / sizeof(fme_tz_ext)));
  HIP_TRY(c->d_tz_sad.reserve(n));
  if (emi) HIP_TRY(c->d_tz_emi.reserve((size_t)2 * n));
  if (nn_in) HIP_TRY(c->d_tz_nn_in.reserve((size_t)9 * n));
  HIP_TRY(hipMemcpyAsync(c->d_jobs.p, jobs, (size_t)n * sizeof(fme_job), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_tz_ext.p, ext, (size_t)n * ext_stride, hipMemcpyHostToDevice, s));
  // rows of jobs without FME_TZ_RING are left untouched: start from the caller's values
  if (nn_in) HIP_TRY(hipMemcpyAsync(c->d_tz_nn_in.p, nn_in, (size_t)9 * n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  int rc = tz_run(c, c->d_jobs.p, c->d_tz_ext.p, c->d_tz_sad.p, n, stream, emi ? c->d_tz_emi.p : nullptr,
                  nn_in ? c->d_tz_nn_in.p : nullptr, ext_stride);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(jobs, c->d_jobs.p, (size_t)n * sizeof(fme_job), hipMemcpyDeviceToHost, s));
  if (sad) HIP_TRY(hipMemcpyAsync(sad, c->d_tz_sad.p, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if (emi) HIP_TRY(hipMemcpyAsync(emi, c->d_tz_emi.p, (size_t)n * 2 * sizeof(int16_t), hipMemcpyDeviceToHost, s));
  if (nn_in) HIP_TRY(hipMemcpyAsync(nn_in, c->d_tz_nn_in.p, (size_t)9 * n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return FME_OK;
}

// The integer searches of a producer's jobs by m_integerMv2Nx2N dependency level.  jobs / ext in
// call order (ext's pred2n already set where src[u] < 0); lvl[u]: the level of job u; src[u]: the
// job whose post-EMI MV is u's m_integerMv2Nx2N, or -1.  One upload, one k_tz_level launch per
// level back to back on the stream (a level reads the earlier levels' MVs from device memory), one
// download: the chain of a 1080p frame (≈ 2,200 levels, most of a few jobs: the bottom CTU row has
// no depth-0 CU) never waits for the host.  emi: the post-EMI integer MV of every job.
struct PiClock;
static void pi_lap(PiClock* clk, int k);
static int tz_by_level(fme_ctx* c, std::vector<fme_job>& jobs, std::vector<fme_tz_ext>& ext,
                       const std::vector<int>& src, const std::vector<int>& lvl, hipStream_t s,
                       std::vector<int16_t>& emi, PiClock* clk = nullptr) {
  const int nu = (int)jobs.size();
  emi.assign((size_t)nu * 2, 0);
  if (nu == 0) return FME_OK;
  int max_level = 0;
  for (int v : lvl) max_level = std::max(max_level, v);
  std::vector<int32_t> off((size_t)max_level + 2, 0), pos((size_t)nu), psrc((size_t)nu);
  std::vector<int> order((size_t)nu);
  for (int u = 0; u < nu; u++) off[lvl[u] + 1]++;
  for (int l = 0; l <= max_level; l++) off[l + 1] += off[l];
  {
    // within a level, the largest PUs first: blocks dispatch in index order, so the longest
    // searches of a wide level start at once instead of forming its tail
    std::vector<int> byarea((size_t)nu), start(64 * 64 + 2, 0);   // counting sort, area descending
    for (int u = 0; u < nu; u++) start[64 * 64 - (int)jobs[u].w * jobs[u].h + 1]++;
    for (size_t a = 1; a < start.size(); a++) start[a] += start[a - 1];
    for (int u = 0; u < nu; u++) byarea[start[64 * 64 - (int)jobs[u].w * jobs[u].h]++] = u;
    std::vector<int32_t> fill(off.begin(), off.end() - 1);
    for (int u : byarea) {
      pos[u] = fill[lvl[u]]++;
      order[pos[u]] = u;
    }
  }
  std::vector<fme_job> lj((size_t)nu);
  std::vector<fme_tz_ext> le((size_t)nu);
  for (int q = 0; q < nu; q++) {
    const int u = order[q];
    lj[q] = jobs[u];
    le[q] = ext[u];
    psrc[q] = ((ext[u].flags & FME_TZ_PRED2NX2N) && src[u] >= 0) ? pos[src[u]] : -1;
  }
  pi_lap(clk, 2);   // the level ordering is host setup; the chain starts with its upload
  HIP_TRY(c->d_jobs.reserve(nu));
  HIP_TRY(c->d_tz_ext.reserve(nu));
  HIP_TRY(c->d_tz_emi.reserve((size_t)2 * nu));
  HIP_TRY(c->d_ch_i32.reserve((size_t)nu));
  HIP_TRY(hipMemcpyAsync(c->d_jobs.p, lj.data(), (size_t)nu * sizeof(fme_job), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_tz_ext.p, le.data(), (size_t)nu * sizeof(fme_tz_ext), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_ch_i32.p, psrc.data(), (size_t)nu * sizeof(int32_t), hipMemcpyHostToDevice, s));
  TzArgs ta{};
  ta.a.jobs = c->d_jobs.p;
  ta.a.keys = c->d_keys.p;
  ta.a.n_keys = (int64_t)c->n_keys;
  ta.a.key_invalid = c->d_key_invalid.p;
  ta.a.mlambda = c->d_mlambda.p;
  ta.a.pics = c->d_pics.p;
  ta.a.n = nu;
  ta.a.use_hadamard = c->cfg.use_hadamard ? 1 : 0;
  ta.a.fen = c->cfg.fast_inter_mode;
  ta.jobs_out = c->d_jobs.p;
  ta.ext = c->d_tz_ext.p;
  ta.ext_stride = (int)sizeof(fme_tz_ext);
  ta.emi_mv = c->d_tz_emi.p;
  const TzChain ch{c->d_ch_i32.p, max_level + 1};
  HIP_TRY(launch_tz_levels(ta, ch, off.data(), c->cfg.bit_depth, s));
  std::vector<int16_t> lemi((size_t)2 * nu);
  HIP_TRY(hipMemcpyAsync(lj.data(), c->d_jobs.p, (size_t)nu * sizeof(fme_job), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(lemi.data(), c->d_tz_emi.p, (size_t)2 * nu * sizeof(int16_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (int q = 0; q < nu; q++) {
    const int u = order[q];
    jobs[u] = lj[q];
    emi[2 * u] = lemi[2 * q];
    emi[2 * u + 1] = lemi[2 * q + 1];
  }
  return FME_OK;
}

extern "C" {

int fme_integer_search_device(fme_ctx* c, fme_job* d_jobs, const fme_tz_ext* d_ext, uint32_t* d_sad, int n,
                              void* stream) {
  return tz_run(c, d_jobs, d_ext, d_sad, n, stream, nullptr);
}

int fme_integer_search(fme_ctx* c, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n, void* stream) {
  return tz_run_host(c, jobs, ext, sad, n, stream, nullptr);
}

int fme_integer_search2_device(fme_ctx* c, fme_job* d_jobs, const fme_tz_ext2* d_ext, uint32_t* d_sad, int n,
                               void* stream) {
  return tz_run(c, d_jobs, reinterpret_cast<const fme_tz_ext*>(d_ext), d_sad, n, stream, nullptr, nullptr,
                (int)sizeof(fme_tz_ext2));
}

int fme_integer_search2(fme_ctx* c, fme_job* jobs, const fme_tz_ext2* ext, uint32_t* sad, int n, void* stream) {
  return tz_run_host(c, jobs, reinterpret_cast<const fme_tz_ext*>(ext), sad, n, stream, nullptr, nullptr,
                     (int)sizeof(fme_tz_ext2));
}

int fme_integer_search_ring_device(fme_ctx* c, fme_job* d_jobs, const fme_tz_ext* d_ext, uint32_t* d_sad,
                                   uint32_t* d_nn_in, int n, void* stream) {
  if (!d_nn_in && n > 0) return fail(FME_E_INVALID, "fme_integer_search_ring_device: null nn_in");
  return tz_run(c, d_jobs, d_ext, d_sad, n, stream, nullptr, d_nn_in);
}

int fme_integer_search_ring(fme_ctx* c, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, uint32_t* nn_in,
                            int n, void* stream) {
  if (!nn_in && n > 0) return fail(FME_E_INVALID, "fme_integer_search_ring: null nn_in");
  return tz_run_host(c, jobs, ext, sad, n, stream, nullptr, nn_in);
}

int fme_integer_search_last_ms(fme_ctx* c, float* ms) {
  if (!c || !ms) return fail(FME_E_INVALID, "fme_integer_search_last_ms: null argument");
  if (!c->tz_timed) return fail(FME_E_STATE, "fme_integer_search_last_ms: no profiled integer search");
  HIP_TRY(hipEventSynchronize(c->ev_tz[1]));
  HIP_TRY(hipEventElapsedTime(ms, c->ev_tz[0], c->ev_tz[1]));
  return FME_OK;
}

// Host arrays: H2D of the jobs, the batch, D2H of the outputs and of the rejected-job count,
// one synchronisation at the end.
static int refine_host(fme_ctx* c, const fme_job* jobs, fme_result* res, fme_mv_result* mv, int n, void* stream,
                       const char* name) {
  if (!c || (n > 0 && (!jobs || (!res && !mv)))) return fail(FME_E_INVALID, "%s: null argument", name);
  if (n <= 0) return n == 0 ? FME_OK : fail(FME_E_INVALID, "%s: n = %d", name, n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(c->d_jobs.reserve(n));
  HIP_TRY(c->d_res.reserve(n));
  if (mv) HIP_TRY(c->d_mv.reserve(n));
  HIP_TRY(hipMemcpyAsync(c->d_jobs.p, jobs, (size_t)n * sizeof(fme_job), hipMemcpyHostToDevice, s));
  int rc = refine_batch(c, c->d_jobs.p, c->d_res.p, mv ? c->d_mv.p : nullptr, n, s);
  if (rc) return rc;
  if (mv)
    HIP_TRY(hipMemcpyAsync(mv, c->d_mv.p, (size_t)n * sizeof(fme_mv_result), hipMemcpyDeviceToHost, s));
  else
    HIP_TRY(hipMemcpyAsync(res, c->d_res.p, (size_t)n * sizeof(fme_result), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(c->h_counts, &c->d_sched.p->invalid, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->h_counts[0] > 0)
    return fail(FME_E_INVALID, "%s: %d job(s) with an unsupported PU size or unset picture/lambda/key", name,
                c->h_counts[0]);
  return FME_OK;
}

int fme_refine(fme_ctx* c, const fme_job* jobs, fme_result* res, int n, void* stream) {
  return refine_host(c, jobs, res, nullptr, n, stream, "fme_refine");
}

int fme_refine_mv(fme_ctx* c, const fme_job* jobs, fme_mv_result* out, int n, void* stream) {
  return refine_host(c, jobs, nullptr, out, n, stream, "fme_refine_mv");
}

// The deeper nets' single NN_pred call: its completion word in pinned, device-mapped host memory.
static int ensure_stage(fme_ctx* c) {
  if (c->stage) return FME_OK;
  void* p = nullptr;
  HIP_TRY(hipHostMalloc(&p, sizeof(SingleStage), hipHostMallocMapped));
  c->stage = static_cast<SingleStage*>(p);
  void* d = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&d, p, 0));
  c->stage_dev = static_cast<uint8_t*>(d);
  HIP_TRY(hipStreamCreateWithFlags(&c->single_stream, hipStreamNonBlocking));
  std::memset(c->stage, 0, sizeof(SingleStage));
  return FME_OK;
}

static int class_of(int w, int h) {
  for (int k = 0; k < kNumClasses; k++)
    if (kClassW[k] == w && kClassH[k] == h) return k;
  return -1;
}

// Wait for a single-PU kernel's completion word (written after its results, system-scope release)
// instead of synchronising the stream; the stream is queried now and then so a kernel that ended
// without writing it (a device error) is reported, not waited on forever.
static int single_wait(fme_ctx* c, uint32_t seq) {
  volatile uint32_t* f = &c->stage->flag;
  for (long it = 1; *f != seq; it++) {
    __builtin_ia32_pause();
    if ((it & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->single_stream);
      if (q != hipErrorNotReady && *f != seq) {
        if (q != hipSuccess) return fail(FME_E_DEVICE, "single-PU kernel: %s", hipGetErrorString(q));
        return fail(FME_E_DEVICE, "single-PU kernel ended without its completion word");
      }
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return FME_OK;
}

// ---- the single-call server (fme_server.hip) ----------------------------------------------------
// One resident workgroup serves fme_frac_dif_single and the master net's fme_nn_pred_single: the
// host writes the request into the mailbox (pinned, device-mapped), releases req_seq and spins on
// the answer block res.  An instance exits after kSrvIdleUs without a call or kSrvLifeMs of life (or on `stop`)
// and writes its epoch to `stopped`; a call that finds its instance gone relaunches one, which
// serves the pending request.
constexpr uint64_t kSrvIdleUs = 2000;
constexpr uint64_t kSrvLifeMs = 100;

static int srv_open(fme_ctx* c) {
  if (c->box) return FME_OK;
  void* p = nullptr;
  HIP_TRY(hipHostMalloc(&p, sizeof(SrvBox), hipHostMallocMapped));
  std::memset(p, 0, sizeof(SrvBox));
  c->box = static_cast<SrvBox*>(p);
  void* d = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&d, p, 0));
  c->box_dev = static_cast<SrvBox*>(d);
  HIP_TRY(hipStreamCreateWithFlags(&c->srv_stream, hipStreamNonBlocking));
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) == hipSuccess && khz > 0)
    c->srv_khz = (uint64_t)khz;
  return FME_OK;
}

static int srv_launch(fme_ctx* c) {
  if (c->srv_orphan) {   // never two instances on one mailbox: relaunch only once the old one has left
    const hipError_t q = hipStreamQuery(c->srv_stream);
    if (q == hipErrorNotReady)
      return fail(FME_E_DEVICE, "single-call server: the instance that timed out is still running");
    (void)hipGetLastError();
    c->srv_orphan = false;
  }
  __atomic_store_n(&c->box->req[0][3], 0u, __ATOMIC_RELEASE);
  const uint32_t epoch = ++c->srv_epoch;
  c->srv_nn_gen = c->nn_gen;
  HIP_TRY(launch_server(c->box_dev, c->nn_loaded ? c->d_nn.p : nullptr, c->srv_done, epoch,
                        kSrvIdleUs * c->srv_khz / 1000, kSrvLifeMs * c->srv_khz, c->srv_stream));
  c->srv_running = true;
  return FME_OK;
}

// The running instance's end: its `stopped` word (or a device error on its stream).
// Host-side bound of a wait on the server (a call, or its stop): far above any call's work (a 64x64
// FracDIF takes ~0.1 ms, an instance lives 100 ms), so only a server that never answers reaches it.
constexpr double kSrvWaitLimitS = 2.0;
static bool srv_waited_too_long(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kSrvWaitLimitS;
}

static int srv_join(fme_ctx* c) {
  volatile uint32_t* st = &c->box->stopped;
  const auto t0 = std::chrono::steady_clock::now();
  for (long it = 1; *st != c->srv_epoch; it++) {
    __builtin_ia32_pause();
    if ((it & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->srv_stream);
      if (q != hipErrorNotReady && *st != c->srv_epoch) {
        c->srv_running = false;
        if (q != hipSuccess) return fail(FME_E_DEVICE, "single-call server: %s", hipGetErrorString(q));
        return fail(FME_E_DEVICE, "single-call server ended without its stop word");
      }
      if (srv_waited_too_long(t0)) {
        c->srv_running = false;
        c->srv_orphan = true;   // srv_launch waits for it to leave srv_stream before a relaunch
        return fail(FME_E_DEVICE, "single-call server: no stop word after %.1f s", kSrvWaitLimitS);
      }
    }
  }
  c->srv_running = false;
  HIP_TRY(hipStreamSynchronize(c->srv_stream));
  return FME_OK;
}

static int srv_stop(fme_ctx* c) {
  if (!c->srv_running) return FME_OK;
  __atomic_store_n(&c->box->req[0][3], 1u, __ATOMIC_RELEASE);
  return srv_join(c);
}

// One call: the request fields and payload are in c->box already.
static int srv_call(fme_ctx* c, bool uses_nn) {
  int rc = FME_OK;
  if (c->srv_running && uses_nn && c->srv_nn_gen != c->nn_gen) rc = srv_stop(c);
  if (!rc && !c->srv_running) rc = srv_launch(c);
  if (rc) return rc;
  const uint32_t seq = c->srv_done + 1;
  __atomic_store_n(&c->box->req[0][0], seq, __ATOMIC_RELEASE);
  volatile uint32_t* done = &c->box->res[0];
  volatile uint32_t* st = &c->box->stopped;
  const auto t0 = std::chrono::steady_clock::now();
  for (long it = 1; *done != seq; it++) {
    __builtin_ia32_pause();
    if (*st == c->srv_epoch && *done != seq) {   // the instance left before it saw the call
      c->srv_running = false;
      HIP_TRY(hipStreamSynchronize(c->srv_stream));
      if (srv_waited_too_long(t0))
        return fail(FME_E_DEVICE, "single-call server: call %u unanswered after %.1f s", seq, kSrvWaitLimitS);
      rc = srv_launch(c);
      if (rc) return rc;
    } else if ((it & 4095) == 0) {
      const hipError_t q = hipStreamQuery(c->srv_stream);
      if (q != hipErrorNotReady && q != hipSuccess) {
        c->srv_running = false;
        return fail(FME_E_DEVICE, "single-call server: %s", hipGetErrorString(q));
      }
      if (srv_waited_too_long(t0)) {   // stop the instance (it exits within its lifetime) and give up
        __atomic_store_n(&c->box->req[0][3], 1u, __ATOMIC_RELEASE);
        if (srv_join(c) != FME_OK) c->srv_orphan = true;
        c->srv_running = false;
        return fail(FME_E_DEVICE, "single-call server: call %u unanswered after %.1f s", seq, kSrvWaitLimitS);
      }
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  c->srv_done = seq;
  return FME_OK;
}

// xPatternSearchFracDIF for one PU, as TEncSearch calls it: the key block (pcPatternKey, HM Pel)
// and the reference window around the integer MV (rows -4..h+3, columns -4..w+3 of the padded
// picture) go into the server's mailbox; the MV predictor is shifted by 4*mv_int so that every
// MV-cost argument (xPatternRefinement's (cMvTest << scale) - pred) is unchanged.
// Bit depth 10: the call runs as a one-job batch (the lane kernel k_search_lane10, bit-exact with
// the main10 batches) on a private 10-bit context with its own stream, so the caller's pictures,
// lambdas, keys and NN state are untouched: the window (rows -4..h+3, columns -4..w+3 around
// mv_int) becomes picture 0 with the PU at (4, 4), the key its key block, the MV predictor is
// shifted by 4*mv_int as for the server.  Latency: a few launches and copies per call.
static int frac_dif_single10(fme_ctx* c, int lossless, const int16_t* key, int key_stride, int w, int h,
                             const int16_t* ref, int ref_stride, int mv_int_x, int mv_int_y, int px, int py,
                             double motion_lambda, int16_t* half_xy, int16_t* qtr_xy, uint32_t* cost) {
  if (!c->single10) {
    fme_config cfg = c->cfg;
    cfg.nn_mode = 0;
    cfg.max_jobs = 64;
    fme_ctx* s = nullptr;
    const int rc = fme_create(c->device, &cfg, &s);
    if (rc) return rc;
    c->single10 = s;
    HIP_TRY(hipStreamCreateWithFlags(&c->single10_stream, hipStreamNonBlocking));
  }
  fme_ctx* s = c->single10;
  const int pw = w + 8, ph = h + 8;
  const int maxv = (1 << c->cfg.bit_depth) - 1;
  std::vector<uint16_t> win((size_t)pw * ph);
  for (int y = 0; y < ph; y++) {
    const int16_t* src = ref + (ptrdiff_t)(mv_int_y - 4 + y) * ref_stride + (mv_int_x - 4);
    for (int x = 0; x < pw; x++) win[(size_t)y * pw + x] = (uint16_t)std::min(maxv, std::max(0, (int)src[x]));
  }
  std::vector<int16_t> kb((size_t)w * h);
  for (int y = 0; y < h; y++) std::memcpy(&kb[(size_t)y * w], key + (ptrdiff_t)y * key_stride, (size_t)w * sizeof(int16_t));
  int rc = fme_set_picture(s, 0, reinterpret_cast<const uint8_t*>(win.data()), pw, pw, ph, c->single10_stream);
  if (!rc) rc = fme_set_motion_lambda(s, 0, motion_lambda);
  if (!rc) rc = fme_set_keys(s, kb.data(), kb.size(), c->single10_stream);
  if (rc) return rc;
  fme_job j{};
  j.x = 4;
  j.y = 4;
  j.w = (uint8_t)w;
  j.h = (uint8_t)h;
  j.org_id = 0;
  j.ref_id = 0;
  j.mvp_x = (int16_t)px;
  j.mvp_y = (int16_t)py;
  j.lt_x = j.lt_y = -1;
  j.rb_x = j.rb_y = 1;
  j.flags = lossless ? FME_JOB_LOSSLESS : 0;
  j.key_offset = 0;
  fme_result r{};
  rc = fme_refine(s, &j, &r, 1, c->single10_stream);
  if (rc) return rc;
  if (r.status & FME_RES_REJECTED) return fail(FME_E_INVALID, "fme_frac_dif_single: job rejected");
  half_xy[0] = r.half_x;
  half_xy[1] = r.half_y;
  qtr_xy[0] = r.qtr_x;
  qtr_xy[1] = r.qtr_y;
  *cost = r.frac_cost;
  return FME_OK;
}

int fme_frac_dif_single(fme_ctx* c, int lossless, const int16_t* key, int key_stride, int w, int h,
                        const int16_t* ref, int ref_stride, int mv_int_x, int mv_int_y, int mvp_x,
                        int mvp_y, double motion_lambda, int16_t* half_xy, int16_t* qtr_xy,
                        uint32_t* cost) {
  if (!c || !key || !ref || !half_xy || !qtr_xy || !cost) return fail(FME_E_INVALID, "fme_frac_dif_single: null argument");
  const int cls = class_of(w, h);
  if (cls < 0) return fail(FME_E_UNSUPPORTED, "fme_frac_dif_single: %dx%d", w, h);
  const int px = mvp_x - 4 * mv_int_x, py = mvp_y - 4 * mv_int_y;
  if (px < -32768 || px > 32767 || py < -32768 || py > 32767) return fail(FME_E_INVALID, "fme_frac_dif_single: predictor out of range");
  HIP_TRY(hipSetDevice(c->device));
  if (c->cfg.bit_depth > 8)
    return frac_dif_single10(c, lossless, key, key_stride, w, h, ref, ref_stride, mv_int_x, mv_int_y, px, py,
                             motion_lambda, half_xy, qtr_xy, cost);
  int rc = srv_open(c);
  if (rc) return rc;
  SrvBox* b = c->box;
  const uint32_t seq = c->srv_done + 1;   // the call's sequence number (srv_call)
  const int pw = w + 8, ph = h + 8, win_bytes = pw * ph, bytes = win_bytes + 2 * w * h;
  // small PUs: window and key ride in the request blocks (kSrvTagged), 12 bytes per block
  const bool tagged = bytes <= kSrvTagBytes;
  alignas(16) uint8_t stream[kSrvTagBytes + 12];
  uint8_t* wdst = tagged ? stream : b->win;
  int16_t* kdst = tagged ? reinterpret_cast<int16_t*>(stream + win_bytes) : b->key;
  for (int y = 0; y < h; y++) std::memcpy(kdst + y * w, key + (ptrdiff_t)y * key_stride, (size_t)w * sizeof(int16_t));
  for (int y = 0; y < ph; y++) {
    const int16_t* src = ref + (ptrdiff_t)(mv_int_y - 4 + y) * ref_stride + (mv_int_x - 4);
    uint8_t* dst = wdst + y * pw;
    for (int x = 0; x < pw; x++) dst[x] = (uint8_t)std::min(255, std::max(0, (int)src[x]));
  }
  if (tagged)
    for (int p = 0; 12 * p < bytes; p++) {
      std::memcpy(&b->req[2 + p][1], stream + 12 * p, 12);
      __atomic_store_n(&b->req[2 + p][0], seq, __ATOMIC_RELEASE);
    }
  uint32_t mlw[2];
  std::memcpy(mlw, &motion_lambda, sizeof(mlw));
  b->req[1][1] = mlw[0];
  b->req[1][2] = mlw[1];
  __atomic_store_n(&b->req[1][0], seq, __ATOMIC_RELEASE);
  b->req[0][1] = (uint32_t)kSrvFrac | ((lossless || !c->cfg.use_hadamard) ? (uint32_t)kSrvSad : 0u) |
                 (tagged ? (uint32_t)kSrvTagged : 0u) | (c->srv_marks ? (uint32_t)kSrvMarks : 0u) |
                 ((uint32_t)(w - 1) << 8) | ((uint32_t)(h - 1) << 16);
  b->req[0][2] = (uint32_t)(uint16_t)px | ((uint32_t)(uint16_t)py << 16);
  rc = srv_call(c, false);
  if (rc) return rc;
  const uint32_t hq = b->res[2];
  half_xy[0] = (int16_t)(int8_t)(hq & 0xFF);
  half_xy[1] = (int16_t)(int8_t)((hq >> 8) & 0xFF);
  qtr_xy[0] = (int16_t)(int8_t)((hq >> 16) & 0xFF);
  qtr_xy[1] = (int16_t)(int8_t)(hq >> 24);
  *cost = b->res[1];
  return FME_OK;
}

int fme_nn_pred_single(fme_ctx* c, const uint32_t* e, uint32_t cc, int pu_h, int pu_w, int* nn_class, int16_t* out4) {
  if (!c || !e || !nn_class) return fail(FME_E_INVALID, "fme_nn_pred_single: null argument");
  const bool deep = c->cfg.nn_mode == 2;
  if (deep ? !c->net_loaded : !c->nn_loaded) return fail(FME_E_STATE, "fme_nn_pred_single: no weights loaded");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if (!deep) {   // the master net: the server, weights in its LDS
    rc = srv_open(c);
    if (rc) return rc;
    const uint32_t in[12] = {e[0], e[1], e[2], e[3], e[4], e[5], e[6], e[7], cc, (uint32_t)pu_h, (uint32_t)pu_w, 0u};
    const uint32_t seq = c->srv_done + 1;   // the call's sequence number (srv_call)
    for (int b = 1; b < 5; b++) {   // each block's inputs, then its sequence word
      for (int k = 0; k < 3; k++) c->box->req[b][1 + k] = in[3 * (b - 1) + k];
      __atomic_store_n(&c->box->req[b][0], seq, __ATOMIC_RELEASE);
    }
    c->box->req[0][1] = kSrvNn | (c->srv_marks ? (uint32_t)kSrvMarks : 0u);
    rc = srv_call(c, true);
    if (rc) return rc;
    *nn_class = (int)c->box->res[1];
  } else {
  // a resident server (a FracDIF call just before) would hold this launch up on a hardware queue
  // its stream shares until its idle exit: stop it first, as the batch entry points do
  rc = srv_stop(c);
  if (!rc) rc = ensure_stage(c);
  if (rc) return rc;
  // inputs in the kernel argument, the class and the completion word through mapped host memory:
  // one launch, a spin on the completion word
  NnIn11 in{};
  for (int s = 0; s < 8; s++) in.v[s] = e[s];
  in.v[8] = cc;
  in.v[9] = (uint32_t)pu_h;
  in.v[10] = (uint32_t)pu_w;
  int32_t* d_out = reinterpret_cast<int32_t*>(c->stage_dev + offsetof(SingleStage, nn_out));
  uint32_t* d_flag = reinterpret_cast<uint32_t*>(c->stage_dev + offsetof(SingleStage, flag));
  const uint32_t seq = ++c->single_seq;
  HIP_TRY(launch_nn_deep_single(c->net, c->d_net.p, in, d_out, d_flag, seq, c->single_stream));
  rc = single_wait(c, seq);
  if (rc) return rc;
  *nn_class = c->stage->nn_out[0];
  }
  const int cls = *nn_class;
  if (out4) {
    // MVX_HALF, MVX_QRTER, MVY_HALF, MVY_QRTER of the switch at TEncSearch.cpp:136-193:
    // the half/quarter split of the offset (cls % 7 - 3, cls / 7 - 3) with the quarter part
    // in {-1, 0, 1} and x = 2 * half + quarter.
    const int ox = cls % 7 - 3, oy = cls / 7 - 3;
    auto split = [](int o, int16_t& hf, int16_t& qt) {
      static const int8_t H[7] = {-1, -1, 0, 0, 0, 1, 1}, Q[7] = {-1, 0, -1, 0, 1, 0, 1};
      hf = H[o + 3];
      qt = Q[o + 3];
    };
    split(ox, out4[0], out4[1]);
    split(oy, out4[2], out4[3]);
  }
  return FME_OK;
}

int fme_single_last_device_us(fme_ctx* c, float* us, int count) {
  if (!c || (count > 0 && !us)) return fail(FME_E_INVALID, "fme_single_last_device_us: null argument");
  const double k = 1000.0 / (double)c->srv_khz;
  if (count > 1) c->srv_marks = true;   // checkpoints cost wall-clock reads: recorded once asked for
  for (int i = 0; i < count && i < 5; i++)
    us[i] = !c->box ? 0.0f : (float)((double)(i == 0 ? c->box->res[3] : c->box->marks[i - 1]) * k);
  return FME_OK;
}

int fme_search_kernel_of_shape(int width, int height) {
  for (int k = 0; k < kNumClasses; k++)
    if (kClassW[k] == width && kClassH[k] == height) {
      return 0;   // every shape runs in the lane kernel
    }
  return -1;
}

// ---- motion compensation ---------------------------------------------------------------------
static const char* mc_job_problem(const fme_ctx* c, const fme_mc_job& j, int width, int height) {
  if (j.w < 4 || j.h < 4 || j.w > 64 || j.h > 64 || (j.w & 3) || (j.h & 3)) return "PU size";
  if (!(j.flags & (FME_MC_L0 | FME_MC_L1)) || (j.flags & ~(FME_MC_L0 | FME_MC_L1 | FME_MC_WP))) return "list flags";
  if ((int)j.x + j.w > width || (int)j.y + j.h > height) return "PU outside the picture";
  for (int l = 0; l < 2; l++) {
    if (!(j.flags & (1u << l))) continue;
    if (j.ref_id[l] >= FME_MAX_PICTURES) return "reference id";
    const PicDesc& p = c->pics[j.ref_id[l]];
    if (!p.luma || !p.cb || !p.cr) return "reference picture without luma + chroma";
    if (p.width != width || p.height != height) return "reference picture dimensions";
  }
  return nullptr;
}

static int mc_launch(fme_ctx* c, const fme_mc_job* d_jobs, int n, uint8_t* y, int ys, uint8_t* cb, uint8_t* cr,
                     int cs, int width, int height, hipStream_t s) {
  HIP_TRY(c->d_mc_invalid.reserve(1));
  HIP_TRY(hipMemsetAsync(c->d_mc_invalid.p, 0, sizeof(int32_t), s));
  if (int e = sync_tables(c, s)) return e;
  if (!c->wp_init) {   // the default weights: 1 << 0, offset 0
    for (auto& l : c->h_wp)
      for (auto& p : l)
        for (auto& q : p) q = fme_wp_param{1, 0, 0, {0, 0, 0}};
    c->wp_init = true;
  }
  if (c->wp_dirty) {   // (pageable source: the runtime stages it before returning)
    HIP_TRY(c->d_mc_wp.reserve(sizeof(c->h_wp) / sizeof(fme_wp_param)));
    HIP_TRY(hipMemcpyAsync(c->d_mc_wp.p, c->h_wp, sizeof(c->h_wp), hipMemcpyHostToDevice, s));
    c->wp_dirty = false;
  }
  McArgs a{};
  a.wp = c->d_mc_wp.p;
  a.jobs = d_jobs;
  a.pics = c->d_pics.p;
  a.y = y;
  a.cb = cb;
  a.cr = cr;
  a.invalid = c->d_mc_invalid.p;
  a.n = n;
  a.y_stride = ys;
  a.c_stride = cs;
  a.width = width;
  a.height = height;
  a.bit_depth = c->cfg.bit_depth;   // 10: uint16 planes, strides in samples (k_mc10)
  if (c->profiling) {
    if (!c->ev_mc[0]) {
      HIP_TRY(hipEventCreate(&c->ev_mc[0]));
      HIP_TRY(hipEventCreate(&c->ev_mc[1]));
    }
    HIP_TRY(hipEventRecord(c->ev_mc[0], s));
  }
  HIP_TRY(launch_mc(a, s));
  if (c->profiling) HIP_TRY(hipEventRecord(c->ev_mc[1], s));
  c->mc_timed = c->profiling;
  return FME_OK;
}

static int mc_check_planes(const void* y, int ys, const void* cb, const void* cr, int cs, int width, int height) {
  if (!y || !cb || !cr) return fail(FME_E_INVALID, "motion compensation: null plane");
  if (width <= 0 || height <= 0 || (width & 1) || (height & 1) || ys < width || cs < width / 2)
    return fail(FME_E_INVALID, "motion compensation: geometry %dx%d strides %d/%d", width, height, ys, cs);
  return FME_OK;
}

int fme_motion_compensate(fme_ctx* c, const fme_mc_job* jobs, int n, uint8_t* y, int ys, uint8_t* cb, uint8_t* cr,
                          int cs, int width, int height, void* stream) {
  if (!c || (n > 0 && !jobs) || n < 0) return fail(FME_E_INVALID, "fme_motion_compensate: bad argument");
  if (int e = mc_check_planes(y, ys, cb, cr, cs, width, height)) return e;
  for (int i = 0; i < n; i++)
    if (const char* why = mc_job_problem(c, jobs[i], width, height))
      return fail(FME_E_INVALID, "fme_motion_compensate: job %d: %s", i, why);
  if (n == 0) return FME_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t bps = c->cfg.bit_depth > 8 ? 2 : 1;   // bytes per sample (10-bit: uint16 planes)
  const size_t ly = (size_t)width * height * bps, lc = ly / 4;
  HIP_TRY(c->d_mc_jobs.reserve(n));
  HIP_TRY(c->d_mc_planes.reserve(ly + 2 * lc));
  uint8_t* dy = c->d_mc_planes.p;
  uint8_t* dcb = dy + ly;
  uint8_t* dcr = dcb + lc;
  const int cw = width / 2, ch = height / 2;
  HIP_TRY(hipMemcpyAsync(c->d_mc_jobs.p, jobs, n * sizeof(fme_mc_job), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpy2DAsync(dy, width * bps, y, ys * bps, width * bps, height, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpy2DAsync(dcb, cw * bps, cb, cs * bps, cw * bps, ch, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpy2DAsync(dcr, cw * bps, cr, cs * bps, cw * bps, ch, hipMemcpyHostToDevice, s));
  if (int e = mc_launch(c, c->d_mc_jobs.p, n, dy, width, dcb, dcr, cw, width, height, s)) return e;
  HIP_TRY(hipMemcpy2DAsync(y, ys * bps, dy, width * bps, width * bps, height, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpy2DAsync(cb, cs * bps, dcb, cw * bps, cw * bps, ch, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpy2DAsync(cr, cs * bps, dcr, cw * bps, cw * bps, ch, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return FME_OK;
}

int fme_motion_compensate_device(fme_ctx* c, const fme_mc_job* d_jobs, int n, uint8_t* d_y, int ys, uint8_t* d_cb,
                                 uint8_t* d_cr, int cs, int width, int height, void* stream) {
  if (!c || (n > 0 && !d_jobs) || n < 0) return fail(FME_E_INVALID, "fme_motion_compensate_device: bad argument");
  if (int e = mc_check_planes(d_y, ys, d_cb, d_cr, cs, width, height)) return e;
  HIP_TRY(hipSetDevice(c->device));
  return mc_launch(c, d_jobs, n, d_y, ys, d_cb, d_cr, cs, width, height, static_cast<hipStream_t>(stream));
}

int fme_mc_invalid_count(fme_ctx* c) {
  if (!c) return fail(FME_E_INVALID, "fme_mc_invalid_count: null ctx");
  if (!c->d_mc_invalid.p) return 0;
  HIP_TRY(hipSetDevice(c->device));
  int32_t v = 0;
  {
    const int rc = drain_ctx(c);   // this context's streams only
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpy(&v, c->d_mc_invalid.p, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

int fme_set_wp(fme_ctx* c, int list, int ref_id, const fme_wp_param* p) {
  if (!c || !p) return fail(FME_E_INVALID, "fme_set_wp: null argument");
  if (list < 0 || list > 1 || ref_id < 0 || ref_id >= FME_MAX_PICTURES)
    return fail(FME_E_INVALID, "fme_set_wp: list %d reference %d", list, ref_id);
  for (int k = 0; k < 3; k++)
    if (p[k].log2_denom > 7) return fail(FME_E_INVALID, "fme_set_wp: log2 denominator %d", (int)p[k].log2_denom);
  if (!c->wp_init) {
    for (auto& l : c->h_wp)
      for (auto& q : l)
        for (auto& r : q) r = fme_wp_param{1, 0, 0, {0, 0, 0}};
    c->wp_init = true;
  }
  for (int k = 0; k < 3; k++) c->h_wp[list][ref_id][k] = p[k];
  c->wp_dirty = true;
  return FME_OK;
}

int fme_mc_last_ms(fme_ctx* c, float* ms) {
  if (!c || !ms) return fail(FME_E_INVALID, "fme_mc_last_ms: null argument");
  if (!c->mc_timed) return fail(FME_E_STATE, "fme_mc_last_ms: no profiled motion compensation");
  HIP_TRY(hipEventSynchronize(c->ev_mc[1]));
  HIP_TRY(hipEventElapsedTime(ms, c->ev_mc[0], c->ev_mc[1]));
  return FME_OK;
}

int fme_set_profiling(fme_ctx* c, int enable) {
  if (!c) return fail(FME_E_INVALID, "fme_set_profiling: null ctx");
  HIP_TRY(hipSetDevice(c->device));
  if (enable && !c->events_made) {
    for (auto& set : c->ev)
      for (auto& e : set) HIP_TRY(hipEventCreate(&e));
    c->events_made = true;
  }
  if (!enable) {
    const int rc = harvest_events(c, true);
    if (rc) return rc;
  }
  c->profiling = enable != 0;
  return FME_OK;
}

int fme_last_timings(fme_ctx* c, float* ms, int count) {
  if (!c || !ms || count < 0) return fail(FME_E_INVALID, "fme_last_timings: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const int rc = harvest_events(c, true);
  if (rc) return rc;
  if (!c->timed) return fail(FME_E_STATE, "fme_last_timings: no profiled batch");
  for (int i = 0; i < count && i < FME_NUM_TIMINGS; i++) ms[i] = c->last_ms[i];
  return FME_OK;
}

int fme_accumulated_timings(fme_ctx* c, double* ms, int count, int reset) {
  if (!c || (count > 0 && !ms) || count < 0) return fail(FME_E_INVALID, "fme_accumulated_timings: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const int rc = harvest_events(c, true);
  if (rc) return rc;
  const int n = c->acc_batches;
  for (int i = 0; i < count && i < FME_NUM_TIMINGS; i++) ms[i] = c->acc_ms[i];
  if (reset) {
    for (double& v : c->acc_ms) v = 0.0;
    c->acc_batches = 0;
  }
  return n;
}

}  // extern "C"

// ---- predInterSearch's P-slice PU / reference loop ---------------------------
namespace {

// xGetMvpIdxBits (TEncSearch.cpp:4258-4284); m_auiMVPIdxCost[idx][num] (412-425)
uint32_t mvp_idx_bits(int idx, int num) {
  if (num == 1) return 0;
  if (idx == 0) return 1;
  return 1u + (uint32_t)(idx - 1) + (num - 1 > idx ? 1u : 0u);
}
// xGetBlkBits (TEncSearch.cpp:4286-4333), P slice: uiBlkBit[0]
uint32_t blk_bits_p(int part_size) {
  return (part_size == FME_PART_2Nx2N || part_size == FME_PART_NxN) ? 1u : 3u;
}
// TComRdCost::xGetExpGolombNumberOfBits (TComRdCost.cpp:172-185)
uint32_t eg_bits(int v) {
  uint32_t t = v <= 0 ? ((uint32_t)(-v) << 1) + 1u : (uint32_t)v << 1;
  uint32_t len = 1;
  while (t != 1) {
    t >>= 1;
    len += 2;
  }
  return len;
}
// TComRdCost::getCost (TComRdCost.h:165)
uint32_t rd_cost(double ml, uint32_t bits) { return (uint32_t)((ml * (double)bits) / 65536.0); }
// TComDataCU::clipMv (TComDataCU.cpp:2773-2786), max CU 64, quarter-pel
void clip_qpel(int& x, int& y, int pw, int ph, int cu_x, int cu_y) {
  x = std::min((pw + 8 - cu_x - 1) << 2, std::max((-64 - 8 - cu_x + 1) * 4, x));
  y = std::min((ph + 8 - cu_y - 1) << 2, std::max((-64 - 8 - cu_y + 1) * 4, y));
}
int round4(int v) { return (v + 2) >> 2; }   // TComMv::divideByPowerOf2(2)

// xGetBlkBits (TEncSearch.cpp:4286-4333), B slice: uiBlkBit[0..2]
void blk_bits_b(int part_size, int part_idx, int last_mode, uint32_t out[3]) {
  static const uint32_t hor[2][3][3] = {{{0, 0, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {7, 5, 7}, {6, 6, 6}}};
  static const uint32_t ver[2][3][3] = {{{0, 2, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {5, 5, 7}, {6, 6, 6}}};
  if (part_size == FME_PART_2Nx2N || part_size == FME_PART_NxN) {
    out[0] = 3; out[1] = 3; out[2] = 5;
    return;
  }
  const bool hz = part_size == FME_PART_2NxN || part_size == FME_PART_2NxnU || part_size == FME_PART_2NxnD;
  const uint32_t* t = hz ? hor[part_idx][last_mode] : ver[part_idx][last_mode];
  out[0] = t[0]; out[1] = t[1]; out[2] = t[2];
}
uint32_t ref_bits(int k, int num_refs) {   // TEncSearch.cpp:3792-3800
  return num_refs <= 1 ? 0u : (uint32_t)k + 1u - (k == num_refs - 1 ? 1u : 0u);
}
// xCheckBestMVP (TEncSearch.cpp:4344-4394), cost scale 0
void check_best_mvp(double ml, const int16_t cand[2][2], int n_cand, int mx, int my, int& idx, uint32_t& bits,
                    uint32_t& cost) {
  if (n_cand < 2) return;
  const int org_bits = (int)(eg_bits(mx - cand[idx][0]) + eg_bits(my - cand[idx][1]) + mvp_idx_bits(idx, 2));
  int best_bits = org_bits, best_idx = idx;
  for (int m = 0; m < n_cand; m++) {
    if (m == idx) continue;
    const int b = (int)(eg_bits(mx - cand[m][0]) + eg_bits(my - cand[m][1]) + mvp_idx_bits(m, 2));
    if (b < best_bits) {
      best_bits = b;
      best_idx = m;
    }
  }
  if (best_idx != idx) {
    idx = best_idx;
    const uint32_t org_total = bits;
    bits = org_total - (uint32_t)org_bits + (uint32_t)best_bits;
    cost = (cost - rd_cost(ml, org_total)) + rd_cost(ml, bits);
  }
}
// xMotionEstimation's cost tail (TEncSearch.cpp:4594-4597) re-priced for bits_in + extra bits: the
// searches do not read bits_in, so a job run with a provisional bits_in gives the exact result.
uint32_t tail_cost(double ml, const fme_result& r, uint32_t bits_in, uint32_t extra, double fw) {
  const uint32_t mvb = r.bits - bits_in;
  const double v = floor(fw * ((double)r.frac_cost - (double)rd_cost(ml, mvb))) + (double)rd_cost(ml, r.bits + extra);
  return (uint32_t)(int64_t)v;
}

bool valid_pu_shape(int w, int h) {
  for (int k = 0; k < kNumClasses; k++)
    if (kClassW[k] == w && kClassH[k] == h) return true;
  return false;
}

}  // namespace

namespace {
struct BPu {
  uint32_t mb[3];
  uint32_t cost[2], bits[2];
  int16_t mv[2][2];
  int ridx[2];
  int mvpi[2][FME_MAX_REFS];
  int16_t mvt[2][FME_MAX_REFS][2];
  uint32_t cost_v1, bits_v1;
  int16_t mv_v1[2];
  int ridx_v1;
  int L;            // list of the current bi-pred iteration
  uint32_t mot[2];  // uiMotBits
  int bi0;          // first bi job of this request in the round's list
  int stage;        // 0 waiting, 1 bi-pred iteration issued, 2 decided, 3 next iteration due
  int last_mode;    // uiLastMode after this request's decision
  // bi-pred iteration state (3871-4022)
  int it, niter;
  int16_t mvbi[2][2];
  int ridxbi[2];
  int mvpibi[2][FME_MAX_REFS];
  uint32_t cost_bi, bits_bi;
  int ps_ref[2];          // m_acYuvPred[l]: the reference and MV list l's stored prediction used
  int16_t ps_mv[2][2];
  int bip_ref, bip_mvp;   // bestBiPRefIdxL1, bestBiPMvpL1 (MvdL1ZeroFlag)
};

int two_part(int part_size) { return part_size != FME_PART_2Nx2N && part_size != FME_PART_NxN; }
int num_parts(int part_size) { return part_size == FME_PART_2Nx2N ? 1 : (part_size == FME_PART_NxN ? 4 : 2); }
}  // namespace

extern "C" {

// xGetTemplateCost (TEncSearch.cpp:4397-4436) of every AMVP candidate of every request, one launch:
// costs[(i * FME_MAX_REFS + k) * 2 + m]; 0xFFFFFFFF for k >= num_refs or m >= n_cand[k].
int fme_template_costs(fme_ctx* c, const fme_pu_req* reqs, uint32_t* costs, int n, void* stream) {
  if (!c || (n > 0 && (!reqs || !costs))) return fail(FME_E_INVALID, "fme_template_costs: null argument");
  if (n <= 0) return n == 0 ? FME_OK : fail(FME_E_INVALID, "fme_template_costs: n = %d", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<AmvpTask> tasks;
  std::vector<int> slot;
  for (int i = 0; i < n; i++) {
    const fme_pu_req& q = reqs[i];
    const PicDesc& org = c->pics[q.org_id < FME_MAX_PICTURES ? q.org_id : 0];
    if (!valid_pu_shape(q.w, q.h) || q.num_refs < 1 || q.num_refs > FME_MAX_REFS || q.org_id >= FME_MAX_PICTURES ||
        !org.luma || q.x + q.w > org.width || q.y + q.h > org.height || q.lambda_id >= FME_MAX_LAMBDAS ||
        !c->lambda_set[q.lambda_id])
      return fail(FME_E_INVALID, "fme_template_costs: request %d invalid", i);
    for (int k = 0; k < FME_MAX_REFS; k++)
      for (int m = 0; m < 2; m++) {
        costs[((size_t)i * FME_MAX_REFS + k) * 2 + m] = 0xFFFFFFFFu;
        if (k >= q.num_refs || m >= q.n_cand[k]) continue;
        if (q.ref_id[k] >= FME_MAX_PICTURES || !c->pics[q.ref_id[k]].luma || q.n_cand[k] > 2 ||
            c->pics[q.ref_id[k]].width != org.width || c->pics[q.ref_id[k]].height != org.height)
          return fail(FME_E_INVALID, "fme_template_costs: request %d reference %d invalid", i, k);
        slot.push_back((i * FME_MAX_REFS + k) * 2 + m);
        tasks.push_back(AmvpTask{q.x, q.y, q.w, q.h, q.org_id, q.ref_id[k], q.cu_x, q.cu_y, q.cand[k][m][0],
                                 q.cand[k][m][1]});
      }
  }
  if (tasks.empty()) return FME_OK;
  int rc = sync_tables(c, s);
  if (rc) return rc;
  std::vector<uint32_t> tsad(tasks.size());
  HIP_TRY(c->d_amvp.reserve(tasks.size()));
  HIP_TRY(c->d_amvp_sad.reserve(tasks.size()));
  HIP_TRY(hipMemcpyAsync(c->d_amvp.p, tasks.data(), tasks.size() * sizeof(AmvpTask), hipMemcpyHostToDevice, s));
  AmvpArgs aa{c->d_amvp.p, c->d_pics.p, c->d_amvp_sad.p, (int32_t)tasks.size(), c->cfg.bit_depth};
  HIP_TRY(launch_amvp_sad(aa, s));
  HIP_TRY(hipMemcpyAsync(tsad.data(), c->d_amvp_sad.p, tasks.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t t = 0; t < tasks.size(); t++) {
    const int i = slot[t] / (2 * FME_MAX_REFS), m = slot[t] & 1;
    const double ml = c->mlambda[reqs[i].lambda_id];
    // calcRdCost(bits, SAD, DF_SAD) with bits = m_auiMVPIdxCost[m][AMVP_MAX_NUM_CANDS] (4423-4433)
    costs[slot[t]] = (uint32_t)((double)tsad[t] + ((double)mvp_idx_bits(m, 2) * ml) / 65536.0);
  }
  return FME_OK;
}

int fme_build_bipred_keys(fme_ctx* c, const fme_bikey_req* reqs, int n, size_t key_count, void* stream) {
  static_assert(sizeof(fme_bikey_req) == sizeof(BiKeyTask), "fme_bikey_req is the kernel's task record");
  if (!c || (n > 0 && !reqs)) return fail(FME_E_INVALID, "fme_build_bipred_keys: null argument");
  if (n < 0) return fail(FME_E_INVALID, "fme_build_bipred_keys: n = %d", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i = 0; i < n; i++) {
    const fme_bikey_req& q = reqs[i];
    const PicDesc& org = c->pics[q.org_id < FME_MAX_PICTURES ? q.org_id : 0];
    const PicDesc& ref = c->pics[q.ref_id < FME_MAX_PICTURES ? q.ref_id : 0];
    if (!valid_pu_shape(q.w, q.h) || q.org_id >= FME_MAX_PICTURES || q.ref_id >= FME_MAX_PICTURES || !org.luma ||
        !ref.luma || ref.width != org.width || ref.height != org.height || q.x + q.w > org.width ||
        q.y + q.h > org.height || q.key_offset < 0 || (q.key_offset & 3) ||
        (size_t)q.key_offset + (size_t)q.w * q.h > key_count || (q.flags & ~FME_PU_CLIP_BIPRED))
      return fail(FME_E_INVALID, "fme_build_bipred_keys: request %d invalid", i);
  }
  int rc = sync_tables(c, s);
  if (!rc) rc = grow_keys(c, key_count);
  if (rc) return rc;
  c->n_keys = key_count;
  HIP_TRY(hipMemsetAsync(c->d_key_invalid.p, 0, sizeof(int32_t), s));   // host-validated: the keys are good
  if (n == 0) return hipStreamSynchronize(s) == hipSuccess ? FME_OK : fail(FME_E_DEVICE, "fme_build_bipred_keys: sync");
  HIP_TRY(c->d_bikey.reserve((size_t)n));
  HIP_TRY(hipMemcpyAsync(c->d_bikey.p, reqs, (size_t)n * sizeof(BiKeyTask), hipMemcpyHostToDevice, s));
  BiKeyArgs ka{c->d_bikey.p, c->d_pics.p, c->d_keys.p, (int32_t)n, nullptr, (int64_t)key_count, c->cfg.bit_depth};
  HIP_TRY(launch_bi_key(ka, s));
  HIP_TRY(hipStreamSynchronize(s));
  return FME_OK;
}

// The frame replay's per-frame form: requests already in device memory, everything stream-ordered
// (no host synchronisation).  Validation runs in k_bi_key; a request that fails it is skipped and
// counted, and every later batch whose jobs read keys is rejected until keys are built again.
int fme_build_bipred_keys_device(fme_ctx* c, const fme_bikey_req* d_reqs, int n, size_t key_count, void* stream) {
  if (!c || (n > 0 && !d_reqs)) return fail(FME_E_INVALID, "fme_build_bipred_keys_device: null argument");
  if (n < 0) return fail(FME_E_INVALID, "fme_build_bipred_keys_device: n = %d", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = sync_tables(c, s);
  if (rc) return rc;
  rc = grow_keys(c, key_count);   // growing frees the old buffer: every queued batch finishes first
  if (rc) return rc;
  c->n_keys = key_count;
  HIP_TRY(hipMemsetAsync(c->d_key_invalid.p, 0, sizeof(int32_t), s));
  if (n == 0) return FME_OK;
  BiKeyArgs ka{reinterpret_cast<const BiKeyTask*>(d_reqs), c->d_pics.p, c->d_keys.p, (int32_t)n,
               c->d_key_invalid.p, (int64_t)key_count, c->cfg.bit_depth};
  HIP_TRY(launch_bi_key(ka, s));
  return FME_OK;
}

// The producers' integer searches by m_integerMv2Nx2N dependency level.  jobs / ext: pinned host
// arrays in request order; src[u]: the job whose post-EMI MV job u reads (-1: none); lvl[u] its
// level.  The jobs go to the device once, are reordered there by level (within a level the largest
// PUs first) for k_tz_level's launches, and come back in request order in c->d_jobs for the sub-pel
// pass; nothing returns to the host.
static int tz_levels_device(fme_ctx* c, const fme_job* jobs, const fme_tz_ext* ext, const std::vector<int>& src,
                            const std::vector<int>& lvl, int nj, int max_level, hipStream_t s) {
  if (nj <= 0) return FME_OK;
  // level order: blocks dispatch in index order, so the longest searches of a wide level start at once
  std::vector<int32_t>& off = c->pi_off;
  std::vector<int32_t>& fill = c->pi_fill;
  std::vector<int>& start = c->pi_start;
  off.assign((size_t)max_level + 2, 0);
  for (int u = 0; u < nj; u++) off[lvl[u] + 1]++;
  for (int l = 0; l <= max_level; l++) off[l + 1] += off[l];
  fill.assign(off.begin(), off.end() - 1);
  start.assign(64 * 64 + 2, 0);   // counting sort by area, descending
  for (int u = 0; u < nj; u++) start[64 * 64 - (int)jobs[u].w * jobs[u].h + 1]++;
  for (size_t a = 1; a < start.size(); a++) start[a] += start[a - 1];
  HIP_TRY(c->h_pi_idx.reserve((size_t)2 * nj));
  HIP_TRY(c->h_pi_psrc.reserve((size_t)nj));
  int32_t* const order = c->h_pi_idx.p;        // level position -> job
  int32_t* const pos = c->h_pi_idx.p + nj;     // job -> level position
  {
    std::vector<int>& byarea = c->pi_byarea;
    byarea.resize((size_t)nj);
    for (int u = 0; u < nj; u++) byarea[start[64 * 64 - (int)jobs[u].w * jobs[u].h]++] = u;
    for (int u : byarea) {
      pos[u] = fill[lvl[u]]++;
      order[pos[u]] = u;
    }
  }
  int32_t* const psrc = c->h_pi_psrc.p;
  par_for(nj, [&](int lo, int hi) {
    for (int q = lo; q < hi; q++) {
      const int u = order[q];
      psrc[q] = ((ext[u].flags & FME_TZ_PRED2NX2N) && src[u] >= 0) ? pos[src[u]] : -1;
    }
  });
  HIP_TRY(c->d_jobs.reserve(nj));
  HIP_TRY(c->d_tz_ext.reserve(nj));
  HIP_TRY(c->d_pi_jobs.reserve(nj));
  HIP_TRY(c->d_pi_ext.reserve(nj));
  HIP_TRY(c->d_pi_idx.reserve((size_t)2 * nj));
  HIP_TRY(c->d_ch_i32.reserve(nj));
  HIP_TRY(c->d_tz_emi.reserve((size_t)2 * nj));
  HIP_TRY(hipMemcpyAsync(c->d_jobs.p, jobs, (size_t)nj * sizeof(fme_job), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_tz_ext.p, ext, (size_t)nj * sizeof(fme_tz_ext), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_pi_idx.p, order, (size_t)2 * nj * sizeof(int32_t), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->d_ch_i32.p, psrc, (size_t)nj * sizeof(int32_t), hipMemcpyHostToDevice, s));
  HIP_TRY(launch_gather_jobs(c->d_jobs.p, c->d_tz_ext.p, c->d_pi_idx.p, c->d_pi_jobs.p, c->d_pi_ext.p, nj, s));
  {
    TzArgs ta{};
    ta.a.jobs = c->d_pi_jobs.p;
    ta.a.keys = c->d_keys.p;
    ta.a.n_keys = (int64_t)c->n_keys;
    ta.a.key_invalid = c->d_key_invalid.p;
    ta.a.mlambda = c->d_mlambda.p;
    ta.a.pics = c->d_pics.p;
    ta.a.n = nj;
    ta.a.use_hadamard = c->cfg.use_hadamard ? 1 : 0;
    ta.a.fen = c->cfg.fast_inter_mode;
    ta.jobs_out = c->d_pi_jobs.p;
    ta.ext = c->d_pi_ext.p;
    ta.ext_stride = (int)sizeof(fme_tz_ext);
    ta.emi_mv = c->d_tz_emi.p;
    const TzChain ch{c->d_ch_i32.p, max_level + 1};
    HIP_TRY(launch_tz_levels(ta, ch, off.data(), c->cfg.bit_depth, s));
  }
  // the searched jobs back in request order for the sub-pel pass, on the device
  HIP_TRY(launch_gather_jobs(c->d_pi_jobs.p, nullptr, c->d_pi_idx.p + nj, c->d_jobs.p, nullptr, nj, s));
  return FME_OK;
}

// Phase clock of the producers (fme_pred_inter_phases): lap(k) adds the time since the last lap to
// phase k.
struct PiClock {
  fme_ctx* c;
  std::chrono::steady_clock::time_point t0, t;
  explicit PiClock(fme_ctx* cc) : c(cc), t0(std::chrono::steady_clock::now()), t(t0) {
    for (double& v : c->pi_ms) v = 0.0;
  }
  void lap(int k) {
    const auto now = std::chrono::steady_clock::now();
    c->pi_ms[k] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
  ~PiClock() { c->pi_ms[7] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

static void pi_lap(PiClock* clk, int k) {
  if (clk) clk->lap(k);
}

int fme_pred_inter_phases(fme_ctx* c, double* ms, int count) {
  if (!c || (count > 0 && !ms)) return fail(FME_E_INVALID, "fme_pred_inter_phases: null argument");
  for (int i = 0; i < count && i < FME_PI_PHASES; i++) ms[i] = c->pi_ms[i];
  return FME_OK;
}

int fme_pred_inter_reset(fme_ctx* c) {
  if (!c) return fail(FME_E_INVALID, "fme_pred_inter_reset: null ctx");
  std::memset(c->int_mv_2n, 0, sizeof(c->int_mv_2n));
  return FME_OK;
}

// The requests run in call order as far as anything observable goes; the GPU sees them as
//   1. one AMVP template-cost launch over every (request, reference, candidate) with two candidates;
//   2. integer searches by dependency level: a request that reads m_integerMv2Nx2N[k] waits for the
//      level of the 2Nx2N request that last wrote it (per CTU the chain of 2Nx2N CUs in xCompressCU
//      order); the search kernels also run the EMI square step and return the post-EMI integer MV
//      that the 2Nx2N requests publish to the levels above;
//   3. one fme_refine over all jobs in request order (the NN's carried state as in the reference);
//   4. xCheckBestMVP and the reference choice on the host.
int fme_pred_inter_p(fme_ctx* c, const fme_pu_req* reqs, fme_pu_res* res, int n, void* stream) {
  if (!c || (n > 0 && (!reqs || !res))) return fail(FME_E_INVALID, "fme_pred_inter_p: null argument");
  if (n <= 0) return n == 0 ? FME_OK : fail(FME_E_INVALID, "fme_pred_inter_p: n = %d", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  PiClock clk(c);
  // ---- validation (nothing runs on a bad batch) ----
  for (int i = 0; i < n; i++) {
    const fme_pu_req& q = reqs[i];
    const PicDesc& org = c->pics[q.org_id < FME_MAX_PICTURES ? q.org_id : 0];
    if (!valid_pu_shape(q.w, q.h) || q.part_size > FME_PART_nRx2N || q.num_refs < 1 || q.num_refs > FME_MAX_REFS ||
        q.org_id >= FME_MAX_PICTURES || !org.luma || q.x + q.w > org.width || q.y + q.h > org.height ||
        q.lambda_id >= FME_MAX_LAMBDAS || !c->lambda_set[q.lambda_id] || (q.flags & ~FME_PU_LOSSLESS))
      return fail(FME_E_INVALID, "fme_pred_inter_p: request %d invalid (shape %dx%d, part %d, refs %d)", i, q.w, q.h,
                  q.part_size, q.num_refs);
    for (int k = 0; k < q.num_refs; k++) {
      if (q.ref_id[k] >= FME_MAX_PICTURES || !c->pics[q.ref_id[k]].luma || q.n_cand[k] < 1 || q.n_cand[k] > 2)
        return fail(FME_E_INVALID, "fme_pred_inter_p: request %d reference %d invalid", i, k);
      const PicDesc& r = c->pics[q.ref_id[k]];
      if (r.width != org.width || r.height != org.height)
        return fail(FME_E_INVALID, "fme_pred_inter_p: request %d reference %d size differs from the original", i, k);
    }
  }
  int rc = sync_tables(c, s);
  if (rc) return rc;
  // ---- 1. xEstimateMvPredAMVP template costs: two tasks per (request, reference) with two
  // candidates, built into pinned memory by the host threads ----
  std::vector<int>& base = c->pi_base;
  std::vector<int>& task_of = c->pi_task;
  base.resize((size_t)n + 1);
  base[0] = 0;
  for (int i = 0; i < n; i++) base[i + 1] = base[i] + reqs[i].num_refs;
  const int nj = base[n];
  task_of.resize((size_t)nj);
  int ntasks = 0;
  for (int i = 0; i < n; i++)
    for (int k = 0; k < reqs[i].num_refs; k++) {
      const bool two = reqs[i].n_cand[k] >= 2;
      task_of[base[i] + k] = two ? ntasks : -1;
      ntasks += two ? 2 : 0;
    }
  HIP_TRY(c->h_pi_tasks.reserve((size_t)ntasks));
  HIP_TRY(c->h_pi_tsad.reserve((size_t)ntasks));
  AmvpTask* const tasks = c->h_pi_tasks.p;
  const uint32_t* const tsad = c->h_pi_tsad.p;
  par_for(n, [&](int lo, int hi) {
    for (int i = lo; i < hi; i++) {
      const fme_pu_req& q = reqs[i];
      for (int k = 0; k < q.num_refs; k++) {
        const int t = task_of[base[i] + k];
        if (t < 0) continue;
        for (int m = 0; m < 2; m++)
          tasks[t + m] = AmvpTask{q.x, q.y, q.w, q.h, q.org_id, q.ref_id[k], q.cu_x, q.cu_y, q.cand[k][m][0],
                                  q.cand[k][m][1]};
      }
    }
  });
  clk.lap(0);
  if (ntasks > 0) {
    HIP_TRY(c->d_amvp.reserve((size_t)ntasks));
    HIP_TRY(c->d_amvp_sad.reserve((size_t)ntasks));
    HIP_TRY(hipMemcpyAsync(c->d_amvp.p, tasks, (size_t)ntasks * sizeof(AmvpTask), hipMemcpyHostToDevice, s));
    AmvpArgs aa{c->d_amvp.p, c->d_pics.p, c->d_amvp_sad.p, (int32_t)ntasks, c->cfg.bit_depth};
    HIP_TRY(launch_amvp_sad(aa, s));
    HIP_TRY(hipMemcpyAsync(c->h_pi_tsad.p, c->d_amvp_sad.p, (size_t)ntasks * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  clk.lap(1);
  // ---- jobs: one xMotionEstimation per (request, reference), in request order ----
  HIP_TRY(c->h_pi_jobs.reserve((size_t)nj));
  HIP_TRY(c->h_pi_ext.reserve((size_t)nj));
  fme_job* const jobs = c->h_pi_jobs.p;
  fme_tz_ext* const ext = c->h_pi_ext.p;
  std::vector<uint8_t>& amvp_idx = c->pi_amvp_idx;
  amvp_idx.resize((size_t)nj);
  par_for(n, [&](int lo, int hi) {
    for (int i = lo; i < hi; i++) {
      const fme_pu_req& q = reqs[i];
      const PicDesc& org = c->pics[q.org_id];
      const double ml = c->mlambda[q.lambda_id];
      const int range = q.search_range ? q.search_range : 64;
      for (int k = 0; k < q.num_refs; k++) {
        const int jx = base[i] + k;
        int idx = 0;
        if (task_of[jx] >= 0) {   // uiBestCost > uiTmpCost: the first least cost wins
          uint32_t best = 0xFFFFFFFFu;
          for (int m = 0; m < 2; m++) {
            const uint32_t cost =
                (uint32_t)((double)tsad[task_of[jx] + m] + ((double)mvp_idx_bits(m, 2) * ml) / 65536.0);
            if (best > cost) {
              best = cost;
              idx = m;
            }
          }
        }
        amvp_idx[jx] = (uint8_t)idx;
        uint32_t bits = blk_bits_p(q.part_size);
        if (q.num_refs > 1) bits += (uint32_t)k + 1u - (k == q.num_refs - 1 ? 1u : 0u);
        bits += mvp_idx_bits(idx, 2);
        const int px = q.cand[k][idx][0], py = q.cand[k][idx][1];
        // xSetSearchRange (TEncSearch.cpp:4602-4624)
        int cx = px, cy = py;
        clip_qpel(cx, cy, org.width, org.height, q.cu_x, q.cu_y);
        int lx = cx - (range << 2), ly = cy - (range << 2), rx = cx + (range << 2), ry = cy + (range << 2);
        clip_qpel(lx, ly, org.width, org.height, q.cu_x, q.cu_y);
        clip_qpel(rx, ry, org.width, org.height, q.cu_x, q.cu_y);
        fme_job& j = jobs[jx];
        j = fme_job{};
        j.x = q.x; j.y = q.y; j.w = q.w; j.h = q.h;
        j.org_id = q.org_id; j.ref_id = q.ref_id[k];
        j.mvp_x = (int16_t)px; j.mvp_y = (int16_t)py;
        j.lt_x = (int16_t)round4(lx); j.lt_y = (int16_t)round4(ly);
        j.rb_x = (int16_t)round4(rx); j.rb_y = (int16_t)round4(ry);
        j.flags = (uint8_t)(FME_JOB_EMI | ((q.flags & FME_PU_LOSSLESS) ? FME_JOB_LOSSLESS : 0u));
        j.lambda_id = q.lambda_id;
        j.bits_in = (uint16_t)bits;
        j.key_offset = -1;
        fme_tz_ext& e = ext[jx];
        e = fme_tz_ext{};
        e.cu_x = q.cu_x; e.cu_y = q.cu_y;
        e.search_range = (uint8_t)range;
        const bool reads = !(q.part_size == FME_PART_2Nx2N && q.depth == 0);
        e.flags = reads ? FME_TZ_PRED2NX2N : 0;
      }
    }
  });
  // ---- 2. integer searches by m_integerMv2Nx2N dependency level ----
  std::vector<int>& level = c->pi_level;
  std::vector<int>& src = c->pi_src;   // job whose post-EMI MV is read
  std::vector<int>& lvl = c->pi_lvl;
  level.assign((size_t)n, 0);
  src.assign((size_t)nj, -1);
  lvl.resize((size_t)nj);
  int last[FME_MAX_REFS] = {-1, -1, -1, -1};
  int max_level = 0;
  for (int i = 0; i < n; i++) {
    const fme_pu_req& q = reqs[i];
    const bool reads = !(q.part_size == FME_PART_2Nx2N && q.depth == 0);
    if (reads)
      for (int k = 0; k < q.num_refs; k++)
        if (last[k] >= 0) {
          level[i] = std::max(level[i], level[last[k]] + 1);
          src[base[i] + k] = base[last[k]] + k;
        }
    if (q.part_size == FME_PART_2Nx2N)
      for (int k = 0; k < q.num_refs; k++) last[k] = i;
    max_level = std::max(max_level, level[i]);
    for (int k = 0; k < q.num_refs; k++) {
      lvl[base[i] + k] = level[i];
      fme_tz_ext& e = ext[base[i] + k];
      if ((e.flags & FME_TZ_PRED2NX2N) && src[base[i] + k] < 0) {
        e.pred2n_x = c->int_mv_2n[0][k][0];
        e.pred2n_y = c->int_mv_2n[0][k][1];
      }
    }
  }
  clk.lap(2);
  rc = tz_levels_device(c, jobs, ext, src, lvl, nj, max_level, s);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(s));   // phase boundary (fme_pred_inter_phases)
  clk.lap(3);
  // ---- 3. the sub-pel path over every job in request order (compact results to the host) ----
  HIP_TRY(c->d_res.reserve(nj));
  HIP_TRY(c->d_mv.reserve(nj));
  HIP_TRY(c->h_pi_mv.reserve((size_t)nj));
  HIP_TRY(c->h_pi_last.reserve(FME_MAX_REFS));
  rc = refine_batch(c, c->d_jobs.p, c->d_res.p, c->d_mv.p, nj, s);
  if (rc) return rc;
  const fme_mv_result* const r = c->h_pi_mv.p;
  HIP_TRY(hipMemcpyAsync(c->h_pi_mv.p, c->d_mv.p, (size_t)nj * sizeof(fme_mv_result), hipMemcpyDeviceToHost, s));
  // m_integerMv2Nx2N[k] after this call: mv_int of the last 2Nx2N request with a reference k
  for (int k = 0; k < FME_MAX_REFS; k++)
    if (last[k] >= 0)
      HIP_TRY(hipMemcpyAsync(c->h_pi_last.p + k, c->d_res.p + base[last[k]] + k, sizeof(fme_result),
                             hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(c->h_counts, &c->d_sched.p->invalid, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->h_counts[0] > 0)
    return fail(FME_E_INVALID, "fme_pred_inter_p: %d job(s) rejected by the refinement batch", c->h_counts[0]);
  clk.lap(4);
  // ---- 4. xCheckBestMVP and the reference choice, per request ----
  par_for(n, [&](int lo, int hi) {
    for (int i = lo; i < hi; i++) {
      const fme_pu_req& q = reqs[i];
      const double ml = c->mlambda[q.lambda_id];
      fme_pu_res& o = res[i];
      o = fme_pu_res{};
      uint32_t best = 0xFFFFFFFFu;
      for (int k = 0; k < q.num_refs; k++) {
        const int jx = base[i] + k;
        const fme_mv_result& rr = r[jx];
        const int mx = rr.mv_x, my = rr.mv_y;
        int idx = amvp_idx[jx];
        uint32_t bits = rr.bits, cost = rr.cost;
        if (q.n_cand[k] >= 2) {
          const int org_bits = (int)(eg_bits(mx - q.cand[k][idx][0]) + eg_bits(my - q.cand[k][idx][1]) +
                                     mvp_idx_bits(idx, 2));
          int best_bits = org_bits, best_idx = idx;
          for (int m = 0; m < q.n_cand[k]; m++) {
            if (m == idx) continue;
            const int b = (int)(eg_bits(mx - q.cand[k][m][0]) + eg_bits(my - q.cand[k][m][1]) + mvp_idx_bits(m, 2));
            if (b < best_bits) {
              best_bits = b;
              best_idx = m;
            }
          }
          if (best_idx != idx) {
            idx = best_idx;
            const uint32_t org_total = bits;
            bits = org_total - (uint32_t)org_bits + (uint32_t)best_bits;
            cost = (cost - rd_cost(ml, org_total)) + rd_cost(ml, bits);
          }
        }
        o.ref_cost[k] = cost;
        o.ref_bits[k] = bits;
        o.ref_mv[k][0] = (int16_t)mx;
        o.ref_mv[k][1] = (int16_t)my;
        o.ref_mvp_idx[k] = (uint8_t)idx;
        if (cost < best) {
          best = cost;
          o.cost = cost;
          o.bits = bits;
          o.mv_x = (int16_t)mx;
          o.mv_y = (int16_t)my;
          o.ref_idx = (uint8_t)k;
          o.mvp_idx = (uint8_t)idx;
          o.mvp_x = q.cand[k][idx][0];
          o.mvp_y = q.cand[k][idx][1];
        }
      }
    }
  });
  for (int k = 0; k < FME_MAX_REFS; k++)
    if (last[k] >= 0) {
      c->int_mv_2n[0][k][0] = c->h_pi_last.p[k].mv_int_x;
      c->int_mv_2n[0][k][1] = c->h_pi_last.p[k].mv_int_y;
    }
  clk.lap(5);
  return FME_OK;
}


// predInterSearch on a B slice (TEncSearch.cpp:3746-4105).  The GPU sees:
//   1. one AMVP template-cost launch over every (request, list, reference) with two candidates;
//   2. the uni-pred integer searches by m_integerMv2Nx2N dependency level (per list and reference);
//   3. one fme_refine over the uni-pred jobs in call order.  Their bits_in leave out uiMbBits,
//      which depends on the previous PU's decision (uiLastMode); the searches never read bits_in,
//      so the host re-prices each tail exactly (tail_cost);
//   4. rounds: every request whose uiLastMode is known gets its uni-pred outcome on the host, then
//      its next bi-pred iteration's key (k_bi_key), integer searches (xPatternSearch jobs) and one
//      fme_refine over the uni jobs plus the round's bi jobs in call order: bi jobs read the carried
//      NN state and write none, so the uni jobs repeat their results and each bi job sees the state
//      of its position (a request's iterations all see the state after its own uni jobs).  FEN 1/2
//      and MvdL1ZeroFlag run one iteration, FEN 0/3 up to four (each on the key of the other list's
//      current bi-pred best); a request whose iteration changed nothing stops.  The round's
//      decisions give the next requests their uiLastMode (only the second PU of a two-PU CU waits,
//      so at most 2 x 4 rounds).

int fme_pred_inter_b(fme_ctx* c, const fme_pu_req_b* reqs, fme_pu_res_b* res, int n, void* stream) {
  if (!c || (n > 0 && (!reqs || !res))) return fail(FME_E_INVALID, "fme_pred_inter_b: null argument");
  if (n <= 0) return n == 0 ? FME_OK : fail(FME_E_INVALID, "fme_pred_inter_b: n = %d", n);
  const int fen = c->cfg.fast_inter_mode;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  PiClock clk(c);
  // ---- validation (nothing runs on a bad batch) ----
  for (int i = 0; i < n; i++) {
    const fme_pu_req_b& q = reqs[i];
    const PicDesc& org = c->pics[q.org_id < FME_MAX_PICTURES ? q.org_id : 0];
    if (!valid_pu_shape(q.w, q.h) || q.part_size > FME_PART_nRx2N || q.part_idx >= num_parts(q.part_size) ||
        q.org_id >= FME_MAX_PICTURES || !org.luma || q.x + q.w > org.width || q.y + q.h > org.height ||
        q.lambda_id >= FME_MAX_LAMBDAS || !c->lambda_set[q.lambda_id] ||
        (q.flags & ~(FME_PU_LOSSLESS | FME_PU_FAST_ME_GEN_B | FME_PU_CLIP_BIPRED | FME_PU_MVD_L1_ZERO)))
      return fail(FME_E_INVALID, "fme_pred_inter_b: request %d invalid (shape %dx%d, part %d/%d)", i, q.w, q.h,
                  q.part_size, q.part_idx);
    if (two_part(q.part_size) && q.part_idx == 1 &&
        (i == 0 || reqs[i - 1].part_idx != 0 || reqs[i - 1].part_size != q.part_size ||
         reqs[i - 1].cu_x != q.cu_x || reqs[i - 1].cu_y != q.cu_y))
      return fail(FME_E_INVALID, "fme_pred_inter_b: request %d (second PU) does not follow its CU's first PU", i);
    for (int l = 0; l < 2; l++) {
      if (q.num_refs[l] < 1 || q.num_refs[l] > FME_MAX_REFS)
        return fail(FME_E_INVALID, "fme_pred_inter_b: request %d list %d: %d references", i, l, q.num_refs[l]);
      for (int k = 0; k < q.num_refs[l]; k++) {
        const int rid = q.ref_id[l][k];
        if (rid >= FME_MAX_PICTURES || !c->pics[rid].luma || q.n_cand[l][k] < 1 || q.n_cand[l][k] > 2 ||
            c->pics[rid].width != org.width || c->pics[rid].height != org.height ||
            (l == 1 && (q.l1_to_l0[k] < -1 || q.l1_to_l0[k] >= q.num_refs[0])))
          return fail(FME_E_INVALID, "fme_pred_inter_b: request %d list %d reference %d invalid", i, l, k);
      }
    }
  }
  int rc = sync_tables(c, s);
  if (rc) return rc;
  auto copied = [&](const fme_pu_req_b& q, int l, int k) {
    return l == 1 && (q.flags & FME_PU_FAST_ME_GEN_B) && q.l1_to_l0[k] >= 0;
  };
  // ---- 1. xEstimateMvPredAMVP template costs over every (request, list, reference) ----
  std::vector<int> amvp((size_t)n * 8, 0);   // chosen AMVP index of (i, l, k) = [i * 8 + l * 4 + k]
  // *puiDistBiP of list-1 references under MvdL1ZeroFlag (one candidate: its template cost, 4214-4217)
  std::vector<uint32_t> bipd((size_t)n * 8, 0xFFFFFFFFu);
  {
    std::vector<int> slot, nc;
    size_t ntasks = 0;
    for (int i = 0; i < n; i++) {
      const fme_pu_req_b& q = reqs[i];
      for (int l = 0; l < 2; l++)
        for (int k = 0; k < q.num_refs[l]; k++) {
          const int m_n = q.n_cand[l][k] >= 2 ? 2 : ((q.flags & FME_PU_MVD_L1_ZERO) && l == 1 ? 1 : 0);
          if (!m_n) continue;
          slot.push_back(i * 8 + l * 4 + k);
          nc.push_back(m_n);
          ntasks += (size_t)m_n;
        }
    }
    HIP_TRY(c->h_pi_tasks.reserve(ntasks));
    HIP_TRY(c->h_pi_tsad.reserve(ntasks));
    AmvpTask* const tasks = c->h_pi_tasks.p;
    for (size_t t = 0, base = 0; t < slot.size(); base += nc[t], t++) {
      const fme_pu_req_b& q = reqs[slot[t] / 8];
      const int l = (slot[t] >> 2) & 1, k = slot[t] & 3;
      for (int m = 0; m < nc[t]; m++)
        tasks[base + m] = AmvpTask{q.x, q.y, q.w, q.h, q.org_id, q.ref_id[l][k], q.cu_x, q.cu_y, q.cand[l][k][m][0],
                                   q.cand[l][k][m][1]};
    }
    clk.lap(0);
    if (ntasks > 0) {
      const uint32_t* const tsad = c->h_pi_tsad.p;
      HIP_TRY(c->d_amvp.reserve(ntasks));
      HIP_TRY(c->d_amvp_sad.reserve(ntasks));
      HIP_TRY(hipMemcpyAsync(c->d_amvp.p, tasks, ntasks * sizeof(AmvpTask), hipMemcpyHostToDevice, s));
      AmvpArgs aa{c->d_amvp.p, c->d_pics.p, c->d_amvp_sad.p, (int32_t)ntasks, c->cfg.bit_depth};
      HIP_TRY(launch_amvp_sad(aa, s));
      HIP_TRY(hipMemcpyAsync(c->h_pi_tsad.p, c->d_amvp_sad.p, ntasks * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      for (size_t t = 0, base = 0; t < slot.size(); base += nc[t], t++) {
        const double ml = c->mlambda[reqs[slot[t] / 8].lambda_id];
        uint32_t best = 0xFFFFFFFFu;
        for (int m = 0; m < nc[t]; m++) {   // uiBestCost > uiTmpCost: the first least cost wins
          const uint32_t cost = (uint32_t)((double)tsad[base + m] + ((double)mvp_idx_bits(m, 2) * ml) / 65536.0);
          if (best > cost) {
            best = cost;
            amvp[slot[t]] = m;
          }
        }
        bipd[slot[t]] = best;
      }
    }
  }
  clk.lap(1);
  // ---- 2. uni-pred jobs in call order (pinned), integer searches by m_integerMv2Nx2N level ----
  std::vector<int> ujob((size_t)n * 8, -1), ubeg(n + 1, 0);
  int nu = 0;
  for (int i = 0; i < n; i++) {
    ubeg[i] = nu;
    for (int l = 0; l < 2; l++)
      for (int k = 0; k < reqs[i].num_refs[l]; k++)
        if (!copied(reqs[i], l, k)) ujob[i * 8 + l * 4 + k] = nu++;
  }
  ubeg[n] = nu;
  HIP_TRY(c->h_pi_jobs.reserve((size_t)nu));
  HIP_TRY(c->h_pi_ext.reserve((size_t)nu));
  fme_job* const uj = c->h_pi_jobs.p;
  fme_tz_ext* const ue = c->h_pi_ext.p;
  std::vector<int> ukey((size_t)nu);   // (list, reference) of each uni job
  par_for(n, [&](int lo, int hi) {
    for (int i = lo; i < hi; i++) {
      const fme_pu_req_b& q = reqs[i];
      const PicDesc& org = c->pics[q.org_id];
      const int range = q.search_range ? q.search_range : 64;
      for (int l = 0; l < 2; l++)
        for (int k = 0; k < q.num_refs[l]; k++) {
          const int u = ujob[i * 8 + l * 4 + k];
          if (u < 0) continue;
          const int idx = amvp[i * 8 + l * 4 + k];
          const int px = q.cand[l][k][idx][0], py = q.cand[l][k][idx][1];
          int cx = px, cy = py;
          clip_qpel(cx, cy, org.width, org.height, q.cu_x, q.cu_y);
          int lx = cx - (range << 2), ly = cy - (range << 2), rx = cx + (range << 2), ry = cy + (range << 2);
          clip_qpel(lx, ly, org.width, org.height, q.cu_x, q.cu_y);
          clip_qpel(rx, ry, org.width, org.height, q.cu_x, q.cu_y);
          fme_job& j = uj[u];
          j = fme_job{};
          j.x = q.x; j.y = q.y; j.w = q.w; j.h = q.h;
          j.org_id = q.org_id; j.ref_id = q.ref_id[l][k];
          j.mvp_x = (int16_t)px; j.mvp_y = (int16_t)py;
          j.lt_x = (int16_t)round4(lx); j.lt_y = (int16_t)round4(ly);
          j.rb_x = (int16_t)round4(rx); j.rb_y = (int16_t)round4(ry);
          j.flags = (uint8_t)(FME_JOB_EMI | ((q.flags & FME_PU_LOSSLESS) ? FME_JOB_LOSSLESS : 0u));
          j.lambda_id = q.lambda_id;
          j.bits_in = (uint16_t)(ref_bits(k, q.num_refs[l]) + mvp_idx_bits(idx, 2));   // + uiMbBits[l] later
          j.key_offset = -1;
          fme_tz_ext& e = ue[u];
          e = fme_tz_ext{};
          e.cu_x = q.cu_x; e.cu_y = q.cu_y;
          e.search_range = (uint8_t)range;
          e.flags = (q.part_size == FME_PART_2Nx2N && q.depth == 0) ? 0 : FME_TZ_PRED2NX2N;
          ukey[u] = l * 4 + k;
        }
    }
  });
  {
    std::vector<int>& src = c->pi_src;
    std::vector<int>& lvl = c->pi_lvl;
    std::vector<int>& level = c->pi_level;
    level.assign((size_t)n, 0);
    src.assign((size_t)nu, -1);
    lvl.resize((size_t)nu);
    int max_level = 0;
    int last[8] = {-1, -1, -1, -1, -1, -1, -1, -1};   // last 2Nx2N writer of m_integerMv2Nx2N[l][k]
    for (int i = 0; i < n; i++) {
      for (int u = ubeg[i]; u < ubeg[i + 1]; u++)
        if ((ue[u].flags & FME_TZ_PRED2NX2N) && last[ukey[u]] >= 0) {
          level[i] = std::max(level[i], level[last[ukey[u]]] + 1);
          src[u] = ujob[last[ukey[u]] * 8 + ukey[u]];
        }
      if (reqs[i].part_size == FME_PART_2Nx2N)
        for (int u = ubeg[i]; u < ubeg[i + 1]; u++) last[ukey[u]] = i;
      max_level = std::max(max_level, level[i]);
      for (int u = ubeg[i]; u < ubeg[i + 1]; u++) {
        lvl[u] = level[i];
        if ((ue[u].flags & FME_TZ_PRED2NX2N) && src[u] < 0) {
          ue[u].pred2n_x = c->int_mv_2n[ukey[u] >> 2][ukey[u] & 3][0];
          ue[u].pred2n_y = c->int_mv_2n[ukey[u] >> 2][ukey[u] & 3][1];
        }
      }
    }
    clk.lap(2);
    rc = tz_levels_device(c, uj, ue, src, lvl, nu, max_level, s);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));   // phase boundary (fme_pred_inter_phases)
  }
  clk.lap(3);
  // ---- 3. the uni-pred sub-pel path in call order (full records: the tails are re-priced) ----
  uint32_t s0[12];
  rc = fme_nn_get_state(c, s0);
  if (rc) return rc;
  HIP_TRY(c->d_res.reserve(nu));
  HIP_TRY(c->h_pi_ures.reserve((size_t)nu));
  rc = refine_batch(c, c->d_jobs.p, c->d_res.p, nullptr, nu, s);
  if (rc) return rc;
  // the searched uni jobs (the rounds replay them) and their records
  HIP_TRY(hipMemcpyAsync(uj, c->d_jobs.p, (size_t)nu * sizeof(fme_job), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(c->h_pi_ures.p, c->d_res.p, (size_t)nu * sizeof(fme_result), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(c->h_counts, &c->d_sched.p->invalid, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->h_counts[0] > 0)
    return fail(FME_E_INVALID, "fme_pred_inter_b: %d job(s) rejected by the refinement batch", c->h_counts[0]);
  const fme_result* const ru = c->h_pi_ures.p;
  uint32_t s_end[12];   // the carried state after the uni jobs (what a bi round must leave)
  rc = fme_nn_get_state(c, s_end);
  if (rc) return rc;
  // rowst[i]: NN_pred's carried array_e slots and C after request i's uni jobs (their EMI pushes over
  // the state before them), the inputs its bi jobs read
  std::vector<uint32_t> rowst((size_t)n * 9);
  {
    uint32_t cur[9];
    for (int k = 0; k < 9; k++) cur[k] = s0[k];
    for (int i = 0; i < n; i++) {
      for (int u = ubeg[i]; u < ubeg[i + 1]; u++)
        if (uj[u].flags & FME_JOB_EMI) {
          for (int k = 0; k < (int)ru[u].n_emi && k < 8; k++) cur[k] = ru[u].emi[k];
          cur[8] = ru[u].c;
        }
      std::memcpy(&rowst[(size_t)9 * i], cur, sizeof(cur));
      // a per-call array_e reset (FME_NN_IN_SLOT_RESET nets): a bi call has no pushes of its own
      if (c->cfg.nn_mode == 2 && (c->net.input_flags & FME_NN_IN_SLOT_RESET))
        std::memset(&rowst[(size_t)9 * i], 0, 8 * sizeof(uint32_t));
    }
  }
  clk.lap(4);
  // ---- 4. rounds of host decisions and bi-pred searches ----
  std::vector<BPu> st((size_t)n);
  for (int i = 0; i < n; i++) st[i].stage = 0;
  auto uni_phase = [&](int i, int last_mode) {
    const fme_pu_req_b& q = reqs[i];
    BPu& p = st[i];
    fme_pu_res_b& o = res[i];
    o = fme_pu_res_b{};
    const double ml = c->mlambda[q.lambda_id];
    blk_bits_b(q.part_size, q.part_idx, last_mode, p.mb);
    p.cost[0] = p.cost[1] = 0xFFFFFFFFu;
    p.bits[0] = p.bits[1] = 0;
    std::memset(p.mv, 0, sizeof(p.mv));
    p.ridx[0] = p.ridx[1] = 0;
    p.cost_v1 = 0xFFFFFFFFu;
    p.bits_v1 = 0xFFFFFFFFu;
    p.mv_v1[0] = p.mv_v1[1] = 0;
    p.ridx_v1 = 0;
    p.bip_ref = p.bip_mvp = 0;
    uint32_t cost_l0[FME_MAX_REFS] = {}, bits_l0[FME_MAX_REFS] = {};
    uint32_t best_bip = 0xFFFFFFFFu;   // bestBiPDist (3805-3810)
    for (int l = 0; l < 2; l++)
      for (int k = 0; k < q.num_refs[l]; k++) {
        int idx = amvp[i * 8 + l * 4 + k];
        if ((q.flags & FME_PU_MVD_L1_ZERO) && l == 1 && bipd[i * 8 + 4 + k] < best_bip) {
          best_bip = bipd[i * 8 + 4 + k];
          p.bip_ref = k;
          p.bip_mvp = idx;
        }
        uint32_t b = p.mb[l] + ref_bits(k, q.num_refs[l]) + mvp_idx_bits(idx, 2), cst;
        if (copied(q, l, k)) {   // TEncSearch.cpp:3814-3827
          const int k0 = q.l1_to_l0[k];
          p.mvt[1][k][0] = p.mvt[0][k0][0];
          p.mvt[1][k][1] = p.mvt[0][k0][1];
          cst = cost_l0[k0] - rd_cost(ml, bits_l0[k0]);
          b += eg_bits(p.mvt[1][k][0] - q.cand[1][k][idx][0]) + eg_bits(p.mvt[1][k][1] - q.cand[1][k][idx][1]);
          cst += rd_cost(ml, b);
        } else {
          const int u = ujob[i * 8 + l * 4 + k];
          const fme_result& r = ru[u];
          p.mvt[l][k][0] = r.mv_x;
          p.mvt[l][k][1] = r.mv_y;
          cst = tail_cost(ml, r, uj[u].bits_in, p.mb[l], 1.0);
          b = r.bits + p.mb[l];
        }
        check_best_mvp(ml, q.cand[l][k], q.n_cand[l][k], p.mvt[l][k][0], p.mvt[l][k][1], idx, b, cst);
        p.mvpi[l][k] = idx;
        o.ref_cost[l][k] = cst;
        o.ref_mv[l][k][0] = p.mvt[l][k][0];
        o.ref_mv[l][k][1] = p.mvt[l][k][1];
        o.ref_mvp_idx[l][k] = (uint8_t)idx;
        if (l == 0) {
          cost_l0[k] = cst;
          bits_l0[k] = b;
        }
        if (cst < p.cost[l]) {
          p.cost[l] = cst;
          p.bits[l] = b;
          p.mv[l][0] = p.mvt[l][k][0];
          p.mv[l][1] = p.mvt[l][k][1];
          p.ridx[l] = k;
        }
        if (l == 1 && cst < p.cost_v1 && q.l1_to_l0[k] < 0) {
          p.cost_v1 = cst;
          p.bits_v1 = b;
          p.mv_v1[0] = p.mvt[1][k][0];
          p.mv_v1[1] = p.mvt[1][k][1];
          p.ridx_v1 = k;
        }
      }
    o.bi_list = 0xFF;
    o.bi_cost = 0xFFFFFFFFu;
    o.uni_cost[0] = p.cost[0];
    o.uni_bits[0] = p.bits[0];
    o.uni_cost[1] = p.cost_v1;
    o.uni_bits[1] = p.bits_v1;
  };
  // the decision (4041-4105); bi-pred outcome already in o.bi_* and mvbi/ridxbi/mvpibi
  auto decide = [&](int i, const int16_t mvbi[2][2], const int ridxbi[2], const int mvpibi[2][FME_MAX_REFS]) {
    const fme_pu_req_b& q = reqs[i];
    BPu& p = st[i];
    fme_pu_res_b& o = res[i];
    if (o.bi_cost <= p.cost[0] && o.bi_cost <= p.cost_v1) {
      p.last_mode = 2;
      o.inter_dir = 3;
      o.bits = o.bi_bits;
      o.cost = o.bi_cost;
      for (int l = 0; l < 2; l++) {
        const int k = ridxbi[l], m = mvpibi[l][k];
        o.ref_idx[l] = (uint8_t)k;
        o.mvp_idx[l] = (uint8_t)m;
        o.mv[l][0] = mvbi[l][0];
        o.mv[l][1] = mvbi[l][1];
        o.mvp[l][0] = q.cand[l][k][m][0];
        o.mvp[l][1] = q.cand[l][k][m][1];
      }
    } else if (p.cost[0] <= p.cost_v1) {
      const int k = p.ridx[0], m = p.mvpi[0][k];
      p.last_mode = 0;
      o.inter_dir = 1;
      o.bits = p.bits[0];
      o.cost = p.cost[0];
      o.ref_idx[0] = (uint8_t)k;
      o.mvp_idx[0] = (uint8_t)m;
      o.mv[0][0] = p.mv[0][0];
      o.mv[0][1] = p.mv[0][1];
      o.mvp[0][0] = q.cand[0][k][m][0];
      o.mvp[0][1] = q.cand[0][k][m][1];
    } else {
      const int k = p.ridx_v1, m = p.mvpi[1][k];
      p.last_mode = 1;
      o.inter_dir = 2;
      o.bits = p.bits_v1;
      o.cost = p.cost_v1;
      o.ref_idx[1] = (uint8_t)k;
      o.mvp_idx[1] = (uint8_t)m;
      o.mv[1][0] = p.mv_v1[0];
      o.mv[1][1] = p.mv_v1[1];
      o.mvp[1][0] = q.cand[1][k][m][0];
      o.mvp[1][1] = q.cand[1][k][m][1];
    }
    p.stage = 2;
  };
  std::vector<fme_job> bj;
  std::vector<fme_tz_ext> be;
  std::vector<BiKeyTask> keyt;
  std::vector<int> issued;
  size_t key_total = 0;
  // bi-pred setup (3871-3916): uiMotBits, and under MvdL1ZeroFlag list 1 at its best predictor
  auto bi_setup = [&](int i) {
    const fme_pu_req_b& q = reqs[i];
    BPu& p = st[i];
    std::memcpy(p.mvbi, p.mv, sizeof(p.mvbi));
    p.ridxbi[0] = p.ridx[0];
    p.ridxbi[1] = p.ridx[1];
    std::memcpy(p.mvpibi, p.mvpi, sizeof(p.mvpibi));
    p.ps_ref[0] = p.ridx[0];
    p.ps_ref[1] = p.ridx[1];
    std::memcpy(p.ps_mv, p.mv, sizeof(p.ps_mv));
    p.cost_bi = 0xFFFFFFFFu;
    p.mot[0] = p.bits[0] - p.mb[0];
    if (q.flags & FME_PU_MVD_L1_ZERO) {
      const int kb = p.bip_ref;
      p.mvpibi[1][kb] = p.bip_mvp;
      p.mvbi[1][0] = p.ps_mv[1][0] = p.mvt[1][kb][0] = q.cand[1][kb][p.bip_mvp][0];
      p.mvbi[1][1] = p.ps_mv[1][1] = p.mvt[1][kb][1] = q.cand[1][kb][p.bip_mvp][1];
      p.ridxbi[1] = p.ps_ref[1] = kb;
      p.mot[1] = p.mb[1] + ref_bits(kb, q.num_refs[1]) + mvp_idx_bits(p.bip_mvp, 2);
    } else {
      p.mot[1] = p.bits[1] - p.mb[1];
    }
    p.bits_bi = p.mb[2] + p.mot[0] + p.mot[1];
    p.it = 0;
    p.niter = (fen == 1 || fen == 2 || (q.flags & FME_PU_MVD_L1_ZERO)) ? 1 : 4;
  };
  // one iteration's key (the other list's stored prediction, 3946-3952 and 4461-4471) and searches
  auto bi_issue = [&](int i) {
    const fme_pu_req_b& q = reqs[i];
    BPu& p = st[i];
    const bool l1z = (q.flags & FME_PU_MVD_L1_ZERO) != 0;
    int L = p.it % 2;
    if (fen == 1 || fen == 2) L = p.cost[0] <= p.cost[1] ? 1 : 0;   // FASTINTERSEARCH_MODE1/2 (3931-3941)
    else if (p.it == 0) L = 0;
    if (p.it == 0 && !l1z) {
      p.ps_ref[1 - L] = p.ridx[1 - L];
      p.ps_mv[1 - L][0] = p.mv[1 - L][0];
      p.ps_mv[1 - L][1] = p.mv[1 - L][1];
    }
    if (l1z) L = 0;
    p.L = L;
    const int key_off = (int)key_total;
    key_total += (size_t)q.w * q.h;
    keyt.push_back(BiKeyTask{q.x, q.y, q.w, q.h, q.org_id, q.ref_id[1 - L][p.ps_ref[1 - L]], q.cu_x, q.cu_y,
                             p.ps_mv[1 - L][0], p.ps_mv[1 - L][1], key_off,
                             (q.flags & FME_PU_CLIP_BIPRED) ? 1u : 0u});
    const PicDesc& org = c->pics[q.org_id];
    const int brange = q.bipred_range ? q.bipred_range : 4;
    p.bi0 = (int)bj.size();
    for (int k = 0; k < q.num_refs[L]; k++) {
      const int m = p.mvpibi[L][k];
      // xSetSearchRange around cMvTemp[L][k], the last ME result of (L, k) (4486-4490)
      int cx = p.mvt[L][k][0], cy = p.mvt[L][k][1];
      clip_qpel(cx, cy, org.width, org.height, q.cu_x, q.cu_y);
      int lx = cx - (brange << 2), ly = cy - (brange << 2), rx = cx + (brange << 2), ry = cy + (brange << 2);
      clip_qpel(lx, ly, org.width, org.height, q.cu_x, q.cu_y);
      clip_qpel(rx, ry, org.width, org.height, q.cu_x, q.cu_y);
      fme_job j{};
      j.x = q.x; j.y = q.y; j.w = q.w; j.h = q.h;
      j.org_id = q.org_id; j.ref_id = q.ref_id[L][k];
      j.mvp_x = q.cand[L][k][m][0]; j.mvp_y = q.cand[L][k][m][1];
      j.lt_x = (int16_t)round4(lx); j.lt_y = (int16_t)round4(ly);
      j.rb_x = (int16_t)round4(rx); j.rb_y = (int16_t)round4(ry);
      j.flags = (uint8_t)(FME_JOB_BIPRED | ((q.flags & FME_PU_LOSSLESS) ? FME_JOB_LOSSLESS : 0u));
      j.lambda_id = q.lambda_id;
      j.bits_in = (uint16_t)(p.mb[2] + p.mot[1 - L] + ref_bits(k, q.num_refs[L]) + mvp_idx_bits(m, 2));
      j.key_offset = key_off;
      fme_tz_ext e{};
      e.cu_x = q.cu_x; e.cu_y = q.cu_y;
      e.search_range = (uint8_t)brange;
      bj.push_back(j);
      be.push_back(e);
    }
    p.stage = 1;
    issued.push_back(i);
  };
  for (;;) {
    bj.clear(); be.clear(); keyt.clear(); issued.clear();
    key_total = 0;
    for (int i = 0; i < n; i++) {
      const fme_pu_req_b& q = reqs[i];
      BPu& p = st[i];
      if (p.stage == 3) {
        bi_issue(i);
        continue;
      }
      if (p.stage != 0) continue;
      const bool dep = two_part(q.part_size) && q.part_idx == 1;
      if (dep && st[i - 1].stage != 2) continue;   // uiLastMode not known yet
      uni_phase(i, dep ? st[i - 1].last_mode : 0);
      const bool restricted = q.cu_w == 8 && (q.w < 8 || q.h < 8);   // isBipredRestriction
      if (restricted) {
        const int16_t mvbi[2][2] = {{p.mv[0][0], p.mv[0][1]}, {p.mv[1][0], p.mv[1][1]}};
        decide(i, mvbi, p.ridx, p.mvpi);
        continue;
      }
      bi_setup(i);
      bi_issue(i);
    }
    if (issued.empty()) break;
    // keys, bi-pred integer searches, then the sub-pel path over uni + bi jobs in call order
    rc = grow_keys(c, key_total);
    if (rc) return rc;
    c->n_keys = key_total;
    HIP_TRY(c->d_bikey.reserve(keyt.size()));
    HIP_TRY(hipMemcpyAsync(c->d_bikey.p, keyt.data(), keyt.size() * sizeof(BiKeyTask), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c->d_key_invalid.p, 0, sizeof(int32_t), s));
    BiKeyArgs ka{c->d_bikey.p, c->d_pics.p, c->d_keys.p, (int32_t)keyt.size(), nullptr, (int64_t)key_total, c->cfg.bit_depth};
    HIP_TRY(launch_bi_key(ka, s));
    // the round's bi jobs alone: in call order each sits right after its request's uni jobs, reads
    // the carried NN state there and writes none (TEncSearch.cpp:88-134), so each is refined as an
    // FME_JOB_NN_IN job whose row is that state (rowst, computed once from the uni records) instead
    // of refining every uni job again around them.  The jobs go up once: the bi-pred integer search
    // (xPatternSearch) writes their MVs in place and the refinement reads them there.
    const int nbj = (int)bj.size();
    HIP_TRY(c->h_pi_seq.reserve((size_t)nbj));
    HIP_TRY(c->h_pi_rs.reserve((size_t)nbj));
    HIP_TRY(c->h_pi_rows.reserve((size_t)nbj * 9));
    fme_job* const seq = c->h_pi_seq.p;
    uint32_t* const rows = c->h_pi_rows.p;
    for (int i : issued) {
      const int nb = reqs[i].num_refs[st[i].L];
      for (int k = 0; k < nb; k++) {
        const int q = st[i].bi0 + k;
        seq[q] = bj[q];
        seq[q].flags = (uint8_t)(seq[q].flags | FME_JOB_NN_IN);
        std::memcpy(rows + (size_t)9 * q, &rowst[(size_t)9 * i], 9 * sizeof(uint32_t));
      }
    }
    HIP_TRY(c->d_jobs.reserve(nbj));
    HIP_TRY(c->d_res.reserve(nbj));
    HIP_TRY(c->d_mv.reserve(nbj));
    HIP_TRY(c->d_tz_ext.reserve(nbj));
    HIP_TRY(c->d_tz_sad.reserve(nbj));
    HIP_TRY(c->d_tz_nn_in.reserve((size_t)nbj * 9));
    HIP_TRY(hipMemcpyAsync(c->d_jobs.p, seq, (size_t)nbj * sizeof(fme_job), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_tz_ext.p, be.data(), (size_t)nbj * sizeof(fme_tz_ext), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_tz_nn_in.p, rows, (size_t)nbj * 9 * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    const uint32_t* const keep_in = c->nn_in;
    const int keep_cap = c->nn_in_cap;
    c->nn_in = c->d_tz_nn_in.p;
    c->nn_in_cap = nbj;
    rc = tz_run(c, c->d_jobs.p, c->d_tz_ext.p, c->d_tz_sad.p, nbj, stream, nullptr);
    if (!rc) rc = refine_batch(c, c->d_jobs.p, c->d_res.p, c->d_mv.p, nbj, s);
    c->nn_in = keep_in;
    c->nn_in_cap = keep_cap;
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->h_pi_rs.p, c->d_mv.p, (size_t)nbj * sizeof(fme_mv_result), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_counts, &c->d_sched.p->invalid, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (c->h_counts[0] > 0)
      return fail(FME_E_INVALID, "fme_pred_inter_b: %d job(s) rejected by a bi-pred round", c->h_counts[0]);
    rc = fme_nn_set_state(c, s_end);   // the bi rows wrote the carried state: back to after the uni jobs
    if (rc) return rc;
    const fme_mv_result* const rs = c->h_pi_rs.p;
    for (size_t t2 = 0; t2 < issued.size(); t2++) {
      const int i = issued[t2];
      const fme_pu_req_b& q = reqs[i];
      BPu& p = st[i];
      fme_pu_res_b& o = res[i];
      const double ml = c->mlambda[q.lambda_id];
      const int L = p.L;
      bool changed = false;
      std::memset(o.bi_ref_cost, 0, sizeof(o.bi_ref_cost));
      std::memset(o.bi_ref_mv, 0, sizeof(o.bi_ref_mv));
      for (int k = 0; k < q.num_refs[L]; k++) {
        const fme_mv_result& r = rs[p.bi0 + k];
        p.mvt[L][k][0] = r.mv_x;
        p.mvt[L][k][1] = r.mv_y;
        uint32_t b = r.bits, cst = r.cost;
        int idx = p.mvpibi[L][k];
        check_best_mvp(ml, q.cand[L][k], q.n_cand[L][k], r.mv_x, r.mv_y, idx, b, cst);
        p.mvpibi[L][k] = idx;
        o.bi_ref_cost[k] = cst;
        o.bi_ref_mv[k][0] = r.mv_x;
        o.bi_ref_mv[k][1] = r.mv_y;
        if (cst < p.cost_bi) {   // 3985-4005
          changed = true;
          p.mvbi[L][0] = r.mv_x;
          p.mvbi[L][1] = r.mv_y;
          p.ridxbi[L] = k;
          p.cost_bi = cst;
          p.mot[L] = b - p.mb[2] - p.mot[1 - L];
          p.bits_bi = b;
          if (p.niter != 1) {   // setAllMv + motionCompensation of list L
            p.ps_ref[L] = k;
            p.ps_mv[L][0] = r.mv_x;
            p.ps_mv[L][1] = r.mv_y;
          }
        }
      }
      o.bi_list = (uint8_t)L;
      o.bi_iters = (uint8_t)(p.it + 1);
      if (changed && p.it + 1 < p.niter) {
        p.it++;
        p.stage = 3;
        continue;
      }
      if (!changed && p.cost_bi <= p.cost[0] && p.cost_bi <= p.cost[1]) {   // 4008-4021
        for (int l = 0; l < ((q.flags & FME_PU_MVD_L1_ZERO) ? 1 : 2); l++) {
          const int k = p.ridxbi[l];
          check_best_mvp(ml, q.cand[l][k], q.n_cand[l][k], p.mvbi[l][0], p.mvbi[l][1], p.mvpibi[l][k], p.bits_bi,
                         p.cost_bi);
        }
      }
      o.bi_cost = p.cost_bi;
      o.bi_bits = p.bits_bi;
      decide(i, p.mvbi, p.ridxbi, p.mvpibi);
    }
  }
  clk.lap(6);
  // ---- m_integerMv2Nx2N: the last 2Nx2N request's post-EMI integer MV per (list, reference) ----
  for (int i = 0; i < n; i++)
    if (reqs[i].part_size == FME_PART_2Nx2N)
      for (int u = ubeg[i]; u < ubeg[i + 1]; u++) {
        c->int_mv_2n[ukey[u] >> 2][ukey[u] & 3][0] = ru[u].mv_int_x;
        c->int_mv_2n[ukey[u] >> 2][ukey[u] & 3][1] = ru[u].mv_int_y;
      }
  return FME_OK;
}

}  // extern "C"
