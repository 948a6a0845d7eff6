// fme_device.h — types shared by the HIP kernels (fme_kernels.hip) and the host runtime
// (fme_api.cpp).  Not part of the public ABI (include/fme.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fme.h"

// 0 (default): k_scatter writes only the permutation and the searches gather jobs[perm[i]];
// 1: k_scatter also copies each job into class order (sjobs) for contiguous reads.  Same search
// time on the 1080p frame (0.901 against 0.896 ms, profiles/r05_ab.log) for 27.6 MB less written
// and read per batch.  A build variant for that A/B, not a second path.
#ifndef FME_SJOBS
#define FME_SJOBS 0
#endif
// 1: the bulk integer search stages each (kernel, reference, CTU) group's search area in LDS
// (fme_tz.hip k_tz_staged); 0: one wave per PU straight from the class order (k_tz_wave)
#ifndef FME_TZ_STAGE
#define FME_TZ_STAGE 1
#endif
// Sub-bands per XCD queue of the search kernel (Schedule::xq): the XCD searches its spatial band
// of the frame in this many consecutive strips, every class of a strip before the next strip, so
// the jobs' lines and the reference windows a strip's PU classes share stay in the XCD's L2.
// 1 = the round-4 order (each XCD's band class by class), the default: 8 strips cut the search's
// fetch by 7 % and cost 6 % of its time (0.955 against 0.899 ms; 16: 0.969 ms, profiles/r05_ab.log).
#ifndef FME_LANE_SUBBANDS
#define FME_LANE_SUBBANDS 1
#endif

namespace fme {

constexpr int kNumClasses = 24;      // HEVC inter PU shapes 4x8 .. 64x64 incl. AMP

// Order in which an XCD's band visits the PU classes (Schedule::xq position -> class id):
// 0 = by class id (smallest PUs first), 1 = reversed (largest first), 2 = smallest and largest
// alternating (0, 23, 1, 22, ...).  A/B on the 1080p batch: 0.876 / 0.880 / 0.884 ms, results
// identical (profiles/r06_ab.log): the band's first class pays its cold start whichever it is.
#ifndef FME_LANE_ORDER
#define FME_LANE_ORDER 0
#endif
__host__ __device__ __forceinline__ constexpr int lane_class_at(int pos) {
  return FME_LANE_ORDER == 1 ? kNumClasses - 1 - pos
         : FME_LANE_ORDER == 2 ? ((pos & 1) ? kNumClasses - 1 - (pos >> 1) : (pos >> 1))
                               : pos;
}
constexpr int kBlock = 256;          // threads per workgroup (4 wavefronts)
constexpr int kJobsPerScanBlock = 1024;  // classify / NN kernels: 4 jobs per thread
constexpr int kKeyedWord = 60;           // counts[]: jobs that read a key block (k_classify)

// PU shape of each class (W, H).  Order: by area, then width.
constexpr int kClassW[kNumClasses] = {4, 8, 8, 4, 16, 8, 16, 12, 16, 16, 8, 32,
                                      16, 32, 24, 32, 32, 16, 64, 32, 64, 48, 64, 64};
constexpr int kClassH[kNumClasses] = {8, 4, 8, 16, 4, 16, 8, 16, 12, 16, 32, 8,
                                      32, 16, 32, 24, 32, 64, 16, 64, 32, 64, 48, 64};

struct PicDesc {
  const uint8_t* luma;
  int32_t stride, width, height;
  const uint8_t* cb;          // 4:2:0 chroma (motion compensation only); null when unset
  const uint8_t* cr;
  int32_t cstride;
  int32_t pad_;
};

// One motion-compensation launch (fme_mc.hip).
struct McArgs {
  const fme_mc_job* jobs;
  const PicDesc* pics;
  uint8_t* y;
  uint8_t* cb;
  uint8_t* cr;
  int32_t* invalid;           // count of skipped jobs
  int32_t n, y_stride, c_stride, width, height;
  int32_t bit_depth;          // 8, or 10: y / cb / cr and the pictures hold uint16 samples (strides in samples)
  const fme_wp_param* wp;     // [2][FME_MAX_PICTURES][3] weighted-prediction parameters (FME_MC_WP jobs)
};
hipError_t launch_mc(const McArgs& a, hipStream_t s);

// xGetTemplateCost's distortion (fme_mc.hip): SAD of the uni-pred luma prediction at one AMVP
// candidate (clipMv'd against the CU origin) against the original, one task per wave.
struct AmvpTask {
  uint16_t x, y;
  uint8_t w, h, org_id, ref_id;
  uint16_t cu_x, cu_y;
  int16_t mv_x, mv_y;
};
static_assert(sizeof(AmvpTask) == 16, "AmvpTask layout");
struct AmvpArgs {
  const AmvpTask* tasks;
  const PicDesc* pics;
  uint32_t* sad;
  int32_t n;
  int32_t bit_depth;          // 8, or 10: uint16 planes (k_amvp_sad<10>)
};
hipError_t launch_amvp_sad(const AmvpArgs& a, hipStream_t s);

// xMotionEstimation(bBi)'s search key (fme_mc.hip): the other list's uni-pred luma prediction at
// its MV (clipMv'd against the CU origin), key = 2 * org - pred (TComYuv::removeHighFreq), clipped
// to 8 bits with ClipForBiPredMe; w*h int16 at keys + key_off.  One task per wave.
struct BiKeyTask {
  uint16_t x, y;
  uint8_t w, h, org_id, ref_id;
  uint16_t cu_x, cu_y;
  int16_t mv_x, mv_y;
  int32_t key_off;
  uint32_t clip;
};
static_assert(sizeof(BiKeyTask) == 24, "BiKeyTask layout");
struct BiKeyArgs {
  const BiKeyTask* tasks;
  const PicDesc* pics;
  int16_t* keys;
  int32_t n;
  int32_t* invalid;           // device-resident requests: validated here, rejected ones counted
  int64_t n_keys;             // (then) the key buffer's length
  int32_t bit_depth;          // 8, or 10: uint16 planes, ClipForBiPredMe to 0..1023 (k_bi_key<10>)
};
hipError_t launch_bi_key(const BiKeyArgs& a, hipStream_t s);


// One batch as the device sees it.
struct BatchArgs {
  const fme_job* jobs;
  fme_result* res;
  const int16_t* keys;
  int64_t n_keys;
  const double* mlambda;      // [FME_MAX_LAMBDAS]
  const PicDesc* pics;        // [FME_MAX_PICTURES]
  int32_t n;
  int32_t use_hadamard;
  int32_t fen;
  int32_t nn_mode;
  const int32_t* key_invalid; // > 0: the last device-built keys had invalid requests; batches
                              // whose jobs read keys are rejected (k_classify)
  const uint32_t* nn_in;      // NN input rows of FME_JOB_NN_IN jobs ([nn_in_cap][9]) or null
  int32_t nn_in_cap;
};

struct Schedule;

// Work buffers (device) for one batch.
struct WorkBufs {
  uint8_t* cls;          // [n] class id, 255 = invalid
  int32_t* perm;         // [n] jobs grouped by class (original index)
  fme_job* sjobs;        // [n] copies of the jobs in class order (FME_SJOBS 1: the searches read
                         // them contiguously; 0: they read jobs[perm[i]] and k_scatter writes none)
  int32_t* counts;       // [kNumClasses + 1]: per-class count, [24] = invalid jobs
  int32_t* cursor;       // [kNumClasses]
  int32_t* blk_agg;      // [nblk * 9] per-block max of the NN writer indices
  int32_t* blk_prefix;   // [nblk * 9] exclusive prefix (carry-in) per block
  uint32_t* nn_state;    // 2 x 12 words: slot[8], c, pu_h, pu_w, written
  Schedule* sched;       // built on the device by k_schedule from counts
  int32_t* tile_ctr;     // [8] lane-kernel tile queue heads (zeroed with counts)
  fme_mv_result* mv_out; // compact per-job output (fme_refine_mv*), or null
};
// The search record of job i (the search writes its records in call order; the tail completes them).
__device__ __forceinline__ const fme_result* search_rec(const BatchArgs& a, const WorkBufs&, int i) { return a.res + i; }

// Schedule of the search kernel (k_schedule builds it on the device): class c's jobs are
// sjobs/perm[class_off[c] .. + class_cnt[c]) and its 64-lane wave tiles [prefix[c], prefix[c+1]).
struct Schedule {
  int32_t prefix[kNumClasses + 1];
  int32_t class_off[kNumClasses];
  int32_t class_cnt[kNumClasses];
  // The lane kernel's per-XCD tile queues.  Every class's wave tiles are split into 8 S
  // contiguous bands (S = FME_LANE_SUBBANDS; band B holds tiles [nt B / 8S, nt (B+1) / 8S) of a
  // class with nt tiles), XCD x owns bands x S .. x S + S - 1, and its queue lists them band by
  // band, class by class inside a band in the order lane_class_at: xq[x][s][i] = the queue's tiles
  // before (band x S + s, class lane_class_at(i)); xq[x][s][kNumClasses] = before band s + 1
  // (xq[x][S-1][kNumClasses] = its length).
  int32_t xq[8][FME_LANE_SUBBANDS][kNumClasses + 1];
  int32_t invalid;            // jobs rejected by k_classify (the whole batch is then skipped)
  int32_t pad_[3];
};

// What k_schedule needs to know about the search kernel: lanes per PU of each class (its unit
// count rounded up to a power of two).
struct SchedParams {
  int32_t lanes[kNumClasses];
};
SchedParams sched_params();

// One integer-search launch (fme_tz.hip): the batch, its class-ordered copy and the outputs.
struct TzArgs {
  BatchArgs a;
  const fme_job* sjobs;
  const int32_t* perm;
  fme_job* jobs_out;          // mv_x / mv_y written per job
  const fme_tz_ext* ext;
  uint32_t* sad;              // may be null
  int16_t* emi_mv;            // [n][2] or null: the MV after the EMI square step (uni-pred EMI jobs)
  uint32_t* nn_in;            // [n][9] or null: FME_TZ_RING jobs' NN inputs (array_e[index_ref..+7], C)
  int32_t ext_stride;         // bytes per ext record: sizeof(fme_tz_ext), or sizeof(fme_tz_ext2) (predictors)
};
// Integer-search ext record i (either layout) and, for fme_tz_ext2 records, neighbour predictor k.
__device__ __forceinline__ fme_tz_ext tz_ext_at(const TzArgs& ta, int i) {
  return *reinterpret_cast<const fme_tz_ext*>(reinterpret_cast<const uint8_t*>(ta.ext) + (size_t)ta.ext_stride * i);
}
__device__ __forceinline__ void tz_pred_at(const TzArgs& ta, int i, int k, int& x, int& y) {
  if (ta.ext_stride < (int)sizeof(fme_tz_ext2)) {
    x = y = 0;
    return;
  }
  const fme_tz_ext2* e = reinterpret_cast<const fme_tz_ext2*>(reinterpret_cast<const uint8_t*>(ta.ext) + (size_t)ta.ext_stride * i);
  x = e->preds[k][0];
  y = e->preds[k][1];
}
int tz_kernel_of(int cls);    // 0: 4x8 units, 1: 8x4, 2: 8x8
int tz_lanes_per_pu(int cls);
// Host-built schedule of the integer-search kernels (passed by value).
struct TzSchedule {
  int32_t prefix[3][kNumClasses + 1];
  int32_t class_off[kNumClasses];
  int32_t class_cnt[kNumClasses];
};
// keyed: some job of the batch reads a key block (bi-pred): the kernels that hold int16 keys;
// otherwise the uni-pred form, whose key rows take half the registers
hipError_t launch_tz_wave(const TzArgs& ta, const TzSchedule& sc, int kid, bool keyed, int bit_depth, hipStream_t s);   // prefix in waves
// The staged bulk search's groups (fme_tz.hip k_tz_staged): PUs by (unit-shape kernel kid,
// reference picture, CTU), np = (bound picture ids) * cw * ch groups per kernel.
struct TzPairs {
  int32_t* cnt;      // [3 np] PUs per group (zeroed before launch_tz_pairs)
  int32_t* cursor;   // [3 np]
  int32_t* off;      // [3 np] first position of each group in perm
  int32_t* seg;      // non-empty groups, kernel-major
  int32_t* nseg;     // [0..3): non-empty groups per kernel, [3..6): each kernel's first in seg
  int32_t* perm;     // [n] jobs grouped
  int32_t np, cw, ch;
};
hipError_t launch_tz_pairs(const TzArgs& ta, const TzPairs& tp, const uint8_t* cls, int n, hipStream_t s);
hipError_t launch_tz_staged(const TzArgs& ta, const TzPairs& tp, int kid, bool keyed, int bit_depth, hipStream_t s);
// The dependency levels of a producer's m_integerMv2Nx2N chain (fme_tz.hip k_tz_level): jobs in
// level order, level l = jobs [lvl_off[l], lvl_off[l+1]), one launch per level, back to back.
struct TzChain {
  const int32_t* psrc;        // [n]: job whose post-EMI MV is m_integerMv2Nx2N, or -1
  int32_t nlev;
};
hipError_t launch_tz_levels(const TzArgs& ta, const TzChain& ch, const int32_t* h_lvl_off, int bit_depth, hipStream_t s);

// Host-side launch helpers (fme_kernels.hip).
hipError_t launch_classify(const BatchArgs& a, const WorkBufs& w, hipStream_t s);
// one block: w.counts -> *w.sched (class offsets, block ranges, XCD queues, invalid count)
hipError_t launch_schedule(const WorkBufs& w, const SchedParams& p, hipStream_t s);
hipError_t launch_scatter(const BatchArgs& a, const WorkBufs& w, hipStream_t s);
// 12 words of NN state written to dst in stream order (reset / set_state)
hipError_t launch_put_state(uint32_t* dst, const uint32_t* v12, hipStream_t s);
// the picture / lambda tables written in stream order from kernel arguments
// One batch's picture / lambda tables (a pinned, device-mapped host slot; k_put_tables copies it).
struct TablesSlot {
  PicDesc pics[FME_MAX_PICTURES];
  double ml[FME_MAX_LAMBDAS];
};
hipError_t launch_put_tables(PicDesc* d_pics, double* d_ml, const TablesSlot* t_dev, hipStream_t s);
// The search kernel reads its schedule from *w.sched (no host round trip); it is launched with
// enough workgroups to fill the chip, each pulling tiles from its XCD's queue (then the other
// XCDs').  `a.n` bounds the work.
// reserve > 0: the grid is the resident workgroups (FME_LANE_WAVES per CU) less `reserve`
hipError_t launch_search_lane(const BatchArgs& a, const WorkBufs& w, int reserve, hipStream_t s);
// Bit depth 10 (main10): the pixel-per-lane search (fme_px.hip), same records as the lane kernel;
// pictures hold uint16 samples (PicDesc::luma reinterpreted, stride in samples).
// s_big (may be null: s): the stream of the large-PU kernel, run beside the small-PU one
hipError_t launch_search_px(const BatchArgs& a, const WorkBufs& w, int bit_depth, hipStream_t s, hipStream_t s_big);
// Bit depth 10: the lane-per-unit search on int16 samples (fme_lane10.hip), the lane kernel's
// classes, schedule and records (the default main10 search; FME_MAIN10_SEARCH=px selects the pixel
// kernel above)
hipError_t launch_search_lane10(const BatchArgs& a, const WorkBufs& w, hipStream_t s);
struct NnIn11 {   // NN_pred() inputs of a single call: array_e slots[8], C, PUHeight, PUWidth
  uint32_t v[11];
};
// The single-call server (fme_server.hip): one resident workgroup polls `req_seq` in this block of
// pinned, device-mapped host memory, serves the call and stores the answer block `res`; `stopped` = the
// epoch of an instance that exited (idle, lifetime or `stop`).  Request fields share the first
// lines, the answer has its own, the payload follows.
enum { kSrvNn = 1, kSrvFrac = 2, kSrvSad = 4, kSrvTagged = 8, kSrvMarks = 16 };
constexpr int kSrvBlocks = 128;                       // request blocks, all read by every poll
constexpr int kSrvTagBytes = 12 * (kSrvBlocks - 2);   // FracDIF payload that rides in the blocks
struct SrvBox {
  // host -> device, in 16-byte blocks that the polling wave reads all at once (two per lane, one
  // load each), so a block's fields are those written before its sequence word.  req[0]: seq,
  // shape = kind (bits 0-1) | kSrvSad (lossless or HADME off) | kSrvTagged | kSrvMarks (record the
  // phase checkpoints in `marks`) | w - 1 (bits 8-15) |
  // h - 1 (bits 16-23), the FracDIF predictor - 4 * integer MV (x low 16 bits, y high 16,
  // quarter-pel), stop (set by the host to end the instance).  The rest carry this call's seq in
  // word 0 and are taken only when every one the call uses does:
  //   NN_pred: req[1..4], three inputs each (array_e[8], C, PUHeight, PUWidth);
  //   FracDIF: req[1] = the motion lambda (TComRdCost::m_motionLambda, a double in words 1-2);
  //   kSrvTagged: req[2..] = the window then the key, 12 bytes per block, when they fit in
  //   kSrvTagBytes (the payload arrives with the request: no second round trip); otherwise they are
  //   in key / win below, read after the request.
  alignas(64) uint32_t req[kSrvBlocks][4];
  // device -> host, one 16-byte store: seq, FracDIF cost / NN class, FracDIF half x, y and quarter
  // x, y as int8 (bytes 0..3), the call's device ticks (request read to answer)
  alignas(64) uint32_t res[4];
  uint32_t marks[4];           // FracDIF checkpoints of the call (fme_single_last_device_us)
  uint32_t stopped;
  alignas(64) int16_t key[64 * 64];   // w * h (a multiple of 16 bytes for every PU shape)
  alignas(16) uint8_t win[72 * 72 + 16];   // (w + 8) x (h + 8) window around the integer MV, stride w + 8
};
hipError_t launch_server(SrvBox* box, const float* nn, uint32_t served, uint32_t epoch, uint64_t idle_ticks,
                         uint64_t life_ticks, hipStream_t s);
int lane_lanes_per_pu(int cls);                    // lanes of a class's PU group (pow2), 0: none
int cu_count(int device);                          // compute units (workgroup budget of a launch)
// Packed NN layout for the tail kernel (nn_pack, fme_kernels.hip): offsets in floats, every
// pair region 8-byte aligned.
constexpr int kNnPkPfx = 0;                       // [64 shapes][22] layer-1 prefix (k = 0..7)
constexpr int kNnPkW1 = kNnPkPfx + 64 * 22;       // [11 row pairs][9 k][2]   (k = 8..16)
constexpr int kNnPkW2 = kNnPkW1 + 11 * 9 * 2;     // [10][22][2]
constexpr int kNnPkW3 = kNnPkW2 + 10 * 22 * 2;    // [25][20][2] (row 49 zero)
constexpr int kNnPkB1 = kNnPkW3 + 25 * 20 * 2;    // 22
constexpr int kNnPkG1 = kNnPkB1 + 22;
constexpr int kNnPkBE1 = kNnPkG1 + 22;
constexpr int kNnPkB2 = kNnPkBE1 + 22;            // 20
constexpr int kNnPkG2 = kNnPkB2 + 20;
constexpr int kNnPkBE2 = kNnPkG2 + 20;
constexpr int kNnPkBout = kNnPkBE2 + 20;          // 50 (row 49 zero)
constexpr int kNnPkGin = kNnPkBout + 50;          // 9 each
constexpr int kNnPkMean = kNnPkGin + 9;
constexpr int kNnPkStd = kNnPkMean + 9;
constexpr int kNnPkFloats = kNnPkStd + 9 + 1;
static_assert(kNnPkW1 % 2 == 0 && kNnPkW2 % 2 == 0 && kNnPkW3 % 2 == 0 && kNnPkB1 % 2 == 0 &&
              kNnPkG1 % 2 == 0 && kNnPkBE1 % 2 == 0 && kNnPkB2 % 2 == 0 && kNnPkG2 % 2 == 0 &&
              kNnPkBE2 % 2 == 0 && kNnPkBout % 2 == 0, "pair regions must be 8-byte aligned");
void nn_pack(const float* params, float* packed);   // FME_NN_PARAMS floats -> kNnPkFloats
// NN_pred()'s embedding rows of PUHeight / PUWidth (the switches of TEncSearch.cpp:93-113)
__device__ __forceinline__ int emb_row_h(int h) {
  return h == 4 ? 1 : h == 8 ? 2 : h == 16 ? 3 : h == 12 ? 4 : h == 24 ? 5 : h == 32 ? 6 : h == 64 ? 7 : 0;
}
__device__ __forceinline__ int emb_row_w(int w) {
  return w == 4 ? 1 : w == 8 ? 2 : w == 12 ? 3 : w == 16 ? 4 : w == 24 ? 5 : w == 32 ? 6 : w == 64 ? 7 : 0;
}
typedef float f2 __attribute__((ext_vector_type(2)));   // a row pair of the packed layout
__device__ __forceinline__ f2 ld2(const float* __restrict__ Q, int o) { return *(const f2*)(Q + o); }
__device__ __forceinline__ f2 relu2(f2 s) {
  s.x = s.x < 0.0f ? 0.0f : s.x;
  s.y = s.y < 0.0f ? 0.0f : s.y;
  return s;
}
// Results download into pinned host memory (fme_download_device): `wgs` workgroups of 64 lanes.
hipError_t launch_download(const void* src, void* dst, size_t n16, int wgs, hipStream_t s);
// dst[q] = src[idx[q]] for q < n (jobs, and the integer-search extensions when both ext pointers are
// set): the producers' request order <-> dependency-level order on the device
hipError_t launch_gather_jobs(const fme_job* src, const fme_tz_ext* src_ext, const int32_t* idx, fme_job* dst,
                              fme_tz_ext* dst_ext, int n, hipStream_t s);
hipError_t launch_nn_tail(const BatchArgs& a, const WorkBufs& w, const float* nn_params,
                          int state_in, hipStream_t s);
// fme_job_packed -> fme_job (fme_refine*_packed_device): one lane per job, key offsets by a
// per-wave scan from key_base[i / 64]
hipError_t launch_unpack_jobs(const fme_job_packed* src, const int32_t* key_base, fme_job* dst, int n,
                              hipStream_t s);

// The tail kernels' output: xMotionEstimation's MV / cost / bits with the NN class and status,
// into the full record or, for fme_refine_mv*, the compact one alone.
// The carried array_e slots a job writes (slots 0 .. n-1) and whether it writes C / PU size:
// FME_JOB_EMI: the EMI square step's pushes (its count by geometry, TEncSearch.cpp:1341-1376);
// FME_JOB_NN_IN: a whole input row (the backups' path: all 8 slots, unpushed ones 0, and C).
__device__ __forceinline__ int nn_pushes(const fme_job& j) {
  if (j.flags & FME_JOB_NN_IN) return 8;
  if (!(j.flags & FME_JOB_EMI)) return 0;
  const bool top = j.mv_y - 1 >= j.lt_y, bot = j.mv_y + 1 <= j.rb_y;
  const bool left = j.mv_x - 1 >= j.lt_x, right = j.mv_x + 1 <= j.rb_x;
  const int cols = 1 + (left ? 1 : 0) + (right ? 1 : 0);
  return (top ? cols : 0) + (left ? 1 : 0) + (right ? 1 : 0) + (bot ? cols : 0);
}
__device__ __forceinline__ bool nn_writes_c(const fme_job& j) { return (j.flags & (FME_JOB_EMI | FME_JOB_NN_IN)) != 0; }

// r: the job's record in call order (full-record output); src: its search record (the search
// writes its fields into r itself, so src == r and only the tail's fields are written here).
__device__ __forceinline__ void store_outputs(fme_result* r, const fme_result* src, fme_mv_result* mv_out, int i,
                                              int fx, int fy, uint32_t cost, uint32_t bits, uint8_t cls,
                                              uint16_t status) {
  if (mv_out) {
    fme_mv_result o;
    o.mv_x = (int16_t)fx;
    o.mv_y = (int16_t)fy;
    o.cost = cost;
    o.bits = bits;
    o.nn_class = cls;
    o.reserved = 0;
    o.status = status;
    mv_out[i] = o;
  } else {
    if (src != r) *r = *src;
    r->mv_x = (int16_t)fx;
    r->mv_y = (int16_t)fy;
    r->cost = cost;
    r->bits = bits;
    r->nn_class = cls;
    r->status = status;
  }
}

// Last-writer scan of NN_pred()'s carried globals (k_nn_tail, k_nn_deep_tail).  Job base + t of
// the block's NW waves (t = threadIdx.x) has run[f] = its index when it writes field f (array_e
// slot f < 8; f = 8: C and the PU size), else -1.  src[f] = the last writer at or before the job
// (carry[f]: the last writer before `base`, or -1); tot[f] = the block's last writer (or carry).
// Writer indices grow with the lane, so the last writer at or below a lane is the highest set bit
// of the wave's write mask at or below it: ballots and wave-uniform reads instead of a
// shuffle scan (each ds_bpermute step of which waited on the previous one).
template <int NW>
__device__ __forceinline__ void writer_scan(const int (&run)[9], const int (&carry)[9], int base,
                                            int32_t (*wave_tot)[9], int (&src)[9], int (&tot)[9]) {
  const int lane = (int)threadIdx.x & 63, wid = (int)threadIdx.x >> 6;
  const int wbase = base + 64 * wid;
  const unsigned long long below = ~0ull >> (63 - lane);
  int incl[9];
#pragma unroll
  for (int f = 0; f < 9; f++) {
    const unsigned long long mask = __ballot(run[f] >= 0);
    const unsigned long long m = mask & below;
    incl[f] = m ? wbase + 63 - __clzll(m) : -1;
    if (lane == 0) wave_tot[wid][f] = mask ? wbase + 63 - __clzll(mask) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 9; f++) {
    const int t = lane < NW ? wave_tot[lane][f] : -1;
    const unsigned long long pm = __ballot(lane < wid && t >= 0);   // earlier waves with a writer
    const unsigned long long am = __ballot(t >= 0);
    const int prev = pm ? __builtin_amdgcn_readlane(t, 63 - __clzll(pm)) : carry[f];
    src[f] = max(incl[f], prev);
    tot[f] = am ? __builtin_amdgcn_readlane(t, 63 - __clzll(am)) : carry[f];
  }
}

// A batch k_classify rejected: every job is marked, nothing else is written, and the NN state
// is carried through unchanged (the host flips the state slot after every batch).
__device__ __forceinline__ void reject_job(const BatchArgs& a, const WorkBufs& w, int i, int state_in) {
  if (w.mv_out)
    w.mv_out[i].status = FME_RES_REJECTED;
  else
    a.res[i].status = FME_RES_REJECTED;
  if (i == 0)
    for (int k = 0; k < 12; k++) w.nn_state[12 * (state_in ^ 1) + k] = w.nn_state[12 * state_in + k];
}
}  // namespace fme
