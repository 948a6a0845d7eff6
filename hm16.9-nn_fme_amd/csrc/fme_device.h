// fme_device.h — types shared by the HIP kernels (fme_kernels.hip) and the host runtime
// (fme_api.cpp).  Not part of the public ABI (include/fme.h is).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fme.h"

namespace fme {

constexpr int kNumClasses = 24;      // HEVC inter PU shapes 4x8 .. 64x64 incl. AMP
constexpr int kBlock = 256;          // threads per workgroup (4 wavefronts)
constexpr int kJobsPerScanBlock = 1024;  // classify / NN kernels: 4 jobs per thread

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
};
hipError_t launch_amvp_sad(const AmvpArgs& a, hipStream_t s);


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
};

// Work buffers (device) for one batch.
struct WorkBufs {
  uint8_t* cls;          // [n] class id, 255 = invalid
  int32_t* perm;         // [n] jobs grouped by class (original index)
  fme_job* sjobs;        // [n] copies of the jobs in class order (search reads them contiguously)
  int32_t* counts;       // [kNumClasses + 1]: per-class count, [24] = invalid jobs
  int32_t* cursor;       // [kNumClasses]
  int32_t* blk_agg;      // [nblk * 9] per-block max of the NN writer indices
  int32_t* blk_prefix;   // [nblk * 9] exclusive prefix (carry-in) per block
  uint32_t* nn_state;    // 2 x 12 words: slot[8], c, pu_h, pu_w, written
};

// Schedule of the search kernels.  Kernel k (lane-per-unit with 4x8 / 8x4 / 8x8 units,
// cooperative 256-lane, cooperative 512-lane) serves class c with its blocks
// [prefix[k][c], prefix[k][c+1]); every class belongs to exactly one kernel
// (search_kernel_of).  Class c's jobs are sjobs/perm[class_off[c] .. + class_cnt[c]).
enum {
  kSearchLane48 = 0, kSearchLane84 = 1, kSearchLane88 = 2, kSearchCoop = 3, kSearchCoopLarge = 4,
  kSearchKernels = 5
};
struct Schedule {
  int32_t prefix[kSearchKernels][kNumClasses + 1];
  int32_t class_off[kNumClasses];
  int32_t class_cnt[kNumClasses];
};

// One integer-search launch (fme_tz.hip): the batch, its class-ordered copy and the outputs.
struct TzArgs {
  BatchArgs a;
  const fme_job* sjobs;
  const int32_t* perm;
  fme_job* jobs_out;          // mv_x / mv_y written per job
  const fme_tz_ext* ext;
  uint32_t* sad;              // may be null
  int32_t defer;              // 1: pass 1 queues raster searches for pass 2 (k_tz_raster)
  uint32_t* rst;              // [n][8] raster hand-off records, by job index
  int32_t* rq;                // [3][n] queued job indices per kernel
  int32_t* rqn;               // [3] queue lengths
  int16_t* emi_mv;            // [n][2] or null: the MV after the EMI square step (uni-pred EMI jobs)
};
int tz_kernel_of(int cls);    // 0: 4x8 units, 1: 8x4, 2: 8x8
int tz_lanes_per_pu(int cls);
hipError_t launch_tz(const TzArgs& ta, const Schedule& sc, int kid, hipStream_t s);
hipError_t launch_tz_raster(const TzArgs& ta, const Schedule& sc, int kid, int nq, hipStream_t s);

// Host-side launch helpers (fme_kernels.hip).
int pus_per_tile(int cls);
size_t lds_bytes_for_class(int cls);
hipError_t launch_classify(const BatchArgs& a, const WorkBufs& w, hipStream_t s);
hipError_t launch_scatter(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, hipStream_t s);
int tiles_per_block();
int search_kernel_of(int cls);                      // kSearchLane48 .. kSearchCoopLarge
int search_blocks_for(int cls, int cnt);           // blocks of its kernel for cnt jobs
hipError_t launch_search_lane(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, hipStream_t s);
// one lane kernel (kSearchLane48 / 84 / 88) on stream s
hipError_t launch_search_lane_one(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, int kern,
                                  hipStream_t s);
hipError_t launch_search_large(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, hipStream_t s);
hipError_t launch_search_small(const BatchArgs& a, const WorkBufs& w, const Schedule& sc, hipStream_t s);
int lane_lanes_per_pu(int cls);                    // 0: not a lane-kernel class
int lane_kernel_of(int cls);                       // kSearchLane48/84/88, -1: not a lane class
int lane_blocks_for(int cls, int cnt);
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
hipError_t launch_nn_tail(const BatchArgs& a, const WorkBufs& w, const float* nn_params,
                          int state_in, hipStream_t s);

}  // namespace fme
