/*
 * fme.h — C-ABI of the MI355X-native fractional-pel motion-estimation path.
 *
 * This is the drop-in boundary for HM-16.9-NN_FME's sub-pel hot path:
 *
 *   TEncSearch::xMotionEstimation tail   (TEncSearch.cpp:4529-4597)
 *     EMI 8-point integer square step    (TEncSearch.cpp:5037-5050, 1324-1377, 1078-1189)
 *     TEncSearch::xPatternSearchFracDIF  (TEncSearch.h:423-432, TEncSearch.cpp:5232-5269)
 *       xExtDIFUpSamplingH/Q             (TEncSearch.cpp:6331-6532)
 *       xPatternRefinement               (TEncSearch.cpp:1591-1645)
 *     NN_pred()                          (TEncSearch.cpp:85-204, globals 55-77)
 *
 * The reference exposes no plugin/FFI API for this path: it is a set of protected members
 * of TEncSearch plus a global function with global state.  This header is what a maintainer
 * binds instead: plain pointers, sizes and POD structs, no torch/HIP
 * types in the signatures (streams are passed as `void*` = hipStream_t, may be NULL).
 *
 * Every entry point returns 0 on success and a negative FME_E_* code on failure; the
 * message of the last failure on the calling thread is available from fme_last_error().
 * Nothing aborts.
 */
#ifndef FME_H
#define FME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FME_ABI_VERSION 18

/* ---- error codes ---------------------------------------------------------------- */
#define FME_OK            0
#define FME_E_INVALID    -1   /* bad argument (null pointer, bad size, unknown id)        */
#define FME_E_DEVICE     -2   /* HIP runtime error                                        */
#define FME_E_NOMEM      -3   /* device or host allocation failed                         */
#define FME_E_UNSUPPORTED -4  /* configuration not supported (bit depth != 8, PU size)     */
#define FME_E_STATE      -5   /* missing picture / weights / lambda for a job             */

/* ---- limits ---------------------------------------------------------------------- */
#define FME_MAX_PICTURES  64   /* picture slots per context (org + reference pictures)    */
#define FME_MAX_LAMBDAS   64   /* motion-lambda table entries per context                 */
#define FME_NN_PARAMS     2060 /* float parameters of the 2-layer master net (17-22-20-49)*/

/* ---- configuration (TAppEncCfg.cpp options the path depends on) ------------------- */
typedef struct fme_config {
  int32_t bit_depth;        /* internal luma bit depth: 8, or 10 for the main10
                               configurations (cfg/encoder_*_main10.cfg InternalBitDepth 10):
                               pictures are then uint16 sample planes (strides in samples);
                               every entry point runs at 10 bits (refinement, single-call
                               FracDIF, integer search, template costs, bi-pred keys, the
                               producers, motion compensation), with TComRdCost's 10-bit
                               distortion shifts; other depths return FME_E_UNSUPPORTED     */
  int32_t use_hadamard;     /* HadamardME (TAppEncCfg.cpp:760): SATD vs SAD in FracDIF   */
  int32_t nn_mode;          /* 0: standard FracDIF MV (TEncSearch.cpp:4587-4588 variant)
                               1: NN_pred() MV (shipped behaviour, TEncSearch.cpp:4590-4591)
                               2: the same with a generic net (fme_load_nn_net, configs[4]) */
  int32_t qp;               /* base QP (-q); selects the weight set like TEncSearch::init
                               (TEncSearch.cpp:472/625/775/925: 27, 32, 37, else 22)     */
  int32_t fast_inter_mode;  /* FEN (TAppEncCfg.cpp:888): 1 or 3 -> even-row SAD for the
                               W in {12,24,48} integer metric when H > 8 (TEncSearch.cpp:1158-1164) */
  int32_t max_jobs;         /* capacity hint for device work buffers (0 = grow on demand) */
} fme_config;

/* ---- one PU sub-pel refinement job (32 bytes) -------------------------------------- *
 * Mirrors what xMotionEstimation hands to the path for one (PU, reference picture):
 *   x, y, w, h       PU luma rectangle in the picture (getPartIndexAndSize)
 *   org_id, ref_id   picture slots of the original and the reference picture
 *   mv_x, mv_y       full-pel integer MV: the TZ-search best before the EMI square step
 *                    when FME_JOB_EMI is set, else the final integer MV (bi-pred full search)
 *   mvp_x, mvp_y     AMVP predictor, quarter-pel (TComRdCost::setPredictor)
 *   lt_*, rb_*       full-pel search range passed to xTZSearch (xSetSearchRange output)
 *   flags            FME_JOB_*
 *   lambda_id        index into the context's motion-lambda table
 *   bits_in          ruiBits on entry to xMotionEstimation
 *   key_offset       FME_JOB_BIPRED: element offset of the W*H int16 key block
 *                    (2*org - pred_other, TComYuv::removeHighFreq) in the key buffer
 *                    set by fme_set_keys(); the block is stored row-major with stride W.
 *                    -1: the key is the original picture at (x, y).
 */
#define FME_JOB_EMI       0x01u  /* run the EMI square step (uni-pred TZ path)           */
#define FME_JOB_BIPRED    0x02u  /* bi-pred iteration: weight 0.5 in the cost tail        */
#define FME_JOB_LOSSLESS  0x04u  /* CU transquant bypass: SAD instead of SATD            */
#define FME_JOB_NN_IN     0x08u  /* the backups' input path (nn_mode 2, FME_NN_IN_TZ_RING):
                                    no EMI step here - mv is the integer search's final MV
                                    (after its square + ring, FME_TZ_RING) and the NN inputs
                                    are row i of the array bound with fme_set_nn_inputs     */

typedef struct fme_job {
  uint16_t x, y;
  uint8_t  w, h;
  uint8_t  org_id, ref_id;
  int16_t  mv_x, mv_y;
  int16_t  mvp_x, mvp_y;
  int16_t  lt_x, lt_y, rb_x, rb_y;
  uint8_t  flags;
  uint8_t  lambda_id;
  uint16_t bits_in;
  int32_t  key_offset;
} fme_job;

/* ---- one result (64 bytes) ---------------------------------------------------------- *
 *   mv_int_*    integer MV after the EMI step (== job mv when no EMI), full-pel
 *   mv_*        final MV, quarter-pel (rcMv after TEncSearch.cpp:4590-4591)
 *   half_xy, qtr_xy FracDIF offsets rcMvHalf / rcMvQter, each in {-1,0,1}
 *   frac_cost   FracDIF ruiCost (best quarter-pel SATD + MV cost)
 *   cost, bits  xMotionEstimation outputs ruiCost, ruiBits (TEncSearch.cpp:4595-4596)
 *   c           C: integer distortion at mv_int (TEncSearch.cpp:5049-5050)
 *   emi[]       the distortions pushed into array_e by this job, n_emi of them
 *   nn_class    NN_pred() class 0..48 (255 when nn_mode == 0)
 *   status      FME_RES_* bits
 */
#define FME_RES_NN_STALE   0x01u  /* NN read at least one slot not written by this job     */
#define FME_RES_NN_UNINIT  0x02u  /* NN read a slot never written in this context (read as 0) */
#define FME_RES_REJECTED   0x8000u /* device batch rejected (an invalid job): nothing else of the
                                      record was written and the NN state is unchanged          */

typedef struct fme_result {
  int16_t  mv_int_x, mv_int_y;
  int16_t  mv_x, mv_y;
  int8_t   half_x, half_y, qtr_x, qtr_y;
  uint32_t frac_cost;
  uint32_t cost;
  uint32_t bits;
  uint32_t c;
  uint32_t emi[8];
  uint8_t  n_emi;
  uint8_t  nn_class;
  uint16_t status;
} fme_result;

/* ---- the xMotionEstimation outputs alone (16 bytes) ------------------------------------- *
 * What TEncSearch::xMotionEstimation hands back to predInterSearch (rcMv, ruiBits, ruiCost,
 * TEncSearch.cpp:4590-4597) plus the NN class and status: the record a caller copies back over
 * PCIe per job when it needs no FracDIF / EMI internals (fme_refine_mv*).                     */
typedef struct fme_mv_result {
  int16_t  mv_x, mv_y;        /* final MV, quarter-pel                                         */
  uint32_t cost;              /* ruiCost                                                       */
  uint32_t bits;              /* ruiBits                                                       */
  uint8_t  nn_class;          /* 0..48, 255 when nn_mode == 0                                  */
  uint8_t  reserved;
  uint16_t status;            /* FME_RES_*                                                     */
} fme_mv_result;

/* ---- the packed upload form of fme_job (16 bytes) ----------------------------------------- *
 * What crosses PCIe per job when a caller hands a frame's jobs to the device (SURVEY.md §8(d)
 * times the jobs' H2D): half of fme_job.  Nothing of xMotionEstimation's inputs is dropped:
 *   pu   x/4 [0,11) | y/4 [11,22) | w/4-1 [22,26) | h/4-1 [26,30)   (HEVC PUs sit on the 4x4 grid)
 *   ctl  org_id [0,6) | ref_id [6,12) | lambda_id [12,17) | FME_JOB_* flags [17,21) |
 *        keyed [21] (key_offset >= 0) | EMI range bits [22,26) | bits_in [26,32)
 *   mv, mvp as in fme_job.
 * The search range enters the sub-pel path only through the EMI square step's four range tests
 * around the TZ best (xTZ8PointSquareSearch, TEncSearch.cpp:1334-1376: mv.y-1 >= top,
 * mv.y+1 <= bottom, mv.x-1 >= left, mv.x+1 <= right), so the packed job carries those four bits
 * (FME_PK_RANGE_*) instead of the four range words.  Key blocks: key_base[w] (one int32 per 64
 * jobs) is the key_offset of wave w's first keyed job (-1: none); the wave's later keyed jobs
 * follow it densely in job order (offset of the previous keyed job + its w*h), which is how the
 * producers and fme_build_bipred_keys lay keys out.  fme_pack_jobs refuses (FME_E_UNSUPPORTED,
 * the first such job named in fme_last_error) a job outside this form: off the 4x4 grid, x or y
 * >= 8192, a slot id >= 64 or lambda_id >= 32, bits_in >= 64, an int16-extreme mv, or a key
 * offset that does not follow the wave's previous keyed block; such batches use fme_job.      */
#define FME_PACK_WAVE        64
#define FME_PK_RANGE_TOP     0x1u
#define FME_PK_RANGE_BOTTOM  0x2u
#define FME_PK_RANGE_LEFT    0x4u
#define FME_PK_RANGE_RIGHT   0x8u
typedef struct fme_job_packed {
  uint32_t pu;
  uint32_t ctl;
  int16_t  mv_x, mv_y;
  int16_t  mvp_x, mvp_y;
} fme_job_packed;

typedef struct fme_ctx fme_ctx;

/* ---- lifecycle -------------------------------------------------------------------- */
int         fme_abi_version(void);
int         fme_create(int device, const fme_config* cfg, fme_ctx** out_ctx);
int         fme_destroy(fme_ctx* ctx);
const char* fme_last_error(void);

/* ---- pictures ----------------------------------------------------------------------- *
 * 8-bit luma planes, unpadded (width x height, row stride in bytes; at bit_depth 10 `luma`
 * points to uint16_t samples and the stride counts samples).  The path reads
 * outside the picture with edge replication, which equals HM's padded TComPicYuv
 * (extendPicBorder, TComPicYuv.cpp:229-276) for every MV TComDataCU::clipMv admits.  */
int fme_set_picture(fme_ctx* ctx, int id, const uint8_t* luma, int stride, int width, int height,
                    void* stream);
/* Zero-copy: bind a device-resident plane owned by the caller (e.g. a buffer filled by an
 * RCCL broadcast).  It must stay valid while jobs that use `id` run. */
int fme_bind_picture_device(fme_ctx* ctx, int id, const uint8_t* d_luma, int stride, int width,
                            int height);

/* 4:2:0 chroma planes of picture `id` (8-bit, (width/2) x (height/2) of its luma plane, which
 * must be set first; setting the luma plane again with other dimensions drops them).  Only
 * motion compensation reads chroma.                                                         */
int fme_set_picture_chroma(fme_ctx* ctx, int id, const uint8_t* cb, const uint8_t* cr, int stride,
                           void* stream);
int fme_bind_picture_chroma_device(fme_ctx* ctx, int id, const uint8_t* d_cb, const uint8_t* d_cr,
                                   int stride);

/* ---- cost parameters ------------------------------------------------------------------ */
/* lambda -> motion lambda exactly as TComRdCost::setLambda + selectMotionLambda(true,0,false):
 * mlambda = 65536.0 * sqrt(lambda)  (TComRdCost.cpp:104-117, TComRdCost.h:159).           */
int fme_set_lambda(fme_ctx* ctx, int lambda_id, double lambda);
int fme_set_motion_lambda(fme_ctx* ctx, int lambda_id, double motion_lambda);

/* Bi-pred key blocks (int16, host memory; copied to the device). */
int fme_set_keys(fme_ctx* ctx, const int16_t* keys, size_t count, void* stream);

/* ---- NN predictor ------------------------------------------------------------------- *
 * Parameters in the order embs0[8][4], embs1[8][4], in_h1[22][17], h1_h2[20][22],
 * h2_out[49][20], b1, BN_gamma_1, BN_beta_1 (22 each), b2, BN_gamma_2, BN_beta_2
 * (20 each), bout[49], BN_gamma_in, mean, stdev (9 each) — FME_NN_PARAMS floats.
 * fme_create() loads nothing; the host mirror loads the per-QP set (weights/nn2_qp<QP>.bin).     */
int fme_load_nn_weights(fme_ctx* ctx, const float* params, int count);
/* ---- generic (deeper) NN_pred nets: BASELINE.json configs[4] ------------------------------- *
 * nn_mode 2 runs a net loaded with fme_load_nn_net in NN_pred()'s place, with the same inputs
 * (array_e slots, C, PUHeight, PUWidth carried across calls exactly as in nn_mode 1) and the same
 * class -> MV offset switch.
 * INPUT PATHS.  Without input flags a deeper net sees the master's EMI step (the SSE square at
 * distance 1 around the TZ MV, TEncSearch.cpp:1324-1377 with save = true; C = its best SSE) with
 * the slots carried as in nn_mode 1.
 * input_flags FME_NN_IN_TZ_RING: the backups' own input path.  Both backups push EVERY
 * xTZSearchHelp distortion into array_e (Backups/4:659, Backups/15:1257), end xTZSearch with
 * xTZ8PointSquareSearch at distance 1 and xTZ8PointSquareSearch2 at distance 2 around the star best
 * (Backups/4:4868-4878, 818-965; their updates move rcMv), and build NN_pred's inputs in
 * xPatternSearchFast (Backups/4:4343-4359, Backups/15:4935-4951): C = the least distortion pushed
 * before the square (index_ref), U1 V1 U2 H1 H2 U3 V2 U4 = array_e[index_ref .. index_ref + 7], then
 * memset(array_e) (Backups/4:4421-4422, Backups/15:4961-4962).  Here fme_integer_search_ring
 * (FME_TZ_RING jobs) runs that xTZSearch and writes the nine inputs per job; fme_refine takes them
 * for FME_JOB_NN_IN jobs from the array bound with fme_set_nn_inputs.  Bi-pred calls never run
 * xPatternSearchFast in the backups, so they reuse the last uni-pred call's class (MVX_HALF ..
 * MVY_QRTER are globals): a job without FME_JOB_NN_IN reads the carried inputs of the last
 * FME_JOB_NN_IN job (its whole row: all 8 slots, C, PU size), which gives that class.  Not
 * combinable with FME_NN_IN_SLOT_RESET or carry_hidden (FME_E_INVALID).
 * input_flags FME_NN_IN_SLOT_RESET (master inputs): the array_e slots a call's own EMI step did not
 * push read 0, as after the backups' per-call memset; C and the PU size stay carried.  The shape
 * follows the reference's deeper nets:
 * Per call: x = ((double|float)raw - mean) / stdev * gamma_in for raw = e0,e1,e2,e3,C,e4,e5,e6,e7;
 * IN = [emb0[rowH] | emb1[rowW] | x] (embedding != NONE) or x; per hidden layer
 * X[i] = relu(sum_k W[i][k] * IN[k] + b[i]) * gamma[i] + beta[i], summed k = 0.. in order with a
 * separate rounding per product and per add (no FMA), starting from 0 - or, for a layer whose bit
 * is set in carry_hidden, from that layer's X of the previous call (Backups/15 never re-zeroes X3,
 * X4: :4957-4961); OUT = Wout * X + bout, then sigmoid with out_act; class = first maximum.
 * Parameters (double, fme_nn_param_count of them), in this order:
 *   [embs0[8][4], embs1[8][4]]            (embedding != NONE)
 *   per hidden layer l: W_l[width_l][in_l], b_l, gamma_l, beta_l   (in_0 = 17 or 9)
 *   Wout[49][width_last], bout[49], gamma_in[9], mean[9], stdev[9]
 * A float net takes each value as (float)value, like the reference's float initialisers.         */
#define FME_NN_MAX_HIDDEN  4
#define FME_NN_MAX_WIDTH   40
#define FME_NN_F32         0
#define FME_NN_F64         1
#define FME_NN_EMB_NONE    0   /* 9 inputs, no PU-size embeddings                             */
#define FME_NN_EMB_MASTER  1   /* rows by H 4,8,16,12,24,32,64 -> 1..7 (TEncSearch.cpp:93-102) */
#define FME_NN_EMB_SWAP    2   /* rows by H 4,8,12,16,24,32,64 -> 1..7 (Backups/15:4979-4988)  */
#define FME_NN_OUT_LINEAR  0
#define FME_NN_OUT_SIGMOID 1   /* 1 / (1 + exp(-x)) before the argmax (Backups/4:297-299)      */
#define FME_NN_ENGINE_EXACT 0  /* one lane per job, the reference's arithmetic bit for bit      */
#define FME_NN_ENGINE_MFMA  1  /* batched GEMM on v_mfma_{f32_16x16x4_f32,f64_16x16x4_f64}: a
                                  k-ordered FMA chain, so classes may differ on near-ties       */

typedef struct fme_nn_net {
  int32_t  precision;                   /* FME_NN_F32 / FME_NN_F64                              */
  int32_t  n_hidden;                    /* 1..FME_NN_MAX_HIDDEN                                 */
  int32_t  width[FME_NN_MAX_HIDDEN];    /* 1..FME_NN_MAX_WIDTH each (unused entries 0)          */
  int32_t  embedding;                   /* FME_NN_EMB_*                                          */
  int32_t  out_act;                     /* FME_NN_OUT_*                                          */
  uint32_t carry_hidden;                /* bit l: hidden layer l starts from the previous call's */
  uint32_t input_flags;                 /* FME_NN_IN_*                                           */
} fme_nn_net;   /* 40 bytes */
#define FME_NN_IN_SLOT_RESET 1u         /* array_e slots not pushed by this call read 0           */
#define FME_NN_IN_TZ_RING    2u         /* the backups' input path (FME_JOB_NN_IN rows)           */

/* The NN input rows of FME_JOB_NN_IN jobs: a device array of `capacity` rows of 9 uint32 (array_e
 * slots 0..7, C), row i for job i of a batch; written by fme_integer_search_ring(_device) for its
 * FME_TZ_RING jobs.  A batch with an FME_JOB_NN_IN job beyond the capacity, or with none bound, is
 * rejected (FME_E_INVALID on the host path, FME_RES_REJECTED on the device path).  NULL unbinds.  */
int fme_set_nn_inputs(fme_ctx* ctx, const uint32_t* d_rows, int capacity);

/* Number of parameters of `net`, or a negative FME_E_* code for an invalid descriptor. */
int fme_nn_param_count(const fme_nn_net* net);
int fme_load_nn_net(fme_ctx* ctx, const fme_nn_net* net, const double* params, int count);
/* FME_NN_ENGINE_EXACT (default) or FME_NN_ENGINE_MFMA for nn_mode 2. */
int fme_set_nn_engine(fme_ctx* ctx, int engine);
/* Optional diagnostic output of nn_mode 2: a device array of n floats that each later batch fills
 * with top-1 minus top-2 of OUT (after the output activation) per job; NULL turns it off. */
int fme_set_nn_margin_output(fme_ctx* ctx, float* d_margin, int capacity);
/* (capacity: elements of d_margin; a later nn_mode 2 batch larger than that is rejected with
 * FME_E_INVALID instead of writing past the caller's array; d_margin null / capacity 0: off) */
/* Optional diagnostic output of nn_mode 2: OUT before the output activation, 49 values per job in
 * the net's precision (float or double), job-major, so the exact engine can be checked against the
 * oracle bit for bit and the MFMA engine against the exact one output by output (the sigmoid's exp
 * is the device's, within 1 ulp of glibc's; the saturation tests pin the class at its ties).
 * capacity in jobs; a larger batch is rejected as for the margin output.                       */
int fme_set_nn_logit_output(fme_ctx* ctx, void* d_logits, int capacity);

/* Forget the array_e/C/PUHeight/PUWidth state carried across calls (process start).  Stream-
 * ordered: it takes effect at the start of the next batch, after every batch already issued. */
int fme_nn_reset_state(fme_ctx* ctx);
/* The carried state as 12 words: array_e slots[8], C, PUHeight, PUWidth, and a written mask
 * (bit s: slot s written since reset, bit 8: C/PU size written).  Lets a frame-sharded run
 * hand the state of frame f-1 to the rank that refines frame f (nnfme/dist.py).
 * get: waits for the device.  set: stream-ordered like reset (takes effect at the next batch). */
int fme_nn_get_state(fme_ctx* ctx, uint32_t* out12);
int fme_nn_set_state(fme_ctx* ctx, const uint32_t* in12);
/* Enqueue on `stream` a device-to-device copy of the state after every batch issued so far
 * (12 words to d_out12): per-frame end states without a host round trip.                    */
int fme_nn_copy_state_device(fme_ctx* ctx, uint32_t* d_out12, void* stream);

/* Optional: a hipEvent_t that every later batch records on its stream right before the search
 * kernel, i.e. once the batch's dispatch-heavy prologue (tables, classify, schedule, scatter) has
 * run; NULL turns it off.  A pipeline waits on it to start the previous batch's results download
 * only when the long search kernel is running: a device-to-host copy's posted PCIe writes hold
 * back every read the device issues behind them (AQL packet and kernel-argument fetches), so a
 * download overlapping a prologue delayed each of its launches by the length of the copy.   */
int fme_set_search_event(fme_ctx* ctx, void* event);

/* Workgroup slots the search kernel leaves free for a few-workgroup kernel on another stream (the
 * results download of fme_download_device, queued beside the next batch's search): 0 (default)
 * sizes the persistent search grid to fill the chip; n > 0 launches n fewer workgroups than fit
 * resident, so such a kernel starts at once instead of after the search.  No replacement of a
 * reference interface (pipeline tuning).                                                      */
int fme_set_search_reserve(fme_ctx* ctx, int workgroups);

/* Download of device records (fme_mv_result / fme_result rows, any 16-byte-multiple span) into
 * pinned host memory (hipHostMalloc, hipHostRegister or a torch pin_memory() tensor) by the
 * library's own copy kernel of at most `workgroups` workgroups of 256 lanes (0: the default, 8),
 * each lane storing 16-byte blocks with non-temporal stores (PCIe-write bound, ~54 GB/s from 8
 * workgroups: tools/probes/d2h_kernel_probe.hip), asynchronous on
 * `stream`.  A hipMemcpyAsync device-to-host copy runs on this ROCm as a blit kernel of hundreds
 * of workgroups, which, queued beside a running batch, took the CUs of the search kernel
 * (23.6 % of GPU time in the round-4 profile); this one holds a few wave slots.  No replacement
 * of a reference interface: the reference keeps its results in host memory.
 * d_src and h_dst must be 16-byte aligned and `bytes` a multiple of 16.                       */
int fme_download_device(fme_ctx* ctx, const void* d_src, void* h_dst, size_t bytes, int workgroups,
                        void* stream);

/* One small host <-> device copy on every SDMA engine of the context's device, both directions,
 * through the HSA runtime the HIP runtime runs on (hsa_amd_memory_async_copy_on_engine), waited
 * for; *engines (may be null) = engines that took both copies.  The HSA runtime creates an
 * engine's queue at its first copy, and the HIP runtime moves a stream's copies to another free
 * engine whenever its previous one is busy: the first copy on each new engine then blocked the
 * submitting thread for 5.6-7.5 ms in the middle of a copy pipeline (profiles/r06_ab.log).  Call
 * once before a copy pipeline's timed part.  Synchronous; no replacement of a reference
 * interface (pipeline set-up).                                                                  */
int fme_warm_copy_engines(fme_ctx* ctx, int* engines);


/* ---- the batch path --------------------------------------------------------------------- *
 * Runs EMI step -> FracDIF -> NN_pred -> xMotionEstimation tail for n jobs, in job order
 * for the NN's carried state (jobs are independent otherwise).
 * fme_refine:        host job/result arrays (copied over PCIe), synchronous on `stream`.
 *                    A batch with an invalid job returns FME_E_INVALID (nothing computed, the
 *                    NN state unchanged).
 * fme_refine_device: device-resident job/result arrays, asynchronous on `stream`: no host
 *                    synchronisation at all (the PU-shape schedule is built on the device), so
 *                    successive batches, and copies on other streams, overlap.  Invalid jobs
 *                    are found on the device: the batch is then skipped (every result gets
 *                    FME_RES_REJECTED, the NN state is unchanged) and fme_refine_status()
 *                    reports it.
 * fme_refine_mv / fme_refine_mv_device: the same batch writing only the 16-byte
 *                    fme_mv_result per job (xMotionEstimation's outputs); the full records
 *                    stay in context-owned device memory.                                     */
int fme_refine(fme_ctx* ctx, const fme_job* jobs, fme_result* results, int n, void* stream);
int fme_refine_device(fme_ctx* ctx, const fme_job* d_jobs, fme_result* d_results, int n,
                      void* stream);
int fme_refine_mv(fme_ctx* ctx, const fme_job* jobs, fme_mv_result* out, int n, void* stream);
int fme_refine_mv_device(fme_ctx* ctx, const fme_job* d_jobs, fme_mv_result* d_out, int n,
                         void* stream);
/* Packed jobs (fme_job_packed).  fme_pack_jobs: host, n jobs -> out[n] and key_base[ceil(n/64)]
 * (pure host code, no context).  fme_unpack_jobs: the inverse, giving each job's canonical
 * fme_job (range words mv -/+ the range bits, key_offset -1 for unkeyed jobs); the device path
 * unpacks the same way.  fme_refine_packed_device / fme_refine_mv_packed_device: the device
 * batch of fme_refine_device / fme_refine_mv_device over device-resident packed jobs (a 16-byte
 * read and a 32-byte write per job in HBM before classify), identical results.               */
int fme_pack_jobs(const fme_job* jobs, int n, fme_job_packed* out, int32_t* key_base);
int fme_unpack_jobs(const fme_job_packed* packed, const int32_t* key_base, int n, fme_job* out);
int fme_refine_packed_device(fme_ctx* ctx, const fme_job_packed* d_jobs, const int32_t* d_key_base,
                             fme_result* d_results, int n, void* stream);
int fme_refine_mv_packed_device(fme_ctx* ctx, const fme_job_packed* d_jobs, const int32_t* d_key_base,
                                fme_mv_result* d_out, int n, void* stream);
/* Waits for the last refinement batch; returns the number of jobs k_classify rejected in it
 * (0: the batch ran), or a negative FME_E_* code. */
int fme_refine_status(fme_ctx* ctx);

/* ---- integer motion estimation ----------------------------------------- *
 * The integer search xMotionEstimation runs before the sub-pel path (TEncSearch.cpp:4504-4527):
 *   uni-pred jobs (no FME_JOB_BIPRED): xPatternSearchFast -> xTZSearch (TEncSearch.cpp:4737-5036)
 *     with the shipped settings (FastSearch = 1 diamond, not extended; FastMEAssumingSmootherMV:
 *     first search stops 3 rounds after the best; raster step 5; star refinement), from the
 *     AMVP predictor job.mvp (clipMv'd against the CU origin, rounded to full-pel), the zero
 *     vector and, with FME_TZ_PRED2NX2N, the 2Nx2N PU's integer MV; diamond / star points are
 *     limited to the job's lt/rb range, the raster to the range re-centred on the best after the
 *     2Nx2N test (xSetSearchRange).  The final EMI square step is NOT run here: it is the first
 *     step of fme_refine (FME_JOB_EMI), so the result is the TZ best before it.
 *   bi-pred jobs: xPatternSearch (TEncSearch.cpp:4627-4680), every point of lt..rb in raster order.
 * The metric is the modified integer-ME one of the batch path (SSE, SAD12/24/48 with FEN row
 * subsampling) plus the MV cost at cost scale 2.  On return job.mv_x/mv_y hold the integer MV
 * (ready for fme_refine) and sad[i] = ruiSAD (distortion at that MV).                             */
#define FME_TZ_PRED2NX2N 0x01u
#define FME_TZ_RING      0x02u   /* the backups' xTZSearch tail: square (distance 1) + ring (distance 2),
                                    every distortion pushed (fme_integer_search_ring; see
                                    FME_NN_IN_TZ_RING): job.mv_x/mv_y and sad[i] are then the MV
                                    after the ring, and its nine NN inputs are written            */
/* The other FastSearch settings of TAppEncCfg.cpp:752 ("0:Full search 1:Diamond 2:Selective
 * 3:Enhanced Diamond"; the default and every shipped cfg use 1), per uni-pred job:
 *   FME_TZ_FULL      FastSearch 0, MESEARCH_FULL: xPatternSearch over the job's lt..rb
 *                    (TEncSearch.cpp:4504-4507, 4627-4695), a strict minimum in raster order, as
 *                    for bi-pred jobs.  The reference runs no EMI square step on this path, so its
 *                    refinement jobs carry no FME_JOB_EMI (NN_pred then reads the carried inputs).
 *   FME_TZ_ENHANCED  FastSearch 3, MESEARCH_DIAMOND_ENHANCED: xTZSearch(..., bExtendedSettings =
 *                    true) (4726-4727, 4749-4768): the left / above / above-right neighbours' MVs
 *                    tested as start points (m_acMvPredictors, xPatternSearchFast 4708-4713; from
 *                    fme_tz_ext2.preds, zero through the 12-byte entry points), diamonds with the
 *                    distance-1 corners, a half-range diamond search around the zero vector when
 *                    the start is not zero, the adaptive raster (step 5, or step 6 over the halved
 *                    range when the best is near), then the star refinement with corners.
 * FastSearch 2 (xTZSearchSelective, 5054-5229) is not provided: with RestrictMESampling off (the
 * default, TAppEncCfg.cpp:756) its xTZSearchHelp (1097-1150) moves pOrg / pCur by stride <<
 * isubShift rows and calls the width's distortion function for iRows rows, and the SSE functions
 * this path's setDistParam selects for widths 4..64 (TComRdCost.cpp:893-1205) ignore iSubShift, so
 * the reference reads up to 8 rows past the PU in the CU-sized original buffer (past the buffer's
 * end for a PU on the CU's bottom row): its result is not a function of the inputs.            */
#define FME_TZ_FULL      0x04u
#define FME_TZ_ENHANCED  0x08u

typedef struct fme_tz_ext {
  uint16_t cu_x, cu_y;          /* luma origin of the PU's CU (TComDataCU::clipMv)              */
  int16_t  pred2n_x, pred2n_y;  /* m_integerMv2Nx2N[list][ref] (full-pel), with FME_TZ_PRED2NX2N */
  uint8_t  flags;               /* FME_TZ_*                                                     */
  uint8_t  search_range;        /* m_iSearchRange (cfg SearchRange, 64): diamond / star bound    */
  uint16_t reserved;
} fme_tz_ext;   /* 12 bytes */

/* fme_tz_ext plus xPatternSearchFast's neighbour predictors (FME_TZ_ENHANCED jobs). */
typedef struct fme_tz_ext2 {
  fme_tz_ext base;
  int16_t    preds[3][2];       /* m_acMvPredictors[MD_LEFT, MD_ABOVE, MD_ABOVE_RIGHT] (getMvPredLeft /
                                   Above / AboveRight, TEncSearch.cpp:4708-4713), quarter-pel     */
} fme_tz_ext2;   /* 24 bytes */

int fme_integer_search(fme_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n,
                       void* stream);
/* The same with fme_tz_ext2 records (host arrays / device arrays). */
int fme_integer_search2(fme_ctx* ctx, fme_job* jobs, const fme_tz_ext2* ext, uint32_t* sad, int n,
                        void* stream);
int fme_integer_search2_device(fme_ctx* ctx, fme_job* d_jobs, const fme_tz_ext2* d_ext, uint32_t* d_sad,
                               int n, void* stream);
int fme_integer_search_device(fme_ctx* ctx, fme_job* d_jobs, const fme_tz_ext* d_ext, uint32_t* d_sad,
                              int n, void* stream);
/* The same searches with the NN inputs of their FME_TZ_RING jobs: nn_in[9 i .. 9 i + 8] =
 * array_e[index_ref .. index_ref + 7] (0 where fewer were pushed), C (host arrays / device arrays;
 * rows of other jobs are left untouched).  Uni-pred bulk searches only (not the producers).       */
int fme_integer_search_ring(fme_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad,
                            uint32_t* nn_in, int n, void* stream);
int fme_integer_search_ring_device(fme_ctx* ctx, fme_job* d_jobs, const fme_tz_ext* d_ext,
                                   uint32_t* d_sad, uint32_t* d_nn_in, int n, void* stream);
/* With profiling on: device milliseconds of the last integer-search launches; waits for them. */
int fme_integer_search_last_ms(fme_ctx* ctx, float* ms);

/* ---- predInterSearch's P-slice PU / reference loop --------------------- *
 * TEncSearch::predInterSearch, uni-directional part for P slices (TEncSearch.cpp:3746-3866), as a
 * batch producer.  Per PU request and reference index k < num_refs, in the encoder's call order:
 *   bits_in = xGetBlkBits(part_size, P slice)[0] (4286-4333) + the reference-index bits
 *             (3792-3800) + m_auiMVPIdxCost[mvp_idx][AMVP_MAX_NUM_CANDS] (3812, 412-425);
 *   xEstimateMvPredAMVP (4186-4256): with two candidates, the first with the least
 *             xGetTemplateCost (4397-4436: luma prediction at the clipMv'd candidate, SAD against
 *             the original, cost (UInt)(SAD + bits * mlambda / 65536.0) with bits = 1);
 *   xMotionEstimation (4439-4599): xSetSearchRange around the predictor, xTZSearch from it and
 *             from m_integerMv2Nx2N[k] when the PU is not a depth-0 2Nx2N PU, the EMI step,
 *             FracDIF, NN_pred, the cost tail; a 2Nx2N PU stores its integer MV (after the EMI
 *             step) in m_integerMv2Nx2N[k] (4511-4526), state this context keeps like TEncSearch;
 *   xCheckBestMVP (4344-4394), then the strict-minimum reference choice (3845-3853).
 * The AMVP candidates are the caller's (TComDataCU::fillMvpCand reads CUs the encoder has already
 * decided); merge, bi-prediction and the mode decision stay with the caller.  The NN state and
 * m_integerMv2Nx2N follow request order exactly; internally requests are grouped into dependency
 * levels so that each GPU batch holds every request whose inputs are known.                       */
#define FME_MAX_REFS     4
#define FME_PU_LOSSLESS  0x01u   /* CU transquant bypass                                          */
/* HM PartSize (TypeDef.h) */
#define FME_PART_2Nx2N 0
#define FME_PART_2NxN  1
#define FME_PART_Nx2N  2
#define FME_PART_NxN   3
#define FME_PART_2NxnU 4
#define FME_PART_2NxnD 5
#define FME_PART_nLx2N 6
#define FME_PART_nRx2N 7

typedef struct fme_pu_req {
  uint16_t x, y;              /* PU luma rectangle (getPartIndexAndSize)                        */
  uint8_t  w, h;
  uint16_t cu_x, cu_y;        /* luma origin of the CU (clipMv)                                 */
  uint8_t  part_size;         /* FME_PART_*                                                     */
  uint8_t  depth;             /* CU depth (0: CTU-sized CU)                                     */
  uint8_t  org_id;            /* original picture slot                                          */
  uint8_t  num_refs;          /* getNumRefIdx(REF_PIC_LIST_0), 1..FME_MAX_REFS                 */
  uint8_t  ref_id[FME_MAX_REFS];    /* picture slot of reference index k                       */
  uint8_t  n_cand[FME_MAX_REFS];    /* AMVPInfo::iN of reference index k (1 or 2)              */
  int16_t  cand[FME_MAX_REFS][2][2];/* AMVPInfo::m_acMvCand, quarter-pel (hor, ver)            */
  uint8_t  lambda_id;         /* motion-lambda slot                                             */
  uint8_t  search_range;      /* m_aaiAdaptSR = cfg SearchRange (0 -> 64)                       */
  uint8_t  flags;             /* FME_PU_*                                                       */
  uint8_t  reserved;
  uint16_t reserved2[3];
} fme_pu_req;   /* 64 bytes */

typedef struct fme_pu_res {
  int16_t  mv_x, mv_y;        /* cMv[0]: MV of the chosen reference, quarter-pel                */
  int16_t  mvp_x, mvp_y;      /* its predictor after xCheckBestMVP                              */
  uint8_t  ref_idx;           /* iRefIdx[0]                                                     */
  uint8_t  mvp_idx;           /* aaiMvpIdx[0][ref_idx]                                          */
  uint16_t reserved;
  uint32_t bits, cost;        /* uiBits[0], uiCost[0]                                           */
  uint32_t ref_cost[FME_MAX_REFS];  /* uiCostTempL0 per reference index (after xCheckBestMVP)  */
  uint32_t ref_bits[FME_MAX_REFS];  /* uiBitsTempL0                                            */
  int16_t  ref_mv[FME_MAX_REFS][2]; /* cMvTemp[0][k], quarter-pel                              */
  uint8_t  ref_mvp_idx[FME_MAX_REFS];
  uint32_t reserved2[2];
} fme_pu_res;   /* 80 bytes */

/* Host arrays, synchronous on `stream`.  A batch with an invalid request is rejected before any
 * work runs. */
int fme_pred_inter_p(fme_ctx* ctx, const fme_pu_req* reqs, fme_pu_res* res, int n, void* stream);
/* Forget m_integerMv2Nx2N (TEncSearch construction: every entry (0, 0)). */
int fme_pred_inter_reset(fme_ctx* ctx);
/* xEstimateMvPredAMVP's template costs alone: xGetTemplateCost (TEncSearch.cpp:4397-4436) of every
 * AMVP candidate m < n_cand[k] of every reference k < num_refs of every request, in one launch:
 * costs[(i * FME_MAX_REFS + k) * 2 + m] (0xFFFFFFFF where there is no candidate).  Host arrays,
 * synchronous. */
int fme_template_costs(fme_ctx* ctx, const fme_pu_req* reqs, uint32_t* costs, int n, void* stream);

/* ---- predInterSearch for B slices ------------------------------------ *
 * TEncSearch::predInterSearch on a B slice (TEncSearch.cpp:3746-4105), every FEN
 * (fme_config.fast_inter_mode): FEN 1/2 (FASTINTERSEARCH_MODE1/2) run one bi-pred iteration over
 * the list opposite the cheaper uni-pred list (3918-3941); FEN 0/3 run up to four, alternating
 * L0, L1, L0, L1, each on the key of the other list's current bi-pred best, stopping at the first
 * iteration that improves nothing (then xCheckBestMVP on the bi MVs, 4008-4021).  MvdL1ZeroFlag
 * (TEncGOP.cpp:1392-1418: lowdelay B, both lists holding the same pictures) is a request flag:
 * list 1 fixed at the AMVP predictor of least template cost over its references (3805-3810,
 * 3878-3909), one L0 iteration.  FastMEForGenBLowDelayEnabled and ClipForBiPredMeEnabled per
 * request flag.
 * Per request, in the encoder's call order:
 *   uiMbBits = xGetBlkBits(part_size, B slice, part_idx, uiLastMode) (4286-4333), uiLastMode being
 *             the decision of the request before (part_idx 1 continues that request's CU);
 *   uni-pred (3786-3865): list 0, then list 1, each reference as fme_pred_inter_p runs it
 *             (m_integerMv2Nx2N per list); with FME_PU_FAST_ME_GEN_B an L1 reference that is also
 *             L0 reference l1_to_l0[k] takes L0's MV, its cost re-priced with L1's predictor;
 *   bi-pred (3868-4022) unless isBipredRestriction (TComDataCU.cpp:2758-2770: 8x8 CU, PU side
 *             < 8): the other list's uni-pred luma prediction at its best MV (motionCompensation),
 *             key = 2 * org - pred (removeHighFreq, TComYuv.cpp:411-455), and per reference of the
 *             searched list xMotionEstimation(bBi) (4461-4534): xSetSearchRange around the
 *             reference's last MV with bipred_range, xPatternSearch (every integer position),
 *             FracDIF on the key, NN_pred on the carried state (no EMI step), fWeight 0.5;
 *             xCheckBestMVP; strict minimum;
 *   decision (4041-4105): bi when uiCostBi <= uiCost[0] and <= the best L1 cost over references
 *             not in L0 (costValidList1); else L0 when uiCost[0] <= costValidList1; else L1.
 * Merge and the AMP merge-only test (bTestNormalMC false) stay with the caller.                 */
#define FME_PU_FAST_ME_GEN_B 0x02u   /* FastMEForGenBLowDelayEnabled (cfg default true)          */
#define FME_PU_CLIP_BIPRED   0x04u   /* ClipForBiPredMeEnabled: key clipped to 8 bits            */
#define FME_PU_MVD_L1_ZERO   0x08u   /* TComSlice::getMvdL1ZeroFlag (GPB slices of lowdelay B,
                                        TEncGOP.cpp:1410-1418): list 1 at its best template-cost
                                        AMVP predictor with zero MVD, one list-0 bi iteration   */

typedef struct fme_pu_req_b {
  uint16_t x, y;              /* PU luma rectangle                                              */
  uint8_t  w, h;
  uint16_t cu_x, cu_y;        /* luma origin of the CU                                          */
  uint8_t  part_size;         /* FME_PART_*                                                     */
  uint8_t  depth;             /* CU depth                                                       */
  uint8_t  org_id;            /* original picture slot                                          */
  uint8_t  part_idx;          /* iPartIdx within the CU                                         */
  uint8_t  cu_w;              /* CU width (getWidth(0), isBipredRestriction)                    */
  uint8_t  lambda_id;
  uint8_t  search_range;      /* m_aaiAdaptSR (0 -> 64)                                         */
  uint8_t  bipred_range;      /* m_bipredSearchRange (0 -> 4)                                   */
  uint8_t  flags;             /* FME_PU_*                                                       */
  uint8_t  num_refs[2];       /* getNumRefIdx(list), 1..FME_MAX_REFS                            */
  uint8_t  ref_id[2][FME_MAX_REFS];     /* picture slot of (list, reference index)              */
  uint8_t  n_cand[2][FME_MAX_REFS];     /* AMVPInfo::iN (1 or 2)                                */
  int8_t   l1_to_l0[FME_MAX_REFS];      /* TComSlice::getList1IdxToList0Idx, -1: not in L0      */
  uint8_t  reserved[7];
  int16_t  cand[2][FME_MAX_REFS][2][2]; /* AMVP candidates, quarter-pel (hor, ver)              */
} fme_pu_req_b;   /* 112 bytes */

typedef struct fme_pu_res_b {
  uint8_t  inter_dir;         /* 1: L0, 2: L1, 3: bi (setInterDirSubParts)                      */
  uint8_t  ref_idx[2];        /* decided reference index per list (0 for an unused list)        */
  uint8_t  mvp_idx[2];        /* its AMVP index                                                 */
  uint8_t  bi_list;           /* list searched by the last bi-pred iteration; 0xFF: none        */
  uint8_t  bi_iters;          /* bi-pred iterations run (FEN 0/3: up to 4)                      */
  uint8_t  reserved;
  int16_t  mv[2][2];          /* decided MVs, quarter-pel (0 for an unused list)                */
  int16_t  mvp[2][2];         /* their predictors                                               */
  uint32_t bits, cost;        /* uiMEBits and the decided cost                                  */
  uint32_t uni_cost[2];       /* uiCost[0], costValidList1                                      */
  uint32_t uni_bits[2];       /* uiBits[0], bitsValidList1                                      */
  uint32_t bi_cost, bi_bits;  /* uiCostBi, uiBits[2] (0xFFFFFFFF / 0: no bi-pred search)        */
  uint32_t ref_cost[2][FME_MAX_REFS];   /* uni uiCostTemp per (list, reference)                 */
  int16_t  ref_mv[2][FME_MAX_REFS][2];  /* uni cMvTemp per (list, reference)                    */
  uint32_t bi_ref_cost[FME_MAX_REFS];   /* bi uiCostTemp per reference of bi_list (last iteration) */
  int16_t  bi_ref_mv[FME_MAX_REFS][2];  /* bi cMvTemp per reference of bi_list (last iteration)    */
  uint8_t  ref_mvp_idx[2][FME_MAX_REFS];/* uni aaiMvpIdx after xCheckBestMVP                    */
} fme_pu_res_b;   /* 160 bytes */

/* Bi-pred search keys on the device for callers that drive fme_refine themselves: per request
 * the other list's uni-pred luma prediction at (mv_x, mv_y) (motionCompensation: clipMv against
 * the CU origin, xPredInterBlk) and key = 2 * org - pred (TComYuv::removeHighFreq, TComYuv.cpp:
 * 411-455; clipped to 8 bits with FME_PU_CLIP_BIPRED), written as the w*h block at key_offset of
 * the context's key buffer (which becomes key_count elements, replacing fme_set_keys' content).
 * key_offset must be a multiple of 4.  Host request array, synchronous. */
typedef struct fme_bikey_req {
  uint16_t x, y;
  uint8_t  w, h, org_id, ref_id;   /* ref_id: the other list's reference picture slot           */
  uint16_t cu_x, cu_y;
  int16_t  mv_x, mv_y;             /* the other list's MV, quarter-pel                          */
  int32_t  key_offset;
  uint32_t flags;                  /* FME_PU_CLIP_BIPRED                                        */
} fme_bikey_req;   /* 24 bytes */
int fme_build_bipred_keys(fme_ctx* ctx, const fme_bikey_req* reqs, int n, size_t key_count, void* stream);
/* The same for a device-resident request array, stream-ordered and without host synchronisation
 * (a per-frame step of a frame pipeline: the other list's MVs are known on the device).  The
 * requests are validated on the device; invalid ones are skipped and counted, and then every later
 * batch with a job that reads keys is rejected (FME_RES_REJECTED, fme_refine_status) until keys
 * are built again.  The key buffer grows (after synchronising `stream`) when key_count exceeds it. */
int fme_build_bipred_keys_device(fme_ctx* ctx, const fme_bikey_req* d_reqs, int n, size_t key_count,
                                 void* stream);

/* Host arrays, synchronous on `stream`; a batch with an invalid request is rejected before any
 * work runs.  m_integerMv2Nx2N (both lists) is the state fme_pred_inter_reset forgets. */
int fme_pred_inter_b(fme_ctx* ctx, const fme_pu_req_b* reqs, fme_pu_res_b* res, int n, void* stream);

/* Wall-clock milliseconds of the last fme_pred_inter_p / fme_pred_inter_b call by phase (host clock
 * around each phase, the device work of a phase included in it, ms[FME_PI_PHASES]):
 *   0 validation and request expansion (host)      1 AMVP template costs (k_amvp_sad round trip)
 *   2 job setup and level ordering (host)           3 the m_integerMv2Nx2N level chain (k_tz_level)
 *   4 the sub-pel refinement (fme_refine)           5 xCheckBestMVP / reference choice (host)
 *   6 B slices: the bi-pred rounds (keys, xPatternSearch, refine, decisions)   7 total
 * No replacement of a reference interface (measurement of the producers). */
#define FME_PI_PHASES 8
int fme_pred_inter_phases(fme_ctx* ctx, double* ms, int count);

/* ---- single-PU entry points with the TEncSearch argument lists ---------------------------- *
 * xPatternSearchFracDIF(bIsLosslessCoded, pcPatternKey, piRefY, iRefStride, pcMvInt,
 *                       rcMvHalf, rcMvQter, ruiCost) with the HM objects flattened:
 *   key/key_stride/w/h = pcPatternKey ROI, ref/ref_stride = piRefY/iRefStride
 *   (host pointer at the PU origin of a padded picture: reads span rows -4..h+3 and
 *   columns -4..w+3 around mv_int), mvp/motion_lambda = the TComRdCost state.
 * Synchronous; latency-bound by construction (one launch per call).  At bit depth 10 the
 * call runs as a one-job batch (k_search_lane10) on a private 10-bit context created at the
 * first such call, key and window in int16 / uint16 samples (a few launches and copies).      */
int fme_frac_dif_single(fme_ctx* ctx, int lossless, const int16_t* key, int key_stride, int w,
                        int h, const int16_t* ref, int ref_stride, int mv_int_x, int mv_int_y,
                        int mvp_x, int mvp_y, double motion_lambda, int16_t* half_xy,
                        int16_t* qtr_xy, uint32_t* cost);

/* NN_pred() on explicit inputs: e[8] = array_e slots, c = C, pu_h/pu_w = PUHeight/PUWidth.
 * Returns the class 0..48 in *nn_class and the four globals MVX_HALF, MVX_QRTER,
 * MVY_HALF, MVY_QRTER in out4 (TEncSearch.cpp:136-193).                                */
int fme_nn_pred_single(fme_ctx* ctx, const uint32_t* e, uint32_t c, int pu_h, int pu_w,
                       int* nn_class, int16_t* out4);

/* ---- motion compensation of decided MVs (luma 8-tap + 4:2:0 chroma 4-tap) ------------------ *
 * TComPrediction::motionCompensation for one PU per job (TComPrediction.cpp:495-560):
 *   xPredInterUni / xPredInterBi (562-614) -> xPredInterBlk (616-668) on the luma plane
 *   (8-tap, quarter-pel) and both chroma planes (4-tap, eighth-pel; TComInterpolationFilter.cpp
 *   :65-75, 341-394), each MV first clipped by TComDataCU::clipMv (TComDataCU.cpp:2773-2786)
 *   against the CU origin; bi-prediction keeps both lists at 14-bit precision and averages them
 *   with TComYuv::addAvg (TComYuv.cpp:354-415); L0 and L1 with the same picture and the same MV
 *   are predicted from L0 alone (xCheckIdenticalMotion, TComPrediction.cpp:476-492).
 * Weighted prediction (xWeightedPredictionUni/Bi) is not supported: the shipped configurations
 * leave WeightedPredP/B off.
 *   x, y, w, h   PU luma rectangle (w, h in 4..64, multiples of 4)
 *   flags        FME_MC_L0 and/or FME_MC_L1 (both: bi-prediction)
 *   ref_id[l]    picture slot of list l's reference (luma and chroma set)
 *   cu_x, cu_y   luma origin of the CU the PU belongs to (clipMv bounds)
 *   mv[l]        list l's MV in quarter-pel luma units (hor, ver), as stored in the CU          */
#define FME_MC_L0 0x01u
#define FME_MC_L1 0x02u
#define FME_MC_WP 0x04u   /* explicit weighted prediction for this PU: the slice's PPS UseWP (P slice)
                             or WPBiPred (B slice) (TComPrediction.cpp:509-512, 539-542, 612-619): the
                             lists' 14-bit predictions go through TComWeightPrediction::addWeightUni /
                             addWeightBi (TComWeightPrediction.cpp:78-245) with the fme_set_wp
                             parameters, and identical bi motion is not collapsed (xCheckIdenticalMotion
                             tests !WPBiPred) */

typedef struct fme_mc_job {
  uint16_t x, y;
  uint8_t  w, h;
  uint8_t  flags;
  uint8_t  reserved;
  uint8_t  ref_id[2];
  uint16_t cu_x, cu_y;
  int16_t  mv[2][2];
  uint16_t reserved2;
} fme_mc_job;   /* 24 bytes */

/* Writes each job's prediction into the destination planes at the PU position (luma
 * width x height, chroma (width/2) x (height/2)); other samples are left as they are.  Jobs
 * must not overlap.  Every reference picture must have the destination's dimensions.
 * fme_motion_compensate: host planes (copied to the device and back), synchronous; a batch
 *   with any invalid job is rejected before anything runs.
 * fme_motion_compensate_device: device planes and jobs, asynchronous on `stream`; invalid jobs
 *   are skipped and counted, fme_mc_invalid_count() waits and returns the count of the last
 *   such call.                                                                              */
int fme_motion_compensate(fme_ctx* ctx, const fme_mc_job* jobs, int n, uint8_t* y, int y_stride,
                          uint8_t* cb, uint8_t* cr, int c_stride, int width, int height, void* stream);
int fme_motion_compensate_device(fme_ctx* ctx, const fme_mc_job* d_jobs, int n, uint8_t* d_y,
                                 int y_stride, uint8_t* d_cb, uint8_t* d_cr, int c_stride, int width,
                                 int height, void* stream);
int fme_mc_invalid_count(fme_ctx* ctx);
/* Weighted-prediction parameters of reference `ref_id` in list `list` (0 / 1) for the jobs with
 * FME_MC_WP, per component Y, Cb, Cr: the slice header's WPScalingParam (TComSlice.h:1239-1254)
 * iWeight, iOffset (in 8-bit units; scaled by 1 << (bitDepth - 8), high-precision offsets off) and
 * uiLog2WeightDenom (luma / chroma denominators; a bi-pred PU takes list 0's).  getWpScaling's
 * derivation (TComWeightPrediction.cpp:247-324) runs in the kernels.  Unset entries are the
 * default weights (1 << 0, offset 0, denominator 0).  Takes effect for later motion compensation. */
typedef struct fme_wp_param {
  int16_t weight;
  int16_t offset;
  uint8_t log2_denom;     /* 0..7 */
  uint8_t reserved[3];
} fme_wp_param;           /* 8 bytes */
int fme_set_wp(fme_ctx* ctx, int list, int ref_id, const fme_wp_param* ycbcr);
/* With profiling on: device milliseconds of the last motion-compensation launch (HIP events on
 * its stream); waits for it. */
int fme_mc_last_ms(fme_ctx* ctx, float* ms);

/* ---- instrumentation (an extension; the reference has no counterpart) ------------------- *
 * With profiling on, fme_refine/fme_refine_device record HIP events around each kernel of
 * the batch on the streams the kernels run on.  Device milliseconds, FME_NUM_TIMINGS values:
 * [0] classify, [1] schedule + scatter, [2] search phase (EMI + FracDIF), [3] NN + tail,
 * [4] whole batch (first kernel start to last kernel end), [5] the search kernel, [6] 0 (an
 * auxiliary search kernel in earlier versions; every PU shape now runs in the one kernel).
 * fme_last_timings waits for the last profiled batch.  fme_accumulated_timings returns the
 * sums over every profiled batch since the last reset (the return value is the batch count);
 * a batch's events are read at the next batch's own host synchronisation, so profiling a
 * run of batches adds no synchronisation.                                                  */
#define FME_NUM_TIMINGS 7
int fme_set_profiling(fme_ctx* ctx, int enable);
/* Which search kernel serves PU shape width x height: 0 the lane kernel (timings[5]; every HEVC
 * inter PU shape), -1 unsupported shape. */
int fme_search_kernel_of_shape(int width, int height);
int fme_last_timings(fme_ctx* ctx, float* ms, int count);
int fme_accumulated_timings(fme_ctx* ctx, double* ms, int count, int reset);
/* The last fme_frac_dif_single / fme_nn_pred_single call as the resident server saw it, device
 * microseconds since it read the request: us[0] to the answer (the rest of the call's wall time
 * is the host, PCIe and polling); FracDIF only, us[1..4] to the payload (key and window) in LDS,
 * the first filter stage, the half stage's distortions, the quarter stage's distortions (NN_pred:
 * us[1] shader cycles / 100 and us[2] the net's own microseconds).  count <= 5 values.  The
 * checkpoints cost the server wall-clock reads, so it records them only once a caller has asked
 * for them (count > 1): from the next call on; until then us[1..4] are zero. */
int fme_single_last_device_us(fme_ctx* ctx, float* us, int count);

#ifdef __cplusplus
}
#endif

#endif /* FME_H */
