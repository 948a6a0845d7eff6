/*
 * fme_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of HM-16.9-NN_FME's sub-pel motion-estimation path (plain C, scalar,
 * -O2 -ffp-contract=off).  It is the parity checker for the HIP path and the CPU baseline
 * timed by bench.py (`cpu_baseline`, kind "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never links it.
 *
 * Pinning: the integer parts (interpolation, SATD/SAD/SSE, MV cost, FracDIF, EMI step,
 * tail) are checked against golden vectors produced by oracle/_ref, which compiles the
 * reference's own TLibCommon sources (TComInterpolationFilter, TComRdCost, TComYuv, ...)
 * and drives them in TEncSearch's plane-based order (oracle/ref_harness.cpp).  The NN is
 * pinned by the reference's weight CSVs only: its host file TEncSearch.cpp needs Eigen
 * 3.3.7, which is absent, so the float summation order at the Eigen boundary is "parity
 * unpinned"; the contract is sequential-k float32 without FMA.
 */
#ifndef FME_ORACLE_H
#define FME_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/fme.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_picture {
  const uint8_t* luma;     /* 8-bit samples, or NULL when luma16 is set                        */
  int stride, width, height;
  const uint16_t* luma16;  /* bit depths 9..12 (main10): 16-bit samples, stride in samples      */
  int bd;                  /* the picture's bit depth (8 with luma)                              */
} orc_picture;

/* Carried NN_pred() global state: array_e storage, C, PUHeight, PUWidth (TEncSearch.cpp:55-57). */
typedef struct orc_nn_state {
  uint32_t slot[8];
  uint32_t c;
  uint32_t pu_h, pu_w;
  uint32_t written;   /* bit s: slot s written since reset; bit 8: C/PU size written */
} orc_nn_state;

/* A generic NN_pred net (nn_mode 2, fme_load_nn_net): descriptor, parameters in the net's own
 * precision, and the hidden layers a carry_hidden net keeps between calls. */
#define ORC_NN_NET_MAX_PARAMS 8060
typedef struct orc_nn_net {
  fme_nn_net d;
  int loaded, count;
  double pd[ORC_NN_NET_MAX_PARAMS];
  float pf[ORC_NN_NET_MAX_PARAMS];
  double carry_d[FME_NN_MAX_HIDDEN][FME_NN_MAX_WIDTH];
  float carry_f[FME_NN_MAX_HIDDEN][FME_NN_MAX_WIDTH];
} orc_nn_net;

typedef struct orc_ctx {
  fme_config cfg;
  orc_picture pics[FME_MAX_PICTURES];
  double mlambda[FME_MAX_LAMBDAS];
  const int16_t* keys;
  size_t n_keys;
  float nn[FME_NN_PARAMS];
  int nn_loaded;
  orc_nn_state nn_state;
  orc_nn_net net;
  int16_t int_mv_2n[2][FME_MAX_REFS][2];   /* m_integerMv2Nx2N[list][ref] (TEncSearch.h:118) */
  const uint32_t* nn_in;                   /* FME_JOB_NN_IN input rows (orc_set_nn_inputs)     */
  int nn_in_n;
} orc_ctx;

/* primitives (exported for unit tests) */
uint32_t orc_eg_bits(int v);                                         /* TComRdCost.cpp:172-185 */
uint32_t orc_cost(double mlambda, uint32_t bits);                    /* TComRdCost.h:165     */
int      orc_pred_sample(const orc_picture* p, int x, int y, int fx, int fy); /* A.2 */
void     orc_pred_block(const orc_picture* p, int x0, int y0, int w, int h, int qx, int qy,
                        int16_t* out);                               /* W*H, stride w */
uint32_t orc_satd(const int16_t* org, int org_stride, const int16_t* cur, int cur_stride, int w,
                  int h);                                            /* TComRdCost.cpp:1428-1495 */
uint32_t orc_sad(const int16_t* org, int org_stride, const int16_t* cur, int cur_stride, int w,
                 int h, int sub_shift);                              /* TComRdCost.cpp:335-860 */
uint32_t orc_sse(const int16_t* org, int org_stride, const int16_t* cur, int cur_stride, int w,
                 int h);                                             /* TComRdCost.cpp:860-1205 */

/* xPatternSearchFracDIF on one PU; key W*H with stride key_stride, reference picture p,
 * PU origin (x0,y0), full-pel mv_int. */
void orc_frac_dif(const orc_picture* p, const int16_t* key, int key_stride, int x0, int y0, int w,
                  int h, int mv_x, int mv_y, int mvp_x, int mvp_y, double mlambda,
                  int use_hadamard, int8_t half[2], int8_t qtr[2], uint32_t* cost);

/* EMI square step; returns number of pushes, fills emi[], final best and C. */
int orc_emi(const orc_picture* p, const int16_t* key, int key_stride, int x0, int y0, int w, int h,
            int sx, int sy, int mvp_x, int mvp_y, int lt_x, int lt_y, int rb_x, int rb_y,
            double mlambda, int fast_inter_mode, uint32_t emi[8], int* best_x, int* best_y,
            uint32_t* c);

/* Number of EMI pushes by geometry alone (TEncSearch.cpp:1341-1376). */
int orc_emi_push_count(int sx, int sy, int lt_x, int lt_y, int rb_x, int rb_y);

/* NN_pred() forward on explicit inputs; returns class 0..48 (TEncSearch.cpp:85-134). */
int orc_nn_forward(const float* params, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                   float* logits /* 49, may be NULL */);

/* Generic nets (nn_mode 2).  orc_nn_net_forward runs one NN_pred() call on explicit inputs
 * (updating the carried hidden layers of a carry_hidden net) and returns the class; logits
 * (49, may be NULL) receive OUT after the output activation, as double. */
int orc_nn_param_count(const fme_nn_net* d);
int orc_load_nn_net(orc_ctx* ctx, const fme_nn_net* d, const double* params, int count);
int orc_nn_net_forward(orc_ctx* ctx, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                       double* logits);
/* The same with OUT before the output activation (pre, 49 values as double) as well. */
int orc_nn_net_forward_pre(orc_ctx* ctx, const uint32_t e[8], uint32_t c, int pu_h, int pu_w,
                           double* logits, double* pre);

/* context helpers */
void orc_init(orc_ctx* ctx, const fme_config* cfg);
void orc_set_picture(orc_ctx* ctx, int id, const uint8_t* luma, int stride, int w, int h);
/* cfg.bit_depth 9..12 (main10 = 10): 16-bit samples, stride in samples */
void orc_set_picture16(orc_ctx* ctx, int id, const uint16_t* luma, int stride, int w, int h);
void orc_set_lambda(orc_ctx* ctx, int id, double lambda);
void orc_set_motion_lambda(orc_ctx* ctx, int id, double mlambda);
void orc_set_keys(orc_ctx* ctx, const int16_t* keys, size_t n);
void orc_load_nn(orc_ctx* ctx, const float* params);
void orc_nn_reset(orc_ctx* ctx);
void orc_nn_get_state(const orc_ctx* ctx, uint32_t out[12]);
void orc_nn_set_state(orc_ctx* ctx, const uint32_t in[12]);

/* Whole path for n jobs in order (the restated xMotionEstimation sub-pel part). Returns
 * 0 or a negative FME_E_* code. */
int orc_refine(orc_ctx* ctx, const fme_job* jobs, fme_result* res, int n);

/* ---- integer motion estimation: xTZSearch / xPatternSearch per job;
 * writes jobs[i].mv_x/mv_y and sad[i].  Returns 0 or a negative FME_E_* code. */
int orc_integer_search(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad, int n);
/* fme_tz_ext2 records: FME_TZ_FULL / FME_TZ_ENHANCED with the neighbour predictors (fme.h) */
int orc_integer_search2(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext2* ext, uint32_t* sad, int n);
/* the same with the backups' tail for FME_TZ_RING jobs: nn_in[9 i ..] = array_e[index_ref .. +7], C */
int orc_integer_search_ring(orc_ctx* ctx, fme_job* jobs, const fme_tz_ext* ext, uint32_t* sad,
                            uint32_t* nn_in, int n);
void orc_set_nn_inputs(orc_ctx* ctx, const uint32_t* rows, int n);
/* points tested / distortion samples read by the integer searches since the last reset */
void orc_tz_counters(uint64_t out[2], int reset);

/* ---- motion compensation ------------------------------------ */
typedef struct orc_yuv {
  const uint8_t *y, *cb, *cr;   /* 8-bit 4:2:0 planes; chroma (width/2) x (height/2) */
  int y_stride, c_stride, width, height;
} orc_yuv;

/* TComPrediction::motionCompensation per job into the planes (TComPrediction.cpp:476-668,
 * TComInterpolationFilter.cpp:94-394, TComYuv.cpp:354-415, TComDataCU.cpp:2773-2786).
 * pics[ref_id] are the reference pictures.  Returns 0, or -1-i for an invalid job i. */
int orc_mc(const orc_yuv* pics, const fme_mc_job* jobs, int n, uint8_t* y, int y_stride,
           uint8_t* cb, uint8_t* cr, int c_stride, int width, int height);
/* Motion compensation with explicit weighted prediction for the jobs with FME_MC_WP (8-bit):
 * wp9 = int[2][FME_MAX_PICTURES][3][3], per list, picture and component {iWeight, iOffset,
 * uiLog2WeightDenom}. */
int orc_mc_wp(const orc_yuv* pics, const fme_mc_job* jobs, int n, const int* wp9, uint8_t* y, int ys,
              uint8_t* cb, uint8_t* cr, int cs, int width, int height);

/* ---- predInterSearch's P-slice PU / reference loop: each request in
 * order, each reference index in order, exactly as TEncSearch.cpp:3746-3866 runs them (AMVP
 * template choice, xMotionEstimation = orc_integer_search + orc_refine on one job, xCheckBestMVP,
 * the reference choice, m_integerMv2Nx2N).  Returns 0 or a negative FME_E_* code. */
int orc_pred_inter_p(orc_ctx* ctx, const fme_pu_req* reqs, fme_pu_res* res, int n);
void orc_pred_inter_reset(orc_ctx* ctx);
uint32_t orc_template_cost(const orc_ctx* ctx, const fme_pu_req* q, int k, int m);   /* TEncSearch.cpp:4397-4436 */
/* predInterSearch for B slices (TEncSearch.cpp:3746-4105, FEN 0-3, MvdL1ZeroFlag per request): uni loop
 * over both lists, the bi-pred iterations on the removeHighFreq key, the decision. */
int orc_pred_inter_b(orc_ctx* ctx, const fme_pu_req_b* reqs, fme_pu_res_b* res, int n);
void orc_bi_key(const orc_ctx* ctx, int org_id, int ref_id, int x, int y, int w, int h, int cu_x, int cu_y,
                int mvx, int mvy, int clip, int16_t* key);   /* TEncSearch.cpp:4461-4471 */

/* helpers for bindings */
size_t orc_ctx_size(void);

#ifdef __cplusplus
}
#endif

#endif
