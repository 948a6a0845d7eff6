// fme_hm.hpp — C++ host adapter over the C-ABI (include/fme.h) with HM's TEncSearch call
// surface, plus the per-CTU-row batch producer the north star asks for.
//
// What a maintainer links into TLibEncoder (INTEGRATION.md shows the call-site edits):
//   fme_hm::FracSearch   the members of TEncSearch this path replaces, same argument lists:
//       xPatternSearchFracDIF  (TEncSearch.h:423-432, TEncSearch.cpp:5232-5269)
//       NN_pred                (TEncSearch.cpp:85-204; the globals array_e/C/PUHeight/PUWidth
//                               in, MVX_HALF/MVX_QRTER/MVY_HALF/MVY_QRTER out, :55-77)
//     and the TComRdCost state they read (setLambda TComRdCost.cpp:104-117, setPredictor
//     TComRdCost.h:165-174, selectMotionLambda .h:159).  Synchronous, one launch per call.
//   fme_hm::CtuRowBatcher   queues the xMotionEstimation sub-pel jobs (EMI step + FracDIF +
//     NN_pred + tail, TEncSearch.cpp:4529-4597, 5037-5050) of one CTU row, hands the row to a
//     worker thread that runs it on the GPU while the caller fills the next row, and returns
//     the results in queue order (the NN's carried state follows queue order across rows).
//
// Pel planes are HM's int16 samples; pictures are converted to the library's 8-bit planes.
// Errors throw fme_hm::Error carrying fme_last_error().
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fme.h"

namespace fme_hm {

typedef int16_t Pel;          // TypeDef.h:228 (8-bit build: values 0..255; bi-pred keys wider)
typedef uint32_t Distortion;  // TypeDef.h:239

struct Mv {                   // TComMv (TComMv.h:51-165): hor/ver in the caller's units
  int hor = 0, ver = 0;
  Mv() = default;
  Mv(int h, int v) : hor(h), ver(v) {}
};

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

struct SearchConfig {
  int device = 0;
  bool useHadamardME = true;  // TEncCfg::getUseHADME()
  int nnMode = 1;             // 0: standard FracDIF MV, 1: NN_pred() MV (shipped behaviour)
  int qp = 22;                // base QP: selects the weight set like TEncSearch::init
  int fastInterMode = 1;      // FEN (SAD12/24/48 row subsampling of the EMI metric)
  int maxJobs = 1 << 16;      // device work buffers sized for this many jobs per row
  std::string weightsDir;     // holds nn2_qp{22,27,32,37}.bin (empty: $FME_WEIGHTS_DIR or the
                              // package's weights/ directory next to libfme_amd.so)
};

// Reads weights/nn2_qp<set>.bin (2060 float64 -> float32, the set TEncSearch::init picks).
std::vector<float> loadWeights(const std::string& dir, int qp);

// The TEncSearch-shaped single-PU surface (and owner of the device context).
class FracSearch {
 public:
  explicit FracSearch(const SearchConfig& cfg);
  ~FracSearch();
  FracSearch(const FracSearch&) = delete;
  FracSearch& operator=(const FracSearch&) = delete;

  // TComRdCost state used by xPatternSearchFracDIF's MV cost.
  void setLambda(double lambda);              // motion lambda = 65536 * sqrt(lambda)
  void setPredictor(const Mv& mvpQpel);       // AMVP predictor, quarter-pel

  // TEncSearch::xPatternSearchFracDIF(bIsLosslessCoded, pcPatternKey, piRefY, iRefStride,
  // pcMvInt, rcMvHalf, rcMvQter, ruiCost): key = pcPatternKey's ROI (width x height, stride
  // keyStride), refY = the padded reference plane at the PU origin.  Outputs the half and
  // quarter offsets in {-1,0,1}^2 and the best quarter-stage cost.
  void xPatternSearchFracDIF(bool bIsLosslessCoded, const Pel* key, int keyStride, int width,
                             int height, const Pel* refY, int refStride, const Mv* mvInt,
                             Mv& rcMvHalf, Mv& rcMvQter, Distortion& ruiCost);

  // NN_pred() on explicit globals; returns the class 0..48.
  int NN_pred(const uint32_t arrayE[8], uint32_t C, int puHeight, int puWidth, int& mvxHalf,
              int& mvxQrter, int& mvyHalf, int& mvyQrter);

  // Pictures for the batch path: an HM luma plane (Pel, may point into a padded buffer at
  // the picture origin) becomes device picture `id` (0..FME_MAX_PICTURES-1).
  void setPicture(int id, const Pel* plane, int stride, int width, int height);
  void setPicture8(int id, const uint8_t* plane, int stride, int width, int height);
  void setLambdaSlot(int lambdaId, double lambda);

  fme_ctx* ctx() const { return ctx_; }
  std::mutex& mutex() { return mu_; }   // serialises context use with a running batcher

 private:
  fme_ctx* ctx_ = nullptr;
  SearchConfig cfg_;
  double mlambda_ = 0.0;
  Mv mvp_;
  std::vector<uint8_t> stage_;
  std::mutex mu_;
};

// TComPrediction::motionCompensation-shaped surface (TComPrediction.cpp:495-668) over the
// FracSearch's context: pictures with 4:2:0 chroma, one fme_mc_job per PU (the CU's
// TComCUMvField entries for the partition, unclipped, plus the CU origin for clipMv), and
// a batch predicted into caller planes.  PUs of a batch must not overlap.
class MotionCompensator {
 public:
  explicit MotionCompensator(FracSearch& search) : search_(search) {}
  // A reconstructed reference picture (TComPicYuv planes at the picture origin).
  void setPictureYuv(int id, const Pel* y, int yStride, const Pel* cb, const Pel* cr, int cStride, int width,
                     int height);
  void setPictureYuv8(int id, const uint8_t* y, int yStride, const uint8_t* cb, const uint8_t* cr, int cStride,
                      int width, int height);
  // Explicit weighted prediction of reference `id` in list `list` (the slice header's
  // WPScalingParam iWeight / iOffset / uiLog2WeightDenom for Y, Cb, Cr; fme_set_wp).
  void setWp(int list, int id, const int weight[3], const int offset[3], const int log2Denom[3]);
  // Queue one PU: uni-pred when only one of mvL0 / mvL1 is given (refIdL* < 0 for the other);
  // weighted: the slice's UseWP (P) / WPBiPred (B) (FME_MC_WP).
  void add(int x, int y, int w, int h, int cuX, int cuY, int refIdL0, const Mv& mvL0, int refIdL1, const Mv& mvL1,
           bool weighted = false);
  int pending() const { return (int)jobs_.size(); }
  // Predict every queued PU into the 8-bit planes (width x height luma) and clear the queue.
  void run(uint8_t* y, int yStride, uint8_t* cb, uint8_t* cr, int cStride, int width, int height);

 private:
  FracSearch& search_;
  std::vector<fme_mc_job> jobs_;
  std::vector<uint8_t> stage_;
};

// TEncSearch::predInterSearch's uni-directional PU / reference loop for P slices
// (TEncSearch.cpp:3746-3866) over the FracSearch's context: AMVP template choice, bits,
// xMotionEstimation, xCheckBestMVP and the reference choice per partition PU, with
// m_integerMv2Nx2N kept like TEncSearch keeps it.  The caller queues one fme_pu_req per PU in
// call order (AMVP candidates from TComDataCU::fillMvpCand) and gets one fme_pu_res per request.
// A queue of one request is the live encoder's path; a frame's worth is trace replay (the
// library batches it by its m_integerMv2Nx2N dependency levels).
class InterSearchP {
 public:
  explicit InterSearchP(FracSearch& search) : search_(search) {}
  int add(const fme_pu_req& req);        // index of the request in the pending batch
  int pending() const { return (int)reqs_.size(); }
  std::vector<fme_pu_res> run();         // the queued requests in order; clears the queue
  void reset();                          // m_integerMv2Nx2N = (0, 0), as a new TEncSearch

 private:
  FracSearch& search_;
  std::vector<fme_pu_req> reqs_;
};

// TEncSearch::predInterSearch for B slices (TEncSearch.cpp:3746-4105; FEN 1/2, MvdL1ZeroFlag
// false): uni-pred over both lists, the one-iteration bi-pred search on the removeHighFreq key and
// the uni / bi decision, one fme_pu_res_b per fme_pu_req_b.  A CU's second PU must be queued right
// after its first (uiLastMode).  Same queue discipline as InterSearchP.
class InterSearchB {
 public:
  explicit InterSearchB(FracSearch& search) : search_(search) {}
  int add(const fme_pu_req_b& req);
  int pending() const { return (int)reqs_.size(); }
  std::vector<fme_pu_res_b> run();
  void reset();                          // m_integerMv2Nx2N of both lists = (0, 0)

 private:
  FracSearch& search_;
  std::vector<fme_pu_req_b> reqs_;
};

// Per-CTU-row batch producer (double-buffered: the caller fills row k+1 while row k runs).
class CtuRowBatcher {
 public:
  typedef uint64_t Ticket;
  explicit CtuRowBatcher(FracSearch& search, int maxRowsInFlight = 2);
  ~CtuRowBatcher();
  CtuRowBatcher(const CtuRowBatcher&) = delete;
  CtuRowBatcher& operator=(const CtuRowBatcher&) = delete;

  // Queue one uni-pred job of the current row; returns its index within the row.
  int add(const fme_job& job);
  // Queue a bi-pred job (TEncSearch.cpp:4461-4471): its key block 2*org - pred_other
  // (width x height, stride keyStride) travels with the row.
  int addBiPred(fme_job job, const int16_t* key, int keyStride);
  int pending() const { return (int)cur_.jobs.size(); }

  // End the current row and hand it to the worker; returns the row's ticket.
  Ticket submit();
  // Block until the row ran; results in add() order.  Throws the row's error if it failed.
  std::vector<fme_result> wait(Ticket t);
  // submit() the current row (if any) and block until every submitted row has run; the
  // results stay collectable with wait().
  void drain();

 private:
  struct Row {
    Ticket ticket = 0;
    std::vector<fme_job> jobs;
    std::vector<int16_t> keys;
    std::vector<fme_result> results;
    bool done = false;
    int rc = 0;
    std::string err;
  };
  void worker();

  FracSearch& search_;
  int maxInFlight_;
  Row cur_;
  Ticket next_ = 1;
  std::deque<std::unique_ptr<Row>> queue_;   // submitted, not yet run
  std::deque<std::unique_ptr<Row>> done_;    // ran, not yet collected
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  int inFlight_ = 0;         // submitted rows not yet run
  Ticket running_ = 0;       // row the worker is running (0: none)
  std::thread thread_;
};

}  // namespace fme_hm
