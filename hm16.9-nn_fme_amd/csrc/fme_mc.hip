// fme_mc.hip — motion compensation of decided MVs (gfx950): luma 8-tap + 4:2:0 chroma 4-tap.
//
// TComPrediction::motionCompensation (TComPrediction.cpp:495-560) for one PU per workgroup
// (one wavefront):
//   * clipMv of each list's MV against the CU origin (TComDataCU.cpp:2773-2786);
//   * xCheckIdenticalMotion (TComPrediction.cpp:476-492): both lists on one picture with one MV
//     -> uni-prediction from L0;
//   * xPredInterBlk (616-668) per component: integer offset mv >> (2 + csx), fraction
//     mv & ((4 << csx) - 1); fraction (0,0) copies, (fx,0) / (0,fy) filter once, otherwise a
//     horizontal first stage over H + N - 1 rows into LDS, then the vertical stage
//     (TComInterpolationFilter.cpp:94-154 filterCopy, 172-257 filter<N, isVert, isFirst, isLast>);
//     uni-prediction ends at 8 bits (isLast), bi-prediction keeps 14-bit intermediates;
//   * TComYuv::addAvg (TComYuv.cpp:354-415): (p0 + p1 + 16448) >> 7, clipped to 8 bits.
// Samples outside a plane are read with edge replication, which equals HM's padded picture for
// every clipped MV (luma margin 80, chroma margin 40: the clipped reads stay within 75 / 38).
#include <hip/hip_runtime.h>

#include "fme_device.h"

namespace fme {
namespace {

constexpr int kMcNT = 64;                 // one wavefront per PU
constexpr int kMcTmp = (64 + 7) * 64;     // first-stage rows of the largest luma PU
constexpr int kInternalOffs = 8192;       // IF_INTERNAL_OFFS (1 << IF_INTERNAL_PREC-1), 14-bit

// TComInterpolationFilter.cpp:57-75
__device__ __forceinline__ int luma_tap(int f, int k) {
  constexpr signed char t[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                   {-1, 4, -10, 58, 17, -5, 1, 0},
                                   {-1, 4, -11, 40, 40, -11, 4, -1},
                                   {0, 1, -5, 17, 58, -10, 4, -1}};
  return t[f][k];
}
__device__ __forceinline__ int chroma_tap(int f, int k) {
  constexpr signed char t[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                   {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};
  return t[f][k];
}

struct Plane {
  const uint8_t* p;
  int stride, w, h;
  __device__ __forceinline__ int at(int x, int y) const {
    x = min(max(x, 0), w - 1);
    y = min(max(y, 0), h - 1);
    return p[(size_t)y * stride + x];
  }
};

// TComDataCU::clipMv (TComDataCU.cpp:2773-2786), max CU 64 (sps.getMaxCUWidth/Height)
__device__ __forceinline__ void clip_mv(int& mx, int& my, int pic_w, int pic_h, int cu_x, int cu_y) {
  const int hor_max = (pic_w + 8 - cu_x - 1) << 2, hor_min = (-64 - 8 - cu_x + 1) * 4;
  const int ver_max = (pic_h + 8 - cu_y - 1) << 2, ver_min = (-64 - 8 - cu_y + 1) * 4;
  mx = min(hor_max, max(hor_min, mx));
  my = min(ver_max, max(ver_min, my));
}

// One list's prediction of one component block (W x H at (x0, y0) of the plane, integer offset
// (ix, iy), fractions (fx, fy)) -> 8-bit into dst (uni) or 14-bit into acc (bi; second list
// averages into dst).  mode: 0 uni, 1 bi first list, 2 bi second list.
template <int N>
__device__ void pred_block(const Plane& ref, int x0, int y0, int W, int H, int ix, int iy, int fx, int fy,
                           int mode, int16_t* tmp, int16_t* acc, uint8_t* dst, int dst_stride) {
  const int lane = threadIdx.x;
  const int bx = x0 + ix, by = y0 + iy;
  const bool last = mode == 0;
  auto tapf = [](int f, int k) { return N == 8 ? luma_tap(f, k) : chroma_tap(f, k); };
  auto emit = [&](int x, int y, int v) {   // v: 8-bit sample (uni) or 14-bit intermediate (bi)
    if (mode == 0) {
      dst[y * dst_stride + x] = (uint8_t)v;
    } else if (mode == 1) {
      acc[y * W + x] = (int16_t)v;
    } else {   // TComYuv::addAvg, shiftNum = 7, offset = (1 << 6) + 2 * IF_INTERNAL_OFFS
      const int s = (acc[y * W + x] + v + 16448) >> 7;
      dst[y * dst_stride + x] = (uint8_t)min(max(s, 0), 255);
    }
  };
  if (fx == 0 && fy == 0) {   // filterCopy(isFirst = true, isLast)
    for (int i = lane; i < W * H; i += kMcNT) {
      const int x = i % W, y = i / W;
      const int s = ref.at(bx + x, by + y);
      emit(x, y, last ? s : (s << 6) - kInternalOffs);
    }
  } else if (fy == 0 || fx == 0) {   // one 1-D filter<N, isVert, isFirst = true, isLast>
    const bool vert = fy != 0;
    const int f = vert ? fy : fx;
    for (int i = lane; i < W * H; i += kMcNT) {
      const int x = i % W, y = i / W;
      int sum = 0;
#pragma unroll
      for (int k = 0; k < N; k++) {
        const int o = k - (N / 2 - 1);
        sum += ref.at(bx + x + (vert ? 0 : o), by + y + (vert ? o : 0)) * tapf(f, k);
      }
      // isLast: shift 6, offset 32, clip; else shift 0, offset -IF_INTERNAL_OFFS
      emit(x, y, last ? min(max((sum + 32) >> 6, 0), 255) : sum - kInternalOffs);
    }
  } else {   // filterHor(isFirst, !isLast) over H + N - 1 rows, then filterVer(!isFirst, isLast)
    const int HT = H + N - 1;
    for (int i = lane; i < W * HT; i += kMcNT) {
      const int x = i % W, r = i / W;
      int sum = 0;
#pragma unroll
      for (int k = 0; k < N; k++) sum += ref.at(bx + x + k - (N / 2 - 1), by + r - (N / 2 - 1)) * tapf(fx, k);
      tmp[r * W + x] = (int16_t)(sum - kInternalOffs);
    }
    __syncthreads();
    for (int i = lane; i < W * H; i += kMcNT) {
      const int x = i % W, y = i / W;
      int sum = 0;
#pragma unroll
      for (int k = 0; k < N; k++) sum += tmp[(y + k) * W + x] * tapf(fy, k);
      // isLast: shift 12, offset 2048 + (IF_INTERNAL_OFFS << 6), clip; else shift 6, offset 0
      emit(x, y, last ? min(max((sum + 2048 + (kInternalOffs << 6)) >> 12, 0), 255) : (sum >> 6));
    }
  }
  __syncthreads();   // tmp / acc reuse by the next call
}

__device__ __forceinline__ bool mc_job_valid(const McArgs& a, const fme_mc_job& j) {
  if (j.w < 4 || j.h < 4 || j.w > 64 || j.h > 64 || (j.w & 3) || (j.h & 3)) return false;
  if (!(j.flags & (FME_MC_L0 | FME_MC_L1)) || (j.flags & ~(FME_MC_L0 | FME_MC_L1))) return false;
  if ((int)j.x + j.w > a.width || (int)j.y + j.h > a.height) return false;
  for (int l = 0; l < 2; l++) {
    if (!(j.flags & (1u << l))) continue;
    if (j.ref_id[l] >= FME_MAX_PICTURES) return false;
    const PicDesc& p = a.pics[j.ref_id[l]];
    if (!p.luma || !p.cb || !p.cr || p.width != a.width || p.height != a.height) return false;
  }
  return true;
}

__global__ __launch_bounds__(kMcNT) void k_mc(McArgs a) {
  __shared__ int16_t tmp[kMcTmp];
  __shared__ int16_t acc[64 * 64];
  const fme_mc_job j = a.jobs[blockIdx.x];
  if (!mc_job_valid(a, j)) {
    if (threadIdx.x == 0) atomicAdd(a.invalid, 1);
    return;
  }
  int nl = 0, lists[2];
  if (j.flags & FME_MC_L0) lists[nl++] = 0;
  if (j.flags & FME_MC_L1) lists[nl++] = 1;
  if (nl == 2 && j.ref_id[0] == j.ref_id[1] && j.mv[0][0] == j.mv[1][0] && j.mv[0][1] == j.mv[1][1])
    nl = 1;   // xCheckIdenticalMotion: same picture, same MV -> xPredInterUni(REF_PIC_LIST_0)
  for (int comp = 0; comp < 3; comp++) {
    const int cs = comp ? 1 : 0;   // getComponentScaleX/Y for 4:2:0 chroma
    const int W = j.w >> cs, H = j.h >> cs, x0 = j.x >> cs, y0 = j.y >> cs;
    uint8_t* dst = comp == 0 ? a.y + (size_t)y0 * a.y_stride + x0
                             : (comp == 1 ? a.cb : a.cr) + (size_t)y0 * a.c_stride + x0;
    const int dst_stride = comp ? a.c_stride : a.y_stride;
    for (int k = 0; k < nl; k++) {
      const int l = lists[k];
      const PicDesc& pd = a.pics[j.ref_id[l]];
      int mx = j.mv[l][0], my = j.mv[l][1];
      clip_mv(mx, my, pd.width, pd.height, j.cu_x, j.cu_y);
      const int sh = 2 + cs, mask = (1 << sh) - 1;
      const Plane ref = comp == 0 ? Plane{pd.luma, pd.stride, pd.width, pd.height}
                                  : Plane{comp == 1 ? pd.cb : pd.cr, pd.cstride, pd.width >> 1, pd.height >> 1};
      const int mode = nl == 1 ? 0 : (k == 0 ? 1 : 2);
      if (comp == 0)
        pred_block<8>(ref, x0, y0, W, H, mx >> sh, my >> sh, mx & mask, my & mask, mode, tmp, acc, dst, dst_stride);
      else
        pred_block<4>(ref, x0, y0, W, H, mx >> sh, my >> sh, mx & mask, my & mask, mode, tmp, acc, dst, dst_stride);
    }
  }
}

}  // namespace

hipError_t launch_mc(const McArgs& a, hipStream_t s) {
  if (a.n > 0) hipLaunchKernelGGL(k_mc, dim3(a.n), dim3(kMcNT), 0, s, a);
  return hipGetLastError();
}

}  // namespace fme
