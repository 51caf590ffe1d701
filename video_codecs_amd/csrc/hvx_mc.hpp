// hvx_mc.hpp -- motion compensation (gfx950): TComPrediction::motionCompensation for one PU
// without weighted prediction (TComPrediction.cpp:517-722: xPredInterUni / xPredInterBi /
// xPredInterBlk / xWeightedAverage; TComYuv::addAvg TComYuv.cpp:352;
// TComInterpolationFilter::filter / filterCopy TComInterpolationFilter.cpp:94-257).
//
// Mapping: one 256-thread workgroup per PU.  Per component and list the prediction follows
// xPredInterBlk's three paths exactly: horizontal-only, vertical-only, or horizontal
// (non-last, into an LDS intermediate of h+N-1 rows) then vertical; for bi-prediction both
// lists stay 14-bit intermediates in LDS and are averaged by addAvg.  8-bit, 4:2:0.
#pragma once
#include "hvx_dev.hpp"

// TComInterpolationFilter::filter<N, *, isFirst, isLast> output stage, 8-bit
// (IF_INTERNAL_PREC 14, IF_FILTER_PREC 6, IF_INTERNAL_OFFS 8192)
__device__ __forceinline__ int mc_fir_out(int sum, bool first, bool last) {
  if (last) {
    const int sh = first ? 6 : 12, off = (1 << (sh - 1)) + (first ? 0 : (8192 << 6));
    return clip_pel((int16_t)((sum + off) >> sh));
  }
  return (int16_t)(first ? sum - 8192 : sum >> 6);
}
// filterCopy (:94) with isFirst = true
__device__ __forceinline__ int mc_copy_first(int v, bool last) { return last ? v : (int16_t)((int16_t)(v << 6) - 8192); }

struct McSmem {
  int16_t tmp[(64 + 7) * 64];  // first-stage intermediate (h + N - 1 rows, stride w)
  int16_t pr[2][64 * 64];      // per-list prediction (stride w)
};

// xPredInterBlk (:668) for one component and list into dst (stride w)
__device__ void mc_pred_blk(bool luma, const int16_t *plane, int stride, int x, int y, int mvx, int mvy, int w, int h,
                            bool bi, int16_t *dst, int16_t *tmp) {
  const int sh = luma ? 2 : 3, n = luma ? 8 : 4;
  const int xf = mvx & ((1 << sh) - 1), yf = mvy & ((1 << sh) - 1);
  const int16_t *ref = plane + (y + (mvy >> sh)) * stride + x + (mvx >> sh);
  const int8_t *cx = luma ? kLumaFilter[xf] : kChromaFilter[xf];
  const int8_t *cy = luma ? kLumaFilter[yf] : kChromaFilter[yf];
  const int half = n / 2 - 1;
  if (yf == 0) {  // filterHor(xf, isLast = !bi): filterCopy when xf == 0
    for (int k = threadIdx.x; k < w * h; k += blockDim.x) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = ref + r * stride + c;
      if (xf == 0) {
        dst[k] = (int16_t)mc_copy_first(p[0], !bi);
      } else {
        int s = 0;
        for (int t = 0; t < n; t++) s += cx[t] * p[t - half];
        dst[k] = (int16_t)mc_fir_out(s, true, !bi);
      }
    }
  } else if (xf == 0) {  // filterVer(yf, isFirst, isLast = !bi)
    for (int k = threadIdx.x; k < w * h; k += blockDim.x) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = ref + r * stride + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cy[t] * p[(t - half) * stride];
      dst[k] = (int16_t)mc_fir_out(s, true, !bi);
    }
  } else {  // filterHor(non-last) into tmp over h + n - 1 rows, then filterVer(non-first, isLast = !bi)
    const int16_t *src = ref - half * stride;
    for (int k = threadIdx.x; k < w * (h + n - 1); k += blockDim.x) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = src + r * stride + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cx[t] * p[t - half];
      tmp[k] = (int16_t)mc_fir_out(s, true, false);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < w * h; k += blockDim.x) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = tmp + (r + half) * w + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cy[t] * p[(t - half) * w];
      dst[k] = (int16_t)mc_fir_out(s, false, !bi);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void mc_clip(const hvx_mc_job &j, int &mx, int &my) {  // TComDataCU::clipMv
  const int hmax = (j.pic_w + 8 - j.cu_x - 1) << 2, hmin = (-j.max_cu - 8 - j.cu_x + 1) << 2;
  const int vmax = (j.pic_h + 8 - j.cu_y - 1) << 2, vmin = (-j.max_cu - 8 - j.cu_y + 1) << 2;
  mx = (int16_t)(mx < hmin ? hmin : mx > hmax ? hmax : mx);
  my = (int16_t)(my < vmin ? vmin : my > vmax ? vmax : my);
}

static __global__ __launch_bounds__(256) void k_mc(const int16_t *const *__restrict__ planes, int ls, int cs,
                                            const hvx_mc_job *__restrict__ jobs, int n, int16_t *__restrict__ out) {
  __shared__ McSmem sm;
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_mc_job j = jobs[jid];
  const bool v0 = j.ref[0] >= 0, v1 = j.ref[1] >= 0;
  const bool identical = (j.flags & HVX_MC_B_SLICE) && v0 && v1 && j.poc[0] == j.poc[1] && j.mv_x[0] == j.mv_x[1] &&
                         j.mv_y[0] == j.mv_y[1];
  const bool bi = v0 && v1 && !identical;
  const int l0 = v0 ? 0 : 1;  // the list of a uni-prediction
  int mx[2] = {j.mv_x[0], j.mv_x[1]}, my[2] = {j.mv_y[0], j.mv_y[1]};
  mc_clip(j, mx[0], my[0]);
  mc_clip(j, mx[1], my[1]);
  int16_t *dst = out + j.dst_offset;
  for (int comp = 0; comp < 3; comp++) {
    const bool luma = comp == 0;
    const int w = luma ? j.w : j.w >> 1, h = luma ? j.h : j.h >> 1;
    const int x = luma ? j.pu_x : j.pu_x >> 1, y = luma ? j.pu_y : j.pu_y >> 1;
    const int stride = luma ? ls : cs;
    int16_t *o = dst + (comp == 0 ? 0 : comp == 1 ? j.w * j.h : j.w * j.h + w * h);
    if (bi) {
      for (int l = 0; l < 2; l++)
        mc_pred_blk(luma, planes[3 * j.ref[l] + comp], stride, x, y, mx[l], my[l], w, h, true, sm.pr[l], sm.tmp);
      for (int k = threadIdx.x; k < w * h; k += blockDim.x)  // addAvg: shift 7, offset 64 + 2*8192
        o[k] = (int16_t)clip_pel((sm.pr[0][k] + sm.pr[1][k] + 16448) >> 7);
    } else {
      mc_pred_blk(luma, planes[3 * j.ref[l0] + comp], stride, x, y, mx[l0], my[l0], w, h, false, sm.pr[0], sm.tmp);
      for (int k = threadIdx.x; k < w * h; k += blockDim.x) o[k] = sm.pr[0][k];
    }
    __syncthreads();
  }
}
