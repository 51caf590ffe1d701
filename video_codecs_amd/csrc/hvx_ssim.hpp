// hvx_ssim.hpp -- SSIM / stVSSIM RDO metric (gfx950), JM stvssim semantics.
// Reference: stvssim_src/stvssimrdo2_att/lencod/src/stvssim.c compute_SSIM :491-566,
// compute_stVSSIM :587-830, orientation filters :116-334, calOrit :336.
//
// Mapping: one wave per block.  Each SSIM window is computed by one lane in the reference's
// float32 accumulation order (the window statistics are order-sensitive float sums); the
// per-window results go to LDS and lane 0 averages them in window raster order, as the
// reference does.  Float literals/promotions follow the reference (double where it uses 2.0).
#pragma once
#include "hvx_dev.hpp"
#include "hvx_ssimw.hpp"

__device__ __forceinline__ float ssim_window(const uint8_t *o, int so, const uint8_t *r, int sr, int wint) {
  const float C1 = 0.01f * 0.01f * (float)(255 * 255), C2 = 0.03f * 0.03f * (float)(255 * 255);
  const float wgt = 1.0f / (float)(wint * wint);
  float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
  for (int n = 0; n < wint; n++)
    for (int m = 0; m < wint; m++) {
      const int po = o[n * so + m], pe = r[n * sr + m];
      mo += wgt * po; me += wgt * pe;
      vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
    }
  const float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
  float s = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
  s /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
  return s;
}

static __global__ __launch_bounds__(64) void k_ssim(const uint8_t *__restrict__ org, const uint8_t *__restrict__ rec,
                                             const hvx_ssim_job *__restrict__ jobs, int n, float *__restrict__ out) {
  __shared__ float win[1024];
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_ssim_job j = jobs[jid];
  const int nx = (j.w - j.wint) / j.overlap + 1, ny = (j.h - j.wint) / j.overlap + 1;
  const int nw = nx * ny;
  for (int base = 0; base < nw; base += 1024) {
    const int cnt = nw - base < 1024 ? nw - base : 1024;
    for (int k = lane_id(); k < cnt; k += HVX_WAVE) {
      const int wi = base + k, wy = wi / nx, wx = wi - wy * nx;
      win[k] = ssim_window(org + j.org_off + wy * j.overlap * j.org_stride + wx * j.overlap, j.org_stride,
                           rec + j.rec_off + wy * j.overlap * j.rec_stride + wx * j.overlap, j.rec_stride, j.wint);
    }
    __syncthreads();
    if (lane_id() == 0) {
      float acc = base ? out[jid] : 0.0f;
      for (int k = 0; k < cnt; k++) acc += win[k];
      out[jid] = acc;
    }
    __syncthreads();
  }
  if (lane_id() == 0) {
    float dist = out[jid] / (float)nw;
    if (dist >= 1.0 && dist < 1.01) dist = 1.0f;
    out[jid] = dist;
  }
}

static __global__ __launch_bounds__(64) void k_stvssim(const uint8_t *const *__restrict__ hist_org,
                                                const uint8_t *const *__restrict__ hist_rec,
                                                const float *__restrict__ dirs, const hvx_stvssim_job *__restrict__ jobs,
                                                int n, float *__restrict__ out4) {
  __shared__ float w3[1024], ws[1024];
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_stvssim_job j = jobs[jid];
  const int used = j.gama < 26 ? j.gama : 26;
  const int uv = j.comp > 0 ? 2 : 1;
  const int wint = j.wint, hs = j.hist_stride;
  const uint8_t *const *ho = hist_org + (size_t)jid * 26;
  const uint8_t *const *hr = hist_rec + (size_t)jid * 26;
  const float wa = 0.6f, wb = 1.0f - wa;
  float wgta[4], wgtb[4];
  if (wint == 4) {
    wgta[0] = wgta[2] = wgta[1] = wgta[3] = wa / (wint * (used));
    wgtb[0] = wgtb[2] = wgtb[1] = wgtb[3] = wb / ((wint * wint - wint) * (used));
  } else {
    wgta[0] = wgta[2] = wa / (3 * wint * (used));
    wgta[1] = wgta[3] = wa / ((3 * wint - 2) * (used));
    wgtb[0] = wgtb[2] = wb / ((wint * wint - 3 * wint) * (used));
    wgtb[1] = wgtb[3] = wb / ((wint * wint - 3 * wint + 2) * (used));
  }
  const float C1 = 0.01f * 0.01f * (float)(255 * 255), C2 = 0.03f * 0.03f * (float)(255 * 255);
  const float kOrient[4] = {0, 3.1415926f / 4, 3.1415926f / 2, 3.1415926f * 3 / 4};
  const int nx = (j.w - wint) / j.overlap + 1, ny = (j.h - wint) / j.overlap + 1, nw = nx * ny;
  const float *dmap = dirs + j.dirs_off;
  for (int k = lane_id(); k < nw && k < 1024; k += HVX_WAVE) {
    const int wy = k / nx, wx = k - wy * nx;
    const int i = wx * j.overlap, jj = wy * j.overlap;
    float s3[4];
    for (int kk = 0; kk < 4; kk++) {
      float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
      for (int o = 0; o < used; o++) {
        const uint8_t *ro = ho[o], *re = hr[o];
        for (int nn = jj; nn < jj + wint; nn++)
          for (int m = i; m < i + wint; m++) {
            const float wgt = orient_weight(kk, wint, nn - jj, m - i, wgta[kk], wgtb[kk]);
            const int po = ro[nn * hs + m], pe = re[nn * hs + m];
            mo += wgt * po; me += wgt * pe;
            vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
          }
      }
      const float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
      float s = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
      s /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
      s3[kk] = s;
      if (s3[kk] >= 1.0 && s3[kk] < 1.01) s3[kk] = 1.0f;
    }
    short orit[4] = {0, 0, 0, 0};
    for (int nn = jj; nn < jj + wint; nn++)
      for (int m = i; m < i + wint; m++) {
        const float od = dmap[(nn * uv) * j.dirs_stride + m * uv];
        float dn[4], dx = 10000.0f;
        for (int q = 0; q < 4; q++) { dn[q] = (float)fabs(od - kOrient[q]); if (dn[q] < dx) dx = dn[q]; }
        for (int q = 0; q < 4; q++) if (fabs(dx - dn[q]) < 0.01f) orit[q]++;
      }
    short tmp = 0, inx = 0;
    for (int q = 0; q < 4; q++) if (orit[q] > tmp) { tmp = orit[q]; inx = (short)q; }
    int q;
    for (q = 0; q < 4; ++q) if ((tmp - orit[q]) < 10 && inx != q) break;
    w3[k] = q == 4 ? s3[inx] : (s3[inx] + s3[q]) / 2;
    ws[k] = ssim_window(ho[used - 1] + jj * hs + i, hs, hr[used - 1] + jj * hs + i, hs, wint);
  }
  __syncthreads();
  if (lane_id() == 0) {
    float s3x = 0, sx = 0, stx = 0;
    for (int k = 0; k < nw && k < 1024; k++) { s3x += w3[k]; sx += ws[k]; stx += ws[k] * w3[k]; }
    s3x /= (float)nw; sx /= (float)nw; stx /= (float)nw;
    const float ret = sx * s3x;
    if (stx >= 1.0 && stx < 1.01) stx = 1.0f;
    out4[jid * 4 + 0] = sx; out4[jid * 4 + 1] = s3x; out4[jid * 4 + 2] = stx; out4[jid * 4 + 3] = ret;
  }
}
