// hvx_lib.hip -- libhvx.so: the C-ABI of include/hvx.h, HIP context and launchers (gfx950).
// Single translation unit: the kernels live in the *.hpp files included below.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hvx_dev.hpp"
#include "hvx_dist_interp.hpp"
#include "hvx_me.hpp"
#include "hvx_ssim.hpp"
#include "hvx_tu.hpp"

struct hvx_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
};

namespace {
thread_local std::string g_err;

int fail(int code, const char *what) {
  g_err = what;
  return code;
}

int hip_fail(hipError_t e, const char *what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return HVX_E_HIP - (int)e;
}

#define HVX_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(e_, #call);   \
  } while (0)

int launched(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, what);
  return HVX_OK;
}

// ---- host generation of the constant tables (HEVC spec rules; TComRom.cpp:192-262) ----
const int kCosH[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
int dct32(int k, int n) {
  if (k == 0) return 64;
  int j = (k * (2 * n + 1)) % 128, sign = 1;
  if (j > 64) j = 128 - j;
  if (j > 32) { j = 64 - j; sign = -1; }
  return sign * kCosH[j];
}

void gen_scan(std::vector<int> &out, int w, int h, int stride, int type, int offx, int offy) {
  if (type == 0) {
    for (int d = 0; d < w + h - 1; d++) {
      int y = d < h - 1 ? d : h - 1, x = d - y;
      while (y >= 0 && x < w) out.push_back((y + offy) * stride + x + offx), y--, x++;
    }
  } else if (type == 1) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) out.push_back((y + offy) * stride + x + offx);
  } else {
    for (int x = 0; x < w; x++)
      for (int y = 0; y < h; y++) out.push_back((y + offy) * stride + x + offx);
  }
}

int upload_tables() {
  uint16_t scan[3][1360];
  uint8_t scan_cg[3][85];
  int16_t mat[1360];
  for (int t = 0; t < 3; t++) {
    int sb = 0, cb = 0;
    for (int l = 0; l < 4; l++) {
      const int n = 4 << l, g = 1 << l;
      std::vector<int> cg, full;
      gen_scan(cg, g, g, g, t, 0, 0);
      for (int i = 0; i < g * g; i++) {
        const int gx = cg[i] % g, gy = cg[i] / g;
        gen_scan(full, 4, 4, n, t, gx * 4, gy * 4);
      }
      for (int i = 0; i < n * n; i++) scan[t][sb + i] = (uint16_t)full[i];
      for (int i = 0; i < g * g; i++) scan_cg[t][cb + i] = (uint8_t)cg[i];
      sb += n * n;
      cb += g * g;
    }
  }
  int mb = 0;
  for (int l = 0; l < 4; l++) {
    const int n = 4 << l;
    for (int k = 0; k < n; k++)
      for (int x = 0; x < n; x++) mat[mb + k * n + x] = (int16_t)dct32(k * (32 / n), x);
    mb += n * n;
  }
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kScan), scan, sizeof(scan)));
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kScanCG), scan_cg, sizeof(scan_cg)));
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kMat), mat, sizeof(mat)));
  return HVX_OK;
}
}  // namespace

template <int MODE>
static int tu_launch(hvx_ctx *ctx, const hvx_tu_desc *desc, const hvx_estbits *est, const int32_t *est_idx,
                     const int64_t *off, int n, const int16_t *res_in, int32_t *temp, int32_t *lev, int32_t *arl,
                     int32_t *abs_sum, int16_t *res_out, uint32_t *sse) {
  // one launch per TU size class; workgroups of TUs of another size exit at once
  hipLaunchKernelGGL((k_tu<0, MODE>), dim3(n), dim3(64), 0, ctx->stream, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse);
  hipLaunchKernelGGL((k_tu<1, MODE>), dim3(n), dim3(64), 0, ctx->stream, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse);
  hipLaunchKernelGGL((k_tu<2, MODE>), dim3(n), dim3(64), 0, ctx->stream, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse);
  hipLaunchKernelGGL((k_tu<3, MODE>), dim3(n), dim3(64), 0, ctx->stream, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse);
  return launched("k_tu");
}


extern "C" {

int hvx_version(void) { return 1; }
const char *hvx_last_error(void) { return g_err.c_str(); }

int hvx_create(int device, hvx_ctx **out) {
  if (!out) return fail(HVX_E_INVALID, "hvx_create: out is NULL");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(HVX_E_NODEV, "hvx_create: no HIP device");
  if (device < 0 || device >= ndev) return fail(HVX_E_INVALID, "hvx_create: bad device index");
  HVX_HIP(hipSetDevice(device));
  int rc = upload_tables();
  if (rc) return rc;
  hvx_ctx *c = new hvx_ctx;
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (e != hipSuccess) { delete c; return hip_fail(e, "hipStreamCreate"); }
  c->stream = c->own;
  *out = c;
  return HVX_OK;
}

int hvx_destroy(hvx_ctx *ctx) {
  if (!ctx) return HVX_OK;
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  delete ctx;
  return HVX_OK;
}

int hvx_set_stream(hvx_ctx *ctx, void *stream) {
  if (!ctx) return fail(HVX_E_INVALID, "hvx_set_stream: NULL ctx");
  ctx->stream = stream ? (hipStream_t)stream : ctx->own;
  return HVX_OK;
}

void *hvx_get_stream(hvx_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int hvx_sync(hvx_ctx *ctx) {
  if (!ctx) return fail(HVX_E_INVALID, "hvx_sync: NULL ctx");
  HVX_HIP(hipStreamSynchronize(ctx->stream));
  return HVX_OK;
}

int hvx_dist_batch(hvx_ctx *ctx, const int16_t *d_org, const int16_t *d_cur, const hvx_dist_job *d_jobs, int n,
                   uint32_t *d_out) {
  if (!ctx || n < 0 || (n && (!d_org || !d_cur || !d_jobs || !d_out))) return fail(HVX_E_INVALID, "hvx_dist_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_dist, dim3((n + 3) / 4), dim3(256), 0, ctx->stream, d_org, d_cur, d_jobs, n, d_out);
  return launched("k_dist");
}

int hvx_interp_batch(hvx_ctx *ctx, const int16_t *d_src, int16_t *d_dst, const hvx_interp_job *d_jobs, int n) {
  if (!ctx || n < 0 || (n && (!d_src || !d_dst || !d_jobs))) return fail(HVX_E_INVALID, "hvx_interp_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_interp, dim3(n), dim3(256), 0, ctx->stream, d_src, d_dst, d_jobs);
  return launched("k_interp");
}

int hvx_tu_forward_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const hvx_estbits *d_est, const int32_t *d_est_idx,
                         const int64_t *d_off, int n, const int16_t *d_residual, int32_t *d_temp, int32_t *d_levels,
                         int32_t *d_arl, int32_t *d_abs_sum) {
  if (!ctx || n < 0 || (n && (!d_desc || !d_est || !d_off || !d_residual || !d_levels)))
    return fail(HVX_E_INVALID, "hvx_tu_forward_batch: bad args");
  if (!n) return HVX_OK;
  return tu_launch<0>(ctx, d_desc, d_est, d_est_idx, d_off, n, d_residual, d_temp, d_levels, d_arl, d_abs_sum, nullptr, nullptr);
}

int hvx_tu_inverse_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, int n, const int32_t *d_levels,
                         int16_t *d_residual_out) {
  if (!ctx || n < 0 || (n && (!d_desc || !d_off || !d_levels || !d_residual_out)))
    return fail(HVX_E_INVALID, "hvx_tu_inverse_batch: bad args");
  if (!n) return HVX_OK;
  return tu_launch<1>(ctx, d_desc, nullptr, nullptr, d_off, n, nullptr, nullptr, const_cast<int32_t *>(d_levels), nullptr,
                      nullptr, d_residual_out, nullptr);
}

int hvx_tu_pipeline_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const hvx_estbits *d_est, const int32_t *d_est_idx,
                          const int64_t *d_off, int n, const int16_t *d_residual, int32_t *d_levels,
                          int32_t *d_abs_sum, int16_t *d_residual_out, uint32_t *d_sse) {
  if (!ctx || n < 0 || (n && (!d_desc || !d_est || !d_off || !d_residual || !d_levels || !d_residual_out)))
    return fail(HVX_E_INVALID, "hvx_tu_pipeline_batch: bad args");
  if (!n) return HVX_OK;
  return tu_launch<2>(ctx, d_desc, d_est, d_est_idx, d_off, n, d_residual, nullptr, d_levels, nullptr, d_abs_sum,
                      d_residual_out, d_sse);
}

int hvx_me_batch(hvx_ctx *ctx, const uint8_t *const *d_cur_planes, const uint8_t *const *d_ref_planes, int stride,
                 const hvx_me_job *d_jobs, int n, hvx_me_result *d_out) {
  if (!ctx || n < 0 || stride <= 0 || (n && (!d_cur_planes || !d_ref_planes || !d_jobs || !d_out)))
    return fail(HVX_E_INVALID, "hvx_me_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_me, dim3(n), dim3(64), 0, ctx->stream, d_cur_planes, d_ref_planes, stride, d_jobs, n, d_out);
  return launched("k_me");
}

int hvx_ssim_batch(hvx_ctx *ctx, const uint8_t *d_org, const uint8_t *d_rec, const hvx_ssim_job *d_jobs, int n,
                   float *d_out) {
  if (!ctx || n < 0 || (n && (!d_org || !d_rec || !d_jobs || !d_out))) return fail(HVX_E_INVALID, "hvx_ssim_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_ssim, dim3(n), dim3(64), 0, ctx->stream, d_org, d_rec, d_jobs, n, d_out);
  return launched("k_ssim");
}

int hvx_stvssim_batch(hvx_ctx *ctx, const uint8_t *const *d_hist_org, const uint8_t *const *d_hist_rec,
                      const float *d_dirs, const hvx_stvssim_job *d_jobs, int n, float *d_out4) {
  if (!ctx || n < 0 || (n && (!d_hist_org || !d_hist_rec || !d_dirs || !d_jobs || !d_out4)))
    return fail(HVX_E_INVALID, "hvx_stvssim_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_stvssim, dim3(n), dim3(64), 0, ctx->stream, d_hist_org, d_hist_rec, d_dirs, d_jobs, n, d_out4);
  return launched("k_stvssim");
}

int hvx_plane_extend(hvx_ctx *ctx, uint8_t *d_plane, int width, int height) {
  if (!ctx || !d_plane || width <= 0 || height <= 0) return fail(HVX_E_INVALID, "hvx_plane_extend: bad args");
  const int M = HVX_PLANE_MARGIN, stride = width + 2 * M;
  hipLaunchKernelGGL(k_plane_extend, dim3((2 * M + 255) / 256, height), dim3(256), 0, ctx->stream, d_plane, stride, width, height, M, 0);
  hipLaunchKernelGGL(k_plane_extend, dim3((stride + 255) / 256, 2 * M), dim3(256), 0, ctx->stream, d_plane, stride, width, height, M, 1);
  return launched("k_plane_extend");
}

int hvx_plane_from_pel(hvx_ctx *ctx, const int16_t *d_pel, int pel_stride, int width, int height, uint8_t *d_plane) {
  if (!ctx || !d_pel || !d_plane || width <= 0 || height <= 0 || pel_stride < width)
    return fail(HVX_E_INVALID, "hvx_plane_from_pel: bad args");
  const int stride = width + 2 * HVX_PLANE_MARGIN;
  hipLaunchKernelGGL(k_plane_from_pel, dim3((width + 255) / 256, height), dim3(256), 0, ctx->stream, d_pel, pel_stride, width, height, d_plane, stride);
  int rc = launched("k_plane_from_pel");
  if (rc) return rc;
  return hvx_plane_extend(ctx, d_plane, width, height);
}

}  // extern "C"
