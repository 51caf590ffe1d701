// hvx_lib.hip -- libhvx.so: the C-ABI of include/hvx.h, HIP context and launchers (gfx950).
// The kernels live in the *.hpp files included below; the HM-exact CTU engine is its own
// translation unit (hvx_hm.hip).  Kernels and constant tables of the headers have internal
// linkage, so each translation unit carries (and uploads) its own copies.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hvx_dev.hpp"
#include "hvx_dist_interp.hpp"
#include "hvx_me.hpp"
#include "hvx_ssim.hpp"
#include "hvx_tu.hpp"
#include "hvx_estbit.hpp"
#include "hvx_mc.hpp"
#include "hvx_cabac.hpp"
#include "hvx_intra.hpp"
#include "hvx_deblock.hpp"
#include "hvx_sao.hpp"
#include "hvx_hmloop.hpp"
#include "hvx_saodec.hpp"
#include "hvx_host.hpp"
#include "hvx_tables.hpp"


// staging layout (bytes): desc | est | off | residual (1024 int16) | levels | arl | abs | resout
#define HVX_STG_DESC 0
#define HVX_STG_EST 128
#define HVX_STG_OFF (HVX_STG_EST + 1024)
#define HVX_STG_RES (HVX_STG_OFF + 64)
#define HVX_STG_LEV (HVX_STG_RES + 2048)
#define HVX_STG_ARL (HVX_STG_LEV + 4096)
#define HVX_STG_ABS (HVX_STG_ARL + 4096)
#define HVX_STG_OUT (HVX_STG_ABS + 64)
#define HVX_STG_SIZE (HVX_STG_OUT + 2048)


namespace hvxi {
thread_local std::string g_err;

int fail(int code, const char *what) {
  g_err = what;
  return code;
}

int hip_fail(hipError_t e, const char *what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return HVX_E_HIP - (int)e;
}

int launched(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, what);
  return HVX_OK;
}
}  // namespace hvxi
using namespace hvxi;

// Batched TU pipeline (k_tu_fwd -> k_tu_rdoq -> k_tu_fin) for one size class over TUs
// [0, n) of the arrays; G TUs per RDOQ wave; scratch arrays hold ceil(n/G)*G*NN words.
template <int L, int MODE>
static void tu_class_launch(hipStream_t st, const hvx_tu_desc *desc, const hvx_estbits *est, const int32_t *est_idx,
                            const int64_t *off, int n, const int16_t *res_in, int32_t *temp, int32_t *lev, int32_t *arl,
                            int32_t *abs_sum, int16_t *res_out, uint32_t *sse, uint32_t *coefI, uint32_t *cxI,
                            int32_t *levI, int32_t *stI, int8_t *flags, int G, int n_est_lds) {
  hipLaunchKernelGGL((k_tu_fwd<L>), dim3(n), dim3(64), 0, st, desc, off, n, res_in, temp, arl, coefI, cxI, levI, abs_sum,
                     flags, G, 0);
  hipLaunchKernelGGL((k_tu_rdoq<L>), dim3((n + G - 1) / G), dim3(64), 0, st, desc, est, est_idx, n, coefI, cxI, levI, stI,
                     abs_sum, flags, G, n_est_lds, 0);
  hipLaunchKernelGGL((k_tu_fin<L, MODE>), dim3(n), dim3(64), 0, st, desc, off, n, res_in, levI, lev, res_out, sse, G,
                     (const uint8_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
}

// TUs per lane-parallel RDOQ wave: enough waves to fill the chip (~2 per SIMD), at most 64
static int tu_group(int n) {
  int g = 1;
  while (g < 64 && (size_t)(g * 2) * 2048 <= (size_t)n) g *= 2;
  return g;
}

template <int MODE>
static int tu_batch(hvx_ctx *ctx, const hvx_tu_desc *desc, const hvx_estbits *est, const int32_t *est_idx,
                    const int64_t *off, int n, const int16_t *res_in, int32_t *temp, int32_t *lev, int32_t *arl,
                    int32_t *abs_sum, int16_t *res_out, uint32_t *sse) {
  const int G = tu_group(n);
  const size_t npad = (size_t)(n + G - 1) / G * G;
  const size_t need = 4 * npad * 1024 * sizeof(int32_t) + npad + 256;
  if (ctx->tu_scr_bytes < need) {
    if (ctx->tu_scr) (void)hipFree(ctx->tu_scr);
    ctx->tu_scr = nullptr;
    ctx->tu_scr_bytes = 0;
    HVX_HIP(hipMalloc(&ctx->tu_scr, need));
    ctx->tu_scr_bytes = need;
  }
  uint32_t *coefI = (uint32_t *)ctx->tu_scr, *cxI = coefI + npad * 1024;
  int32_t *levI = (int32_t *)(cxI + npad * 1024), *stI = levI + npad * 1024;
  int8_t *flags = (int8_t *)(stI + npad * 1024);
  hipStream_t st = ctx->stream;
  // one pipeline per size class; workgroups / lanes of TUs of another size exit at once
  tu_class_launch<0, MODE>(st, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse, coefI, cxI, levI, stI, flags, G, 0);
  tu_class_launch<1, MODE>(st, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse, coefI, cxI, levI, stI, flags, G, 0);
  tu_class_launch<2, MODE>(st, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse, coefI, cxI, levI, stI, flags, G, 0);
  tu_class_launch<3, MODE>(st, desc, est, est_idx, off, n, res_in, temp, lev, arl, abs_sum, res_out, sse, coefI, cxI, levI, stI, flags, G, 0);
  return launched("tu_batch");
}

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
  if (const char *st = getenv("HVX_STACK_LIMIT")) HVX_HIP(hipDeviceSetLimit(hipLimitStackSize, (size_t)atol(st)));  // debugging
  int rc = upload_tables();
  if (rc) return rc;
  rc = hvx_hm_module_init();
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
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->tu_scr) (void)hipFree(ctx->tu_scr);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
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
  return tu_batch<0>(ctx, d_desc, d_est, d_est_idx, d_off, n, d_residual, d_temp, d_levels, d_arl, d_abs_sum, nullptr, nullptr);
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
  return tu_batch<2>(ctx, d_desc, d_est, d_est_idx, d_off, n, d_residual, nullptr, d_levels, nullptr, d_abs_sum,
                     d_residual_out, d_sse);
}

static int staging(hvx_ctx *ctx) {
  if (!ctx->scratch) {
    HVX_HIP(hipMalloc(&ctx->scratch, HVX_STG_SIZE));
    HVX_HIP(hipHostMalloc(&ctx->pinned, HVX_STG_SIZE, 0));
  }
  return HVX_OK;
}

int hvx_tu_forward_host(hvx_ctx *ctx, const hvx_tu_desc *h_desc, const hvx_estbits *h_est, const int16_t *h_residual,
                        int residual_stride, int32_t *h_levels, int32_t *h_arl, int32_t *h_abs_sum) {
  if (!ctx || !h_desc || !h_est || !h_residual || !h_levels || !h_abs_sum) return fail(HVX_E_INVALID, "hvx_tu_forward_host: NULL");
  const int w = h_desc->width, h = h_desc->height;
  if (w != h || (w != 4 && w != 8 && w != 16 && w != 32) || residual_stride < w) return fail(HVX_E_INVALID, "hvx_tu_forward_host: TU size");
  int rc = staging(ctx);
  if (rc) return rc;
  char *p = ctx->pinned;
  memcpy(p + HVX_STG_DESC, h_desc, sizeof(hvx_tu_desc));
  memcpy(p + HVX_STG_EST, h_est, sizeof(hvx_estbits));
  *(int64_t *)(p + HVX_STG_OFF) = 0;
  for (int y = 0; y < h; y++) memcpy(p + HVX_STG_RES + y * w * 2, h_residual + (size_t)y * residual_stride, w * 2);
  hipStream_t st = ctx->stream;
  char *d = ctx->scratch;
  HVX_HIP(hipMemcpyAsync(d, p, HVX_STG_LEV, hipMemcpyHostToDevice, st));
  const hvx_tu_desc *dd = (const hvx_tu_desc *)(d + HVX_STG_DESC);
  const hvx_estbits *de = (const hvx_estbits *)(d + HVX_STG_EST);
  const int64_t *doff = (const int64_t *)(d + HVX_STG_OFF);
  const int16_t *dres = (const int16_t *)(d + HVX_STG_RES);
  int32_t *dlev = (int32_t *)(d + HVX_STG_LEV), *darl = (int32_t *)(d + HVX_STG_ARL), *dabs = (int32_t *)(d + HVX_STG_ABS);
  switch (w) {  // one size class: no idle launches
    case 4: hipLaunchKernelGGL((k_tu<0, 0>), dim3(1), dim3(64), 0, st, dd, de, nullptr, doff, 1, dres, nullptr, dlev, darl, dabs, nullptr, nullptr); break;
    case 8: hipLaunchKernelGGL((k_tu<1, 0>), dim3(1), dim3(64), 0, st, dd, de, nullptr, doff, 1, dres, nullptr, dlev, darl, dabs, nullptr, nullptr); break;
    case 16: hipLaunchKernelGGL((k_tu<2, 0>), dim3(1), dim3(64), 0, st, dd, de, nullptr, doff, 1, dres, nullptr, dlev, darl, dabs, nullptr, nullptr); break;
    default: hipLaunchKernelGGL((k_tu<3, 0>), dim3(1), dim3(64), 0, st, dd, de, nullptr, doff, 1, dres, nullptr, dlev, darl, dabs, nullptr, nullptr); break;
  }
  rc = launched("hvx_tu_forward_host");
  if (rc) return rc;
  HVX_HIP(hipMemcpyAsync(p + HVX_STG_LEV, d + HVX_STG_LEV, HVX_STG_OUT - HVX_STG_LEV, hipMemcpyDeviceToHost, st));
  HVX_HIP(hipStreamSynchronize(st));
  memcpy(h_levels, p + HVX_STG_LEV, (size_t)w * h * 4);
  if (h_arl) memcpy(h_arl, p + HVX_STG_ARL, (size_t)w * h * 4);
  *h_abs_sum = *(int32_t *)(p + HVX_STG_ABS);
  return HVX_OK;
}

int hvx_tu_inverse_host(hvx_ctx *ctx, const hvx_tu_desc *h_desc, const int32_t *h_levels, int16_t *h_residual,
                        int residual_stride) {
  if (!ctx || !h_desc || !h_levels || !h_residual) return fail(HVX_E_INVALID, "hvx_tu_inverse_host: NULL");
  const int w = h_desc->width, h = h_desc->height;
  if (w != h || (w != 4 && w != 8 && w != 16 && w != 32) || residual_stride < w) return fail(HVX_E_INVALID, "hvx_tu_inverse_host: TU size");
  int rc = staging(ctx);
  if (rc) return rc;
  char *p = ctx->pinned;
  memcpy(p + HVX_STG_DESC, h_desc, sizeof(hvx_tu_desc));
  *(int64_t *)(p + HVX_STG_OFF) = 0;
  memcpy(p + HVX_STG_LEV, h_levels, (size_t)w * h * 4);
  hipStream_t st = ctx->stream;
  char *d = ctx->scratch;
  HVX_HIP(hipMemcpyAsync(d, p, HVX_STG_ARL, hipMemcpyHostToDevice, st));
  const hvx_tu_desc *dd = (const hvx_tu_desc *)(d + HVX_STG_DESC);
  const int64_t *doff = (const int64_t *)(d + HVX_STG_OFF);
  int32_t *dlev = (int32_t *)(d + HVX_STG_LEV);
  int16_t *dout = (int16_t *)(d + HVX_STG_OUT);
  switch (w) {
    case 4: hipLaunchKernelGGL((k_tu<0, 1>), dim3(1), dim3(64), 0, st, dd, nullptr, nullptr, doff, 1, nullptr, nullptr, dlev, nullptr, nullptr, dout, nullptr); break;
    case 8: hipLaunchKernelGGL((k_tu<1, 1>), dim3(1), dim3(64), 0, st, dd, nullptr, nullptr, doff, 1, nullptr, nullptr, dlev, nullptr, nullptr, dout, nullptr); break;
    case 16: hipLaunchKernelGGL((k_tu<2, 1>), dim3(1), dim3(64), 0, st, dd, nullptr, nullptr, doff, 1, nullptr, nullptr, dlev, nullptr, nullptr, dout, nullptr); break;
    default: hipLaunchKernelGGL((k_tu<3, 1>), dim3(1), dim3(64), 0, st, dd, nullptr, nullptr, doff, 1, nullptr, nullptr, dlev, nullptr, nullptr, dout, nullptr); break;
  }
  rc = launched("hvx_tu_inverse_host");
  if (rc) return rc;
  HVX_HIP(hipMemcpyAsync(p + HVX_STG_OUT, d + HVX_STG_OUT, (size_t)w * h * 2, hipMemcpyDeviceToHost, st));
  HVX_HIP(hipStreamSynchronize(st));
  for (int y = 0; y < h; y++) memcpy(h_residual + (size_t)y * residual_stride, p + HVX_STG_OUT + y * w * 2, w * 2);
  return HVX_OK;
}

int hvx_me_batch(hvx_ctx *ctx, const uint8_t *const *d_cur_planes, const uint8_t *const *d_ref_planes, int stride,
                 const hvx_me_job *d_jobs, int n, hvx_me_result *d_out) {
  if (!ctx || n < 0 || stride <= 0 || (n && (!d_cur_planes || !d_ref_planes || !d_jobs || !d_out)))
    return fail(HVX_E_INVALID, "hvx_me_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_me_int, dim3(n), dim3(64), 0, ctx->stream, d_cur_planes, d_ref_planes, stride, d_jobs, n, d_out);
  hipLaunchKernelGGL(k_me_frac, dim3(n), dim3(256), 0, ctx->stream, d_cur_planes, d_ref_planes, stride, d_jobs, n, d_out);
  return launched("k_me");
}

int hvx_mc_batch(hvx_ctx *ctx, const int16_t *const *d_planes, int luma_stride, int chroma_stride,
                 const hvx_mc_job *d_jobs, int n, int16_t *d_dst) {
  if (!ctx || n < 0 || luma_stride <= 0 || chroma_stride <= 0 || (n && (!d_planes || !d_jobs || !d_dst)))
    return fail(HVX_E_INVALID, "hvx_mc_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_mc, dim3(n), dim3(256), 0, ctx->stream, d_planes, luma_stride, chroma_stride, d_jobs, n, d_dst);
  return launched("k_mc");
}

int hvx_intra_pred_batch(hvx_ctx *ctx, const uint8_t *d_rec, int stride, const hvx_intra_job *d_jobs, int n,
                         uint8_t *d_pred, const int64_t *d_pred_off, int16_t *d_ref_out) {
  if (!ctx || n < 0 || stride <= 0 || (n && (!d_rec || !d_jobs || !d_pred || !d_pred_off)))
    return fail(HVX_E_INVALID, "hvx_intra_pred_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_intra_pred, dim3(n), dim3(64), 0, ctx->stream, d_rec, stride, d_jobs, n, d_pred, d_pred_off,
                     d_ref_out);
  return launched("k_intra_pred");
}

int hvx_intra_search_batch(hvx_ctx *ctx, const uint8_t *d_org, const uint8_t *d_rec, int stride,
                           const hvx_intra_job *d_jobs, int n, const int32_t *d_entropy_bits,
                           hvx_intra_search_result *d_out) {
  if (!ctx || n < 0 || stride <= 0 || (n && (!d_org || !d_rec || !d_jobs || !d_entropy_bits || !d_out)))
    return fail(HVX_E_INVALID, "hvx_intra_search_batch: bad args");
  if (!n) return HVX_OK;
  // 16x16..64x64 PUs: one wave per PU; 4x4 / 8x8 PUs: one PU per lane (each launch skips the
  // other sizes' jobs)
  hipLaunchKernelGGL(k_intra_search, dim3(n < 16384 ? n : 16384), dim3(64), 0, ctx->stream, d_org, d_rec, stride, d_jobs,
                     n, d_entropy_bits, d_out, 1);
  hipLaunchKernelGGL(k_intra_search_lane<2>, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, d_org, d_rec, stride, d_jobs,
                     n, d_entropy_bits, d_out);
  hipLaunchKernelGGL(k_intra_search_lane<3>, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, d_org, d_rec, stride, d_jobs,
                     n, d_entropy_bits, d_out);
  return launched("k_intra_search");
}

int hvx_deblock(hvx_ctx *ctx, uint8_t *d_y, int y_stride, uint8_t *d_cb, uint8_t *d_cr, int c_stride,
                const uint8_t *d_bs_ver, const uint8_t *d_bs_hor, const int8_t *d_qp, const hvx_deblock_params *h_params) {
  if (!ctx || !d_y || !d_cb || !d_cr || !d_bs_ver || !d_bs_hor || !d_qp || !h_params)
    return fail(HVX_E_INVALID, "hvx_deblock: NULL argument");
  const hvx_deblock_params P = *h_params;
  if (P.pic_w <= 0 || P.pic_h <= 0 || P.pic_w % 8 || P.pic_h % 8 || y_stride < P.pic_w || c_stride < P.pic_w / 2 ||
      P.beta_offset_div2 < -6 || P.beta_offset_div2 > 6 || P.tc_offset_div2 < -6 || P.tc_offset_div2 > 6 ||
      P.cb_qp_offset < -12 || P.cb_qp_offset > 12 || P.cr_qp_offset < -12 || P.cr_qp_offset > 12 || P.flags)
    return fail(HVX_E_INVALID, "hvx_deblock: bad parameters");
  const int nv = (P.pic_w / 8 - 1) * (P.pic_h / 4), nh = (P.pic_h / 8 - 1) * (P.pic_w / 4);
  if (nv > 0)
    hipLaunchKernelGGL(k_deblock<0>, dim3((nv + 255) / 256), dim3(256), 0, ctx->stream, d_y, y_stride, d_cb, d_cr,
                       c_stride, d_bs_ver, d_qp, P);
  if (nh > 0)
    hipLaunchKernelGGL(k_deblock<1>, dim3((nh + 255) / 256), dim3(256), 0, ctx->stream, d_y, y_stride, d_cb, d_cr,
                       c_stride, d_bs_hor, d_qp, P);
  return launched("k_deblock");
}

int hvx_sao_stats(hvx_ctx *ctx, const uint8_t *d_org_y, const uint8_t *d_org_cb, const uint8_t *d_org_cr,
                  int org_y_stride, int org_c_stride, const uint8_t *d_rec_y, const uint8_t *d_rec_cb,
                  const uint8_t *d_rec_cr, int rec_y_stride, int rec_c_stride, int pic_w, int pic_h,
                  hvx_sao_stat *d_stats) {
  if (!ctx || !d_org_y || !d_rec_y || !d_stats) return fail(HVX_E_INVALID, "hvx_sao_stats: NULL argument");
  const bool chroma = d_org_cb || d_org_cr || d_rec_cb || d_rec_cr;
  if (chroma && !(d_org_cb && d_org_cr && d_rec_cb && d_rec_cr))
    return fail(HVX_E_INVALID, "hvx_sao_stats: chroma planes must be all set or all NULL");
  if (pic_w <= 0 || pic_h <= 0 || pic_w % 8 || pic_h % 8 || org_y_stride < pic_w || rec_y_stride < pic_w ||
      (chroma && (org_c_stride < pic_w / 2 || rec_c_stride < pic_w / 2)))
    return fail(HVX_E_INVALID, "hvx_sao_stats: bad geometry");
  const int nctu = ((pic_w + 63) / 64) * ((pic_h + 63) / 64);
  hipLaunchKernelGGL(k_sao_stats, dim3(nctu, chroma ? 3 : 1), dim3(256), 0, ctx->stream, d_org_y, d_org_cb, d_org_cr,
                     org_y_stride, org_c_stride, d_rec_y, d_rec_cb, d_rec_cr, rec_y_stride, rec_c_stride, pic_w, pic_h,
                     d_stats);
  return launched("k_sao_stats");
}

int hvx_sao_apply(hvx_ctx *ctx, const uint8_t *d_src_y, const uint8_t *d_src_cb, const uint8_t *d_src_cr,
                  int src_y_stride, int src_c_stride, uint8_t *d_dst_y, uint8_t *d_dst_cb, uint8_t *d_dst_cr,
                  int dst_y_stride, int dst_c_stride, int pic_w, int pic_h, const hvx_sao_ctu *d_params) {
  if (!ctx || !d_src_y || !d_dst_y || !d_params) return fail(HVX_E_INVALID, "hvx_sao_apply: NULL argument");
  const bool chroma = d_src_cb || d_src_cr || d_dst_cb || d_dst_cr;
  if (chroma && !(d_src_cb && d_src_cr && d_dst_cb && d_dst_cr))
    return fail(HVX_E_INVALID, "hvx_sao_apply: chroma planes must be all set or all NULL");
  if (pic_w <= 0 || pic_h <= 0 || pic_w % 8 || pic_h % 8 || src_y_stride < pic_w || dst_y_stride < pic_w ||
      (chroma && (src_c_stride < pic_w / 2 || dst_c_stride < pic_w / 2)))
    return fail(HVX_E_INVALID, "hvx_sao_apply: bad geometry");
  if (d_src_y == d_dst_y || (chroma && (d_src_cb == d_dst_cb || d_src_cr == d_dst_cr)))
    return fail(HVX_E_INVALID, "hvx_sao_apply: src and dst planes must differ");
  const int groups = ((pic_w + 3) / 4) * pic_h;
  const int blocks = (groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096;
  hipLaunchKernelGGL(k_sao_apply, dim3(blocks, chroma ? 3 : 1), dim3(256), 0, ctx->stream, d_src_y, d_src_cb, d_src_cr,
                     src_y_stride, src_c_stride, d_dst_y, d_dst_cb, d_dst_cr, dst_y_stride, dst_c_stride, pic_w, pic_h,
                     d_params);
  return launched("k_sao_apply");
}

int hvx_alloc(hvx_ctx *ctx, size_t bytes, void **d_out) {
  if (!ctx || !d_out) return fail(HVX_E_INVALID, "hvx_alloc: NULL");
  HVX_HIP(hipMalloc(d_out, bytes ? bytes : 1));
  return HVX_OK;
}
int hvx_free(hvx_ctx *ctx, void *d) {
  if (!ctx) return fail(HVX_E_INVALID, "hvx_free: NULL ctx");
  if (d) HVX_HIP(hipFree(d));
  return HVX_OK;
}
int hvx_upload(hvx_ctx *ctx, void *d_dst, const void *h_src, size_t bytes) {
  if (!ctx || (bytes && (!d_dst || !h_src))) return fail(HVX_E_INVALID, "hvx_upload: NULL");
  if (bytes) HVX_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return HVX_OK;
}
int hvx_download(hvx_ctx *ctx, void *h_dst, const void *d_src, size_t bytes) {
  if (!ctx || (bytes && (!d_src || !h_dst))) return fail(HVX_E_INVALID, "hvx_download: NULL");
  if (bytes) HVX_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return HVX_OK;
}

int hvx_estbits_update(const uint8_t *ctx_states, const int32_t *entropy_bits, const uint32_t *rice_stats, int width,
                       int height, int ch_type, hvx_estbits *inout) {
  if (!ctx_states || !entropy_bits || !rice_stats || !inout) return fail(HVX_E_INVALID, "hvx_estbits_update: NULL");
  if (width != height || (width != 4 && width != 8 && width != 16 && width != 32) || ch_type < 0 || ch_type > 1)
    return fail(HVX_E_INVALID, "hvx_estbits_update: bad TU geometry");
  estbit_update(ctx_states, entropy_bits, rice_stats, width, height, ch_type, inout);
  return HVX_OK;
}

int hvx_estbits_batch(hvx_ctx *ctx, const uint8_t *d_states, const int32_t *d_entropy_bits, const uint32_t *d_rice,
                      const hvx_estbit_job *d_jobs, int n, hvx_estbits *d_inout) {
  if (!ctx || n < 0 || (n && (!d_states || !d_entropy_bits || !d_rice || !d_jobs || !d_inout)))
    return fail(HVX_E_INVALID, "hvx_estbits_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_estbits, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, d_states, d_entropy_bits, d_rice, d_jobs, n,
                     d_inout);
  return launched("k_estbits");
}

int hvx_coeff_bits_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, int n, const int32_t *d_levels,
                         const int32_t *d_entropy_bits, uint8_t *d_states, hvx_coeff_bits *d_out) {
  if (!ctx || n < 0 || (n && (!d_desc || !d_off || !d_levels || !d_entropy_bits || !d_states || !d_out)))
    return fail(HVX_E_INVALID, "hvx_coeff_bits_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_coeff_bits, dim3((n + 63) / 64), dim3(64), 0, ctx->stream, d_desc, d_off, n, d_levels,
                     d_entropy_bits, d_states, HVX_NUM_CTX, d_out);
  return launched("k_coeff_bits");
}

int hvx_coeff_write_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, const int32_t *d_levels,
                          const int32_t *d_stream_first, int n_streams, uint8_t *d_states, hvx_cabac_regs *d_regs,
                          uint8_t *d_out, const int64_t *d_out_off, int out_cap, int32_t *d_out_len) {
  if (!ctx || n_streams < 0 || out_cap < 0 ||
      (n_streams && (!d_desc || !d_off || !d_levels || !d_stream_first || !d_states || !d_regs || !d_out ||
                     !d_out_off || !d_out_len)))
    return fail(HVX_E_INVALID, "hvx_coeff_write_batch: bad args");
  if (!n_streams) return HVX_OK;
  hipLaunchKernelGGL(k_coeff_write, dim3((n_streams + kWriteRuns - 1) / kWriteRuns), dim3(64), 0, ctx->stream, d_desc, d_off, d_levels,
                     d_stream_first, n_streams, d_states, d_regs, d_out, d_out_off, out_cap, d_out_len);
  return launched("k_coeff_write");
}

int hvx_me_full_batch(hvx_ctx *ctx, const int16_t *const *d_tgt_planes, int tgt_stride,
                      const uint8_t *const *d_ref_planes, int stride, const hvx_me_job *d_jobs, int n,
                      hvx_me_result *d_out) {
  if (!ctx || n < 0 || stride <= 0 || tgt_stride <= 0 || (n && (!d_tgt_planes || !d_ref_planes || !d_jobs || !d_out)))
    return fail(HVX_E_INVALID, "hvx_me_full_batch: bad args");
  if (!n) return HVX_OK;
  hipLaunchKernelGGL(k_me_full, dim3(n), dim3(256), 0, ctx->stream, d_tgt_planes, tgt_stride, d_ref_planes, stride, d_jobs,
                     n, d_out);
  return launched("k_me_full");
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
  uint8_t *origin = d_plane + (size_t)M * stride + M;  // d_plane = start of the padded allocation
  hipLaunchKernelGGL(k_plane_extend, dim3((2 * M + 255) / 256, height), dim3(256), 0, ctx->stream, origin, stride, width, height, M, 0);
  hipLaunchKernelGGL(k_plane_extend, dim3((stride + 255) / 256, 2 * M), dim3(256), 0, ctx->stream, origin, stride, width, height, M, 1);
  return launched("k_plane_extend");
}

int hvx_plane_from_pel(hvx_ctx *ctx, const int16_t *d_pel, int pel_stride, int width, int height, uint8_t *d_plane) {
  if (!ctx || !d_pel || !d_plane || width <= 0 || height <= 0 || pel_stride < width)
    return fail(HVX_E_INVALID, "hvx_plane_from_pel: bad args");
  const int stride = width + 2 * HVX_PLANE_MARGIN;
  uint8_t *origin = d_plane + (size_t)HVX_PLANE_MARGIN * stride + HVX_PLANE_MARGIN;
  hipLaunchKernelGGL(k_plane_from_pel, dim3((width + 255) / 256, height), dim3(256), 0, ctx->stream, d_pel, pel_stride, width, height, origin, stride);
  int rc = launched("k_plane_from_pel");
  if (rc) return rc;
  return hvx_plane_extend(ctx, d_plane, width, height);
}


int hvx_hm_finish_picture(hvx_ctx *ctx, const hvx_hm_picture *h_pic, const hvx_deblock_params *h_dbk, uint8_t *d_work,
                          int16_t *d_col_field, uint8_t *d_ref8, int ref8_stride, int16_t *d_ref16_y, int16_t *d_ref16_cb,
                          int16_t *d_ref16_cr, int ref16_stride_y, int ref16_stride_c) {
  if (!ctx || !h_pic) return fail(HVX_E_INVALID, "hvx_hm_finish_picture: NULL argument");
  const hvx_hm_picture &P = *h_pic;
  const int w = P.w, h = P.h;
  if (w <= 0 || h <= 0 || w % 8 || h % 8 || P.w_ctus != (w + 63) / 64 || P.h_ctus != (h + 63) / 64 || !P.ctus ||
      !P.rec[0] || !P.rec[1] || !P.rec[2] || P.rec_stride[0] < w || P.rec_stride[1] < w / 2)
    return fail(HVX_E_INVALID, "hvx_hm_finish_picture: bad picture");
  const bool ref16 = d_ref16_y || d_ref16_cb || d_ref16_cr;
  if ((ref16 && !(d_ref16_y && d_ref16_cb && d_ref16_cr && ref16_stride_y >= w + 2 * 80 && ref16_stride_c >= w / 2 + 2 * 40)) ||
      (d_ref8 && (ref8_stride < w + 2 * HVX_PLANE_MARGIN || ref8_stride % 4)))
    return fail(HVX_E_INVALID, "hvx_hm_finish_picture: bad reference planes");
  const int nctu = P.w_ctus * P.h_ctus;
  if (h_dbk) {  // loopFilterPic (TEncGOP.cpp:1465)
    if (!d_work || h_dbk->pic_w != w || h_dbk->pic_h != h) return fail(HVX_E_INVALID, "hvx_hm_finish_picture: bad deblocking args");
    LfPic L{w, h, P.w_ctus, P.slice_type == 0 ? 1 : 0, {}};
    for (int l = 0; l < 2; l++)
      for (int i = 0; i < 4; i++) L.ref_poc[l][i] = P.ref_poc[l][i];
    const size_t nu = (size_t)(w / 4) * (h / 4);
    uint8_t *bv = d_work, *bh = d_work + nu;
    int8_t *qp = (int8_t *)(d_work + 2 * nu);
    hipLaunchKernelGGL(k_hm_lf_params, dim3((unsigned)((nu + 255) / 256)), dim3(256), 0, ctx->stream, P.ctus, L, bv, bh, qp);
    int rc = launched("k_hm_lf_params");
    if (rc) return rc;
    rc = hvx_deblock(ctx, P.rec[0], P.rec_stride[0], P.rec[1], P.rec[2], P.rec_stride[1], bv, bh, qp, h_dbk);
    if (rc) return rc;
  }
  if (d_col_field) {  // TComPic::compressMotion (TEncGOP.cpp:1629)
    hipLaunchKernelGGL(k_hm_col_field, dim3((nctu * 16 + 255) / 256), dim3(256), 0, ctx->stream, P.ctus, w, h, P.w_ctus, nctu,
                       d_col_field);
    const int rc = launched("k_hm_col_field");
    if (rc) return rc;
  }
  // the reference formats with extended borders (TComSlice::setRefPicList -> extendPicBorder, TComSlice.cpp:351)
  if (d_ref8) {
    const int m = HVX_PLANE_MARGIN;
    hipLaunchKernelGGL(k_ref_plane<uint8_t>, dim3((w + 2 * m + 255) / 256, h + 2 * m), dim3(256), 0, ctx->stream,
                       (const uint8_t *)P.rec[0], P.rec_stride[0], w, h, m, d_ref8, ref8_stride);
    const int rc = launched("k_ref_plane");
    if (rc) return rc;
  }
  if (ref16) {
    int16_t *dst[3] = {d_ref16_y, d_ref16_cb, d_ref16_cr};
    for (int c = 0; c < 3; c++) {
      const int cw = c ? w / 2 : w, ch = c ? h / 2 : h, m = c ? 40 : 80;
      hipLaunchKernelGGL(k_ref_plane<int16_t>, dim3((cw + 2 * m + 255) / 256, ch + 2 * m), dim3(256), 0, ctx->stream,
                         (const uint8_t *)P.rec[c], P.rec_stride[c ? 1 : 0], cw, ch, m, dst[c], c ? ref16_stride_c : ref16_stride_y);
      const int rc = launched("k_ref_plane");
      if (rc) return rc;
    }
  }
  return HVX_OK;
}


int hvx_sao_decide(hvx_ctx *ctx, const hvx_sao_decide_job *d_jobs, int n_jobs) {
  if (!ctx || (n_jobs > 0 && !d_jobs) || n_jobs < 0) return fail(HVX_E_INVALID, "hvx_sao_decide: bad args");
  if (n_jobs == 0) return HVX_OK;
  hipLaunchKernelGGL(k_sao_decide, dim3(n_jobs), dim3(64), 0, ctx->stream, d_jobs, n_jobs);
  return launched("k_sao_decide");
}

}  // extern "C"

