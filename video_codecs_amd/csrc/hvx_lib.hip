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
#include "hvx_ctu.hpp"
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

#ifndef HVX_D3_NC
#define HVX_D3_NC 4  // 8x8 CUs per wave of the depth-3 residual pass (8: 0.499 vs 0.473 ms isolated)
#endif
namespace {
size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }
// interleaved RDOQ scratch of the CTU pass: the 3 TU classes (8n 32x32, 16n 16x16, 64n 8x8),
// each padded to whole groups of kCtuG TUs
constexpr int kCtuG = 64;
size_t pad_g(size_t n) { return (n + kCtuG - 1) / kCtuG * kCtuG; }
size_t ctu_il_off16(int n) { return pad_g((size_t)8 * n) * 1024; }
size_t ctu_il_off8(int n) { return ctu_il_off16(n) + pad_g((size_t)16 * n) * 256; }
// 4:2:0 chroma classes: 16x16 (16n TUs), 8x8 (32n), 4x4 (128n + 128n transform-skip twins)
size_t ctu_il_offc16(int n) { return ctu_il_off8(n) + pad_g((size_t)64 * n) * 64; }
size_t ctu_il_offc8(int n) { return ctu_il_offc16(n) + pad_g((size_t)16 * n) * 256; }
size_t ctu_il_offc4(int n) { return ctu_il_offc8(n) + pad_g((size_t)32 * n) * 64; }
size_t ctu_il_words(int n) { return ctu_il_offc4(n) + pad_g((size_t)256 * n) * 16; }  // 4x4 TUs + their TS twins
struct CtuWs {
  size_t jobs, res, desc, off, est_idx, resid, lev, res_out, abs, sse, ptr, coefI, cxI, levI, stI, flags, cbits, bsv, bsh,
      qpm, pred, zd, csse, total;
};
CtuWs ctu_ws_layout(const CtuLayout &L) {
  CtuWs w;
  size_t o = 0;
  const size_t ncu = (size_t)L.nctu * HVX_CUS_PER_CTU, ntu = (size_t)L.ntu(), nres = (size_t)L.nres();
  w.jobs = o; o = align_up(o + ncu * L.nref * sizeof(hvx_me_job));
  w.res = o; o = align_up(o + ncu * L.nref * sizeof(hvx_me_result));
  w.desc = o; o = align_up(o + ntu * sizeof(hvx_tu_desc));
  w.off = o; o = align_up(o + ntu * sizeof(int64_t));
  w.est_idx = o; o = align_up(o + ntu * sizeof(int32_t));
  w.resid = o; o = align_up(o + nres * sizeof(int16_t));
  w.lev = o; o = align_up(o + nres * sizeof(int32_t));
  w.res_out = o; o = align_up(o + nres * sizeof(int16_t));
  w.abs = o; o = align_up(o + ntu * sizeof(int32_t));
  w.sse = o; o = align_up(o + ntu * sizeof(uint32_t));
  w.ptr = o; o = align_up(o + 8 * sizeof(void *));
  const size_t nil = ctu_il_words(L.nctu);
  w.coefI = o; o = align_up(o + nil * sizeof(int32_t));
  w.cxI = o; o = align_up(o + nil * sizeof(int32_t));
  w.levI = o; o = align_up(o + nil * sizeof(int32_t));
  w.stI = o; o = align_up(o + nil * sizeof(int32_t));
  w.flags = o; o = align_up(o + ntu);
  w.cbits = o; o = align_up(o + ntu * sizeof(hvx_coeff_bits));
  const size_t nunit = (size_t)L.nctu * 256;  // deblocking maps of the reference picture (>= (w/4)*(h/4))
  w.bsv = o; o = align_up(o + nunit);
  w.bsh = o; o = align_up(o + nunit);
  w.qpm = o; o = align_up(o + nunit);
  w.pred = o; o = align_up(o + nres);                     // 8-bit prediction, residual layout
  w.zd = o; o = align_up(o + ntu * sizeof(uint32_t));     // per TU: zero-residual distortion
  w.csse = o; o = align_up(o + ntu * sizeof(uint32_t));   // per TU: clipped-reconstruction distortion
  w.total = o;
  return w;
}
CtuLayout ctu_layout(int w, int h, int nref) {
  CtuLayout L;
  L.nctu_x = (w + 63) / 64; L.nctu_y = (h + 63) / 64; L.nctu = L.nctu_x * L.nctu_y; L.nref = nref;
  return L;
}
}  // namespace

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

namespace {
}  // namespace

static void fold_timing(hvx_ctx *ctx) {
  for (int k = 0; k < ctx->ntev; k++) {
    float ms = 0;
    (void)hipEventSynchronize(ctx->tev[2 * k + 1]);
    if (hipEventElapsedTime(&ms, ctx->tev[2 * k], ctx->tev[2 * k + 1]) == hipSuccess) ctx->phase_ms[ctx->tphase[k]] += ms;
  }
  ctx->ntev = 0;
}

// time the launches between t_begin and t_end on stream st as phase `phase` (no-op unless timing)
static int t_begin(hvx_ctx *ctx, hipStream_t st, int phase) {
  if (!ctx || !ctx->timing || !ctx->ev_ok || ctx->ntev >= hvx_ctx::kMaxTimed) return -1;
  const int k = ctx->ntev++;
  ctx->tphase[k] = phase;
  (void)hipEventRecord(ctx->tev[2 * k], st);
  return k;
}
static void t_end(hvx_ctx *ctx, hipStream_t st, int k) {
  if (k >= 0) (void)hipEventRecord(ctx->tev[2 * k + 1], st);
}

// Batched TU pipeline (k_tu_fwd -> k_tu_rdoq -> k_tu_fin) for one size class over TUs
// [0, n) of the arrays; G TUs per RDOQ wave; scratch arrays hold ceil(n/G)*G*NN words.
template <int L, int MODE>
static void tu_class_launch(hipStream_t st, const hvx_tu_desc *desc, const hvx_estbits *est, const int32_t *est_idx,
                            const int64_t *off, int n, const int16_t *res_in, int32_t *temp, int32_t *lev, int32_t *arl,
                            int32_t *abs_sum, int16_t *res_out, uint32_t *sse, uint32_t *coefI, uint32_t *cxI,
                            int32_t *levI, int32_t *stI, int8_t *flags, int G, int n_est_lds, hvx_ctx *tctx = nullptr,
                            int phase0 = 0, hipEvent_t after_rdoq = nullptr, const uint8_t *pred = nullptr,
                            uint32_t *zd = nullptr, uint32_t *csse = nullptr) {
  int k = t_begin(tctx, st, phase0);
  // the CTU pass's 4x4 / 8x8 TUs (RDOQ, inter: pred != nullptr marks that pass): one TU per lane
  const bool lane = L <= 1 && pred && G == 64 && !temp && !arl;
  // 16x16 / 32x32 of that pass: the forward kernel (wave per TU) writes the RDOQ inputs TU-major
  const int tm = L >= 2 && pred && !temp && !arl ? 1 : 0;
  if (lane)
    hipLaunchKernelGGL((k_tu_fwd_lane<L < 2 ? L : 1>), dim3((n + 63) / 64), dim3(64), 0, st, desc, off, n, res_in, coefI,
                       cxI, flags);
  else
    hipLaunchKernelGGL((k_tu_fwd<L>), dim3(n), dim3(64), 0, st, desc, off, n, res_in, temp, arl, coefI, cxI, levI, abs_sum,
                       flags, G, tm);
  t_end(tctx, st, k);
  k = t_begin(tctx, st, phase0 + 1);
  hipLaunchKernelGGL((k_tu_rdoq<L>), dim3((n + G - 1) / G), dim3(64), 0, st, desc, est, est_idx, n, coefI, cxI, levI, stI,
                     abs_sum, flags, G, n_est_lds, tm);
  t_end(tctx, st, k);
  if (after_rdoq) (void)hipEventRecord(after_rdoq, st);  // the levels are final: their rate may be counted beside k_tu_fin
  k = t_begin(tctx, st, phase0 + 2);
  if (lane && MODE == 2)
    hipLaunchKernelGGL((k_tu_fin_lane<L < 2 ? L : 1>), dim3((n + 63) / 64), dim3(64), 0, st, desc, off, n, res_in, levI,
                       lev, res_out, sse, pred, zd, csse);
  else
    hipLaunchKernelGGL((k_tu_fin<L, MODE>), dim3(n), dim3(64), 0, st, desc, off, n, res_in, levI, lev, res_out, sse, G,
                       pred, zd, csse);
  t_end(tctx, st, k);
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
  const char *ser = getenv("HVX_SERIAL_STREAMS");
  c->serial = ser && ser[0] == '1';
  // the side streams carry few, latency-bound workgroups (RDOQ chains): highest priority, so
  // they dispatch ahead of the ME kernels' backlog instead of waiting behind it
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = 0;
  for (int i = 0; i < 3 && e == hipSuccess; i++) e = hipStreamCreateWithPriority(&c->aux[i], hipStreamNonBlocking, prio_hi);
  for (int i = 0; i < 8 && e == hipSuccess; i++) e = hipEventCreateWithFlags(&c->fj[i], hipEventDisableTiming);
  if (e != hipSuccess) { hvx_destroy(c); return hip_fail(e, "hvx_create: streams/events"); }
  *out = c;
  return HVX_OK;
}

int hvx_destroy(hvx_ctx *ctx) {
  if (!ctx) return HVX_OK;
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->tu_scr) (void)hipFree(ctx->tu_scr);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  for (int i = 0; i < 3; i++)
    if (ctx->aux[i]) (void)hipStreamDestroy(ctx->aux[i]);
  for (int i = 0; i < 8; i++)
    if (ctx->fj[i]) (void)hipEventDestroy(ctx->fj[i]);
  if (ctx->ev_ok)
    for (int i = 0; i < 2 * hvx_ctx::kMaxTimed; i++) (void)hipEventDestroy(ctx->tev[i]);
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

int hvx_set_timing(hvx_ctx *ctx, int on) {
  if (!ctx) return fail(HVX_E_INVALID, "hvx_set_timing: NULL ctx");
  if (on && !ctx->ev_ok) {
    for (int i = 0; i < 2 * hvx_ctx::kMaxTimed; i++) HVX_HIP(hipEventCreate(&ctx->tev[i]));
    ctx->ev_ok = true;
  }
  ctx->timing = on;
  return HVX_OK;
}

int hvx_phase_times(hvx_ctx *ctx, double *ms_out, int n, int reset) {
  if (!ctx || !ms_out || n < HVX_NPHASE) return fail(HVX_E_INVALID, "hvx_phase_times: bad args");
  fold_timing(ctx);
  for (int i = 0; i < HVX_NPHASE; i++) ms_out[i] = ctx->phase_ms[i];
  if (reset)
    for (int i = 0; i < HVX_NPHASE; i++) ctx->phase_ms[i] = 0;
  return HVX_OK;
}

int hvx_ctu_workspace_size(int pic_w, int pic_h, int n_ref, size_t *bytes) {
  if (!bytes || pic_w <= 0 || pic_h <= 0 || n_ref <= 0 || n_ref > 8) return fail(HVX_E_INVALID, "hvx_ctu_workspace_size: bad args");
  *bytes = ctu_ws_layout(ctu_layout(pic_w, pic_h, n_ref)).total;
  return HVX_OK;
}

// cnt_states != NULL (hvx_ctu_encode): each TU size class's coefficient rate is counted on the
// class's own stream right behind its TU pipeline, so it overlaps the remaining searches
// the device-side view of hvx_chroma_planes (C.on = 0 without one)
static CtuChroma ctu_chroma(const hvx_chroma_planes *cp) {
  CtuChroma C;
  memset(&C, 0, sizeof(C));
  if (cp) {
    C.cur[0] = cp->cur_cb; C.cur[1] = cp->cur_cr; C.refs = cp->refs_c;
    C.recon[0] = cp->recon_cb; C.recon[1] = cp->recon_cr; C.stride = cp->c_stride; C.on = 1;
  }
  return C;
}

// chroma != NULL: 4:2:0 (P.chroma_format 1, d_est4 = 7 tables: luma 4x4..32x32, chroma 4x4..16x16)
static int ctu_analyze_impl(hvx_ctx *ctx, const uint8_t *d_cur, const uint8_t *const *d_refs, int stride,
                            const hvx_ctu_params *h_params, const hvx_estbits *d_est4, void *d_workspace, size_t ws_bytes,
                            hvx_cu_result *d_out, const uint8_t *cnt_states, const int32_t *cnt_eb,
                            const hvx_chroma_planes *chroma = nullptr) {
  if (!ctx || !d_cur || !d_refs || !h_params || !d_est4 || !d_workspace || !d_out)
    return fail(HVX_E_INVALID, "hvx_ctu_analyze: NULL argument");
  const hvx_ctu_params P = *h_params;
  if (P.pic_w <= 0 || P.pic_h <= 0 || P.n_ref <= 0 || P.n_ref > 8 || P.qp < 0 || P.qp > 51 ||
      stride < P.pic_w + 2 * HVX_PLANE_MARGIN || stride % 4 != 0 || P.search_range <= 0 || P.search_range > 256)
    return fail(HVX_E_INVALID, "hvx_ctu_analyze: bad parameters");
  if (P.chroma_format != (chroma ? 1 : 0))
    return fail(HVX_E_INVALID, "hvx_ctu_analyze: chroma_format must be 0 (luma entry points) or 1 (hvx_ctu_encode_yuv)");
  if (chroma && (!chroma->cur_cb || !chroma->cur_cr || !chroma->refs_c || chroma->c_stride % 4 != 0 ||
                 chroma->c_stride < P.pic_w / 2 + HVX_PLANE_MARGIN || P.pic_w % 8 || P.pic_h % 8 ||
                 P.qp_chroma < 0 || P.qp_chroma > 51 || !(P.chroma_weight > 0.0)))
    return fail(HVX_E_INVALID, "hvx_ctu_encode_yuv: bad chroma planes / parameters");
  const CtuChroma C = ctu_chroma(chroma);
  const int n_est = chroma ? 7 : 4;
  const CtuLayout L = ctu_layout(P.pic_w, P.pic_h, P.n_ref);
  const CtuWs W = ctu_ws_layout(L);
  if (ws_bytes < W.total) return fail(HVX_E_INVALID, "hvx_ctu_analyze: workspace too small");
  char *ws = (char *)d_workspace;
  hvx_me_job *jobs = (hvx_me_job *)(ws + W.jobs);
  hvx_me_result *res = (hvx_me_result *)(ws + W.res);
  hvx_tu_desc *desc = (hvx_tu_desc *)(ws + W.desc);
  int64_t *off = (int64_t *)(ws + W.off);
  int32_t *est_idx = (int32_t *)(ws + W.est_idx);
  int16_t *resid = (int16_t *)(ws + W.resid);
  int32_t *lev = (int32_t *)(ws + W.lev);
  int16_t *res_out = (int16_t *)(ws + W.res_out);
  int32_t *abs_sum = (int32_t *)(ws + W.abs);
  uint32_t *sse = (uint32_t *)(ws + W.sse);
  uint8_t *pred = (uint8_t *)(ws + W.pred);
  uint32_t *zd = (uint32_t *)(ws + W.zd), *csse = (uint32_t *)(ws + W.csse);
  const uint8_t **cur_slot = (const uint8_t **)(ws + W.ptr);
  // Three streams, joined back into ctx->stream before the per-CU totals:
  //   A (ctx->stream): ME depth 0 -> 1 -> 2 -> 3 (depth d+1 starts from depth d's integer MVs),
  //                    then residuals + the 8x8 TU pipeline of depth 3
  //   B (aux[0], high priority): residuals of depths 0-1 and the 32x32 TU pipeline -- its
  //                    latency-bound RDOQ waves run beside the depth 2/3 searches, not after them
  //   C (aux[1], high priority): residuals of depth 2 and the 16x16 TU pipeline
  // The 64x64 fractional refinement stays on A after depth 0 (it fills the chip by itself).
  hipStream_t st = ctx->stream, sb = ctx->aux[0], sc = ctx->aux[1], se = ctx->aux[2];
  if (ctx->serial) sb = sc = se = st;
  fold_timing(ctx);  // a previous call's events must be read before they are re-recorded
  hipLaunchKernelGGL(k_set_ptr, dim3(1), dim3(1), 0, st, cur_slot, d_cur);
  const uint8_t *const *cs = (const uint8_t *const *)cur_slot;
  const bool fen = (P.me_flags & HVX_ME_FEN) != 0;
  const int n = L.nctu;
  CtuMc M;
  M.L = L; M.P = P; M.cur = d_cur; M.refs = d_refs; M.stride = stride; M.res = res; M.resid = resid; M.pred_out = pred;
  M.descs = desc; M.offs = off; M.est_idx = est_idx; M.out = d_out; M.C = C;
  auto resid_depth = [&](hipStream_t s, int d) {
    const dim3 grid(n << (2 * d)), blk(64);
    if (d == 0) hipLaunchKernelGGL(k_ctu_pred_resid<64>, grid, blk, 0, s, M, 0);
    if (d == 1) hipLaunchKernelGGL(k_ctu_pred_resid<32>, grid, blk, 0, s, M, 0);
    if (d == 2) hipLaunchKernelGGL(k_ctu_pred_resid<16>, grid, blk, 0, s, M, 0);
    if (d == 3) hipLaunchKernelGGL(k_ctu_pred_resid8q<HVX_D3_NC>, dim3(n * (64 / HVX_D3_NC)), blk, 0, s, M);  // NC 8x8 CUs per wave
  };
  for (int d = 0; d < 4; d++) {
    const int ncu = 1 << (2 * d), nt = L.nctu * ncu * L.nref;
    const int tk = t_begin(ctx, st, d);
    hipLaunchKernelGGL(k_ctu_me_jobs, dim3((nt + 255) / 256), dim3(256), 0, st, L, P, d, res, jobs);
    // the depth's jobs are contiguous per CTU but interleaved across CTUs: launch over all CUs of
    // this depth via a per-depth view (blocks of other depths return at once)
    const int first = d == 0 ? 0 : d == 1 ? 1 : d == 2 ? 5 : 21;
    const dim3 grid(L.nctu * ncu * L.nref);
    switch (d) {  // block size, FEN row subsampling and waves per job are compile-time per depth
      case 0:  // 64x64: integer search here, fractional refinement by k_me_frac_ctu on stream B
        if (fen) hipLaunchKernelGGL((k_me_int_ctu<64, 1, 4>), grid, dim3(256), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        else hipLaunchKernelGGL((k_me_int_ctu<64, 0, 4>), grid, dim3(256), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        break;
      case 1:  // fused integer + fractional search
        if (fen) hipLaunchKernelGGL((k_me_ctu<32, 1, 2>), grid, dim3(128), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        else hipLaunchKernelGGL((k_me_ctu<32, 0, 2>), grid, dim3(128), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        break;
      case 2:
        if (fen) hipLaunchKernelGGL((k_me_ctu<16, 1, 1>), grid, dim3(64), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        else hipLaunchKernelGGL((k_me_ctu<16, 0, 1>), grid, dim3(64), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        break;
      default:  // 8x8: FEN never applies (rows <= 8)
        hipLaunchKernelGGL((k_me_ctu<8, 0, 1>), grid, dim3(64), 0, st, cs, d_refs, stride, jobs, res, L.nref, ncu, first);
        break;
    }
    t_end(ctx, st, tk);
    if (d == 0) {  // fractional refinement of the 64x64 depth (the others are fused above)
      const int tf = t_begin(ctx, st, 4);
      hipLaunchKernelGGL((k_me_frac_ctu<64, 4>), dim3(L.nctu * L.nref), dim3(256), 0, st, cs, d_refs, stride, jobs, res,
                         L.nref, 1, 0);
      t_end(ctx, st, tf);
    }
    if (d == 1) HVX_HIP(hipEventRecord(ctx->fj[1], st));
    if (d == 2) HVX_HIP(hipEventRecord(ctx->fj[2], st));
  }
  // kCtuG = 64 TUs per RDOQ wave for every class: measured best at 2160p (G = 8/16/32/64 for
  // 32x32: 3.1/2.9/2.6/2.5 ms) -- the per-lane chain is latency-bound, so wider waves win
  const int g32 = kCtuG, g16 = kCtuG, g8 = kCtuG;
  uint32_t *coefI = (uint32_t *)(ws + W.coefI), *cxI = (uint32_t *)(ws + W.cxI);
  int32_t *levI = (int32_t *)(ws + W.levI), *stI = (int32_t *)(ws + W.stI);
  int8_t *flags = (int8_t *)(ws + W.flags);
  hvx_coeff_bits *cb = (hvx_coeff_bits *)(ws + W.cbits);
  auto count_class = [&](hipStream_t s, int first, int cnt, size_t il_off, int L2) {
    if (!cnt_states) return;
    const int tc = t_begin(ctx, s, 16);
    const dim3 grid((cnt + 63) / 64);
    if (L2 == 3) hipLaunchKernelGGL((k_coeff_bits_il<3>), grid, dim3(64), 0, s, desc + first, cnt, levI + il_off, cnt_eb, cnt_states, cb + first);
    else if (L2 == 2) hipLaunchKernelGGL((k_coeff_bits_il<2>), grid, dim3(64), 0, s, desc + first, cnt, levI + il_off, cnt_eb, cnt_states, cb + first);
    else if (L2 == 1) hipLaunchKernelGGL((k_coeff_bits_il<1>), grid, dim3(64), 0, s, desc + first, cnt, levI + il_off, cnt_eb, cnt_states, cb + first);
    else hipLaunchKernelGGL((k_coeff_bits_il<0>), grid, dim3(64), 0, s, desc + first, cnt, levI + il_off, cnt_eb, cnt_states, cb + first);
    t_end(ctx, s, tc);
  };
  // size classes are contiguous: [0,8n) 32x32 | [8n,24n) 16x16 | [24n,88n) 8x8; their
  // interleaved scratch regions start at 0, ctu_il_off16(n), ctu_il_off8(n)
  {  // stream B; with counting (hvx_ctu_encode) the 32x32 class's rate runs on stream E beside k_tu_fin
    HVX_HIP(hipStreamWaitEvent(sb, ctx->fj[1], 0));
    const int tk = t_begin(ctx, sb, 5);
    resid_depth(sb, 0);
    resid_depth(sb, 1);
    t_end(ctx, sb, tk);
    if (C.on) {  // the chroma 16x16 TUs of these CUs on stream E, beside the luma 32x32 pipeline
      HVX_HIP(hipEventRecord(ctx->fj[7], sb));
      HVX_HIP(hipStreamWaitEvent(se, ctx->fj[7], 0));
      const size_t o = ctu_il_offc16(n);
      tu_class_launch<2, 2>(se, desc + 88 * n, d_est4, est_idx + 88 * n, off + 88 * n, 16 * n, resid, nullptr, lev,
                            nullptr, abs_sum + 88 * n, res_out, sse + 88 * n, coefI + o, cxI + o, levI + o, stI + o,
                            flags + 88 * n, kCtuG, n_est, ctx, 9, nullptr, pred, zd + 88 * n, csse + 88 * n);
      count_class(se, 88 * n, 16 * n, o, 2);
    }
    tu_class_launch<3, 2>(sb, desc, d_est4, est_idx, off, 8 * n, resid, nullptr, lev, nullptr, abs_sum, res_out, sse,
                          coefI, cxI, levI, stI, flags, g32, n_est, ctx, 6, cnt_states ? ctx->fj[5] : nullptr, pred, zd,
                          csse);
    if (cnt_states) {
      HVX_HIP(hipStreamWaitEvent(se, ctx->fj[5], 0));
      count_class(se, 0, 8 * n, 0, 3);
    }
    HVX_HIP(hipEventRecord(ctx->fj[6], se));
  }
  {  // stream C
    HVX_HIP(hipStreamWaitEvent(sc, ctx->fj[2], 0));
    const int tk = t_begin(ctx, sc, 5);
    resid_depth(sc, 2);
    t_end(ctx, sc, tk);
    const size_t o = ctu_il_off16(n);
    tu_class_launch<2, 2>(sc, desc + 8 * n, d_est4, est_idx + 8 * n, off + 8 * n, 16 * n, resid, nullptr, lev, nullptr,
                          abs_sum + 8 * n, res_out, sse + 8 * n, coefI + o, cxI + o, levI + o, stI + o, flags + 8 * n, g16,
                          n_est, ctx, 9, nullptr, pred, zd + 8 * n, csse + 8 * n);
    count_class(sc, 8 * n, 16 * n, o, 2);
    if (C.on) {
      const size_t oc = ctu_il_offc8(n);
      tu_class_launch<1, 2>(sc, desc + 104 * n, d_est4, est_idx + 104 * n, off + 104 * n, 32 * n, resid, nullptr, lev,
                            nullptr, abs_sum + 104 * n, res_out, sse + 104 * n, coefI + oc, cxI + oc, levI + oc, stI + oc,
                            flags + 104 * n, kCtuG, n_est, ctx, 12, nullptr, pred, zd + 104 * n, csse + 104 * n);
      count_class(sc, 104 * n, 32 * n, oc, 1);
    }
    HVX_HIP(hipEventRecord(ctx->fj[4], sc));
  }
  {  // stream A: depth 3 (its 4x4 chroma TUs go to stream B, idle by then, beside the luma 8x8 pipeline)
    const int tk = t_begin(ctx, st, 5);
    resid_depth(st, 3);
    t_end(ctx, st, tk);
    if (C.on) HVX_HIP(hipEventRecord(ctx->fj[0], st));
    const size_t o = ctu_il_off8(n);
    tu_class_launch<1, 2>(st, desc + 24 * n, d_est4, est_idx + 24 * n, off + 24 * n, 64 * n, resid, nullptr, lev, nullptr,
                          abs_sum + 24 * n, res_out, sse + 24 * n, coefI + o, cxI + o, levI + o, stI + o, flags + 24 * n, g8,
                          n_est, ctx, 12, nullptr, pred, zd + 24 * n, csse + 24 * n);
    count_class(st, 24 * n, 64 * n, o, 1);
  }
  if (C.on) {  // stream B, after its 32x32 pipeline: the 4x4 chroma TUs of depth 3 (+ transform-skip twins)
    HVX_HIP(hipStreamWaitEvent(sb, ctx->fj[0], 0));
    const size_t oc = ctu_il_offc4(n);
    tu_class_launch<0, 2>(sb, desc + 136 * n, d_est4, est_idx + 136 * n, off + 136 * n, 256 * n, resid, nullptr, lev,
                          nullptr, abs_sum + 136 * n, res_out, sse + 136 * n, coefI + oc, cxI + oc, levI + oc, stI + oc,
                          flags + 136 * n, kCtuG, n_est, ctx, 12, nullptr, pred, zd + 136 * n, csse + 136 * n);
    count_class(sb, 136 * n, 256 * n, oc, 0);
  }
  HVX_HIP(hipEventRecord(ctx->fj[3], sb));
  HVX_HIP(hipStreamWaitEvent(st, ctx->fj[3], 0));
  HVX_HIP(hipStreamWaitEvent(st, ctx->fj[4], 0));
  HVX_HIP(hipStreamWaitEvent(st, ctx->fj[6], 0));
  const int tk = t_begin(ctx, st, 15);
  hipLaunchKernelGGL(k_ctu_finalize, dim3((n * HVX_CUS_PER_CTU + 255) / 256), dim3(256), 0, st, L, abs_sum, sse, d_out);
  t_end(ctx, st, tk);
  return launched("hvx_ctu_analyze");
}

int hvx_ctu_analyze(hvx_ctx *ctx, const uint8_t *d_cur, const uint8_t *const *d_refs, int stride,
                    const hvx_ctu_params *h_params, const hvx_estbits *d_est4, void *d_workspace, size_t ws_bytes,
                    hvx_cu_result *d_out) {
  return ctu_analyze_impl(ctx, d_cur, d_refs, stride, h_params, d_est4, d_workspace, ws_bytes, d_out, nullptr, nullptr);
}

static int ctu_decide_impl(hvx_ctx *ctx, const uint8_t *d_cur, int stride, const hvx_ctu_params *h_params,
                           const uint8_t *d_ctx_states, const int32_t *d_entropy_bits, void *d_workspace, size_t ws_bytes,
                           const hvx_cu_result *d_cu, hvx_cu_decision *d_dec, uint8_t *d_recon, uint8_t *d_ref_pic,
                           bool count, const hvx_chroma_planes *chroma = nullptr) {
  if (!ctx || !d_cur || !h_params || !d_ctx_states || !d_entropy_bits || !d_workspace || !d_cu || !d_dec || !d_recon)
    return fail(HVX_E_INVALID, "hvx_ctu_decide: NULL argument");
  const hvx_ctu_params P = *h_params;
  if (P.pic_w <= 0 || P.pic_h <= 0 || P.pic_w % 8 || P.pic_h % 8 || P.n_ref <= 0 || P.n_ref > 8 ||
      stride < P.pic_w + 2 * HVX_PLANE_MARGIN || stride % 4 != 0 || (P.rd_metric != HVX_RD_SSE && P.rd_metric != HVX_RD_SSIM))
    return fail(HVX_E_INVALID, "hvx_ctu_decide: bad parameters");
  const CtuLayout L = ctu_layout(P.pic_w, P.pic_h, P.n_ref);
  const CtuWs W = ctu_ws_layout(L);
  if (ws_bytes < W.total) return fail(HVX_E_INVALID, "hvx_ctu_decide: workspace too small");
  char *ws = (char *)d_workspace;
  hipStream_t st = ctx->stream;
  const int n = L.nctu;
  const hvx_tu_desc *desc = (const hvx_tu_desc *)(ws + W.desc);
  hvx_coeff_bits *cb = (hvx_coeff_bits *)(ws + W.cbits);
  // 1. coefficient rate of every TU, one lane per TU, per size class (no mixed-size waves), from
  //    the RDOQ's interleaved scan-order levels; every TU counts from the same context snapshot
  int tk = -1;
  const int32_t *levI = (const int32_t *)(ws + W.levI);
  if (count) {
  tk = t_begin(ctx, st, 16);
  hipLaunchKernelGGL((k_coeff_bits_il<3>), dim3((8 * n + 63) / 64), dim3(64), 0, st, desc, 8 * n, levI, d_entropy_bits,
                     d_ctx_states, cb);
  hipLaunchKernelGGL((k_coeff_bits_il<2>), dim3((16 * n + 63) / 64), dim3(64), 0, st, desc + 8 * n, 16 * n,
                     levI + ctu_il_off16(n), d_entropy_bits, d_ctx_states, cb + 8 * n);
  hipLaunchKernelGGL((k_coeff_bits_il<1>), dim3((64 * n + 63) / 64), dim3(64), 0, st, desc + 24 * n, 64 * n,
                     levI + ctu_il_off8(n), d_entropy_bits, d_ctx_states, cb + 24 * n);
  t_end(ctx, st, tk);
  }
  // 2. the CU tree of every CTU, 3. the reconstruction of its leaves + border extension
  tk = t_begin(ctx, st, 17);
  DecideArgs A;
  A.L = L; A.pic_w = P.pic_w; A.pic_h = P.pic_h; A.lambda = P.lambda;
  A.cu = d_cu; A.res = (const hvx_me_result *)(ws + W.res); A.cb = cb;
  A.st = d_ctx_states; A.eb = d_entropy_bits; A.dec = d_dec;
  A.metric = P.rd_metric; A.lambda_ssim = P.lambda_ssim;
  A.C = ctu_chroma(chroma); A.cw = P.chroma_weight;
  if (chroma && (!chroma->recon_cb || !chroma->recon_cr || (d_ref_pic && (!chroma->ref_pic_cb || !chroma->ref_pic_cr))))
    return fail(HVX_E_INVALID, "hvx_ctu_encode_yuv: NULL chroma reconstruction / reference plane");
  hipLaunchKernelGGL(k_ctu_leaf, dim3((n * HVX_CUS_PER_CTU + 63) / 64), dim3(64), 0, st, A, (const int32_t *)(ws + W.abs),
                     (const uint32_t *)(ws + W.sse), (const uint32_t *)(ws + W.zd), (const uint32_t *)(ws + W.csse));
  if (P.rd_metric == HVX_RD_SSIM)
    hipLaunchKernelGGL(k_ctu_leaf_ssim, dim3(n * HVX_CUS_PER_CTU), dim3(64), 0, st, A, d_cur, stride,
                       (const int16_t *)(ws + W.resid), (const int16_t *)(ws + W.res_out));
  hipLaunchKernelGGL(k_ctu_decide, dim3(n), dim3(64), 0, st, A);  // one wave per CTU
  // the reference picture (if asked for) gets the reconstructed samples in the same pass; its
  // margins are extended after deblocking
  uint8_t *rp_y = d_ref_pic != d_recon ? d_ref_pic : nullptr;
  uint8_t *rp_cb = chroma && d_ref_pic && chroma->ref_pic_cb != chroma->recon_cb ? chroma->ref_pic_cb : nullptr;
  uint8_t *rp_cr = chroma && d_ref_pic && chroma->ref_pic_cr != chroma->recon_cr ? chroma->ref_pic_cr : nullptr;
  // the boundary strengths (for the reference picture's deblocking) run in the reconstruction launch
  const int M = HVX_PLANE_MARGIN, Mc = M / 2, cw = P.pic_w / 2, ch = P.pic_h / 2;
  uint8_t *bsv = (uint8_t *)(ws + W.bsv), *bsh = (uint8_t *)(ws + W.bsh);
  int8_t *qpm = (int8_t *)(ws + W.qpm);
  CtuBsArgs B = {d_cu, d_ref_pic ? bsv : nullptr, bsh, qpm, P.qp};
  hipLaunchKernelGGL(k_ctu_recon, dim3(n), dim3(256), 0, st, L, P.pic_w, P.pic_h, d_cur, stride, (const hvx_cu_decision *)d_dec,
                     (const int16_t *)(ws + W.resid), (const int16_t *)(ws + W.res_out), d_recon, A.C, rp_y, rp_cb, rp_cr, B);
  // extendPicBorder of Y (and Cb, Cr): one launch
  auto extend = [&](uint8_t *y, uint8_t *cb, uint8_t *cr) {
    PlaneSet E = {{y, cb, cr}, {stride, chroma ? chroma->c_stride : 0, chroma ? chroma->c_stride : 0},
                  {P.pic_w, cw, cw}, {P.pic_h, ch, ch}, {M, Mc, Mc}};
    const int np = chroma ? 3 : 1, nm = 2 * M * P.pic_h + 2 * M * (P.pic_w + 2 * M);
    hipLaunchKernelGGL(k_planes_extend, dim3((nm + 255) / 256, np), dim3(256), 0, st, E);
  };
  extend(d_recon, chroma ? chroma->recon_cb : nullptr, chroma ? chroma->recon_cr : nullptr);
  t_end(ctx, st, tk);
  if (d_ref_pic) {
    // 4. the reference picture: the reconstruction deblocked (boundary strengths of the decided
    //    trees, computed above; TComLoopFilter::loopFilterPic, luma) with borders extended again
    tk = t_begin(ctx, st, 18);
    hvx_deblock_params dp = {};
    dp.pic_w = P.pic_w; dp.pic_h = P.pic_h;
    // loopFilterPic: luma, and at 4:2:0 the chroma edges (filtered only where bs == 2, i.e. never
    // between the inter CUs of this pass)
    uint8_t *dcb = chroma ? chroma->ref_pic_cb : nullptr, *dcr = chroma ? chroma->ref_pic_cr : nullptr;
    const int dcs = chroma ? chroma->c_stride : 0;
    const int nv = (P.pic_w / 8 - 1) * (P.pic_h / 4), nh = (P.pic_h / 8 - 1) * (P.pic_w / 4);
    if (nv > 0)
      hipLaunchKernelGGL(k_deblock<0>, dim3((nv + 255) / 256), dim3(256), 0, st, d_ref_pic, stride, dcb, dcr, dcs, bsv, qpm,
                         dp);
    if (nh > 0)
      hipLaunchKernelGGL(k_deblock<1>, dim3((nh + 255) / 256), dim3(256), 0, st, d_ref_pic, stride, dcb, dcr, dcs, bsh, qpm,
                         dp);
    extend(d_ref_pic, chroma ? chroma->ref_pic_cb : nullptr, chroma ? chroma->ref_pic_cr : nullptr);
    t_end(ctx, st, tk);
  }
  return launched("hvx_ctu_decide");
}

int hvx_ctu_decide(hvx_ctx *ctx, const uint8_t *d_cur, int stride, const hvx_ctu_params *h_params,
                   const uint8_t *d_ctx_states, const int32_t *d_entropy_bits, void *d_workspace, size_t ws_bytes,
                   const hvx_cu_result *d_cu, hvx_cu_decision *d_dec, uint8_t *d_recon, uint8_t *d_ref_pic) {
  return ctu_decide_impl(ctx, d_cur, stride, h_params, d_ctx_states, d_entropy_bits, d_workspace, ws_bytes, d_cu, d_dec,
                         d_recon, d_ref_pic, true);
}

int hvx_ctu_encode(hvx_ctx *ctx, const uint8_t *d_cur, const uint8_t *const *d_refs, int stride,
                   const hvx_ctu_params *h_params, const hvx_estbits *d_est4, const uint8_t *d_ctx_states,
                   const int32_t *d_entropy_bits, void *d_workspace, size_t ws_bytes, hvx_cu_result *d_cu,
                   hvx_cu_decision *d_dec, uint8_t *d_recon, uint8_t *d_ref_pic) {
  if (!d_ctx_states || !d_entropy_bits || !d_dec || !d_recon) return fail(HVX_E_INVALID, "hvx_ctu_encode: NULL argument");
  const int rc = ctu_analyze_impl(ctx, d_cur, d_refs, stride, h_params, d_est4, d_workspace, ws_bytes, d_cu, d_ctx_states,
                                  d_entropy_bits);
  if (rc) return rc;
  return ctu_decide_impl(ctx, d_cur, stride, h_params, d_ctx_states, d_entropy_bits, d_workspace, ws_bytes, d_cu, d_dec,
                         d_recon, d_ref_pic, false);
}

int hvx_ctu_encode_yuv(hvx_ctx *ctx, const uint8_t *d_cur, const uint8_t *const *d_refs, int stride,
                       const hvx_chroma_planes *h_chroma, const hvx_ctu_params *h_params, const hvx_estbits *d_est7,
                       const uint8_t *d_ctx_states, const int32_t *d_entropy_bits, void *d_workspace, size_t ws_bytes,
                       hvx_cu_result *d_cu, hvx_cu_decision *d_dec, uint8_t *d_recon, uint8_t *d_ref_pic) {
  if (!h_chroma || !d_ctx_states || !d_entropy_bits || !d_dec || !d_recon)
    return fail(HVX_E_INVALID, "hvx_ctu_encode_yuv: NULL argument");
  const int rc = ctu_analyze_impl(ctx, d_cur, d_refs, stride, h_params, d_est7, d_workspace, ws_bytes, d_cu, d_ctx_states,
                                  d_entropy_bits, h_chroma);
  if (rc) return rc;
  return ctu_decide_impl(ctx, d_cur, stride, h_params, d_ctx_states, d_entropy_bits, d_workspace, ws_bytes, d_cu, d_dec,
                         d_recon, d_ref_pic, false, h_chroma);
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

