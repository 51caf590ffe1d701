// hvx_hm.hip -- the HM-exact CTU decision of libhvx.so (its own translation unit: the engine is
// one large kernel, compiled apart from the leaf-kernel library in hvx_lib.hip).
// the engine's tool set has no extended precision processing: RDOQ's rate is the branch-free form
#define HVX_TU_NO_EXT 1
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "hvx_dev.hpp"
#include "hvx_hm.hpp"
#include "hvx_hmwrite.hpp"
#include "hvx_host.hpp"
#include "hvx_tables.hpp"

using namespace hvxi;


// hvx_hm_write_slices: one workgroup (one wave) per slice
static __global__ __launch_bounds__(64) void k_hm_write_slices(const hvx_hm_picture *__restrict__ pics, int n_pics,
                                                               const hvx_hm_slice *__restrict__ slices, int n_slices,
                                                               char *state_base, size_t state_bytes,
                                                               hvx_hm_slice_result *__restrict__ res) {
  using namespace hm;
  const int jid = blockIdx.x;
  if (jid >= n_slices) return;
  const int l = threadIdx.x;
  const hvx_hm_slice &j = slices[jid];
  hvx_hm_slice_result *o = &res[jid];
  int bad = 0;
  if (j.pic < 0 || j.pic >= n_pics) bad = HVX_HM_BAD_PIC;
  else {
    const hvx_hm_picture &P = pics[j.pic];
    const int n = P.w_ctus * P.h_ctus;
    if (P.w <= 0 || P.h <= 0 || (P.w & 7) || (P.h & 7) || P.w_ctus != (P.w + 63) / 64 || P.h_ctus != (P.h + 63) / 64 ||
        !P.ctus)
      bad = HVX_HM_BAD_GEOMETRY;
    else if (j.first_ctu < 0 || j.n_ctus < 1 || j.first_ctu + j.n_ctus > n) bad = HVX_HM_BAD_CTUS;
    else if (!j.out || j.out_cap < 0 || ((j.sao_enabled[0] | j.sao_enabled[1] | j.sao_enabled[2]) && !j.sao_coded))
      bad = HVX_HM_BAD_OUT;
  }
  if (bad) {
    if (l == 0) o->status = -bad;
    return;
  }
  State *S = (State *)(state_base + (size_t)jid * state_bytes);
  copy_words(&hm_e.P, &pics[j.pic], (int)sizeof(hvx_hm_picture));
  wsync();
  hm_fill_pk(hm_e.P.entropy_bits, l);
  hm_e.S = S;
  if (l < 4) hm_e.dbg[l] = 0;
  hm_e.stage = 0;
  hm_e.stop = 0;
  hm_e.tsp = 0;
  hm_e.slice_start = j.first_ctu;
  hm_e.slice_end = j.first_ctu + j.n_ctus - 1;
  hm_e.slice_qp = hm_e.P.qp;
  for (int d = 0; d < 4; d++) {
    hm_e.best[d] = d;
    hm_e.temp[d] = 4 + d;
    for (int k = 0; k < 7; k++) hm_e.yi[k][d] = k * 4 + d;
  }
  // TEncBinCABAC::start() and the slice-start contexts
  hm_w.low = 0; hm_w.range = 510; hm_w.bits_left = 23; hm_w.nbuf = 0; hm_w.buffered = 0xff; hm_w.bins = 0;
  hm_w.nout = 0; hm_w.cap = j.out_cap; hm_w.out = j.out;
  if (l < 7) hm_w.coded[l] = 0;
  for (int i = l; i < HVX_NUM_CTX; i += 64) hm_w.st[i] = j.entry.st[i];
  wsync();
  const int sao = j.sao_enabled[0] | j.sao_enabled[1] | j.sao_enabled[2];
  const int en[3] = {j.sao_enabled[0], j.sao_enabled[1], j.sao_enabled[2]};
  for (int k = 0; k < j.n_ctus; k++) {
    const int addr = j.first_ctu + k;
    hm_e.ctu_addr = addr;
    hm_e.ctu_x = addr % hm_e.P.w_ctus;
    hm_e.ctu_y = addr / hm_e.P.w_ctus;
    // the CTU's data (TComPic::getCtu): the current CTU's partitions and its depth-0 view
    const hvx_hm_ctu *src = &hm_e.P.ctus[addr];
    Cu *v = &S->view;
    wsync();
    v->depth = 0; v->zidx = 0; v->width = 64; v->nparts = 256;
    v->x = hm_e.ctu_x * 64; v->y = hm_e.ctu_y * 64;
    copy_words(S->ctu_p, src->p, (int)sizeof(Part) * 256);
    copy_words(v->p, src->p, (int)sizeof(Part) * 256);
    copy_words(v->coef, src->coef, 2 * 6144);
    wsync();
    if (sao) write_sao(j.sao_coded, en, addr, j.first_ctu);
    write_cu<0>(0, addr == hm_e.slice_end);
  }
  wsync();
  if (l == 0) {
    o->low = hm_w.low; o->range = hm_w.range; o->bits_left = hm_w.bits_left; o->num_buffered = hm_w.nbuf;
    o->buffered_byte = hm_w.buffered; o->bins = hm_w.bins; o->n_bytes = hm_w.nout; o->status = 0; o->pad_ = 0;
  }
  if (l < 7) o->coded[l] = hm_w.coded[l];
  for (int i = l; i < 208; i += 64) o->states[i] = i < HVX_NUM_CTX ? hm_w.st[i] : 0;
}

// hvx_hm_stv_prepare: one thread per window of the three stv_sums tables (hm::stv_hist_acc)
static __global__ __launch_bounds__(256) void k_stv_hist(const uint8_t *const *__restrict__ hist, int n_hist, int w, int h,
                                                         int hs_y, int hs_c, float *__restrict__ sums) {
  using namespace hm;
  const int nx0 = (w - 8) / 4 + 1, ny0 = (h - 8) / 4 + 1, nx1 = ((w >> 1) - 8) / 4 + 1, ny1 = ((h >> 1) - 8) / 4 + 1;
  const int nx2 = ((w >> 1) - 4) / 4 + 1, ny2 = ((h >> 1) - 4) / 4 + 1;
  const long n0 = (long)nx0 * ny0, n1 = (long)nx1 * ny1, n2 = (long)nx2 * ny2;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n0 + n1 + n2) return;
  int c, wint, px, py;
  if (i < n0) { c = 0; wint = 8; py = (int)(i / nx0) * 4; px = (int)(i % nx0) * 4; }
  else if (i < n0 + n1) { c = 1; wint = 8; py = (int)((i - n0) / nx1) * 4; px = (int)((i - n0) % nx1) * 4; }
  else { c = 1; wint = 4; py = (int)((i - n0 - n1) / nx2) * 4; px = (int)((i - n0 - n1) % nx2) * 4; }
  float wgta[4], wgtb[4], acc[20];
  stv_weights(wint, n_hist + 1, wgta, wgtb);
  for (int k = 0; k < 20; k++) acc[k] = 0.0f;
  stv_hist_acc(hist, n_hist, c, c ? hs_c : hs_y, wint, px, py, wgta, wgtb, acc);
  float *o = sums + 20 * i;
  for (int k = 0; k < 20; k++) o[k] = acc[k];
}

int hvx_hm_module_init() { return upload_tables(); }

extern "C" {

int hvx_hm_state_size(size_t *bytes) {
  if (!bytes) return fail(HVX_E_INVALID, "hvx_hm_state_size: NULL");
  *bytes = (sizeof(hm::State) + 255) / 256 * 256;
  return HVX_OK;
}

int hvx_hm_compress(hvx_ctx *ctx, const hvx_hm_picture *d_pics, int n_pics, const hvx_hm_job *d_jobs, int n_jobs,
                    int n_out, void *d_state, hvx_hm_ctu *d_out_ctu, uint8_t *d_out_rec, hvx_hm_coder *d_out_coder) {
  if (!ctx || !d_pics || n_pics < 1 || !d_jobs || n_jobs < 0 || n_out < 0 || !d_state || !d_out_ctu || !d_out_rec)
    return fail(HVX_E_INVALID, "hvx_hm_compress: bad args");
  if (n_jobs == 0) return HVX_OK;
  size_t sb = 0;
  hvx_hm_state_size(&sb);
  const int grid = n_jobs;
  hipLaunchKernelGGL(k_hm_compress, dim3(grid), dim3(64), 0, ctx->stream, d_pics, n_pics, d_jobs, n_jobs, n_out,
                     (char *)d_state, sb, d_out_ctu, d_out_rec, d_out_coder);
  return launched("k_hm_compress");
}

int hvx_hm_job_status(hvx_ctx *ctx, const void *d_state, int n_jobs, int32_t *h_status) {
  if (!ctx || !d_state || n_jobs < 0 || (n_jobs && !h_status)) return fail(HVX_E_INVALID, "hvx_hm_job_status: bad args");
  if (n_jobs == 0) return HVX_OK;
  size_t sb = 0;
  hvx_hm_state_size(&sb);
  // State.status[0] of every job's state (strided): 0 = ran, -HVX_HM_BAD_* = refused
  if (hipMemcpy2DAsync(h_status, sizeof(int32_t), d_state, sb, sizeof(int32_t), (size_t)n_jobs, hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return fail(HVX_E_HIP, "hvx_hm_job_status: copy failed");
  return HVX_OK;
}

int hvx_hm_stv_sums_size(int w, int h, size_t *bytes) {
  if (!bytes || w < 16 || h < 16 || (w & 7) || (h & 7)) return fail(HVX_E_INVALID, "hvx_hm_stv_sums_size: bad args");
  const size_t n = (size_t)((w - 8) / 4 + 1) * ((h - 8) / 4 + 1) + (size_t)((w / 2 - 8) / 4 + 1) * ((h / 2 - 8) / 4 + 1) +
                   (size_t)((w / 2 - 4) / 4 + 1) * ((h / 2 - 4) / 4 + 1);
  *bytes = n * 20 * sizeof(float);
  return HVX_OK;
}

int hvx_hm_stv_prepare(hvx_ctx *ctx, const hvx_hm_picture *h_pic, float *d_sums) {
  size_t bytes = 0;
  if (!ctx || !h_pic || !d_sums || hvx_hm_stv_sums_size(h_pic->w, h_pic->h, &bytes) != HVX_OK ||
      h_pic->hist_n < 0 || h_pic->hist_n > HVX_STV_HIST || (h_pic->hist_n > 0 && !h_pic->hist) ||
      (h_pic->hist_n > 0 && (h_pic->hist_stride[0] < h_pic->w || h_pic->hist_stride[1] < h_pic->w / 2)))
    return fail(HVX_E_INVALID, "hvx_hm_stv_prepare: bad args");
  const long n = (long)(bytes / (20 * sizeof(float)));
  hipLaunchKernelGGL(k_stv_hist, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, h_pic->hist, h_pic->hist_n,
                     h_pic->w, h_pic->h, h_pic->hist_stride[0], h_pic->hist_stride[1], d_sums);
  return launched("k_stv_hist");
}

int hvx_hm_write_slices(hvx_ctx *ctx, const hvx_hm_picture *d_pics, int n_pics, const hvx_hm_slice *d_slices,
                        int n_slices, void *d_state, hvx_hm_slice_result *d_out) {
  if (!ctx || !d_pics || n_pics < 1 || !d_slices || n_slices < 0 || !d_state || !d_out)
    return fail(HVX_E_INVALID, "hvx_hm_write_slices: bad args");
  if (n_slices == 0) return HVX_OK;
  size_t sb = 0;
  hvx_hm_state_size(&sb);
  hipLaunchKernelGGL(k_hm_write_slices, dim3(n_slices), dim3(64), 0, ctx->stream, d_pics, n_pics, d_slices, n_slices,
                     (char *)d_state, sb, d_out);
  return launched("k_hm_write_slices");
}

}  // extern "C"
