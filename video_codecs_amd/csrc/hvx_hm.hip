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
#include "hvx_host.hpp"
#include "hvx_tables.hpp"

using namespace hvxi;

int hvx_hm_module_init() { return upload_tables(); }

extern "C" {

int hvx_hm_state_size(size_t *bytes) {
  if (!bytes) return fail(HVX_E_INVALID, "hvx_hm_state_size: NULL");
#ifdef HM_STATE_ODD_LINES
  // an odd number of 128-byte lines between consecutive chains' states, so the same field of
  // different chains falls into different cache sets / memory channels
  *bytes = ((sizeof(hm::State) + 127) / 128 | 1) * 128;
#else
  *bytes = (sizeof(hm::State) + 255) / 256 * 256;
#endif
  return HVX_OK;
}

int hvx_hm_compress(hvx_ctx *ctx, const hvx_hm_picture *d_pics, int n_pics, const hvx_hm_job *d_jobs, int n_jobs,
                    int n_out, void *d_state, hvx_hm_ctu *d_out_ctu, uint8_t *d_out_rec, hvx_hm_coder *d_out_coder) {
  if (!ctx || !d_pics || n_pics < 1 || !d_jobs || n_jobs < 0 || n_out < 0 || !d_state || !d_out_ctu || !d_out_rec)
    return fail(HVX_E_INVALID, "hvx_hm_compress: bad args");
  if (n_jobs == 0) return HVX_OK;
  size_t sb = 0;
  hvx_hm_state_size(&sb);
#ifdef HM_XCD_GROUP
  const int grid = 8 * ((n_jobs + 7) / 8);
#else
  const int grid = n_jobs;
#endif
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

}  // extern "C"
