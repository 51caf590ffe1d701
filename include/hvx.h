/* hvx.h -- C-ABI of the MI355X-native HM-16.5rc1 CU mode-decision hot path (libhvx.so).
 *
 * Plain pointers and sizes only (no torch / HIP types in signatures).  All
 * batch entry points are asynchronous on the context's HIP stream; every
 * pointer argument named d_* is DEVICE memory (hipMalloc'd or a torch tensor),
 * h_* is host memory.  The caller owns all buffers; the context owns only its
 * stream and constant tables.  Every function returns 0 on success or a
 * negative HVX_E_* code (HIP errors are mapped to HVX_E_HIP - hipError_t);
 * hvx_last_error() gives the message.  HM itself has no return codes and
 * fails fast (assert/exit, TComTrQuant.cpp:891,913), so the C++ shims over this
 * ABI abort() on a negative status.
 *
 * Each entry point replaces a reference interface (paths relative to
 * /root/reference/hm-16.5rc1/source/Lib, or stvssim_src/...):
 *
 *   hvx_dist_batch        TComRdCost::setDistParam + DistParam::DistFunc, getDistPart
 *                         (TComRdCost.h:60,153-158,221; TComRdCost.cpp:294-451) -- the
 *                         FpDistFunc function pointer is HM's native plug-in seam.
 *   hvx_interp_batch      TComInterpolationFilter::filterHor / filterVer
 *                         (TComInterpolationFilter.h:56-77; .cpp:341,377)
 *   hvx_tu_forward_batch  TComTrQuant::transformNxN (TComTrQuant.h:98-337; .cpp:1460)
 *   hvx_tu_inverse_batch  TComTrQuant::invTransformNxN (TComTrQuant.cpp:1547)
 *   hvx_tu_pipeline_batch transformNxN + invTransformNxN + TComRdCost::getDistPart(SSE)
 *                         as called back-to-back per TU by TEncSearch::xEstimateInterResidualQT
 *                         (TEncSearch.cpp:4632-4711) and xIntraCodingTUBlock (:1262-1384)
 *   hvx_me_batch          TEncSearch::xMotionEstimation, uni-prediction path
 *                         (TEncSearch.h:126-215; TEncSearch.cpp:3663-3760, xTZSearch :3881,
 *                         xPatternSearchFracDIF :4240)
 *   hvx_ssim_batch        compute_SSIM (stvssim_src/stvssimrdo2_att/lencod/src/stvssim.c:491)
 *   hvx_stvssim_batch     compute_stVSSIM (stvssim.c:587)
 *   hvx_estbits_update / hvx_estbits_batch   TEncSbac::estBit (TEncSbac.cpp:1726)
 *   hvx_mc_batch          TComPrediction::motionCompensation (TComPrediction.cpp:517)
 *   hvx_coeff_bits_batch  TEncEntropy::encodeCoeffNxN -> TEncSbac::codeCoeffNxN (TEncEntropy.cpp:654,
 *                         TEncSbac.cpp:1181) under TEncBinCABACCounter (TEncBinCoderCABACCounter.cpp:74):
 *                         the RD search's coefficient rate (TEncSearch.cpp:969, 4706, 4875, 5136)
 *   hvx_coeff_write_batch TEncSbac::codeCoeffNxN (TEncSbac.cpp:1181) through the slice writer's
 *                         arithmetic coder TEncBinCABAC (TEncBinCoderCABAC.cpp:200-460): the residual
 *                         syntax of TU runs written as CABAC bytes (TEncSlice::encodeSlice path)
 *   hvx_me_full_batch     TEncSearch::xMotionEstimation with xPatternSearch (:3786), incl. bBi
 *   hvx_intra_pred_batch  TComPrediction::initIntraPatternChType (TComPattern.cpp:115, reference
 *                         samples + smoothing) + predIntraAng (TComPrediction.cpp:455)
 *   hvx_intra_search_batch TEncSearch::estIntraPredLumaQT's first pass (TEncSearch.cpp:2244-2323):
 *                         35-mode Hadamard cost ranking + MPM candidates per luma PU
 *   hvx_deblock           TComLoopFilter::loopFilterPic (TComLoopFilter.cpp:130, xEdgeFilterLuma :560,
 *                         xEdgeFilterChroma :679) on given boundary strengths
 *   hvx_sao_stats         TEncSampleAdaptiveOffset::getStatistics (TEncSampleAdaptiveOffset.cpp:285,
 *                         getBlkStats :892): per-CTU SAO statistics of a deblocked picture
 *   hvx_sao_apply         TComSampleAdaptiveOffset::offsetCTU (TComSampleAdaptiveOffset.cpp:554,
 *                         offsetBlock :313) of every CTU with given (merge-resolved) parameters
 *   hvx_plane_from_pel    TComPicYuv int16 padded plane -> device 8-bit padded plane, with
 *                         TComPicYuv::extendPicBorder (TComPicYuv.cpp:197)
 */
#ifndef HVX_H
#define HVX_H
#include <stddef.h>
#include <stdint.h>
#include "hvx_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HVX_OK 0
#define HVX_E_INVALID -1   /* bad argument (shape/size the kernel does not support) */
#define HVX_E_NODEV -2     /* no HIP device */
#define HVX_E_HIP -1000    /* HVX_E_HIP - (int)hipError_t */

typedef struct hvx_ctx hvx_ctx;

int hvx_create(int device, hvx_ctx **out);
int hvx_destroy(hvx_ctx *ctx);
/* Run subsequent batches on an external stream (hipStream_t passed as void*); NULL = own stream. */
int hvx_set_stream(hvx_ctx *ctx, void *stream);
void *hvx_get_stream(hvx_ctx *ctx);
int hvx_sync(hvx_ctx *ctx);
const char *hvx_last_error(void);
int hvx_version(void);

/* ---------------------------------------------------------------------------------------
 * Distortion.  kind: HVX_DIST_* below.  org/cur are int16 (HM Pel) sample arrays; each
 * job gives element offsets and strides into d_org / d_cur.  Output: Distortion (uint32).
 * ------------------------------------------------------------------------------------- */
#define HVX_DIST_SAD_ME 0   /* setDistParam(pattern) dispatch: 4/8/16/32/64/12/24/48 honour sub_shift */
#define HVX_DIST_SAD 1      /* getDistPart(DF_SAD) / xGetSAD: all rows (sub_shift ignored) */
#define HVX_DIST_SATD 2     /* xGetHADs: 8x8 / 4x4 / 2x2 Hadamard tiles */
#define HVX_DIST_SSE 3      /* getDistPart(DF_SSE), luma */
#define HVX_DIST_SSE_W 4    /* getDistPart(DF_SSE), chroma: (uint32)(weight * sse) */

typedef struct hvx_dist_job {
  int32_t kind, w, h, sub_shift;
  int64_t org_off, cur_off;       /* element offsets */
  int32_t org_stride, cur_stride; /* elements */
  double weight;                  /* m_distortionWeight[compID] for HVX_DIST_SSE_W */
} hvx_dist_job;

int hvx_dist_batch(hvx_ctx *ctx, const int16_t *d_org, const int16_t *d_cur, const hvx_dist_job *d_jobs, int n,
                   uint32_t *d_out);

/* ---------------------------------------------------------------------------------------
 * Interpolation.  One job = one filterHor (vertical=0) or filterVer (vertical=1) call.
 * is_luma: 8-tap quarter-pel luma, else 4-tap eighth-pel chroma (4:2:0 frac index).
 * src_off points at the block origin (the filter reads (N/2-1) samples before it).
 * ------------------------------------------------------------------------------------- */
typedef struct hvx_interp_job {
  int32_t is_luma, vertical, frac, is_first, is_last, w, h, pad_;
  int64_t src_off, dst_off;
  int32_t src_stride, dst_stride;
} hvx_interp_job;

int hvx_interp_batch(hvx_ctx *ctx, const int16_t *d_src, int16_t *d_dst, const hvx_interp_job *d_jobs, int n);

/* ---------------------------------------------------------------------------------------
 * Transform units.  TU i reads its desc d_desc[i], its estBits table d_est[d_est_idx[i]]
 * (d_est_idx may be NULL: TU i uses d_est[i]) and w*h contiguous elements at element
 * offset d_off[i] of every per-TU array (residual in/out int16 row-major, levels int32,
 * optional temp (transform output) / arl (adaptive-QP levels) int32, may be NULL).
 * d_abs_sum[i] receives uiAbsSum.
 * ------------------------------------------------------------------------------------- */
int hvx_tu_forward_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const hvx_estbits *d_est, const int32_t *d_est_idx,
                         const int64_t *d_off, int n, const int16_t *d_residual, int32_t *d_temp, int32_t *d_levels,
                         int32_t *d_arl, int32_t *d_abs_sum);
int hvx_tu_inverse_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, int n, const int32_t *d_levels,
                         int16_t *d_residual_out);
/* forward + inverse + SSE(residual, reconstructed residual) = distortion of the coded TU */
int hvx_tu_pipeline_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const hvx_estbits *d_est, const int32_t *d_est_idx,
                          const int64_t *d_off, int n, const int16_t *d_residual, int32_t *d_levels,
                          int32_t *d_abs_sum, int16_t *d_residual_out, uint32_t *d_sse);

/* Synchronous single-TU convenience forms over HOST memory (the per-call seam used by the
 * HM shim in integration/; staged through a device scratch buffer owned by the context). */
int hvx_tu_forward_host(hvx_ctx *ctx, const hvx_tu_desc *h_desc, const hvx_estbits *h_est, const int16_t *h_residual,
                        int residual_stride, int32_t *h_levels, int32_t *h_arl, int32_t *h_abs_sum);
int hvx_tu_inverse_host(hvx_ctx *ctx, const hvx_tu_desc *h_desc, const int32_t *h_levels, int16_t *h_residual,
                        int residual_stride);

/* ---------------------------------------------------------------------------------------
 * Motion estimation.  Planes are 8-bit padded planes (margin HVX_PLANE_MARGIN on every
 * side, luma stride `stride` bytes); d_cur_planes[j.cur_idx] / d_ref_planes[j.ref_idx]
 * point at sample (0,0) of each picture (device pointers, array itself in device memory).
 * ------------------------------------------------------------------------------------- */
#define HVX_PLANE_MARGIN 80
int hvx_me_batch(hvx_ctx *ctx, const uint8_t *const *d_cur_planes, const uint8_t *const *d_ref_planes, int stride,
                 const hvx_me_job *d_jobs, int n, hvx_me_result *d_out);

/* ---------------------------------------------------------------------------------------
 * SSIM metric (float32, JM stvssim semantics).  Blocks are 8-bit with their own strides.
 * ------------------------------------------------------------------------------------- */
typedef struct hvx_ssim_job {
  int32_t w, h, wint, overlap;
  int64_t org_off, rec_off;
  int32_t org_stride, rec_stride;
} hvx_ssim_job;
/* xMotionEstimation with the integer FULL search (TEncSearch.cpp:3663-3760 with
 * FastSearch=0 or bBi; xPatternSearch :3786) + xPatternSearchFracDIF.  The search pattern is an
 * int16 plane: d_tgt_planes[job.cur_idx] (stride tgt_stride) at (pu_x, pu_y) -- the original,
 * or for bi-prediction refinement the removeHighFreq target 2*org - pred(other list)
 * (TComYuv.cpp:409).  Search range: job.search_range (BipredSearchRange for bBi) around
 * (center_x, center_y); HVX_ME_BI weights the final cost by 0.5.  Result as hvx_me_batch
 * (mv_int/sad_int are the full-search result). */
int hvx_me_full_batch(hvx_ctx *ctx, const int16_t *const *d_tgt_planes, int tgt_stride,
                      const uint8_t *const *d_ref_planes, int stride, const hvx_me_job *d_jobs, int n,
                      hvx_me_result *d_out);

int hvx_ssim_batch(hvx_ctx *ctx, const uint8_t *d_org, const uint8_t *d_rec, const hvx_ssim_job *d_jobs, int n,
                   float *d_out);

/* stVSSIM: job j uses frames d_hist_org[j*26 + o], d_hist_rec[j*26 + o] (o < min(gama,26);
 * entry min(gama,26)-1 is the current frame) with stride hist_stride, and the per-pixel
 * direction map d_dirs + dirs_off (float, stride dirs_stride, luma resolution).
 * Output per job: {ssim, ssim3d, stvssim, return value}. */
typedef struct hvx_stvssim_job {
  int32_t w, h, wint, overlap, gama, comp, hist_stride, dirs_stride;
  int64_t dirs_off;
} hvx_stvssim_job;
int hvx_stvssim_batch(hvx_ctx *ctx, const uint8_t *const *d_hist_org, const uint8_t *const *d_hist_rec,
                      const float *d_dirs, const hvx_stvssim_job *d_jobs, int n, float *d_out4);

/* ---------------------------------------------------------------------------------------
 * Motion compensation (hvx_types.h hvx_mc_job): TComPrediction::motionCompensation /
 * xPredInterUni / xPredInterBi / xPredInterBlk / xWeightedAverage (TComPrediction.cpp:517-722)
 * and TComYuv::addAvg (TComYuv.cpp:352).  d_planes: device array of 3*n_refs pointers, entry
 * 3*r + c = sample (0,0) of component c (0 Y, 1 Cb, 2 Cr) of reference r, HM TComPicYuv int16
 * planes (margins >= the MV clip range + filter reach, e.g. HM's 80/40); luma_stride /
 * chroma_stride in samples.  d_dst receives int16 prediction samples.
 * ------------------------------------------------------------------------------------- */
int hvx_mc_batch(hvx_ctx *ctx, const int16_t *const *d_planes, int luma_stride, int chroma_stride,
                 const hvx_mc_job *d_jobs, int n, int16_t *d_dst);

/* Device memory helpers for callers without HIP headers (ordered on the context's stream). */
int hvx_alloc(hvx_ctx *ctx, size_t bytes, void **d_out);
int hvx_free(hvx_ctx *ctx, void *d);
int hvx_upload(hvx_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);   /* async */
int hvx_download(hvx_ctx *ctx, void *h_dst, const void *d_src, size_t bytes); /* async */

/* ---------------------------------------------------------------------------------------
 * Rate tables from CABAC state: TEncSbac::estBit (TEncSbac.cpp:1726-1950), i.e.
 * estCBFBit, estSignificantCoeffGroupMapBit, estSignificantMapBit,
 * estLastSignificantPositionBit, estSignificantCoefficientsBit + the Golomb-Rice statistics.
 * ctx_states: the encoder's context models in TEncSbac::m_contextModels order, one
 * ContextModel::m_ucState byte (state << 1 | MPS) each, HVX_NUM_CTX of them;
 * entropy_bits: ContextModel::m_entropyBits (128 entries, ContextModel.cpp:106 -- the caller
 * passes the encoder's own table); rice_stats: m_golombRiceAdaptationStatistics[4].  Exactly
 * the entries the reference writes for a width x height TU of channel type ch_type are
 * written; the rest of *inout is left as it was (the reference keeps a persistent table).
 * ------------------------------------------------------------------------------------- */
#define HVX_CTX_QT_CBF 28      /* 2 sets x 5 (blockCbpBits) */
#define HVX_CTX_QT_ROOT_CBF 41 /* estCBFBit reads 4 models from here (the reference's loop bound) */
#define HVX_CTX_SIG_CG 42      /* [chType][2] */
#define HVX_CTX_SIG 46         /* 28 luma + 16 chroma */
#define HVX_CTX_LAST_X 90      /* [chType][15] */
#define HVX_CTX_LAST_Y 120     /* [chType][15] */
#define HVX_CTX_ONE 150        /* 16 luma + 8 chroma */
#define HVX_CTX_ABS 174        /* 4 luma + 2 chroma */
typedef struct hvx_estbit_job { int32_t width, height, ch_type, pad_; } hvx_estbit_job;
/* host form (no device work; usable from the encoder thread) */
int hvx_estbits_update(const uint8_t *ctx_states, const int32_t *entropy_bits, const uint32_t *rice_stats, int width,
                       int height, int ch_type, hvx_estbits *inout);
/* batched device form: job i reads d_states[i*HVX_NUM_CTX ..], d_rice[i*4 ..], updates d_inout[i] */
int hvx_estbits_batch(hvx_ctx *ctx, const uint8_t *d_states, const int32_t *d_entropy_bits, const uint32_t *d_rice,
                      const hvx_estbit_job *d_jobs, int n, hvx_estbits *d_inout);

/* ---------------------------------------------------------------------------------------
 * Coefficient rate: TEncSbac::codeCoeffNxN counted by TEncBinCABACCounter (the RD search's
 * bit estimate of one TU's levels; TEncSbac.cpp:1181).  TU i reads its desc d_desc[i] (comp,
 * width == height in {4,8,16,32}, scan_type, transform_skip, pps_tskip, sign_hiding,
 * transquant_bypass, golomb_rice_stat, persistent_rice, ts_context, extended_precision,
 * max_log2_tr_range), w*h raster int32 levels at element offset d_off[i] of d_levels, and
 * the RD coder's context states d_states[i*HVX_NUM_CTX ..] (m_contextModels order, advanced in
 * place bin by bin as the counter does).  d_entropy_bits = ContextModel::m_entropyBits (128).
 * d_out[i].frac_bits = increase of m_fracBits (bits = frac >> 15); num_sig = 0 for an all-zero
 * TU (nothing coded; the reference refuses such a call), 0xffffffff for an unsupported shape.
 * ------------------------------------------------------------------------------------- */
int hvx_coeff_bits_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, int n, const int32_t *d_levels,
                         const int32_t *d_entropy_bits, uint8_t *d_states, hvx_coeff_bits *d_out);

/* ---------------------------------------------------------------------------------------
 * CABAC residual writer (replaces TEncSbac::codeCoeffNxN with TEncBinCABAC as m_pcBinIf,
 * TEncSbac.cpp:1181 / TEncBinCoderCABAC.cpp:200-460; called by TEncEntropy::encodeCoeffNxN,
 * TEncEntropy.cpp:654, on the TEncSlice::encodeSlice path).  n_streams independent bitstream
 * runs, one lane each: run k codes TUs [d_stream_first[k], d_stream_first[k+1]) (hvx_tu_desc
 * and raster levels as in hvx_coeff_bits_batch) in order through ONE arithmetic coder whose
 * registers start at d_regs[k] (TEncBinCABAC::start() = {0, 510, 23, 0, 0xff}) and whose context
 * states start at d_states[k*HVX_NUM_CTX ..]; both are advanced in place.  The bytes the coder
 * completes are written to d_out + d_out_off[k] (at most out_cap bytes) and counted in
 * d_out_len[k] (-1: more than out_cap, -2: a TU of the run is unsupported -- non-square, not
 * 4..32, scan type > 2, or persistent_rice set -- checked before anything is coded, so the run's
 * registers and states are left untouched).  d_regs[k].coded accumulates the context models the
 * run coded a bin with (the caller sets their m_binsCoded).  Bytes still held in the
 * registers (low, the buffered 0xff run) belong to the next call or to TEncBinCABAC::finish().
 * ------------------------------------------------------------------------------------- */
int hvx_coeff_write_batch(hvx_ctx *ctx, const hvx_tu_desc *d_desc, const int64_t *d_off, const int32_t *d_levels,
                          const int32_t *d_stream_first, int n_streams, uint8_t *d_states, hvx_cabac_regs *d_regs,
                          uint8_t *d_out, const int64_t *d_out_off, int out_cap, int32_t *d_out_len);

/* ---------------------------------------------------------------------------------------
 * Intra (hvx_types.h hvx_intra_job).  d_rec = sample (0,0) of the 8-bit plane holding the
 * reconstructed neighbours (any stride; only samples of available units are read), d_org the
 * original with the same stride.  hvx_intra_pred_batch writes job i's (1<<log2_size)^2
 * prediction of job.mode at d_pred + d_pred_off[i] (row-major), and, when d_ref_out is not NULL,
 * its unfiltered and filtered reference borders (2 x 257 int16 per job, hvx_types.h layout; the
 * filtered one is zero for chroma).  hvx_intra_search_batch runs the first pass of luma PU jobs
 * (rates from ctx_state / frac_bits with d_entropy_bits = ContextModel::m_entropyBits, 128
 * int32).  A job with an out-of-range size, channel or unit is skipped (its output untouched).
 * ------------------------------------------------------------------------------------- */
int hvx_intra_pred_batch(hvx_ctx *ctx, const uint8_t *d_rec, int stride, const hvx_intra_job *d_jobs, int n,
                         uint8_t *d_pred, const int64_t *d_pred_off, int16_t *d_ref_out);
int hvx_intra_search_batch(hvx_ctx *ctx, const uint8_t *d_org, const uint8_t *d_rec, int stride,
                           const hvx_intra_job *d_jobs, int n, const int32_t *d_entropy_bits,
                           hvx_intra_search_result *d_out);

/* ---------------------------------------------------------------------------------------
 * Deblocking in place (hvx_types.h hvx_deblock_params): d_y / d_cb / d_cr = sample (0,0) of the
 * reconstructed 8-bit planes (4:2:0, any strides >= the plane widths), d_bs_ver / d_bs_hor /
 * d_qp = (pic_w/4) x (pic_h/4) per-4x4-unit maps on the device.  Two launches on the context
 * stream: all vertical edges, then all horizontal edges.
 * ------------------------------------------------------------------------------------- */
int hvx_deblock(hvx_ctx *ctx, uint8_t *d_y, int y_stride, uint8_t *d_cb, uint8_t *d_cr, int c_stride,
                const uint8_t *d_bs_ver, const uint8_t *d_bs_hor, const int8_t *d_qp, const hvx_deblock_params *h_params);

/* ---------------------------------------------------------------------------------------
 * SAO (hvx_types.h hvx_sao_*), single slice and tile, 8-bit 4:2:0, pic_w / pic_h multiples of 8.
 * Plane pointers = sample (0,0); chroma pointers may both be NULL (luma only).
 * hvx_sao_stats: d_stats = [ctu][3][5] hvx_sao_stat (components not computed are untouched) of
 * the deblocked picture d_rec_* against the original d_org_* -- SAOProcess's statistics with
 * SAOLcuBoundary (pre-deblocking samples) off.  hvx_sao_apply: every sample of d_dst_* = d_src_*
 * with its CTU's offsets (d_params: one hvx_sao_ctu per CTU, raster order); d_dst must not
 * overlap d_src (edge classes read the unmodified neighbours, as offsetCTU reads SAOProcess's copy).
 * ------------------------------------------------------------------------------------- */
int hvx_sao_stats(hvx_ctx *ctx, const uint8_t *d_org_y, const uint8_t *d_org_cb, const uint8_t *d_org_cr,
                  int org_y_stride, int org_c_stride, const uint8_t *d_rec_y, const uint8_t *d_rec_cb,
                  const uint8_t *d_rec_cr, int rec_y_stride, int rec_c_stride, int pic_w, int pic_h,
                  hvx_sao_stat *d_stats);
int hvx_sao_apply(hvx_ctx *ctx, const uint8_t *d_src_y, const uint8_t *d_src_cb, const uint8_t *d_src_cr,
                  int src_y_stride, int src_c_stride, uint8_t *d_dst_y, uint8_t *d_dst_cb, uint8_t *d_dst_cr,
                  int dst_y_stride, int dst_c_stride, int pic_w, int pic_h, const hvx_sao_ctu *d_params);
/* SAO's RD decision for n_jobs pictures, one wave each (TEncSampleAdaptiveOffset::decideBlkParams
 * TEncSampleAdaptiveOffset.cpp:763: deriveModeNewRDO :566 / deriveModeMergeRDO :709 per CTU in raster
 * order, deriveOffsets :447 with estIterOffset :414, getDistortion :370, the SAO syntax rate
 * TEncSbac::codeSAOBlkParam TEncSbac.cpp:1683 on the RD counter carried CTU to CTU, the picture-level
 * disable test :846): the coded and the applied (merge-resolved, hvx_sao_apply-ready) parameters. */
int hvx_sao_decide(hvx_ctx *ctx, const hvx_sao_decide_job *d_jobs, int n_jobs);

/* ---------------------------------------------------------------------------------------
 * Picture upload: HM int16 plane (width x height samples, any stride, device copy) ->
 * 8-bit padded plane (stride = width + 2*HVX_PLANE_MARGIN), borders extended.  d_plane is
 * the START of the padded allocation ((height + 2*M) rows); sample (0,0) is at M*stride + M.
 * ------------------------------------------------------------------------------------- */
int hvx_plane_from_pel(hvx_ctx *ctx, const int16_t *d_pel, int pel_stride, int width, int height, uint8_t *d_plane);
int hvx_plane_extend(hvx_ctx *ctx, uint8_t *d_plane, int width, int height);

/* ---------------------------------------------------------------------------------------
 * HM-exact CTU decision: TEncCu::compressCtu (hm-16.5rc1 TEncCu.cpp:228, called from
 * TEncSlice::compressSlice TEncSlice.cpp:814) followed by the CTU syntax walk of
 * TEncCu::encodeCtu (TEncCu.cpp:252) on the RD coder, whose context states start the next CTU
 * (TEncSlice.cpp:821-828).  Replaces, per CTU, the whole xCompressCU recursion: merge/skip
 * (xCheckRDCostMerge2Nx2N :1166), 2Nx2N / Nx2N / 2NxN / AMP inter search with AMVP, merge
 * estimation and AMP_MRG (xCheckRDCostInter :1291, TEncSearch::predInterSearch :2912), the RQT
 * (xEstimateInterResidualQT :4426), intra-in-inter and NxN intra (xCheckRDCostIntra :1330,
 * estIntraPredLumaQT :2176, estIntraPredChromaQT :2563), split decisions and xCheckBestMode.
 * Tool set of encoder_lowdelay_P_main.cfg (hvx_types.h hvx_hm_picture): CTU 64, depth 4, TU
 * 4..32 with QuadtreeTUMaxDepthInter/Intra 3, RDOQ + RDOQTS, sign hiding, transform skip with
 * TransformSkipFast, FEN, FDM, AMP, TZ search with HadamardME, TMVP, 5 merge candidates, no
 * ECU/ESD/CFM, no PCM, no delta QP, no lossless, no weighted prediction; I, P and B slices (B:
 * encoder_randomaccess_main.cfg's bi-prediction with BipredSearchRange, FastMEForGenBLowDelay,
 * MvdL1Zero); the TEncCu comparisons on HM's SSE cost or the stvssim SSIM cost (rd_metric).
 * One wave per job (hvx_hm_job): the chain's CTUs are decided in raster order with the contexts
 * carried; d_state = n_jobs * hvx_hm_state_size() bytes of device scratch.  Outputs per CTU
 * slot: d_out_ctu (the CTU's final TComDataCU data and RD totals), d_out_rec (6144 bytes: its
 * pre-loop-filter reconstruction, Y 64x64 | Cb 32x32 | Cr 32x32, 0 outside the picture),
 * d_out_coder (optional: the RD coder after encodeCtu).
 * Preconditions of every job, checked on the device before it runs (a job violating one is
 * skipped -- nothing of it is written -- and its status word holds -HVX_HM_BAD_*; read with
 * hvx_hm_job_status): 0 <= pic < n_pics; the picture's w, h positive multiples of 8 with
 * w_ctus / h_ctus = ceil(w / 64) / ceil(h / 64); slice_type 0..2 with nref[0] 1..4 (P, B),
 * nref[1] 0..4 (B only), I without references; every used ref_plane in 0..7 with its planes set;
 * org / rec / ctus / entropy_bits (and col_field when col_valid) set; 0 <= slice_start <=
 * first_ctu, n_ctus >= 1, first_ctu + n_ctus - 1 <= slice_end < w_ctus * h_ctus; 0 <= out and,
 * when n_out > 0 (the slots of the output arrays), out + n_ctus <= n_out.
 * ------------------------------------------------------------------------------------- */
#define HVX_HM_BAD_PIC 1
#define HVX_HM_BAD_GEOMETRY 2
#define HVX_HM_BAD_REFS 3
#define HVX_HM_BAD_PLANES 4
#define HVX_HM_BAD_CTUS 5
#define HVX_HM_BAD_OUT 6
int hvx_hm_state_size(size_t *bytes);
int hvx_hm_compress(hvx_ctx *ctx, const hvx_hm_picture *d_pics, int n_pics, const hvx_hm_job *d_jobs, int n_jobs,
                    int n_out, void *d_state, hvx_hm_ctu *d_out_ctu, uint8_t *d_out_rec, hvx_hm_coder *d_out_coder);
/* the status word of each of the last launch's jobs (0: ran; -HVX_HM_BAD_*: refused); synchronises
 * the context's stream */
int hvx_hm_job_status(hvx_ctx *ctx, const void *d_state, int n_jobs, int32_t *h_status);
/* The slice data of decided pictures: TEncSlice::encodeSlice's CTU loop
 * (TEncSlice.cpp:920) through TEncBinCABAC -- per CTU the SAO syntax (TEncSbac::codeSAOBlkParam
 * TEncSbac.cpp:1683) and TEncCu::encodeCtu (TEncCu.cpp:252: xEncodeCU :940, finishCU :885) -- one wave
 * per slice (hvx_types.h hvx_hm_slice).  d_state = n_slices * hvx_hm_state_size() bytes of scratch;
 * d_out = n_slices results.  The caller ends each slice as encodeSlice does: the terminating bin 1,
 * TEncBinCABAC::finish (TEncBinCoderCABAC.cpp:81) and the byte alignment, from the result's registers. */
int hvx_hm_write_slices(hvx_ctx *ctx, const hvx_hm_picture *d_pics, int n_pics, const hvx_hm_slice *d_slices,
                        int n_slices, void *d_state, hvx_hm_slice_result *d_out);
/* HVX_RD_STVSSIM's history part, once per picture (hvx_hm_picture.stv_sums): compute_stVSSIM's
 * (stvssim.c:651-702) five directional accumulators of every window after the hist_n history frames,
 * for the windows the CU decision can evaluate -- luma 8x8 windows and chroma 8x8 / 4x4 windows on the
 * 4-sample grid -- from h_pic's hist / hist_n / hist_stride / w / h (host copy of the descriptor).
 * Layout (floats): luma [(h-8)/4+1][(w-8)/4+1][4 directions][mo, me, vo, ve, cov], then chroma 8x8
 * [(h/2-8)/4+1][(w/2-8)/4+1][4][5], then chroma 4x4 [(h/2-4)/4+1][(w/2-4)/4+1][4][5]; chroma from the Cb
 * history planes (which Cr reads too, hvx_types.h).  d_sums: hvx_hm_stv_sums_size bytes. */
int hvx_hm_stv_sums_size(int w, int h, size_t *bytes);
int hvx_hm_stv_prepare(hvx_ctx *ctx, const hvx_hm_picture *h_pic, float *d_sums);

/* ---------------------------------------------------------------------------------------
 * The picture-level steps TEncGOP runs after compressSlice (TEncGOP.cpp:1465-1629), on a picture
 * whose every CTU hvx_hm_compress has decided (h_pic: the host copy of its hvx_hm_picture; its
 * ctus and rec complete), in stream order:
 *   h_dbk != NULL: TComLoopFilter::loopFilterPic (TComLoopFilter.cpp:130) on rec in place, with the
 *     boundary strengths and QP map derived on the device from the CTU data exactly as
 *     xDeblockCU / xGetBoundaryStrengthSingle do (:170-557; LFCrossSliceBoundaryFlag on, filter
 *     enabled; h_dbk->pic_w / pic_h = the picture's).  d_work: 3 * (w/4) * (h/4) bytes that receive
 *     the bs_ver, bs_hor and QP maps of hvx_deblock (in that order).  NULL = deblocking disabled.
 *   d_col_field != NULL: TComPic::compressMotion -- the picture's hvx_hm_picture.col_field rows
 *     ([w_ctus*h_ctus][16][8]) for the pictures that take it as their collocated picture.
 *   d_ref8 / d_ref16_*: the filtered picture as the engine's reference formats (hvx_hm_picture
 *     ref8 / ref16, sample (0,0) pointers): 8-bit luma with HVX_PLANE_MARGIN, int16 Y / Cb / Cr with
 *     80 / 40 samples of border, TComPicYuv::extendPicBorder (TComSlice.cpp:351).  Either may be NULL.
 * SAO is not applied here (hvx_sao_apply with decided parameters).  w, h multiples of 8.
 * ------------------------------------------------------------------------------------- */
int hvx_hm_finish_picture(hvx_ctx *ctx, const hvx_hm_picture *h_pic, const hvx_deblock_params *h_dbk, uint8_t *d_work,
                          int16_t *d_col_field, uint8_t *d_ref8, int ref8_stride, int16_t *d_ref16_y, int16_t *d_ref16_cb,
                          int16_t *d_ref16_cr, int ref16_stride_y, int ref16_stride_c);

#ifdef __cplusplus
}
#endif
#endif
