/* hvx_oracle.h -- CPU restatement of the HM-16.5rc1 CU mode-decision kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may call it,
 * as the checker, never as the product path.  The product is the HIP library
 * video_codecs_amd/libhvx.so (include/hvx.h).
 *
 * Pinned against golden vectors produced by the reference itself
 * (oracle/golden_gen.cpp, oracle/tu_capture.cpp -> tests/golden/).
 * All types mirror HM's Main-profile build: Pel=int16, TCoeff=int32,
 * Distortion=uint32 (hm-16.5rc1/source/Lib/TLibCommon/TypeDef.h:211-230).
 */
#ifndef HVX_ORACLE_H
#define HVX_ORACLE_H
#include <stdint.h>
#include "../include/hvx_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- distortion (TComRdCost.cpp:294-451, 461-1593) ---- */
uint32_t hvxo_sad(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, int sub_shift);
uint32_t hvxo_sad_me(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, int sub_shift);
uint32_t hvxo_satd(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h);
uint32_t hvxo_sse(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h);
uint32_t hvxo_sse_weighted(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, double weight);
uint32_t hvxo_eg_bits(int v);

/* ---- interpolation (TComInterpolationFilter.cpp:94-394) ---- */
void hvxo_filter_hor(int is_luma, const int16_t *src, int ss, int16_t *dst, int ds, int w, int h, int frac, int is_last);
void hvxo_filter_ver(int is_luma, const int16_t *src, int ss, int16_t *dst, int ds, int w, int h, int frac,
                     int is_first, int is_last);

/* ---- transforms (TComTrQuant.cpp:388-987) ---- */
void hvxo_fwd_transform(const int32_t *block, int32_t *coeff, int n, int use_dst);
void hvxo_inv_transform(const int32_t *coeff, int32_t *block, int n, int use_dst);

/* ---- TU-level forward path: transformNxN (TComTrQuant.cpp:1460) = xT/xTransformSkip + xQuant
 *      (RDOQ xRateDistOptQuant :2129 / selective RDOQ :1257 / scalar quant + SBH :1126,991) ---- */
void hvxo_transform_nxn(const hvx_tu_desc *tu, const hvx_estbits *est, const int16_t *residual, int stride,
                        int32_t *temp_coeff, int32_t *levels, int32_t *arl, int32_t *abs_sum);
/* quantisation only, on transform output `coeff` (raster, w*h) */
void hvxo_quant(const hvx_tu_desc *tu, const hvx_estbits *est, const int32_t *coeff, int32_t *levels,
                int32_t *arl, int32_t *abs_sum);
/* ---- TU-level inverse path: invTransformNxN (TComTrQuant.cpp:1547) = xDeQuant :1314 + xIT/xITransformSkip ---- */
void hvxo_inv_transform_nxn(const hvx_tu_desc *tu, const int32_t *levels, int16_t *residual, int stride);

/* ---- motion estimation (TEncSearch.cpp:3663-3760 uni-pred path) on 8-bit padded planes ---- */
void hvxo_motion_estimation(const uint8_t *cur, int cur_stride, const uint8_t *ref, int ref_stride,
                            const hvx_me_job *job, hvx_me_result *res);
/* quarter-sample luma interpolation of one block at quarter-pel MV (standard two-stage, 8-bit) */
void hvxo_luma_block_qpel(const uint8_t *ref, int stride, int x, int y, int mvx, int mvy, int w, int h, int16_t *out, int os);

/* ---- SSIM metric (stvssim.c:491-566, 587-830, 1565-1806) ---- */
float hvxo_ssim(const uint8_t *org, int so, const uint8_t *rec, int sr, int w, int h, int wint, int overlap);
float hvxo_stvssim(const uint8_t *const *org_hist, const uint8_t *const *rec_hist, int hist_stride,
                   const float *dirs, int dirs_stride, int w, int h, int wint, int overlap, int gama, int comp,
                   float *ssim, float *ssim3d, float *stvssim);
double hvxo_lambda_2(int qp);
/* TComPrediction::motionCompensation for one PU, no WP (TComPrediction.cpp:517-722) + addAvg
 * (TComYuv.cpp:352): planes[3*r + c] = sample (0,0) of component c of reference r (HM int16
 * planes); out = Y w*h, Cb, Cr (w/2)*(h/2) */
void hvxo_mc(const int16_t *const *planes, int luma_stride, int chroma_stride, const hvx_mc_job *j, int16_t *out);
/* xMotionEstimation with the integer full search (FastSearch=0 / bBi), int16 pattern plane */
void hvxo_me_full(const int16_t *tgt, int tstride, const uint8_t *refp, int ref_stride, const hvx_me_job *j,
                  hvx_me_result *r);
void hvxo_me_full_pat(const int16_t *pat, int pstride, const uint8_t *refp, int ref_stride, const hvx_me_job *j,
                      hvx_me_result *r);
/* TComYuv::addAvg per sample, 8-bit (TComYuv.cpp:352) */
void hvxo_add_avg(const int16_t *a, const int16_t *b, int16_t *dst, int n);
/* TEncSbac::estBit (TEncSbac.cpp:1726): context states (TEncSbac::m_contextModels order,
 * m_ucState bytes) + ContextModel::m_entropyBits -> the estBits entries for a w x h TU of
 * channel type ch (other entries untouched) */
void hvxo_estbits_update(const uint8_t *states, const int32_t *entropy_bits, const uint32_t *rice, int w, int h, int ch,
                         hvx_estbits *e);
double hvxo_adjust_lambda(double lambda, double eta);
/* TEncSbac::codeCoeffNxN counted by TEncBinCABACCounter (TEncSbac.cpp:1181): coef = w*h levels
 * (raster), states = the RD coder's HVX_NUM_CTX context states (advanced in place), eb =
 * ContextModel::m_entropyBits (128) */
void hvxo_coeff_bits(const hvx_tu_desc *tu, const int32_t *coef, uint8_t *states, const int32_t *eb, hvx_coeff_bits *out);
/* TEncSbac::codeCoeffNxN written by TEncBinCABAC (TEncBinCoderCABAC.cpp): the same syntax, the
 * bins driving *regs, the bytes the call completes into out (capacity cap); returns the byte
 * count, -1 past cap */
int hvxo_coeff_write(const hvx_tu_desc *tu, const int32_t *coef, uint8_t *states, hvx_cabac_regs *regs, uint8_t *out,
                     int cap);

/* ---- intra (border layout: hvx_oracle.c "Intra prediction") ---- */
/* fillReferenceSamples (TComPattern.cpp:364): raw border samples + bNeighborFlags -> border */
void hvxo_intra_fill(const int16_t *raw, const uint32_t *avail, int n, int unit_log2, int16_t *border);
/* initIntraPatternChType's [1 2 1] / strong smoothing (TComPattern.cpp:190-330) */
void hvxo_intra_filter(const int16_t *border, int n, int is_luma, int strong_enabled, int16_t *out);
/* filteringIntraReferenceSamples (TComPattern.cpp:544), 4:2:0 */
int hvxo_intra_use_filter(int mode, int n, int is_luma);
/* predIntraAng (TComPrediction.cpp:455): pred = n*n */
void hvxo_intra_pred(const int16_t *border, int n, int is_luma, int mode, uint8_t *pred);
/* estIntraPredLumaQT's first pass (TEncSearch.cpp:2244-2323); eb = ContextModel::m_entropyBits */
void hvxo_intra_search(const uint8_t *org, const int16_t *raw, const hvx_intra_job *j, const int32_t *eb,
                       hvx_intra_search_result *r);

/* ---- deblocking: loopFilterPic on given BS / QP maps, planes in place ---- */
void hvxo_deblock(uint8_t *y, int ys, uint8_t *cb, uint8_t *cr, int cs, const uint8_t *bs_ver, const uint8_t *bs_hor,
                  const int8_t *qp, const hvx_deblock_params *p);

/* ---- SAO, one plane (comp 0 luma / 1, 2 chroma 4:2:0; ctu = 64 >> (comp > 0)) ---- */
/* TEncSampleAdaptiveOffset::getStatistics / getBlkStats (non-pre-deblocking samples): out[ctu][5] */
void hvxo_sao_stats(const uint8_t *org, int os, const uint8_t *rec, int rs, int w, int h, int comp, hvx_sao_stat *out);
/* TComSampleAdaptiveOffset::offsetCTU of every CTU: dst = src with the CTU's offsets (dst != src) */
void hvxo_sao_apply(const uint8_t *src, int ss, uint8_t *dst, int ds, int w, int h, int comp,
                    const hvx_sao_ctu *params);

/* SAO's RD decision (TEncSampleAdaptiveOffset::decideBlkParams, TEncSampleAdaptiveOffset.cpp:763,
 * with deriveModeNewRDO :566, deriveModeMergeRDO :709, deriveOffsets :447, estIterOffset :414,
 * getDistortion :370 and the SAO syntax rate of TEncSbac::codeSAOBlkParam TEncSbac.cpp:1683 on the
 * RD counter), 8-bit 4:2:0, one tile.  stats = [ctu][comp 3][type 5][diff 32, count 32] (int64);
 * slice_enabled = decidePicParams' flags (Y, Cb, Cr); sao_states = the sao_merge / sao_type_idx
 * context states of the picture-start coder and frac_lo the low 15 bits of its fractional bit
 * count; slice_ctus = CTUs per slice (SliceMode 1; 0: one slice; merges stay inside a slice);
 * test_off = bTestSAODisableAtPictureLevel.  out = [ctu][comp][mode (0 off, 1 new, 2 merge), type,
 * band position, offsets of EO classes 0..4 / of the 4 bands]; recon (optional) = the parameters
 * offsetCTU applied, merges resolved ([ctu][comp] hvx_sao_ctu form; kept when the picture-level test
 * then disables SAO, which clears only the coded parameters and slice_enabled, as the reference
 * does).  Returns decideBlkParams' total cost. */
double hvxo_sao_decide(int w, int h, const int64_t *stats, const double *lambdas, int *slice_enabled,
                       const uint8_t *sao_states, int frac_lo, const int32_t *entropy_bits, int slice_ctus, int test_off,
                       int32_t *out, hvx_sao_ctu *recon);
/* decidePicParams (:332): the slice-enabled flags of a picture at temporal layer `layer` from the
 * SAO-off rates of the earlier pictures (disabled_rate [3][7]); and decideBlkParams' rate update
 * (:861-888) from a decided picture's reconstructed parameters (recon: [ctu][comp]). */
void hvxo_sao_pic_params(int layer, const double *disabled_rate, double rate, double rate_chroma, int *slice_enabled);
void hvxo_sao_update_rates(int layer, const hvx_sao_ctu *recon, int nctu, double rate, double rate_chroma,
                           double *disabled_rate);

/* boundary strengths of hvx_ctu_decide's CU trees (the bench step's deblocking input); cu/dec =
 * nctu*85 records of the whole picture, maps (pic_w/4) x (pic_h/4) */

/* tables (generated, HEVC spec values) */
void hvxo_dct_matrix(int n, int16_t *m /* n*n, [k][x] */);
const uint32_t *hvxo_scan(int grouped, int scan_type, int log2w, int log2h);

void hvxo_init_tables(void);

#ifdef __cplusplus
}
#endif
#endif
