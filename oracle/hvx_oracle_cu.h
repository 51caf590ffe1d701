/* hvx_oracle_cu.h -- CPU restatement of HM-16.5rc1's CTU mode decision (TEncCu::compressCtu,
 * TEncCu.cpp:228) and CTU syntax walk (TEncCu::encodeCtu, :252).
 *
 * TEST INFRASTRUCTURE ONLY: the parity oracle of the HM-exact CTU path (tests/, smoke()).
 * Pinned against the reference's own CTU decisions (oracle/cu_capture.cpp -> tests/golden/ctu_*.bin).
 */
#ifndef HVX_ORACLE_CU_H
#define HVX_ORACLE_CU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* an RD coder: TEncSbac's context states (m_ucState) + TEncBinCABACCounter::m_fracBits */
typedef struct hvxo_hm_coder {
  uint8_t st[202];
  uint64_t frac;
} hvxo_hm_coder;

/* the picture-level state the CU decision reads (TComSlice / TComRdCost / TComTrQuant) */
typedef struct hvxo_hm_pic {
  int w, h, w_ctus, h_ctus, poc, slice_type, qp;
  int nref[2], ref_poc[2][4], ref_plane_idx[2][4];
  int chroma_qp[2];
  int max_merge, tmvp, check_ldc, col_from_l0, col_valid, col_poc;
  int col_ref_poc[2][4];
  int mvd_l1_zero;                      /* TComSlice::getMvdL1ZeroFlag (TEncGOP.cpp:1311-1336) */
  int l1_to_l0[4];                      /* TComSlice::getList1IdxToList0Idx (TComSlice.cpp:302) */
  const int16_t *col_field;             /* the collocated picture, [ctu][16 blocks of 16x16][8] (cu_capture.cpp) */
  double lambda, sqrt_lambda, chroma_weight[2], tq_lambda[3];
  uint32_t lambda_motion;
  int search_range, amp;
  int bipred_range;                     /* BipredSearchRange (TEncSearch::m_bipredSearchRange) */
  int rd_metric;                        /* 0: HM's SSE cost; 1: the stvssim SSIM cost, 2: its stVSSIM cost in
                                           TEncCu's comparisons (include/hvx_types.h HVX_RD_*) */
  double lambda_ssim;                   /* rd_metric 1, 2: lambda_2(QP) * eta^0.85 (stvssim.c:1805, :1707) */
  const uint8_t *const *hist;           /* rd_metric 2: the stVSSIM history (hvx_hm_picture.hist layout) */
  int hist_n, hist_stride[2];
  const float *dirs;                    /* rd_metric 2: direction map, one float per 4x4 luma block */
  int dirs_stride;
  const int32_t *entropy_bits;          /* ContextModel::m_entropyBits[128] */
  const int16_t *org[3];                /* original, sample (0,0) */
  int org_stride[3];
  const uint8_t *org8;                  /* original luma, 8-bit (ME pattern) */
  int org8_stride;
  const int16_t *const *ref_planes16;   /* [3 * plane + comp] sample (0,0), margins >= 80 / 40 */
  int ref_stride16[2];
  const uint8_t *const *ref_planes8;    /* [plane] luma sample (0,0), margin >= 80 */
  int ref_stride8;
} hvxo_hm_pic;

/* mvd_l1_zero and l1_to_l0 from the slice type and the reference POC lists, as HM derives them:
 * a B slice whose L1 equals L0 entry by entry (GPB) codes no L1 MVD of bi-predicted PUs
 * (TEncGOP.cpp:1311-1336); l1_to_l0[i] = the first L0 index of L1 entry i's picture, or -1. */
void hvxo_hm_derive_lists(hvxo_hm_pic *pic);

/* the picture's CTU data (TComPic::getCtu): opaque, hvxo_hm_ctu_data_size() bytes per CTU */
typedef struct hvxo_hm_ctu_data hvxo_hm_ctu_data;
#define HVXO_HM_PART_FIELDS 29   /* the ctu_parts fields of cu_capture.cpp, in order */

size_t hvxo_hm_ctu_data_size(void);
void hvxo_hm_unpack_parts(const hvxo_hm_ctu_data *d, int16_t *out /* [256][HVXO_HM_PART_FIELDS] */);
void hvxo_hm_pack_parts(hvxo_hm_ctu_data *d, const int16_t *in);

/* TEncCu::compressCtu of CTU ctu_addr: ctus = the picture's CTU data (the CTUs before ctu_addr
 * hold their final decisions; ctu_addr's is written), rec = the picture reconstruction planes
 * (sample (0,0), sized to whole CTUs), entry = m_pppcRDSbacCoder[0][CI_CURR_BEST] on entry,
 * int2n = TEncSearch::m_integerMv2Nx2N [2][4][2] on entry.  after_encode (optional) = that coder
 * after TEncCu::encodeCtu, i.e. the next CTU's entry state. */
void hvxo_hm_compress_ctu(const hvxo_hm_pic *pic, hvxo_hm_ctu_data *ctus, int16_t *const *rec, const int *rec_stride,
                          int ctu_addr, const hvxo_hm_coder *entry, const int16_t *int2n, hvxo_hm_coder *after_encode);

/* The same for a CTU of a SliceMode=1 slice [slice_start, slice_end] (CTU addresses): neighbours
 * before the slice are unavailable, the slice's last CTU ends without the end_of_slice bin;
 * int2n_out (optional) receives m_integerMv2Nx2N after the decision (the next CTU's). */
void hvxo_hm_compress_ctu_slice(const hvxo_hm_pic *pic, hvxo_hm_ctu_data *ctus, int16_t *const *rec, const int *rec_stride,
                                int ctu_addr, int slice_start, int slice_end, const hvxo_hm_coder *entry,
                                const int16_t *int2n, int16_t *int2n_out, hvxo_hm_coder *after_encode);

/* Replay one captured picture (tests/golden/ctu_*.bin arrays, cu_capture.cpp layouts).
 * mode 0: every CTU from the reference's own entry state and its left/above CTUs' final data;
 * mode 1: the CTUs in raster order, each from the previous CTU's restated encodeCtu state.
 * slice_ctus > 0: SliceMode=1 slices of that many CTUs (each slice starts from the captured state).
 * Outputs per CTU (n = pic's CTU count): parts [n][256][29], coef [n][6144], recon [n][6144],
 * cost [n], bits_dist [n][2], states/frac after encodeCtu [n][202] / [n]. */
int hvxo_hm_replay_picture(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                           const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                           const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                           const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                           int slice_ctus, int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon, double *out_cost,
                           uint32_t *out_bits_dist, uint8_t *out_states, int64_t *out_frac);

/* The same with the CU decision's cost selected: rd_metric 0 = HM's SSE cost (as above), 1 = the
 * stvssim SSIM cost with lambda_ssim (hvxo_hm_pic.rd_metric) */
int hvxo_hm_replay_picture_rd(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                              const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                              const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                              const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                              int slice_ctus, int rd_metric, double lambda_ssim, int16_t *out_parts, int32_t *out_coef,
                              uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist, uint8_t *out_states,
                              int64_t *out_frac);

/* The stVSSIM inputs of rd_metric 2 (hvx_hm_picture.hist / dirs, include/hvx_types.h): hist[6k + c]
 * original / hist[6k + 3 + c] reconstruction of the k-th most recent previous picture (8-bit, strides
 * hist_stride[0] luma / [1] chroma), k < hist_n <= 25; dirs: orientation per 4x4 luma block. */
typedef struct hvxo_stv {
  const uint8_t *const *hist;
  int hist_n, hist_stride[2];
  const float *dirs;
  int dirs_stride;
} hvxo_stv;
int hvxo_hm_replay_picture_stv(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                               const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                               const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                               const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                               int slice_ctus, int rd_metric, double lambda_ssim, const hvxo_stv *stv, int16_t *out_parts,
                               int32_t *out_coef, uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist,
                               uint8_t *out_states, int64_t *out_frac);

/* Independent SliceMode=1 slice chains (slices of slice_ctus CTUs): chain k decides CTUs
 * chain_first[k] .. + ctus_per_chain - 1 from entry_states (the slice-start contexts) and a zero
 * m_integerMv2Nx2N, carrying both CTU to CTU (a chain crossing into the next slice restarts from
 * entry_states there and carries m_integerMv2Nx2N on); the chains run on n_threads threads.  Picture
 * arrays as hvxo_hm_replay_picture; outputs per (chain, CTU) in that order. */
int hvxo_hm_chains(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                   int n_refpics, const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states,
                   int n_chains, const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads,
                   int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist);

int hvxo_hm_chains_rd(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                      int n_refpics, const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states,
                      int n_chains, const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads,
                      int rd_metric, double lambda_ssim, int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon,
                      double *out_cost, uint32_t *out_bits_dist);
int hvxo_hm_chains_stv(const int32_t *pic_i32, const double *pic_f64, const uint8_t *org, const uint8_t *refpics,
                       int n_refpics, const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states,
                       int n_chains, const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads,
                       int rd_metric, double lambda_ssim, const hvxo_stv *stv, int16_t *out_parts, int32_t *out_coef,
                       uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist);

/* The picture-level loop after compressSlice (TEncGOP.cpp:1465-1480) on a decided picture's CTU data
 * (hm_parts = [n_ctus][256][HVXO_HM_PART_FIELDS], the cu_capture.cpp rows):
 * hvxo_hm_boundary_strength: TComLoopFilter::loopFilterPic's per-4x4-unit boundary strengths of the
 *   left (bs_ver) and top (bs_hor) edge, (w/4) x (h/4) raster, 0 off the 8x8 edge grid -- exactly the
 *   m_aapucBS values xEdgeFilterLuma/Chroma read (xDeblockCU :170, xSetLoopfilterParam :362,
 *   xSetEdgefilterTU :274, xSetEdgefilterPU :299, xGetBoundaryStrengthSingle :417), with
 *   LFCrossSliceBoundaryFlag on and the deblocking filter enabled; qp = each unit's QpY (getQP).
 *   ref_poc = the slice's [2][4] reference POCs (reference identity), is_b = B slice.
 * hvxo_hm_col_field: TComPic::compressMotion (TComDataCU::compressMV, TComDataCU.cpp:3320): the
 *   hvx_hm_picture.col_field rows [n_ctus][16][8] the next picture's TMVP reads -- per 16x16 block
 *   its top-left 4x4 unit's {pred mode (-1 outside the picture), ref idx L0, L1, MV L0 x, y, L1 x, y, 0}. */
void hvxo_hm_boundary_strength(int w, int h, const int16_t *hm_parts, const int32_t *ref_poc, int is_b,
                               uint8_t *bs_ver, uint8_t *bs_hor, int8_t *qp);
void hvxo_hm_col_field(int w, int h, const int16_t *hm_parts, int16_t *col_field);

#ifdef __cplusplus
}
#endif
#endif
