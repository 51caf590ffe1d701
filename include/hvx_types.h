/* hvx_types.h -- plain-C data structures shared by the hvx C-ABI (hvx.h) and its
 * CPU parity oracle (oracle/hvx_oracle.h).  No torch / HIP types.
 *
 * Every struct below is a snapshot of the HM-16.5rc1 object state that the
 * reference kernel reads at call time ("Threading":
 * lambda, predictor, cost scale, estBits, ... are mutated by the callers, so
 * each batched job carries its own copy).
 */
#ifndef HVX_TYPES_H
#define HVX_TYPES_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Layout-identical to HM's estBitsSbacStruct (hm-16.5rc1 TComTrQuant.h:60-73,
 * context counts from ContextTables.h): the fractional-bit tables (15-bit fixed
 * point) that TEncSbac::estBit (TEncSbac.cpp:1726) derives from the CABAC state. */
typedef struct hvx_estbits {
  int32_t significantCoeffGroupBits[2][2];
  int32_t significantBits[44][2];
  int32_t lastXBits[2][10];
  int32_t lastYBits[2][10];
  int32_t greaterOneBits[24][2];
  int32_t levelAbsBits[6][2];
  int32_t blockCbpBits[10][2];
  int32_t blockRootCbpBits[4][2];
  int32_t golombRiceAdaptationStatistics[4];
} hvx_estbits;

/* One transform unit (TComTU + the TComDataCU/TComSlice/TComTrQuant state the
 * forward/inverse TU path reads: TComTrQuant.cpp:1126-1676, 2129-2671). */
typedef struct hvx_tu_desc {
  int32_t comp;               /* ComponentID: 0 Y, 1 Cb, 2 Cr */
  int32_t width, height;      /* TU rectangle of this component */
  int32_t log2_size;          /* TComTU::GetEquivalentLog2TrSize */
  int32_t scan_type;          /* TComDataCU::getCoefScanIdx: 0 diag, 1 hor, 2 ver */
  int32_t use_dst;            /* TComTU::useDST (4x4 intra luma) */
  int32_t transform_skip;
  int32_t is_intra;
  int32_t tr_idx;             /* TComDataCU::getTransformIdx(absPartIdx) */
  int32_t ctx_qt_cbf;         /* TComDataCU::getCtxQtCbf(rTu, chType) */
  int32_t slice_type;         /* HM SliceType: 0 B, 1 P, 2 I */
  int32_t qp_per, qp_rem;     /* QpParam */
  int32_t sign_hiding;        /* PPS sign_data_hiding */
  int32_t use_rdoq, use_rdoq_ts, selective_rdoq, adaptive_qp_select;
  int32_t transquant_bypass;
  int32_t golomb_rice_stat;   /* estBits->golombRiceAdaptationStatistics[statIdx] */
  int32_t persistent_rice, extended_precision, ts_context;
  int32_t max_log2_tr_range;  /* 15 for 8-bit Main */
  int32_t bit_depth;          /* 8 */
  int32_t pps_tskip;          /* PPS transform_skip_enabled_flag (read by codeCoeffNxN's
                                 codeTransformSkipFlags only; log2MaxTransformSkipBlockSize 2) */
  double lambda;              /* TComTrQuant::m_dLambda after selectLambda(compID) */
} hvx_tu_desc;

/* CABAC context models of HM's TEncSbac (m_contextModels, constructor order TEncSbac.cpp:62-92) */
#define HVX_NUM_CTX 202

/* TEncSbac::codeCoeffNxN (TEncSbac.cpp:1181) counted by TEncBinCABACCounter
 * (TEncBinCoderCABACCounter.cpp:74-120): the rate of one TU's coefficients as the RD search
 * measures it, from the RD coder's context states (which the count also advances). */
typedef struct hvx_coeff_bits {
  uint64_t frac_bits;         /* increase of TEncBinCABACCounter::m_fracBits (15-bit fixed point) */
  uint32_t rice_stat;         /* m_golombRiceAdaptationStatistics[statIdx] after the call */
  uint32_t num_sig;           /* non-zero coefficients (0: the reference's empty-TU exit, nothing coded) */
} hvx_coeff_bits;

/* The registers of the slice writer's arithmetic coder, TEncBinCABAC (TEncBinCoderCABAC.h):
 * m_uiLow, m_uiRange, m_bitsLeft, m_numBufferedBytes, m_bufferedByte.  TEncBinCABAC::start()
 * is {0, 510, 23, 0, 0xff}.  bins counts the bins coded (context, bypass), as m_uiBinsCoded
 * does with m_binCountIncrement 1; the writer adds to it.  coded: bit (m - 42) of the 160-bit map
 * is set for every context model m (42..184, the residual syntax) the writer codes a bin with --
 * ContextModel::setBinsCoded(1) in encodeBin (TEncBinCoderCABAC.cpp:203), which
 * ContextModel3DBuffer::calcCost reads for the cabac_init_flag choice; OR-accumulated. */
typedef struct hvx_cabac_regs {
  uint32_t low, range;
  int32_t bits_left, num_buffered;
  uint32_t buffered_byte, bins;
  uint32_t coded[5];
} hvx_cabac_regs;

/* One uni-prediction motion search: TEncSearch::xMotionEstimation with bBi=false
 * (TEncSearch.cpp:3663-3760): TZ integer search + half/quarter refinement. */
typedef struct hvx_me_job {
  int32_t pic_w, pic_h;       /* SPS picture size in luma samples (clipMv, TComDataCU.cpp:2788) */
  int32_t max_cu;             /* SPS max CU width/height (64) */
  int32_t cu_x, cu_y;         /* TComDataCU::m_uiCUPelX/Y of the CU owning the PU */
  int32_t pu_x, pu_y, w, h;   /* PU rectangle in luma samples */
  int32_t pred_x, pred_y;     /* AMVP predictor (quarter-pel) */
  int32_t use_int2nx2n;       /* pIntegerMv2Nx2NPred != 0 (TEncSearch.cpp:3734) */
  int32_t i2_x, i2_y;         /* m_integerMv2Nx2N[list][ref] (integer-pel) */
  int32_t bits_in;            /* ruiBits on entry */
  int32_t search_range;       /* m_iSearchRange (SearchRange cfg) */
  uint32_t lambda_motion;     /* TComRdCost m_uiLambdaMotionSAD[0] = floor(65536*sqrt(lambda)) */
  int32_t flags;              /* HVX_ME_* below */
  int32_t ref_idx;            /* index into the reference-plane array of a batch */
  int32_t cur_idx;            /* index into the current-plane array of a batch */
  int32_t center_x, center_y; /* hvx_me_full_batch: xSetSearchRange centre (quarter-pel) -- the
                                 predictor (FastSearch=0) or the list's current MV rcMv (bBi) */
  int32_t pad_;
} hvx_me_job;

#define HVX_ME_FEN        1   /* FEN: subsampled SAD when rows > 8 (TEncSearch.cpp:346) */
#define HVX_ME_HADME      2   /* HadamardME: SATD in fractional refinement */
#define HVX_ME_SMOOTHMV   4   /* FastMEAssumingSmootherMV: stop first search after 3 rounds */
#define HVX_ME_BI         8   /* bi-prediction refinement (bBi): final cost weight 0.5 (TEncSearch.cpp:3759) */

typedef struct hvx_me_result {
  int32_t mv_int_x, mv_int_y; /* integer-pel TZ result */
  uint32_t sad_int;           /* ruiSAD after xTZSearch (SAD without MV cost) */
  int32_t half_x, half_y;     /* cMvHalf */
  int32_t qtr_x, qtr_y;       /* cMvQter */
  uint32_t cost_frac;         /* ruiCost after xPatternSearchFracDIF */
  int32_t mv_x, mv_y;         /* final quarter-pel MV */
  uint32_t bits;              /* ruiBits on exit */
  uint32_t cost;              /* ruiCost on exit */
} hvx_me_result;

/* CU-level distortion of the HM engine's mode / split comparisons (hvx_hm_picture.rd_metric):
 * HVX_RD_SSE = HM's calcRdCost(bits, SSE); HVX_RD_SSIM = the stvssim encoder's distortionSSIM cost,
 * HVX_RD_STVSSIM = its active distortionstVSSIM cost (BASELINE config 4; see
 * hvx_hm_picture). */
#define HVX_RD_SSE 0
#define HVX_RD_SSIM 1
#define HVX_RD_STVSSIM 2
/* HVX_RD_STVSSIM: the most previous pictures of the stVSSIM history (REFNUM 26 - 1, att_stv.h) */
#define HVX_STV_HIST 25

/* One intra block: TComPrediction::initIntraPatternChType's reference
 * samples (TComPattern.cpp:115-360: fillReferenceSamples :364 substitution + the [1 2 1] /
 * strong bilinear smoothing), predIntraAng (TComPrediction.cpp:455: planar :756, DC :183 +
 * xDCPredFiltering :816, angular xPredIntraAng :247 with its edge filters), and
 * TEncSearch::estIntraPredLumaQT's first pass (TEncSearch.cpp:2244-2323: Hadamard SATD of all 35
 * modes + xModeBitsIntra :5222 rate, sqrt-lambda cost, xUpdateCandList :5254, MPM append).
 * The block is square, size 1 << log2_size, at (x, y) of an 8-bit padded plane; 8-bit video. */
#define HVX_INTRA_STRONG   1   /* SPS strong_intra_smoothing_enabled_flag (luma 32x32) */
#define HVX_INTRA_FAST_MPM 2   /* FastUDIUseMPM: g_aucIntraModeNumFast_UseMPM + MPM append */
typedef struct hvx_intra_job {
  int32_t x, y;              /* block origin in its plane, samples */
  int32_t log2_size;         /* 2..6 luma, 2..5 chroma */
  int32_t ch_type;           /* 0 luma, 1 chroma (4:2:0: no reference smoothing, no edge/DC filters) */
  int32_t unit_log2;         /* neighbour unit in samples (minimum CU/TU grid): 2 luma, 1 chroma 4:2:0 */
  uint32_t avail[3];         /* bNeighborFlags (TComPattern.cpp:140-147), bit i = unit i: 0..L-1 the left and
                                below-left units bottom-up (L = 2*size >> unit_log2), L the above-left unit,
                                L+1..2L the above and above-right units left to right */
  int32_t mode;              /* hvx_intra_pred_batch: 0 planar, 1 DC, 2..34 angular */
  int32_t flags;             /* HVX_INTRA_STRONG | HVX_INTRA_FAST_MPM */
  int32_t left_dir, above_dir; /* first pass: the intra dirs TComDataCU::getIntraDirPredictor reads
                                  (TComDataCU.cpp:1413-1428; DC = 1 when unavailable / not intra) */
  int32_t ctx_state;         /* first pass: m_ucState of prev_intra_luma_pred_flag's context */
  int32_t frac_bits;         /* first pass: m_fracBits & 32767 of the bin counter of the coder xModeBitsIntra
                                loads from (m_pppcRDSbacCoder[depth][CI_CURR_BEST]): loadIntraDirMode copies
                                it (TEncSbac.cpp:403) and resetBits keeps those bits (TEncBinCoderCABAC.cpp:172) */
  double sqrt_lambda;        /* first pass: TComRdCost::getSqrtLambda */
} hvx_intra_job;

/* First-pass result of one intra PU (estIntraPredLumaQT's uiRdModeList / CandCostList). */
typedef struct hvx_intra_search_result {
  double cand_cost[8];       /* CandCostList[0..num_rd), ascending */
  uint32_t satd[35];         /* Hadamard SATD of each mode's prediction against the original */
  uint8_t mode_bits[35];     /* xModeBitsIntra of each mode */
  uint8_t num_rd;            /* numModesForFullRD before the MPM append */
  uint8_t n_cand;            /* candidates after the MPM append (<= 11) */
  uint8_t cand[11];          /* uiRdModeList */
  uint8_t pad_[4];
} hvx_intra_search_result;

/* Deblocking of a reconstructed picture (TComLoopFilter::loopFilterPic,
 * TComLoopFilter.cpp:130): all vertical edges, then all horizontal edges, on the 8x8 grid (luma)
 * and the 16x16-luma grid (4:2:0 chroma, bs 2 only).  Edge inputs are per 4x4 luma unit,
 * raster over (pic_w/4) x (pic_h/4): bs_ver = boundary strength 0..2 of the unit's LEFT edge (read
 * where x % 8 == 0), bs_hor = of its TOP edge (read where y % 8 == 0) -- xGetBoundaryStrengthSingle
 * (:417) values, 0 where no TU/PU edge or at the picture border; qp = the unit's QpY
 * (TComDataCU::getQP).  8-bit video, no PCM / transquant-bypass units. */
typedef struct hvx_deblock_params {
  int32_t pic_w, pic_h;            /* luma samples, multiples of 8 */
  int32_t beta_offset_div2, tc_offset_div2;  /* slice_beta_offset_div2, slice_tc_offset_div2 */
  int32_t cb_qp_offset, cr_qp_offset;        /* pps_cb_qp_offset, pps_cr_qp_offset */
  int32_t flags, pad_;             /* reserved, 0 */
} hvx_deblock_params;

/* SAO parameters of one CTU component as offsetCTU applies them (TComSampleAdaptiveOffset.cpp:554:
 * the decided parameters with merges resolved and offsets de-quantised, reconstructBlkSAOParam
 * :248).  type: -1 off, 0..3 edge offset EO_0 / EO_90 / EO_135 / EO_45, 4 band offset.
 * EO: offset[] = full valley, half valley, half peak, full peak (the plain class adds 0).
 * BO: band = first of the 4 consecutive bands (mod 32) whose offsets are offset[0..3]. */
#define HVX_SAO_OFF (-1)
#define HVX_SAO_BO 4
typedef struct hvx_sao_offset {
  int8_t type;
  uint8_t band;
  int8_t offset[4];
  int8_t pad_[2];
} hvx_sao_offset;                  /* 8 bytes */
typedef struct hvx_sao_ctu {
  hvx_sao_offset comp[3];          /* Y, Cb, Cr */
} hvx_sao_ctu;                     /* 24 bytes, one per CTU in raster order */

/* SAO statistics of one CTU component and type (SAOStatData, TEncSampleAdaptiveOffset.h:66):
 * EO: classes 0..4 (edge type + 2); BO: the 32 bands. */
#define HVX_SAO_TYPES 5
#define HVX_SAO_CLASSES 32
typedef struct hvx_sao_stat {
  int64_t diff[HVX_SAO_CLASSES];   /* sum of org - rec */
  int64_t count[HVX_SAO_CLASSES];
} hvx_sao_stat;                    /* 512 bytes; a picture: [ctu][comp 3][type 5] */

/* One picture's SAO RD decision (hvx_sao_decide: TEncSampleAdaptiveOffset::decideBlkParams,
 * TEncSampleAdaptiveOffset.cpp:763), 8-bit 4:2:0, one tile.  Device pointers; the job array itself
 * is on the device. */
typedef struct hvx_sao_decide_job {
  int32_t pic_w, pic_h;
  int32_t slice_ctus;              /* CTUs per slice (SliceMode 1), 0: one slice -- merges stay in a slice */
  int32_t test_off;                /* bTestSAODisableAtPictureLevel */
  int32_t slice_enabled[3];        /* decidePicParams' flags Y, Cb, Cr (host: the SAO-off rates of earlier pictures) */
  int32_t frac_lo;                 /* low 15 bits of the picture-start RD coder's fractional bit count */
  uint8_t sao_states[2];           /* its sao_merge_left/up_flag and sao_type_idx context states (m_ucState) */
  uint8_t pad_[6];
  double lambda[3];                /* SAOProcess's lambdas */
  const hvx_sao_stat *stats;       /* [ctu][3][5] statistics (hvx_sao_stats) */
  const int32_t *entropy_bits;     /* ContextModel::m_entropyBits[128] */
  int32_t *coded;                  /* out [ctu][3][8]: mode (0 off, 1 new, 2 merge), type (EO 0-3 / BO 4, or merge
                                      0 left / 1 above), band position, offsets of EO classes 0..4 / of the 4 bands */
  hvx_sao_ctu *recon;              /* out [ctu]: the parameters offsetCTU applies (merges resolved) */
  int32_t *slice_enabled_out;      /* out [3]: cleared when the picture-level test disables SAO */
  double *total_cost;              /* out: decideBlkParams' total cost */
} hvx_sao_decide_job;

/* One PU's motion compensation (TComPrediction::motionCompensation for one partition, no
 * weighted prediction; TComPrediction.cpp:517-722).  Lists with ref >= 0 are used: both ->
 * bi-prediction (14-bit intermediates + TComYuv::addAvg), unless HVX_MC_B_SLICE is set and the
 * two lists carry identical motion (same POC and MV: xCheckIdenticalMotion :500), which
 * predicts from list 0 alone; one -> uni-prediction from that list.  MVs are clipped here as
 * xPredInterUni does (TComDataCU::clipMv).  4:2:0, 8-bit. */
#define HVX_MC_B_SLICE 1
typedef struct hvx_mc_job {
  int32_t pic_w, pic_h, max_cu;  /* clipMv */
  int32_t cu_x, cu_y;            /* CU origin, luma samples (clipMv) */
  int32_t pu_x, pu_y, w, h;      /* PU, luma samples */
  int32_t ref[2];                /* per list: reference picture index into the plane table, -1 = unused */
  int32_t poc[2];                /* per list: the reference's POC (identical-motion check) */
  int32_t mv_x[2], mv_y[2];      /* per list: quarter-pel MV before clipMv */
  int32_t flags;                 /* HVX_MC_B_SLICE */
  int64_t dst_offset;            /* element offset of the output: Y w*h, Cb, Cr (w/2)*(h/2) each */
} hvx_mc_job;


/* ---------------------------------------------------------------------------------------
 * HM-exact CTU decision (hvx_hm_compress; TEncCu::compressCtu TEncCu.cpp:228 + the CTU syntax
 * walk TEncCu::encodeCtu :252 that carries the CABAC contexts to the next CTU,
 * TEncSlice.cpp:814-828).  4:2:0 8-bit, the encoder_lowdelay_P_main.cfg / encoder_randomaccess_main.cfg
 * tool set (see hvx.h): I, P and B slices.
 * ------------------------------------------------------------------------------------- */
/* An RD coder of TEncCu: TEncSbac's 202 context states (m_ucState) + TEncBinCABACCounter::m_fracBits
 * (TEncSbac::load/store copy both, TEncSbac.cpp:396-425). */
typedef struct hvx_hm_coder {
  uint8_t st[202];
  uint8_t pad_[6];
  uint64_t frac;
} hvx_hm_coder;

/* The per-partition fields of TComDataCU (TComDataCU.h) for one 4x4 partition (z-order). */
typedef struct hvx_hm_part {
  int8_t depth, part, pred, skip, merge, merge_idx, inter_dir, tr_idx;  /* part: PartSize, pred: PredMode */
  int8_t ref[2], mvp_idx[2], mvp_num[2];                                 /* per list */
  int16_t mv[2][2], mvd[2][2];                                           /* per list (x, y), quarter-pel */
  uint8_t idir[2];                                                       /* intra dir luma / chroma (36 = DM) */
  uint8_t ts[3], cbf[3];                                                 /* transform skip, cbf (bit = TU depth) */
  uint8_t width;
  int8_t qp;
} hvx_hm_part;

/* The final data of one CTU (TComPic::getCtu(addr)): partitions in z-order and the coefficients
 * (m_pcTrCoeff: luma 64x64 then Cb, Cr 32x32, in the CU/TU z-order packing of TComDataCU). */
typedef struct hvx_hm_ctu {
  hvx_hm_part p[256];
  int16_t coef[6144];
  uint32_t bits, dist;       /* TComDataCU::getTotalBits / getTotalDistortion of the CTU */
  double cost;               /* getTotalCost */
} hvx_hm_ctu;

/* One picture as the decision reads it (TComSlice / TComRdCost / TComTrQuant state + planes).
 * All pointers are device pointers to sample (0,0).  org: 8-bit planes (strides org_stride[0]
 * luma, [1] chroma).  rec: the picture reconstruction (TComPic::getPicYuvRec before the loop
 * filters; read for intra neighbours outside the CTU being decided, written by chained jobs).
 * ref8[i]: luma of reference plane i, 8-bit with HVX_PLANE_MARGIN on every side (stride
 * ref8_stride, a multiple of 4, >= w + 2*margin); ref16[i][c]: the same picture as int16 planes
 * with margins >= 80 (luma) / 40 (chroma) (strides ref16_stride[0/1]).  ctus: the picture's CTU
 * array (neighbours of the CTU being decided; chained jobs write each CTU they finish).
 * col_field: the collocated picture's compressed motion, [ctu][16 blocks of 16x16][8] =
 * {pred mode (-1 outside), ref0, ref1, mv0x, mv0y, mv1x, mv1y, 0}. */
typedef struct hvx_hm_picture {
  int32_t w, h, w_ctus, h_ctus, poc, slice_type, qp;
  int32_t nref[2], ref_poc[2][4], ref_plane[2][4];   /* ref_plane: index into ref8 / ref16 */
  int32_t chroma_qp[2];
  int32_t max_merge, tmvp, check_ldc, col_from_l0, col_valid, col_poc;
  int32_t col_ref_poc[2][4];
  int32_t search_range, amp;
  uint32_t lambda_motion;    /* m_uiLambdaMotionSAD[0] */
  int32_t bipred_range;      /* BipredSearchRange (TEncSearch::m_bipredSearchRange, B slices) */
  double lambda, sqrt_lambda, chroma_weight[2], tq_lambda[3];
  const int16_t *col_field;
  const uint8_t *org[3];
  uint8_t *rec[3];
  int32_t org_stride[2], rec_stride[2];
  hvx_hm_ctu *ctus;
  const uint8_t *ref8[8];
  const int16_t *ref16[8][3];
  int32_t ref8_stride, ref16_stride[2];
  int32_t mvd_l1_zero;       /* TComSlice::getMvdL1ZeroFlag: L1 = L0 entry by entry (TEncGOP.cpp:1311-1336) */
  int32_t l1_to_l0[4];       /* TComSlice::getList1IdxToList0Idx (TComSlice.cpp:302), -1: not in L0 */
  const int32_t *entropy_bits;  /* ContextModel::m_entropyBits[128] */
  /* The cost TEncCu's comparisons use (xCheckBestMode TEncCu.cpp:1444 and the split cost):
   * HVX_RD_SSE = HM's calcRdCost(bits, SSE); HVX_RD_SSIM = the stvssim encoder's SSIM cost
   * J = D + lambda_ssim * max(0.5, bits) (rdopt.c:1631), D = sum over the CU's 8x8 luma / 4x4 chroma
   * blocks of (1 - SSIM) / 4 (compute_SSIM stvssim.c:491, one window per block), lambda_ssim =
   * lambda_2(QP) * eta^0.85 (stvssim.c:1805, :1707) computed by the caller.  The searches, merge
   * estimation, RQT and RDOQ keep HM's SSE / SATD costs in both. */
  int32_t rd_metric, pad3_;
  double lambda_ssim;
  /* HVX_RD_STVSSIM (distortionstVSSIM, stvssim.c:831-855, active by att_stv.h:5 / rdopt.c:223):
   * D of a CU = the sum over its 16x16 luma areas (one JM macroblock each, raster order) of
   * (1 - stVSSIM_Y) + (1 - stVSSIM_Cb) + (1 - stVSSIM_Cr) (WeightY/Cb/Cr 1, encoder.cfg:289-291),
   * compute_stVSSIM (:587) over the area's 16x16 luma (8x8 windows stepped by SSIMOverlapSize 4,
   * encoder.cfg:280) and 8x8 Cb, Cr blocks; an 8x8 CU is one 8x8 luma window + 4x4 chroma windows,
   * weighted 1/4.  The 3-D terms read the co-located samples of hist_n (<= HVX_STV_HIST) previous
   * pictures in coding order, most recent first (storeRefAndEncFrames :362, img->number + 1 frames
   * with the current one): hist[6k + c] = picture k's original component c, hist[6k + 3 + c] = its
   * final reconstruction, 8-bit, strides hist_stride[0] (luma) / [1] (chroma) -- Cr's history is read
   * from the Cb planes, as compute_stVSSIM is called with comp 1 for both chroma components (:846,
   * :850).  dirs: the direction map (pic_directions2: orientation in radians, one float per 4x4
   * luma block, dirs_stride floats per row of blocks; getDirection_macroblock :1369).
   * stv_sums (optional, hvx_hm_stv_prepare): the history frames' part of every window's five
   * directional sums, so a window adds only the current picture's samples (the same float sequence). */
  const uint8_t *const *hist;
  const float *dirs;
  const float *stv_sums;
  int32_t hist_n, dirs_stride, hist_stride[2];
} hvx_hm_picture;

/* One chain of CTUs decided in raster order by one wave: CTUs first_ctu .. first_ctu+n_ctus-1 of
 * picture pic, the first from `entry` (m_pppcRDSbacCoder[0][CI_CURR_BEST] on entry) and
 * int2n (TEncSearch::m_integerMv2Nx2N [2][4][2]), each later one from the previous CTU's
 * encodeCtu state and search state.  Neighbours outside [slice_start, slice_end] are unavailable
 * (TComDataCU::getPU* with the slice restriction; SliceMode=1 slices of whole CTUs), and the
 * slice's last CTU ends without the end_of_slice_segment_flag bin.  chained = 1: every finished CTU is written into the
 * picture (ctus[addr] and rec) before the next starts; 0: the picture is only read (n_ctus = 1,
 * independent CTUs against a fixed neighbourhood).  Outputs go to slot out + k of the output
 * arrays for the k-th CTU of the chain. */
typedef struct hvx_hm_job {
  int32_t pic, first_ctu, n_ctus, chained, out;
  int32_t slice_start, slice_end;  /* the slice holding the chain: first / last CTU address (raster) */
  int32_t flags;                   /* HVX_HM_RESUME; bits 8..15: 0 (debugging builds: stop stage) */
  hvx_hm_coder entry;
  int16_t int2n[16];
} hvx_hm_job;
/* hvx_hm_job.flags: continue the chain of the previous launch with the same job index -- the entry
 * coder and m_integerMv2Nx2N come from that job's state (d_state), not from entry / int2n */
#define HVX_HM_RESUME 1
/* hvx_hm_job.flags bits 16..30: SliceMode=1 slices of that many CTUs (0: one slice, [slice_start,
 * slice_end]).  The chain may then run over consecutive slices: each slice's first CTU starts from
 * `entry` (the slice-start context states) and ends its predecessor without the end-of-slice bin,
 * while m_integerMv2Nx2N carries from CTU to CTU across the slice boundary, as in TAppEncoder --
 * where a slice whose first CTU is a picture-boundary CTU (the partial bottom row) reads it. */
#define HVX_HM_SLICE_CTUS(n) ((int32_t)(n) << 16)

/* One slice's data written by hvx_hm_write_slices (TEncSlice::encodeSlice, TEncSlice.cpp:920): CTUs
 * first_ctu .. first_ctu + n_ctus - 1 (raster) of picture pic, whose ctus array holds the decided
 * CTUs (hvx_hm_compress chained jobs, or a caller's TComDataCU data); each CTU's SAO syntax when
 * sao_enabled (the slice's sao flags Y / Cb / Cr) from sao_coded ([ctu][3][8] of the picture, the
 * layout of hvx_sao_decide_job.coded), then its CU syntax, from the slice-start context states
 * `entry` (resetEntropy).  The completed bytes go to out (at most out_cap). */
typedef struct hvx_hm_slice {
  int32_t pic, first_ctu, n_ctus, out_cap;
  int32_t sao_enabled[3], pad_;
  const int32_t *sao_coded;
  uint8_t *out;
  hvx_hm_coder entry;
} hvx_hm_slice;
/* The writer's state after the slice's last CTU (before its terminating end_of_slice_segment_flag 1
 * and TEncBinCABAC::finish, which the caller codes from these registers): TEncBinCABAC's m_uiLow,
 * m_uiRange, m_bitsLeft, m_numBufferedBytes, m_bufferedByte, m_uiBinsCoded; the bytes written
 * (n_bytes > out_cap: the output was truncated at out_cap); status 0, or -HVX_HM_BAD_* (nothing
 * written); the context states after the slice and the models it coded (bit m % 32 of word m / 32). */
typedef struct hvx_hm_slice_result {
  uint32_t low, range;
  int32_t bits_left, num_buffered;
  uint32_t buffered_byte, bins;
  int32_t n_bytes, status;
  uint32_t coded[7], pad_;
  uint8_t states[208];
} hvx_hm_slice_result;
#define HVX_HM_SLICE_CTUS_OF(flags) (((flags) >> 16) & 0x7fff)

#ifdef __cplusplus
}
#endif
#endif
