// hm_access.hpp -- the HM-16.5rc1 members the seams read and write that HM keeps private or
// protected, reached without editing HM's headers and without redefining access keywords.
//
// A pointer to member is formed inside an explicit template instantiation, where access checking
// does not apply to the template arguments ([temp.spec]/6 in C++17), and handed out through a
// friend function the instantiation defines.  Each HM_ACCESS line names one member; a seam uses it
// as  HM(obj_ptr, Tag)  (an lvalue: read or assign).  Everything reachable through HM's public
// getters (TComDataCU's per-partition arrays, the totals, ContextModel's state / MPS, ...) is used
// through those instead.
#pragma once
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/ContextModel.h"
#include "TLibCommon/TComLoopFilter.h"
#include "TLibCommon/TComMotionInfo.h"
#include "TLibCommon/TComPrediction.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#include "TLibEncoder/TEncCu.h"
#include "TLibEncoder/TEncSampleAdaptiveOffset.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncSlice.h"

template <class T> using hm_type = T;
template <class Tag, typename Tag::type M> struct HmAccess {
  friend constexpr typename Tag::type hm_member(Tag) { return M; }
};
#define HM_ACCESS(TAG, CLASS, TYPE, MEMBER)                                     \
  struct TAG {                                                                  \
    typedef hm_type<TYPE> CLASS::*type;                                         \
    friend constexpr type hm_member(TAG);                                       \
  };                                                                            \
  template struct HmAccess<TAG, &CLASS::MEMBER>
#define HM(PTR, TAG) ((PTR)->*hm_member(TAG()))

// the encoder objects TEncCu / TEncSlice hold
HM_ACCESS(TEncCu_cfg, TEncCu, TEncCfg *, m_pcEncCfg);
HM_ACCESS(TEncCu_search, TEncCu, TEncSearch *, m_pcPredSearch);
HM_ACCESS(TEncCu_rdcost, TEncCu, TComRdCost *, m_pcRdCost);
HM_ACCESS(TEncCu_trquant, TEncCu, TComTrQuant *, m_pcTrQuant);
HM_ACCESS(TEncCu_rdcoders, TEncCu, TEncSbac ***, m_pppcRDSbacCoder);
HM_ACCESS(TEncSlice_cfg, TEncSlice, TEncCfg *, m_pcCfg);
HM_ACCESS(TEncSlice_sbac, TEncSlice, TEncSbac *, m_pcSbacCoder);
HM_ACCESS(TEncSlice_cabac, TEncSlice, TEncBinCABAC *, m_pcBinCABAC);
HM_ACCESS(TEncSlice_entropy, TEncSlice, TEncEntropy *, m_pcEntropyCoder);
HM_ACCESS(TEncSlice_trquant, TEncSlice, TComTrQuant *, m_pcTrQuant);
HM_ACCESS(TEncSlice_cabac_idx, TEncSlice, SliceType, m_encCABACTableIdx);
// TEncSearch's search state
HM_ACCESS(TEncSearch_bipred_range, TEncSearch, Int, m_bipredSearchRange);
HM_ACCESS(TEncSearch_int2n, TEncSearch, TComMv[NUM_REF_PIC_LIST_01][MAX_NUM_REF], m_integerMv2Nx2N);
// the RD scalars
HM_ACCESS(TComRdCost_lambda_motion_sad, TComRdCost, UInt[2], m_uiLambdaMotionSAD);
HM_ACCESS(TComRdCost_sqrt_lambda, TComRdCost, Double, m_sqrtLambda);
HM_ACCESS(TComRdCost_dist_weight, TComRdCost, Double[MAX_NUM_COMPONENT], m_distortionWeight);
HM_ACCESS(TComTrQuant_lambdas, TComTrQuant, Double[MAX_NUM_COMPONENT], m_lambdas);
// the CABAC coders
HM_ACCESS(TEncSbac_models, TEncSbac, ContextModel[MAX_NUM_CTX_MOD], m_contextModels);
HM_ACCESS(TEncSbac_n_models, TEncSbac, Int, m_numContextModels);
HM_ACCESS(TEncSbac_bin, TEncSbac, TEncBinIf *, m_pcBinIf);
HM_ACCESS(TEncBinCABAC_low, TEncBinCABAC, UInt, m_uiLow);
HM_ACCESS(TEncBinCABAC_range, TEncBinCABAC, UInt, m_uiRange);
HM_ACCESS(TEncBinCABAC_buffered_byte, TEncBinCABAC, UInt, m_bufferedByte);
HM_ACCESS(TEncBinCABAC_n_buffered, TEncBinCABAC, Int, m_numBufferedBytes);
HM_ACCESS(TEncBinCABAC_bits_left, TEncBinCABAC, Int, m_bitsLeft);
HM_ACCESS(TEncBinCABAC_bins, TEncBinCABAC, UInt, m_uiBinsCoded);
HM_ACCESS(TEncBinCABAC_bin_inc, TEncBinCABAC, Int, m_binCountIncrement);
HM_ACCESS(TEncBinCABAC_frac, TEncBinCABAC, UInt64, m_fracBits);
HM_ACCESS(TEncBinCABAC_bitif, TEncBinCABAC, TComBitIf *, m_pcTComBitIf);
// TComCUMvField's reference indices (no per-partition setter)
HM_ACCESS(TComCUMvField_ref_idx, TComCUMvField, Char *, m_piRefIdx);
// TComTrQuant's RDOQ configuration and current lambda (hm_tu_seam.cpp)
HM_ACCESS(TComTrQuant_lambda, TComTrQuant, Double, m_dLambda);
HM_ACCESS(TComTrQuant_rdoq, TComTrQuant, Bool, m_useRDOQ);
HM_ACCESS(TComTrQuant_rdoq_ts, TComTrQuant, Bool, m_useRDOQTS);
HM_ACCESS(TComTrQuant_selective_rdoq, TComTrQuant, Bool, m_useSelectiveRDOQ);
HM_ACCESS(TComTrQuant_adapt_qp, TComTrQuant, Bool, m_bUseAdaptQpSelect);
// the intra border TComPrediction built (hm_intra_seam.cpp)
HM_ACCESS(TComPrediction_yuv_ext, TComPrediction, Pel *[MAX_NUM_COMPONENT][NUM_PRED_BUF], m_piYuvExt);
// TComLoopFilter's boundary-strength derivation, run on a private filter object (hm_lf_seam.cpp)
HM_ACCESS(TComLoopFilter_n_parts, TComLoopFilter, UInt, m_uiNumPartitions);
HM_ACCESS(TComLoopFilter_bs, TComLoopFilter, UChar *[NUM_EDGE_DIR], m_aapucBS);
HM_ACCESS(TComLoopFilter_edge, TComLoopFilter, Bool *[NUM_EDGE_DIR], m_aapbEdgeFilter);
HM_ACCESS(TComLoopFilter_cross_tile, TComLoopFilter, Bool, m_bLFCrossTileBoundary);
HM_ACCESS(TComLoopFilter_set_param, TComLoopFilter, Void(TComDataCU *, UInt), xSetLoopfilterParam);
HM_ACCESS(TComLoopFilter_set_tu, TComLoopFilter, Void(TComTU &), xSetEdgefilterTU);
HM_ACCESS(TComLoopFilter_set_pu, TComLoopFilter, Void(TComDataCU *, UInt), xSetEdgefilterPU);
HM_ACCESS(TComLoopFilter_bs_single, TComLoopFilter, Void(TComDataCU *, DeblockEdgeDir, UInt), xGetBoundaryStrengthSingle);
// SAOProcess's steps (hm_sao_seam.cpp)
HM_ACCESS(TEncSao_stat, TEncSampleAdaptiveOffset, SAOStatData ***, m_statData);
HM_ACCESS(TEncSao_lambda, TEncSampleAdaptiveOffset, Double[MAX_NUM_COMPONENT], m_lambda);
HM_ACCESS(TEncSao_decide_pic, TEncSampleAdaptiveOffset, Void(Bool *, Int, const Double, const Double), decidePicParams);
HM_ACCESS(TEncSao_decide_blk, TEncSampleAdaptiveOffset,
          Void(TComPic *, Bool *, SAOStatData ***, TComPicYuv *, TComPicYuv *, SAOBlkParam *, SAOBlkParam *, const Bool,
               const Double, const Double),
          decideBlkParams);
HM_ACCESS(TComSao_temp_yuv, TComSampleAdaptiveOffset, TComPicYuv *, m_tempPicYuv);
HM_ACCESS(TComSao_width, TComSampleAdaptiveOffset, Int, m_picWidth);
HM_ACCESS(TComSao_height, TComSampleAdaptiveOffset, Int, m_picHeight);
HM_ACCESS(TComSao_ctu_w, TComSampleAdaptiveOffset, Int, m_maxCUWidth);
HM_ACCESS(TComSao_ctu_h, TComSampleAdaptiveOffset, Int, m_maxCUHeight);
HM_ACCESS(TComSao_n_ctus, TComSampleAdaptiveOffset, Int, m_numCTUsPic);

// a context model's state byte (m_ucState = state << 1 | MPS) through its public accessors
inline UChar hm_ctx_state(ContextModel &m) { return (UChar)((m.getState() << 1) | m.getMps()); }
inline void hm_set_ctx_state(ContextModel &m, UChar s) { m.setStateAndMps(s >> 1, s & 1); }
