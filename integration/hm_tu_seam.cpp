// hm_tu_seam.cpp -- drop-in of the hvx TU kernels under an UNCHANGED HM-16.5rc1 TAppEncoder.
//
// Linked into the reference encoder with
//   -Wl,--wrap=<TComTrQuant::transformNxN> -Wl,--wrap=<TComTrQuant::invTransformNxN>
// every call TEncSearch makes into the reference transform/quant (TEncSearch.cpp:1262,1277,
// 4632,4640,4711 -> TComTrQuant.cpp:1460,1547) is served by libhvx.so on the MI355X through
// the C-ABI (hvx_tu_forward_host / hvx_tu_inverse_host).  The shim snapshots exactly the
// state the reference reads (hvx_tu_desc, estBits, lambda) and reproduces transformNxN's one
// side effect on the CU (the CBF flags, TComTrQuant.cpp:1543).  No HM source is modified;
// a negative ABI status aborts, matching HM's fail-fast convention.
//
// RDPCM (RExt) and non-square TUs (4:2:2) are not on the ported path; such calls fall through
// to the reference implementation (never taken in Main-profile 4:2:0 configs).
#include <sstream>
#include <iostream>
#include <vector>
#include <list>
#include <map>
#include <set>
#include <string>
#include <algorithm>
#include <cassert>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <memory>
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComChromaFormat.h"
#include "hm_access.hpp"
#include "hvx.h"

#define FWD_SYM _ZN11TComTrQuant12transformNxNER6TComTU11ComponentIDPsjPiS4_RiRK7QpParam
#define INV_SYM _ZN11TComTrQuant15invTransformNxNER6TComTU11ComponentIDPsjPiRK7QpParam
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" {
void CAT(__real_, FWD_SYM)(TComTrQuant *, TComTU &, ComponentID, Pel *, UInt, TCoeff *, TCoeff *, TCoeff &, const QpParam &);
void CAT(__real_, INV_SYM)(TComTrQuant *, TComTU &, ComponentID, Pel *, UInt, TCoeff *, const QpParam &);
}

static_assert(sizeof(estBitsSbacStruct) == sizeof(hvx_estbits), "estBits layout");

static hvx_ctx *g_ctx = nullptr;
static long long g_calls = 0;

static hvx_ctx *ctx() {
  if (!g_ctx) {
    int rc = hvx_create(0, &g_ctx);
    if (rc) { fprintf(stderr, "hvx_create failed (%d): %s\n", rc, hvx_last_error()); abort(); }
    atexit([] { fprintf(stderr, "hm_tu_seam: %lld TU calls served by libhvx\n", g_calls); });
  }
  return g_ctx;
}

// the one libhvx context of the process, shared with hm_mc_seam.cpp
hvx_ctx *hvx_seam_ctx() { return ctx(); }

static bool ported(TComTU &rTu, ComponentID compID) {
  TComDataCU *cu = rTu.getCU();
  const UInt idx = rTu.GetAbsPartIdxTU();
  const TComRectangle &r = rTu.getRect(compID);
  const bool rdpcm = cu->isRDPCMEnabled(idx) && (cu->getTransformSkip(idx, compID) || cu->getCUTransquantBypass(idx));
  return !rdpcm && r.width == r.height;
}

static void fill_desc(TComTrQuant *self, TComTU &rTu, ComponentID compID, const QpParam &qp, hvx_tu_desc &d) {
  TComDataCU *cu = rTu.getCU();
  const UInt idx = rTu.GetAbsPartIdxTU();
  const TComRectangle &rect = rTu.getRect(compID);
  const ChannelType ch = toChannelType(compID);
  const TComSlice *sl = cu->getSlice();
  const TComSPS *sps = sl->getSPS();
  memset(&d, 0, sizeof(d));
  d.comp = compID;
  d.width = rect.width;
  d.height = rect.height;
  d.log2_size = rTu.GetEquivalentLog2TrSize(compID);
  d.scan_type = cu->getCoefScanIdx(idx, rect.width, rect.height, compID);
  d.use_dst = rTu.useDST(compID) ? 1 : 0;
  d.transform_skip = cu->getTransformSkip(idx, compID);
  d.is_intra = cu->isIntra(idx) ? 1 : 0;
  d.tr_idx = cu->getTransformIdx(idx);
  d.ctx_qt_cbf = cu->getCtxQtCbf(rTu, ch);
  d.slice_type = sl->getSliceType();
  d.qp_per = qp.per;
  d.qp_rem = qp.rem;
  d.sign_hiding = sl->getPPS()->getSignHideFlag() ? 1 : 0;
  d.use_rdoq = HM(self, TComTrQuant_rdoq);
  d.use_rdoq_ts = HM(self, TComTrQuant_rdoq_ts);
  d.selective_rdoq = HM(self, TComTrQuant_selective_rdoq);
  d.adaptive_qp_select = HM(self, TComTrQuant_adapt_qp);
  d.transquant_bypass = cu->getCUTransquantBypass(idx) ? 1 : 0;
  d.golomb_rice_stat = self->m_pcEstBitsSbac->golombRiceAdaptationStatistics[rTu.getGolombRiceStatisticsIndex(compID)];
  d.persistent_rice = sps->getSpsRangeExtension().getPersistentRiceAdaptationEnabledFlag() ? 1 : 0;
  d.extended_precision = sps->getSpsRangeExtension().getExtendedPrecisionProcessingFlag() ? 1 : 0;
  d.ts_context = sps->getSpsRangeExtension().getTransformSkipContextEnabledFlag() ? 1 : 0;
  d.max_log2_tr_range = sps->getMaxLog2TrDynamicRange(ch);
  d.bit_depth = sps->getBitDepth(ch);
  d.lambda = HM(self, TComTrQuant_lambda);
}

extern "C" void CAT(__wrap_, FWD_SYM)(TComTrQuant *self, TComTU &rTu, ComponentID compID, Pel *res, UInt stride,
                                      TCoeff *coeff, TCoeff *arl, TCoeff &absSum, const QpParam &qp) {
  if (!ported(rTu, compID)) { CAT(__real_, FWD_SYM)(self, rTu, compID, res, stride, coeff, arl, absSum, qp); return; }
  hvx_tu_desc d;
  fill_desc(self, rTu, compID, qp, d);
  const bool rdoq_path = !d.transquant_bypass && (d.transform_skip ? d.use_rdoq_ts : d.use_rdoq);
  int32_t abs_sum = 0;
  int rc = hvx_tu_forward_host(ctx(), &d, (const hvx_estbits *)self->m_pcEstBitsSbac, res, (int)stride, coeff,
                               (d.adaptive_qp_select || rdoq_path) ? arl : nullptr, &abs_sum);
  if (rc) { fprintf(stderr, "hvx_tu_forward_host failed (%d): %s\n", rc, hvx_last_error()); abort(); }
  absSum = abs_sum;
  g_calls++;
  TComDataCU *cu = rTu.getCU();
  cu->setCbfPartRange((((absSum > 0) ? 1 : 0) << rTu.GetTransformDepthRel()), compID, rTu.GetAbsPartIdxTU(),
                      rTu.GetAbsPartIdxNumParts(compID));
}

extern "C" void CAT(__wrap_, INV_SYM)(TComTrQuant *self, TComTU &rTu, ComponentID compID, Pel *res, UInt stride,
                                      TCoeff *coeff, const QpParam &qp) {
  if (!ported(rTu, compID)) { CAT(__real_, INV_SYM)(self, rTu, compID, res, stride, coeff, qp); return; }
  hvx_tu_desc d;
  fill_desc(self, rTu, compID, qp, d);
  int rc = hvx_tu_inverse_host(ctx(), &d, coeff, res, (int)stride);
  if (rc) { fprintf(stderr, "hvx_tu_inverse_host failed (%d): %s\n", rc, hvx_last_error()); abort(); }
  g_calls++;
}
