// hm_me_seam.cpp -- drop-in of the hvx motion search under an UNCHANGED HM-16.5rc1 TAppEncoder.
//
// Replaces TEncSearch::xMotionEstimation (TEncSearch.cpp:3663-3760): every (PU, list, ref)
// search predInterSearch makes (TEncSearch.cpp:3105, 3256 uni-pred; 3259 bi-pred
// refinement) is served by libhvx.so on the MI355X through the C-ABI:
//   - FastSearch=1 (TZ, the LDP/LDB/RA configs): hvx_me_batch -- xTZSearch (:3881) +
//     xPatternSearchFracDIF (:4240) with the job's own snapshot of the search state;
//   - FastSearch=0 or bBi (bi-pred refinement over BipredSearchRange around rcMv):
//     hvx_me_full_batch -- xPatternSearch (:3786) + xPatternSearchFracDIF on the int16
//     target (the removeHighFreq pattern for bBi, TComYuv.cpp:409).
//
// xMotionEstimation and its caller predInterSearch live in the same translation unit, so
// the linker's --wrap cannot reach it.  The seam build instead takes the reference's own
// TEncSearch object, marks its xMotionEstimation WEAK and adds a __real_ alias at the same
// address (objcopy, oracle/Makefile target _ref/TEncSearch_meseam.o); the strong definition
// below then wins every call.  Nothing in the reference source changes.
//
// The shim snapshots what the reference reads (search range incl. the adaptive range,
// predictor, 2Nx2N integer predictor, lambda, FEN/HADME/smooth-MV switches), runs one job
// and reproduces the reference's side effects: m_iSearchRange, m_integerMv2Nx2N, the bBi
// target in m_cYuvPredTemp and the TComRdCost state (cost scale 0, predictor, motion cost).
// Weighted prediction, lossless CUs, non-8-bit video and FastSearch=2 (selective) are not on
// the ported path and fall through to the reference implementation.
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
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComPicYuv.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComYuv.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncCfg.h"
#include "hm_access.hpp"
#include "hvx.h"

#define ME_SYM _ZN10TEncSearch17xMotionEstimationEP10TComDataCUP7TComYuvi10RefPicListP6TComMviRS5_RjS8_b
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

// the reference implementation, kept reachable under an alias by the objcopy step
extern "C" void CAT(__real_, ME_SYM)(TEncSearch *, TComDataCU *, TComYuv *, Int, RefPicList, TComMv *, Int, TComMv &,
                                     UInt &, Distortion &, Bool);

hvx_ctx *hvx_seam_ctx();  // shared with hm_tu_seam.cpp / hm_mc_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

struct DevRef {  // 8-bit padded luma plane of one reference picture (HVX_PLANE_MARGIN = HM's 80)
  const TComPicYuv *pic = nullptr;
  Int poc = -1 << 30;
  void *plane = nullptr;     // start of the padded allocation
  const uint8_t *org = nullptr;
};

struct MeSeam {
  std::vector<DevRef> refs;
  void *d_pel = nullptr;     // int16 staging of one HM plane (for hvx_plane_from_pel)
  size_t pel_bytes = 0;
  void *d_cur = nullptr, *d_tgt = nullptr, *d_ptrs = nullptr, *d_job = nullptr, *d_res = nullptr;
  std::vector<uint8_t> h_cur;
  std::vector<int16_t> h_tgt;
  long long uni = 0, bi = 0, full = 0, fallback = 0;
  ~MeSeam() {
    fprintf(stderr, "hm_me_seam: %lld xMotionEstimation calls served by libhvx (%lld TZ, %lld full search, %lld bi-pred "
                    "refinement), %lld fell through\n", uni + full + bi, uni, full, bi, fallback);
  }

  const uint8_t *ref(TComPicYuv *p, Int poc) {
    for (auto &d : refs)
      if (d.pic == p && d.poc == poc) return d.org;
    DevRef *slot = nullptr;
    for (auto &d : refs)
      if (d.pic == p) slot = &d;  // the buffer now holds another picture: replace
    if (!slot) { refs.emplace_back(); slot = &refs.back(); }
    hvx_ctx *c = hvx_seam_ctx();
    const int w = p->getWidth(COMPONENT_Y), h = p->getHeight(COMPONENT_Y);
    const int S = w + 2 * HVX_PLANE_MARGIN;
    const size_t n = (size_t)p->getStride(COMPONENT_Y) * p->getTotalHeight(COMPONENT_Y) * sizeof(Pel);
    if (n > pel_bytes) {
      if (d_pel) check(hvx_free(c, d_pel), "hvx_free");
      check(hvx_alloc(c, n, &d_pel), "hvx_alloc");
      pel_bytes = n;
    }
    if (!slot->plane) check(hvx_alloc(c, (size_t)S * (h + 2 * HVX_PLANE_MARGIN), &slot->plane), "hvx_alloc");
    check(hvx_upload(c, d_pel, p->getBuf(COMPONENT_Y), n), "hvx_upload");
    const int16_t *pel0 = (const int16_t *)d_pel + (p->getAddr(COMPONENT_Y) - p->getBuf(COMPONENT_Y));
    check(hvx_plane_from_pel(c, pel0, p->getStride(COMPONENT_Y), w, h, (uint8_t *)slot->plane), "hvx_plane_from_pel");
    slot->pic = p;
    slot->poc = poc;
    slot->org = (const uint8_t *)slot->plane + (size_t)HVX_PLANE_MARGIN * S + HVX_PLANE_MARGIN;
    return slot->org;
  }
};
MeSeam g_me;
}  // namespace

Void TEncSearch::xMotionEstimation(TComDataCU *pcCU, TComYuv *pcYuvOrg, Int iPartIdx, RefPicList eRefPicList,
                                   TComMv *pcMvPred, Int iRefIdxPred, TComMv &rcMv, UInt &ruiBits, Distortion &ruiCost,
                                   Bool bBi) {
  TComSlice *sl = pcCU->getSlice();
  UInt uiPartAddr;
  Int w, h;
  pcCU->getPartIndexAndSize(iPartIdx, uiPartAddr, w, h);
  const bool lossless = pcCU->getCUTransquantBypass(uiPartAddr) != 0;
  const bool wp = (sl->getSliceType() == P_SLICE && sl->getPPS()->getUseWP()) ||
                  (sl->getSliceType() == B_SLICE && sl->getPPS()->getWPBiPred());
  if (wp || lossless || sl->getSPS()->getBitDepth(CHANNEL_TYPE_LUMA) != 8 || (m_iFastSearch != 0 && m_iFastSearch != 1)) {
    g_me.fallback++;
    CAT(__real_, ME_SYM)(this, pcCU, pcYuvOrg, iPartIdx, eRefPicList, pcMvPred, iRefIdxPred, rcMv, ruiBits, ruiCost, bBi);
    return;
  }
  hvx_ctx *c = hvx_seam_ctx();

  m_iSearchRange = m_aaiAdaptSR[eRefPicList][iRefIdxPred];  // side effect the reference makes (:3681)
  const Int iSrchRng = bBi ? m_bipredSearchRange : m_iSearchRange;
  TComYuv *pcYuv = pcYuvOrg;
  if (bBi) {  // the bi-pred refinement target, built exactly as the reference does (:3694-3701)
    TComYuv *pcYuvOther = &m_acYuvPred[1 - (Int)eRefPicList];
    pcYuv = &m_cYuvPredTemp;
    pcYuvOrg->copyPartToPartYuv(pcYuv, uiPartAddr, w, h);
    pcYuv->removeHighFreq(pcYuvOther, uiPartAddr, w, h, sl->getSPS()->getBitDepths().recon,
                          m_pcEncCfg->getClipForBiPredMeEnabled());
  }

  // PU position in the picture (the reference's piRefY offset, :3717)
  TComPicYuv *rec = sl->getRefPic(eRefPicList, iRefIdxPred)->getPicYuvRec();
  const Int ls = rec->getStride(COMPONENT_Y);
  const ptrdiff_t d = rec->getAddr(COMPONENT_Y, pcCU->getCtuRsAddr(), pcCU->getZorderIdxInCtu() + uiPartAddr) -
                      rec->getAddr(COMPONENT_Y);
  hvx_me_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = sl->getSPS()->getPicWidthInLumaSamples();
  j.pic_h = sl->getSPS()->getPicHeightInLumaSamples();
  j.max_cu = sl->getSPS()->getMaxCUWidth();
  j.cu_x = pcCU->getCUPelX();
  j.cu_y = pcCU->getCUPelY();
  j.pu_x = (int)(d % ls);
  j.pu_y = (int)(d / ls);
  j.w = w;
  j.h = h;
  j.pred_x = pcMvPred->getHor();
  j.pred_y = pcMvPred->getVer();
  const bool tz = m_iFastSearch && !bBi;
  if (tz && (pcCU->getPartitionSize(0) != SIZE_2Nx2N || pcCU->getDepth(0) != 0)) {  // :3733-3737
    j.use_int2nx2n = 1;
    j.i2_x = m_integerMv2Nx2N[eRefPicList][iRefIdxPred].getHor();
    j.i2_y = m_integerMv2Nx2N[eRefPicList][iRefIdxPred].getVer();
  }
  j.bits_in = (int32_t)ruiBits;
  j.search_range = iSrchRng;
  j.lambda_motion = HM(m_pcRdCost, TComRdCost_lambda_motion_sad)[0];
  j.flags = (m_pcEncCfg->getUseFastEnc() ? HVX_ME_FEN : 0) | (m_pcEncCfg->getUseHADME() ? HVX_ME_HADME : 0) |
            (m_pcEncCfg->getFastMEAssumingSmootherMVEnabled() ? HVX_ME_SMOOTHMV : 0) | (bBi ? HVX_ME_BI : 0);
  const TComMv centre = bBi ? rcMv : *pcMvPred;  // xSetSearchRange centre (:3723-3730)
  j.center_x = centre.getHor();
  j.center_y = centre.getVer();

  const Pel *src = pcYuv->getAddr(COMPONENT_Y, uiPartAddr);
  const UInt ss = pcYuv->getStride(COMPONENT_Y);
  const uint8_t *refp = g_me.ref(rec, sl->getRefPic(eRefPicList, iRefIdxPred)->getPOC());
  const int S = rec->getWidth(COMPONENT_Y) + 2 * HVX_PLANE_MARGIN;
  if (!g_me.d_job) {
    check(hvx_alloc(c, 2 * sizeof(void *), &g_me.d_ptrs), "hvx_alloc");
    check(hvx_alloc(c, sizeof(hvx_me_job), &g_me.d_job), "hvx_alloc");
    check(hvx_alloc(c, sizeof(hvx_me_result), &g_me.d_res), "hvx_alloc");
    check(hvx_alloc(c, (size_t)65 * S + 64, &g_me.d_cur), "hvx_alloc");
    check(hvx_alloc(c, (size_t)65 * 64 * sizeof(int16_t), &g_me.d_tgt), "hvx_alloc");
  }
  // The kernels address the pattern at (pu_x, pu_y) of a picture-sized plane; only the PU's
  // rows are shipped, so the table entry is the PU block's base rebased to sample (0,0).
  const void *ptrs[2];
  ptrs[1] = refp;
  if (tz) {
    g_me.h_cur.assign((size_t)h * S, 0);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) g_me.h_cur[(size_t)y * S + x] = (uint8_t)src[y * ss + x];
    check(hvx_upload(c, g_me.d_cur, g_me.h_cur.data(), g_me.h_cur.size()), "hvx_upload");
    ptrs[0] = (const uint8_t *)g_me.d_cur - ((ptrdiff_t)j.pu_y * S + j.pu_x);
  } else {
    g_me.h_tgt.assign((size_t)h * 64, 0);
    for (int y = 0; y < h; y++) memcpy(&g_me.h_tgt[(size_t)y * 64], src + y * ss, w * sizeof(Pel));
    check(hvx_upload(c, g_me.d_tgt, g_me.h_tgt.data(), g_me.h_tgt.size() * sizeof(int16_t)), "hvx_upload");
    ptrs[0] = (const int16_t *)g_me.d_tgt - ((ptrdiff_t)j.pu_y * 64 + j.pu_x);
  }
  j.cur_idx = 0;
  j.ref_idx = 0;
  check(hvx_upload(c, g_me.d_ptrs, ptrs, sizeof(ptrs)), "hvx_upload");
  check(hvx_upload(c, g_me.d_job, &j, sizeof(j)), "hvx_upload");
  const void *const *dp = (const void *const *)g_me.d_ptrs;
  if (tz)
    check(hvx_me_batch(c, (const uint8_t *const *)dp, (const uint8_t *const *)dp + 1, S, (const hvx_me_job *)g_me.d_job,
                       1, (hvx_me_result *)g_me.d_res), "hvx_me_batch");
  else
    check(hvx_me_full_batch(c, (const int16_t *const *)dp, 64, (const uint8_t *const *)dp + 1, S,
                            (const hvx_me_job *)g_me.d_job, 1, (hvx_me_result *)g_me.d_res), "hvx_me_full_batch");
  hvx_me_result r;
  check(hvx_download(c, &r, g_me.d_res, sizeof(r)), "hvx_download");
  check(hvx_sync(c), "hvx_sync");

  if (tz && pcCU->getPartitionSize(0) == SIZE_2Nx2N) m_integerMv2Nx2N[eRefPicList][iRefIdxPred].set(r.mv_int_x, r.mv_int_y);
  rcMv.set(r.mv_x, r.mv_y);
  ruiBits = r.bits;
  ruiCost = r.cost;
  // TComRdCost state on exit of the reference (:3745-3755)
  m_pcRdCost->getMotionCost(true, 0, lossless);
  m_pcRdCost->setPredictor(*pcMvPred);
  m_pcRdCost->setCostScale(0);
  (bBi ? g_me.bi : tz ? g_me.uni : g_me.full)++;
}
