// hm_intra_seam.cpp -- drop-in of the hvx intra prediction under an UNCHANGED HM-16.5rc1 TAppEncoder.
//
// Linked into the reference encoder with -Wl,--wrap=<TComPrediction::predIntraAng>: when the
// environment sets HVX_SEAM_INTRA=1, every intra prediction TEncSearch asks for (the first-pass
// 35-mode scan TEncSearch.cpp:2283, the full-RD TU predictions :1131-1160, chroma included) is
// computed by libhvx.so on the MI355X through the C-ABI (hvx_intra_pred_batch).  The reference
// samples enter as HM already has them: initIntraPatternChType's UNFILTERED border
// (m_piYuvExt[PRED_BUF_UNFILTERED], substitution done) is laid out around the block of a small
// 8-bit plane with every neighbour unit marked available, so the device rebuilds exactly that
// border, applies its own smoothing decision and prediction, and the block comes back into
// piPred.  Calls outside the ported subset (RDPCM/lossless, non-square, 4:2:2/4:4:4, a filter
// flag other than filteringIntraReferenceSamples') fall through to the reference.
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
#include "TLibCommon/TComPrediction.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComSlice.h"
#include "hm_access.hpp"
#include "hvx.h"

#define PRED_SYM _ZN14TComPrediction12predIntraAngE11ComponentIDjPsjS1_jR6TComTUbbbb
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, PRED_SYM)(TComPrediction *, ComponentID, UInt, Pel *, UInt, Pel *, UInt, TComTU &, Bool, Bool,
                                       Bool, Bool);

hvx_ctx *hvx_seam_ctx();  // shared with hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

constexpr int kStride = 2 * MAX_CU_SIZE + 4;      // the staging plane: block at (1, 1)
constexpr int kRows = 2 * MAX_CU_SIZE + 2;

struct IntraSeam {
  bool on = false;
  void *d_plane = nullptr, *d_job = nullptr, *d_pred = nullptr, *d_off = nullptr;
  std::vector<uint8_t> plane, pred;
  long long served = 0, fell = 0;
  IntraSeam() { const char *e = getenv("HVX_SEAM_INTRA"); on = e && e[0] == '1'; }
  ~IntraSeam() {
    if (on) fprintf(stderr, "hm_intra_seam: %lld predIntraAng calls served by libhvx, %lld fell through\n", served, fell);
  }
  void init() {
    if (d_plane) return;
    hvx_ctx *c = hvx_seam_ctx();
    check(hvx_alloc(c, (size_t)kStride * kRows, &d_plane), "hvx_alloc");
    check(hvx_alloc(c, sizeof(hvx_intra_job), &d_job), "hvx_alloc");
    check(hvx_alloc(c, MAX_CU_SIZE * MAX_CU_SIZE, &d_pred), "hvx_alloc");
    check(hvx_alloc(c, sizeof(int64_t), &d_off), "hvx_alloc");
    const int64_t zero = 0;
    check(hvx_upload(c, d_off, &zero, sizeof(zero)), "hvx_upload");
    plane.assign((size_t)kStride * kRows, 0);
    pred.resize(MAX_CU_SIZE * MAX_CU_SIZE);
  }
};
IntraSeam g;
}  // namespace

extern "C" void CAT(__wrap_, PRED_SYM)(TComPrediction *self, ComponentID compID, UInt mode, Pel *piOrg, UInt orgStride,
                                        Pel *piPred, UInt predStride, TComTU &rTu, Bool bAbove, Bool bLeft,
                                        Bool bUseFilt, Bool bDPCM) {
  if (!g.on) {
    CAT(__real_, PRED_SYM)(self, compID, mode, piOrg, orgStride, piPred, predStride, rTu, bAbove, bLeft, bUseFilt, bDPCM);
    return;
  }
  TComDataCU *cu = rTu.getCU();
  const TComSPS &sps = *cu->getSlice()->getSPS();
  const TComRectangle &rect = rTu.getRect(compID);
  const int n = rect.width;
  const ChromaFormat fmt = cu->getPic()->getChromaFormat();
  const bool luma = isLuma(compID);
  int log2 = 0;
  while ((1 << log2) < n) log2++;
  const UInt absIdx = rTu.GetAbsPartIdxTU();
  const bool enable_edge = !(cu->isRDPCMEnabled(absIdx) && cu->getCUTransquantBypass(absIdx));
  const bool ok = !bDPCM && rect.height == n && (1 << log2) == n && n >= 4 && n <= (luma ? 64 : 32) &&
                  (luma || fmt == CHROMA_420) && bAbove && bLeft && enable_edge &&
                  sps.getBitDepth(toChannelType(compID)) == 8 &&
                  bUseFilt == TComPrediction::filteringIntraReferenceSamples(
                                  compID, mode, n, n, fmt, sps.getSpsRangeExtension().getIntraSmoothingDisabledFlag());
  if (!ok) {
    g.fell++;
    CAT(__real_, PRED_SYM)(self, compID, mode, piOrg, orgStride, piPred, predStride, rTu, bAbove, bLeft, bUseFilt, bDPCM);
    return;
  }
  g.init();
  hvx_ctx *c = hvx_seam_ctx();
  // HM's unfiltered border around the block at (1, 1) of the staging plane (stride 2n+1 buffer)
  const Pel *B = HM(self, TComPrediction_yuv_ext)[compID][PRED_BUF_UNFILTERED];
  const int s = 2 * n + 1;
  uint8_t *P = g.plane.data();
  P[0] = (uint8_t)B[0];
  for (int i = 0; i < 2 * n; i++) P[1 + i] = (uint8_t)B[1 + i];
  for (int j = 0; j < 2 * n; j++) P[(1 + j) * kStride] = (uint8_t)B[(j + 1) * s];
  hvx_intra_job job;
  memset(&job, 0, sizeof(job));
  job.x = 1; job.y = 1; job.log2_size = log2; job.ch_type = luma ? 0 : 1;
  job.unit_log2 = luma ? 2 : 1;
  const int units = ((4 * n) >> job.unit_log2) + 1;  // every unit available: the border is taken as is
  for (int u = 0; u < units; u++) job.avail[u >> 5] |= 1u << (u & 31);
  job.mode = (int)mode;
  job.flags = (luma && sps.getUseStrongIntraSmoothing()) ? HVX_INTRA_STRONG : 0;
  check(hvx_upload(c, g.d_plane, P, (size_t)kStride * (2 * n + 1)), "hvx_upload");
  check(hvx_upload(c, g.d_job, &job, sizeof(job)), "hvx_upload");
  check(hvx_intra_pred_batch(c, (const uint8_t *)g.d_plane, kStride, (const hvx_intra_job *)g.d_job, 1,
                             (uint8_t *)g.d_pred, (const int64_t *)g.d_off, nullptr),
        "hvx_intra_pred_batch");
  check(hvx_download(c, g.pred.data(), g.d_pred, (size_t)n * n), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++) piPred[y * predStride + x] = (Pel)g.pred[y * n + x];
  g.served++;
}
