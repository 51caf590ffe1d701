// tu_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_capture) with
//   -Wl,--wrap=<TComTrQuant::transformNxN>,--wrap=<TComTrQuant::invTransformNxN>
// so that every call TEncSearch makes into the reference transform/quant
// (TEncSearch.cpp:1262,1277,4632,4640,4711 -> TComTrQuant.cpp:1460,1547) is
// observed: the TU geometry, QP, lambda, the CABAC-derived estBits table,
// the residual in, and the quantised levels / reconstructed residual out.
// A bounded, bucketed sample of those calls is written as golden vectors
// (tests/golden/tu_*.bin).  The reference code itself runs unmodified.
#include <sstream>
#include <iostream>
#include <fstream>
#include <vector>
#include <list>
#include <map>
#include <set>
#include <string>
#include <algorithm>
#include <cassert>
#include <cstring>
#include <cstdio>
#include <cmath>
#include <limits>
#include <memory>
#include <cstdlib>
#define private public
#define protected public
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComChromaFormat.h"
#undef private
#undef protected
#include "golden_writer.h"

#define FWD_SYM _ZN11TComTrQuant12transformNxNER6TComTU11ComponentIDPsjPiS4_RiRK7QpParam
#define INV_SYM _ZN11TComTrQuant15invTransformNxNER6TComTU11ComponentIDPsjPiRK7QpParam
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" {
void CAT(__real_, FWD_SYM)(TComTrQuant *, TComTU &, ComponentID, Pel *, UInt, TCoeff *, TCoeff *, TCoeff &, const QpParam &);
void CAT(__real_, INV_SYM)(TComTrQuant *, TComTU &, ComponentID, Pel *, UInt, TCoeff *, const QpParam &);
}

namespace {
const int kEstInts = sizeof(estBitsSbacStruct) / sizeof(Int);

struct Store {
  std::vector<int32_t> fmeta, fest, fcoefout, ftemp, imeta, icoef;
  std::vector<int16_t> fres, ires;
  std::vector<double> flambda;
  std::vector<int64_t> foff, ioff;
  std::map<int, int> fcount, icount;
  long long ncalls = 0, nicalls = 0;
  int nf = 0, ni = 0;
  SplitMix64 rng{0x5EED2001};
  ~Store() { flush(); }
  void flush() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out || (!nf && !ni)) return;
    GoldenWriter gw;
    gw.add("fwd_meta", "i32", {(uint32_t)nf, 28}, fmeta);
    gw.add("fwd_lambda", "f64", {(uint32_t)nf}, flambda);
    gw.add("fwd_estbits", "i32", {(uint32_t)nf, (uint32_t)kEstInts}, fest);
    gw.add("fwd_off", "i64", {(uint32_t)nf}, foff);
    gw.add("fwd_res", "i16", {(uint32_t)fres.size()}, fres);
    gw.add("fwd_temp", "i32", {(uint32_t)ftemp.size()}, ftemp);
    gw.add("fwd_coef", "i32", {(uint32_t)fcoefout.size()}, fcoefout);
    gw.add("inv_meta", "i32", {(uint32_t)ni, 12}, imeta);
    gw.add("inv_off", "i64", {(uint32_t)ni}, ioff);
    gw.add("inv_coef", "i32", {(uint32_t)icoef.size()}, icoef);
    gw.add("inv_res", "i16", {(uint32_t)ires.size()}, ires);
    gw.write(out);
    fprintf(stderr, "tu_capture: %lld fwd calls (%d kept), %lld inv calls (%d kept)\n", ncalls, nf, nicalls, ni);
  }
} g_store;

int cap_per_bucket() {
  const char *e = getenv("HVX_CAPTURE_PER_BUCKET");
  return e ? atoi(e) : 10;
}
}  // namespace

extern "C" void CAT(__wrap_, FWD_SYM)(TComTrQuant *self, TComTU &rTu, ComponentID compID, Pel *res, UInt stride,
                                      TCoeff *coeff, TCoeff *arl, TCoeff &absSum, const QpParam &qp) {
  TComDataCU *cu = rTu.getCU();
  const UInt idx = rTu.GetAbsPartIdxTU();
  const TComRectangle &rect = rTu.getRect(compID);
  const Int w = rect.width, h = rect.height;
  const ChannelType ch = toChannelType(compID);
  const Int tskip = cu->getTransformSkip(idx, compID);
  const Int intra = cu->isIntra(idx) ? 1 : 0;
  const Int bypass = cu->getCUTransquantBypass(idx) ? 1 : 0;
  // snapshot inputs before the call (the reference overwrites nothing it reads, but be safe)
  std::vector<int16_t> r(w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) r[y * w + x] = res[y * stride + x];
  std::vector<int32_t> est((int32_t *)self->m_pcEstBitsSbac, (int32_t *)self->m_pcEstBitsSbac + kEstInts);
  const double lambda = self->m_dLambda;
  const UInt gr = self->m_pcEstBitsSbac->golombRiceAdaptationStatistics[rTu.getGolombRiceStatisticsIndex(compID)];
  const Int ctxQtCbf = cu->getCtxQtCbf(rTu, ch);
  const Int trIdx = cu->getTransformIdx(idx);
  const Int scan = cu->getCoefScanIdx(idx, w, h, compID);
  const Int dst = rTu.useDST(compID) ? 1 : 0;
  const Int log2 = rTu.GetEquivalentLog2TrSize(compID);

  CAT(__real_, FWD_SYM)(self, rTu, compID, res, stride, coeff, arl, absSum, qp);
  g_store.ncalls++;

  const TComSlice *sl = cu->getSlice();
  const Int rdoqMode = tskip ? self->m_useRDOQTS : self->m_useRDOQ;
  int key = (ch << 12) | (log2 << 8) | (intra << 7) | (tskip << 6) | (rdoqMode << 5) | ((absSum >= 2) << 4) | (dst << 3) | (scan & 3);
  int &cnt = g_store.fcount[key];
  bool keep = cnt < cap_per_bucket() || (g_store.rng.next() % 4000 == 0);
  if (!keep) return;
  cnt++;
  Int meta[28] = {compID, w, h, log2, scan, dst, tskip, intra, trIdx, ctxQtCbf,
                  sl->getSliceType(), qp.Qp, qp.per, qp.rem,
                  sl->getPPS()->getSignHideFlag() ? 1 : 0, self->m_useRDOQ, self->m_useRDOQTS, self->m_useSelectiveRDOQ,
                  self->m_bUseAdaptQpSelect, bypass, (Int)gr,
                  sl->getSPS()->getSpsRangeExtension().getPersistentRiceAdaptationEnabledFlag() ? 1 : 0,
                  sl->getSPS()->getSpsRangeExtension().getExtendedPrecisionProcessingFlag() ? 1 : 0,
                  sl->getSPS()->getMaxLog2TrDynamicRange(ch), sl->getSPS()->getBitDepth(ch),
                  (Int)absSum, sl->getSPS()->getSpsRangeExtension().getTransformSkipContextEnabledFlag() ? 1 : 0,
                  cu->getPredictionMode(idx)};
  g_store.fmeta.insert(g_store.fmeta.end(), meta, meta + 28);
  g_store.flambda.push_back(lambda);
  g_store.fest.insert(g_store.fest.end(), est.begin(), est.end());
  g_store.foff.push_back((int64_t)g_store.fres.size());
  g_store.fres.insert(g_store.fres.end(), r.begin(), r.end());
  for (int i = 0; i < w * h; i++) {
    g_store.ftemp.push_back(self->m_plTempCoeff[i]);
    g_store.fcoefout.push_back(coeff[i]);
  }
  g_store.nf++;
}

extern "C" void CAT(__wrap_, INV_SYM)(TComTrQuant *self, TComTU &rTu, ComponentID compID, Pel *res, UInt stride,
                                      TCoeff *coeff, const QpParam &qp) {
  TComDataCU *cu = rTu.getCU();
  const UInt idx = rTu.GetAbsPartIdxTU();
  const TComRectangle &rect = rTu.getRect(compID);
  const Int w = rect.width, h = rect.height;
  std::vector<int32_t> c(coeff, coeff + w * h);
  const Int tskip = cu->getTransformSkip(idx, compID);
  const Int dst = rTu.useDST(compID) ? 1 : 0;
  const Int bypass = cu->getCUTransquantBypass(idx) ? 1 : 0;
  const Int log2 = rTu.GetEquivalentLog2TrSize(compID);

  CAT(__real_, INV_SYM)(self, rTu, compID, res, stride, coeff, qp);
  g_store.nicalls++;

  bool nz = false;
  for (auto v : c) nz |= v != 0;
  int key = (toChannelType(compID) << 8) | (log2 << 4) | (tskip << 3) | (dst << 2) | (nz << 1);
  int &cnt = g_store.icount[key];
  if (!(cnt < cap_per_bucket() || (g_store.rng.next() % 4000 == 0))) return;
  cnt++;
  const TComSlice *sl = cu->getSlice();
  Int meta[12] = {compID, w, h, log2, dst, tskip, qp.Qp, qp.per, qp.rem, bypass,
                  sl->getSPS()->getMaxLog2TrDynamicRange(toChannelType(compID)), sl->getSPS()->getBitDepth(toChannelType(compID))};
  g_store.imeta.insert(g_store.imeta.end(), meta, meta + 12);
  g_store.ioff.push_back((int64_t)g_store.ires.size());
  g_store.icoef.insert(g_store.icoef.end(), c.begin(), c.end());
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) g_store.ires.push_back(res[y * stride + x]);
  g_store.ni++;
}
