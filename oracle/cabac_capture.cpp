// cabac_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_cabcap) with -Wl,--wrap=<TEncEntropy::encodeCoeffNxN>.  The RD search
// (TEncSearch.cpp:969, 4706, 4875, 5136) counts coefficient bits through
// TEncEntropy::encodeCoeffNxN (TEncEntropy.cpp:654) -> TEncSbac::codeCoeffNxN
// (TEncSbac.cpp:1181) with a TEncBinCABACCounter as the bin coder.  Each sampled call where
// the bin coder is that counter records the TU geometry and flags, the coefficients, the 202
// CABAC context states before and after, the Golomb-Rice statistic before and after, and the
// counter's m_fracBits before and after -- golden vectors for the coefficient-rate
// restatement (tests/golden/cabac.bin).  The reference code itself runs unmodified.
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
#include "TLibCommon/ContextModel.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComChromaFormat.h"
#include "TLibEncoder/TEncEntropy.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABACCounter.h"
#undef private
#undef protected
#include "golden_writer.h"

#define COEF_SYM _ZN11TEncEntropy14encodeCoeffNxNER6TComTUPi11ComponentID
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, COEF_SYM)(TEncEntropy *, TComTU &, TCoeff *, ComponentID);

namespace {
const int kMaxCtx = 256;
const int kMeta = 14;

struct Store {
  std::vector<int32_t> meta, rice_after;
  std::vector<int16_t> coef;  // levels are clipped to 16 bits (TComTrQuant.cpp:1178, RDOQ entropyCodingMaximum)
  std::vector<uint8_t> before, after;
  std::vector<int64_t> frac;
  std::map<int, int> count;
  long long ncalls = 0, counted = 0;
  int n = 0;
  SplitMix64 rng{0x5EED3003};
  ~Store() { flush(); }
  void flush() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out || !n) return;
    std::vector<int32_t> ent(ContextModel::m_entropyBits, ContextModel::m_entropyBits + 128);
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, (uint32_t)kMeta}, meta);
    gw.add("coef", "i16", {(uint32_t)n, 1024}, coef);
    gw.add("states_before", "u8", {(uint32_t)n, (uint32_t)kMaxCtx}, before);
    gw.add("states_after", "u8", {(uint32_t)n, (uint32_t)kMaxCtx}, after);
    gw.add("frac", "i64", {(uint32_t)n, 2}, frac);
    gw.add("rice_after", "i32", {(uint32_t)n}, rice_after);
    gw.add("entropy_bits", "i32", {128}, ent);
    gw.write(out);
    fprintf(stderr, "cabac_capture: %lld calls, %lld counted, %d kept\n", ncalls, counted, n);
  }
};
Store g;
}  // namespace

extern "C" void CAT(__wrap_, COEF_SYM)(TEncEntropy *self, TComTU &rTu, TCoeff *pcCoef, ComponentID compID) {
  g.ncalls++;
  TEncSbac *sbac = dynamic_cast<TEncSbac *>(self->m_pcEntropyCoderIf);
  TEncBinCABACCounter *ctr = sbac ? dynamic_cast<TEncBinCABACCounter *>(sbac->m_pcBinIf) : nullptr;
  bool keep = false;
  const TComRectangle &rect = rTu.getRect(compID);
  const int w = rect.width, h = rect.height;
  if (ctr && sbac->m_numContextModels <= kMaxCtx) {
    g.counted++;
    TComDataCU *cu = rTu.getCU();
    const UInt abs = rTu.GetAbsPartIdxTU(compID);
    const int intra = cu->isIntra(abs) ? 1 : 0;
    const int tskip = cu->getTransformSkip(abs, compID) ? 1 : 0;
    // bucket by (size, channel, intra, transform skip): first 30, then a 1/32 sample, max 60 each
    const int key = (w << 8) | (h << 2) | ((compID != COMPONENT_Y) << 1) | intra | (tskip << 16);
    int &c = g.count[key];
    keep = c < 60 && (c < 30 || (g.rng.next() & 31) == 0);
    if (keep) {
      c++;
      TUEntropyCodingParameters cp;
      getTUEntropyCodingParameters(cp, rTu, compID);
      const TComPPS *pps = cu->getSlice()->getPPS();
      const TComSPS *sps = cu->getSlice()->getSPS();
      UInt &rice = sbac->m_golombRiceAdaptationStatistics[rTu.getGolombRiceStatisticsIndex(compID)];
      g.meta.insert(g.meta.end(),
                    {w, h, (int)compID, (int)cp.scanType, tskip, pps->getUseTransformSkip() ? 1 : 0,
                     pps->getSignHideFlag() ? 1 : 0, cu->getCUTransquantBypass(abs) ? 1 : 0, intra, (int)rice,
                     sps->getSpsRangeExtension().getPersistentRiceAdaptationEnabledFlag() ? 1 : 0,
                     sps->getSpsRangeExtension().getTransformSkipContextEnabledFlag() ? 1 : 0,
                     sps->getSpsRangeExtension().getExtendedPrecisionProcessingFlag() ? 1 : 0,
                     sps->getMaxLog2TrDynamicRange(toChannelType(compID))});
      for (int i = 0; i < 1024; i++) g.coef.push_back((int16_t)(i < w * h ? pcCoef[i] : 0));
      for (int i = 0; i < kMaxCtx; i++)
        g.before.push_back(i < sbac->m_numContextModels ? sbac->m_contextModels[i].m_ucState : 0);
      g.frac.push_back((int64_t)ctr->m_fracBits);
    }
  }
  CAT(__real_, COEF_SYM)(self, rTu, pcCoef, compID);
  if (keep) {
    const UInt rice = sbac->m_golombRiceAdaptationStatistics[rTu.getGolombRiceStatisticsIndex(compID)];
    for (int i = 0; i < kMaxCtx; i++)
      g.after.push_back(i < sbac->m_numContextModels ? sbac->m_contextModels[i].m_ucState : 0);
    g.frac.push_back((int64_t)ctr->m_fracBits);
    g.rice_after.push_back((int32_t)rice);
    g.n++;
  }
}
