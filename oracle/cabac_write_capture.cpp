// cabac_write_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_cabwcap) with -Wl,--wrap=<TEncEntropy::encodeCoeffNxN>.  The RD search calls
// TEncEntropy::encodeCoeffNxN (TEncEntropy.cpp:654) from TEncSearch.cpp for every candidate TU
// (the slice writer's calls stay inside TEncEntropy.cpp, where a link-time wrap cannot see
// them).  For each sampled call the harness hands the same TU (the live TComTU, coefficients
// and component) and the live context states (TEncSbac::loadContexts, :1973) to a second,
// harness-owned TEncSbac whose bin coder is the reference's real arithmetic coder TEncBinCABAC
// (TEncBinCoderCABAC.cpp) writing into its own TComOutputBitstream, and calls
// TEncSbac::codeCoeffNxN (TEncSbac.cpp:1181) on it.  That writer runs as one continuous stream
// over all sampled calls, so every call starts from a reachable coder state.  Each record holds
// the TU geometry and flags, the coefficients, the context states before and after, the
// arithmetic coder registers (m_uiLow, m_uiRange, m_bitsLeft, m_numBufferedBytes,
// m_bufferedByte) before and after, and the bytes the call appended -- golden vectors for the
// device CABAC residual writer (tests/golden/cabac_write.bin).  The RD search itself then runs
// unmodified.
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
#include "TLibCommon/TComBitStream.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComChromaFormat.h"
#include "TLibEncoder/TEncEntropy.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
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

void coder_regs(const TEncBinCABAC *b, std::vector<int64_t> &v) {
  v.insert(v.end(), {(int64_t)b->m_uiLow, (int64_t)b->m_uiRange, (int64_t)b->m_bitsLeft,
                     (int64_t)b->m_numBufferedBytes, (int64_t)b->m_bufferedByte});
}

struct Store {
  std::vector<int32_t> meta;
  std::vector<int16_t> coef;
  std::vector<uint8_t> before, after, bytes;
  std::vector<int64_t> regs, byte_off{0};
  std::map<int, int> count;
  long long ncalls = 0, written = 0;
  int n = 0;
  SplitMix64 rng{0x5EED3005};
  ~Store() { flush(); }
  void flush() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out || !n) return;
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, (uint32_t)kMeta}, meta);
    gw.add("coef", "i16", {(uint32_t)n, 1024}, coef);
    gw.add("states_before", "u8", {(uint32_t)n, (uint32_t)kMaxCtx}, before);
    gw.add("states_after", "u8", {(uint32_t)n, (uint32_t)kMaxCtx}, after);
    gw.add("regs", "i64", {(uint32_t)n, 10}, regs);  // low, range, bits_left, num_buffered, buffered: before | after
    gw.add("bytes", "u8", {(uint32_t)bytes.size()}, bytes);
    gw.add("byte_off", "i64", {(uint32_t)byte_off.size()}, byte_off);
    gw.write(out);
    fprintf(stderr, "cabac_write_capture: %lld calls, %lld written, %d kept, %zu bytes\n", ncalls, written, n,
            bytes.size());
  }
};
Store g;
}  // namespace

struct Writer {
  TComOutputBitstream bs;
  TEncBinCABAC bin;
  TEncSbac sbac;
  Writer() {
    bin.init(&bs);
    bin.start();
    sbac.init(&bin);
  }
};

extern "C" void CAT(__wrap_, COEF_SYM)(TEncEntropy *self, TComTU &rTu, TCoeff *pcCoef, ComponentID compID) {
  static Writer wr;
  g.ncalls++;
  TEncSbac *sbac = dynamic_cast<TEncSbac *>(self->m_pcEntropyCoderIf);
  const TComRectangle &rect = rTu.getRect(compID);
  const int w = rect.width, h = rect.height;
  bool nz = false;  // the reference asserts on an empty TU (TEncSbac.cpp:1233); TEncEntropy skips cbf = 0
  for (int i = 0; i < w * h && !nz; i++) nz = pcCoef[i] != 0;
  if (nz && sbac && sbac->m_numContextModels <= kMaxCtx && wr.sbac.m_numContextModels == sbac->m_numContextModels) {
    g.written++;
    TComDataCU *cu = rTu.getCU();
    const UInt abs = rTu.GetAbsPartIdxTU(compID);
    const int intra = cu->isIntra(abs) ? 1 : 0;
    const int tskip = cu->getTransformSkip(abs, compID) ? 1 : 0;
    // bucket by (size, channel, intra, transform skip): first 30, then a 1/32 sample, max 60 each
    const int key = (w << 8) | (h << 2) | ((compID != COMPONENT_Y) << 1) | intra | (tskip << 16);
    int &c = g.count[key];
    if (c < 60 && (c < 30 || (g.rng.next() & 31) == 0)) {
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
      wr.sbac.loadContexts(sbac);
      for (int i = 0; i < kMaxCtx; i++)
        g.before.push_back(i < wr.sbac.m_numContextModels ? wr.sbac.m_contextModels[i].m_ucState : 0);
      coder_regs(&wr.bin, g.regs);
      const size_t n0 = wr.bs.getFIFO().size();
      wr.sbac.codeCoeffNxN(rTu, pcCoef, compID);
      for (int i = 0; i < kMaxCtx; i++)
        g.after.push_back(i < wr.sbac.m_numContextModels ? wr.sbac.m_contextModels[i].m_ucState : 0);
      coder_regs(&wr.bin, g.regs);
      g.bytes.insert(g.bytes.end(), wr.bs.getFIFO().begin() + n0, wr.bs.getFIFO().end());
      g.byte_off.push_back((int64_t)g.bytes.size());
      g.n++;
    }
  }
  CAT(__real_, COEF_SYM)(self, rTu, pcCoef, compID);
}
