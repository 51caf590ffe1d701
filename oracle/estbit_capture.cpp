// estbit_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_estcap) with -Wl,--wrap=<TEncEntropy::estimateBit>.  TEncSearch calls
// TEncEntropy::estimateBit (TEncEntropy.cpp) before every transform/quant of the RD search,
// which forwards to TEncSbac::estBit (TEncSbac.cpp:1726).  Each sampled call records the
// CABAC context states of the RD coder (TEncSbac::m_contextModels, one state byte per model),
// its Golomb-Rice statistics, the TU geometry / channel type, and the estBitsSbacStruct
// before and after -- golden vectors for the estBit restatement (tests/golden/estbit.bin).
// ContextModel::m_entropyBits (the table estBit reads) is recorded once.  The reference code
// itself runs unmodified.
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
#include "TLibCommon/TComTrQuant.h"
#include "TLibEncoder/TEncEntropy.h"
#include "TLibEncoder/TEncSbac.h"
#undef private
#undef protected
#include "golden_writer.h"

#define EST_SYM _ZN11TEncEntropy11estimateBitEP17estBitsSbacStructii11ChannelType
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, EST_SYM)(TEncEntropy *, estBitsSbacStruct *, Int, Int, ChannelType);

namespace {
const int kEstInts = sizeof(estBitsSbacStruct) / sizeof(Int);
const int kMaxCtx = 256;

struct Store {
  std::vector<int32_t> meta, before, after, rice;
  std::vector<uint8_t> states;
  std::map<int, int> count;
  long long ncalls = 0;
  int n = 0, nctx = 0;
  SplitMix64 rng{0x5EED2002};
  ~Store() { flush(); }
  void flush() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out || !n) return;
    std::vector<int32_t> ent(ContextModel::m_entropyBits, ContextModel::m_entropyBits + 128);
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, 4}, meta);
    gw.add("states", "u8", {(uint32_t)n, (uint32_t)kMaxCtx}, states);
    gw.add("rice", "i32", {(uint32_t)n, 4}, rice);
    gw.add("before", "i32", {(uint32_t)n, (uint32_t)kEstInts}, before);
    gw.add("after", "i32", {(uint32_t)n, (uint32_t)kEstInts}, after);
    gw.add("entropy_bits", "i32", {128}, ent);
    gw.write(out);
    fprintf(stderr, "estbit_capture: %lld calls (%d kept), %d context models\n", ncalls, n, nctx);
  }
};
Store g;
}  // namespace

extern "C" void CAT(__wrap_, EST_SYM)(TEncEntropy *self, estBitsSbacStruct *est, Int w, Int h, ChannelType ch) {
  g.ncalls++;
  TEncSbac *sbac = dynamic_cast<TEncSbac *>(self->m_pcEntropyCoderIf);
  // bucket by (size, channel): keep the first 24 of each bucket, then a 1/64 sample, max 40 each
  const int key = (w << 8) | (h << 1) | (int)ch;
  int &c = g.count[key];
  const bool keep = sbac && sbac->m_numContextModels <= kMaxCtx && c < 40 && (c < 24 || (g.rng.next() & 63) == 0);
  if (keep) {
    c++;
    g.nctx = sbac->m_numContextModels;
    g.meta.insert(g.meta.end(), {w, h, (int)ch, sbac->m_numContextModels});
    for (int i = 0; i < kMaxCtx; i++) g.states.push_back(i < sbac->m_numContextModels ? sbac->m_contextModels[i].m_ucState : 0);
    for (int i = 0; i < 4; i++) g.rice.push_back((int32_t)sbac->m_golombRiceAdaptationStatistics[i]);
    const Int *b = (const Int *)est;
    g.before.insert(g.before.end(), b, b + kEstInts);
  }
  CAT(__real_, EST_SYM)(self, est, w, h, ch);
  if (keep) {
    const Int *a = (const Int *)est;
    g.after.insert(g.after.end(), a, a + kEstInts);
    g.n++;
  }
}
