// saodec_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target _ref/TAppEncoder_saodec)
// with -Wl,--wrap=<TEncSampleAdaptiveOffset::SAOProcess>.  For each picture TEncGOP runs SAO on
// (TEncGOP.cpp:1500) it records the inputs and outputs of the SAO RD decision
// (decidePicParams TEncSampleAdaptiveOffset.cpp:332, decideBlkParams :763 with deriveModeNewRDO
// :566, deriveModeMergeRDO :709, deriveOffsets :447, estIterOffset :414):
//   * meta: width, height, CTUs, picture temporal layer (TComSlice::getDepth), bTestSAODisableAtPictureLevel,
//     the slice-enabled flags SAOProcess returned (Y, Cb, Cr), the SAO context states of the
//     picture-start RD coder (m_pppcRDSbacCoder[SAO_CABACSTATE_PIC_INIT]: sao_merge_left/up flag,
//     sao_type_idx) and the low 15 bits of its fractional bit count;
//   * f64: the three lambdas, SAOEncodingRate / SAOEncodingRateChroma, m_saoDisabledRate before
//     and after (3 components x 7 temporal layers each);
//   * the per-CTU statistics the decision reads (m_statData: diff[32], count[32] per component
//     and type);
//   * the coded parameters it decided per CTU and component (TComPicSym::getSAOBlkParam):
//     mode (0 off, 1 new, 2 merge), type (EO 0-3 / BO 4, or the merge direction), band position,
//     offsets of classes 0..4 (EO) or of the 4 bands from the band position (BO).
// The reference code itself runs unmodified.
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
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComPicSym.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComSampleAdaptiveOffset.h"
#include "TLibEncoder/TEncSampleAdaptiveOffset.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#undef private
#undef protected
#include "golden_writer.h"

#define SAO_SYM _ZN24TEncSampleAdaptiveOffset10SAOProcessEP7TComPicPbPKdbddb
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, SAO_SYM)(TEncSampleAdaptiveOffset *, TComPic *, Bool *, const Double *, const Bool,
                                      const Double, const Double, Bool);

namespace {
const int kMeta = 12, kF64 = 5 + 2 * 3 * MAX_TLAYER;
struct Store {
  std::vector<int32_t> meta;   // per picture: kMeta ints (see the header)
  std::vector<double> f64;     // per picture: lambdas[3], rate, rate chroma, disabled rate before / after [3][MAX_TLAYER]
  std::vector<int64_t> stats;  // per CTU: [comp 3][type 5][diff 32, count 32]
  std::vector<int32_t> params; // per CTU: [comp 3][mode, type, band, offset[5]]
  int n = 0;
  ~Store() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out) return;
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, kMeta}, meta);
    gw.add("f64", "f64", {(uint32_t)n, kF64}, f64);
    gw.add("stats", "i64", {(uint32_t)(stats.size() / 960), 3, 5, 64}, stats);
    gw.add("params", "i32", {(uint32_t)(params.size() / 24), 3, 8}, params);
    gw.write(out);
    fprintf(stderr, "saodec_capture: %d pictures\n", n);
  }
};
Store g;
}  // namespace

extern "C" void CAT(__wrap_, SAO_SYM)(TEncSampleAdaptiveOffset *self, TComPic *pic, Bool *sliceEnabled,
                                       const Double *lambdas, const Bool testOff, const Double rate,
                                       const Double rateChroma, Bool preDbf) {
  const bool keep = !preDbf && pic->getChromaFormat() == CHROMA_420 && pic->getPicSym()->getNumTiles() == 1;
  double before[3][MAX_TLAYER];
  int st_merge = 0, st_type = 0, frac_lo = 0;
  if (keep) {
    for (int c = 0; c < 3; c++)
      for (int t = 0; t < MAX_TLAYER; t++) before[c][t] = self->m_saoDisabledRate[c][t];
    TEncSbac *init = self->m_pppcRDSbacCoder[SAO_CABACSTATE_PIC_INIT];
    st_merge = init->m_cSaoMergeSCModel.get(0, 0, 0).m_ucState;
    st_type = init->m_cSaoTypeIdxSCModel.get(0, 0, 0).m_ucState;
    frac_lo = (int)(((TEncBinCABAC *)init->m_pcBinIf)->m_fracBits & 32767);
  }
  CAT(__real_, SAO_SYM)(self, pic, sliceEnabled, lambdas, testOff, rate, rateChroma, preDbf);
  if (!keep) return;
  const int nctu = self->m_numCTUsPic;
  g.meta.insert(g.meta.end(), {self->m_picWidth, self->m_picHeight, nctu, pic->getSlice(0)->getDepth(), testOff ? 1 : 0,
                               sliceEnabled[0] ? 1 : 0, sliceEnabled[1] ? 1 : 0, sliceEnabled[2] ? 1 : 0, st_merge, st_type,
                               frac_lo, pic->getNumAllocatedSlice()});
  g.f64.insert(g.f64.end(), {lambdas[0], lambdas[1], lambdas[2], rate, rateChroma});
  for (int c = 0; c < 3; c++)
    for (int t = 0; t < MAX_TLAYER; t++) g.f64.push_back(before[c][t]);
  for (int c = 0; c < 3; c++)
    for (int t = 0; t < MAX_TLAYER; t++) g.f64.push_back(self->m_saoDisabledRate[c][t]);
  for (int a = 0; a < nctu; a++)
    for (int k = 0; k < 3; k++)
      for (int t = 0; t < NUM_SAO_NEW_TYPES; t++) {
        const SAOStatData &s = self->m_statData[a][k][t];
        g.stats.insert(g.stats.end(), s.diff, s.diff + 32);
        g.stats.insert(g.stats.end(), s.count, s.count + 32);
      }
  SAOBlkParam *coded = pic->getPicSym()->getSAOBlkParam();
  for (int a = 0; a < nctu; a++)
    for (int k = 0; k < 3; k++) {
      const SAOOffset &o = coded[a][k];
      int32_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      r[0] = o.modeIdc == SAO_MODE_OFF ? 0 : o.modeIdc == SAO_MODE_NEW ? 1 : 2;
      if (o.modeIdc != SAO_MODE_OFF) {
        r[1] = o.typeIdc;
        if (o.modeIdc == SAO_MODE_NEW) {
          r[2] = o.typeAuxInfo;
          if (o.typeIdc == SAO_TYPE_BO)
            for (int i = 0; i < 4; i++) r[3 + i] = o.offset[(o.typeAuxInfo + i) % NUM_SAO_BO_CLASSES];
          else
            for (int i = 0; i < 5; i++) r[3 + i] = o.offset[i];
        }
      }
      g.params.insert(g.params.end(), r, r + 8);
    }
  g.n++;
}
