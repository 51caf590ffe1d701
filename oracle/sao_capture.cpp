// sao_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target _ref/TAppEncoder_saocap)
// with -Wl,--wrap=<TEncSampleAdaptiveOffset::SAOProcess>.  For each of the first pictures
// TEncGOP runs SAO on (TEncGOP.cpp:1500) it records
//   * the original and the deblocked reconstruction (SAOProcess's input), Y, Cb, Cr (8-bit video);
//   * the per-CTU statistics SAOProcess gathered (m_statData after the call:
//     TEncSampleAdaptiveOffset::getStatistics / getBlkStats, TEncSampleAdaptiveOffset.cpp:285, 892):
//     diff[32] and count[32] (int64) of every component and SAO type;
//   * every CTU's SAO parameters as offsetCTU applied them: the coded parameters the reference
//     decided (TComPicSym::getSAOBlkParam) resolved through the reference's own getMergeList and
//     reconstructBlkSAOParam (TComSampleAdaptiveOffset.cpp:192, 248), exactly as decideBlkParams
//     (TEncSampleAdaptiveOffset.cpp:845-848) does before offsetCTU;
//   * the picture after SAO (SAOProcess's output);
//   * for the first picture of a run, one more record: random parameters (every type, OFF
//     included, on every CTU and component) applied to the same input by the reference's own
//     TComSampleAdaptiveOffset::offsetCTU (TComSampleAdaptiveOffset.cpp:554), so every edge
//     class and boundary rule is pinned even where the encoder chose band offsets (meta[3] = 1).
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
#undef private
#undef protected
#include "golden_writer.h"

#define SAO_SYM _ZN24TEncSampleAdaptiveOffset10SAOProcessEP7TComPicPbPKdbddb
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, SAO_SYM)(TEncSampleAdaptiveOffset *, TComPic *, Bool *, const Double *, const Bool,
                                      const Double, const Double, Bool);

namespace {
struct Store {
  std::vector<int32_t> meta;  // per record: w, h, ctus, synthetic
  std::vector<uint8_t> org, pre, post;
  std::vector<int64_t> stats;  // per CTU: [comp 3][type 5][diff 32, count 32]
  std::vector<int32_t> params; // per CTU: [comp 3][type (-1 off, 0..3 EO, 4 BO), band position, offset[4]]
  int n = 0, pics = 0;
  SplitMix64 rng{0x5A0C0DEull};
  ~Store() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out) return;
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, 4}, meta);
    gw.add("org", "u8", {(uint32_t)org.size()}, org);    // per picture: Y w*h, Cb, Cr (w/2)*(h/2)
    gw.add("pre", "u8", {(uint32_t)pre.size()}, pre);
    gw.add("post", "u8", {(uint32_t)post.size()}, post);
    gw.add("stats", "i64", {(uint32_t)(stats.size() / 960), 3, 5, 64}, stats);  // diff[32] then count[32]
    gw.add("params", "i32", {(uint32_t)(params.size() / 18), 3, 6}, params);
    gw.write(out);
    fprintf(stderr, "sao_capture: %d pictures\n", n);
  }
};
Store g;

void planes(TComPicYuv *p, std::vector<uint8_t> &dst) {
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int w = p->getWidth(id), h = p->getHeight(id), s = p->getStride(id);
    const Pel *a = p->getAddr(id);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst.push_back((uint8_t)a[y * s + x]);
  }
}
}  // namespace

extern "C" void CAT(__wrap_, SAO_SYM)(TEncSampleAdaptiveOffset *self, TComPic *pic, Bool *sliceEnabled,
                                       const Double *lambdas, const Bool testOff, const Double rate,
                                       const Double rateChroma, Bool preDbf) {
  const bool keep = g.n < 3 && !preDbf && pic->getChromaFormat() == CHROMA_420;
  if (keep) {
    planes(pic->getPicYuvOrg(), g.org);
    planes(pic->getPicYuvRec(), g.pre);
  }
  CAT(__real_, SAO_SYM)(self, pic, sliceEnabled, lambdas, testOff, rate, rateChroma, preDbf);
  if (!keep) return;
  const int nctu = self->m_numCTUsPic;
  g.meta.insert(g.meta.end(), {self->m_picWidth, self->m_picHeight, nctu, 0});
  for (int c = 0; c < nctu; c++)
    for (int k = 0; k < 3; k++)
      for (int t = 0; t < NUM_SAO_NEW_TYPES; t++) {
        const SAOStatData &s = self->m_statData[c][k][t];
        g.stats.insert(g.stats.end(), s.diff, s.diff + 32);
        g.stats.insert(g.stats.end(), s.count, s.count + 32);
      }
  // the parameters offsetCTU applied: decideBlkParams' reconParams, rebuilt with the reference's code
  SAOBlkParam *coded = pic->getPicSym()->getSAOBlkParam();
  std::vector<SAOBlkParam> recon(nctu);
  for (int c = 0; c < nctu; c++) {
    SAOBlkParam *merge[NUM_SAO_MERGE_TYPES] = {NULL};
    self->getMergeList(pic, c, recon.data(), merge);
    recon[c] = coded[c];
    self->reconstructBlkSAOParam(recon[c], merge);
    for (int k = 0; k < 3; k++) {
      const SAOOffset &o = recon[c][k];
      int32_t rec[6] = {-1, 0, 0, 0, 0, 0};
      if (o.modeIdc != SAO_MODE_OFF) {
        assert(o.modeIdc == SAO_MODE_NEW);
        rec[0] = o.typeIdc;
        if (o.typeIdc == SAO_TYPE_BO) {
          rec[1] = o.typeAuxInfo;
          for (int i = 0; i < 4; i++) rec[2 + i] = o.offset[(o.typeAuxInfo + i) % NUM_SAO_BO_CLASSES];
        } else {
          const int cls[4] = {SAO_CLASS_EO_FULL_VALLEY, SAO_CLASS_EO_HALF_VALLEY, SAO_CLASS_EO_HALF_PEAK,
                              SAO_CLASS_EO_FULL_PEAK};
          for (int i = 0; i < 4; i++) rec[2 + i] = o.offset[cls[i]];
        }
      }
      g.params.insert(g.params.end(), rec, rec + 6);
    }
  }
  planes(pic->getPicYuvRec(), g.post);
  g.n++;
  if (g.pics++ > 0) return;
  // synthetic record: random reconstructed parameters through the reference's offsetCTU, from
  // SAOProcess's own extended copy of the deblocked picture (m_tempPicYuv) into a fresh picture
  TComPicYuv *src = self->m_tempPicYuv;
  TComPicYuv res;
  const TComSPS &sps = pic->getPicSym()->getSPS();
  res.create(self->m_picWidth, self->m_picHeight, pic->getChromaFormat(), sps.getMaxCUWidth(), sps.getMaxCUHeight(),
             sps.getMaxTotalCUDepth(), true);
  src->copyToPic(&res);
  std::vector<SAOBlkParam> syn(nctu);
  for (int c = 0; c < nctu; c++)
    for (int k = 0; k < 3; k++) {
      SAOOffset &o = syn[c][k];
      o.reset();
      int32_t rec[6] = {-1, 0, 0, 0, 0, 0};
      const int t = g.rng.range(-1, 4);
      if (t >= 0) {
        o.modeIdc = SAO_MODE_NEW;
        o.typeIdc = t;
        rec[0] = t;
        if (t == SAO_TYPE_BO) {
          o.typeAuxInfo = g.rng.range(0, 31);
          rec[1] = o.typeAuxInfo;
          for (int i = 0; i < 4; i++) rec[2 + i] = o.offset[(o.typeAuxInfo + i) % NUM_SAO_BO_CLASSES] = g.rng.range(-7, 7);
        } else {
          const int cls[4] = {SAO_CLASS_EO_FULL_VALLEY, SAO_CLASS_EO_HALF_VALLEY, SAO_CLASS_EO_HALF_PEAK,
                              SAO_CLASS_EO_FULL_PEAK};
          for (int i = 0; i < 4; i++) rec[2 + i] = o.offset[cls[i]] = i < 2 ? g.rng.range(0, 7) : g.rng.range(-7, 0);
        }
      }
      g.params.insert(g.params.end(), rec, rec + 6);
    }
  for (int c = 0; c < nctu; c++) self->offsetCTU(c, src, &res, syn[c], pic);
  g.meta.insert(g.meta.end(), {self->m_picWidth, self->m_picHeight, nctu, 1});
  const size_t plane_bytes = g.post.size() / g.n;
  g.org.insert(g.org.end(), g.org.end() - plane_bytes, g.org.end());
  g.pre.insert(g.pre.end(), g.pre.end() - plane_bytes, g.pre.end());
  g.stats.insert(g.stats.end(), g.stats.end() - (size_t)nctu * 960, g.stats.end());
  planes(&res, g.post);
  res.destroy();
  g.n++;
}
