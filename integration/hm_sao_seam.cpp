// hm_sao_seam.cpp -- drop-in of the hvx SAO kernels under an UNCHANGED HM-16.5rc1 TAppEncoder.
//
// Linked into the reference encoder with -Wl,--wrap=<TEncSampleAdaptiveOffset::SAOProcess> and
// -Wl,--wrap=<TComSampleAdaptiveOffset::offsetCTU>.  For every picture TEncGOP runs SAO on
// (TEncGOP.cpp:1500) the wrapper performs SAOProcess's steps (TEncSampleAdaptiveOffset.cpp:241-264)
// with the two sample-level stages on the MI355X through the C-ABI:
//   1. the deblocked picture is copied and border-extended as the reference does (m_tempPicYuv);
//   2. the statistics of every CTU, component and type come from hvx_sao_stats and are written
//      into the encoder's m_statData -- in place of getStatistics;
//   3. the reference's own decidePicParams and decideBlkParams make the RD decisions (CABAC-rate
//      estimates carried CTU to CTU, merges); decideBlkParams' per-CTU offsetCTU calls only record
//      the merge-resolved parameters (the wrapped offsetCTU, while the seam is active);
//   4. hvx_sao_apply applies every CTU's parameters to the copy and the result becomes the
//      picture's reconstruction -- in place of offsetCTU.
// Pictures outside the ported subset (pre-deblocking statistics, not 8-bit 4:2:0, several slices
// or tiles, sizes not multiples of 8) fall through to the reference.
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
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComPicSym.h"
#include "TLibCommon/TComPicYuv.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComSampleAdaptiveOffset.h"
#include "TLibEncoder/TEncSampleAdaptiveOffset.h"
#include "hm_access.hpp"
#include "hvx.h"

#define SAO_SYM _ZN24TEncSampleAdaptiveOffset10SAOProcessEP7TComPicPbPKdbddb
#define OFF_SYM _ZN24TComSampleAdaptiveOffset9offsetCTUEiP10TComPicYuvS1_R11SAOBlkParamP7TComPic
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, SAO_SYM)(TEncSampleAdaptiveOffset *, TComPic *, Bool *, const Double *, const Bool,
                                      const Double, const Double, Bool);
extern "C" void CAT(__real_, OFF_SYM)(TComSampleAdaptiveOffset *, Int, TComPicYuv *, TComPicYuv *, SAOBlkParam &,
                                      TComPic *);

hvx_ctx *hvx_seam_ctx();  // shared with hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

struct SaoSeam {
  void *d_org[3] = {}, *d_src[3] = {}, *d_dst[3] = {}, *d_stats = nullptr, *d_params = nullptr;
  size_t org_bytes[3] = {}, src_bytes[3] = {}, dst_bytes[3] = {}, stats_bytes = 0, params_bytes = 0;
  std::vector<uint8_t> host[3];
  std::vector<hvx_sao_stat> stats;
  std::vector<hvx_sao_ctu> params;
  bool deferring = false;
  long long pictures = 0, fell = 0;
  ~SaoSeam() { fprintf(stderr, "hm_sao_seam: %lld pictures through libhvx SAO, %lld fell through\n", pictures, fell); }
  void ensure(void *&p, size_t &have, size_t need) {
    if (have >= need) return;
    if (p) check(hvx_free(hvx_seam_ctx(), p), "hvx_free");
    check(hvx_alloc(hvx_seam_ctx(), need, &p), "hvx_alloc");
    have = need;
  }
};
SaoSeam g;

void upload(TComPicYuv *p, void *const d[3]) {
  for (int k = 0; k < 3; k++) {
    const ComponentID id = ComponentID(k);
    const int w = p->getWidth(id), h = p->getHeight(id), s = p->getStride(id);
    const Pel *a = p->getAddr(id);
    g.host[k].resize((size_t)w * h);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) g.host[k][(size_t)y * w + x] = (uint8_t)a[y * s + x];
    check(hvx_upload(hvx_seam_ctx(), d[k], g.host[k].data(), g.host[k].size()), "hvx_upload");
    check(hvx_sync(hvx_seam_ctx()), "hvx_sync");  // the staging vector is reused by the next plane
  }
}
}  // namespace

// while the seam runs decideBlkParams: keep the parameters offsetCTU would apply
extern "C" void CAT(__wrap_, OFF_SYM)(TComSampleAdaptiveOffset *self, Int ctu, TComPicYuv *src, TComPicYuv *res,
                                       SAOBlkParam &prm, TComPic *pic) {
  if (!g.deferring) {
    CAT(__real_, OFF_SYM)(self, ctu, src, res, prm, pic);
    return;
  }
  hvx_sao_ctu &o = g.params[ctu];
  for (int k = 0; k < 3; k++) {
    const SAOOffset &s = prm[k];
    hvx_sao_offset &d = o.comp[k];
    memset(&d, 0, sizeof(d));
    d.type = HVX_SAO_OFF;
    if (s.modeIdc == SAO_MODE_OFF) continue;
    if (s.modeIdc != SAO_MODE_NEW) abort();  // reconstructBlkSAOParam resolved every merge before this call
    d.type = (int8_t)s.typeIdc;
    if (s.typeIdc == SAO_TYPE_BO) {
      d.band = (uint8_t)s.typeAuxInfo;
      for (int i = 0; i < 4; i++) d.offset[i] = (int8_t)s.offset[(s.typeAuxInfo + i) % NUM_SAO_BO_CLASSES];
    } else {
      d.offset[0] = (int8_t)s.offset[SAO_CLASS_EO_FULL_VALLEY];
      d.offset[1] = (int8_t)s.offset[SAO_CLASS_EO_HALF_VALLEY];
      d.offset[2] = (int8_t)s.offset[SAO_CLASS_EO_HALF_PEAK];
      d.offset[3] = (int8_t)s.offset[SAO_CLASS_EO_FULL_PEAK];
    }
  }
}

extern "C" void CAT(__wrap_, SAO_SYM)(TEncSampleAdaptiveOffset *self, TComPic *pic, Bool *sliceEnabled,
                                       const Double *lambdas, const Bool testOff, const Double rate,
                                       const Double rateChroma, Bool preDbf) {
  const TComSPS &sps = pic->getPicSym()->getSPS();
  const int W = HM(self, TComSao_width), H = HM(self, TComSao_height);
  const bool ok = !preDbf && pic->getChromaFormat() == CHROMA_420 && sps.getBitDepth(CHANNEL_TYPE_LUMA) == 8 &&
                  sps.getBitDepth(CHANNEL_TYPE_CHROMA) == 8 && W % 8 == 0 && H % 8 == 0 &&
                  pic->getNumAllocatedSlice() == 1 && pic->getPicSym()->getNumTiles() == 1 &&
                  HM(self, TComSao_ctu_w) == 64 && HM(self, TComSao_ctu_h) == 64;
  if (!ok) {
    g.fell++;
    CAT(__real_, SAO_SYM)(self, pic, sliceEnabled, lambdas, testOff, rate, rateChroma, preDbf);
    return;
  }
  hvx_ctx *c = hvx_seam_ctx();
  const int nctu = HM(self, TComSao_n_ctus);
  // SAOProcess :243-249
  TComPicYuv *orgYuv = pic->getPicYuvOrg(), *resYuv = pic->getPicYuvRec();
  memcpy(HM(self, TEncSao_lambda), lambdas, sizeof(HM(self, TEncSao_lambda)));
  TComPicYuv *srcYuv = HM(self, TComSao_temp_yuv);
  resYuv->copyToPic(srcYuv);
  srcYuv->setBorderExtension(false);
  srcYuv->extendPicBorder();
  // :252 getStatistics -> hvx_sao_stats
  const size_t pb[3] = {(size_t)W * H, (size_t)(W / 2) * (H / 2), (size_t)(W / 2) * (H / 2)};
  for (int k = 0; k < 3; k++) {
    g.ensure(g.d_org[k], g.org_bytes[k], pb[k]);
    g.ensure(g.d_src[k], g.src_bytes[k], pb[k]);
    g.ensure(g.d_dst[k], g.dst_bytes[k], pb[k]);
  }
  g.ensure(g.d_stats, g.stats_bytes, (size_t)nctu * 15 * sizeof(hvx_sao_stat));
  g.ensure(g.d_params, g.params_bytes, (size_t)nctu * sizeof(hvx_sao_ctu));
  upload(orgYuv, g.d_org);
  upload(srcYuv, g.d_src);
  check(hvx_sao_stats(c, (const uint8_t *)g.d_org[0], (const uint8_t *)g.d_org[1], (const uint8_t *)g.d_org[2], W, W / 2,
                      (const uint8_t *)g.d_src[0], (const uint8_t *)g.d_src[1], (const uint8_t *)g.d_src[2], W, W / 2, W,
                      H, (hvx_sao_stat *)g.d_stats),
        "hvx_sao_stats");
  g.stats.resize((size_t)nctu * 15);
  check(hvx_download(c, g.stats.data(), g.d_stats, g.stats.size() * sizeof(hvx_sao_stat)), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  for (int u = 0; u < nctu; u++)
    for (int k = 0; k < 3; k++)
      for (int t = 0; t < NUM_SAO_NEW_TYPES; t++) {
        const hvx_sao_stat &s = g.stats[((size_t)u * 3 + k) * HVX_SAO_TYPES + t];
        SAOStatData &d = HM(self, TEncSao_stat)[u][k][t];
        for (int i = 0; i < MAX_NUM_SAO_CLASSES; i++) { d.diff[i] = s.diff[i]; d.count[i] = s.count[i]; }
      }
  // :257-262 the reference's decisions; its offsetCTU calls are recorded, not applied
  HM(self, TEncSao_decide_pic)(sliceEnabled, pic->getSlice(0)->getDepth(), rate, rateChroma);
  SAOBlkParam *reconParams = new SAOBlkParam[nctu];
  hvx_sao_ctu off;
  memset(&off, 0, sizeof(off));
  for (int k = 0; k < 3; k++) off.comp[k].type = HVX_SAO_OFF;
  g.params.assign(nctu, off);
  g.deferring = true;
  HM(self, TEncSao_decide_blk)(pic, sliceEnabled, HM(self, TEncSao_stat), srcYuv, resYuv, reconParams,
                        pic->getPicSym()->getSAOBlkParam(), testOff, rate, rateChroma);
  g.deferring = false;
  delete[] reconParams;
  // offsetCTU of every CTU -> hvx_sao_apply from the copy into the reconstruction
  check(hvx_upload(c, g.d_params, g.params.data(), (size_t)nctu * sizeof(hvx_sao_ctu)), "hvx_upload");
  check(hvx_sao_apply(c, (const uint8_t *)g.d_src[0], (const uint8_t *)g.d_src[1], (const uint8_t *)g.d_src[2], W, W / 2,
                      (uint8_t *)g.d_dst[0], (uint8_t *)g.d_dst[1], (uint8_t *)g.d_dst[2], W, W / 2, W, H,
                      (const hvx_sao_ctu *)g.d_params),
        "hvx_sao_apply");
  for (int k = 0; k < 3; k++) {
    g.host[k].resize(pb[k]);
    check(hvx_download(c, g.host[k].data(), g.d_dst[k], pb[k]), "hvx_download");
  }
  check(hvx_sync(c), "hvx_sync");
  for (int k = 0; k < 3; k++) {
    const ComponentID id = ComponentID(k);
    const int w = resYuv->getWidth(id), h = resYuv->getHeight(id), s = resYuv->getStride(id);
    Pel *dst = resYuv->getAddr(id);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst[y * s + x] = (Pel)g.host[k][(size_t)y * w + x];
  }
  g.pictures++;
}
