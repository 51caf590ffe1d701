// hm_lf_seam.cpp -- drop-in of the hvx deblocking filter under an UNCHANGED HM-16.5rc1 TAppEncoder.
//
// Linked into the reference encoder with -Wl,--wrap=<TComLoopFilter::loopFilterPic>: every
// picture TEncGOP deblocks (TEncGOP.cpp:1465) is filtered by libhvx.so on the MI355X through the
// C-ABI (hvx_deblock) instead of the reference's loop filter.  The host side is what HM already
// derives per CU: the boundary strength of every 4x4 unit's left/top edge (the reference's own
// xSetLoopfilterParam / xSetEdgefilterTU / xSetEdgefilterPU / xGetBoundaryStrengthSingle, run on
// a private TComLoopFilter object while walking each CTU's CU tree as xDeblockCU does) and each
// unit's QP.  The three planes go to the device once per picture (8-bit), are filtered in place
// and come back into the TComPicYuv.  Pictures with PCM/transquant-bypass units fall through.
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
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComLoopFilter.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComPicYuv.h"
#include "TLibCommon/TComSlice.h"
#include "hm_access.hpp"
#include "hvx.h"

#define LF_SYM _ZN14TComLoopFilter13loopFilterPicEP7TComPic
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, LF_SYM)(TComLoopFilter *, TComPic *);

hvx_ctx *hvx_seam_ctx();  // shared with hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

// the boundary-strength walk of xDeblockCU (TComLoopFilter.cpp:170-218), without the filtering
void bs_walk(TComLoopFilter &lf, TComDataCU *cu, UInt abs, UInt depth, DeblockEdgeDir dir) {
  if (cu->getPic() == 0 || cu->getPartitionSize(abs) == NUMBER_OF_PART_SIZES) return;
  TComPic *pic = cu->getPic();
  const UInt cur = pic->getNumPartitionsInCtu() >> (depth << 1), q = cur >> 2;
  const TComSPS &sps = *(cu->getSlice()->getSPS());
  if (cu->getDepth(abs) > depth) {
    for (UInt k = 0; k < 4; k++, abs += q) {
      const UInt x = cu->getCUPelX() + g_auiRasterToPelX[g_auiZscanToRaster[abs]];
      const UInt y = cu->getCUPelY() + g_auiRasterToPelY[g_auiZscanToRaster[abs]];
      if (x < sps.getPicWidthInLumaSamples() && y < sps.getPicHeightInLumaSamples()) bs_walk(lf, cu, abs, depth + 1, dir);
    }
    return;
  }
  HM(&lf, TComLoopFilter_set_param)(cu, abs);
  TComTURecurse tu(cu, abs);
  HM(&lf, TComLoopFilter_set_tu)(tu);
  HM(&lf, TComLoopFilter_set_pu)(cu, abs);
  const UInt pels = sps.getMaxCUWidth() >> sps.getMaxTotalCUDepth();
  for (UInt p = abs; p < abs + cur; p++) {
    const UInt chk = pels == 4 ? ((dir == EDGE_VER && p % 2 == 0) || (dir == EDGE_HOR && (p - ((p >> 2) << 2)) / 2 == 0)) : 1;
    if (HM(&lf, TComLoopFilter_edge)[dir][p] && chk) HM(&lf, TComLoopFilter_bs_single)(cu, dir, p);
  }
}

struct LfSeam {
  void *d_plane[3] = {}, *d_map[3] = {};
  size_t plane_bytes[3] = {}, map_bytes[3] = {};
  std::vector<uint8_t> host[3], bs[2];
  std::vector<int8_t> qp;
  long long pictures = 0, fell = 0;
  ~LfSeam() { fprintf(stderr, "hm_lf_seam: %lld pictures deblocked by libhvx, %lld fell through\n", pictures, fell); }
  void ensure(void *&p, size_t &have, size_t need) {
    if (have >= need) return;
    if (p) check(hvx_free(hvx_seam_ctx(), p), "hvx_free");
    check(hvx_alloc(hvx_seam_ctx(), need, &p), "hvx_alloc");
    have = need;
  }
};
LfSeam g;
}  // namespace

extern "C" void CAT(__wrap_, LF_SYM)(TComLoopFilter *self, TComPic *pic) {
  TComSlice *sl = pic->getSlice(0);
  const TComSPS &sps = *sl->getSPS();
  const TComPPS &pps = *sl->getPPS();
  const int W = sps.getPicWidthInLumaSamples(), H = sps.getPicHeightInLumaSamples();
  bool ok = W % 8 == 0 && H % 8 == 0 && !pps.getTransquantBypassEnableFlag() && !sps.getUsePCM() &&
            pic->getChromaFormat() == CHROMA_420 && sps.getBitDepth(CHANNEL_TYPE_LUMA) == 8 &&
            sps.getBitDepth(CHANNEL_TYPE_CHROMA) == 8 && pic->getNumAllocatedSlice() == 1;
  if (!ok) {
    g.fell++;
    CAT(__real_, LF_SYM)(self, pic);
    return;
  }
  hvx_ctx *c = hvx_seam_ctx();
  const int uw = W / 4, uh = H / 4;
  // 1. BS / QP maps from the CU data (the reference's own derivation)
  for (int d = 0; d < 2; d++) g.bs[d].assign((size_t)uw * uh, 0);
  g.qp.assign((size_t)uw * uh, 0);
  {
    TComLoopFilter lf;
    lf.create(sps.getMaxTotalCUDepth());
    lf.setCfg(HM(self, TComLoopFilter_cross_tile));
    const int ctu_w = sps.getMaxCUWidth(), ctus_x = (W + ctu_w - 1) / ctu_w;
    for (int dir = 0; dir < 2; dir++)
      for (UInt a = 0; a < pic->getNumberOfCtusInFrame(); a++) {
        TComDataCU *ctu = pic->getCtu(a);
        memset(HM(&lf, TComLoopFilter_bs)[dir], 0, HM(&lf, TComLoopFilter_n_parts));
        memset(HM(&lf, TComLoopFilter_edge)[dir], 0, HM(&lf, TComLoopFilter_n_parts));
        bs_walk(lf, ctu, 0, 0, (DeblockEdgeDir)dir);
        const int x0 = (a % ctus_x) * ctu_w, y0 = (a / ctus_x) * ctu_w;
        for (UInt p = 0; p < HM(&lf, TComLoopFilter_n_parts); p++) {
          const int x = x0 + g_auiRasterToPelX[g_auiZscanToRaster[p]], y = y0 + g_auiRasterToPelY[g_auiZscanToRaster[p]];
          if (x >= W || y >= H) continue;
          g.bs[dir][(y / 4) * uw + x / 4] = HM(&lf, TComLoopFilter_bs)[dir][p];
          if (dir == 0) g.qp[(y / 4) * uw + x / 4] = (int8_t)ctu->getQP(p);
        }
      }
    lf.destroy();
  }
  // 2. planes to the device (8-bit, stride = width), deblock in place, back into the picture
  TComPicYuv *rec = pic->getPicYuvRec();
  for (int k = 0; k < 3; k++) {
    const ComponentID id = ComponentID(k);
    const int w = rec->getWidth(id), h = rec->getHeight(id), s = rec->getStride(id);
    const Pel *src = rec->getAddr(id);
    g.host[k].resize((size_t)w * h);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) g.host[k][(size_t)y * w + x] = (uint8_t)src[y * s + x];
    g.ensure(g.d_plane[k], g.plane_bytes[k], g.host[k].size());
    check(hvx_upload(c, g.d_plane[k], g.host[k].data(), g.host[k].size()), "hvx_upload");
  }
  for (int k = 0; k < 3; k++) g.ensure(g.d_map[k], g.map_bytes[k], (size_t)uw * uh);
  check(hvx_upload(c, g.d_map[0], g.bs[EDGE_VER].data(), (size_t)uw * uh), "hvx_upload");
  check(hvx_upload(c, g.d_map[1], g.bs[EDGE_HOR].data(), (size_t)uw * uh), "hvx_upload");
  check(hvx_upload(c, g.d_map[2], g.qp.data(), (size_t)uw * uh), "hvx_upload");
  hvx_deblock_params dp = {W, H, sl->getDeblockingFilterBetaOffsetDiv2(), sl->getDeblockingFilterTcOffsetDiv2(),
                           pps.getQpOffset(COMPONENT_Cb), pps.getQpOffset(COMPONENT_Cr), 0, 0};
  if (sl->getDeblockingFilterDisable()) {  // bs maps are all zero then; nothing to do
    check(hvx_sync(c), "hvx_sync");
    g.pictures++;
    return;
  }
  check(hvx_deblock(c, (uint8_t *)g.d_plane[0], W, (uint8_t *)g.d_plane[1], (uint8_t *)g.d_plane[2], W / 2,
                    (const uint8_t *)g.d_map[0], (const uint8_t *)g.d_map[1], (const int8_t *)g.d_map[2], &dp),
        "hvx_deblock");
  for (int k = 0; k < 3; k++) check(hvx_download(c, g.host[k].data(), g.d_plane[k], g.host[k].size()), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  for (int k = 0; k < 3; k++) {
    const ComponentID id = ComponentID(k);
    const int w = rec->getWidth(id), h = rec->getHeight(id), s = rec->getStride(id);
    Pel *dst = rec->getAddr(id);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst[y * s + x] = (Pel)g.host[k][(size_t)y * w + x];
  }
  g.pictures++;
}
