// deblock_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_dbkcap) with -Wl,--wrap=<TComLoopFilter::loopFilterPic>.  For each of the
// first pictures TEncGOP deblocks (TEncGOP.cpp:1465) it records
//   * the reconstruction before and after the reference's loopFilterPic (TComLoopFilter.cpp:130),
//     Y, Cb, Cr (8-bit video);
//   * the boundary strength every 4x4 luma unit's left (vertical) and top (horizontal) edge gets,
//     exactly as xEdgeFilterLuma/Chroma read it (m_aapucBS): derived by a SEPARATE TComLoopFilter
//     object through the reference's own xSetLoopfilterParam, xSetEdgefilterTU, xSetEdgefilterPU
//     and xGetBoundaryStrengthSingle (TComLoopFilter.cpp:195-218), walking each CTU's CU tree as
//     xDeblockCU does (:170-193) -- the encoder's own loop filter is not touched;
//   * each unit's QP (TComDataCU::getQP) and the slice's beta/tc offsets and chroma QP offsets.
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
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComLoopFilter.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComSlice.h"
#undef private
#undef protected
#include "golden_writer.h"

#define LF_SYM _ZN14TComLoopFilter13loopFilterPicEP7TComPic
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, LF_SYM)(TComLoopFilter *, TComPic *);

namespace {
struct Store {
  std::vector<int32_t> meta;  // per picture: w, h, beta_offset_div2, tc_offset_div2, cb_qp_offset, cr_qp_offset, bypass
  std::vector<uint8_t> pre, post, bs_ver, bs_hor;
  std::vector<int8_t> qp;
  std::vector<int32_t> poc;
  int n = 0;
  ~Store() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out) return;
    GoldenWriter gw;
    gw.add("meta", "i32", {(uint32_t)n, 7}, meta);
    gw.add("pre", "u8", {(uint32_t)pre.size()}, pre);    // per picture: Y w*h, Cb, Cr (w/2)*(h/2)
    gw.add("post", "u8", {(uint32_t)post.size()}, post);
    gw.add("bs_ver", "u8", {(uint32_t)bs_ver.size()}, bs_ver);  // per picture: (w/4)*(h/4), raster
    gw.add("bs_hor", "u8", {(uint32_t)bs_hor.size()}, bs_hor);
    gw.add("qp", "i8", {(uint32_t)qp.size()}, qp);
    gw.add("poc", "i32", {(uint32_t)n}, poc);
    gw.write(out);
    fprintf(stderr, "deblock_capture: %d pictures\n", n);
  }
};
Store g;

void planes(TComPic *pic, std::vector<uint8_t> &dst) {
  TComPicYuv *rec = pic->getPicYuvRec();
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int w = rec->getWidth(id), h = rec->getHeight(id), s = rec->getStride(id);
    const Pel *p = rec->getAddr(id);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst.push_back((uint8_t)p[y * s + x]);
  }
}

// xDeblockCU's walk (TComLoopFilter.cpp:170-218) without the filtering: the BS of every part
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
  lf.xSetLoopfilterParam(cu, abs);
  TComTURecurse tu(cu, abs);
  lf.xSetEdgefilterTU(tu);
  lf.xSetEdgefilterPU(cu, abs);
  const UInt pels = sps.getMaxCUWidth() >> sps.getMaxTotalCUDepth();
  for (UInt p = abs; p < abs + cur; p++) {
    const UInt check = pels == 4 ? ((dir == EDGE_VER && p % 2 == 0) || (dir == EDGE_HOR && (p - ((p >> 2) << 2)) / 2 == 0)) : 1;
    if (lf.m_aapbEdgeFilter[dir][p] && check) lf.xGetBoundaryStrengthSingle(cu, dir, p);
  }
}
// HVX_CAPTURE_POCS=<poc,poc,...>: record the pictures of these POCs (default: the first two deblocked)
bool keep_picture(int poc) {
  const char *s = getenv("HVX_CAPTURE_POCS");
  if (!s || !*s) return g.n < 2;
  for (const char *p = s; *p;) {
    char *end;
    const long v = strtol(p, &end, 10);
    if (end == p) break;
    if (v == poc) return true;
    p = *end ? end + 1 : end;
  }
  return false;
}
}  // namespace

extern "C" void CAT(__wrap_, LF_SYM)(TComLoopFilter *self, TComPic *pic) {
  const bool keep = keep_picture(pic->getPOC());
  if (keep) {
    TComSlice *sl = pic->getSlice(0);
    const TComSPS &sps = *sl->getSPS();
    const TComPPS &pps = *sl->getPPS();
    const int W = sps.getPicWidthInLumaSamples(), H = sps.getPicHeightInLumaSamples(), uw = W / 4, uh = H / 4;
    g.meta.insert(g.meta.end(), {W, H, sl->getDeblockingFilterBetaOffsetDiv2(), sl->getDeblockingFilterTcOffsetDiv2(),
                                 pps.getQpOffset(COMPONENT_Cb), pps.getQpOffset(COMPONENT_Cr),
                                 pps.getTransquantBypassEnableFlag() ? 1 : 0});
    g.poc.push_back(pic->getPOC());
    planes(pic, g.pre);
    std::vector<uint8_t> bs[2] = {std::vector<uint8_t>(uw * uh, 0), std::vector<uint8_t>(uw * uh, 0)};
    std::vector<int8_t> qp(uw * uh, 0);
    TComLoopFilter lf;
    lf.create(sps.getMaxTotalCUDepth());
    lf.setCfg(self->m_bLFCrossTileBoundary);
    const int ctu_w = sps.getMaxCUWidth(), ctus_x = (W + ctu_w - 1) / ctu_w;
    for (int dir = 0; dir < 2; dir++)
      for (UInt a = 0; a < pic->getNumberOfCtusInFrame(); a++) {
        TComDataCU *ctu = pic->getCtu(a);
        memset(lf.m_aapucBS[dir], 0, lf.m_uiNumPartitions);
        memset(lf.m_aapbEdgeFilter[dir], 0, lf.m_uiNumPartitions);
        bs_walk(lf, ctu, 0, 0, (DeblockEdgeDir)dir);
        const int x0 = (a % ctus_x) * ctu_w, y0 = (a / ctus_x) * ctu_w;
        for (UInt p = 0; p < lf.m_uiNumPartitions; p++) {
          const int x = x0 + g_auiRasterToPelX[g_auiZscanToRaster[p]], y = y0 + g_auiRasterToPelY[g_auiZscanToRaster[p]];
          if (x >= W || y >= H) continue;
          // only the 8x8 edge grid is filtered (xEdgeFilterLuma's iEdge step, :220): keep those
          const bool on_grid = dir == EDGE_VER ? (x % 8 == 0) : (y % 8 == 0);
          bs[dir][(y / 4) * uw + x / 4] = on_grid ? lf.m_aapucBS[dir][p] : 0;
          if (dir == 0) qp[(y / 4) * uw + x / 4] = (int8_t)ctu->getQP(p);
        }
      }
    lf.destroy();
    g.bs_ver.insert(g.bs_ver.end(), bs[EDGE_VER].begin(), bs[EDGE_VER].end());
    g.bs_hor.insert(g.bs_hor.end(), bs[EDGE_HOR].begin(), bs[EDGE_HOR].end());
    g.qp.insert(g.qp.end(), qp.begin(), qp.end());
  }
  CAT(__real_, LF_SYM)(self, pic);
  if (keep) {
    planes(pic, g.post);
    g.n++;
  }
}
