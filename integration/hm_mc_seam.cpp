// hm_mc_seam.cpp -- drop-in of the hvx motion compensation under an UNCHANGED HM-16.5rc1
// TAppEncoder.
//
// Linked into the reference encoder with -Wl,--wrap=<TComPrediction::motionCompensation>:
// every call TEncSearch / TEncCu make into the reference MC (TComPrediction.cpp:517; merge
// candidates, AMVP/bi-pred targets, final PU predictions) is served by libhvx.so on the
// MI355X through the C-ABI (hvx_mc_batch).  Reference pictures are uploaded once per
// (picture buffer, POC) -- they are final while they serve as references -- and each call
// ships its PU jobs, runs one hvx_mc_batch and copies the prediction into the TComYuv.
// Weighted prediction is not on the ported path and falls through to the reference.
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
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComPicYuv.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComYuv.h"
#include "hm_access.hpp"
#include "hvx.h"

#define MC_SYM _ZN14TComPrediction18motionCompensationEP10TComDataCUP7TComYuv10RefPicListi
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, MC_SYM)(TComPrediction *, TComDataCU *, TComYuv *, RefPicList, Int);

hvx_ctx *hvx_seam_ctx();  // shared with hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

struct DevPic {  // device copy of one reference picture's three planes
  const TComPicYuv *pic = nullptr;
  Int poc = -1 << 30;
  void *buf[3] = {};
  const int16_t *org[3] = {};
};

struct McSeam {
  std::vector<DevPic> pics;
  void *d_ptrs = nullptr, *d_jobs = nullptr, *d_out = nullptr;
  long long calls = 0, pus = 0;
  ~McSeam() { fprintf(stderr, "hm_mc_seam: %lld motionCompensation calls (%lld PUs) served by libhvx\n", calls, pus); }

  // device origin pointers of a reference picture (uploaded on first use for this POC)
  const DevPic &pic(TComPicYuv *p, Int poc) {
    for (auto &d : pics)
      if (d.pic == p && d.poc == poc) return d;
    DevPic *slot = nullptr;
    for (auto &d : pics)
      if (d.pic == p) slot = &d;  // the buffer now holds another picture: replace
    if (!slot) { pics.emplace_back(); slot = &pics.back(); }
    hvx_ctx *c = hvx_seam_ctx();
    for (int comp = 0; comp < 3; comp++) {
      const ComponentID id = ComponentID(comp);
      const size_t n = (size_t)p->getStride(id) * p->getTotalHeight(id);
      if (!slot->buf[comp]) check(hvx_alloc(c, n * sizeof(Pel), &slot->buf[comp]), "hvx_alloc");
      check(hvx_upload(c, slot->buf[comp], p->getBuf(id), n * sizeof(Pel)), "hvx_upload");
      slot->org[comp] = (const int16_t *)slot->buf[comp] + (p->getAddr(id) - p->getBuf(id));
    }
    slot->pic = p;
    slot->poc = poc;
    return *slot;
  }
};
McSeam g_mc;
}  // namespace

extern "C" void CAT(__wrap_, MC_SYM)(TComPrediction *self, TComDataCU *cu, TComYuv *pred, RefPicList list, Int partIdx) {
  TComSlice *sl = cu->getSlice();
  if (sl->getPPS()->getUseWP() || sl->getPPS()->getWPBiPred() || cu->getPic()->getChromaFormat() != CHROMA_420 ||
      sl->getSPS()->getBitDepth(CHANNEL_TYPE_LUMA) != 8) {
    CAT(__real_, MC_SYM)(self, cu, pred, list, partIdx);
    return;
  }
  hvx_ctx *c = hvx_seam_ctx();
  const int first = partIdx >= 0 ? partIdx : 0, last = partIdx >= 0 ? partIdx : cu->getNumPartitions() - 1;
  const TComSPS *sps = sl->getSPS();
  TComPicYuv *cur = cu->getPic()->getPicYuvRec();
  const Int ls = cur->getStride(COMPONENT_Y);
  std::vector<hvx_mc_job> jobs;
  std::vector<const int16_t *> ptrs;
  std::vector<UInt> addrs;
  std::vector<int64_t> offs;
  int64_t off = 0;
  for (int part = first; part <= last; part++) {
    UInt addr;
    Int w, h;
    cu->getPartIndexAndSize(part, addr, w, h);
    hvx_mc_job j;
    memset(&j, 0, sizeof(j));
    j.pic_w = sps->getPicWidthInLumaSamples();
    j.pic_h = sps->getPicHeightInLumaSamples();
    j.max_cu = sps->getMaxCUWidth();
    j.cu_x = cu->getCUPelX();
    j.cu_y = cu->getCUPelY();
    const Pel *pa = cur->getAddr(COMPONENT_Y, cu->getCtuRsAddr(), cu->getZorderIdxInCtu() + addr);
    const ptrdiff_t d = pa - cur->getAddr(COMPONENT_Y);
    j.pu_x = (int)(d % ls);
    j.pu_y = (int)(d / ls);
    j.w = w;
    j.h = h;
    for (int l = 0; l < 2; l++) {
      const RefPicList rl = l ? REF_PIC_LIST_1 : REF_PIC_LIST_0;
      const bool want = list == REF_PIC_LIST_X || list == rl;
      const Int ri = want ? cu->getCUMvField(rl)->getRefIdx(addr) : -1;
      j.ref[l] = -1;
      if (ri < 0) continue;
      TComPic *rp = sl->getRefPic(rl, ri);
      const DevPic &dp = g_mc.pic(rp->getPicYuvRec(), rp->getPOC());
      j.ref[l] = (int)ptrs.size() / 3;
      for (int comp = 0; comp < 3; comp++) ptrs.push_back(dp.org[comp]);
      j.poc[l] = rp->getPOC();
      const TComMv mv = cu->getCUMvField(rl)->getMv(addr);
      j.mv_x[l] = mv.getHor();
      j.mv_y[l] = mv.getVer();
    }
    // motionCompensation(list X) takes xCheckIdenticalMotion's shortcut in B slices without WP
    j.flags = (list == REF_PIC_LIST_X && sl->isInterB()) ? HVX_MC_B_SLICE : 0;
    j.dst_offset = off;
    offs.push_back(off);
    off += w * h + 2 * (w / 2) * (h / 2);
    jobs.push_back(j);
    addrs.push_back(addr);
  }
  // ptrs/jobs/out staging on the device (grown on demand: at most 4 PUs x 2 lists per call)
  static std::vector<int16_t> host_out;
  if (!g_mc.d_ptrs) {
    check(hvx_alloc(c, 24 * sizeof(void *), &g_mc.d_ptrs), "hvx_alloc");
    check(hvx_alloc(c, 4 * sizeof(hvx_mc_job), &g_mc.d_jobs), "hvx_alloc");
    check(hvx_alloc(c, 4 * 64 * 64 * 3 / 2 * sizeof(int16_t), &g_mc.d_out), "hvx_alloc");
  }
  host_out.resize((size_t)off);
  check(hvx_upload(c, g_mc.d_ptrs, ptrs.data(), ptrs.size() * sizeof(void *)), "hvx_upload");
  check(hvx_upload(c, g_mc.d_jobs, jobs.data(), jobs.size() * sizeof(hvx_mc_job)), "hvx_upload");
  check(hvx_mc_batch(c, (const int16_t *const *)g_mc.d_ptrs, ls, cur->getStride(COMPONENT_Cb),
                     (const hvx_mc_job *)g_mc.d_jobs, (int)jobs.size(), (int16_t *)g_mc.d_out), "hvx_mc_batch");
  check(hvx_download(c, host_out.data(), g_mc.d_out, (size_t)off * sizeof(int16_t)), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  for (size_t k = 0; k < jobs.size(); k++) {
    const hvx_mc_job &j = jobs[k];
    const int16_t *src = host_out.data() + offs[k];
    for (int comp = 0; comp < 3; comp++) {
      const ComponentID id = ComponentID(comp);
      const int w = comp ? j.w / 2 : j.w, h = comp ? j.h / 2 : j.h;
      Pel *dst = pred->getAddr(id, addrs[k]);
      const UInt st = pred->getStride(id);
      for (int y = 0; y < h; y++) memcpy(dst + y * st, src + y * w, w * sizeof(Pel));
      src += w * h;
    }
  }
  g_mc.calls++;
  g_mc.pus += (long long)jobs.size();
}
