// hm_cu_seam.cpp -- drop-in of the HM-exact CTU decision (hvx_hm_compress) under an UNCHANGED
// HM-16.5rc1 TAppEncoder: the L3 boundary of SURVEY.md section 1.
//
// Replaces TEncCu::compressCtu (TEncCu.cpp:228, called once per CTU by TEncSlice::compressSlice,
// TEncSlice.cpp:814).  Per picture (first CTU of a new POC) the seam describes the picture to the
// device once (hvx_hm_picture: slice / RD scalars as initEncSlice and setUpLambda left them in
// TComSlice / TComRdCost / TComTrQuant, the original, the reference pictures' reconstructions as
// padded 8-bit and int16 planes, the collocated picture's motion field for TMVP, an empty
// reconstruction and CTU array).  Per CTU it sends one chained job (one wave): the RD coder the
// decision starts from (m_pppcRDSbacCoder[0][CI_CURR_BEST]: context states and m_fracBits) and
// TEncSearch::m_integerMv2Nx2N; the device decides the CTU exactly as xCompressCU, writes it into
// its picture (the neighbourhood of the next CTU) and returns the CTU data.  The seam then writes
// what copyToPic would have written into the picture's TComDataCU (per 4x4 partition: depth,
// width, partition size, prediction mode, skip / merge, motion, MVDs, MVP indices, intra modes,
// transform index / skip, CBFs, QP; the coefficients; total bits / distortion / cost) and the
// reconstruction into TComPicYuv rec (xCopyYuv2Pic).  HM's own encodeCtu, loop filters, SAO and
// slice writer then run on that data unchanged.
//
// Served: I, P and B slices (the engine's tool set: HM's lowdelay_P / randomaccess settings, 4:2:0
// 8-bit, CTU 64, no dQP / TQ bypass / RDPCM / cross-component prediction / weighted prediction / PCM /
// rate control / adaptive search range); anything else falls through to the reference's
// compressCtu (counted).  HVX_SEAM_CU=1 enables the seam.
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
#include "TLibCommon/ContextModel.h"
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibEncoder/TEncCfg.h"
#include "TLibEncoder/TEncCu.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#include "hm_access.hpp"
#include "hvx.h"

#define CU_SYM _ZN6TEncCu11compressCtuEP10TComDataCU
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, CU_SYM)(TEncCu *, TComDataCU *);
hvx_ctx *hvx_seam_ctx();  // hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

const int kM8 = HVX_PLANE_MARGIN, kM16 = 80, kM16C = 40;

struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  void *get(size_t bytes) {
    if (bytes > n) {
      if (p) check(hvx_free(hvx_seam_ctx(), p), "hvx_free");
      check(hvx_alloc(hvx_seam_ctx(), bytes, &p), "hvx_alloc");
      n = bytes;
    }
    return p;
  }
};

// A reference picture's planes as the engine reads them (hm.DeviceFrame): 8-bit luma with
// HVX_PLANE_MARGIN, int16 Y / Cb / Cr with 80 / 40 samples of border (TComPicYuv::extendPicBorder
// replicates the edge samples, as HM's own reconstruction borders do)
struct RefPlanes {
  int poc = -1;
  DevBuf y8, p16[3];
  int s8 = 0, s16[2] = {0, 0};
  const uint8_t *o8 = nullptr;
  const int16_t *o16[3] = {nullptr, nullptr, nullptr};
};

struct CuSeam {
  int enabled = -1, batch = -1;
  long long served = 0, fallback = 0, pictures = 0, batched = 0, launches = 0, state_mismatch = 0;
  int cur_poc = -1000000;
  bool cur_ok = false;
  int w = 0, h = 0, wc = 0, hc = 0;
  DevBuf org[3], rec[3], ctus, col, eb, pic, job, state, out_ctu, out_rec, out_cod;
  // batched mode: every chain of the picture decided by one launch at its first compressCtu call
  bool pic_batched = false;
  std::vector<hvx_hm_ctu> b_ctu;
  std::vector<uint8_t> b_rec;
  std::vector<hvx_hm_coder> b_cod;
  std::vector<uint8_t> slice_first;  // per CTU: a slice starts here (the entry state is resetEntropy's)
  std::vector<RefPlanes> refs = std::vector<RefPlanes>(8);
  hvx_hm_picture P;
  std::vector<uint8_t> stage;
  ~CuSeam() {
    if (enabled == 1)
      fprintf(stderr, "hm_cu_seam: %lld compressCtu calls served by libhvx (%lld pictures), %lld fell through\n", served,
              pictures, fallback);
    if (enabled == 1 && batch == 1)
      fprintf(stderr, "hm_cu_seam batched: %lld CTUs from %lld launches, %lld entry-state mismatches\n", batched, launches,
              state_mismatch);
  }
  bool on() {
    if (enabled < 0) {
      const char *e = getenv("HVX_SEAM_CU");
      enabled = (e && e[0] == '1') ? 1 : 0;
    }
    if (batch < 0) {
      const char *e = getenv("HVX_SEAM_CU_BATCH");
      batch = (e && e[0] == '1') ? 1 : 0;
    }
    return enabled == 1;
  }
};
CuSeam g;

void upload(void *d, const void *h, size_t n) { check(hvx_upload(hvx_seam_ctx(), d, h, n), "hvx_upload"); }

// pad a plane of Pel into an 8-bit or int16 buffer with margin m (edge replication)
template <class T>
void pad_plane(const Pel *src, int stride, int w, int h, int m, std::vector<uint8_t> &out, int &pstride) {
  pstride = w + 2 * m;
  if (sizeof(T) == 1) pstride = (pstride + 3) & ~3;  // ref8_stride: a multiple of 4
  out.assign((size_t)pstride * (h + 2 * m) * sizeof(T), 0);
  T *o = (T *)out.data();
  for (int y = -m; y < h + m; y++) {
    const int sy = std::min(std::max(y, 0), h - 1);
    T *row = o + (size_t)(y + m) * pstride;
    for (int x = -m; x < w + m; x++) row[x + m] = (T)src[sy * stride + std::min(std::max(x, 0), w - 1)];
  }
}

const RefPlanes &ref_planes(int slot, TComPic *pic) {
  RefPlanes &r = g.refs[slot];
  if (r.poc == pic->getPOC()) return r;
  TComPicYuv *y = pic->getPicYuvRec();
  r.poc = pic->getPOC();
  int ps = 0;
  pad_plane<uint8_t>(y->getAddr(COMPONENT_Y), y->getStride(COMPONENT_Y), g.w, g.h, kM8, g.stage, ps);
  uint8_t *d8 = (uint8_t *)r.y8.get(g.stage.size());
  upload(d8, g.stage.data(), g.stage.size());
  r.s8 = ps;
  r.o8 = d8 + (size_t)kM8 * ps + kM8;
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int m = c ? kM16C : kM16, cw = c ? g.w / 2 : g.w, ch = c ? g.h / 2 : g.h;
    pad_plane<int16_t>(y->getAddr(id), y->getStride(id), cw, ch, m, g.stage, ps);
    int16_t *d16 = (int16_t *)r.p16[c].get(g.stage.size());
    upload(d16, g.stage.data(), g.stage.size());
    r.s16[c ? 1 : 0] = ps;
    r.o16[c] = d16 + (size_t)m * ps + m;
  }
  return r;
}

// the picture description (cu_capture.cpp records the same fields from the same objects)
bool begin_picture(TEncCu *cu, TComDataCU *ctu) {
  TComPic *pic = ctu->getPic();
  TComSlice *s = ctu->getSlice();
  const TComSPS &sps = *s->getSPS();
  const TComPPS &pps = *s->getPPS();
  const int st = s->getSliceType();
  const bool ok = (st == I_SLICE || st == P_SLICE || st == B_SLICE) && sps.getChromaFormatIdc() == CHROMA_420 &&
                  sps.getBitDepth(CHANNEL_TYPE_LUMA) == 8 && sps.getBitDepth(CHANNEL_TYPE_CHROMA) == 8 &&
                  sps.getMaxCUWidth() == 64 && sps.getMaxCUHeight() == 64 && sps.getMaxTotalCUDepth() == 4 &&
                  !pps.getUseDQP() && !pps.getTransquantBypassEnableFlag() && !pps.getUseWP() &&
                  !pps.getWPBiPred() && !s->getUseChromaQpAdj() && s->getNumRefIdx(REF_PIC_LIST_0) <= 4 &&
                  (st != B_SLICE || s->getNumRefIdx(REF_PIC_LIST_1) <= 4) && !sps.getUsePCM() &&
                  pic->getPicSym()->getNumTiles() == 1 && !sps.getScalingListFlag() &&
                  sps.getQuadtreeTULog2MaxSize() == 5 && sps.getQuadtreeTULog2MinSize() == 2 &&
                  sps.getQuadtreeTUMaxDepthInter() == 3 && sps.getQuadtreeTUMaxDepthIntra() == 3 &&
                  sps.getUseStrongIntraSmoothing() && !pps.getConstrainedIntraPred() && pps.getSignHideFlag() &&
                  pps.getUseTransformSkip() && pps.getPpsRangeExtension().getLog2MaxTransformSkipBlockSize() == 2;
  // the encoder tool set the engine decides with (encoder_lowdelay_P_main.cfg's search and RD options)
  TEncCfg *cfg = HM(cu, TEncCu_cfg);
  const bool tools = cfg->getUseRDOQ() && cfg->getUseRDOQTS() && !cfg->getUseSelectiveRDOQ() && cfg->getFastSearch() == 1 &&
                     cfg->getUseHADME() && cfg->getUseFastEnc() && cfg->getUseFastDecisionForMerge() &&
                     !cfg->getUseEarlySkipDetection() && !cfg->getUseCbfFastMode() && !cfg->getUseEarlyCU() &&
                     cfg->getUseTransformSkipFast() && !cfg->getUseAdaptQpSelect() && !cfg->getUseRateCtrl() &&
                     !cfg->getUsePCM() && !cfg->getUseASR() && !cfg->getUseAdaptiveQP() &&
                     cfg->getFastMEForGenBLowDelayEnabled() && !cfg->getClipForBiPredMeEnabled();
  if (!ok || !tools) return false;
  g.w = sps.getPicWidthInLumaSamples();
  g.h = sps.getPicHeightInLumaSamples();
  g.wc = (g.w + 63) / 64;
  g.hc = (g.h + 63) / 64;
  hvx_hm_picture &P = g.P;
  memset(&P, 0, sizeof(P));
  P.w = g.w; P.h = g.h; P.w_ctus = g.wc; P.h_ctus = g.hc;
  P.poc = s->getPOC();
  P.slice_type = st;
  P.qp = s->getSliceQp();
  // reference lists: list 0's pictures take planes 0.., a list-1 picture list 0 does not hold the next one
  const int nref = st == I_SLICE ? 0 : s->getNumRefIdx(REF_PIC_LIST_0);
  const int nref1 = st == B_SLICE ? s->getNumRefIdx(REF_PIC_LIST_1) : 0;
  P.nref[0] = nref;
  P.nref[1] = nref1;
  TComPic *plane_pic[8] = {};
  int nplanes = 0;
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < 4; i++) {
      const int n = l ? nref1 : nref;
      P.ref_poc[l][i] = i < n ? s->getRefPOC(RefPicList(l), i) : 0;
      P.ref_plane[l][i] = 0;
      if (i >= n) continue;
      TComPic *rp = s->getRefPic(RefPicList(l), i);
      int k = 0;
      while (k < nplanes && plane_pic[k]->getPOC() != rp->getPOC()) k++;
      if (k == nplanes) plane_pic[nplanes++] = rp;
      P.ref_plane[l][i] = k;
    }
  P.mvd_l1_zero = st == B_SLICE && s->getMvdL1ZeroFlag();
  for (int i = 0; i < 4; i++) P.l1_to_l0[i] = (st == B_SLICE && i < nref1) ? s->getList1IdxToList0Idx(i) : -1;
  P.bipred_range = HM(HM(cu, TEncCu_search), TEncSearch_bipred_range);
  for (int c = 1; c < 3; c++) {
    const QpParam q(*ctu, ComponentID(c));  // getScaledChromaQP of the slice QP
    P.chroma_qp[c - 1] = q.Qp;
  }
  P.max_merge = s->getMaxNumMergeCand();
  P.tmvp = s->getEnableTMVPFlag();
  P.check_ldc = s->getCheckLDC();
  P.col_from_l0 = s->getColFromL0Flag();
  P.search_range = HM(cu, TEncCu_cfg)->getSearchRange();
  P.amp = sps.getUseAMP();
  P.lambda_motion = HM(HM(cu, TEncCu_rdcost), TComRdCost_lambda_motion_sad)[0];
  P.lambda = HM(cu, TEncCu_rdcost)->getLambda();
  P.sqrt_lambda = HM(HM(cu, TEncCu_rdcost), TComRdCost_sqrt_lambda);
  P.chroma_weight[0] = HM(HM(cu, TEncCu_rdcost), TComRdCost_dist_weight)[1];
  P.chroma_weight[1] = HM(HM(cu, TEncCu_rdcost), TComRdCost_dist_weight)[2];
  for (int c = 0; c < 3; c++) P.tq_lambda[c] = HM(HM(cu, TEncCu_trquant), TComTrQuant_lambdas)[c];
  // the original (8-bit planes, stride = width)
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    TComPicYuv *o = pic->getPicYuvOrg();
    const int cw = c ? g.w / 2 : g.w, ch = c ? g.h / 2 : g.h;
    g.stage.resize((size_t)cw * ch);
    for (int y = 0; y < ch; y++)
      for (int x = 0; x < cw; x++) g.stage[(size_t)y * cw + x] = (uint8_t)o->getAddr(id)[y * o->getStride(id) + x];
    void *d = g.org[c].get(g.stage.size());
    upload(d, g.stage.data(), g.stage.size());
    P.org[c] = (const uint8_t *)d;
  }
  P.org_stride[0] = g.w;
  P.org_stride[1] = g.w / 2;
  // the reconstruction the chained jobs write (whole CTUs) and the CTU array, both empty
  const int rw = g.wc * 64, rh = g.hc * 64;
  for (int c = 0; c < 3; c++) {
    const size_t n = (size_t)(c ? rw / 2 : rw) * (c ? rh / 2 : rh);
    g.stage.assign(n, 0);
    void *d = g.rec[c].get(n);
    upload(d, g.stage.data(), n);
    P.rec[c] = (uint8_t *)d;
  }
  P.rec_stride[0] = rw;
  P.rec_stride[1] = rw / 2;
  const size_t nct = (size_t)g.wc * g.hc * sizeof(hvx_hm_ctu);
  g.stage.assign(nct, 0);
  void *dct = g.ctus.get(nct);
  upload(dct, g.stage.data(), nct);
  P.ctus = (hvx_hm_ctu *)dct;
  // references: the reconstructed (loop-filtered) reference pictures of both lists
  for (int i = 0; i < nplanes; i++) {
    const RefPlanes &r = ref_planes(i, plane_pic[i]);
    P.ref8[i] = r.o8;
    P.ref8_stride = r.s8;
    for (int c = 0; c < 3; c++) P.ref16[i][c] = r.o16[c];
    P.ref16_stride[0] = r.s16[0];
    P.ref16_stride[1] = r.s16[1];
  }
  // the collocated picture's compressed motion field (xGetColMVP, TComDataCU.cpp:3061)
  if (st != I_SLICE && s->getEnableTMVPFlag()) {
    TComPic *colp = s->getRefPic(RefPicList(s->isInterB() ? 1 - s->getColFromL0Flag() : 0), s->getColRefIdx());
    TComSlice *cs = colp->getSlice(0);
    P.col_valid = 1;
    P.col_poc = cs->getPOC();
    const int cst = cs->getSliceType();
    for (int l = 0; l < 2; l++) {
      const int n = cst == I_SLICE ? 0 : (l == 1 && cst == P_SLICE ? 0 : cs->getNumRefIdx(RefPicList(l)));
      for (int i = 0; i < 4; i++) P.col_ref_poc[l][i] = i < n ? cs->getRefPOC(RefPicList(l), i) : -1;
    }
    const int nctu = colp->getPicSym()->getNumberOfCtusInFrame();
    std::vector<int16_t> f;
    f.reserve((size_t)nctu * 16 * 8);
    for (int a = 0; a < nctu; a++) {
      TComDataCU *cc = colp->getCtu(a);
      for (int z = 0; z < 256; z += 16) {
        const int ps = cc->getPartitionSize(z);
        f.push_back((int16_t)(ps == NUMBER_OF_PART_SIZES ? -1 : cc->getPredictionMode(z)));
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getRefIdx(z));
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getRefIdx(z));
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getMv(z).getHor());
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getMv(z).getVer());
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getMv(z).getHor());
        f.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getMv(z).getVer());
        f.push_back(0);
      }
    }
    void *d = g.col.get(f.size() * sizeof(int16_t));
    upload(d, f.data(), f.size() * sizeof(int16_t));
    P.col_field = (const int16_t *)d;
  }
  // ContextModel::m_entropyBits (the counter's rate table)
  int32_t ebits[128];
  for (int i = 0; i < 128; i++) {  // m_entropyBits[state byte i], through a model in that state
    ContextModel m;
    hm_set_ctx_state(m, (UChar)i);
    ebits[i] = (int32_t)m.getEntropyBits(0);
  }
  void *deb = g.eb.get(sizeof(ebits));
  upload(deb, ebits, sizeof(ebits));
  P.entropy_bits = (const int32_t *)deb;
  upload(g.pic.get(sizeof(P)), &P, sizeof(P));
  size_t sb = 0;
  check(hvx_hm_state_size(&sb), "hvx_hm_state_size");
  g.state.get(sb);
  g.job.get(sizeof(hvx_hm_job));
  g.out_ctu.get(sizeof(hvx_hm_ctu));
  g.out_rec.get(6144);
  g.pictures++;
  return true;
}

// what TComDataCU::copyToPic (TComDataCU.cpp:945) writes for the decided CTU
void write_ctu(TComDataCU *ctu, const hvx_hm_ctu &o) {
  for (int z = 0; z < 256; z++) {
    const hvx_hm_part &p = o.p[z];
    ctu->getDepth()[z] = (UChar)p.depth;
    ctu->getWidth()[z] = ctu->getHeight()[z] = p.width;
    ctu->getPartitionSize()[z] = p.part;
    ctu->getPredictionMode()[z] = p.pred;
    ctu->getSkipFlag()[z] = p.skip != 0;
    ctu->getMergeFlag()[z] = p.merge != 0;
    ctu->getMergeIndex()[z] = (UChar)p.merge_idx;
    ctu->getInterDir()[z] = (UChar)p.inter_dir;
    for (int l = 0; l < 2; l++) {
      TComCUMvField *f = ctu->getCUMvField(RefPicList(l));
      const_cast<TComMv &>(f->getMv(z)) = TComMv(p.mv[l][0], p.mv[l][1]);
      const_cast<TComMv &>(f->getMvd(z)) = TComMv(p.mvd[l][0], p.mvd[l][1]);
      HM(f, TComCUMvField_ref_idx)[z] = p.ref[l];
      ctu->getMVPIdx(RefPicList(l))[z] = p.mvp_idx[l];
      ctu->getMVPNum(RefPicList(l))[z] = p.mvp_num[l];
    }
    ctu->getIntraDir(CHANNEL_TYPE_LUMA)[z] = p.idir[0];
    ctu->getIntraDir(CHANNEL_TYPE_CHROMA)[z] = p.idir[1];
    ctu->getTransformIdx()[z] = (UChar)p.tr_idx;
    for (int c = 0; c < 3; c++) {
      ctu->getTransformSkip(ComponentID(c))[z] = p.ts[c];
      ctu->getCbf(ComponentID(c))[z] = p.cbf[c];
    }
    ctu->getQP()[z] = p.qp;
  }
  for (int c = 0; c < 3; c++) {
    const int n = c ? 1024 : 4096, off = c == 0 ? 0 : c == 1 ? 4096 : 5120;
    TCoeff *dst = ctu->getCoeff(ComponentID(c));
    for (int i = 0; i < n; i++) dst[i] = o.coef[off + i];
  }
  ctu->getTotalBits() = o.bits;
  ctu->getTotalDistortion() = o.dist;
  ctu->getTotalCost() = o.cost;
}

// xCopyYuv2Pic of the CTU's reconstruction (the window; samples outside the picture are not written)
void write_rec(TComDataCU *ctu, const uint8_t *w) {
  TComPicYuv *rec = ctu->getPic()->getPicYuvRec();
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int cs = c ? 32 : 64, s = rec->getStride(id), pw = rec->getWidth(id), ph = rec->getHeight(id);
    const int x0 = ctu->getCUPelX() >> (c ? 1 : 0), y0 = ctu->getCUPelY() >> (c ? 1 : 0);
    const uint8_t *src = w + (c == 0 ? 0 : c == 1 ? 4096 : 5120);
    Pel *a = rec->getAddr(id);
    for (int y = 0; y < cs && y0 + y < ph; y++)
      for (int x = 0; x < cs && x0 + x < pw; x++) a[(y0 + y) * s + x0 + x] = src[y * cs + x];
  }
}

// The throughput form of the seam (HVX_SEAM_CU_BATCH=1): at a picture's first compressCtu call
// every slice of the picture is decided in ONE launch, one chain per slice (TEncSlice::
// compressSlice's CTU loop, TEncSlice.cpp:727-897, for all slices at once), the chains' outputs
// kept for the following calls.  A slice whose first CTU is a picture-boundary CTU (it reads
// TEncSearch::m_integerMv2Nx2N as the previous CTU left it) runs in the previous slice's chain
// (HVX_HM_SLICE_CTUS).  Every slice starts from the same resetEntropy state (one slice type and
// QP per picture): the entry state of the picture's first CTU.  Only SliceMode 0 / 1 (whole
// CTUs) pictures batch.
bool batch_picture(TEncCu *self, TComDataCU *ctu) {
  TComSlice *s = ctu->getSlice();
  const int n = g.wc * g.hc;
  const int mode = s->getSliceMode();
  if (ctu->getCtuRsAddr() != 0 || (mode != 0 && mode != 1) || s->getSliceSegmentMode() != 0) return false;
  const int S = mode == 0 ? n : (int)s->getSliceArgument();
  if (S <= 0) return false;
  auto boundary = [&](int a) { return ((a % g.wc) + 1) * 64 > g.w || ((a / g.wc) + 1) * 64 > g.h; };
  std::vector<hvx_hm_job> jobs;
  hvx_hm_job j;
  memset(&j, 0, sizeof(j));
  TEncSbac *sb = HM(self, TEncCu_rdcoders)[0][CI_CURR_BEST];
  for (int i = 0; i < HVX_NUM_CTX; i++) j.entry.st[i] = i < (int)HM(sb, TEncSbac_n_models) ? hm_ctx_state(HM(sb, TEncSbac_models)[i]) : 0;
  j.entry.frac = HM((TEncBinCABAC *)HM(sb, TEncSbac_bin), TEncBinCABAC_frac);
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < 4; i++) {
      j.int2n[(l * 4 + i) * 2] = (int16_t)HM(HM(self, TEncCu_search), TEncSearch_int2n)[l][i].getHor();
      j.int2n[(l * 4 + i) * 2 + 1] = (int16_t)HM(HM(self, TEncCu_search), TEncSearch_int2n)[l][i].getVer();
    }
  j.chained = 1;
  g.slice_first.assign(n, 0);
  for (int a0 = 0; a0 < n; a0 += S) {
    const int a1 = std::min(a0 + S, n) - 1;
    g.slice_first[a0] = 1;
    if (a0 > 0 && boundary(a0)) {  // continue the previous chain into this slice
      hvx_hm_job &p = jobs.back();
      p.n_ctus = a1 - p.first_ctu + 1;
      p.flags = HVX_HM_SLICE_CTUS(S);
      continue;
    }
    j.first_ctu = a0;
    j.n_ctus = a1 - a0 + 1;
    j.out = a0;  // output slot = CTU address
    j.slice_start = a0;
    j.slice_end = a1;
    j.flags = 0;
    jobs.push_back(j);
  }
  hvx_ctx *c = hvx_seam_ctx();
  size_t sb_bytes = 0;
  check(hvx_hm_state_size(&sb_bytes), "hvx_hm_state_size");
  g.state.get(sb_bytes * jobs.size());
  g.job.get(sizeof(hvx_hm_job) * jobs.size());
  g.out_ctu.get(sizeof(hvx_hm_ctu) * n);
  g.out_rec.get((size_t)6144 * n);
  g.out_cod.get(sizeof(hvx_hm_coder) * n);
  upload(g.job.p, jobs.data(), sizeof(hvx_hm_job) * jobs.size());
  check(hvx_hm_compress(c, (const hvx_hm_picture *)g.pic.p, 1, (const hvx_hm_job *)g.job.p, (int)jobs.size(), n, g.state.p,
                        (hvx_hm_ctu *)g.out_ctu.p, (uint8_t *)g.out_rec.p, (hvx_hm_coder *)g.out_cod.p),
        "hvx_hm_compress");
  std::vector<int32_t> st(jobs.size());
  check(hvx_hm_job_status(c, g.state.p, (int)jobs.size(), st.data()), "hvx_hm_job_status");
  for (size_t k = 0; k < st.size(); k++)
    if (st[k]) { fprintf(stderr, "hm_cu_seam: batched job %zu refused (%d)\n", k, st[k]); abort(); }
  g.b_ctu.resize(n);
  g.b_rec.resize((size_t)6144 * n);
  g.b_cod.resize(n);
  check(hvx_download(c, g.b_ctu.data(), g.out_ctu.p, sizeof(hvx_hm_ctu) * n), "hvx_download");
  check(hvx_download(c, g.b_rec.data(), g.out_rec.p, (size_t)6144 * n), "hvx_download");
  check(hvx_download(c, g.b_cod.data(), g.out_cod.p, sizeof(hvx_hm_coder) * n), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  g.launches++;
  return true;
}
}  // namespace

extern "C" void CAT(__wrap_, CU_SYM)(TEncCu *self, TComDataCU *ctu) {
  if (!g.on()) {
    CAT(__real_, CU_SYM)(self, ctu);
    return;
  }
  const int poc = ctu->getSlice()->getPOC();
  if (poc != g.cur_poc) {
    g.cur_poc = poc;
    g.cur_ok = begin_picture(self, ctu);
    g.pic_batched = g.cur_ok && g.batch == 1 && batch_picture(self, ctu);
  }
  if (!g.cur_ok) {
    g.fallback++;
    CAT(__real_, CU_SYM)(self, ctu);
    return;
  }
  if (g.pic_batched) {
    const int a = ctu->getCtuRsAddr();
    // the entry coder HM holds now must be the one the device chain carried into this CTU (the
    // previous CTU's encodeCtu state), except at slice starts (resetEntropy)
    if (a > 0 && !g.slice_first[a]) {
      TEncSbac *sb = HM(self, TEncCu_rdcoders)[0][CI_CURR_BEST];
      bool same = HM((TEncBinCABAC *)HM(sb, TEncSbac_bin), TEncBinCABAC_frac) == g.b_cod[a - 1].frac;
      for (int i = 0; i < (int)HM(sb, TEncSbac_n_models) && i < HVX_NUM_CTX; i++)
        same = same && hm_ctx_state(HM(sb, TEncSbac_models)[i]) == g.b_cod[a - 1].st[i];
      if (!same) g.state_mismatch++;
    }
    write_ctu(ctu, g.b_ctu[a]);
    write_rec(ctu, &g.b_rec[(size_t)6144 * a]);
    g.served++;
    g.batched++;
    return;
  }
  hvx_ctx *c = hvx_seam_ctx();
  TComSlice *s = ctu->getSlice();
  const int addr = ctu->getCtuRsAddr();
  hvx_hm_job j;
  memset(&j, 0, sizeof(j));
  j.pic = 0;
  j.first_ctu = addr;
  j.n_ctus = 1;
  j.chained = 1;  // the decided CTU is written into the device picture: the next CTU's neighbourhood
  j.out = 0;
  j.slice_start = (int)s->getSliceCurStartCtuTsAddr();  // one tile: TS order = raster order
  j.slice_end = (int)s->getSliceCurEndCtuTsAddr() - 1;
  // the RD coder the decision starts from and the search's integer 2Nx2N MVs (cu_capture.cpp)
  TEncSbac *sb = HM(self, TEncCu_rdcoders)[0][CI_CURR_BEST];
  for (int i = 0; i < HVX_NUM_CTX; i++) j.entry.st[i] = i < (int)HM(sb, TEncSbac_n_models) ? hm_ctx_state(HM(sb, TEncSbac_models)[i]) : 0;
  j.entry.frac = HM((TEncBinCABAC *)HM(sb, TEncSbac_bin), TEncBinCABAC_frac);
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < 4; i++) {
      j.int2n[(l * 4 + i) * 2] = (int16_t)HM(HM(self, TEncCu_search), TEncSearch_int2n)[l][i].getHor();
      j.int2n[(l * 4 + i) * 2 + 1] = (int16_t)HM(HM(self, TEncCu_search), TEncSearch_int2n)[l][i].getVer();
    }
  upload(g.job.p, &j, sizeof(j));
  check(hvx_hm_compress(c, (const hvx_hm_picture *)g.pic.p, 1, (const hvx_hm_job *)g.job.p, 1, 1, g.state.p,
                        (hvx_hm_ctu *)g.out_ctu.p, (uint8_t *)g.out_rec.p, nullptr),
        "hvx_hm_compress");
  static hvx_hm_ctu o;
  static uint8_t w[6144];
  check(hvx_download(c, &o, g.out_ctu.p, sizeof(o)), "hvx_download");
  check(hvx_download(c, w, g.out_rec.p, sizeof(w)), "hvx_download");
  check(hvx_sync(c), "hvx_sync");
  write_ctu(ctu, o);
  write_rec(ctu, w);
  g.served++;
}
