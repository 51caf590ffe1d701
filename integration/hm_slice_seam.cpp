// hm_slice_seam.cpp -- the slice writer of an UNCHANGED HM-16.5rc1 TAppEncoder served by libhvx.so:
// SURVEY.md 8(f) item 4 (bitstream emission).
//
// Replaces TEncSlice::encodeSlice (TEncSlice.cpp:920, called per slice by TEncGOP::compressGOP,
// TEncGOP.cpp:1570).  For a slice of consecutive CTUs (no tiles, no wavefronts, no dependent slice
// segments) the seam initialises the entropy coder as encodeSlice does (TEncSbac::init with the
// slice's TEncBinCABAC, resetEntropy, bin counting on), describes the picture to the device
// (geometry, slice type / QP, reference counts, merge candidates, AMP, MvdL1Zero; every CTU of the
// slice packed from the picture's TComDataCU objects -- what copyToPic left there; the SAO
// parameters of TComPicSym::getSAOBlkParam) and hands the slice-start context states over;
// hvx_hm_write_slices codes every CTU's SAO and CU syntax through the device TEncBinCABAC.  The
// seam appends the returned bytes to the slice's substream, loads the returned registers, bin count
// and context states (with their coded marks) into HM's coder, and ends the slice as encodeSlice
// does: encodeTerminatingBit(1), encodeSliceFinish, writeByteAlignment, the cabac_init_idx choice
// for the next slice (determineCabacInitIdx) and numBinsCoded.  Anything else falls through to
// the reference's encodeSlice (counted).  HVX_SEAM_SLICE=1 enables the seam.
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
#include "TLibCommon/TComBitStream.h"
#include "TLibCommon/TComSampleAdaptiveOffset.h"
#include "TLibEncoder/TEncCfg.h"
#include "TLibEncoder/TEncSlice.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#include "TLibEncoder/TEncEntropy.h"
#include "hm_access.hpp"
#include "hvx.h"

#define SLICE_SYM _ZN9TEncSlice11encodeSliceEP7TComPicP19TComOutputBitstreamRj
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, SLICE_SYM)(TEncSlice *, TComPic *, TComOutputBitstream *, UInt &);
hvx_ctx *hvx_seam_ctx();  // hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

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

struct SliceSeam {
  int enabled = -1;
  long long served = 0, fallback = 0, bytes = 0;
  DevBuf pic, ctus, sao, job, state, res, out;
  ~SliceSeam() {
    if (enabled == 1)
      fprintf(stderr, "hm_slice_seam: %lld slices written by libhvx (%lld bytes), %lld fell through\n", served, bytes,
              fallback);
  }
  bool on() {
    if (enabled < 0) {
      const char *e = getenv("HVX_SEAM_SLICE");
      enabled = (e && e[0] == '1') ? 1 : 0;
    }
    return enabled == 1;
  }
};
SliceSeam g;

void upload(void *d, const void *h, size_t n) { check(hvx_upload(hvx_seam_ctx(), d, h, n), "hvx_upload"); }

// the decided CTU as TComDataCU holds it (copyToPic, TComDataCU.cpp:945) -> hvx_hm_ctu
void pack_ctu(TComDataCU *ctu, hvx_hm_ctu &o) {
  memset(&o, 0, sizeof(o));
  for (int z = 0; z < 256; z++) {
    hvx_hm_part &p = o.p[z];
    p.depth = (int8_t)ctu->getDepth(z);
    p.width = ctu->getWidth(z);
    p.part = (int8_t)ctu->getPartitionSize(z);
    p.pred = (int8_t)ctu->getPredictionMode(z);
    p.skip = ctu->getSkipFlag(z) ? 1 : 0;
    p.merge = ctu->getMergeFlag(z) ? 1 : 0;
    p.merge_idx = (int8_t)ctu->getMergeIndex(z);
    p.inter_dir = (int8_t)ctu->getInterDir(z);
    for (int l = 0; l < 2; l++) {
      const TComCUMvField *f = ctu->getCUMvField(RefPicList(l));
      p.mv[l][0] = (int16_t)f->getMv(z).getHor();
      p.mv[l][1] = (int16_t)f->getMv(z).getVer();
      p.mvd[l][0] = (int16_t)f->getMvd(z).getHor();
      p.mvd[l][1] = (int16_t)f->getMvd(z).getVer();
      p.ref[l] = (int8_t)f->getRefIdx(z);
      p.mvp_idx[l] = (int8_t)ctu->getMVPIdx(RefPicList(l))[z];
      p.mvp_num[l] = (int8_t)ctu->getMVPNum(RefPicList(l))[z];
    }
    p.idir[0] = ctu->getIntraDir(CHANNEL_TYPE_LUMA, z);
    p.idir[1] = ctu->getIntraDir(CHANNEL_TYPE_CHROMA, z);
    p.tr_idx = (int8_t)ctu->getTransformIdx(z);
    for (int c = 0; c < 3; c++) {
      p.ts[c] = ctu->getTransformSkip(z, ComponentID(c));
      p.cbf[c] = ctu->getCbf(z, ComponentID(c));
    }
    p.qp = ctu->getQP(z);
  }
  for (int c = 0; c < 3; c++) {
    const int n = c ? 1024 : 4096, off = c == 0 ? 0 : c == 1 ? 4096 : 5120;
    const TCoeff *src = ctu->getCoeff(ComponentID(c));
    for (int i = 0; i < n; i++) o.coef[off + i] = (int16_t)src[i];
  }
}

// SAOBlkParam -> the [3][8] layout of hvx_sao_decide_job.coded: mode (0 off, 1 new, 2 merge),
// type (EO 0-3 / BO 4; merge 0 left / 1 above), band position, offsets (EO classes 0..4 / the 4 bands)
void pack_sao(SAOBlkParam &b, int32_t *r) {
  for (int c = 0; c < 3; c++) {
    const SAOOffset &o = b[c];
    int32_t *q = r + c * 8;
    for (int i = 0; i < 8; i++) q[i] = 0;
    q[0] = o.modeIdc == SAO_MODE_OFF ? 0 : o.modeIdc == SAO_MODE_NEW ? 1 : 2;
    if (o.modeIdc == SAO_MODE_OFF) continue;
    q[1] = o.typeIdc;
    if (o.modeIdc == SAO_MODE_NEW) {
      q[2] = o.typeAuxInfo;
      if (o.typeIdc == SAO_TYPE_BO)
        for (int i = 0; i < 4; i++) q[3 + i] = o.offset[(o.typeAuxInfo + i) % NUM_SAO_BO_CLASSES];
      else
        for (int i = 0; i < 5; i++) q[3 + i] = o.offset[i];
    }
  }
}

// the slices the device writer takes (SliceMode 0 / 1 slices of whole CTUs, 4:2:0 8-bit, CTU 64,
// the engine's tool set)
bool supported(TEncSlice *self, TComPic *pic, TComSlice *s) {
  const TComSPS &sps = *s->getSPS();
  const TComPPS &pps = *s->getPPS();
  if (pps.getDependentSliceSegmentsEnabledFlag() || pps.getEntropyCodingSyncEnabledFlag()) return false;
  if (pps.getNumTileColumnsMinus1() != 0 || pps.getNumTileRowsMinus1() != 0) return false;
  if (pps.getTransquantBypassEnableFlag() || pps.getUseDQP() || s->getUseChromaQpAdj()) return false;
  if (sps.getMaxCUWidth() != 64 || sps.getMaxCUHeight() != 64 || sps.getChromaFormatIdc() != CHROMA_420) return false;
  if (sps.getBitDepth(CHANNEL_TYPE_LUMA) != 8 || sps.getBitDepth(CHANNEL_TYPE_CHROMA) != 8) return false;
  if (sps.getUsePCM() || s->getSliceSegmentCurStartCtuTsAddr() != s->getSliceCurStartCtuTsAddr()) return false;
  if (pps.getPpsRangeExtension().getLog2MaxTransformSkipBlockSize() != 2) return false;  // transform_skip_flag: 4x4
  // the syntax the device writer hard-codes (hm_cu_seam.cpp begin_picture's tool check): sign hiding on and the
  // transform_skip_flag coded (hvx_tu_desc sign_hiding / pps_tskip), the TU quadtree 32..4 to depth 3
  // (write_transform's split flags), an 8x8 minimum CU (the split flag is skipped only at depth 3)
  if (!pps.getSignHideFlag() || !pps.getUseTransformSkip()) return false;
  if (sps.getQuadtreeTULog2MaxSize() != 5 || sps.getQuadtreeTULog2MinSize() != 2 || sps.getQuadtreeTUMaxDepthInter() != 3 ||
      sps.getQuadtreeTUMaxDepthIntra() != 3 || sps.getMaxTotalCUDepth() != 4)
    return false;
  if (sps.getSpsRangeExtension().getRdpcmEnabledFlag(RDPCM_SIGNAL_IMPLICIT) ||
      sps.getSpsRangeExtension().getRdpcmEnabledFlag(RDPCM_SIGNAL_EXPLICIT) ||
      sps.getSpsRangeExtension().getPersistentRiceAdaptationEnabledFlag() ||
      sps.getSpsRangeExtension().getCabacBypassAlignmentEnabledFlag() ||
      sps.getSpsRangeExtension().getExtendedPrecisionProcessingFlag() ||
      pps.getPpsRangeExtension().getCrossComponentPredictionEnabledFlag())
    return false;
  (void)self;
  (void)pic;
  return true;
}
}  // namespace

extern "C" void CAT(__wrap_, SLICE_SYM)(TEncSlice *self, TComPic *pic, TComOutputBitstream *subs, UInt &num_bins) {
  TComSlice *const s = pic->getSlice(self->getSliceIdx());
  if (!g.on() || !supported(self, pic, s)) {
    if (g.on()) g.fallback++;
    CAT(__real_, SLICE_SYM)(self, pic, subs, num_bins);
    return;
  }
  TComPicSym *sym = pic->getPicSym();
  const int start = (int)s->getSliceSegmentCurStartCtuTsAddr(), bound = (int)s->getSliceSegmentCurEndCtuTsAddr();
  const int wc = (int)sym->getFrameWidthInCtus(), nctu = (int)sym->getNumberOfCtusInFrame();
  // TEncSlice::encodeSlice's set-up (TEncSlice.cpp:930-938)
  TEncSbac *sb = HM(self, TEncSlice_sbac);
  TEncBinCABAC *bin = HM(self, TEncSlice_cabac);
  TEncEntropy *ent = HM(self, TEncSlice_entropy);
  sb->init((TEncBinIf *)bin);
  ent->setEntropyCoder(sb);
  ent->resetEntropy(s);
  num_bins = 0;
  bin->setBinCountingEnableFlag(true);
  bin->setBinsCoded(0);
  TComOutputBitstream &bs = subs[pic->getSubstreamForCtuAddr(sym->getCtuTsToRsAddrMap(start), true, s)];
  ent->setBitstream(&bs);

  // the picture as the writer reads it (hvx_hm_picture: geometry, slice parameters, the CTU array)
  hvx_hm_picture P;
  memset(&P, 0, sizeof(P));
  const TComSPS &sps = *s->getSPS();
  P.w = (int)sps.getPicWidthInLumaSamples();
  P.h = (int)sps.getPicHeightInLumaSamples();
  P.w_ctus = wc;
  P.h_ctus = (P.h + 63) / 64;
  P.poc = s->getPOC();
  P.slice_type = s->getSliceType();
  P.qp = s->getSliceQp();
  for (int l = 0; l < 2; l++) P.nref[l] = s->isIntra() || (l == 1 && !s->isInterB()) ? 0 : s->getNumRefIdx(RefPicList(l));
  P.max_merge = (int)s->getMaxNumMergeCand();
  P.amp = sps.getUseAMP() ? 1 : 0;
  P.mvd_l1_zero = s->getMvdL1ZeroFlag() ? 1 : 0;
  std::vector<hvx_hm_ctu> ctus(nctu);
  std::vector<int32_t> sao((size_t)nctu * 24, 0);
  const bool use_sao = sps.getUseSAO();
  for (int ts = start; ts < bound; ts++) {
    const int a = (int)sym->getCtuTsToRsAddrMap(ts);
    pack_ctu(pic->getCtu(a), ctus[a]);
    if (use_sao) pack_sao(sym->getSAOBlkParam()[a], &sao[(size_t)a * 24]);
  }
  void *dctus = g.ctus.get(ctus.size() * sizeof(hvx_hm_ctu));
  upload(dctus, ctus.data(), ctus.size() * sizeof(hvx_hm_ctu));
  P.ctus = (hvx_hm_ctu *)dctus;
  void *dpic = g.pic.get(sizeof(P));
  upload(dpic, &P, sizeof(P));

  hvx_hm_slice j;
  memset(&j, 0, sizeof(j));
  j.pic = 0;
  j.first_ctu = (int)sym->getCtuTsToRsAddrMap(start);
  j.n_ctus = bound - start;
  if (use_sao) {
    for (int c = 0; c < 3; c++) j.sao_enabled[c] = s->getSaoEnabledFlag(toChannelType(ComponentID(c))) ? 1 : 0;
    void *dsao = g.sao.get(sao.size() * sizeof(int32_t));
    upload(dsao, sao.data(), sao.size() * sizeof(int32_t));
    j.sao_coded = (const int32_t *)dsao;
  }
  const int cap = 1 << 24;
  j.out = (uint8_t *)g.out.get(cap);
  j.out_cap = cap;
  for (int i = 0; i < HVX_NUM_CTX; i++) j.entry.st[i] = i < (int)HM(sb, TEncSbac_n_models) ? hm_ctx_state(HM(sb, TEncSbac_models)[i]) : 0;
  void *djob = g.job.get(sizeof(j));
  upload(djob, &j, sizeof(j));
  size_t sbytes = 0;
  check(hvx_hm_state_size(&sbytes), "hvx_hm_state_size");
  void *dstate = g.state.get(sbytes);
  void *dres = g.res.get(sizeof(hvx_hm_slice_result));
  check(hvx_hm_write_slices(hvx_seam_ctx(), (const hvx_hm_picture *)dpic, 1, (const hvx_hm_slice *)djob, 1, dstate,
                            (hvx_hm_slice_result *)dres),
        "hvx_hm_write_slices");
  hvx_hm_slice_result r;
  check(hvx_download(hvx_seam_ctx(), &r, dres, sizeof(r)), "hvx_download");
  if (r.status != 0 || r.n_bytes > cap) {
    fprintf(stderr, "hm_slice_seam: slice at CTU %d refused (%d, %d bytes)\n", j.first_ctu, r.status, r.n_bytes);
    abort();
  }
  std::vector<uint8_t> bytes(r.n_bytes);
  if (r.n_bytes) check(hvx_download(hvx_seam_ctx(), bytes.data(), j.out, bytes.size()), "hvx_download");
  // the bytes TEncBinCABAC::writeOut wrote, then its registers, bin count and the contexts
  for (uint8_t b : bytes) bs.write(b, 8);
  HM(bin, TEncBinCABAC_low) = r.low;
  HM(bin, TEncBinCABAC_range) = r.range;
  HM(bin, TEncBinCABAC_bits_left) = r.bits_left;
  HM(bin, TEncBinCABAC_n_buffered) = r.num_buffered;
  HM(bin, TEncBinCABAC_buffered_byte) = r.buffered_byte;
  HM(bin, TEncBinCABAC_bins) += r.bins * HM(bin, TEncBinCABAC_bin_inc);
  ContextModel *models = HM(sb, TEncSbac_models);
  for (int m = 0; m < (int)HM(sb, TEncSbac_n_models) && m < HVX_NUM_CTX; m++) {
    hm_set_ctx_state(models[m], r.states[m]);
    if ((r.coded[m >> 5] >> (m & 31)) & 1u) models[m].setBinsCoded(1);
  }
  // the end of the slice (TEncSlice.cpp:1084-1090) and of encodeSlice (:1097-1114)
  ent->encodeTerminatingBit(1);
  ent->encodeSliceFinish();
  bs.writeByteAlignment();
#if ADAPTIVE_QP_SELECTION
  if (HM(self, TEncSlice_cfg)->getUseAdaptQpSelect()) HM(self, TEncSlice_trquant)->storeSliceQpNext(s);
#endif
  if (s->getPPS()->getCabacInitPresentFlag() && !s->getPPS()->getDependentSliceSegmentsEnabledFlag())
    HM(self, TEncSlice_cabac_idx) = ent->determineCabacInitIdx(s);
  else
    HM(self, TEncSlice_cabac_idx) = s->getSliceType();
  num_bins = bin->getBinsCoded();
  g.served++;
  g.bytes += r.n_bytes;
}
