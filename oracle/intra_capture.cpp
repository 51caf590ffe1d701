// intra_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target
// _ref/TAppEncoder_intracap) with
//   -Wl,--wrap=<TComPrediction::initIntraPatternChType>,--wrap=<TComPrediction::predIntraAng>
// so that the intra calls TEncSearch makes (TEncSearch.cpp:2256, 2283, 1131-1160) are
// observed.  Three record kinds go to the golden container named by $HVX_CAPTURE:
//
//  ref_*   initIntraPatternChType (TComPattern.cpp:115-360 + fillReferenceSamples :364-540):
//          the block geometry, the neighbour flags (recomputed with the reference's own
//          isAboveLeftAvailable/isAboveAvailable/... of TComPattern.cpp:571-749), the raw
//          reconstructed samples at every neighbour position, and the unfiltered / filtered
//          reference borders the reference built (m_piYuvExt).
//  pred_*  predIntraAng (TComPrediction.cpp:455-516): mode, filter choice, the reference border
//          it read and the prediction block it wrote.
//  fp_*    estIntraPredLumaQT's first pass (TEncSearch.cpp:2244-2323): a luma PU for which
//          predIntraAng is called with modes 0..34 in order.  Per mode the reference's own
//          Hadamard SATD (TComRdCost::setDistParam + DistFunc, as :2276-2284 does) and
//          xModeBitsIntra (:5222); the sqrt-lambda, the MPM inputs/outputs
//          (TComDataCU::getIntraDirPredictor :1401) and the candidate list produced by the
//          reference's xUpdateCandList (:5254) with the MPM append of :2299-2321.
//
// Border layout (all record kinds): B[0] = top-left corner, B[1..2N] = above + above-right
// row left to right, B[2N+1..4N] = left + below-left column top to bottom (N = block size).
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
#include "TLibCommon/TComPrediction.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncCfg.h"
#include "TLibEncoder/TEncBinCoderCABACCounter.h"
#include "TLibCommon/TComBitCounter.h"
#undef private
#undef protected
#include "golden_writer.h"

#define INIT_SYM _ZN14TComPrediction22initIntraPatternChTypeER6TComTURbS2_11ComponentIDb
#define PRED_SYM _ZN14TComPrediction12predIntraAngE11ComponentIDjPsjS1_jR6TComTUbbbb
#define MPM_SYM _ZN10TComDataCU20getIntraDirPredictorEjPi11ComponentIDS0_
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" {
void CAT(__real_, INIT_SYM)(TComPrediction *, TComTU &, Bool &, Bool &, ComponentID, Bool);
void CAT(__real_, PRED_SYM)(TComPrediction *, ComponentID, UInt, Pel *, UInt, Pel *, UInt, TComTU &, Bool, Bool, Bool, Bool);
void CAT(__real_, MPM_SYM)(TComDataCU *, UInt, Int *, ComponentID, Int *);
}
// the reference's neighbour-availability functions (TComPattern.cpp:571-749, external linkage)
Bool isAboveLeftAvailable(TComDataCU *pcCU, UInt uiPartIdxLT);
Int isAboveAvailable(TComDataCU *pcCU, UInt uiPartIdxLT, UInt uiPartIdxRT, Bool *bValidFlags);
Int isLeftAvailable(TComDataCU *pcCU, UInt uiPartIdxLT, UInt uiPartIdxLB, Bool *bValidFlags);
Int isAboveRightAvailable(TComDataCU *pcCU, UInt uiPartIdxLT, UInt uiPartIdxRT, Bool *bValidFlags);
Int isBelowLeftAvailable(TComDataCU *pcCU, UInt uiPartIdxLT, UInt uiPartIdxLB, Bool *bValidFlags);

namespace {
const int kB = 257;     // border samples of a 64x64 block
const int kF = 65;      // neighbour units of a 64x64 luma block (4-sample units)
const int kBlk = 4096;

int log2i(int v) { int l = 0; while ((1 << l) < v) l++; return l; }

// HM's 2-D reference buffer (stride 2N+1) -> border layout
void border_from_buf(const Pel *buf, int n, int16_t *B) {
  const int s = 2 * n + 1;
  for (int i = 0; i <= 2 * n; i++) B[i] = buf[i];
  for (int j = 0; j < 2 * n; j++) B[2 * n + 1 + j] = buf[(j + 1) * s];
}

struct Nbr {  // the inputs of one initIntraPatternChType call
  const TComDataCU *cu = nullptr;
  UInt abs = 0;
  int comp = -1, n = 0, unit = 0, nflags = 0;
  uint8_t flags[kF];
  int16_t raw[kB];
};

struct FirstPass {
  bool active = false;
  const TComDataCU *cu = nullptr;
  UInt abs = 0;
  int n = 0, next = 0;
  Nbr nbr;
  int16_t unf[kB], filt[kB];
  uint8_t org[kBlk];
  double sqrt_lambda = 0;
  uint32_t satd[35], bits[35];
  int ctx_state = -1, frac_in[35], mpm_calls = 0;
  TEncSearch *enc = nullptr;
};

struct Store {
  // ref records
  std::vector<int32_t> ref_meta;
  std::vector<uint8_t> ref_flags;
  std::vector<int16_t> ref_raw, ref_unf, ref_filt;
  // pred records
  std::vector<int32_t> pred_meta;
  std::vector<int16_t> pred_border;
  std::vector<uint8_t> pred_out;
  // first-pass records
  std::vector<int32_t> fp_meta, fp_cand;
  std::vector<uint8_t> fp_flags, fp_org;
  std::vector<int16_t> fp_raw;
  std::vector<uint32_t> fp_satd, fp_bits;
  std::vector<double> fp_lambda, fp_cost, fp_cand_cost;
  std::vector<int32_t> fp_frac_in;
  std::map<int, int> ref_count, pred_count, fp_count;
  int nref = 0, npred = 0, nfp = 0;
  long long ninit = 0, npredcalls = 0, nfpseen = 0;
  Nbr last;
  FirstPass fp;
  SplitMix64 rng{0x5EED4004};
  ~Store() { flush(); }
  bool take(std::map<int, int> &m, int key, int first, int cap, int one_in) {
    int &c = m[key];
    if (c >= cap || !(c < first || (rng.next() % one_in) == 0)) return false;
    c++;
    return true;
  }
  void flush() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out) return;
    GoldenWriter gw;
    gw.add("ref_meta", "i32", {(uint32_t)nref, 6}, ref_meta);
    gw.add("ref_flags", "u8", {(uint32_t)nref, (uint32_t)kF}, ref_flags);
    gw.add("ref_raw", "i16", {(uint32_t)nref, (uint32_t)kB}, ref_raw);
    gw.add("ref_unf", "i16", {(uint32_t)nref, (uint32_t)kB}, ref_unf);
    gw.add("ref_filt", "i16", {(uint32_t)nref, (uint32_t)kB}, ref_filt);
    gw.add("pred_meta", "i32", {(uint32_t)npred, 6}, pred_meta);
    gw.add("pred_border", "i16", {(uint32_t)npred, (uint32_t)kB}, pred_border);
    gw.add("pred_out", "u8", {(uint32_t)pred_out.size()}, pred_out);  // N*N per record, in record order
    gw.add("fp_meta", "i32", {(uint32_t)nfp, 12}, fp_meta);  // log2n ctx_state left_dir above_dir iMode mpm0..2 num_rd n_cand fast_mpm frac0
    gw.add("fp_flags", "u8", {(uint32_t)nfp, (uint32_t)kF}, fp_flags);
    gw.add("fp_raw", "i16", {(uint32_t)nfp, (uint32_t)kB}, fp_raw);
    gw.add("fp_org", "u8", {(uint32_t)fp_org.size()}, fp_org);  // N*N per record, in record order
    gw.add("fp_lambda", "f64", {(uint32_t)nfp}, fp_lambda);
    gw.add("fp_satd", "u32", {(uint32_t)nfp, 35}, fp_satd);
    gw.add("fp_bits", "u32", {(uint32_t)nfp, 35}, fp_bits);
    gw.add("fp_cost", "f64", {(uint32_t)nfp, 35}, fp_cost);
    gw.add("fp_cand", "i32", {(uint32_t)nfp, 11}, fp_cand);
    gw.add("fp_cand_cost", "f64", {(uint32_t)nfp, 8}, fp_cand_cost);
    gw.add("fp_frac_in", "i32", {(uint32_t)nfp, 35}, fp_frac_in);  // the source coder's m_fracBits & 32767 at each mode
    gw.write(out);
    fprintf(stderr, "intra_capture: %lld pattern calls (%d kept), %lld predIntraAng calls (%d kept), "
            "%lld first passes (%d kept)\n", ninit, nref, npredcalls, npred, nfpseen, nfp);
  }
};
Store g;

// neighbour flags + raw samples exactly as initIntraPatternChType derives them (TComPattern.cpp:120-160)
void observe_pattern(TComTU &rTu, ComponentID compID, Nbr &nb) {
  TComDataCU *pcCU = rTu.getCU();
  const TComSPS &sps = *(pcCU->getSlice()->getSPS());
  const UInt zo = rTu.GetAbsPartIdxTU();
  const int w = rTu.getRect(compID).width, h = rTu.getRect(compID).height;
  const int base = sps.getMaxCUWidth() >> sps.getMaxTotalCUDepth();
  const int uw = base >> pcCU->getPic()->getPicYuvRec()->getComponentScaleX(compID);
  const int uh = base >> pcCU->getPic()->getPicYuvRec()->getComponentScaleY(compID);
  const int wu = w / uw, hu = h / uh, aboveU = wu << 1, leftU = hu << 1;
  const int ps = pcCU->getPic()->getNumPartInCtuWidth();
  const UInt lt = pcCU->getZorderIdxInCtu() + zo;
  const UInt rt = g_auiRasterToZscan[g_auiZscanToRaster[lt] + wu - 1];
  const UInt lb = g_auiRasterToZscan[g_auiZscanToRaster[lt] + ((hu - 1) * ps)];
  Bool f[4 * MAX_NUM_PART_IDXS_IN_CTU_WIDTH + 1];
  memset(f, 0, sizeof(f));
  f[leftU] = isAboveLeftAvailable(pcCU, lt);
  isAboveAvailable(pcCU, lt, rt, f + leftU + 1);
  isAboveRightAvailable(pcCU, lt, rt, f + leftU + 1 + wu);
  isLeftAvailable(pcCU, lt, lb, f + leftU - 1);
  isBelowLeftAvailable(pcCU, lt, lb, f + leftU - 1 - hu);
  nb.cu = pcCU; nb.abs = zo; nb.comp = (int)compID; nb.n = w; nb.unit = uw;
  nb.nflags = aboveU + leftU + 1;
  memset(nb.flags, 0, sizeof(nb.flags));
  for (int i = 0; i < nb.nflags && i < kF; i++) nb.flags[i] = f[i] ? 1 : 0;
  const Pel *o = pcCU->getPic()->getPicYuvRec()->getAddr(compID, pcCU->getCtuRsAddr(), pcCU->getZorderIdxInCtu() + zo);
  const int st = pcCU->getPic()->getStride(compID);
  memset(nb.raw, 0, sizeof(nb.raw));
  nb.raw[0] = o[-st - 1];
  for (int i = 0; i < 2 * w; i++) nb.raw[1 + i] = o[-st + i];
  for (int j = 0; j < 2 * h; j++) nb.raw[2 * w + 1 + j] = o[j * st - 1];
}
}  // namespace

static void finish_first_pass(TComDataCU *cu, UInt abs);

extern "C" void CAT(__wrap_, INIT_SYM)(TComPrediction *self, TComTU &rTu, Bool &bAbove, Bool &bLeft, ComponentID compID,
                                        Bool bFilter) {
  g.ninit++;
  observe_pattern(rTu, compID, g.last);
  CAT(__real_, INIT_SYM)(self, rTu, bAbove, bLeft, compID, bFilter);
  const Nbr &nb = g.last;
  const int n = nb.n;
  int navail = 0;
  for (int i = 0; i < nb.nflags; i++) navail += nb.flags[i];
  const int cls = navail == 0 ? 0 : navail == nb.nflags ? 1 : 2;
  const int key = (isLuma(compID) ? 0 : 1) | (log2i(n) << 1) | (cls << 4);
  if (!g.take(g.ref_count, key, 10, 24, 32)) return;
  g.ref_meta.insert(g.ref_meta.end(), {log2i(n), isLuma(compID) ? 0 : 1, log2i(nb.unit), bFilter ? 1 : 0,
                                       (bAbove ? 1 : 0) | (bLeft ? 2 : 0), nb.nflags});
  g.ref_flags.insert(g.ref_flags.end(), nb.flags, nb.flags + kF);
  g.ref_raw.insert(g.ref_raw.end(), nb.raw, nb.raw + kB);
  int16_t B[kB];
  memset(B, 0, sizeof(B));
  border_from_buf(self->m_piYuvExt[compID][PRED_BUF_UNFILTERED], n, B);
  g.ref_unf.insert(g.ref_unf.end(), B, B + kB);
  memset(B, 0, sizeof(B));
  if (bFilter) border_from_buf(self->m_piYuvExt[compID][PRED_BUF_FILTERED], n, B);
  g.ref_filt.insert(g.ref_filt.end(), B, B + kB);
  g.nref++;
}

extern "C" void CAT(__wrap_, PRED_SYM)(TComPrediction *self, ComponentID compID, UInt mode, Pel *piOrg, UInt orgStride,
                                        Pel *piPred, UInt predStride, TComTU &rTu, Bool bAbove, Bool bLeft,
                                        Bool bUseFilt, Bool bDPCM) {
  g.npredcalls++;
  CAT(__real_, PRED_SYM)(self, compID, mode, piOrg, orgStride, piPred, predStride, rTu, bAbove, bLeft, bUseFilt, bDPCM);
  const int n = rTu.getRect(compID).width;
  if (bDPCM || rTu.getRect(compID).height != n) return;
  // (1) the prediction itself
  const int key = (isLuma(compID) ? 0 : 1) | (log2i(n) << 1) | (mode << 4) | ((bUseFilt ? 1 : 0) << 10);
  if (g.take(g.pred_count, key, n >= 32 ? 1 : 2, n >= 32 ? 2 : 4, 64)) {
    g.pred_meta.insert(g.pred_meta.end(), {log2i(n), isLuma(compID) ? 0 : 1, (int)mode, bUseFilt ? 1 : 0, bAbove ? 1 : 0,
                                           bLeft ? 1 : 0});
    int16_t B[kB];
    memset(B, 0, sizeof(B));
    border_from_buf(self->getPredictorPtr(compID, bUseFilt), n, B);
    g.pred_border.insert(g.pred_border.end(), B, B + kB);
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) g.pred_out.push_back((uint8_t)piPred[y * predStride + x]);
    g.npred++;
  }
  // (2) estIntraPredLumaQT's first pass: modes 0..34 in order on one luma PU
  TEncSearch *enc = dynamic_cast<TEncSearch *>(self);
  FirstPass &fp = g.fp;
  if (!enc || !isLuma(compID) || !piOrg) { fp.active = false; return; }
  TComDataCU *cu = rTu.getCU();
  const UInt abs = rTu.GetAbsPartIdxTU();
  if (mode == 0) {
    fp.active = g.last.cu == cu && g.last.abs == abs && g.last.comp == (int)compID && g.last.n == n;
    if (!fp.active) return;
    fp.cu = cu; fp.abs = abs; fp.n = n; fp.next = 0; fp.nbr = g.last;
    memset(fp.unf, 0, sizeof(fp.unf)); memset(fp.filt, 0, sizeof(fp.filt)); memset(fp.org, 0, sizeof(fp.org));
    border_from_buf(self->m_piYuvExt[compID][PRED_BUF_UNFILTERED], n, fp.unf);
    border_from_buf(self->m_piYuvExt[compID][PRED_BUF_FILTERED], n, fp.filt);
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) fp.org[y * n + x] = (uint8_t)piOrg[y * orgStride + x];
    fp.sqrt_lambda = enc->m_pcRdCost->getSqrtLambda();
  } else if (!fp.active || fp.cu != cu || fp.abs != abs || fp.n != n || (int)mode != fp.next) {
    fp.active = false;
    return;
  }
  // the reference's SATD (TEncSearch.cpp:2276-2284) and mode bits (:2287)
  DistParam dp;
  enc->m_pcRdCost->setDistParam(dp, cu->getSlice()->getSPS()->getBitDepth(CHANNEL_TYPE_LUMA), piOrg, orgStride, piPred,
                                predStride, n, n, true);
  dp.bApplyWeight = false;
  fp.satd[mode] = dp.DistFunc(&dp);
  // the state xModeBitsIntra loads (TEncSearch.cpp:5225) and the RD counter it counts with.
  // HM's own count of mode m-1 is READ (not recomputed) from that counter here, before mode
  // m's resetBits: getNumberOfWrittenBits is a pure read, so the encode is not perturbed.
  const int st = enc->m_pppcRDSbacCoder[cu->getDepth(0)][CI_CURR_BEST]->m_cCUIntraPredSCModel.get(0, 0, 0).m_ucState;
  TEncBinCABAC *live = dynamic_cast<TEncBinCABAC *>(enc->m_pcRDGoOnSbacCoder->m_pcBinIf);
  if (!live) { fp.active = false; return; }
  if (mode > 0) fp.bits[mode - 1] = enc->m_pcRDGoOnSbacCoder->getNumberOfWrittenBits();
  // loadIntraDirMode copies the bin coder state (m_fracBits included) from that same source
  // coder before resetBits keeps its low 15 bits (TEncSbac.cpp:403, TEncBinCoderCABAC.cpp:172)
  TEncBinCABAC *src = dynamic_cast<TEncBinCABAC *>(enc->m_pppcRDSbacCoder[cu->getDepth(0)][CI_CURR_BEST]->m_pcBinIf);
  if (!src) { fp.active = false; return; }
  fp.frac_in[mode] = (int)(src->m_fracBits & 32767);
  if (mode == 0) { fp.ctx_state = st; fp.enc = enc; fp.mpm_calls = 0; }
  else if (st != fp.ctx_state || fp.frac_in[mode] != fp.frac_in[0]) { fp.active = false; return; }
  fp.next++;
  // mode 34's count is read in the getIntraDirPredictor wrap that follows the loop (:2303)
}

// called right after the first pass's mode loop (TEncSearch.cpp:2303, FastUDIUseMPM)
extern "C" void CAT(__wrap_, MPM_SYM)(TComDataCU *cu, UInt abs, Int *preds, ComponentID compID, Int *piMode) {
  // every xModeBitsIntra also calls it (TEncSbac::codeIntraDirLumaAng, TEncSbac.cpp:654) before
  // counting: after mode 34 the first call is that one, the second is the loop's own
  FirstPass &fp = g.fp;
  bool done = false;
  if (fp.active && fp.next == 35 && fp.cu == cu && fp.abs == abs && compID == COMPONENT_Y && fp.enc) {
    if (++fp.mpm_calls == 2) {
      fp.bits[34] = fp.enc->m_pcRDGoOnSbacCoder->getNumberOfWrittenBits();
      fp.active = false;
      done = true;
    }
  }
  CAT(__real_, MPM_SYM)(cu, abs, preds, compID, piMode);
  if (done) finish_first_pass(cu, abs);
}

static void finish_first_pass(TComDataCU *cu, UInt abs) {
  FirstPass &fp = g.fp;
  TEncSearch *enc = fp.enc;
  const int n = fp.n;
  g.nfpseen++;
  const int fkey = log2i(n);
  if (!g.take(g.fp_count, fkey, n >= 32 ? 12 : 24, n >= 32 ? 24 : 60, 8)) return;
  // MPM inputs as getIntraDirPredictor reads them (TComDataCU.cpp:1413-1428) and its output
  UInt li = MAX_UINT, ai = MAX_UINT;
  TComDataCU *lc = cu->getPULeft(li, cu->getZorderIdxInCtu() + abs);
  TComDataCU *ac = cu->getPUAbove(ai, cu->getZorderIdxInCtu() + abs, true, true);
  const int ldir = lc ? (lc->isIntra(li) ? lc->getIntraDir(CHANNEL_TYPE_LUMA, li) : DC_IDX) : DC_IDX;
  const int adir = ac ? (ac->isIntra(ai) ? ac->getIntraDir(CHANNEL_TYPE_LUMA, ai) : DC_IDX) : DC_IDX;
  Int preds[NUM_MOST_PROBABLE_MODES] = {-1, -1, -1};
  Int iMode = -1;
  CAT(__real_, MPM_SYM)(cu, abs, preds, COMPONENT_Y, &iMode);
  // the candidate list (TEncSearch.cpp:2244-2323) through the reference's xUpdateCandList
  const Bool fastMpm = enc->m_pcEncCfg->getFastUDIUseMPMEnabled();
  const UInt wbit = cu->getIntraSizeIdx(0);
  Int numFull = fastMpm ? g_aucIntraModeNumFast_UseMPM[wbit] : g_aucIntraModeNumFast_NotUseMPM[wbit];
  UInt list[FAST_UDI_MAX_RDMODE_NUM];
  Double ccost[FAST_UDI_MAX_RDMODE_NUM];
  for (int i = 0; i < FAST_UDI_MAX_RDMODE_NUM; i++) { list[i] = 0; ccost[i] = MAX_DOUBLE; }
  double cost[35];
  for (int m = 0; m < 35; m++) {
    cost[m] = (Double)fp.satd[m] + (Double)fp.bits[m] * fp.sqrt_lambda;
    enc->xUpdateCandList(m, cost[m], numFull, list, ccost);
  }
  const int numRD = numFull;
  if (fastMpm) {
    const Int numCand = (iMode >= 0) ? iMode : Int(NUM_MOST_PROBABLE_MODES);
    for (Int j = 0; j < numCand; j++) {
      Bool inc = false;
      for (Int i = 0; i < numFull; i++) inc |= (preds[j] == (Int)list[i]);
      if (!inc) list[numFull++] = preds[j];
    }
  }
  g.fp_meta.insert(g.fp_meta.end(), {log2i(n), fp.ctx_state, ldir, adir, iMode, preds[0], preds[1], preds[2], numRD,
                                     numFull, fastMpm ? 1 : 0, fp.frac_in[0]});
  g.fp_flags.insert(g.fp_flags.end(), fp.nbr.flags, fp.nbr.flags + kF);
  g.fp_raw.insert(g.fp_raw.end(), fp.nbr.raw, fp.nbr.raw + kB);
  g.fp_org.insert(g.fp_org.end(), fp.org, fp.org + n * n);
  g.fp_lambda.push_back(fp.sqrt_lambda);
  g.fp_satd.insert(g.fp_satd.end(), fp.satd, fp.satd + 35);
  g.fp_bits.insert(g.fp_bits.end(), fp.bits, fp.bits + 35);
  g.fp_cost.insert(g.fp_cost.end(), cost, cost + 35);
  g.fp_frac_in.insert(g.fp_frac_in.end(), fp.frac_in, fp.frac_in + 35);
  for (int i = 0; i < 11; i++) g.fp_cand.push_back(i < numFull ? (int32_t)list[i] : -1);
  for (int i = 0; i < 8; i++) g.fp_cand_cost.push_back(i < numRD ? ccost[i] : 0.0);
  g.nfp++;
}
