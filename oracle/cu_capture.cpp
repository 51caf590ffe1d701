// cu_capture.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target _ref/TAppEncoder_cucap)
// with -Wl,--wrap=<TEncCu::compressCtu>.  Every CTU the reference compresses
// (TEncSlice.cpp:814 -> TEncCu.cpp:228) is recorded:
//   * per picture (at its first CTU): the slice parameters the CU decision reads (POC, type, QP,
//     lambdas, chroma distortion weights, reference lists and POCs, the collocated picture used
//     by TMVP and its compressed motion field, merge-candidate count), the original picture and
//     every reference picture's reconstruction;
//   * per CTU, on entry: the RD coder the decision starts from (m_pppcRDSbacCoder[0][CI_CURR_BEST]:
//     context states and the bin counter's m_fracBits) and TEncSearch::m_integerMv2Nx2N;
//   * per CTU, on exit: the whole TComDataCU the decision wrote (per 4x4 partition: depth, part
//     size, prediction mode, skip/merge, motion, MVD, MVP index, intra modes, transform index,
//     transform-skip flags, CBFs), the quantised coefficients, the reconstruction (before the loop
//     filters) and the CTU's total bits / distortion / RD cost.
// The reference code itself runs unmodified.  Output: HVX_CAPTURE=<file> (tests/golden/ctu_*.bin).
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
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComPic.h"
#include "TLibCommon/TComSlice.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibEncoder/TEncCu.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#undef private
#undef protected
#include "golden_writer.h"

#define CU_SYM _ZN6TEncCu11compressCtuEP10TComDataCU
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, CU_SYM)(TEncCu *, TComDataCU *);

namespace {
// per-picture integer fields (pic_i32 rows)
enum {
  P_W, P_H, P_POC, P_SLICE_TYPE, P_QP, P_NREF0, P_NREF1, P_REFPOC0, P_REFPOC1 = P_REFPOC0 + 4,
  P_REFPIC0 = P_REFPOC1 + 4, P_REFPIC1 = P_REFPIC0 + 4, P_COL_FROM_L0 = P_REFPIC1 + 4, P_COL_REF_IDX, P_CHECK_LDC,
  P_TMVP, P_MAX_MERGE, P_COL_POC, P_COL_NREF0, P_COL_NREF1, P_COL_REFPOC0, P_COL_REFPOC1 = P_COL_REFPOC0 + 4,
  P_CHROMA_QP_CB = P_COL_REFPOC1 + 4, P_CHROMA_QP_CR, P_FIRST_CTU, P_NCTU, P_LAMBDA_MOTION, P_CABAC_TABLE,
  P_COL_VALID, P_NFIELDS
};
enum { F_LAMBDA, F_SQRT_LAMBDA, F_WEIGHT_CB, F_WEIGHT_CR, F_TQ_LAMBDA_Y, F_TQ_LAMBDA_CB, F_TQ_LAMBDA_CR, F_NFIELDS };
// per-partition fields (ctu_parts rows: 256 per CTU, z-order)
enum {
  U_DEPTH, U_PART, U_PRED, U_SKIP, U_MERGE, U_MERGE_IDX, U_INTER_DIR, U_REF0, U_REF1, U_MV0X, U_MV0Y, U_MV1X, U_MV1Y,
  U_MVD0X, U_MVD0Y, U_MVD1X, U_MVD1Y, U_MVP0, U_MVP1, U_IDIR_Y, U_IDIR_C, U_TRIDX, U_TS_Y, U_TS_CB, U_TS_CR, U_CBF_Y,
  U_CBF_CB, U_CBF_CR, U_QP, U_NFIELDS
};

struct Store {
  std::vector<int32_t> pic_i32;
  std::vector<double> pic_f64;
  std::vector<uint8_t> org, refpic, ctu_states, ctu_recon;
  std::vector<int32_t> refpic_poc, ctu_coef, ctu_meta;
  std::vector<int64_t> ctu_frac;
  std::vector<int16_t> ctu_parts, ctu_int2n, col_field;
  std::vector<double> ctu_cost;
  std::map<int, int> refpic_index;  // POC -> index into refpic
  int npic = 0, nctu = 0, cur_poc = -1000000;
  int max_pics = 1 << 30;
  ~Store() {
    const char *out = getenv("HVX_CAPTURE");
    if (!out || !nctu) return;
    GoldenWriter gw;
    gw.add("pic_i32", "i32", {(uint32_t)npic, (uint32_t)P_NFIELDS}, pic_i32);
    gw.add("pic_f64", "f64", {(uint32_t)npic, (uint32_t)F_NFIELDS}, pic_f64);
    gw.add("org", "u8", {(uint32_t)org.size()}, org);                 // per picture: Y w*h, Cb, Cr
    gw.add("refpic", "u8", {(uint32_t)refpic.size()}, refpic);        // per reference picture, same layout
    gw.add("refpic_poc", "i32", {(uint32_t)refpic_poc.size()}, refpic_poc);
    gw.add("col_field", "i16", {(uint32_t)(col_field.size() / 8), 8}, col_field);  // per picture, per 16x16 of the col pic
    gw.add("ctu_meta", "i32", {(uint32_t)nctu, 4}, ctu_meta);          // picture index, ctu rs addr, bits, dist
    gw.add("ctu_states", "u8", {(uint32_t)nctu, (uint32_t)HVX_CTX}, ctu_states);
    gw.add("ctu_frac", "i64", {(uint32_t)nctu}, ctu_frac);
    gw.add("ctu_int2n", "i16", {(uint32_t)nctu, 2 * 4 * 2}, ctu_int2n);  // [list][ref][x,y]
    gw.add("ctu_parts", "i16", {(uint32_t)nctu, 256, (uint32_t)U_NFIELDS}, ctu_parts);
    gw.add("ctu_coef", "i32", {(uint32_t)nctu, 4096 + 2048}, ctu_coef);  // Y 4096, Cb 1024, Cr 1024 (HM coefficient layout)
    gw.add("ctu_recon", "u8", {(uint32_t)nctu, 4096 + 2048}, ctu_recon);  // Y 64x64, Cb 32x32, Cr 32x32 (0 outside picture)
    gw.add("ctu_cost", "f64", {(uint32_t)nctu}, ctu_cost);
    gw.write(out);
    fprintf(stderr, "cu_capture: %d pictures, %d CTUs\n", npic, nctu);
  }
  static const int HVX_CTX = 202;
};
Store g;

void put_planes(TComPicYuv *p, std::vector<uint8_t> &dst) {
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int w = p->getWidth(id), h = p->getHeight(id), s = p->getStride(id);
    const Pel *a = p->getAddr(id);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst.push_back((uint8_t)a[y * s + x]);
  }
}

int ref_index(TComPic *pic) {
  const int poc = pic->getPOC();
  auto it = g.refpic_index.find(poc);
  if (it != g.refpic_index.end()) return it->second;
  const int idx = (int)g.refpic_poc.size();
  g.refpic_index[poc] = idx;
  g.refpic_poc.push_back(poc);
  put_planes(pic->getPicYuvRec(), g.refpic);
  return idx;
}

void capture_picture(TEncCu *cu, TComDataCU *ctu) {
  TComPic *pic = ctu->getPic();
  TComSlice *s = ctu->getSlice();
  std::vector<int32_t> r(P_NFIELDS, 0);
  r[P_W] = s->getSPS()->getPicWidthInLumaSamples();
  r[P_H] = s->getSPS()->getPicHeightInLumaSamples();
  r[P_POC] = s->getPOC();
  r[P_SLICE_TYPE] = s->getSliceType();
  r[P_QP] = s->getSliceQp();
  for (int l = 0; l < 2; l++) {
    const int n = s->getSliceType() == I_SLICE ? 0 : (l == 1 && s->getSliceType() == P_SLICE ? 0 : s->getNumRefIdx(RefPicList(l)));
    r[l ? P_NREF1 : P_NREF0] = n;
    for (int i = 0; i < 4; i++) {
      r[(l ? P_REFPOC1 : P_REFPOC0) + i] = i < n ? s->getRefPOC(RefPicList(l), i) : -1;
      r[(l ? P_REFPIC1 : P_REFPIC0) + i] = i < n ? ref_index(s->getRefPic(RefPicList(l), i)) : -1;
    }
  }
  r[P_COL_FROM_L0] = s->getColFromL0Flag();
  r[P_COL_REF_IDX] = s->getColRefIdx();
  r[P_CHECK_LDC] = s->getCheckLDC();
  r[P_TMVP] = s->getEnableTMVPFlag();
  r[P_MAX_MERGE] = s->getMaxNumMergeCand();
  r[P_CABAC_TABLE] = s->getEncCABACTableIdx();
  r[P_FIRST_CTU] = g.nctu;
  r[P_NCTU] = pic->getPicSym()->getNumberOfCtusInFrame();
  r[P_LAMBDA_MOTION] = (int32_t)cu->m_pcRdCost->m_uiLambdaMotionSAD[0];
  for (int c = 1; c < 3; c++) {
    const QpParam q(*ctu, ComponentID(c));  // getScaledChromaQP of the slice QP (no CU QP offsets here)
    r[c == 1 ? P_CHROMA_QP_CB : P_CHROMA_QP_CR] = q.Qp;
  }
  // the collocated picture's compressed motion field (TComDataCU::xGetColMVP, TComDataCU.cpp:3061)
  if (s->getSliceType() != I_SLICE && s->getEnableTMVPFlag()) {
    TComPic *col = s->getRefPic(RefPicList(s->isInterB() ? 1 - s->getColFromL0Flag() : 0), s->getColRefIdx());
    TComSlice *cs = col->getSlice(0);
    r[P_COL_VALID] = 1;
    r[P_COL_POC] = cs->getPOC();
    for (int l = 0; l < 2; l++) {
      const int n = cs->getSliceType() == I_SLICE ? 0 : (l == 1 && cs->getSliceType() == P_SLICE ? 0 : cs->getNumRefIdx(RefPicList(l)));
      r[l ? P_COL_NREF1 : P_COL_NREF0] = n;
      for (int i = 0; i < 4; i++) r[(l ? P_COL_REFPOC1 : P_COL_REFPOC0) + i] = i < n ? cs->getRefPOC(RefPicList(l), i) : -1;
    }
    const int nctu = col->getPicSym()->getNumberOfCtusInFrame();
    for (int a = 0; a < nctu; a++) {
      TComDataCU *cc = col->getCtu(a);
      for (int z = 0; z < 256; z += 16) {
        const int ps = cc->getPartitionSize(z);
        g.col_field.push_back((int16_t)(ps == NUMBER_OF_PART_SIZES ? -1 : cc->getPredictionMode(z)));
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getRefIdx(z));
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getRefIdx(z));
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getMv(z).getHor());
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_0)->getMv(z).getVer());
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getMv(z).getHor());
        g.col_field.push_back((int16_t)cc->getCUMvField(REF_PIC_LIST_1)->getMv(z).getVer());
        g.col_field.push_back(0);
      }
    }
  }
  g.pic_i32.insert(g.pic_i32.end(), r.begin(), r.end());
  TComRdCost *rd = cu->m_pcRdCost;
  TComTrQuant *tq = cu->m_pcTrQuant;
  double f[F_NFIELDS] = {rd->getLambda(), rd->m_sqrtLambda, rd->m_distortionWeight[1], rd->m_distortionWeight[2],
                         tq->m_lambdas[0], tq->m_lambdas[1], tq->m_lambdas[2]};
  g.pic_f64.insert(g.pic_f64.end(), f, f + F_NFIELDS);
  put_planes(pic->getPicYuvOrg(), g.org);
  g.npic++;
}

void capture_entry(TEncCu *cu, TComDataCU *ctu) {
  TEncSbac *sb = cu->m_pppcRDSbacCoder[0][CI_CURR_BEST];
  for (int i = 0; i < Store::HVX_CTX; i++) g.ctu_states.push_back(sb->m_contextModels[i].m_ucState);
  g.ctu_frac.push_back(((TEncBinCABAC *)sb->m_pcBinIf)->m_fracBits);
  TEncSearch *se = cu->m_pcPredSearch;
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < 4; i++) {
      g.ctu_int2n.push_back((int16_t)se->m_integerMv2Nx2N[l][i].getHor());
      g.ctu_int2n.push_back((int16_t)se->m_integerMv2Nx2N[l][i].getVer());
    }
}

void capture_exit(TComDataCU *ctu) {
  TComPic *pic = ctu->getPic();
  const int addr = ctu->getCtuRsAddr();
  g.ctu_meta.push_back(g.npic - 1);
  g.ctu_meta.push_back(addr);
  g.ctu_meta.push_back((int32_t)ctu->getTotalBits());
  g.ctu_meta.push_back((int32_t)ctu->getTotalDistortion());
  g.ctu_cost.push_back(ctu->getTotalCost());
  for (int z = 0; z < 256; z++) {
    int16_t u[U_NFIELDS];
    u[U_DEPTH] = ctu->getDepth(z);
    u[U_PART] = ctu->getPartitionSize(z);
    u[U_PRED] = ctu->getPredictionMode(z);
    u[U_SKIP] = ctu->getSkipFlag(z);
    u[U_MERGE] = ctu->getMergeFlag(z);
    u[U_MERGE_IDX] = ctu->getMergeIndex(z);
    u[U_INTER_DIR] = ctu->getInterDir(z);
    for (int l = 0; l < 2; l++) {
      TComCUMvField *f = ctu->getCUMvField(RefPicList(l));
      u[U_REF0 + l] = f->getRefIdx(z);
      u[U_MV0X + 2 * l] = f->getMv(z).getHor();
      u[U_MV0Y + 2 * l] = f->getMv(z).getVer();
      u[U_MVD0X + 2 * l] = f->getMvd(z).getHor();
      u[U_MVD0Y + 2 * l] = f->getMvd(z).getVer();
      u[U_MVP0 + l] = ctu->getMVPIdx(RefPicList(l), z);
    }
    u[U_IDIR_Y] = ctu->getIntraDir(CHANNEL_TYPE_LUMA, z);
    u[U_IDIR_C] = ctu->getIntraDir(CHANNEL_TYPE_CHROMA, z);
    u[U_TRIDX] = ctu->getTransformIdx(z);
    for (int c = 0; c < 3; c++) {
      u[U_TS_Y + c] = ctu->getTransformSkip(z, ComponentID(c));
      u[U_CBF_Y + c] = ctu->getCbf(ComponentID(c))[z];
    }
    u[U_QP] = ctu->getQP(z);
    g.ctu_parts.insert(g.ctu_parts.end(), u, u + U_NFIELDS);
  }
  for (int c = 0; c < 3; c++) {
    const int n = c ? 1024 : 4096;
    const TCoeff *p = ctu->getCoeff(ComponentID(c));
    g.ctu_coef.insert(g.ctu_coef.end(), p, p + n);
  }
  TComPicYuv *rec = pic->getPicYuvRec();
  for (int c = 0; c < 3; c++) {
    const ComponentID id = ComponentID(c);
    const int sz = c ? 32 : 64, s = rec->getStride(id);
    const int x0 = ctu->getCUPelX() >> (c ? 1 : 0), y0 = ctu->getCUPelY() >> (c ? 1 : 0);
    const int w = rec->getWidth(id), h = rec->getHeight(id);
    const Pel *a = rec->getAddr(id);
    for (int y = 0; y < sz; y++)
      for (int x = 0; x < sz; x++)
        g.ctu_recon.push_back((x0 + x < w && y0 + y < h) ? (uint8_t)a[(y0 + y) * s + x0 + x] : 0);
  }
  g.nctu++;
}

// HVX_CAPTURE_POCS=<poc,poc,...>: record only the pictures of these POCs (the others are encoded
// unrecorded; their reconstructions still enter the capture when a recorded picture references them)
bool poc_selected(int poc) {
  const char *s = getenv("HVX_CAPTURE_POCS");
  if (!s || !*s) return true;
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

extern "C" void CAT(__wrap_, CU_SYM)(TEncCu *self, TComDataCU *ctu) {
  const int poc = ctu->getSlice()->getPOC();
  if (!poc_selected(poc)) {
    CAT(__real_, CU_SYM)(self, ctu);
    return;
  }
  if (poc != g.cur_poc) {
    g.cur_poc = poc;
    capture_picture(self, ctu);
  }
  capture_entry(self, ctu);
  CAT(__real_, CU_SYM)(self, ctu);
  capture_exit(ctu);
}
