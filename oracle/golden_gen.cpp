// golden_gen.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Links the reference HM-16.5rc1 objects (built by oracle/Makefile from
// /root/reference, into oracle/_ref/) and the reference stvssim.c, calls the
// reference functions on seeded synthetic inputs and writes golden vectors
// (inputs + expected outputs) to tests/golden/*.bin ("HVXG" container,
// golden_writer.h).  Those fixtures pin oracle/hvx_oracle.c and the HIP path.
//
// Access to HM's protected/private members is obtained the usual white-box
// way (access specifiers redefined for this translation unit only); no
// reference source is modified or copied.
//
// Reference functions exercised (file:line under hm-16.5rc1/source/Lib):
//   TComRdCost::setDistParam/DistFunc/getDistPart    TLibCommon/TComRdCost.cpp:294-451
//   TComInterpolationFilter::filterHor/filterVer     TLibCommon/TComInterpolationFilter.cpp:341,377
//   xTrMxN / xITrMxN                                 TLibCommon/TComTrQuant.cpp:860,927
//   TEncSearch::xSetSearchRange/xTZSearch/xPatternSearchFracDIF and the
//   final-cost lines of xMotionEstimation            TLibEncoder/TEncSearch.cpp:3663-3760,3881,4240
//   compute_SSIM / compute_stVSSIM                   stvssim_src/.../stvssim.c:491,587
// standard headers first: the access-specifier redefinition must not reach them
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
#define private public
#define protected public
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/TComRom.h"
#include "TLibCommon/TComRdCost.h"
#include "TLibCommon/TComYuv.h"
#include "TLibCommon/TComInterpolationFilter.h"
#include "TLibCommon/TComTrQuant.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComSlice.h"
#include "TLibEncoder/TEncSearch.h"
#include "TLibEncoder/TEncCfg.h"
#undef private
#undef protected
#include "golden_writer.h"
#include <cmath>
#include <cstdlib>

extern Void xTrMxN(Int bitDepth, TCoeff *block, TCoeff *coeff, Int iWidth, Int iHeight, Bool useDST, const Int maxLog2TrDynamicRange);
extern Void xITrMxN(Int bitDepth, TCoeff *coeff, TCoeff *block, Int iWidth, Int iHeight, Bool useDST, const Int maxLog2TrDynamicRange);

extern "C" {
float stv_compute_ssim(const uint8_t *org, const uint8_t *rec, int w, int h, int wint, int overlap, int comp);
float stv_compute_stvssim(const uint8_t *org_hist, const uint8_t *rec_hist, const float *dirs,
                          int w, int h, int wint, int overlap, int gama, int comp,
                          float *ssim, float *ssim3d, float *stvssim);
double stv_lambda_2(int qp);
double stv_adjust_lambda(double lambda, double eta);
}

static std::string g_out = "tests/golden";

// ---------------------------------------------------------------------------------------------
// PU shapes of a 64x64 CTU (2Nx2N, 2NxN, Nx2N, NxN, AMP) -- TComDataCU::getPartIndexAndSize
static std::vector<std::pair<int, int>> pu_shapes() {
  std::vector<std::pair<int, int>> v;
  for (int s = 64; s >= 8; s >>= 1) {
    v.push_back({s, s}); v.push_back({s, s / 2}); v.push_back({s / 2, s});
    if (s > 8) {  // NxN inter only at min CU; AMP only for CU >= 16
      v.push_back({s, s / 4}); v.push_back({s, 3 * s / 4});
      v.push_back({s / 4, s}); v.push_back({3 * s / 4, s});
    }
  }
  v.push_back({4, 8}); v.push_back({8, 4}); v.push_back({4, 4});
  return v;
}

// ---------------------------------------------------------------------------------------------
static void gen_dist() {
  // kinds: 0 = ME SAD (setDistParam(pattern) + FEN subsampling),  1 = ME SAD without FEN,
  //        2 = HADs (setDistParam(rcDP, ..., bHadamard=true)), 3 = SSE luma (getDistPart DF_SSE),
  //        4 = SSE chroma weighted (getDistPart COMPONENT_Cb), 5 = SAD generic (getDistPart DF_SAD)
  TComRdCost rd;
  rd.init();
  SplitMix64 rng(0x5EED1001);
  std::vector<int32_t> meta;
  std::vector<uint8_t> org, cur;
  std::vector<uint32_t> out;
  std::vector<double> weight;
  auto shapes = pu_shapes();
  int n = 0;
  for (int kind = 0; kind < 6; kind++) {
    for (auto wh : shapes) {
      int w = wh.first, h = wh.second;
      if (kind == 2 && ((w % 2) || (h % 2))) continue;
      for (int rep = 0; rep < 2; rep++) {
        std::vector<uint8_t> o(64 * 64), c(64 * 64);
        int mode = rng.range(0, 2);  // 0: uniform, 1: correlated (small diffs), 2: extreme
        for (int i = 0; i < 64 * 64; i++) {
          o[i] = rng.u8();
          if (mode == 0) c[i] = rng.u8();
          else if (mode == 1) { int v = o[i] + rng.range(-12, 12); c[i] = v < 0 ? 0 : v > 255 ? 255 : v; }
          else { o[i] = (rng.next() & 1) ? 255 : 0; c[i] = (rng.next() & 1) ? 255 : 0; }
        }
        Pel po[64 * 64], pc[64 * 64];
        for (int i = 0; i < 64 * 64; i++) { po[i] = o[i]; pc[i] = c[i]; }
        Distortion d = 0;
        int sub = 0;
        double wgt = 1.0;
        DistParam dp;
        dp.bApplyWeight = false;
        dp.bitDepth = 8;
        if (kind == 0 || kind == 1) {
          TComPattern pat;
          pat.initPattern(po, w, h, 64, 8);
          rd.setDistParam(&pat, pc, 64, dp);
          if (kind == 0 && dp.iRows > 8) dp.iSubShift = 1;
          sub = dp.iSubShift;
          dp.bitDepth = 8; dp.bApplyWeight = false; dp.compIdx = COMPONENT_Y;
          d = dp.DistFunc(&dp);
        } else if (kind == 2) {
          rd.setDistParam(dp, 8, po, 64, pc, 64, w, h, true);
          dp.bApplyWeight = false; dp.compIdx = COMPONENT_Y;
          d = dp.DistFunc(&dp);
        } else if (kind == 3) {
          d = rd.getDistPart(8, pc, 64, po, 64, w, h, COMPONENT_Y, DF_SSE);
        } else if (kind == 4) {
          wgt = 1.0 + (rng.next() % 1000) / 997.0;  // chroma distortion weight (TEncSlice.cpp:158)
          rd.setDistortionWeight(COMPONENT_Cb, wgt);
          d = rd.getDistPart(8, pc, 64, po, 64, w, h, COMPONENT_Cb, DF_SSE);
        } else {
          d = rd.getDistPart(8, pc, 64, po, 64, w, h, COMPONENT_Y, DF_SAD);
        }
        meta.insert(meta.end(), {kind, w, h, sub});
        org.insert(org.end(), o.begin(), o.end());
        cur.insert(cur.end(), c.begin(), c.end());
        out.push_back(d);
        weight.push_back(wgt);
        n++;
      }
    }
  }
  GoldenWriter gw;
  gw.add("meta", "i32", {(uint32_t)n, 4}, meta);
  gw.add("org", "u8", {(uint32_t)n, 64, 64}, org);
  gw.add("cur", "u8", {(uint32_t)n, 64, 64}, cur);
  gw.add("weight", "f64", {(uint32_t)n}, weight);
  gw.add("out", "u32", {(uint32_t)n}, out);
  gw.write(g_out + "/dist.bin");
}

// ---------------------------------------------------------------------------------------------
static void gen_interp() {
  TComInterpolationFilter ifl;
  SplitMix64 rng(0x5EED1002);
  std::vector<int32_t> meta;
  std::vector<int16_t> src, out;
  int n = 0;
  const int S = 80, O = 8;  // src buffer 80x80, block origin at (8,8)
  int sizes[][2] = {{64, 64}, {32, 16}, {16, 64}, {8, 8}, {8, 4}, {4, 8}, {12, 16}, {48, 64}, {64, 65}, {65, 64}, {2, 4}, {4, 2}, {16, 16}};
  for (int isLuma = 1; isLuma >= 0; isLuma--) {
    int nfrac = isLuma ? 4 : 8;
    for (int dir = 0; dir < 2; dir++) {
      for (int frac = 0; frac < nfrac; frac++) {
        for (int fl = 0; fl < 4; fl++) {
          bool isFirst = fl & 1, isLast = (fl >> 1) & 1;
          if (dir == 0 && !isFirst) continue;  // filterHor is always first
          for (int pick = 0; pick < 2; pick++) {
            auto &sz = sizes[rng.range(0, (int)(sizeof(sizes) / sizeof(sizes[0])) - 1)];
            int w = sz[0], h = sz[1];
            if (w > 64 + 8 || h > 64 + 8) continue;
            std::vector<int16_t> s(S * S);
            Pel ps[S * S], pd[80 * 80];
            if (isFirst) {
              for (int i = 0; i < S * S; i++) s[i] = rng.u8();
            } else {  // intermediate-domain input: output of a non-last first stage
              for (int i = 0; i < S * S; i++) {
                int v = (int)rng.u8() * 64 - 8192 + rng.range(-600, 600);
                s[i] = v < -14312 ? -14312 : v > 14248 ? 14248 : v;
              }
            }
            for (int i = 0; i < S * S; i++) ps[i] = s[i];
            for (int i = 0; i < 80 * 80; i++) pd[i] = 0;
            ComponentID comp = isLuma ? COMPONENT_Y : COMPONENT_Cb;
            if (dir == 0) ifl.filterHor(comp, ps + O * S + O, S, pd, 80, w, h, frac, isLast, CHROMA_420, 8);
            else ifl.filterVer(comp, ps + O * S + O, S, pd, 80, w, h, frac, isFirst, isLast, CHROMA_420, 8);
            std::vector<int16_t> o(80 * 80);
            for (int i = 0; i < 80 * 80; i++) o[i] = pd[i];
            meta.insert(meta.end(), {isLuma, dir, frac, (int)isFirst, (int)isLast, w, h});
            src.insert(src.end(), s.begin(), s.end());
            out.insert(out.end(), o.begin(), o.end());
            n++;
          }
        }
      }
    }
  }
  GoldenWriter gw;
  gw.add("meta", "i32", {(uint32_t)n, 7}, meta);
  gw.add("src", "i16", {(uint32_t)n, S, S}, src);   // block origin at [8][8], stride 80
  gw.add("out", "i16", {(uint32_t)n, 80, 80}, out);  // stride 80
  gw.write(g_out + "/interp.bin");
}

// ---------------------------------------------------------------------------------------------
static void gen_xform() {
  SplitMix64 rng(0x5EED1003);
  std::vector<int32_t> meta, fin, fout, iin, iout;
  int n = 0;
  for (int log2 = 2; log2 <= 5; log2++) {
    int N = 1 << log2;
    for (int dst = 0; dst < (N == 4 ? 2 : 1); dst++) {
      for (int rep = 0; rep < 6; rep++) {
        TCoeff blk[32 * 32] = {0}, co[32 * 32] = {0}, ci[32 * 32] = {0}, ro[32 * 32] = {0};
        int mode = rep % 3;
        for (int i = 0; i < N * N; i++) {
          if (mode == 0) blk[i] = rng.range(-255, 255);
          else if (mode == 1) blk[i] = rng.range(-20, 20);
          else blk[i] = (rng.next() & 1) ? 255 : -255;
        }
        xTrMxN(8, blk, co, N, N, dst, 15);
        for (int i = 0; i < N * N; i++) {
          if (mode == 2) ci[i] = (rng.next() & 1) ? 32767 : -32768;  // clip stress
          else ci[i] = rng.range(-4000, 4000) >> (mode * 3);
        }
        TCoeff cin[32 * 32];
        memcpy(cin, ci, sizeof(ci));
        xITrMxN(8, cin, ro, N, N, dst, 15);
        std::vector<int32_t> a(32 * 32, 0), b(32 * 32, 0), c(32 * 32, 0), d(32 * 32, 0);
        for (int i = 0; i < N * N; i++) { a[i] = blk[i]; b[i] = co[i]; c[i] = ci[i]; d[i] = ro[i]; }
        meta.insert(meta.end(), {N, dst});
        fin.insert(fin.end(), a.begin(), a.end()); fout.insert(fout.end(), b.begin(), b.end());
        iin.insert(iin.end(), c.begin(), c.end()); iout.insert(iout.end(), d.begin(), d.end());
        n++;
      }
    }
  }
  GoldenWriter gw;
  gw.add("meta", "i32", {(uint32_t)n, 2}, meta);
  gw.add("fwd_in", "i32", {(uint32_t)n, 32 * 32}, fin);
  gw.add("fwd_out", "i32", {(uint32_t)n, 32 * 32}, fout);
  gw.add("inv_in", "i32", {(uint32_t)n, 32 * 32}, iin);
  gw.add("inv_out", "i32", {(uint32_t)n, 32 * 32}, iout);
  gw.write(g_out + "/xform.bin");
}

// ---------------------------------------------------------------------------------------------
// Motion estimation: xMotionEstimation's uni-prediction path (TZ integer search + half/quarter
// refinement + final cost), TEncSearch.cpp:3663-3760, on synthetic padded 8-bit planes.
static const int MARGIN = 80;

struct Plane {
  int w, h, stride;
  std::vector<Pel> buf;
  Pel *org() { return buf.data() + MARGIN * stride + MARGIN; }
  void init(int W, int H) { w = W; h = H; stride = W + 2 * MARGIN; buf.assign((size_t)stride * (H + 2 * MARGIN), 0); }
  void extend() {  // TComPicYuv::extendPicBorder (replicate edges)
    Pel *p = org();
    for (int y = 0; y < h; y++) {
      for (int x = -MARGIN; x < 0; x++) p[y * stride + x] = p[y * stride];
      for (int x = w; x < w + MARGIN; x++) p[y * stride + x] = p[y * stride + w - 1];
    }
    for (int y = -MARGIN; y < 0; y++) memcpy(p + y * stride - MARGIN, p - MARGIN, stride * sizeof(Pel));
    for (int y = h; y < h + MARGIN; y++) memcpy(p + y * stride - MARGIN, p + (h - 1) * stride - MARGIN, stride * sizeof(Pel));
  }
};

static void gen_me() {
  const int W = 416, H = 240;
  SplitMix64 rng(0x5EED1004);
  GoldenWriter gw;
  std::vector<int32_t> jobs, res;
  std::vector<double> lambdas;
  std::vector<uint8_t> planes;
  int njobs = 0;

  TEncCfg cfg;
  cfg.m_iFastSearch = 1;
  cfg.m_bUseFastEnc = true;
  cfg.m_bFastMEAssumingSmootherMVEnabled = true;
  cfg.m_bUseHADME = true;
  cfg.m_iSearchRange = 64;
  TComRdCost rd;
  rd.init();
  TEncSearch es;
  es.m_pcEncCfg = &cfg;
  es.m_pcRdCost = &rd;
  es.m_iSearchRange = 64;
  es.m_iFastSearch = 1;
  es.initTempBuff(CHROMA_420);
  es.m_cDistParam.bApplyWeight = false;

  TComSPS sps;
  sps.setPicWidthInLumaSamples(W);
  sps.setPicHeightInLumaSamples(H);
  sps.setMaxCUWidth(64);
  sps.setMaxCUHeight(64);
  sps.setBitDepth(CHANNEL_TYPE_LUMA, 8);
  sps.setBitDepth(CHANNEL_TYPE_CHROMA, 8);
  TComSlice slice;
  slice.setSPS(&sps);
  TComDataCU cu;
  cu.m_pcSlice = &slice;

  for (int pair = 0; pair < 3; pair++) {
    Plane cur, ref;
    cur.init(W, H); ref.init(W, H);
    // pair 0: independent uniform random frames (the bench workload)
    // pair 1: ref = smooth texture, cur = ref shifted by (dx,dy) + noise (real motion)
    // pair 2: same as 1 with a larger shift
    int dx = pair == 1 ? 3 : -17, dy = pair == 1 ? -2 : 9;
    std::vector<int> tex((W + 64) * (H + 64));
    for (int y = 0; y < H + 64; y++)
      for (int x = 0; x < W + 64; x++)
        tex[y * (W + 64) + x] = (int)(128 + 60 * sin(x * 0.11 + y * 0.05) + 40 * cos(y * 0.13 - x * 0.03)) + rng.range(-6, 6);
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        if (pair == 0) { ref.org()[y * ref.stride + x] = rng.u8(); cur.org()[y * cur.stride + x] = rng.u8(); }
        else {
          int v = tex[(y + 32) * (W + 64) + x + 32];
          ref.org()[y * ref.stride + x] = v < 0 ? 0 : v > 255 ? 255 : v;
          int u = tex[(y + 32 + dy) * (W + 64) + x + 32 + dx] + rng.range(-3, 3);
          cur.org()[y * cur.stride + x] = u < 0 ? 0 : u > 255 ? 255 : u;
        }
      }
    cur.extend(); ref.extend();
    for (auto &p : {&cur, &ref})
      for (auto v : p->buf) planes.push_back((uint8_t)v);

    auto shapes = pu_shapes();
    for (int j = 0; j < 110; j++) {
      // random CTU, random CU depth, random PU inside it
      auto wh = shapes[rng.range(0, (int)shapes.size() - 1)];
      int pw = wh.first, ph = wh.second;
      int cuSize = 64;
      while (cuSize > 8 && (cuSize / 2 >= pw && cuSize / 2 >= ph)) cuSize >>= 1;
      if (pw < cuSize && ph < cuSize && cuSize > 8) cuSize = std::max(pw, ph);
      int ctux = rng.range(0, (W - 1) / 64), ctuy = rng.range(0, (H - 1) / 64);
      int cux = ctux * 64 + rng.range(0, 64 / cuSize - 1) * cuSize;
      int cuy = ctuy * 64 + rng.range(0, 64 / cuSize - 1) * cuSize;
      int pux = cux + (pw < cuSize ? rng.range(0, (cuSize - pw) / 4) * 4 : 0);
      int puy = cuy + (ph < cuSize ? rng.range(0, (cuSize - ph) / 4) * 4 : 0);
      if (pux + pw > cux + cuSize) pux = cux + cuSize - pw;
      if (puy + ph > cuy + cuSize) puy = cuy + cuSize - ph;
      // The reference pads partial CTUs; restrict PUs to lie in the picture like HM does.
      if (pux + pw > W || puy + ph > H) { j--; continue; }
      cu.m_uiCUPelX = cux;
      cu.m_uiCUPelY = cuy;
      int qp = rng.range(22, 37);
      double lambda = 0.57 * pow(2.0, (qp - 12) / 3.0) * (rng.range(0, 1) ? 1.0 : 0.68);
      rd.setLambda(lambda, sps.getBitDepths());
      TComMv pred(rng.range(-40, 40), rng.range(-40, 40));
      if (j % 5 == 0) pred.set(0, 0);
      if (j % 7 == 1) pred.set(rng.range(-700, 700), rng.range(-500, 500));  // far / clipped predictor
      int use2Nx2N = (j % 3 == 0);
      TComMv int2Nx2N(rng.range(-30, 30), rng.range(-30, 30));
      UInt bitsIn = rng.range(0, 9);

      // ---- xMotionEstimation (uni-pred, TEncSearch.cpp:3663-3760) ----
      TComPattern pat;
      pat.initPattern(cur.org() + puy * cur.stride + pux, pw, ph, cur.stride, 8);
      Pel *piRefY = ref.org() + puy * ref.stride + pux;
      TComMv lt, rb, mv;
      es.xSetSearchRange(&cu, pred, 64, lt, rb);
      rd.getMotionCost(true, 0, false);
      rd.setPredictor(pred);
      rd.setCostScale(2);
      mv = pred;
      Distortion sad = 0;
      TComMv i2 = int2Nx2N;
      es.xTZSearch(&cu, &pat, piRefY, ref.stride, &lt, &rb, mv, sad, use2Nx2N ? &i2 : NULL);
      TComMv mvInt = mv;
      Distortion sadInt = sad;
      rd.getMotionCost(true, 0, false);
      rd.setCostScale(1);
      TComMv half, qter;
      Distortion cost = 0;
      es.xPatternSearchFracDIF(false, &pat, piRefY, ref.stride, &mv, half, qter, cost);
      TComMv mvHalf = half, mvQ = qter;
      Distortion costFrac = cost;
      rd.setCostScale(0);
      mv <<= 2;
      mv += (half <<= 1);
      mv += qter;
      UInt mvBits = rd.getBits(mv.getHor(), mv.getVer());
      UInt bits = bitsIn + mvBits;
      Distortion fin = (Distortion)(floor(1.0 * ((Double)costFrac - (Double)rd.getCost(mvBits))) + (Double)rd.getCost(bits));

      jobs.insert(jobs.end(), {pair, cux, cuy, pux, puy, pw, ph, pred.getHor(), pred.getVer(), use2Nx2N,
                               int2Nx2N.getHor(), int2Nx2N.getVer(), (int)bitsIn, qp});
      lambdas.push_back(lambda);
      res.insert(res.end(), {mvInt.getHor(), mvInt.getVer(), (int)sadInt, mvHalf.getHor(), mvHalf.getVer(),
                             mvQ.getHor(), mvQ.getVer(), (int)costFrac, mv.getHor(), mv.getVer(), (int)bits, (int)fin});
      njobs++;
    }
  }
  gw.add("dims", "i32", {4}, std::vector<int32_t>{W, H, MARGIN, 64});
  gw.add("planes", "u8", {3, 2, (uint32_t)(H + 2 * MARGIN), (uint32_t)(W + 2 * MARGIN)}, planes);
  gw.add("jobs", "i32", {(uint32_t)njobs, 14}, jobs);
  gw.add("lambda", "f64", {(uint32_t)njobs}, lambdas);
  gw.add("res", "i32", {(uint32_t)njobs, 12}, res);
  gw.write(g_out + "/me.bin");
  es.m_pcEncCfg = NULL;  // TEncSearch::init() was not run; keep its destructor off the layer buffers
  cu.m_pcSlice = NULL;
}

// ---------------------------------------------------------------------------------------------
static void gen_ssim() {
  SplitMix64 rng(0x5EED1005);
  const int HN = 26, B = 32;
  std::vector<int32_t> meta;
  std::vector<uint8_t> orgh, rech;
  std::vector<float> dirs, out;
  std::vector<double> lam;
  int n = 0;
  int shapes[][2] = {{16, 16}, {8, 8}, {32, 32}, {16, 8}, {32, 16}};
  for (int rep = 0; rep < 20; rep++) {
    int w = shapes[rep % 5][0], h = shapes[rep % 5][1];
    int comp = (rep / 5) % 2;
    int gama = rep < 10 ? 1 + rep : (rep * 7) % 40 + 1;
    int wint = (rep % 7 == 3) ? 4 : 8;
    int overlap = (rep % 4 == 1) ? 2 : 4;
    std::vector<uint8_t> o(HN * B * B), r(HN * B * B);
    for (int f = 0; f < HN; f++)
      for (int i = 0; i < B * B; i++) {
        int base = (int)(120 + 50 * sin(i * 0.07 + f * 0.3)) + rng.range(-20, 20);
        o[f * B * B + i] = base < 0 ? 0 : base > 255 ? 255 : base;
        int v = o[f * B * B + i] + rng.range(-(rep % 6) * 4, (rep % 6) * 4);
        r[f * B * B + i] = v < 0 ? 0 : v > 255 ? 255 : v;
      }
    std::vector<float> d(2 * B * 2 * B);
    for (auto &x : d) x = (float)((rng.next() % 3142) / 1000.0);
    float ssim = stv_compute_ssim(o.data() + (HN - 1) * B * B, r.data() + (HN - 1) * B * B, w, h, wint, overlap, comp);
    float s1, s2, s3;
    float ret = stv_compute_stvssim(o.data(), r.data(), d.data(), w, h, wint, overlap, gama, comp, &s1, &s2, &s3);
    meta.insert(meta.end(), {w, h, wint, overlap, gama, comp});
    orgh.insert(orgh.end(), o.begin(), o.end());
    rech.insert(rech.end(), r.begin(), r.end());
    dirs.insert(dirs.end(), d.begin(), d.end());
    out.insert(out.end(), {ssim, s1, s2, s3, ret});
    n++;
  }
  for (int qp = 0; qp <= 51; qp++) {
    lam.push_back(stv_lambda_2(qp));
    lam.push_back(stv_adjust_lambda(stv_lambda_2(qp), 0.25 + qp * 0.05));
  }
  GoldenWriter gw;
  gw.add("meta", "i32", {(uint32_t)n, 6}, meta);
  gw.add("org_hist", "u8", {(uint32_t)n, HN, B, B}, orgh);  // [HN-1] is the current frame
  gw.add("rec_hist", "u8", {(uint32_t)n, HN, B, B}, rech);
  gw.add("dirs", "f32", {(uint32_t)n, 2 * B, 2 * B}, dirs);
  gw.add("out", "f32", {(uint32_t)n, 5}, out);
  gw.add("lambda", "f64", {52, 2}, lam);
  gw.write(g_out + "/ssim.bin");
}

// xMotionEstimation with the integer full search (TEncSearch.cpp:3663-3760, xPatternSearch
// :3786): FastSearch=0 jobs (SR 16/64 around the predictor, pattern = the original) and
// bi-prediction refinement jobs (bBi: pattern = removeHighFreq target 2*org - other,
// TComYuv.cpp:409, unclipped; SR = BipredSearchRange 4 around the list's current MV; final
// cost weighted by 0.5).
static void gen_me_full() {
  const int W = 416, H = 240;
  SplitMix64 rng(0x5EED1005);
  GoldenWriter gw;
  std::vector<int32_t> jobs, res;
  std::vector<double> lambdas;
  std::vector<uint8_t> planes;
  std::vector<int16_t> targets;
  int njobs = 0;

  TEncCfg cfg;
  cfg.m_iFastSearch = 0;
  cfg.m_bUseFastEnc = true;
  cfg.m_bUseHADME = true;
  cfg.m_iSearchRange = 64;
  TComRdCost rd;
  rd.init();
  TEncSearch es;
  es.m_pcEncCfg = &cfg;
  es.m_pcRdCost = &rd;
  es.m_iSearchRange = 64;
  es.m_iFastSearch = 0;
  es.initTempBuff(CHROMA_420);
  es.m_cDistParam.bApplyWeight = false;

  TComSPS sps;
  sps.setPicWidthInLumaSamples(W);
  sps.setPicHeightInLumaSamples(H);
  sps.setMaxCUWidth(64);
  sps.setMaxCUHeight(64);
  sps.setBitDepth(CHANNEL_TYPE_LUMA, 8);
  sps.setBitDepth(CHANNEL_TYPE_CHROMA, 8);
  TComSlice slice;
  slice.setSPS(&sps);
  TComDataCU cu;
  cu.m_pcSlice = &slice;

  for (int pair = 0; pair < 2; pair++) {
    Plane cur, ref;
    cur.init(W, H); ref.init(W, H);
    std::vector<int> tex((W + 64) * (H + 64));
    for (int y = 0; y < H + 64; y++)
      for (int x = 0; x < W + 64; x++)
        tex[y * (W + 64) + x] = (int)(128 + 60 * sin(x * 0.09 + y * 0.04) + 40 * cos(y * 0.12 - x * 0.05)) + rng.range(-6, 6);
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        if (pair == 0) { ref.org()[y * ref.stride + x] = rng.u8(); cur.org()[y * cur.stride + x] = rng.u8(); }
        else {
          int v = tex[(y + 32) * (W + 64) + x + 32];
          ref.org()[y * ref.stride + x] = v < 0 ? 0 : v > 255 ? 255 : v;
          int u = tex[(y + 32 - 5) * (W + 64) + x + 32 + 7] + rng.range(-3, 3);
          cur.org()[y * cur.stride + x] = u < 0 ? 0 : u > 255 ? 255 : u;
        }
      }
    cur.extend(); ref.extend();
    for (auto &p : {&cur, &ref})
      for (auto v : p->buf) planes.push_back((uint8_t)v);

    auto shapes = pu_shapes();
    for (int j = 0; j < 60; j++) {
      auto wh = shapes[rng.range(0, (int)shapes.size() - 1)];
      int pw = wh.first, ph = wh.second;
      int cuSize = 64;
      while (cuSize > 8 && (cuSize / 2 >= pw && cuSize / 2 >= ph)) cuSize >>= 1;
      if (pw < cuSize && ph < cuSize && cuSize > 8) cuSize = std::max(pw, ph);
      int ctux = rng.range(0, (W - 1) / 64), ctuy = rng.range(0, (H - 1) / 64);
      int cux = ctux * 64 + rng.range(0, 64 / cuSize - 1) * cuSize;
      int cuy = ctuy * 64 + rng.range(0, 64 / cuSize - 1) * cuSize;
      int pux = cux + (pw < cuSize ? rng.range(0, (cuSize - pw) / 4) * 4 : 0);
      int puy = cuy + (ph < cuSize ? rng.range(0, (cuSize - ph) / 4) * 4 : 0);
      if (pux + pw > cux + cuSize) pux = cux + cuSize - pw;
      if (puy + ph > cuy + cuSize) puy = cuy + cuSize - ph;
      if (pux + pw > W || puy + ph > H) { j--; continue; }
      cu.m_uiCUPelX = cux;
      cu.m_uiCUPelY = cuy;
      int qp = rng.range(22, 37);
      double lambda = 0.57 * pow(2.0, (qp - 12) / 3.0) * (rng.range(0, 1) ? 1.0 : 0.68);
      rd.setLambda(lambda, sps.getBitDepths());
      const bool bi = (j % 2) == 1;
      const int sr = bi ? 4 : ((j % 4) == 0 ? 64 : 16);
      TComMv pred(rng.range(-40, 40), rng.range(-40, 40));
      if (j % 7 == 3) pred.set(rng.range(-700, 700), rng.range(-500, 500));  // far / clipped predictor
      TComMv center = bi ? TComMv(pred.getHor() + rng.range(-24, 24), pred.getVer() + rng.range(-24, 24)) : pred;
      if (bi && j % 9 == 5) center.set(rng.range(-600, 600), rng.range(-400, 400));
      UInt bitsIn = rng.range(0, 9);

      // the search pattern: the original, or the bi target 2*org - other (removeHighFreq, no clip)
      std::vector<Pel> tgt(64 * 64, 0);
      for (int y = 0; y < ph; y++)
        for (int x = 0; x < pw; x++) {
          const int o = cur.org()[(puy + y) * cur.stride + pux + x];
          const int other = bi ? (int)((o + rng.range(-40, 40)) < 0 ? 0 : (o + rng.range(-40, 40)) > 255 ? 255 : (o + rng.range(-40, 40))) : 0;
          tgt[y * 64 + x] = (Pel)(bi ? 2 * o - other : o);
        }
      TComPattern pat;
      pat.initPattern(tgt.data(), pw, ph, 64, 8);
      Pel *piRefY = ref.org() + puy * ref.stride + pux;
      TComMv lt, rb, mv;
      es.xSetSearchRange(&cu, center, sr, lt, rb);
      rd.getMotionCost(true, 0, false);
      rd.setPredictor(pred);
      rd.setCostScale(2);
      Distortion sad = 0;
      es.xPatternSearch(&pat, piRefY, ref.stride, &lt, &rb, mv, sad);
      TComMv mvInt = mv;
      Distortion sadInt = sad;
      rd.getMotionCost(true, 0, false);
      rd.setCostScale(1);
      TComMv half, qter;
      Distortion cost = 0;
      es.xPatternSearchFracDIF(false, &pat, piRefY, ref.stride, &mv, half, qter, cost);
      TComMv mvHalf = half, mvQ = qter;
      Distortion costFrac = cost;
      rd.setCostScale(0);
      mv <<= 2;
      mv += (half <<= 1);
      mv += qter;
      UInt mvBits = rd.getBits(mv.getHor(), mv.getVer());
      UInt bits = bitsIn + mvBits;
      const double wgt = bi ? 0.5 : 1.0;
      Distortion fin = (Distortion)(floor(wgt * ((Double)costFrac - (Double)rd.getCost(mvBits))) + (Double)rd.getCost(bits));

      jobs.insert(jobs.end(), {pair, cux, cuy, pux, puy, pw, ph, pred.getHor(), pred.getVer(), bi ? 1 : 0,
                               center.getHor(), center.getVer(), (int)bitsIn, qp, sr});
      lambdas.push_back(lambda);
      targets.insert(targets.end(), tgt.begin(), tgt.end());
      res.insert(res.end(), {mvInt.getHor(), mvInt.getVer(), (int)sadInt, mvHalf.getHor(), mvHalf.getVer(),
                             mvQ.getHor(), mvQ.getVer(), (int)costFrac, mv.getHor(), mv.getVer(), (int)bits, (int)fin});
      njobs++;
    }
  }
  gw.add("dims", "i32", {4}, std::vector<int32_t>{W, H, MARGIN, 64});
  gw.add("planes", "u8", {2, 2, (uint32_t)(H + 2 * MARGIN), (uint32_t)(W + 2 * MARGIN)}, planes);
  gw.add("jobs", "i32", {(uint32_t)njobs, 15}, jobs);
  gw.add("lambda", "f64", {(uint32_t)njobs}, lambdas);
  gw.add("targets", "i16", {(uint32_t)njobs, 64, 64}, targets);
  gw.add("res", "i32", {(uint32_t)njobs, 12}, res);
  gw.write(g_out + "/me_full.bin");
  es.m_pcEncCfg = NULL;
  cu.m_pcSlice = NULL;
}

// TComYuv::addAvg (TComYuv.cpp:352) on random 14-bit intermediates, 4:2:0, several PU sizes
static void gen_addavg() {
  SplitMix64 rng(0x5EED0A06);
  const int shapes[][2] = {{64, 64}, {32, 32}, {16, 16}, {8, 8}, {16, 8}, {8, 16}, {64, 16}, {12, 16}, {32, 24}, {8, 4}, {4, 8}};
  const int n = sizeof(shapes) / sizeof(shapes[0]);
  std::vector<int32_t> meta;
  std::vector<int16_t> in0, in1, out;
  BitDepths bd;
  bd.recon[CHANNEL_TYPE_LUMA] = 8;
  bd.recon[CHANNEL_TYPE_CHROMA] = 8;
  for (int i = 0; i < n; i++) {
    const int w = shapes[i][0], h = shapes[i][1];
    TComYuv a, b, d;
    a.create(64, 64, CHROMA_420);
    b.create(64, 64, CHROMA_420);
    d.create(64, 64, CHROMA_420);
    for (int c = 0; c < 3; c++) {
      const ComponentID id = ComponentID(c);
      for (int k = 0; k < a.getHeight(id) * a.getStride(id); k++) {
        // first-stage-like intermediates: (sample << 6) - 8192 plus filter overshoot
        a.getAddr(id)[k] = (Pel)rng.range(-8192 - 2600, 8192 + 2600);
        b.getAddr(id)[k] = (Pel)rng.range(-8192 - 2600, 8192 + 2600);
      }
    }
    d.addAvg(&a, &b, 0, w, h, bd);
    meta.insert(meta.end(), {w, h});
    for (int c = 0; c < 3; c++) {
      const ComponentID id = ComponentID(c);
      const int cw = c ? w >> 1 : w, ch = c ? h >> 1 : h, st = a.getStride(id);
      for (int y = 0; y < ch; y++)
        for (int x = 0; x < cw; x++) {
          in0.push_back(a.getAddr(id)[y * st + x]);
          in1.push_back(b.getAddr(id)[y * st + x]);
          out.push_back(d.getAddr(id)[y * st + x]);
        }
    }
    a.destroy();
    b.destroy();
    d.destroy();
  }
  GoldenWriter gw;
  gw.add("meta", "i32", {(uint32_t)n, 2}, meta);
  gw.add("in0", "i16", {(uint32_t)in0.size()}, in0);
  gw.add("in1", "i16", {(uint32_t)in1.size()}, in1);
  gw.add("out", "i16", {(uint32_t)out.size()}, out);
  gw.write(g_out + "/addavg.bin");
}

int main(int argc, char **argv) {
  if (argc > 1) g_out = argv[1];
  initROM();
  gen_dist();
  gen_interp();
  gen_xform();
  gen_me();
  gen_ssim();
  gen_addavg();
  gen_me_full();
  destroyROM();
  return 0;
}
