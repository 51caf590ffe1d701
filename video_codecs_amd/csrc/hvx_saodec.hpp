// hvx_saodec.hpp -- SAO's RD decision on the device (hvx_sao_decide, include/hvx.h):
// TEncSampleAdaptiveOffset::decideBlkParams (TEncSampleAdaptiveOffset.cpp:763) for one picture per
// wave.  Restates oracle/hvx_oracle.c hvxo_sao_decide, pinned against the reference's SAOProcess
// decisions (tests/golden/saodec.bin).
//
// The decision is serial over the picture's CTUs (the RD coder's two SAO contexts and the merge
// candidates carry from CTU to CTU), but per CTU the 15 (component, type) offset derivations
// (deriveOffsets :447 with its estIterOffset :414 searches, invertQuantOffsets, getDistortion :370)
// are independent: lanes 0..14 compute them into LDS, then lane 0 runs the mode comparisons, the
// SAO syntax rates (TEncSbac::codeSAOBlkParam TEncSbac.cpp:1683, codeSAOOffsetParam :1605) and the
// parameter reconstruction with the reference's operations in the reference's order.  8-bit only:
// DISTORTION_PRECISION_ADJUSTMENT 0, offset step log2 0, maximum offset 7.
#pragma once
#include "hvx_dev.hpp"

namespace hvxi {
namespace saod {

struct Off {  // SAOOffset: modeIdc (0 off, 1 new, 2 merge), typeIdc, typeAuxInfo, offset[32]
  int mode, type, aux;
  int8_t offset[32];
};
struct Blk { Off c[3]; };
struct Coder { uint8_t st[2]; uint64_t frac; };  // the RD counter: sao_merge, sao_type_idx
struct Env { const int32_t *eb; const double *lambda; const int *en; };

__device__ __forceinline__ void bin(const Env &e, Coder &c, int ctx, int v) {  // TEncBinCABACCounter::encodeBin
  const int s = c.st[ctx], p = s >> 1, mps = s & 1;
  c.frac += (uint64_t)(uint32_t)e.eb[s ^ v];
  if (v == mps) c.st[ctx] = (uint8_t)(((p < 62 ? p + 1 : p) << 1) | mps);
  else c.st[ctx] = (uint8_t)((cab::kTransIdxLps[p] << 1) | (p == 0 ? mps ^ 1 : mps));
}
__device__ __forceinline__ void ep(Coder &c, int n) { c.frac += 32768ull * (uint64_t)n; }
__device__ __forceinline__ uint32_t written(const Coder &c) { return (uint32_t)(c.frac >> 15); }
__device__ __forceinline__ void reset_bits(Coder &c) { c.frac &= 32767; }

// codeSAOOffsetParam (TEncSbac.cpp:1605), codeSaoMaxUvlc (:1548) with maxSymbol 7
__device__ void code_offset(const Env &e, Coder &c, int comp, const Off &p) {
  if (!e.en[comp]) return;
  const bool first = comp != 2;
  if (first) {
    const int sym = p.mode == 0 ? 0 : p.type == 4 ? 1 : 2;
    bin(e, c, 1, sym != 0);
    if (sym) ep(c, 1);
  }
  if (p.mode == 1) {
    int off[4], k = 0;
    const int ncls = p.type == 4 ? 4 : 5;
    for (int i = 0; i < ncls; i++) {
      if (p.type != 4 && i == 2) continue;
      off[k++] = p.offset[p.type == 4 ? (p.aux + i) % 32 : i];
    }
    for (int i = 0; i < 4; i++) {
      const int a = off[i] < 0 ? -off[i] : off[i];
      ep(c, a == 0 ? 1 : a + (a < 7 ? 1 : 0));
    }
    if (p.type == 4) {
      for (int i = 0; i < 4; i++)
        if (off[i]) ep(c, 1);
      ep(c, 5);
    } else if (first) {
      ep(c, 2);
    }
  }
}
// codeSAOBlkParam (:1683)
__device__ void code_blk(const Env &e, Coder &c, const Blk &b, bool left, bool above, bool only_merge) {
  bool is_left = false, is_above = false;
  if (left) {
    is_left = b.c[0].mode == 2 && b.c[0].type == 0;
    bin(e, c, 0, is_left);
  }
  if (above && !is_left) {
    is_above = b.c[0].mode == 2 && b.c[0].type == 1;
    bin(e, c, 0, is_above);
  }
  if (only_merge) return;
  if (!is_left && !is_above)
    for (int k = 0; k < 3; k++) code_offset(e, c, k, b.c[k]);
}

__device__ __forceinline__ int64_t est_dist(int64_t count, int64_t offset, int64_t diff) {
  return (count * offset * offset - diff * offset * 2) >> 0;
}
// estIterOffset (:414)
__device__ int iter_offset(int type, double lambda, int in, int64_t count, int64_t diff, int64_t &best_dist, double &best_cost) {
  int it = in, out = 0;
  double min_cost = lambda;
  while (it != 0) {
    int64_t rate = type == 4 ? (abs(it) + 2) : (abs(it) + 1);
    if (abs(it) == 7) rate--;
    const int64_t dist = est_dist(count, (int64_t)it, diff);
    const double cost = ((double)dist + lambda * (double)rate);
    if (cost < min_cost) {
      min_cost = cost;
      out = it;
      best_dist = dist;
      best_cost = cost;
    }
    it = it > 0 ? it - 1 : it + 1;
  }
  return out;
}
// deriveOffsets (:447) -> coded offsets q[32] and band position; then invertQuantOffsets (step 1)
// and getDistortion (:370)
__device__ int64_t derive(double lambda, int type, const hvx_sao_stat &s, int8_t *q, int &aux) {
  int qq[32];
  for (int i = 0; i < 32; i++) qq[i] = 0;
  const int ncls = type == 4 ? 32 : 5;
  for (int i = 0; i < ncls; i++) {
    if (type != 4 && i == 2) continue;
    if (s.count[i] == 0) continue;
    const double x = (double)s.diff[i] / (double)s.count[i];
    const int v = (int)(x >= 0 ? (double)(int)(x + 0.5) : (double)(int)(x - 0.5));  // xRoundIbdi (8-bit)
    qq[i] = v < -7 ? -7 : v > 7 ? 7 : v;
  }
  aux = 0;
  if (type != 4) {
    for (int i = 0; i < 5; i++) {
      if ((i == 0 || i == 1) && qq[i] < 0) qq[i] = 0;
      if ((i == 3 || i == 4) && qq[i] > 0) qq[i] = 0;
      if (qq[i] != 0) {
        int64_t d = 0;
        double cst = 0;
        qq[i] = iter_offset(type, lambda, qq[i], s.count[i], s.diff[i], d, cst);
      }
    }
  } else {
    double cost_bo[32];
    for (int i = 0; i < 32; i++) {
      int64_t d = 0;
      cost_bo[i] = lambda;
      if (qq[i] != 0) qq[i] = iter_offset(type, lambda, qq[i], s.count[i], s.diff[i], d, cost_bo[i]);
    }
    double min_cost = 1.7e308;
    for (int b = 0; b < 32 - 4 + 1; b++) {
      double cst = cost_bo[b];
      cst += cost_bo[b + 1];
      cst += cost_bo[b + 2];
      cst += cost_bo[b + 3];
      if (cst < min_cost) { min_cost = cst; aux = b; }
    }
    int keep[32];
    for (int i = 0; i < 32; i++) keep[i] = 0;
    for (int i = 0; i < 4; i++) keep[(aux + i) % 32] = qq[(aux + i) % 32];
    for (int i = 0; i < 32; i++) qq[i] = keep[i];
  }
  for (int i = 0; i < 32; i++) q[i] = (int8_t)qq[i];
  // the de-quantised offsets are the coded ones (step 1), zero outside the coded classes
  int64_t d = 0;
  if (type != 4) {
    for (int i = 0; i < 5; i++) d += est_dist(s.count[i], qq[i], s.diff[i]);
  } else {
    for (int i = aux; i < aux + 4; i++) {
      const int b = i % 32;
      d += est_dist(s.count[b], qq[b], s.diff[b]);
    }
  }
  return d;
}
// getDistortion of reconstructed parameters (a merge candidate)
__device__ int64_t distortion(const Off &o, const hvx_sao_stat &s) {
  int64_t d = 0;
  if (o.type != 4) {
    for (int i = 0; i < 5; i++) d += est_dist(s.count[i], o.offset[i], s.diff[i]);
  } else {
    for (int i = o.aux; i < o.aux + 4; i++) {
      const int b = i % 32;
      d += est_dist(s.count[b], o.offset[b], s.diff[b]);
    }
  }
  return d;
}
// an hvx_sao_ctu component (applied form) back to a reconstructed SAOOffset
__device__ void from_applied(const hvx_sao_offset &a, Off &o) {
  o.mode = a.type < 0 ? 0 : 1;
  o.type = a.type < 0 ? 0 : a.type;
  o.aux = 0;
  for (int i = 0; i < 32; i++) o.offset[i] = 0;
  if (a.type == 4) {
    o.aux = a.band;
    for (int i = 0; i < 4; i++) o.offset[(a.band + i) % 32] = a.offset[i];
  } else if (a.type >= 0) {
    o.offset[0] = a.offset[0];
    o.offset[1] = a.offset[1];
    o.offset[3] = a.offset[2];
    o.offset[4] = a.offset[3];
  }
}

struct Shared {
  int8_t q[15][32];  // coded offsets of (component, type) k = comp * 5 + type
  int aux[15];
  int64_t dist[15];
};

enum { PIC_INIT = 0, CUR = 1, NEXT = 2, MID = 3, TEMP = 4, GO = 5 };

// deriveModeNewRDO (:566), lane 0
__device__ void mode_new(const Env &e, const Shared &sh, bool left, bool above, Coder *coders, Blk &mode, double &norm_cost) {
  int64_t dist[3] = {0, 0, 0}, mdist[3] = {0, 0, 0};
  Off test[3];
  for (int k = 0; k < 3; k++) { test[k].mode = 0; test[k].type = 0; test[k].aux = 0; }
  double min_cost, cost;
  mode.c[0].mode = 0;
  Coder go = coders[CUR];
  code_blk(e, go, mode, left, above, true);
  coders[MID] = go;
  {
    mode.c[0].mode = 0;
    reset_bits(go);
    code_offset(e, go, 0, mode.c[0]);
    mdist[0] = 0;
    min_cost = e.lambda[0] * ((double)written(go));
    coders[TEMP] = go;
    if (e.en[0]) {
      for (int t = 0; t < 5; t++) {
        test[0].mode = 1;
        test[0].type = t;
        test[0].aux = sh.aux[t];
        for (int i = 0; i < 32; i++) test[0].offset[i] = sh.q[t][i];
        dist[0] = sh.dist[t];
        go = coders[MID];
        reset_bits(go);
        code_offset(e, go, 0, test[0]);
        const int rate = (int)written(go);
        cost = (double)dist[0] + e.lambda[0] * ((double)rate);
        if (cost < min_cost) {
          min_cost = cost;
          mdist[0] = dist[0];
          mode.c[0] = test[0];
          coders[TEMP] = go;
        }
      }
    }
    go = coders[TEMP];
    coders[MID] = go;
  }
  cost = 0;
  uint32_t prev = 0;
  reset_bits(go);
  for (int k = 1; k < 3; k++) {
    mode.c[k].mode = 0;
    mdist[k] = 0;
    code_offset(e, go, k, mode.c[k]);
    const uint32_t now = written(go);
    cost += e.lambda[k] * (now - prev);
    prev = now;
  }
  min_cost = cost;
  for (int t = 0; t < 5; t++) {
    go = coders[MID];
    reset_bits(go);
    prev = 0;
    cost = 0;
    for (int k = 1; k < 3; k++) {
      if (!e.en[k]) {
        test[k].mode = 0;
        dist[k] = 0;
        continue;
      }
      const int ix = k * 5 + t;
      test[k].mode = 1;
      test[k].type = t;
      test[k].aux = sh.aux[ix];
      for (int i = 0; i < 32; i++) test[k].offset[i] = sh.q[ix][i];
      dist[k] = sh.dist[ix];
      code_offset(e, go, k, test[k]);
      const uint32_t now = written(go);
      cost += dist[k] + (e.lambda[k] * (now - prev));
      prev = now;
    }
    if (cost < min_cost) {
      min_cost = cost;
      for (int k = 1; k < 3; k++) {
        mdist[k] = dist[k];
        mode.c[k] = test[k];
      }
    }
  }
  norm_cost = 0;
  for (int k = 0; k < 3; k++) norm_cost += (double)mdist[k] / e.lambda[k];
  go = coders[CUR];
  reset_bits(go);
  code_blk(e, go, mode, left, above, false);
  norm_cost += (double)written(go);
  coders[GO] = go;
}

// deriveModeMergeRDO (:709), lane 0; cand[mt] = the reconstructed candidate (valid if has[mt])
__device__ void mode_merge(const Env &e, const hvx_sao_stat *st, const Blk *cand, const bool *has, Coder *coders, Blk &mode,
                           double &norm_cost) {
  norm_cost = 1.7e308;
  for (int mt = 0; mt < 2; mt++) {
    if (!has[mt]) continue;
    Blk test = cand[mt];
    double nd = 0;
    for (int k = 0; k < 3; k++) {
      test.c[k].mode = 2;
      test.c[k].type = mt;
      const Off &m = cand[mt].c[k];
      if (m.mode != 0) nd += (((double)distortion(m, st[k * 5 + m.type])) / e.lambda[k]);
    }
    Coder go = coders[CUR];
    reset_bits(go);
    code_blk(e, go, test, has[0], has[1], false);
    const int rate = (int)written(go);
    const double cost = nd + (double)rate;
    if (cost < norm_cost) {
      norm_cost = cost;
      mode = test;
      coders[TEMP] = go;
    }
  }
  coders[GO] = coders[TEMP];
}

__device__ void to_applied(const Off &q, hvx_sao_offset &d) {
  d.type = (int8_t)(q.mode == 0 ? -1 : q.type);
  d.band = 0;
  d.offset[0] = d.offset[1] = d.offset[2] = d.offset[3] = 0;
  d.pad_[0] = d.pad_[1] = 0;
  if (q.mode != 0) {
    if (q.type == 4) {
      d.band = (uint8_t)q.aux;
      for (int i = 0; i < 4; i++) d.offset[i] = q.offset[(q.aux + i) % 32];
    } else {
      d.offset[0] = q.offset[0];
      d.offset[1] = q.offset[1];
      d.offset[2] = q.offset[3];
      d.offset[3] = q.offset[4];
    }
  }
}

}  // namespace saod

// one wave per picture
static __global__ __launch_bounds__(64) void k_sao_decide(const hvx_sao_decide_job *__restrict__ jobs, int n_jobs) {
  using namespace saod;
  __shared__ Shared sh;
  const int j = blockIdx.x, l = threadIdx.x;
  if (j >= n_jobs) return;
  const hvx_sao_decide_job J = jobs[j];
  if (J.pic_w <= 0 || J.pic_h <= 0 || J.pic_w > 16384 || J.pic_h > 16384 || !J.stats || !J.entropy_bits || !J.coded ||
      !J.recon || !J.slice_enabled_out || !J.total_cost)
    return;  // a malformed job is skipped whole
  const int wc = (J.pic_w + 63) / 64, hc = (J.pic_h + 63) / 64, n = wc * hc;
  int en[3] = {J.slice_enabled[0] != 0, J.slice_enabled[1] != 0, J.slice_enabled[2] != 0};
  const Env e{J.entropy_bits, J.lambda, en};
  const bool all_off = !en[0] && !en[1] && !en[2];
  Coder coders[6];
  coders[PIC_INIT].st[0] = J.sao_states[0];
  coders[PIC_INIT].st[1] = J.sao_states[1];
  coders[PIC_INIT].frac = (uint64_t)(uint32_t)J.frac_lo;
  coders[GO] = coders[PIC_INIT];
  double total = 0;
  for (int a = 0; a < n; a++) {
    const hvx_sao_stat *st = J.stats + (size_t)a * 15;
    if (all_off) {
      if (l < 3) {
        for (int i = 0; i < 8; i++) J.coded[((size_t)a * 3 + l) * 8 + i] = 0;
        Off z;
        z.mode = 0; z.type = 0; z.aux = 0;
        for (int i = 0; i < 32; i++) z.offset[i] = 0;
        to_applied(z, J.recon[a].comp[l]);
      }
      continue;
    }
    // the 15 offset derivations, one per lane
    if (l < 15) {
      const int comp = l / 5, t = l % 5;
      if (en[comp]) {
        int aux = 0;
        sh.dist[l] = derive(J.lambda[comp], t, st[l], sh.q[l], aux);
        sh.aux[l] = aux;
      }
    }
    __syncthreads();
    if (l == 0) {
      coders[CUR] = coders[GO];
      const int x = a % wc, y = a / wc, s0 = J.slice_ctus > 0 ? a - a % J.slice_ctus : 0;
      bool has[2] = {x > 0 && a - 1 >= s0, y > 0 && a - wc >= s0};  // getMergeList: left, above (same slice)
      Blk cand[2];
      for (int mt = 0; mt < 2; mt++)
        if (has[mt])
          for (int k = 0; k < 3; k++) from_applied(J.recon[mt == 0 ? a - 1 : a - wc].comp[k], cand[mt].c[k]);
      double min_cost = 1.7e308, cost;
      Blk mode, best;
      for (int k = 0; k < 3; k++) { mode.c[k].mode = 0; mode.c[k].type = 0; mode.c[k].aux = 0; best.c[k] = mode.c[k]; }
      for (int m = 1; m < 3; m++) {
        if (m == 1) mode_new(e, sh, has[0], has[1], coders, mode, cost);
        else mode_merge(e, st, cand, has, coders, mode, cost);
        if (cost < min_cost) {
          min_cost = cost;
          best = mode;
          coders[NEXT] = coders[GO];
        }
      }
      total += min_cost;
      coders[GO] = coders[NEXT];
      for (int k = 0; k < 3; k++) {
        const Off &o = best.c[k];
        int32_t *r = J.coded + ((size_t)a * 3 + k) * 8;
        for (int i = 0; i < 8; i++) r[i] = 0;
        r[0] = o.mode;
        if (o.mode != 0) {
          r[1] = o.type;
          if (o.mode == 1) {
            r[2] = o.aux;
            if (o.type == 4)
              for (int i = 0; i < 4; i++) r[3 + i] = o.offset[(o.aux + i) % 32];
            else
              for (int i = 0; i < 5; i++) r[3 + i] = o.offset[i];
          }
        }
        // reconstructBlkSAOParam: a merge takes the candidate's reconstructed parameters
        to_applied(o.mode == 2 ? cand[o.type].c[k] : o, J.recon[a].comp[k]);
      }
    }
    __syncthreads();
  }
  if (l == 0) {
    int eo[3] = {en[0], en[1], en[2]};
    if (!all_off && total >= 0 && J.test_off) {  // the coded parameters only (offsetCTU has run, :840-859)
      for (size_t i = 0; i < (size_t)n * 24; i++) J.coded[i] = 0;
      eo[0] = eo[1] = eo[2] = 0;
    }
    for (int k = 0; k < 3; k++) J.slice_enabled_out[k] = eo[k];
    *J.total_cost = total;
  }
}

}  // namespace hvxi
