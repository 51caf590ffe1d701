// hvx_tu.hpp -- transform-unit kernels (gfx950): forward DCT/DST + quant/RDOQ, dequant +
// inverse, and the fused TU pipeline (forward -> inverse -> SSE).
//
// Reference: TComTrQuant.cpp (transformNxN :1460, xT :1952, xTrMxN :860, xQuant :1126,
// signBitHidingHDQ :991, xRateDistOptQuant :2129-2671 and its context helpers :2682-3052,
// xDeQuant :1314, invTransformNxN :1547, xIT :1988, xTransformSkip :2021/:2070) and
// TComRdCost::getDistPart SSE (TComRdCost.cpp:429).
//
// Mapping: one 64-lane wave (one workgroup) per TU, templated on the TU size so the LDS
// image is sized exactly (4x4: ~1 KB ... 32x32: ~62 KB).  The integer transforms are
// LDS-tiled matrix products (partial butterflies compute the same exact integer sums; no
// MFMA -- small integer transforms).  The two stages are laid out so that every LDS access
// in the inner loops is either lane-consecutive or wave-uniform (broadcast): no bank
// conflicts.  Quantisation / RDOQ per-coefficient work (scaled levels, uncoded costs,
// candidate distortions) runs across the 64 lanes; the inherently serial RDOQ state
// machine (c1/c2/Rice/context-set carry in reverse scan order, CG zero-out, last-position
// search, RD sign hiding) runs on lane 0 over the LDS image in the reference's exact
// operation order, in double precision (the build uses -ffp-contract=off), so the
// decisions are bit-identical.
#pragma once
#include "hvx_dev.hpp"

template <int L>
struct TuSmem {
  static constexpr int N = 4 << L, NN = N * N, NCG = NN / 16;
  int32_t mt[NN];     // transform matrix, transposed: mt[x*N + k] = M[k][x]
  int32_t m[NN];      // transform matrix: m[k*N + x]
  int32_t a[NN];      // residual (int) / intermediate
  int32_t coef[NN];   // transform output (raster)
  int32_t lev[NN];    // levels (raster)
  int32_t ld[NN];     // RDOQ lLevelDouble per scan position
  int32_t rup[NN], rdown[NN], sigd[NN], du[NN];  // raster (SBH inputs)
  double cc[NN], cs[NN], cc0[NN];                 // per scan position
  double cgsig[NCG];
  uint32_t sigcg[NCG];
  int16_t res[NN];    // input residual (kept for the pipeline SSE)
  int32_t scal[4];
};

struct TuCoding {
  const uint16_t *scan;    // grouped scan -> raster
  const uint8_t *scan_cg;  // CG scan -> CG raster
  int wg, first_sig, scan_type;
};

__device__ __forceinline__ int tu_transform_shift(const hvx_tu_desc &d) {
  int s = d.max_log2_tr_range - d.bit_depth - d.log2_size;
  if (d.transform_skip && d.extended_precision && s < 0) s = 0;
  return s;
}

// getTUEntropyCodingParameters (TComChromaFormat.cpp:96) for square TUs
template <int L>
__device__ __forceinline__ TuCoding tu_coding(const hvx_tu_desc &d) {
  constexpr int N = 4 << L;
  TuCoding c;
  const int ch = d.comp ? 1 : 0;
  c.scan = kScan[d.scan_type] + scan_base(L);
  c.scan_cg = kScanCG[d.scan_type] + cg_base(L);
  c.wg = N >> 2;
  c.scan_type = d.scan_type;
  const int start4 = 0, start8 = 9, startN = ch ? 12 : 21, single = ch ? 15 : 27;
  if (d.ts_context && (d.transquant_bypass || d.transform_skip)) c.first_sig = single;
  else if (N == 4) c.first_sig = start4;
  else if (N == 8) c.first_sig = start8 + ((d.scan_type != 0 && !ch) ? 6 : 0);
  else c.first_sig = startN;
  return c;
}

// ----------------------------------------------------------------------------------- transforms
template <int L>
__device__ void tu_load_matrix(TuSmem<L> &s, bool dst) {
  constexpr int N = 4 << L, NN = N * N;
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int k = i / N, x = i % N;
    const int v = dst ? kDst4[i] : kMat[mat_base(L) + i];
    s.m[i] = v;
    s.mt[x * N + k] = v;
  }
}

// xTrMxN (:860): in s.a (int residual), out s.coef
template <int L>
__device__ void tu_forward_transform(TuSmem<L> &s) {
  constexpr int N = 4 << L, NN = N * N, LOG2 = L + 2;
  const int s1 = LOG2 - 1, s2 = LOG2 + 6;
  const int a1 = s1 > 0 ? 1 << (s1 - 1) : 0, a2 = 1 << (s2 - 1);
  int32_t *tmpT = s.lev;  // scratch: tmpT[y*N + u]
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int x = 0; x < N; x++) acc += s.mt[x * N + u] * s.a[y * N + x];
    tmpT[y * N + u] = (acc + a1) >> s1;
  }
  __syncthreads();
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int v = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int y = 0; y < N; y++) acc += s.m[v * N + y] * tmpT[y * N + u];
    s.coef[v * N + u] = (acc + a2) >> s2;
  }
  __syncthreads();
}

// xITrMxN (:927): in `in` (dequantised, raster), out int16 residual (stride N) in s.res? no: `out`
template <int L>
__device__ void tu_inverse_transform(TuSmem<L> &s, const int32_t *in, int32_t *out) {
  constexpr int N = 4 << L, NN = N * N;
  int32_t *tmp = s.rup;  // scratch: tmp[y*N + u]
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int v = 0; v < N; v++) acc += s.m[v * N + y] * in[v * N + u];
    tmp[y * N + u] = clip3(-32768, 32767, (acc + 64) >> 7);
  }
  __syncthreads();
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, x = i % N;
    int acc = 0;
#pragma unroll 8
    for (int u = 0; u < N; u++) acc += s.m[u * N + x] * tmp[y * N + u];
    out[y * N + x] = clip3(-32768, 32767, (acc + 2048) >> 12);
  }
  __syncthreads();
}

// ----------------------------------------------------------------------------------- RDOQ helpers
struct RdState {
  const hvx_estbits *est;
  double lambda;
};

__device__ __forceinline__ double rd_icost(const RdState &r, double rate) { return r.lambda * rate; }

// xGetICRate (:2891)
__device__ int rd_ic_rate(const RdState &r, uint32_t level, int ctx_one, int ctx_abs, int rice, uint32_t c1_idx,
                          uint32_t c2_idx, int limited, int max_log2) {
  int rate = 32768;
  const uint32_t base = (c1_idx < 8) ? (2 + (c2_idx < 1)) : 1;
  if (level >= base) {
    uint32_t symbol = level - base;
    if (symbol < (3u << rice)) {
      rate += (int)(((symbol >> rice) + 1 + rice) << 15);
    } else if (limited) {
      const uint32_t maxp = 32 - (3 + max_log2);
      uint32_t prefix = 0, suffix = (symbol >> rice) - 3;
      while (prefix < maxp && suffix > ((2u << prefix) - 2)) prefix++;
      const uint32_t sl = prefix == maxp ? (uint32_t)(max_log2 - rice) : prefix + 1;
      rate += (int)((3 + prefix + sl + rice) << 15);
    } else {
      uint32_t len = rice;
      symbol -= (3u << rice);
      while (symbol >= (1u << len)) { symbol -= (1u << (len++)); }
      rate += (int)((3 + len + 1 - rice + len) << 15);
    }
    if (c1_idx < 8) {
      rate += r.est->greaterOneBits[ctx_one][1];
      if (c2_idx < 1) rate += r.est->levelAbsBits[ctx_abs][1];
    }
  } else if (level == 1) {
    rate += r.est->greaterOneBits[ctx_one][0];
  } else if (level == 2) {
    rate += r.est->greaterOneBits[ctx_one][1];
    rate += r.est->levelAbsBits[ctx_abs][0];
  } else {
    rate = 0;
  }
  return rate;
}

// getSigCtxInc (:2717) for square TUs (log2 width = log2 height = LOG2)
template <int L>
__device__ __forceinline__ int rd_sig_ctx(int pattern, const TuCoding &c, int sp, int ch) {
  constexpr int LOG2 = L + 2;
  const int single = ch ? 15 : 27;
  if (c.first_sig == single) return single;
  const int raster = c.scan[sp];
  const int py = raster >> LOG2, px = raster - (py << LOG2);
  if (px + py == 0) return 0;
  int offset;
  if (L == 0) {
    offset = kCtxIndMap4x4[4 * py + px];
  } else {
    int cnt;
    if (pattern == 0) { const int t = (px & 3) + (py & 3); cnt = t >= 3 ? 0 : t >= 1 ? 1 : 2; }
    else if (pattern == 1) { const int y = py & 3; cnt = y >= 2 ? 0 : y >= 1 ? 1 : 2; }
    else if (pattern == 2) { const int x = px & 3; cnt = x >= 2 ? 0 : x >= 1 ? 1 : 2; }
    else cnt = 2;
    const int nf = ((px >> 2) + (py >> 2)) > 0;
    offset = (nf ? (ch ? 0 : 3) : 0) + cnt;
  }
  return c.first_sig + offset;
}

__device__ __forceinline__ double rd_rate_last(const RdState &r, int px, int py, int ch) {
  const int cx = kGroupIdx[px], cy = kGroupIdx[py];
  double c = (double)(r.est->lastXBits[ch][cx] + r.est->lastYBits[ch][cy]);
  if (cx > 3) c += 32768.0 * ((cx - 2) >> 1);
  if (cy > 3) c += 32768.0 * ((cy - 2) >> 1);
  return rd_icost(r, c);
}

// xRateDistOptQuant (:2129-2671).  Input s.coef (raster); output s.lev (signed levels), returns uiAbsSum.
template <int L>
__device__ int32_t tu_rdoq(TuSmem<L> &s, const hvx_tu_desc &d, const hvx_estbits *est, int32_t *arl_out) {
  constexpr int N = 4 << L, NN = N * N, NCG = NN / 16, LOG2 = L + 2;
  const int ch = d.comp ? 1 : 0, comp = d.comp;
  const int ts = tu_transform_shift(d);
  const int qbits = 14 + d.qp_per + ts;
  const int qc = kQuantScales[d.qp_rem];
  const int ext = d.extended_precision, max_log2 = d.max_log2_tr_range;
  const int32_t ecmax = (1 << max_log2) - 1, ecmin = -(1 << max_log2);
  // setErrScaleCoeff (:3106) for the flat list
  const int tsn = d.max_log2_tr_range - d.bit_depth - d.log2_size;
  double escale = (double)(1 << 15);
  escale = escale * ldexp(1.0, -2 * tsn);  // == pow(2.0, -2.0*tsn) exactly
  escale = escale / qc / qc / (1 << 0);
  const TuCoding c = tu_coding<L>(d);
  const int64_t lim = (int64_t)2147483647 - ((int64_t)1 << (qbits - 1));
  const int qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);

  // ---- per-coefficient work across lanes ----
  for (int sp = lane_id(); sp < NN; sp += HVX_WAVE) {
    const int blk = c.scan[sp];
    const int64_t t = (int64_t)abs(s.coef[blk]) * qc;
    const int32_t ld = (int32_t)(t < lim ? t : lim);
    s.ld[sp] = ld;
    const double e = (double)ld;
    s.cc0[sp] = e * e * escale;
    s.cc[sp] = 0.0;
    s.cs[sp] = 0.0;
    s.rup[blk] = 0; s.rdown[blk] = 0; s.sigd[blk] = 0; s.du[blk] = 0;
    if (arl_out) arl_out[blk] = d.adaptive_qp_select ? (ld + add_c) >> qbits_c : 0;
  }
  for (int g = lane_id(); g < NCG; g += HVX_WAVE) { s.cgsig[g] = 0.0; s.sigcg[g] = 0; }
  __syncthreads();

  if (lane_id() == 0) {
    const RdState r = {est, d.lambda};
    const uint32_t rice0 = (uint32_t)d.golomb_rice_stat / 4;
    uint32_t rice = rice0, ctx_set = 0, c1_idx = 0, c2_idx = 0;
    int c1 = 1, c2 = 0, last = -1, cg_last = -1;
    double block_uncoded = 0, base_cost = 0;
    const int sig_off = ch ? 28 : 0;
    for (int cgp = NCG - 1; cgp >= 0; cgp--) {
      const int cgblk = c.scan_cg[cgp];
      const int cy = cgblk / c.wg, cx = cgblk - cy * c.wg;
      int nnz0 = 0;
      double coded_ld = 0, uncoded = 0, sig_cost = 0, sig_cost0 = 0;
      int pattern = 0;
      if (NCG > 1) {
        const int rr = cx < c.wg - 1 ? (s.sigcg[cy * c.wg + cx + 1] != 0) : 0;
        const int bb = cy < c.wg - 1 ? (s.sigcg[(cy + 1) * c.wg + cx] != 0) : 0;
        pattern = rr + (bb << 1);
      }
      for (int pin = 15; pin >= 0; pin--) {
        const int sp = cgp * 16 + pin;
        const int blk = c.scan[sp];
        const int32_t ld = s.ld[sp];
        const uint32_t q = (uint32_t)((ld + (1 << (qbits - 1))) >> qbits);
        const uint32_t max_abs = (uint32_t)ecmax < q ? (uint32_t)ecmax : q;
        block_uncoded += s.cc0[sp];
        int32_t out = (int32_t)max_abs;
        if (max_abs > 0 && last < 0) {
          last = sp;
          ctx_set = (comp ? 4 : 0) + ((comp == 0 && (sp >> 4) > 0) ? 2 : 0);
          cg_last = cgp;
        }
        if (last >= 0) {
          const int ctx_one = 4 * (int)ctx_set + c1, ctx_abs = (int)ctx_set + c2;
          // xGetCodedLevel (:2822)
          const bool is_last = sp == last;
          int ctx_sig = sig_off;
          if (!is_last) ctx_sig = sig_off + rd_sig_ctx<L>(pattern, c, sp, ch);
          double cur_sig = 0, cost, cost_sig = 0;
          uint32_t best = 0;
          bool done = false;
          if (!is_last && max_abs < 3) {
            cost_sig = rd_icost(r, (double)est->significantBits[ctx_sig][0]);
            cost = s.cc0[sp] + cost_sig;
            if (max_abs == 0) done = true;
          } else {
            cost = 1.7e+308;
          }
          if (!done) {
            if (!is_last) cur_sig = rd_icost(r, (double)est->significantBits[ctx_sig][1]);
            const uint32_t min_abs = max_abs > 1 ? max_abs - 1 : 1;
            for (int lv = (int)max_abs; lv >= (int)min_abs; lv--) {
              const double err = (double)sub32(ld, shl32(lv, qbits));
              double cc = err * err * escale +
                          rd_icost(r, (double)rd_ic_rate(r, (uint32_t)lv, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2));
              cc += cur_sig;
              if (cc < cost) { best = (uint32_t)lv; cost = cc; cost_sig = cur_sig; }
            }
          }
          s.cc[sp] = cost;
          s.cs[sp] = cost_sig;
          const uint32_t level = best;
          if (!is_last) s.sigd[blk] = est->significantBits[ctx_sig][1] - est->significantBits[ctx_sig][0];
          s.du[blk] = sub32(ld, shl32((int32_t)level, qbits)) >> (qbits - 8);
          if (level > 0) {
            const int now = rd_ic_rate(r, level, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2);
            s.rup[blk] = rd_ic_rate(r, level + 1, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2) - now;
            s.rdown[blk] = rd_ic_rate(r, level - 1, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2) - now;
          } else {
            s.rup[blk] = est->greaterOneBits[ctx_one][0];
          }
          out = (int32_t)level;
          base_cost += s.cc[sp];
          const uint32_t base = (c1_idx < 8) ? (2 + (c2_idx < 1)) : 1;
          if (level >= base && level > 3u * (1u << rice)) rice = d.persistent_rice ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
          if (level >= 1) c1_idx++;
          if (level > 1) { c1 = 0; c2 += (c2 < 2); c2_idx++; }
          else if (c1 < 3 && c1 > 0 && level) c1++;
          if ((sp % 16 == 0) && sp > 0) {
            ctx_set = (comp ? 4 : 0) + ((comp == 0 && ((sp - 1) >> 4) > 0) ? 2 : 0) + (c1 == 0 ? 1 : 0);
            c1 = 1; c2 = 0; c1_idx = 0; c2_idx = 0;
            rice = rice0;
          }
        } else {
          base_cost += s.cc0[sp];
        }
        s.lev[blk] = out;
        sig_cost += s.cs[sp];
        if (pin == 0) sig_cost0 = s.cs[sp];
        if (out) {
          s.sigcg[cgblk] = 1;
          coded_ld += s.cc[sp] - s.cs[sp];
          uncoded += s.cc0[sp];
          if (pin != 0) nnz0++;
        }
      }
      if (cg_last >= 0) {
        if (cgp) {
          const int rr = cx < c.wg - 1 ? (s.sigcg[cy * c.wg + cx + 1] != 0) : 0;
          const int bb = cy < c.wg - 1 ? (s.sigcg[(cy + 1) * c.wg + cx] != 0) : 0;
          const int ctx = (rr + bb) != 0;
          if (s.sigcg[cgblk] == 0) {
            base_cost += rd_icost(r, (double)est->significantCoeffGroupBits[ctx][0]) - sig_cost;
            s.cgsig[cgp] = rd_icost(r, (double)est->significantCoeffGroupBits[ctx][0]);
          } else if (cgp < cg_last) {
            if (nnz0 == 0) { base_cost -= sig_cost0; sig_cost -= sig_cost0; }
            double zero_cost = base_cost;
            base_cost += rd_icost(r, (double)est->significantCoeffGroupBits[ctx][1]);
            zero_cost += rd_icost(r, (double)est->significantCoeffGroupBits[ctx][0]);
            s.cgsig[cgp] = rd_icost(r, (double)est->significantCoeffGroupBits[ctx][1]);
            zero_cost += uncoded;
            zero_cost -= coded_ld;
            zero_cost -= sig_cost;
            if (zero_cost < base_cost) {
              s.sigcg[cgblk] = 0;
              base_cost = zero_cost;
              s.cgsig[cgp] = rd_icost(r, (double)est->significantCoeffGroupBits[ctx][0]);
              for (int pin = 15; pin >= 0; pin--) {
                const int sp = cgp * 16 + pin;
                const int blk = c.scan[sp];
                if (s.lev[blk]) { s.lev[blk] = 0; s.cc[sp] = s.cc0[sp]; s.cs[sp] = 0; }
              }
            }
          }
        } else {
          s.sigcg[cgblk] = 1;
        }
      }
    }

    int32_t abs_sum = 0;
    if (last >= 0) {
      double best_cost;
      int best_p1 = 0;
      if (!d.is_intra && ch == 0 && d.tr_idx == 0) {
        best_cost = block_uncoded + rd_icost(r, (double)est->blockRootCbpBits[0][0]);
        base_cost += rd_icost(r, (double)est->blockRootCbpBits[0][1]);
      } else {
        const int ctx = d.ctx_qt_cbf + (ch ? 5 : 0);
        best_cost = block_uncoded + rd_icost(r, (double)est->blockCbpBits[ctx][0]);
        base_cost += rd_icost(r, (double)est->blockCbpBits[ctx][1]);
      }
      bool found = false;
      for (int cgp = cg_last; cgp >= 0 && !found; cgp--) {
        const int cgblk = c.scan_cg[cgp];
        base_cost -= s.cgsig[cgp];
        if (s.sigcg[cgblk]) {
          for (int pin = 15; pin >= 0; pin--) {
            const int sp = cgp * 16 + pin;
            if (sp > last) continue;
            const int blk = c.scan[sp];
            if (s.lev[blk]) {
              const int py = blk >> LOG2, px = blk - (py << LOG2);
              const double cl = c.scan_type == 2 ? rd_rate_last(r, py, px, ch) : rd_rate_last(r, px, py, ch);
              const double total = base_cost + cl - s.cs[sp];
              if (total < best_cost) { best_p1 = sp + 1; best_cost = total; }
              if (s.lev[blk] > 1) { found = true; break; }
              base_cost -= s.cc[sp];
              base_cost += s.cc0[sp];
            } else {
              base_cost -= s.cs[sp];
            }
          }
        }
      }
      for (int sp = 0; sp < best_p1; sp++) {
        const int blk = c.scan[sp];
        const int32_t lv = s.lev[blk];
        abs_sum += lv;
        s.lev[blk] = s.coef[blk] < 0 ? -lv : lv;
      }
      for (int sp = best_p1; sp <= last; sp++) s.lev[c.scan[sp]] = 0;

      if (d.sign_hiding && abs_sum >= 2) {
        const double iq = (double)kInvQuantScales[d.qp_rem];
        const int64_t rdf = (int64_t)(iq * iq * (1 << (2 * d.qp_per)) / d.lambda / 16 / (1 << 0) + 0.5);
        int last_cg = -1;
        for (int sub = (NN - 1) >> 4; sub >= 0; sub--) {
          const int pos = sub << 4;
          int first_nz = 16, last_nz = -1, abs_in = 0, k;
          for (k = 15; k >= 0; k--) if (s.lev[c.scan[k + pos]]) { last_nz = k; break; }
          for (k = 0; k < 16; k++) if (s.lev[c.scan[k + pos]]) { first_nz = k; break; }
          for (k = first_nz; k <= last_nz; k++) abs_in += s.lev[c.scan[k + pos]];
          if (last_nz >= 0 && last_cg == -1) last_cg = 1;
          if (last_nz - first_nz >= 4) {
            const uint32_t signbit = s.lev[c.scan[pos + first_nz]] > 0 ? 0 : 1;
            if (signbit != (uint32_t)(abs_in & 1)) {
              int64_t min_inc = INT64_MAX, cur = INT64_MAX;
              int min_pos = -1, fch = 0, cch = 0;
              for (k = (last_cg == 1 ? last_nz : 15); k >= 0; k--) {
                const int blk = c.scan[k + pos];
                const int32_t lv = s.lev[blk];
                if (lv != 0) {
                  const int64_t up = rdf * (-s.du[blk]) + s.rup[blk];
                  int64_t down = rdf * (s.du[blk]) + s.rdown[blk] - ((abs(lv) == 1) ? s.sigd[blk] : 0);
                  if (last_cg == 1 && last_nz == k && abs(lv) == 1) down -= (4 << 15);
                  if (up < down) { cur = up; cch = 1; }
                  else { cch = -1; cur = (k == first_nz && abs(lv) == 1) ? INT64_MAX : down; }
                } else {
                  cur = rdf * (-(abs(s.du[blk]))) + (1 << 15) + s.rup[blk] + s.sigd[blk];
                  cch = 1;
                  if (k < first_nz) {
                    const uint32_t tsb = s.coef[blk] >= 0 ? 0 : 1;
                    if (tsb != signbit) cur = INT64_MAX;
                  }
                }
                if (cur < min_inc) { min_inc = cur; fch = cch; min_pos = blk; }
              }
              if (s.lev[min_pos] == ecmax || s.lev[min_pos] == ecmin) fch = -1;
              if (s.coef[min_pos] >= 0) s.lev[min_pos] += fch;
              else s.lev[min_pos] -= fch;
            }
          }
          if (last_cg == 1) last_cg = 0;
        }
      }
    }
    s.scal[0] = abs_sum;
  }
  __syncthreads();
  return s.scal[0];
}

// xQuant (:1126) non-RDOQ path + signBitHidingHDQ (:991).  Input s.coef, output s.lev.
template <int L>
__device__ int32_t tu_quant_plain(TuSmem<L> &s, const hvx_tu_desc &d, int32_t *arl_out) {
  constexpr int NN = (4 << L) * (4 << L);
  const int ts = tu_transform_shift(d);
  const int qbits = 14 + d.qp_per + ts;
  const int qc = kQuantScales[d.qp_rem];
  const int add = (d.slice_type == 2 ? 171 : 85) << (qbits - 9);
  const int qbits8 = qbits - 8, qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
  const int32_t ecmax = (1 << d.max_log2_tr_range) - 1, ecmin = -(1 << d.max_log2_tr_range);
  int part = 0;
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int32_t lv = s.coef[i];
    const int sign = lv < 0 ? -1 : 1;
    const int64_t t = (int64_t)abs(lv) * qc;
    if (arl_out) arl_out[i] = d.adaptive_qp_select ? (int32_t)((t + add_c) >> qbits_c) : 0;
    const int32_t qm = (int32_t)((t + add) >> qbits);
    s.du[i] = (int32_t)((t - (int64_t)shl32(qm, qbits)) >> qbits8);
    part += qm;
    s.lev[i] = clip3(ecmin, ecmax, qm * sign);
  }
  const int32_t abs_sum = wave_sum_i32(part);
  __syncthreads();
  if (d.sign_hiding && abs_sum >= 2 && lane_id() == 0) {
    const TuCoding c = tu_coding<L>(d);
    int last_cg = -1;
    for (int sub = (NN - 1) >> 4; sub >= 0; sub--) {
      const int pos = sub << 4;
      int first_nz = 16, last_nz = -1, abs_in = 0, k;
      for (k = 15; k >= 0; k--) if (s.lev[c.scan[k + pos]]) { last_nz = k; break; }
      for (k = 0; k < 16; k++) if (s.lev[c.scan[k + pos]]) { first_nz = k; break; }
      for (k = first_nz; k <= last_nz; k++) abs_in += s.lev[c.scan[k + pos]];
      if (last_nz >= 0 && last_cg == -1) last_cg = 1;
      if (last_nz - first_nz >= 4) {
        const uint32_t signbit = s.lev[c.scan[pos + first_nz]] > 0 ? 0 : 1;
        if (signbit != (uint32_t)(abs_in & 1)) {
          int32_t cur = INT32_MAX, min_inc = INT32_MAX;
          int min_pos = -1, fch = 0, cch = 0;
          for (k = (last_cg == 1 ? last_nz : 15); k >= 0; k--) {
            const int blk = c.scan[k + pos];
            const int32_t q = s.lev[blk];
            if (q != 0) {
              if (s.du[blk] > 0) { cur = -s.du[blk]; cch = 1; }
              else if (k == first_nz && abs(q) == 1) cur = INT32_MAX;
              else { cur = s.du[blk]; cch = -1; }
            } else if (k < first_nz) {
              const uint32_t tsb = s.coef[blk] >= 0 ? 0 : 1;
              if (tsb != signbit) cur = INT32_MAX;
              else { cur = -s.du[blk]; cch = 1; }
            } else {
              cur = -s.du[blk]; cch = 1;
            }
            if (cur < min_inc) { min_inc = cur; fch = cch; min_pos = blk; }
          }
          if (s.lev[min_pos] == ecmax || s.lev[min_pos] == ecmin) fch = -1;
          if (s.coef[min_pos] >= 0) s.lev[min_pos] += fch;
          else s.lev[min_pos] -= fch;
        }
      }
      if (last_cg == 1) last_cg = 0;
    }
  }
  __syncthreads();
  return abs_sum;
}

// transformNxN (:1460) on s.res (int16, raster N*N).  Leaves s.coef (transform output) and
// s.lev (levels); returns uiAbsSum.
template <int L>
__device__ int32_t tu_forward(TuSmem<L> &s, const hvx_tu_desc &d, const hvx_estbits *est, int32_t *arl_out) {
  constexpr int N = 4 << L, NN = N * N;
  if (d.transquant_bypass) {
    int part = 0;
    for (int i = lane_id(); i < NN; i += HVX_WAVE) { s.lev[i] = s.res[i]; s.coef[i] = s.res[i]; part += abs((int)s.res[i]); }
    __syncthreads();
    return wave_sum_i32(part);
  }
  if (d.transform_skip) {
    const int ts = tu_transform_shift(d);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int32_t v = s.res[i];
      s.coef[i] = ts >= 0 ? shl32(v, ts) : (v + (1 << (-ts - 1))) >> -ts;
    }
    __syncthreads();
  } else {
    tu_load_matrix<L>(s, d.use_dst && N == 4);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) s.a[i] = s.res[i];
    __syncthreads();
    tu_forward_transform<L>(s);
  }
  const int use_rdoq = d.transform_skip ? d.use_rdoq_ts : d.use_rdoq;
  if (use_rdoq) {
    bool need = true;
    if (d.selective_rdoq) {  // xNeedRDOQ (:1257)
      const int ts = tu_transform_shift(d);
      const int qbits = 14 + d.qp_per + ts;
      const int add = (d.comp == 0 ? 171 : 256) << (qbits - 9);
      int any = 0;
      for (int i = lane_id(); i < NN; i += HVX_WAVE)
        any |= ((int32_t)(((int64_t)abs(s.coef[i]) * kQuantScales[d.qp_rem] + add) >> qbits)) != 0;
      need = wave_sum_i32(any) != 0;
    }
    if (need) return tu_rdoq<L>(s, d, est, arl_out);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      s.lev[i] = 0;
      if (arl_out) arl_out[i] = 0;
    }
    __syncthreads();
    return 0;
  }
  return tu_quant_plain<L>(s, d, arl_out);
}

// invTransformNxN (:1547) on levels `in` (raster) -> `out` (int32 raster, values fit Pel).
template <int L>
__device__ void tu_inverse(TuSmem<L> &s, const hvx_tu_desc &d, const int32_t *in, int32_t *out) {
  constexpr int N = 4 << L, NN = N * N;
  if (d.transquant_bypass) {
    for (int i = lane_id(); i < NN; i += HVX_WAVE) out[i] = (int16_t)in[i];
    __syncthreads();
    return;
  }
  const int ts = tu_transform_shift(d);
  const int max_log2 = d.max_log2_tr_range;
  const int32_t tmin = -(1 << max_log2), tmax = (1 << max_log2) - 1;
  const int right = 6 - (ts + d.qp_per);
  const int scale = kInvQuantScales[d.qp_rem];
  int tib = 32 + right - 7;
  if (max_log2 + 1 < tib) tib = max_log2 + 1;
  const int32_t imin = -(1 << (tib - 1)), imax = (1 << (tib - 1)) - 1;
  int32_t *deq = s.a;
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int32_t c = clip3(imin, imax, in[i]);
    const int32_t v = right > 0 ? (c * scale + (1 << (right - 1))) >> right : shl32(c * scale, -right);
    deq[i] = clip3(tmin, tmax, v);
  }
  __syncthreads();
  if (d.transform_skip) {
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int32_t v = deq[i];
      out[i] = (int16_t)(ts >= 0 ? (v + (ts == 0 ? 0 : 1 << (ts - 1))) >> ts : shl32(v, -ts));
    }
    __syncthreads();
  } else {
    tu_load_matrix<L>(s, d.use_dst && N == 4);
    __syncthreads();
    tu_inverse_transform<L>(s, deq, out);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) out[i] = (int16_t)out[i];
    __syncthreads();
  }
}

__device__ __forceinline__ int tu_class(const hvx_tu_desc &d) { return d.log2_size - 2; }

// mode: 0 forward, 1 inverse, 2 pipeline
template <int L, int MODE>
__global__ __launch_bounds__(64) void k_tu(const hvx_tu_desc *__restrict__ descs, const hvx_estbits *__restrict__ est,
                                           const int32_t *__restrict__ est_idx, const int64_t *__restrict__ offs,
                                           int n, const int16_t *__restrict__ res_in, int32_t *__restrict__ temp_out,
                                           int32_t *__restrict__ lev_io, int32_t *__restrict__ arl_out,
                                           int32_t *__restrict__ abs_out, int16_t *__restrict__ res_out,
                                           uint32_t *__restrict__ sse_out) {
  constexpr int N = 4 << L, NN = N * N;
  __shared__ TuSmem<L> s;
  const int t = blockIdx.x;
  if (t >= n) return;
  const hvx_tu_desc d = descs[t];
  if (d.width != N || d.height != N) return;  // another size class handles this TU
  const int64_t off = offs[t];
  if (MODE == 1) {
    for (int i = lane_id(); i < NN; i += HVX_WAVE) s.lev[i] = lev_io[off + i];
    __syncthreads();
    tu_inverse<L>(s, d, s.lev, s.coef);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) res_out[off + i] = (int16_t)s.coef[i];
    return;
  }
  const hvx_estbits *e = est + (est_idx ? est_idx[t] : t);
  for (int i = lane_id(); i < NN; i += HVX_WAVE) s.res[i] = res_in[off + i];
  __syncthreads();
  const int32_t abs_sum = tu_forward<L>(s, d, e, arl_out ? arl_out + off : nullptr);
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    lev_io[off + i] = s.lev[i];
    if (temp_out) temp_out[off + i] = s.coef[i];
  }
  if (lane_id() == 0 && abs_out) abs_out[t] = abs_sum;
  if (MODE == 2) {
    __syncthreads();
    tu_inverse<L>(s, d, s.lev, s.rdown);
    uint32_t part = 0;
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int r = (int16_t)s.rdown[i];
      res_out[off + i] = (int16_t)r;
      const int df = (int)s.res[i] - r;
      part += (uint32_t)(df * df);
    }
    const uint32_t sse = wave_sum_u32(part);
    if (lane_id() == 0 && sse_out) sse_out[t] = sse;
  }
}
