// hvx_tu.hpp -- transform-unit kernels (gfx950): forward DCT/DST + quant/RDOQ, dequant +
// inverse, and the fused TU pipeline (forward -> inverse -> SSE).
//
// Reference: TComTrQuant.cpp (transformNxN :1460, xT :1952, xTrMxN :860, xQuant :1126,
// signBitHidingHDQ :991, xRateDistOptQuant :2129-2671 and its context helpers :2682-3052,
// xDeQuant :1314, invTransformNxN :1547, xIT :1988, xTransformSkip :2021/:2070) and
// TComRdCost::getDistPart SSE (TComRdCost.cpp:429).
//
// Mapping: one 64-lane wave (one workgroup) per TU, templated on the TU size.  The LDS
// image is three int32 planes of the TU (12 KB at 32x32) so that several TUs stay resident
// per SIMD to hide the latency of RDOQ's serial part:
//   a    : residual -> (RDOQ) context state per scan position -> dequantised coefficients
//   coef : transform output -> inverse-transform scratch
//   lev  : forward-transform scratch -> levels -> reconstructed residual
// The integer transforms are matrix products over LDS (partial butterflies compute the same
// exact integer sums; small integer transforms, no MFMA) with the DCT/DST matrix read from
// the constant table; every LDS access in the inner loops is lane-consecutive or
// wave-uniform (broadcast).  RDOQ: see tu_rdoq.
#pragma once
#include "hvx_dev.hpp"

template <int L>
struct TuSmem {
  static constexpr int N = 4 << L, NN = N * N, NCG = NN / 16;
  alignas(16) int32_t a[NN];
  alignas(16) int32_t coef[NN];
  alignas(16) int32_t lev[NN];
  int32_t cgr[NCG];  // RDOQ coded-group flag rate per CG scan position
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
// M[k][x] of the TU's transform (the 4x4 DST for intra luma 4x4)
template <int L>
__device__ __forceinline__ int tu_mat(bool dst, int k, int x) {
  constexpr int N = 4 << L;
  if (L == 0 && dst) return kDst4[k * 4 + x];
  return kMat[mat_base(L) + k * N + x];
}

// xTrMxN (:860): in s.a (int residual), out s.coef; s.lev is scratch
template <int L>
__device__ void tu_forward_transform(TuSmem<L> &s, bool dst) {
  constexpr int N = 4 << L, NN = N * N, LOG2 = L + 2;
  const int s1 = LOG2 - 1, s2 = LOG2 + 6;
  const int a1 = s1 > 0 ? 1 << (s1 - 1) : 0, a2 = 1 << (s2 - 1);
  int32_t *tmpT = s.lev;  // tmpT[y*N + u]
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int x = 0; x < N; x++) acc += tu_mat<L>(dst, u, x) * s.a[y * N + x];
    tmpT[y * N + u] = (acc + a1) >> s1;
  }
  __syncthreads();
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int v = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int y = 0; y < N; y++) acc += tu_mat<L>(dst, v, y) * tmpT[y * N + u];
    s.coef[v * N + u] = (acc + a2) >> s2;
  }
  __syncthreads();
}

// ---- 16-bit transform form for the 16x16 / 32x32 TUs of 8-bit video with the 15-bit dynamic
// range (the CTU pass): every operand of both directions is int16 there -- residuals, the
// forward first stage ((sum + a1) >> s1 <= 2048 * 255 / 2^s1 in magnitude, the DCT rows' largest
// absolute sum being 64N), dequantised coefficients (clipped to [-2^15, 2^15)) and the inverse
// first stage (clipped) -- so each product pair is one v_dot2_i32_i16 on int16 pairs, and the
// lane's matrix row (lane & (N-1), the same row in both passes) stays in registers.  The sums
// are the same integers as tu_forward_transform / tu_inverse_transform.
template <int L>
__device__ __forceinline__ void tu_mat_row(const int16_t *tab, int r, uint32_t (&w)[(4 << L) / 2]) {
  constexpr int N = 4 << L;
  const uint4 *p = reinterpret_cast<const uint4 *>(tab + mat_base(L) + r * N);
#pragma unroll
  for (int q = 0; q < N / 8; q++) {
    const uint4 v = p[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}
// sum over the N/2 int16 pairs of a 16-byte aligned LDS row against the register row
template <int L>
__device__ __forceinline__ int tu_dot_row(const uint32_t (&m)[(4 << L) / 2], const int16_t *row, int acc) {
  constexpr int N = 4 << L;
  typedef short s2 __attribute__((ext_vector_type(2)));
  const uint4 *p = reinterpret_cast<const uint4 *>(row);
#pragma unroll
  for (int q = 0; q < N / 8; q++) {
    const uint4 v = p[q];
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, m[4 * q]), __builtin_bit_cast(s2, v.x), acc, false);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, m[4 * q + 1]), __builtin_bit_cast(s2, v.y), acc, false);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, m[4 * q + 2]), __builtin_bit_cast(s2, v.z), acc, false);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, m[4 * q + 3]), __builtin_bit_cast(s2, v.w), acc, false);
  }
  return acc;
}
template <int N> constexpr int tu_p16() { return N + 8; }  // int16 pitch of the transposed planes (16-byte rows)

// xTrMxN: aH = int16 residual [y][x] (pitch N) -> coefT = int32 coefficient (v, u) at u*N + v;
// tT (int16, N x tu_p16) is scratch
template <int L>
__device__ void tu_forward_dot2(const int16_t *aH, int16_t *tT, int32_t *coefT) {
  constexpr int N = 4 << L, LOG2 = L + 2, P = tu_p16<N>(), R = HVX_WAVE / N;
  static_assert(L >= 2, "16x16 / 32x32 only");
  const int s1 = LOG2 - 1, s2 = LOG2 + 6, a1 = 1 << (s1 - 1), a2 = 1 << (s2 - 1);
  const int lane = lane_id(), r = lane & (N - 1), g = lane / N;
  uint32_t m[N / 2];
  tu_mat_row<L>(kMat, r, m);
#pragma unroll 2
  for (int k = 0; k < N / R; k++) {  // out1[y][u = r] -> tT[u][y]
    const int y = g + R * k;
    tT[r * P + y] = (int16_t)(tu_dot_row<L>(m, aH + y * N, a1) >> s1);
  }
  __syncthreads();
#pragma unroll 2
  for (int k = 0; k < N / R; k++) {  // coefficient (v = r, u)
    const int u = g + R * k;
    coefT[u * N + r] = tu_dot_row<L>(m, tT + u * P, a2) >> s2;
  }
  __syncthreads();
}

// xITrMxN: deqT = int16 dequantised coefficient (v, u) at u*P + v -> out = int32 residual [y][x]
// (pitch N, values clipped to int16); tmp (int16, N x P) is scratch
template <int L>
__device__ void tu_inverse_dot2(const int16_t *deqT, int16_t *tmp, int32_t *out) {
  constexpr int N = 4 << L, P = tu_p16<N>(), R = HVX_WAVE / N;
  static_assert(L >= 2, "16x16 / 32x32 only");
  const int lane = lane_id(), r = lane & (N - 1), g = lane / N;
  uint32_t m[N / 2];
  tu_mat_row<L>(kMatT, r, m);  // M^T row r: M[.][r]
#pragma unroll 2
  for (int k = 0; k < N / R; k++) {  // tmp[y = r][u] = sum_v M[v][y] in[v][u]
    const int u = g + R * k;
    tmp[r * P + u] = (int16_t)clip3(-32768, 32767, tu_dot_row<L>(m, deqT + u * P, 64) >> 7);
  }
  __syncthreads();
#pragma unroll 2
  for (int k = 0; k < N / R; k++) {  // out[y][x = r] = sum_u M[u][x] tmp[y][u]
    const int y = g + R * k;
    out[y * N + r] = clip3(-32768, 32767, tu_dot_row<L>(m, tmp + y * P, 2048) >> 12);
  }
  __syncthreads();
}

// xITrMxN (:927): in (dequantised, raster) -> out (clipped to Pel range); tmp is scratch
template <int L>
__device__ void tu_inverse_transform(bool dst, const int32_t *in, int32_t *tmp, int32_t *out) {
  constexpr int N = 4 << L, NN = N * N;
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, u = i % N;
    int acc = 0;
#pragma unroll 8
    for (int v = 0; v < N; v++) acc += tu_mat<L>(dst, v, y) * in[v * N + u];
    tmp[y * N + u] = clip3(-32768, 32767, (acc + 64) >> 7);
  }
  __syncthreads();
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int y = i / N, x = i % N;
    int acc = 0;
#pragma unroll 8
    for (int u = 0; u < N; u++) acc += tu_mat<L>(dst, u, x) * tmp[y * N + u];
    out[y * N + x] = clip3(-32768, 32767, (acc + 2048) >> 12);
  }
  __syncthreads();
}

// ----------------------------------------------------------------------------------- RDOQ helpers
// xGetICRate (:2891) with the context's table entries already fetched:
// g0/g1 = greaterOneBits[ctx_one][0/1], a0/a1 = levelAbsBits[ctx_abs][0/1];
// c1ok = c1Idx < 8, c2ok = c2Idx < 1
__device__ __forceinline__ int rd_ic_rate(uint32_t level, int rice, bool c1ok, bool c2ok, int g0, int g1, int a0,
                                          int a1, int limited, int max_log2) {
  int rate = 32768;
  const uint32_t base = c1ok ? (c2ok ? 3u : 2u) : 1u;
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
      // the reference's loop `while (symbol >= (1 << len)) symbol -= 1 << len++` from
      // len = rice runs floor(log2((symbol >> rice) + 1)) times
      const uint32_t v = ((symbol - (3u << rice)) >> rice) + 1;
      const uint32_t len = (uint32_t)rice + (31u - (uint32_t)__clz(v));
      rate += (int)((3 + len + 1 - rice + len) << 15);
    }
    if (c1ok) {
      rate += g1;
      if (c2ok) rate += a1;
    }
  } else if (level == 1) {
    rate += g0;
  } else if (level == 2) {
    rate += g1;
    rate += a0;
  } else {
    rate = 0;
  }
  return rate;
}

// xGetICRate (:2891) without branches (the rate of one candidate level; lanes are different
// TUs, so every branch of the reference's form would be divergent).  Not for the limited-prefix
// (extended precision) escape code, which keeps rd_ic_rate.
__device__ __forceinline__ int rd_ic_rate_bf(uint32_t level, uint32_t rice, bool c1ok, bool c2ok, int g0, int g1, int a0,
                                             int a1) {
  const uint32_t base = c1ok ? (c2ok ? 3u : 2u) : 1u;
  const uint32_t symbol = level - base, r3 = 3u << rice;
  const int small = (int)(((symbol >> rice) + 1 + rice) << 15);
  const uint32_t v = ((symbol - r3) >> rice) + 1;
  const uint32_t len = rice + (31u - (uint32_t)__clz(v));
  const int big = (int)((3 + len + 1 - rice + len) << 15);
  const int esc = (symbol < r3 ? small : big) + (c1ok ? g1 + (c2ok ? a1 : 0) : 0);
  const int lo = level == 1 ? g0 : g1 + a0;  // level 2 below base (c1ok && c2ok)
  return level == 0 ? 0 : 32768 + (level >= base ? esc : lo);
}

// getSigCtxInc (:2717) for square TUs (log2 width = log2 height = LOG2)
template <int L>
__device__ __forceinline__ int rd_sig_ctx_raster(int pattern, int first_sig, int raster, int ch);
template <int L>
__device__ __forceinline__ int rd_sig_ctx(int pattern, const TuCoding &c, int sp, int ch) {
  return rd_sig_ctx_raster<L>(pattern, c.first_sig, c.scan[sp], ch);
}
// the same with the position's raster index given (a compile-time scan)
template <int L>
__device__ __forceinline__ int rd_sig_ctx_raster(int pattern, int first_sig, int raster, int ch) {
  constexpr int LOG2 = L + 2;
  const int single = ch ? 15 : 27;
  TuCoding c;
  c.first_sig = first_sig;
  if (c.first_sig == single) return single;
  const int py = raster >> LOG2, px = raster - (py << LOG2);
  if (px + py == 0) return 0;
  int offset;
  if (L == 0) {
    constexpr int8_t map4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};  // ctxIndMap4x4
    offset = map4[4 * py + px];
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

__device__ __forceinline__ double rd_rate_last(const hvx_estbits *est, double lambda, int px, int py, int ch) {
  const int cx = kGroupIdx[px], cy = kGroupIdx[py];
  double c = (double)(est->lastXBits[ch][cx] + est->lastYBits[ch][cy]);
  if (cx > 3) c += 32768.0 * ((cx - 2) >> 1);
  if (cy > 3) c += 32768.0 * ((cy - 2) >> 1);
  return lambda * c;
}

__device__ __forceinline__ int rl(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ double rld(double v, int lane) {
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// speculative rounds of the RDOQ reverse scan before the serial fallback (tu_rdoq).  Each round
// makes at least one more position exact (the first mispredicted one is decided from an exact
// state), so 16 rounds always finish a group: the serial fallback is then never reached
#ifndef HVX_RDOQ_ROUNDS
#define HVX_RDOQ_ROUNDS 16
#endif
// The c1 / c2 / Rice / c1Idx / c2Idx update after a position's decision (:2281-2330)
__device__ __forceinline__ void rd_step(uint32_t level, int &c1, int &c2, uint32_t &c1_idx, uint32_t &c2_idx, uint32_t &rice,
                                        bool persistent) {
  const bool c1ok = c1_idx < 8, c2ok = c2_idx < 1;
  const uint32_t base = c1ok ? (c2ok ? 3u : 2u) : 1u;
  if (level >= base && level > 3u * (1u << rice)) rice = persistent ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
  if (level >= 1) c1_idx++;
  if (level > 1) { c1 = 0; c2 += (c2 < 2); c2_idx++; }
  else if (c1 < 3 && c1 > 0 && level) c1++;
}
// xGetICRate: the branch-free form when extended precision is compiled out (HVX_TU_NO_EXT)
__device__ __forceinline__ int rd_rate(uint32_t level, uint32_t rice, bool c1ok, bool c2ok, int g0, int g1, int a0, int a1,
                                       int ext, int max_log2) {
#ifdef HVX_TU_NO_EXT
  (void)ext; (void)max_log2;
  return rd_ic_rate_bf(level, rice, c1ok, c2ok, g0, g1, a0, a1);
#else
  return rd_ic_rate(level, (int)rice, c1ok, c2ok, g0, g1, a0, a1, ext, max_log2);
#endif
}

// Per scan position, the RDOQ pass keeps one packed int in s.a:
//   before the serial pass: the significance context under each of the 4 neighbour-CG
//     patterns (6 bits each);
//   after it: the context state of its decision -- ctx_one | ctx_abs<<5 | rice<<8 |
//     c1ok<<13 | c2ok<<14 | has_sig<<15 | ctx_sig<<16 | sig_sel<<22, where sig_sel says
//     which significance-flag rate its cost carried (0 none, 1 sig=0, 2 sig=1).
// From it (and the level and lLevelDouble) every per-position quantity the later passes
// need -- the chosen cost, the flag cost, the sign-hiding rate deltas -- is recomputed
// with the same operations, hence bit-identically.
struct RdCtx {
  int ctx_one, ctx_abs, rice, ctx_sig, sig_sel;
  bool c1ok, c2ok, has_sig;
};
__device__ __forceinline__ int rd_pack(int one, int abs_, int rice, bool c1ok, bool c2ok, bool has_sig, int sig,
                                       int sel) {
  return one | (abs_ << 5) | (rice << 8) | ((int)c1ok << 13) | ((int)c2ok << 14) | ((int)has_sig << 15) |
         (sig << 16) | (sel << 22);
}
__device__ __forceinline__ RdCtx rd_unpack(int v) {
  RdCtx r;
  r.ctx_one = v & 31; r.ctx_abs = (v >> 5) & 7; r.rice = (v >> 8) & 31;
  r.c1ok = (v >> 13) & 1; r.c2ok = (v >> 14) & 1; r.has_sig = (v >> 15) & 1; r.ctx_sig = (v >> 16) & 63;
  r.sig_sel = (v >> 22) & 3;
  return r;
}

// lLevelDouble (:2210) of a coefficient
__device__ __forceinline__ int32_t rd_level_double(int32_t coef, int qc, int64_t lim) {
  const int64_t t = (int64_t)abs(coef) * qc;
  return (int32_t)(t < lim ? t : lim);
}

// xRateDistOptQuant (:2129-2671).  Input s.coef (raster); output s.lev (signed levels), returns uiAbsSum.
//
// The reverse-scan state machine (c1/c2/Rice/context-set carry, CG zero-out, last-position
// search) is inherently serial; it runs as WAVE-UNIFORM code: every lane executes the same
// scalar control flow, the estBits tables it indexes with state-dependent contexts sit in
// lane slices of four VGPRs and are fetched with v_readlane (no dependent memory loads),
// each coefficient group's 16 inputs are loaded in one batch (one per lane, read back by
// v_readlane), and the 16 per-position results are gathered into lanes 0..15 and stored
// once per group.  Double precision with the reference's exact operation order
// (-ffp-contract=off) keeps every decision identical.  Sign hiding then runs one
// coefficient group per lane (groups are independent), with the rate deltas recomputed
// from the packed context state of each position.
// scan / scan_cg: optional copies of the TU's scan tables (e.g. staged in LDS by a caller that
// runs many TUs serially: the serial passes then read no global memory); nullptr: kScan / kScanCG
template <int L>
__device__ int32_t tu_rdoq(TuSmem<L> &s, const hvx_tu_desc &d, const hvx_estbits *est, int32_t *arl_out,
                           const uint16_t *scan = nullptr, const uint8_t *scan_cg = nullptr) {
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
  const double lambda = d.lambda;
  TuCoding c = tu_coding<L>(d);
  if (scan) c.scan = scan;
  if (scan_cg) c.scan_cg = scan_cg;
  const int64_t lim = (int64_t)2147483647 - ((int64_t)1 << (qbits - 1));
  const int qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
  const int lane = lane_id();
  const int sig_off = ch ? 28 : 0;
  int32_t *st = s.a;  // the residual is dead once the forward transform has run

#ifdef HVX_TU_PROF_HOOK
  uint64_t t_ph = __builtin_amdgcn_s_memtime();
#define HVX_RDOQ_PHASE(k) do { const uint64_t t_n = __builtin_amdgcn_s_memtime(); HVX_TU_PROF_HOOK(28 + (k), t_n - t_ph); t_ph = t_n; } while (0)
#else
#define HVX_RDOQ_PHASE(k) ((void)0)
#endif
// sub-phases of the reverse scan (profile builds with HVX_RDOQ_PROF_SUB: slots 12..15)
#define HVX_RDOQ_SUB(k) ((void)0)
  // ---- A. per-coefficient work across lanes ----
  bool anyq = false;
  for (int sp = lane; sp < NN; sp += HVX_WAVE) {
    const int blk = c.scan[sp];
    const int32_t ld = rd_level_double(s.coef[blk], qc, lim);
    if (arl_out) arl_out[blk] = d.adaptive_qp_select ? (ld + add_c) >> qbits_c : 0;
    anyq |= ((ld + (1 << (qbits - 1))) >> qbits) > 0;
    int info = 0;
#pragma unroll
    for (int pat = 0; pat < 4; pat++) info |= (sig_off + rd_sig_ctx<L>(pat, c, sp, ch)) << (6 * pat);
    st[sp] = info;
  }
  // every rounded level 0: the decisions all keep level 0 (no last position, nothing to hide), so
  // the reverse scan would only price them -- its outputs are all-zero levels and uiAbsSum 0
  if (__ballot(anyq) == 0) {
    for (int i = lane; i < NN; i += HVX_WAVE) s.lev[i] = 0;
    __syncthreads();
    return 0;
  }
  // estBits in lane slices: entry [ctx][0] in lane ctx, [ctx][1] in lane 32 + ctx (or own VGPR)
  const int t_sb0 = lane < 44 ? est->significantBits[lane][0] : 0;
  const int t_sb1 = lane < 44 ? est->significantBits[lane][1] : 0;
  const int t_g = lane < 24 ? est->greaterOneBits[lane][0] : (lane >= 32 && lane < 56) ? est->greaterOneBits[lane - 32][1] : 0;
  const int t_a = lane < 6 ? est->levelAbsBits[lane][0] : (lane >= 32 && lane < 38) ? est->levelAbsBits[lane - 32][1] : 0;
  __syncthreads();

  HVX_RDOQ_PHASE(0);
  // ---- B. reverse-scan decisions (wave-uniform) ----
  const uint32_t rice0 = (uint32_t)d.golomb_rice_stat / 4;
  const bool persistent = d.persistent_rice != 0;
  uint32_t rice = rice0, ctx_set = 0, c1_idx = 0, c2_idx = 0;
  int c1 = 1, c2 = 0, last = -1, cg_last = -1;
  double block_uncoded = 0, base_cost = 0;
  uint64_t sigmask = 0;  // coded_sub_block_flag by CG raster index
  for (int cgp = NCG - 1; cgp >= 0; cgp--) {
    const int cgblk = c.scan_cg[cgp];
    const int cy = cgblk / c.wg, cx = cgblk - cy * c.wg;
    int pattern = 0;
    if (NCG > 1) {
      const int rr = cx < c.wg - 1 ? (int)((sigmask >> (cgblk + 1)) & 1) : 0;
      const int bb = cy < c.wg - 1 ? (int)((sigmask >> (cgblk + c.wg)) & 1) : 0;
      pattern = rr + (bb << 1);
    }
    // the group's 16 inputs, one per lane (read back with v_readlane), and everything of a
    // position's decision that does not depend on the serial c1 / c2 / Rice state, computed
    // lane-parallel with the serial pass's own operations (same values bit for bit): the
    // quantised magnitude, the uncoded cost, the distortion term of both candidate levels, the
    // significance context and its two flag costs
    const int myblk = c.scan[cgp * 16 + (lane & 15)];
    const int ldl = rd_level_double(s.coef[myblk], qc, lim);
    const int infl = st[cgp * 16 + (lane & 15)];
    const int shp = 6 * pattern;
    const uint32_t q_l = (uint32_t)((ldl + (1 << (qbits - 1))) >> qbits);
    const uint32_t ma_l = (uint32_t)ecmax < q_l ? (uint32_t)ecmax : q_l;
    const double e_l = (double)ldl;
    const double cc0_l = e_l * e_l * escale;
    const double er1 = (double)sub32(ldl, shl32((int32_t)ma_l, qbits));
    const double d1_l = er1 * er1 * escale;  // distortion term of level max_abs
    const double er2 = (double)sub32(ldl, shl32((int32_t)ma_l - 1, qbits));
    const double d2_l = er2 * er2 * escale;  // ... of level max_abs - 1
    const int ctxs_l = (infl >> shp) & 63;
    const double ls0_l = lambda * (double)est->significantBits[ctxs_l][0];
    const double ls1_l = lambda * (double)est->significantBits[ctxs_l][1];
    int nnz0 = 0;
    bool any = false;
    double coded_ld = 0, uncoded = 0, sig_cost = 0, sig_cost0 = 0;
    int o_lev = 0, o_st = 0;  // lane pin: results of scan position cgp*16 + pin
    // the reference's per-position decision on the serial state (xGetCodedLevel :2822 and the
    // c1 / c2 / Rice updates :2281-2330), for positions pin_hi .. 0 of a group holding or
    // following the last significant position; the group-end reset is the caller's
    auto serial_from = [&](int pin_hi) {
      for (int pin = pin_hi; pin >= 0; pin--) {
        const int sp = cgp * 16 + pin;
        const uint32_t max_abs = (uint32_t)rl((int)ma_l, pin);
        const double cc0 = rld(cc0_l, pin);
        block_uncoded += cc0;
        const int ctx_one = 4 * (int)ctx_set + c1, ctx_abs = (int)ctx_set + c2;
        const int g0 = rl(t_g, ctx_one), g1 = rl(t_g, ctx_one + 32), a0 = rl(t_a, ctx_abs), a1 = rl(t_a, ctx_abs + 32);
        const bool c1ok = c1_idx < 8, c2ok = c2_idx < 1;
        const bool is_last = sp == last;
        const int ctx_sig = is_last ? 0 : rl(ctxs_l, pin);
        double cur_sig = 0, cost, cost_sig = 0;
        int sel = 0;
        uint32_t best = 0;
        bool done = false;
        if (!is_last && max_abs < 3) {
          cost_sig = rld(ls0_l, pin);  // lambda * significantBits[ctx][0]
          sel = 1;
          cost = cc0 + cost_sig;
          if (max_abs == 0) done = true;
        } else {
          cost = 1.7e+308;
        }
        if (!done) {
          if (!is_last) cur_sig = rld(ls1_l, pin);
          const double dist1 = rld(d1_l, pin), dist2 = rld(d2_l, pin);
          // the candidates max_abs and (max_abs > 1) max_abs - 1, tried in that order with the
          // strict comparison of the reference's loop; both costs are formed independently
          const bool two = max_abs > 1;
          const uint32_t lv2 = two ? max_abs - 1 : max_abs;
          const int r1 = rd_rate(max_abs, rice, c1ok, c2ok, g0, g1, a0, a1, ext, max_log2);
          const int r2 = rd_rate(lv2, rice, c1ok, c2ok, g0, g1, a0, a1, ext, max_log2);
          double cl1 = dist1 + lambda * (double)r1;
          cl1 += cur_sig;
          double cl2 = dist2 + lambda * (double)r2;
          cl2 += cur_sig;
          if (cl1 < cost) { best = max_abs; cost = cl1; cost_sig = cur_sig; sel = is_last ? 0 : 2; }
          if (two && cl2 < cost) { best = lv2; cost = cl2; cost_sig = cur_sig; sel = is_last ? 0 : 2; }
        }
        const double cc = cost, cs = cost_sig;
        const int stv = rd_pack(ctx_one, ctx_abs, (int)rice, c1ok, c2ok, !is_last, ctx_sig, sel);
        base_cost += cc;
        rd_step(best, c1, c2, c1_idx, c2_idx, rice, persistent);
        sig_cost += cs;
        if (pin == 0) sig_cost0 = cs;
        if (best) {
          any = true;
          coded_ld += cc - cs;
          uncoded += cc0;
          if (pin != 0) nnz0++;
        }
        if (lane == pin) { o_lev = (int32_t)best; o_st = stv; }
      }
    };
    HVX_RDOQ_SUB(0);
    // the decided positions: from the last significant one (its group) or the whole group
    int start = 15;
    if (last < 0) {
      const uint64_t nz = __ballot(lane < 16 && ma_l > 0);
      start = nz ? 63 - (int)__clzll(nz) : -1;
      if (nz) {
        last = cgp * 16 + start;
        ctx_set = (comp ? 4 : 0) + ((comp == 0 && cgp > 0) ? 2 : 0);
        cg_last = cgp;
      }
    }
    // above it: uncoded costs only (every level there is 0)
    for (int pin = 15; pin > start; pin--) {
      const double cc0 = rld(cc0_l, pin);
      block_uncoded += cc0;
      base_cost += cc0;
    }
    if (start >= 0) {
      // Speculation in rounds: the serial state at each decided position is predicted from guessed
      // levels of the positions before it (scalar, integers only), and every position's decision
      // is then evaluated lane-parallel from its predicted state with the serial pass's own
      // operations.  The guesses start at max_abs and are the previous round's decisions after
      // that.  A position whose state update from its decision differs from the one from its
      // guess invalidates the predictions below it; every position down to the first such one is
      // exact (its predecessors' updates all matched).  After the last round the rest of the
      // group runs the serial pass from the true state.
      uint32_t guess = ma_l;
      int pst_l = 0, f = -1;
      double cost = 0, cost_sig = 0;
      uint32_t best = 0;
      int stv_l = 0;
      for (int round = 0;; round++) {
        {
          // rd_step's updates in closed form over the positions decided before this lane's (pins
          // start .. pin+1): c1Idx / c2Idx count the levels >= 1 / > 1, c2 saturates at 2, c1 is 0
          // after a level > 1 and otherwise counts the 1s up to 3 (from a nonzero start); the Rice
          // parameter can only move at a level > 3 (a level > 3 << rice is always >= base), so it
          // is scanned over those positions alone
          const int pin_l = lane & 15;
          const uint32_t mdec = (2u << start) - 1u;
          const uint32_t above = mdec & ~((2u << pin_l) - 1u);
          const uint32_t nzg = (uint32_t)__ballot(lane < 16 && guess >= 1u) & mdec;
          const uint32_t g1g = (uint32_t)__ballot(lane < 16 && guess > 1u) & mdec;
          const int n_nz = __popc(nzg & above), n_g1 = __popc(g1g & above);
          const int c2s = c2 + n_g1 < 2 ? c2 + n_g1 : 2;
          const int c1n = c1 + (n_nz - n_g1);
          const int c1s = n_g1 ? 0 : (c1 == 0 ? 0 : (c1n < 3 ? c1n : 3));
          uint32_t rs = rice;
          uint32_t big = (uint32_t)__ballot(lane < 16 && guess > 3u) & mdec;
          if (big) {
            uint32_t r = rice;
            while (big) {
              const int p = 31 - (int)__clz(big);
              big &= ~(1u << p);
              if ((uint32_t)rl((int)guess, p) > 3u * (1u << r)) r = persistent ? r + 1 : (r + 1 < 4 ? r + 1 : 4);
              if (pin_l < p) rs = r;
            }
          }
          pst_l = c1s | (c2s << 2) | ((int)(c1_idx + n_nz) << 4) | ((int)(c2_idx + n_g1) << 9) | ((int)rs << 14);
        }
        const int c1p = pst_l & 3, c2p = (pst_l >> 2) & 3;
        const uint32_t c1ip = (uint32_t)(pst_l >> 4) & 31, c2ip = (uint32_t)(pst_l >> 9) & 31, rp = (uint32_t)(pst_l >> 14) & 31;
        const int ctx_one_l = 4 * (int)ctx_set + c1p, ctx_abs_l = (int)ctx_set + c2p;
        const int g0l = __shfl(t_g, ctx_one_l, HVX_WAVE), g1l = __shfl(t_g, ctx_one_l + 32, HVX_WAVE);
        const int a0l = __shfl(t_a, ctx_abs_l, HVX_WAVE), a1l = __shfl(t_a, ctx_abs_l + 32, HVX_WAVE);
        const bool c1okl = c1ip < 8, c2okl = c2ip < 1;
        const int pin_l = lane & 15;
        const bool is_last_l = cgp * 16 + pin_l == last;
        const int ctx_sig_l = is_last_l ? 0 : ctxs_l;
        double cur_sig = 0;
        cost_sig = 0;
        int sel = 0;
        best = 0;
        bool done = false;
        if (!is_last_l && ma_l < 3) {
          cost_sig = ls0_l;
          sel = 1;
          cost = cc0_l + cost_sig;
          if (ma_l == 0) done = true;
        } else {
          cost = 1.7e+308;
        }
        if (!done) {
          if (!is_last_l) cur_sig = ls1_l;
          const bool two = ma_l > 1;
          const uint32_t lv2 = two ? ma_l - 1 : ma_l;
          const int r1 = rd_rate(ma_l, rp, c1okl, c2okl, g0l, g1l, a0l, a1l, ext, max_log2);
          const int r2 = rd_rate(lv2, rp, c1okl, c2okl, g0l, g1l, a0l, a1l, ext, max_log2);
          double cl1 = d1_l + lambda * (double)r1;
          cl1 += cur_sig;
          double cl2 = d2_l + lambda * (double)r2;
          cl2 += cur_sig;
          if (cl1 < cost) { best = ma_l; cost = cl1; cost_sig = cur_sig; sel = is_last_l ? 0 : 2; }
          if (two && cl2 < cost) { best = lv2; cost = cl2; cost_sig = cur_sig; sel = is_last_l ? 0 : 2; }
        }
        stv_l = rd_pack(ctx_one_l, ctx_abs_l, (int)rp, c1okl, c2okl, !is_last_l, ctx_sig_l, sel);
        bool ok;
        {
          int a1c = c1p, a2c = c2p, b1c = c1p, b2c = c2p;
          uint32_t a1i = c1ip, a2i = c2ip, ar = rp, b1i = c1ip, b2i = c2ip, br = rp;
          rd_step(best, a1c, a2c, a1i, a2i, ar, persistent);
          rd_step(guess, b1c, b2c, b1i, b2i, br, persistent);
          ok = a1c == b1c && a2c == b2c && a1i == b1i && a2i == b2i && ar == br;
        }
        const uint64_t bad = __ballot(lane <= start && !ok);
        f = bad ? 63 - (int)__clzll(bad) : -1;  // the first position (in scan order) whose update differs
        if (f <= 0 || round == HVX_RDOQ_ROUNDS - 1) break;
        guess = best;
      }
      HVX_RDOQ_SUB(1);
      const double dlt_l = cost - cost_sig;  // coded_ld's term (the serial pass's cc - cs)
      const uint32_t nzm = (uint32_t)__ballot(lane <= start && best != 0);
      const int lo = f < 0 ? 0 : f;
      for (int pin = start; pin >= lo; pin--) {
        const double cc0 = rld(cc0_l, pin);
        block_uncoded += cc0;
        const double cc = rld(cost, pin), cs = rld(cost_sig, pin);
        base_cost += cc;
        sig_cost += cs;
        if (pin == 0) sig_cost0 = cs;
        if ((nzm >> pin) & 1u) {
          any = true;
          coded_ld += rld(dlt_l, pin);
          uncoded += cc0;
          if (pin != 0) nnz0++;
        }
      }
      if (lane <= start && lane >= lo) { o_lev = (int32_t)best; o_st = stv_l; }
      if (f < 0) {  // every prediction held: the state after position 0 is the predicted one
        const int pk = rl(pst_l, 0);
        c1 = pk & 3; c2 = (pk >> 2) & 3; c1_idx = (uint32_t)(pk >> 4) & 31; c2_idx = (uint32_t)(pk >> 9) & 31;
        rice = (uint32_t)(pk >> 14) & 31;
        rd_step((uint32_t)rl((int)best, 0), c1, c2, c1_idx, c2_idx, rice, persistent);
      } else {  // the true state after position f, then the serial pass for the rest of the group
        const int pk = rl(pst_l, f);
        c1 = pk & 3; c2 = (pk >> 2) & 3; c1_idx = (uint32_t)(pk >> 4) & 31; c2_idx = (uint32_t)(pk >> 9) & 31;
        rice = (uint32_t)(pk >> 14) & 31;
        rd_step((uint32_t)rl((int)best, f), c1, c2, c1_idx, c2_idx, rice, persistent);
        if (f > 0) serial_from(f - 1);
      }
      HVX_RDOQ_SUB(2);
      if (cgp > 0) {  // the next group's context set and counters (:2262-2266)
        ctx_set = (comp ? 4 : 0) + ((comp == 0 && cgp - 1 > 0) ? 2 : 0) + (c1 == 0 ? 1 : 0);
        c1 = 1; c2 = 0; c1_idx = 0; c2_idx = 0;
        rice = rice0;
      }
    }
    if (any) sigmask |= 1ull << cgblk;
    int cgrate = 0;
    if (cg_last >= 0) {
      if (cgp) {
        const int rr = cx < c.wg - 1 ? (int)((sigmask >> (cgblk + 1)) & 1) : 0;
        const int bb = cy < c.wg - 1 ? (int)((sigmask >> (cgblk + c.wg)) & 1) : 0;
        const int ctx = (rr + bb) != 0;
        const int r0 = est->significantCoeffGroupBits[ctx][0], r1 = est->significantCoeffGroupBits[ctx][1];
        if (!any) {
          base_cost += lambda * (double)r0 - sig_cost;
          cgrate = r0;
        } else if (cgp < cg_last) {
          if (nnz0 == 0) { base_cost -= sig_cost0; sig_cost -= sig_cost0; }
          double zero_cost = base_cost;
          base_cost += lambda * (double)r1;
          zero_cost += lambda * (double)r0;
          cgrate = r1;
          zero_cost += uncoded;
          zero_cost -= coded_ld;
          zero_cost -= sig_cost;
          if (zero_cost < base_cost) {  // the whole group is zeroed (its cost/flag entries are never read again)
            sigmask &= ~(1ull << cgblk);
            base_cost = zero_cost;
            cgrate = r0;
            o_lev = 0;
          }
        }
      } else {
        sigmask |= 1ull << cgblk;
      }
    }
    if (lane < 16) {
      s.lev[myblk] = o_lev;
      st[cgp * 16 + lane] = o_st;
    }
    if (lane == 0) s.cgr[cgp] = cgrate;
    HVX_RDOQ_SUB(3);
  }
  __syncthreads();

  HVX_RDOQ_PHASE(1);
  if (last < 0) return 0;  // every level is 0 (written above)

  // ---- C. best last position (wave-uniform) ----
  double best_cost;
  int best_p1 = 0;
  if (!d.is_intra && ch == 0 && d.tr_idx == 0) {
    best_cost = block_uncoded + lambda * (double)est->blockRootCbpBits[0][0];
    base_cost += lambda * (double)est->blockRootCbpBits[0][1];
  } else {
    const int ctx = d.ctx_qt_cbf + (ch ? 5 : 0);
    best_cost = block_uncoded + lambda * (double)est->blockCbpBits[ctx][0];
    base_cost += lambda * (double)est->blockCbpBits[ctx][1];
  }
  bool found = false;
  for (int cgp = cg_last; cgp >= 0 && !found; cgp--) {
    const int cgblk = c.scan_cg[cgp];
    base_cost -= lambda * (double)s.cgr[cgp];
    if ((sigmask >> cgblk) & 1) {
      for (int pin = 15; pin >= 0; pin--) {
        const int sp = cgp * 16 + pin;
        if (sp > last) continue;
        const int blk = c.scan[sp];
        const int lvv = s.lev[blk];
        const RdCtx x = rd_unpack(st[sp]);
        // the flag cost this position's decision carried
        const int sbr = x.sig_sel == 1 ? rl(t_sb0, x.ctx_sig) : x.sig_sel == 2 ? rl(t_sb1, x.ctx_sig) : 0;
        const double cs = x.sig_sel ? lambda * (double)sbr : 0.0;
        if (lvv) {
          const int py = blk >> LOG2, px = blk - (py << LOG2);
          const double cl = c.scan_type == 2 ? rd_rate_last(est, lambda, py, px, ch) : rd_rate_last(est, lambda, px, py, ch);
          const double total = base_cost + cl - cs;
          if (total < best_cost) { best_p1 = sp + 1; best_cost = total; }
          if (lvv > 1) { found = true; break; }
          // the cost of the chosen level 1, recomputed as the serial pass computed it
          const int32_t ld = rd_level_double(s.coef[blk], qc, lim);
          const double err = (double)sub32(ld, shl32(1, qbits));
          const int rate = rd_ic_rate(1u, x.rice, x.c1ok, x.c2ok, rl(t_g, x.ctx_one), rl(t_g, x.ctx_one + 32),
                                      rl(t_a, x.ctx_abs), rl(t_a, x.ctx_abs + 32), ext, max_log2);
          double cc = err * err * escale + lambda * (double)rate;
          cc += x.has_sig ? lambda * (double)rl(t_sb1, x.ctx_sig) : 0.0;
          base_cost -= cc;
          const double e = (double)ld;
          base_cost += e * e * escale;
        } else {
          base_cost -= cs;
        }
      }
    }
  }
  __syncthreads();

  HVX_RDOQ_PHASE(2);
  // ---- D. signs, zeroing past the chosen last position, uiAbsSum (lanes) ----
  int part = 0;
  for (int sp = lane; sp <= last; sp += HVX_WAVE) {
    const int blk = c.scan[sp];
    if (sp < best_p1) {
      const int32_t lv = s.lev[blk];
      part += lv;
      s.lev[blk] = s.coef[blk] < 0 ? -lv : lv;
    } else {
      s.lev[blk] = 0;
    }
  }
  const int32_t abs_sum = wave_sum_i32(part);
  __syncthreads();

  // ---- E. RD sign-bit hiding (:2541-2660): one coefficient group per lane ----
  if (d.sign_hiding && abs_sum >= 2) {
    const double iq = (double)kInvQuantScales[d.qp_rem];
    const int64_t rdf = (int64_t)(iq * iq * (1 << (2 * d.qp_per)) / d.lambda / 16 / (1 << 0) + 0.5);
    if constexpr (L <= 1) {
      // TUs up to 8x8: every position in its own lane (lane = group * 16 + k).  A group's
      // first / last non-zero come from its ballot, its level sum (signed, as the reference sums
      // it: positions outside [first_nz, last_nz] hold 0) from a 16-lane reduction, and the
      // reverse loop's strict-minimum search from a 16-lane argmin keeping the highest k on ties
      // (the first minimum the descending loop meets) -- the same change at the same position.
      const int sub = lane >> 4, k = lane & 15, pos = sub << 4;
      const bool valid = sub < NCG;
      const int blk = valid ? c.scan[pos + k] : 0;
      const int32_t lv = valid ? s.lev[blk] : 0;
      const int32_t cf = valid ? s.coef[blk] : 0;
      const int stv = valid ? st[pos + k] : 0;
      const uint64_t nzm = __ballot(lv != 0);
      const uint32_t m16 = (uint32_t)(nzm >> pos) & 0xffffu;
      const int last_nz = m16 ? 31 - __clz(m16) : -1, first_nz = m16 ? __builtin_ctz(m16) : 16;
      const int top = nzm ? (63 - (int)__clzll(nzm)) >> 4 : -1;
      int abs_in = lv;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) abs_in += __shfl_xor(abs_in, o, HVX_WAVE);
      const int lv_first = __shfl(lv, (pos + (first_nz & 15)) & 63, HVX_WAVE);
      const uint32_t signbit = lv_first > 0 ? 0 : 1;
      const bool act = valid && last_nz - first_nz >= 4 && signbit != (uint32_t)(abs_in & 1);
      const bool is_top = sub == top;
      long long cur = INT64_MAX;
      int cch = 0;
      if (act && k <= (is_top ? last_nz : 15)) {
        const uint32_t lev0 = (uint32_t)abs(lv);
        const int32_t ld = rd_level_double(cf, qc, lim);
        const int32_t du = sub32(ld, shl32((int32_t)lev0, qbits)) >> (qbits - 8);
        const RdCtx x = rd_unpack(stv);
        const int g0 = est->greaterOneBits[x.ctx_one][0];
        const int sigd = x.has_sig ? est->significantBits[x.ctx_sig][1] - est->significantBits[x.ctx_sig][0] : 0;
        int rup = g0, rdown = 0;
        if (lev0 > 0) {
          const int g1 = est->greaterOneBits[x.ctx_one][1];
          const int a0 = est->levelAbsBits[x.ctx_abs][0], a1 = est->levelAbsBits[x.ctx_abs][1];
          const int now = rd_ic_rate(lev0, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2);
          rup = rd_ic_rate(lev0 + 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
          rdown = rd_ic_rate(lev0 - 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
        }
        if (lv != 0) {
          const int64_t up = rdf * (-du) + rup;
          int64_t down = rdf * (du) + rdown - ((abs(lv) == 1) ? sigd : 0);
          if (is_top && last_nz == k && abs(lv) == 1) down -= (4 << 15);
          if (up < down) { cur = up; cch = 1; }
          else { cch = -1; cur = (k == first_nz && abs(lv) == 1) ? INT64_MAX : down; }
        } else {
          cur = rdf * (-(abs(du))) + (1 << 15) + rup + sigd;
          cch = 1;
          if (k < first_nz) {
            const uint32_t tsb = cf >= 0 ? 0 : 1;
            if (tsb != signbit) cur = INT64_MAX;
          }
        }
      }
      // argmin over the group: the smallest cost, the highest k among equal costs
      long long bc = cur;
      int bk = cur < INT64_MAX ? k : -1;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        const long long oc = __shfl_xor(bc, o, HVX_WAVE);
        const int ok = __shfl_xor(bk, o, HVX_WAVE);
        if (oc < bc || (oc == bc && ok > bk)) { bc = oc; bk = ok; }
      }
      const int src = (pos + (bk < 0 ? 0 : bk)) & 63;
      const int min_pos = bk < 0 ? -1 : __shfl(blk, src, HVX_WAVE);
      int fch = __shfl(cch, src, HVX_WAVE);
      if (bk < 0) fch = 0;
      if (act && k == 0) {
        if (s.lev[min_pos] == ecmax || s.lev[min_pos] == ecmin) fch = -1;
        if (s.coef[min_pos] >= 0) s.lev[min_pos] += fch;
        else s.lev[min_pos] -= fch;
      }
      __syncthreads();
      HVX_RDOQ_PHASE(3);
      return abs_sum;
    }
    const int sub = lane, pos = sub << 4;
    int first_nz = 16, last_nz = -1, abs_in = 0;
    if (sub < NCG) {
      for (int k = 15; k >= 0; k--) if (s.lev[c.scan[k + pos]]) { last_nz = k; break; }
      for (int k = 0; k < 16; k++) if (s.lev[c.scan[k + pos]]) { first_nz = k; break; }
      for (int k = first_nz; k <= last_nz; k++) abs_in += s.lev[c.scan[k + pos]];
    }
    // the highest group holding a level is the reference's lastCG
    int top = last_nz >= 0 ? sub : -1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) top = max(top, __shfl_xor(top, o, HVX_WAVE));
    if (sub < NCG && last_nz - first_nz >= 4) {
      const uint32_t signbit = s.lev[c.scan[pos + first_nz]] > 0 ? 0 : 1;
      if (signbit != (uint32_t)(abs_in & 1)) {
        const bool is_top = sub == top;
        int64_t min_inc = INT64_MAX, cur = INT64_MAX;
        int min_pos = -1, fch = 0, cch = 0;
        for (int k = (is_top ? last_nz : 15); k >= 0; k--) {
          const int sp = k + pos;
          const int blk = c.scan[sp];
          const int32_t lv = s.lev[blk];
          const uint32_t lev0 = (uint32_t)abs(lv);  // == the serial pass's level at every position scanned here
          const int32_t ld = rd_level_double(s.coef[blk], qc, lim);
          const int32_t du = sub32(ld, shl32((int32_t)lev0, qbits)) >> (qbits - 8);
          const RdCtx x = rd_unpack(st[sp]);
          const int g0 = est->greaterOneBits[x.ctx_one][0];
          const int sigd = x.has_sig ? est->significantBits[x.ctx_sig][1] - est->significantBits[x.ctx_sig][0] : 0;
          int rup = g0, rdown = 0;
          if (lev0 > 0) {
            const int g1 = est->greaterOneBits[x.ctx_one][1];
            const int a0 = est->levelAbsBits[x.ctx_abs][0], a1 = est->levelAbsBits[x.ctx_abs][1];
            const int now = rd_ic_rate(lev0, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2);
            rup = rd_ic_rate(lev0 + 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
            rdown = rd_ic_rate(lev0 - 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
          }
          if (lv != 0) {
            const int64_t up = rdf * (-du) + rup;
            int64_t down = rdf * (du) + rdown - ((abs(lv) == 1) ? sigd : 0);
            if (is_top && last_nz == k && abs(lv) == 1) down -= (4 << 15);
            if (up < down) { cur = up; cch = 1; }
            else { cch = -1; cur = (k == first_nz && abs(lv) == 1) ? INT64_MAX : down; }
          } else {
            cur = rdf * (-(abs(du))) + (1 << 15) + rup + sigd;
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
    __syncthreads();
  }
  HVX_RDOQ_PHASE(3);
#undef HVX_RDOQ_PHASE
  return abs_sum;
}

// xQuant (:1126) non-RDOQ path + signBitHidingHDQ (:991).  Input s.coef, output s.lev;
// deltaU is kept in s.a.
template <int L>
__device__ int32_t tu_quant_plain(TuSmem<L> &s, const hvx_tu_desc &d, int32_t *arl_out) {
  constexpr int NN = (4 << L) * (4 << L);
  const int ts = tu_transform_shift(d);
  const int qbits = 14 + d.qp_per + ts;
  const int qc = kQuantScales[d.qp_rem];
  const int add = (d.slice_type == 2 ? 171 : 85) << (qbits - 9);
  const int qbits8 = qbits - 8, qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
  const int32_t ecmax = (1 << d.max_log2_tr_range) - 1, ecmin = -(1 << d.max_log2_tr_range);
  int32_t *du = s.a;
  int part = 0;
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int32_t lv = s.coef[i];
    const int sign = lv < 0 ? -1 : 1;
    const int64_t t = (int64_t)abs(lv) * qc;
    if (arl_out) arl_out[i] = d.adaptive_qp_select ? (int32_t)((t + add_c) >> qbits_c) : 0;
    const int32_t qm = (int32_t)((t + add) >> qbits);
    du[i] = (int32_t)((t - (int64_t)shl32(qm, qbits)) >> qbits8);
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
              if (du[blk] > 0) { cur = -du[blk]; cch = 1; }
              else if (k == first_nz && abs(q) == 1) cur = INT32_MAX;
              else { cur = du[blk]; cch = -1; }
            } else if (k < first_nz) {
              const uint32_t tsb = s.coef[blk] >= 0 ? 0 : 1;
              if (tsb != signbit) cur = INT32_MAX;
              else { cur = -du[blk]; cch = 1; }
            } else {
              cur = -du[blk]; cch = 1;
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

// transformNxN (:1460) on s.a (the residual as int, raster N*N).  Leaves s.coef (transform
// output) and s.lev (levels); returns uiAbsSum.
template <int L>
__device__ int32_t tu_forward(TuSmem<L> &s, const hvx_tu_desc &d, const hvx_estbits *est, int32_t *arl_out,
                              const uint16_t *scan = nullptr, const uint8_t *scan_cg = nullptr) {
  constexpr int N = 4 << L, NN = N * N;
  if (d.transquant_bypass) {
    int part = 0;
    for (int i = lane_id(); i < NN; i += HVX_WAVE) { s.lev[i] = s.a[i]; s.coef[i] = s.a[i]; part += abs(s.a[i]); }
    __syncthreads();
    return wave_sum_i32(part);
  }
#ifdef HVX_TU_PROF_HOOK
  const uint64_t t_x0 = __builtin_amdgcn_s_memtime();
#endif
  if (d.transform_skip) {
    const int ts = tu_transform_shift(d);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int32_t v = s.a[i];
      s.coef[i] = ts >= 0 ? shl32(v, ts) : (v + (1 << (-ts - 1))) >> -ts;
    }
    __syncthreads();
  } else {
    tu_forward_transform<L>(s, d.use_dst && N == 4);
  }
#ifdef HVX_TU_PROF_HOOK
  HVX_TU_PROF_HOOK(22, __builtin_amdgcn_s_memtime() - t_x0);
#endif
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
#ifdef HVX_TU_PROF_HOOK
    if (need) {
      const uint64_t t_r0 = __builtin_amdgcn_s_memtime();
      const int32_t r = tu_rdoq<L>(s, d, est, arl_out, scan, scan_cg);
      HVX_TU_PROF_HOOK(23, __builtin_amdgcn_s_memtime() - t_r0);
      return r;
    }
#else
    if (need) return tu_rdoq<L>(s, d, est, arl_out, scan, scan_cg);
#endif
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      s.lev[i] = 0;
      if (arl_out) arl_out[i] = 0;
    }
    __syncthreads();
    return 0;
  }
  return tu_quant_plain<L>(s, d, arl_out);
}

// invTransformNxN (:1547) on the levels in s.lev (raster) -> reconstructed residual in s.lev
// (values fit Pel); s.a and s.coef are scratch.
template <int L>
__device__ void tu_inverse(TuSmem<L> &s, const hvx_tu_desc &d) {
  constexpr int N = 4 << L, NN = N * N;
  if (d.transquant_bypass) {
    for (int i = lane_id(); i < NN; i += HVX_WAVE) s.lev[i] = (int16_t)s.lev[i];
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
    const int32_t c = clip3(imin, imax, s.lev[i]);
    const int32_t v = right > 0 ? (c * scale + (1 << (right - 1))) >> right : shl32(c * scale, -right);
    deq[i] = clip3(tmin, tmax, v);
  }
  __syncthreads();
  if (d.transform_skip) {
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int32_t v = deq[i];
      s.lev[i] = (int16_t)(ts >= 0 ? (v + (ts == 0 ? 0 : 1 << (ts - 1))) >> ts : shl32(v, -ts));
    }
    __syncthreads();
  } else {
    tu_inverse_transform<L>(d.use_dst && N == 4, deq, s.coef, s.lev);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) s.lev[i] = (int16_t)s.lev[i];
    __syncthreads();
  }
}

// mode: 0 forward, 1 inverse, 2 pipeline
template <int L, int MODE>
static __global__ __launch_bounds__(64) void k_tu(const hvx_tu_desc *__restrict__ descs, const hvx_estbits *__restrict__ est,
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
    tu_inverse<L>(s, d);
    for (int i = lane_id(); i < NN; i += HVX_WAVE) res_out[off + i] = (int16_t)s.lev[i];
    return;
  }
  const hvx_estbits *e = est + (est_idx ? est_idx[t] : t);
  for (int i = lane_id(); i < NN; i += HVX_WAVE) s.a[i] = res_in[off + i];
  __syncthreads();
  const int32_t abs_sum = tu_forward<L>(s, d, e, arl_out ? arl_out + off : nullptr);
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    lev_io[off + i] = s.lev[i];
    if (temp_out) temp_out[off + i] = s.coef[i];
  }
  if (lane_id() == 0 && abs_out) abs_out[t] = abs_sum;
  if (MODE == 2) {
    __syncthreads();
    tu_inverse<L>(s, d);
    uint32_t part = 0;
    for (int i = lane_id(); i < NN; i += HVX_WAVE) {
      const int r = (int16_t)s.lev[i];
      res_out[off + i] = (int16_t)r;
      const int df = (int)res_in[off + i] - r;
      part += (uint32_t)(df * df);
    }
    const uint32_t sse = wave_sum_u32(part);
    if (lane_id() == 0 && sse_out) sse_out[t] = sse;
  }
}

// =======================================================================================
// Batched TU pipeline with lane-parallel RDOQ.
//
// The wave-uniform tu_rdoq above leaves 63 of 64 lanes idle and is bound by the SIMD's
// scalar issue rate (one SALU instruction per 4 cycles, shared by the SIMD's waves).  For
// batches, the serial xRateDistOptQuant instead runs ONE TU PER LANE: G TUs of a size class
// advance through their reverse scans together, so every VALU instruction serves G TUs.
// Three kernels per size class:
//   k_tu_fwd  (wave per TU)  transform + the non-RDOQ quantisers; for RDOQ TUs the
//                            coefficients go to an interleaved scan-order array
//   k_tu_rdoq (lane per TU)  rdoq_lane: decisions, last position, sign hiding
//   k_tu_fin  (wave per TU)  scan-order levels -> raster output, dequant + inverse + SSE
// Per-TU scratch arrays are interleaved so that the G lanes of a wave touch G consecutive
// words: element sp of TU t lives at ((t / G) * NN + sp) * G + t % G.
// =======================================================================================
__device__ __forceinline__ size_t tu_il(int t, int sp, int NN, int G) {
  return ((size_t)(t / G) * NN + sp) * G + (t % G);
}

// xRateDistOptQuant (:2129-2671) for one TU by one lane.  ldI/cxI/lev/st: the TU's
// interleaved arrays (element sp at [sp * G]), all in scan order:
//   ldI  lLevelDouble (:2210) | sign of the coefficient << 31       (k_tu_fwd)
//   cxI  significance context (getSigCtxInc :2717, + the chroma offset) under each of the 4
//        neighbour-group patterns, 6 bits per pattern               (k_tu_fwd)
//   lev  receives the signed final levels; st the packed context state of every decided
//        position (rd_pack), which the last-position and sign-hiding passes replay.
// Returns uiAbsSum.  Same operations, in the same order, as tu_rdoq and the reference; the
// decision pass is branch-free per position (selects on both candidate levels), keeps the
// group's greater-one / level-abs rate pairs in registers (the context set is fixed inside a
// group: xRateDistOptQuant resets c1/c2/Rice at every group start), and stages each group's 16
// inputs in the lane's LDS column while the next group's are in flight.
struct RdLaneStage {
  uint32_t ld[16][64], cx[16][64];
  int32_t lv[16][64], st[16][64];
};

// FAST: the wave's tables are in LDS and no TU of the wave uses extended precision (the
// limited-prefix escape code), so every table read is a ds_read and the rate has no branch.
// TM: ldI / cxI are TU-major (element sp at [sp], written coalesced by the wave-per-TU forward
// kernel); otherwise interleaved like lev / st.
template <int L, bool FAST, bool TM>
__device__ int32_t rdoq_lane(const hvx_tu_desc &d, const hvx_estbits *est, const uint32_t *ldI, const uint32_t *cxI,
                             int32_t *lev, int32_t *st, int G, RdLaneStage &sg, int lane) {
  constexpr int N = 4 << L, NN = N * N, NCG = NN / 16;
  constexpr int LOG2 = L + 2;
  const int ch = d.comp ? 1 : 0, comp = d.comp;
  const int ts = tu_transform_shift(d);
  const int qbits = 14 + d.qp_per + ts;
  const int qc = kQuantScales[d.qp_rem];
  const int ext = d.extended_precision, max_log2 = d.max_log2_tr_range;
  const int32_t ecmax = (1 << max_log2) - 1, ecmin = -(1 << max_log2);
  const int tsn = d.max_log2_tr_range - d.bit_depth - d.log2_size;
  double escale = (double)(1 << 15);
  escale = escale * ldexp(1.0, -2 * tsn);
  escale = escale / qc / qc / (1 << 0);
  const double lambda = d.lambda;
  const TuCoding c = tu_coding<L>(d);
  const size_t g16 = (size_t)16 * G;
  const size_t gi = TM ? 1 : (size_t)G, gi16 = 16 * gi;  // ldI / cxI stride
  const int32_t rnd = 1 << (qbits - 1);
  const int set0 = comp ? 4 : 0;
  const bool persistent = d.persistent_rice != 0;

  // ---- reverse-scan decisions ----
  const uint32_t rice0 = (uint32_t)d.golomb_rice_stat / 4;
  int last = -1, cg_last = -1;
  bool carry = false;  // c1 == 0 at the end of the previous group (decided lanes only)
  double block_uncoded = 0, base_cost = 0;
  uint64_t sigmask = 0;
  int32_t tot = 0;  // sum of the decided levels (after the group zero-outs)
  uint32_t nld[16], ncx[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    nld[k] = ldI[(NCG - 1) * gi16 + (size_t)k * gi];
    ncx[k] = cxI[(NCG - 1) * gi16 + (size_t)k * gi];
  }
  for (int cgp = NCG - 1; cgp >= 0; cgp--) {
#pragma unroll
    for (int k = 0; k < 16; k++) { sg.ld[k][lane] = nld[k]; sg.cx[k][lane] = ncx[k]; }
    if (cgp > 0) {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        nld[k] = ldI[(cgp - 1) * gi16 + (size_t)k * gi];
        ncx[k] = cxI[(cgp - 1) * gi16 + (size_t)k * gi];
      }
    }
    const int cgblk = c.scan_cg[cgp];
    const int cy = cgblk / c.wg, cx = cgblk - cy * c.wg;
    int pattern = 0;
    if (NCG > 1) {
      const int rr = cx < c.wg - 1 ? (int)((sigmask >> (cgblk + 1)) & 1) : 0;
      const int bb = cy < c.wg - 1 ? (int)((sigmask >> (cgblk + c.wg)) & 1) : 0;
      pattern = rr + (bb << 1);
    }
    const int psh = 6 * pattern;
    // the group's context set: a lane whose last position lies in this group starts it here
    // without the carry (:2262-2266), a decided lane carries c1 == 0 of the previous group
    const int ctx_set = set0 + ((comp == 0 && cgp > 0) ? 2 : 0) + ((last >= 0 && carry) ? 1 : 0);
    int G0[4], G1[4], A0[3], A1[3];
#pragma unroll
    for (int k = 0; k < 4; k++) { G0[k] = est->greaterOneBits[4 * ctx_set + k][0]; G1[k] = est->greaterOneBits[4 * ctx_set + k][1]; }
#pragma unroll
    for (int k = 0; k < 3; k++) { A0[k] = est->levelAbsBits[ctx_set + k][0]; A1[k] = est->levelAbsBits[ctx_set + k][1]; }
    int c1 = 1, c2 = 0;
    uint32_t c1_idx = 0, c2_idx = 0, rice = rice0;
    int nnz0 = 0, cgsum = 0;
    bool any = false;
    double coded_ld = 0, uncoded = 0, sig_cost = 0, sig_cost0 = 0;
#pragma unroll 2
    for (int pin = 15; pin >= 0; pin--) {
      const int sp = cgp * 16 + pin;
      const uint32_t w = sg.ld[pin][lane], cxw = sg.cx[pin][lane];
      const int32_t ld = (int32_t)(w & 0x7fffffffu);
      const uint32_t q = (uint32_t)((ld + rnd) >> qbits);
      const uint32_t max_abs = (uint32_t)ecmax < q ? (uint32_t)ecmax : q;
      const double e = (double)ld;
      const double cc0 = e * e * escale;
      block_uncoded += cc0;
      const bool found = max_abs > 0 && last < 0;
      last = found ? sp : last;
      cg_last = found ? cgp : cg_last;
      const bool act = last >= 0, is_last = sp == last;
      const int ctx_sig = is_last ? 0 : (int)((cxw >> psh) & 63u);
      const int sb0 = est->significantBits[ctx_sig][0], sb1 = est->significantBits[ctx_sig][1];
      const int g0 = c1 == 0 ? G0[0] : c1 == 1 ? G0[1] : c1 == 2 ? G0[2] : G0[3];
      const int g1 = c1 == 0 ? G1[0] : c1 == 1 ? G1[1] : c1 == 2 ? G1[2] : G1[3];
      const int a0 = c2 == 0 ? A0[0] : c2 == 1 ? A0[1] : A0[2];
      const int a1 = c2 == 0 ? A1[0] : c2 == 1 ? A1[1] : A1[2];
      const bool c1ok = c1_idx < 8, c2ok = c2_idx < 1;
      // xGetCodedLevel (:2822): level 0 (when allowed), then max, then max - 1
      const bool zero_ok = !is_last && max_abs < 3;
      const double sig0 = lambda * (double)sb0;
      double cost = zero_ok ? cc0 + sig0 : 1.7e+308;
      double cost_sig = zero_ok ? sig0 : 0.0;
      int sel = zero_ok ? 1 : 0;
      uint32_t best = 0;
      const double cur_sig = is_last ? 0.0 : lambda * (double)sb1;
      const int sel_nz = is_last ? 0 : 2;
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const uint32_t lv = max_abs - (uint32_t)k;
        const int r = (!FAST && ext) ? rd_ic_rate(lv, (int)rice, c1ok, c2ok, g0, g1, a0, a1, ext, max_log2)
                                     : rd_ic_rate_bf(lv, rice, c1ok, c2ok, g0, g1, a0, a1);
        const double err = (double)sub32(ld, shl32((int32_t)lv, qbits));
        double cl = err * err * escale + lambda * (double)r;
        cl += cur_sig;
        const bool take = max_abs >= (uint32_t)(k + 1) && cl < cost;
        best = take ? lv : best;
        cost = take ? cl : cost;
        cost_sig = take ? cur_sig : cost_sig;
        sel = take ? sel_nz : sel;
      }
      const uint32_t level = act ? best : 0u;
      const double cs = act ? cost_sig : 0.0;
      sg.st[pin][lane] = rd_pack(4 * ctx_set + c1, ctx_set + c2, (int)rice, c1ok, c2ok, !is_last, ctx_sig, sel);
      sg.lv[pin][lane] = (int32_t)level;
      cgsum += (int)level;
      base_cost += act ? cost : cc0;
      // context state after the level (:2300-2325): Rice parameter, c1Idx, c1/c2
      const uint32_t base = c1ok ? (c2ok ? 3u : 2u) : 1u;
      const bool rup = level >= base && level > (3u << rice);
      rice = rup ? (persistent ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4)) : rice;
      c1_idx += level >= 1 ? 1u : 0u;
      const bool gt1 = level > 1;
      c2_idx += gt1 ? 1u : 0u;
      c2 = gt1 ? c2 + (c2 < 2) : c2;
      c1 = gt1 ? 0 : ((c1 < 3 && c1 > 0 && level) ? c1 + 1 : c1);
      sig_cost += cs;
      if (pin == 0) sig_cost0 = cs;
      const bool nz = level != 0;
      any = any || nz;
      coded_ld = nz ? coded_ld + (cost - cs) : coded_ld;
      uncoded = nz ? uncoded + cc0 : uncoded;
      nnz0 += (nz && pin != 0) ? 1 : 0;
    }
    carry = c1 == 0;
    if (any) sigmask |= 1ull << cgblk;
    if (cg_last >= 0) {
      if (cgp) {
        const int rr = cx < c.wg - 1 ? (int)((sigmask >> (cgblk + 1)) & 1) : 0;
        const int bb = cy < c.wg - 1 ? (int)((sigmask >> (cgblk + c.wg)) & 1) : 0;
        const int ctx = (rr + bb) != 0;
        const int r0 = est->significantCoeffGroupBits[ctx][0], r1 = est->significantCoeffGroupBits[ctx][1];
        if (!any) {
          base_cost += lambda * (double)r0 - sig_cost;
        } else if (cgp < cg_last) {
          if (nnz0 == 0) { base_cost -= sig_cost0; sig_cost -= sig_cost0; }
          double zero_cost = base_cost;
          base_cost += lambda * (double)r1;
          zero_cost += lambda * (double)r0;
          zero_cost += uncoded;
          zero_cost -= coded_ld;
          zero_cost -= sig_cost;
          if (zero_cost < base_cost) {
            sigmask &= ~(1ull << cgblk);
            base_cost = zero_cost;
            cgsum = 0;
#pragma unroll
            for (int pin = 0; pin < 16; pin++) sg.lv[pin][lane] = 0;
          }
        }
      } else {
        sigmask |= 1ull << cgblk;
      }
    }
    tot += cgsum;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      lev[cgp * g16 + (size_t)k * G] = sg.lv[k][lane];
      st[cgp * g16 + (size_t)k * G] = sg.st[k][lane];
    }
  }
  if (last < 0) return 0;

  // ---- best last position ----
  double best_cost;
  int best_p1 = 0;
  if (!d.is_intra && ch == 0 && d.tr_idx == 0) {
    best_cost = block_uncoded + lambda * (double)est->blockRootCbpBits[0][0];
    base_cost += lambda * (double)est->blockRootCbpBits[0][1];
  } else {
    const int ctx = d.ctx_qt_cbf + (ch ? 5 : 0);
    best_cost = block_uncoded + lambda * (double)est->blockCbpBits[ctx][0];
    base_cost += lambda * (double)est->blockCbpBits[ctx][1];
  }
  bool found = false;
  int32_t above = 0, drop = 0;  // levels past the scanned position / past the best last one
  for (int cgp = cg_last; cgp >= 0 && !found; cgp--) {
    const int cgblk = c.scan_cg[cgp];
    // the coded-group flag rate the decision pass added for this group: 0 for the first
    // and the last coded group, else the flag's final value under the right/below context
    // (those neighbours were final before this group was decided)
    int cgrate = 0;
    if (cgp && cgp < cg_last) {
      const int cy = cgblk / c.wg, cx = cgblk - cy * c.wg;
      const int rr = cx < c.wg - 1 ? (int)((sigmask >> (cgblk + 1)) & 1) : 0;
      const int bb = cy < c.wg - 1 ? (int)((sigmask >> (cgblk + c.wg)) & 1) : 0;
      cgrate = est->significantCoeffGroupBits[(rr + bb) != 0][(sigmask >> cgblk) & 1];
    }
    base_cost -= lambda * (double)cgrate;
    if ((sigmask >> cgblk) & 1) {
      {
        int32_t a16[16], b16[16];
        uint32_t c16[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
          a16[k] = lev[cgp * g16 + (size_t)k * G];
          b16[k] = st[cgp * g16 + (size_t)k * G];
          c16[k] = ldI[cgp * gi16 + (size_t)k * gi];
        }
#pragma unroll
        for (int k = 0; k < 16; k++) { sg.lv[k][lane] = a16[k]; sg.st[k][lane] = b16[k]; sg.ld[k][lane] = c16[k]; }
      }
      for (int pin = 15; pin >= 0; pin--) {
        const int sp = cgp * 16 + pin;
        if (sp > last) continue;
        const int lvv = sg.lv[pin][lane];
        const RdCtx x = rd_unpack(sg.st[pin][lane]);
        const int sbr = x.sig_sel == 1 ? est->significantBits[x.ctx_sig][0]
                                       : x.sig_sel == 2 ? est->significantBits[x.ctx_sig][1] : 0;
        const double cs = x.sig_sel ? lambda * (double)sbr : 0.0;
        if (lvv) {
          const int blk = c.scan[sp];
          const int py = blk >> LOG2, px = blk - (py << LOG2);
          const double cl = c.scan_type == 2 ? rd_rate_last(est, lambda, py, px, ch) : rd_rate_last(est, lambda, px, py, ch);
          const double total = base_cost + cl - cs;
          if (total < best_cost) { best_p1 = sp + 1; best_cost = total; drop = above; }
          above += lvv;
          if (lvv > 1) { found = true; break; }
          const int32_t ld = (int32_t)(sg.ld[pin][lane] & 0x7fffffffu);
          const double err = (double)sub32(ld, shl32(1, qbits));
          const int g0 = est->greaterOneBits[x.ctx_one][0], g1 = est->greaterOneBits[x.ctx_one][1];
          const int a0 = est->levelAbsBits[x.ctx_abs][0], a1 = est->levelAbsBits[x.ctx_abs][1];
          const int rate = FAST ? rd_ic_rate_bf(1u, (uint32_t)x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1)
                                : rd_ic_rate(1u, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2);
          double cc = err * err * escale + lambda * (double)rate;
          cc += x.has_sig ? lambda * (double)est->significantBits[x.ctx_sig][1] : 0.0;
          base_cost -= cc;
          const double e = (double)ld;
          base_cost += e * e * escale;
        } else {
          base_cost -= cs;
        }
      }
    }
  }

  // uiAbsSum over the kept levels (:2530-2538)
  const int32_t abs_sum = best_p1 ? tot - drop : 0;

  // ---- signs, zeroing past the chosen last position, RD sign-bit hiding (:2541-2660) ----
  // one pass over the groups from the top: HM's sign loop and its SBH loop see each group with
  // the same final levels, and the groups above the last position are all zero
  const bool sbh = d.sign_hiding && abs_sum >= 2;
  const double iq = (double)kInvQuantScales[d.qp_rem];
  const int64_t rdf = sbh ? (int64_t)(iq * iq * (1 << (2 * d.qp_per)) / d.lambda / 16 / (1 << 0) + 0.5) : 0;
  int last_cg = -1;
  for (int sub = last >> 4; sub >= 0; sub--) {
    int32_t v[16];
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      v[k] = lev[sub * g16 + (size_t)k * G];
      w[k] = ldI[sub * gi16 + (size_t)k * gi];
    }
    uint32_t nzm = 0, negm = 0;
    int abs_in = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int32_t a = sub * 16 + k < best_p1 ? v[k] : 0;
      v[k] = (w[k] >> 31) ? -a : a;
      nzm |= (a != 0 ? 1u : 0u) << k;
      negm |= (w[k] >> 31) << k;
      abs_in += v[k];
    }
    if (sbh && nzm) {
      const int last_nz = 31 - __builtin_clz(nzm), first_nz = __builtin_ctz(nzm);
      if (last_cg == -1) last_cg = 1;
      const uint32_t signbit = (negm >> first_nz) & 1u;
      if (last_nz - first_nz >= 4 && signbit != (uint32_t)(abs_in & 1)) {
        {
          int32_t b16[16];
#pragma unroll
          for (int q = 0; q < 16; q++) b16[q] = st[sub * g16 + (size_t)q * G];
#pragma unroll
          for (int q = 0; q < 16; q++) { sg.lv[q][lane] = v[q]; sg.ld[q][lane] = w[q]; sg.st[q][lane] = b16[q]; }
        }
        int64_t min_inc = INT64_MAX, cur = INT64_MAX;
        int min_k = -1, fch = 0, cch = 0;
        for (int k = (last_cg == 1 ? last_nz : 15); k >= 0; k--) {
          const int32_t lv = sg.lv[k][lane];
          const uint32_t lev0 = (uint32_t)abs(lv);
          const uint32_t wk = sg.ld[k][lane];
          const int32_t ld = (int32_t)(wk & 0x7fffffffu);
          const int32_t du = sub32(ld, shl32((int32_t)lev0, qbits)) >> (qbits - 8);
          const RdCtx x = rd_unpack(sg.st[k][lane]);
          const int g0 = est->greaterOneBits[x.ctx_one][0];
          const int sigd = x.has_sig ? est->significantBits[x.ctx_sig][1] - est->significantBits[x.ctx_sig][0] : 0;
          int rup = g0, rdown = 0;
          if (lev0 > 0) {
            const int g1 = est->greaterOneBits[x.ctx_one][1];
            const int a0 = est->levelAbsBits[x.ctx_abs][0], a1 = est->levelAbsBits[x.ctx_abs][1];
            if (FAST) {  // no extended precision in the wave: the branch-free rate
              const uint32_t rc = (uint32_t)x.rice;
              const int now = rd_ic_rate_bf(lev0, rc, x.c1ok, x.c2ok, g0, g1, a0, a1);
              rup = rd_ic_rate_bf(lev0 + 1, rc, x.c1ok, x.c2ok, g0, g1, a0, a1) - now;
              rdown = rd_ic_rate_bf(lev0 - 1, rc, x.c1ok, x.c2ok, g0, g1, a0, a1) - now;
            } else {
              const int now = rd_ic_rate(lev0, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2);
              rup = rd_ic_rate(lev0 + 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
              rdown = rd_ic_rate(lev0 - 1, x.rice, x.c1ok, x.c2ok, g0, g1, a0, a1, ext, max_log2) - now;
            }
          }
          if (lv != 0) {
            const int64_t up = rdf * (-du) + rup;
            int64_t down = rdf * (du) + rdown - ((abs(lv) == 1) ? sigd : 0);
            if (last_cg == 1 && last_nz == k && abs(lv) == 1) down -= (4 << 15);
            if (up < down) { cur = up; cch = 1; }
            else { cch = -1; cur = (k == first_nz && abs(lv) == 1) ? INT64_MAX : down; }
          } else {
            cur = rdf * (-(abs(du))) + (1 << 15) + rup + sigd;
            cch = 1;
            if (k < first_nz) {
              const uint32_t tsb = wk >> 31;
              if (tsb != signbit) cur = INT64_MAX;
            }
          }
          if (cur < min_inc) { min_inc = cur; fch = cch; min_k = k; }
        }
        int32_t mv = sg.lv[min_k][lane];
        if (mv == ecmax || mv == ecmin) fch = -1;
        if (!(sg.ld[min_k][lane] >> 31)) mv += fch;
        else mv -= fch;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = k == min_k ? mv : v[k];
      }
      if (last_cg == 1) last_cg = 0;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) lev[sub * g16 + (size_t)k * G] = v[k];
  }
  return abs_sum;
}

// transformNxN up to (not including) RDOQ, wave per TU.  RDOQ TUs: per scan position the
// state-independent inputs of the lane-parallel RDOQ (lLevelDouble | sign -> ldI, the
// significance context under each neighbour pattern -> cxI), flag 1.  Others (bypass, plain quant, RDOQ not needed): final levels in
// scan order -> levI, uiAbsSum -> abs_out, flag 0.
template <int L>
static __global__ __launch_bounds__(64) void k_tu_fwd(const hvx_tu_desc *__restrict__ descs, const int64_t *__restrict__ offs,
                                               int n, const int16_t *__restrict__ res_in, int32_t *__restrict__ temp_out,
                                               int32_t *__restrict__ arl_out, uint32_t *__restrict__ ldI,
                                               uint32_t *__restrict__ cxI, int32_t *__restrict__ levI,
                                               int32_t *__restrict__ abs_out, int8_t *__restrict__ flags, int G,
                                               int tm) {
  constexpr int N = 4 << L, NN = N * N;
  __shared__ TuSmem<L> s;
  const int t = blockIdx.x;
  if (t >= n) return;
  const hvx_tu_desc d = descs[t];
  if (d.width != N || d.height != N) return;
  const int64_t off = offs[t];
  const int lane = lane_id();
  const TuCoding c = tu_coding<L>(d);
  if constexpr (L >= 2) {
    // the CTU pass's 16x16 / 32x32 TUs (8-bit, RDOQ): the 16-bit transform, coefficients transposed
    if (!temp_out && !arl_out && d.bit_depth == 8 && d.max_log2_tr_range == 15 && !d.transquant_bypass &&
        !d.transform_skip && !d.extended_precision && d.use_rdoq && !d.selective_rdoq) {
      constexpr int LOG2 = L + 2;
      int16_t *aH = reinterpret_cast<int16_t *>(s.a);
      const uint32_t *src = reinterpret_cast<const uint32_t *>(res_in + off);
      for (int i = lane; i < NN / 2; i += HVX_WAVE) reinterpret_cast<uint32_t *>(aH)[i] = src[i];
      __syncthreads();
      tu_forward_dot2<L>(aH, reinterpret_cast<int16_t *>(s.lev), s.coef);
      const int qbits = 14 + d.qp_per + tu_transform_shift(d);
      const int qc = kQuantScales[d.qp_rem];
      const int64_t lim = (int64_t)2147483647 - ((int64_t)1 << (qbits - 1));
      const int ch = d.comp ? 1 : 0, sig_off = ch ? 28 : 0;
      for (int sp = lane; sp < NN; sp += HVX_WAVE) {
        const int blk = c.scan[sp];
        const int32_t cf = s.coef[(blk & (N - 1)) * N + (blk >> LOG2)];
        const int32_t ld = rd_level_double(cf, qc, lim);
        const size_t il = tm ? (size_t)t * NN + sp : tu_il(t, sp, NN, G);
        ldI[il] = (uint32_t)ld | (cf < 0 ? 0x80000000u : 0u);
        uint32_t cx = 0;
#pragma unroll
        for (int p = 0; p < 4; p++) cx |= (uint32_t)(sig_off + rd_sig_ctx<L>(p, c, sp, ch)) << (6 * p);
        cxI[il] = cx;
      }
      if (lane == 0) flags[t] = 1;
      return;
    }
  }
  for (int i = lane; i < NN; i += HVX_WAVE) s.a[i] = res_in[off + i];
  __syncthreads();
  int32_t *arl = arl_out ? arl_out + off : nullptr;
  bool rdoq = false;
  int32_t abs_sum = 0;
  if (d.transquant_bypass) {
    int part = 0;
    for (int i = lane; i < NN; i += HVX_WAVE) { s.lev[i] = s.a[i]; s.coef[i] = s.a[i]; part += abs(s.a[i]); }
    abs_sum = wave_sum_i32(part);
    __syncthreads();
  } else {
    if (d.transform_skip) {
      const int ts = tu_transform_shift(d);
      for (int i = lane; i < NN; i += HVX_WAVE) {
        const int32_t v = s.a[i];
        s.coef[i] = ts >= 0 ? shl32(v, ts) : (v + (1 << (-ts - 1))) >> -ts;
      }
      __syncthreads();
    } else {
      tu_forward_transform<L>(s, d.use_dst && N == 4);
    }
    const int use_rdoq = d.transform_skip ? d.use_rdoq_ts : d.use_rdoq;
    const int ts = tu_transform_shift(d);
    const int qbits = 14 + d.qp_per + ts;
    const int qc = kQuantScales[d.qp_rem];
    if (use_rdoq) {
      bool need = true;
      if (d.selective_rdoq) {  // xNeedRDOQ (:1257)
        const int add = (d.comp == 0 ? 171 : 256) << (qbits - 9);
        int any = 0;
        for (int i = lane; i < NN; i += HVX_WAVE) any |= ((int32_t)(((int64_t)abs(s.coef[i]) * qc + add) >> qbits)) != 0;
        need = wave_sum_i32(any) != 0;
      }
      if (need) {
        rdoq = true;
        const int64_t lim = (int64_t)2147483647 - ((int64_t)1 << (qbits - 1));
        const int qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
        const int ch = d.comp ? 1 : 0, sig_off = ch ? 28 : 0;
        for (int sp = lane; sp < NN; sp += HVX_WAVE) {
          const int blk = c.scan[sp];
          const int32_t cf = s.coef[blk];
          const int32_t ld = rd_level_double(cf, qc, lim);
          const size_t il = tm ? (size_t)t * NN + sp : tu_il(t, sp, NN, G);
          ldI[il] = (uint32_t)ld | (cf < 0 ? 0x80000000u : 0u);
          uint32_t cx = 0;
#pragma unroll
          for (int p = 0; p < 4; p++) cx |= (uint32_t)(sig_off + rd_sig_ctx<L>(p, c, sp, ch)) << (6 * p);
          cxI[il] = cx;
          if (arl) arl[blk] = d.adaptive_qp_select ? (ld + add_c) >> qbits_c : 0;
        }
      } else {
        for (int i = lane; i < NN; i += HVX_WAVE) {
          s.lev[i] = 0;
          if (arl) arl[i] = 0;
        }
        __syncthreads();
      }
    } else {
      abs_sum = tu_quant_plain<L>(s, d, arl);
    }
  }
  if (temp_out)
    for (int i = lane; i < NN; i += HVX_WAVE) temp_out[off + i] = s.coef[i];
  if (!rdoq) {
    for (int sp = lane; sp < NN; sp += HVX_WAVE) levI[tu_il(t, sp, NN, G)] = s.lev[c.scan[sp]];
    if (lane == 0 && abs_out) abs_out[t] = abs_sum;
  }
  if (lane == 0) flags[t] = rdoq ? 1 : 0;
}

// xRateDistOptQuant, one TU per lane: wave w handles TUs w*G .. w*G+G-1 of the launch.
// n_est_lds > 0: the launch's TUs index the first n_est_lds tables of `est` (est_idx); the
// (at most two consecutive) tables the wave's TUs use are staged in LDS -- a class launch of the
// CTU pass uses one -- so the wave's LDS stays at the lane stage + 2 tables (8 waves per CU).
// Otherwise each lane reads its own table from global memory.
template <int L>
static __global__ __launch_bounds__(64) void k_tu_rdoq(const hvx_tu_desc *__restrict__ descs, const hvx_estbits *__restrict__ est,
                                                const int32_t *__restrict__ est_idx, int n,
                                                const uint32_t *__restrict__ ldI, const uint32_t *__restrict__ cxI,
                                                int32_t *__restrict__ levI, int32_t *__restrict__ stI,
                                                int32_t *__restrict__ abs_out, const int8_t *__restrict__ flags, int G,
                                                int n_est_lds, int tm) {
  constexpr int N = 4 << L, NN = N * N;
  __shared__ hvx_estbits tbl[2];
  __shared__ RdLaneStage stage;
  const int lane = lane_id();
  const int t = blockIdx.x * G + lane;
  const bool live = lane < G && t < n;
  int e0 = 0;
  bool staged = false;
  if (n_est_lds > 0) {
    const int my = live ? (est_idx ? est_idx[t] : t) : -1;
    int lo = live ? my : INT_MAX, hi = my;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, HVX_WAVE));
      hi = max(hi, __shfl_xor(hi, o, HVX_WAVE));
    }
    lo = __builtin_amdgcn_readfirstlane(lo); hi = __builtin_amdgcn_readfirstlane(hi);
    if (hi >= 0 && lo >= 0 && hi - lo <= 1 && hi < n_est_lds) {
      const int32_t *src = (const int32_t *)(est + lo);
      int32_t *dst = (int32_t *)tbl;
      const int words = (hi - lo + 1) * (int)(sizeof(hvx_estbits) / 4);
      for (int i = lane; i < words; i += HVX_WAVE) dst[i] = src[i];
      __syncthreads();
      e0 = lo; staged = true;
    }
  }
  if (!live) return;
  if (!flags[t]) return;
  const hvx_tu_desc d = descs[t];
  if (d.width != N || d.height != N) return;
  const int ei = est_idx ? est_idx[t] : t;
  const hvx_estbits *e = staged ? &tbl[ei - e0] : est + ei;
  const size_t base = tu_il(t, 0, NN, G);
  const bool any_ext = __builtin_amdgcn_ballot_w64(d.extended_precision != 0) != 0;
  int32_t a;
  if (tm) {  // TU-major inputs (the CTU pass's 16x16 / 32x32 classes)
    if (staged && !any_ext)
      a = rdoq_lane<L, true, true>(d, e, ldI + (size_t)t * NN, cxI + (size_t)t * NN, levI + base, stI + base, G, stage, lane);
    else
      a = rdoq_lane<L, false, true>(d, e, ldI + (size_t)t * NN, cxI + (size_t)t * NN, levI + base, stI + base, G, stage, lane);
  } else if (staged && !any_ext) {
    a = rdoq_lane<L, true, false>(d, e, ldI + base, cxI + base, levI + base, stI + base, G, stage, lane);
  } else {
    a = rdoq_lane<L, false, false>(d, e, ldI + base, cxI + base, levI + base, stI + base, G, stage, lane);
  }
  if (abs_out) abs_out[t] = a;
}

// Levels (scan order, interleaved) -> raster lev_io; MODE 2 also dequant + inverse + SSE.  With
// zd_out: the zero-residual distortion sum(res_in^2); with pred (8-bit, residual layout) and
// csse_out: the distortion of the clipped reconstruction, sum((pred + res_in - clip(pred + r))^2)
// (TComYuv::addClip + getDistPart over the TU).
// tu_inverse for the CTU pass's 16x16 / 32x32 TUs (8-bit, 15-bit range, transform, no bypass):
// dequantised coefficients transposed as int16, the 16-bit inverse transform; s.lev ends with
// the reconstructed residual (raster) exactly as tu_inverse leaves it
template <int L>
__device__ void tu_inverse_fast(TuSmem<L> &s, const hvx_tu_desc &d) {
  constexpr int N = 4 << L, NN = N * N, LOG2 = L + 2, P = tu_p16<N>();
  const int ts = tu_transform_shift(d);
  const int right = 6 - (ts + d.qp_per);
  const int scale = kInvQuantScales[d.qp_rem];
  int tib = 32 + right - 7;
  if (16 < tib) tib = 16;
  const int32_t imin = -(1 << (tib - 1)), imax = (1 << (tib - 1)) - 1;
  int16_t *deqT = reinterpret_cast<int16_t *>(s.a);
  for (int i = lane_id(); i < NN; i += HVX_WAVE) {
    const int32_t c = clip3(imin, imax, s.lev[i]);
    const int32_t v = right > 0 ? (c * scale + (1 << (right - 1))) >> right : shl32(c * scale, -right);
    deqT[(i & (N - 1)) * P + (i >> LOG2)] = (int16_t)clip3(-32768, 32767, v);
  }
  __syncthreads();
  tu_inverse_dot2<L>(deqT, reinterpret_cast<int16_t *>(s.coef), s.lev);
}

template <int L, int MODE>
static __global__ __launch_bounds__(64) void k_tu_fin(const hvx_tu_desc *__restrict__ descs, const int64_t *__restrict__ offs,
                                               int n, const int16_t *__restrict__ res_in,
                                               const int32_t *__restrict__ levI, int32_t *__restrict__ lev_io,
                                               int16_t *__restrict__ res_out, uint32_t *__restrict__ sse_out, int G,
                                               const uint8_t *__restrict__ pred, uint32_t *__restrict__ zd_out,
                                               uint32_t *__restrict__ csse_out) {
  constexpr int N = 4 << L, NN = N * N;
  __shared__ TuSmem<L> s;
  const int t = blockIdx.x;
  if (t >= n) return;
  const hvx_tu_desc d = descs[t];
  if (d.width != N || d.height != N) return;
  const int64_t off = offs[t];
  const int lane = lane_id();
  const TuCoding c = tu_coding<L>(d);
  for (int sp = lane; sp < NN; sp += HVX_WAVE) s.lev[c.scan[sp]] = levI[tu_il(t, sp, NN, G)];
  __syncthreads();
  for (int i = lane; i < NN; i += HVX_WAVE) lev_io[off + i] = s.lev[i];
  if (MODE == 2) {
    __syncthreads();
    bool fast = false;
    if constexpr (L >= 2)
      fast = d.bit_depth == 8 && d.max_log2_tr_range == 15 && !d.transquant_bypass && !d.transform_skip &&
             !d.extended_precision;
    if constexpr (L >= 2) {
      if (fast) tu_inverse_fast<L>(s, d);
      else tu_inverse<L>(s, d);
    } else {
      tu_inverse<L>(s, d);
    }
    uint32_t part = 0, pz = 0, pc = 0;
    for (int i = lane; i < NN; i += HVX_WAVE) {
      const int r = (int16_t)s.lev[i];
      res_out[off + i] = (int16_t)r;
      const int ri = res_in[off + i];
      const int df = ri - r;
      part += (uint32_t)(df * df);
      pz += (uint32_t)(ri * ri);
      if (pred) {
        const int p = pred[off + i], v = p + r, c = ri + p - (v < 0 ? 0 : v > 255 ? 255 : v);
        pc += (uint32_t)(c * c);
      }
    }
    const uint32_t sse = wave_sum_u32(part);
    if (lane == 0 && sse_out) sse_out[t] = sse;
    if (zd_out) {
      const uint32_t z = wave_sum_u32(pz);
      if (lane == 0) zd_out[t] = z;
    }
    if (pred && csse_out) {
      const uint32_t c = wave_sum_u32(pc);
      if (lane == 0) csse_out[t] = c;
    }
  }
}
