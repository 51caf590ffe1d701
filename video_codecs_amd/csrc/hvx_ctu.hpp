// hvx_ctu.hpp -- the CTU analysis pass on the device (the bench workload; hvx_types.h,
// DESIGN.md).  All CTUs of a picture are independent here (no neighbour-dependent
// predictors), so the pass is a fixed sequence of wide launches:
//   for depth 0..3: k_ctu_me_jobs (one thread per CU x reference) -> k_me
//   k_ctu_pred_resid<S> (one wave per CU: best reference, separable luma/chroma MC over LDS, residual, TU descriptors)
//   k_tu<L,pipeline> per TU size class over contiguous class ranges
//   k_ctu_finalize (per-CU sums)
// The composition is restated on the CPU by hvxo_ctu_analyze (oracle/hvx_oracle.c).
#pragma once
#include "hvx_dev.hpp"
#include "hvx_me.hpp"

struct CtuLayout {
  int nctu_x, nctu_y, nctu, nref;
  // TU classes, contiguous: luma [0,8n) 32x32 | [8n,24n) 16x16 | [24n,88n) 8x8, then (4:2:0) chroma
  // [88n,104n) 16x16 (the 64x64 and 32x32 CUs) | [104n,136n) 8x8 | [136n,264n) 4x4 | [264n,392n) the
  // transform-skip twins of the 4x4 TUs (same residual, transform_skip = 1)
  __host__ __device__ int ntu() const { return 392 * nctu; }
  __host__ __device__ int64_t nres() const { return (int64_t)26624 * nctu; }
};

// the chroma planes of a 4:2:0 pass (hvx_chroma_planes on the device side); on == 0: luma only
struct CtuChroma {
  const uint8_t *cur[2];
  const uint8_t *const *refs;  // 2 * nref origins: Cb of each reference, then Cr
  uint8_t *recon[2];
  int stride, on;
};

__device__ __forceinline__ void cu_geom(int ci, int &d, int &j, int &S, int &g) {
  if (ci == 0) { d = 0; j = 0; }
  else if (ci < 5) { d = 1; j = ci - 1; }
  else if (ci < 21) { d = 2; j = ci - 5; }
  else { d = 3; j = ci - 21; }
  S = 64 >> d;
  g = 1 << d;
}

__device__ __forceinline__ int depth_base(int d) { return d == 0 ? 0 : d == 1 ? 1 : d == 2 ? 5 : 21; }

// TU index and residual offset of TU t of component c (0 Y, 1 Cb, 2 Cr) of CU (ctu, d, j)
__device__ __forceinline__ int ctu_tu_index(const CtuLayout &L, int ctu, int d, int j, int t, int c = 0) {
  const int n = L.nctu;
  if (c == 0) {
    if (d == 0) return ctu * 8 + t;
    if (d == 1) return ctu * 8 + 4 + j;
    if (d == 2) return 8 * n + ctu * 16 + j;
    return 24 * n + ctu * 64 + j;
  }
  if (d == 0) return 88 * n + ctu * 16 + (c - 1) * 4 + t;
  if (d == 1) return 88 * n + ctu * 16 + 8 + (c - 1) * 4 + j;
  if (d == 2) return 104 * n + ctu * 32 + (c - 1) * 16 + j;
  return 136 * n + ctu * 128 + (c - 1) * 64 + j;
}
__device__ __forceinline__ int64_t ctu_tu_offset(const CtuLayout &L, int tu) {
  const int64_t n = L.nctu;
  if (tu < 8 * n) return (int64_t)tu * 1024;
  if (tu < 24 * n) return 8 * n * 1024 + (int64_t)(tu - 8 * n) * 256;
  if (tu < 88 * n) return 8 * n * 1024 + 16 * n * 256 + (int64_t)(tu - 24 * n) * 64;
  const int64_t c0 = 16384 * n;
  if (tu < 104 * n) return c0 + (int64_t)(tu - 88 * n) * 256;
  if (tu < 136 * n) return c0 + 4096 * n + (int64_t)(tu - 104 * n) * 64;
  return c0 + 6144 * n + (int64_t)(tu - 136 * n) * 16;  // the 4x4 TUs and their twins
}
// the transform-skip twin of a 4x4 chroma TU
__device__ __forceinline__ int ctu_tu_ts(const CtuLayout &L, int tu) { return tu + 128 * L.nctu; }

// xPredInterBlk for one 4:2:0 chroma sample, uni-prediction (hvxo_chroma_block_epel): the luma
// quarter-pel MV in 1/8 chroma samples, 4-tap filters, first (+ last) stage(s) of
// TComInterpolationFilter (8-bit: the single stage rounds by 32 >> 6, the two-stage path keeps
// the -8192-offset int16 intermediate, TComInterpolationFilter.cpp:94-257)
__device__ __forceinline__ int ctu_epel_sample(const uint8_t *ref, int sr, int x, int y, int mvx, int mvy) {
  const int fx = mvx & 7, fy = mvy & 7;
  const uint8_t *p = ref + (y + (mvy >> 3)) * sr + x + (mvx >> 3);
  if (!fx && !fy) return p[0];
  if (!fy) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) s += kChromaFilter[fx][k] * p[k - 1];
    return clip_pel((s + 32) >> 6);
  }
  if (!fx) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) s += kChromaFilter[fy][k] * p[(k - 1) * sr];
    return clip_pel((s + 32) >> 6);
  }
  int s2 = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) s += kChromaFilter[fx][k] * p[(t - 1) * sr + k - 1];
    s2 += kChromaFilter[fy][t] * (int16_t)(s - 8192);
  }
  return clip_pel((s2 + (1 << 11) + (8192 << 6)) >> 12);
}

static __global__ void k_set_ptr(const uint8_t **slot, const uint8_t *p) { *slot = p; }

// one thread per (ctu, cu of this depth, ref)
static __global__ __launch_bounds__(256) void k_ctu_me_jobs(CtuLayout L, hvx_ctu_params P, int depth,
                                                     const hvx_me_result *__restrict__ res, hvx_me_job *__restrict__ jobs) {
  const int g = 1 << depth, ncu = g * g;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L.nctu * ncu * L.nref) return;
  const int ref = t % L.nref, j = (t / L.nref) % ncu, ctu = t / (L.nref * ncu);
  const int S = 64 >> depth, cy = j / g, cx = j % g;
  const int x = (ctu % L.nctu_x) * 64 + cx * S, y = (ctu / L.nctu_x) * 64 + cy * S;
  const int ci = depth_base(depth) + j;
  hvx_me_job jb;
  jb.pic_w = P.pic_w; jb.pic_h = P.pic_h; jb.max_cu = 64;
  jb.cu_x = jb.pu_x = x; jb.cu_y = jb.pu_y = y;
  const bool valid = x + S <= P.pic_w && y + S <= P.pic_h;
  jb.w = jb.h = valid ? S : 0;
  jb.pred_x = jb.pred_y = 0;
  jb.use_int2nx2n = 0; jb.i2_x = jb.i2_y = 0;
  if (depth > 0) {
    const int pg = g >> 1, pj = (cy >> 1) * pg + (cx >> 1);
    const int pS = S * 2, px = (ctu % L.nctu_x) * 64 + (cx >> 1) * pS, py = (ctu / L.nctu_x) * 64 + (cy >> 1) * pS;
    if (px + pS <= P.pic_w && py + pS <= P.pic_h) {
      const hvx_me_result &pr = res[((size_t)ctu * HVX_CUS_PER_CTU + depth_base(depth - 1) + pj) * L.nref + ref];
      jb.use_int2nx2n = 1; jb.i2_x = pr.mv_int_x; jb.i2_y = pr.mv_int_y;
    }
  }
  jb.bits_in = 0;
  jb.search_range = P.search_range;
  jb.lambda_motion = P.lambda_motion;
  jb.flags = P.me_flags;
  jb.ref_idx = ref; jb.cur_idx = 0; jb.center_x = jb.center_y = 0; jb.pad_ = 0;
  jobs[((size_t)ctu * HVX_CUS_PER_CTU + ci) * L.nref + ref] = jb;
}

// one wave per CU of size S: best reference, luma MC (standard two-stage quarter-pel), residual
// into the TU-class layout, TU descriptors (hvxo_ctu_tu_desc semantics).  The MC is separable
// over LDS: the (S+7)^2 reference window is staged once, the first (horizontal) stage is
// computed once per row of the window, the second stage reads it (the same int16 intermediate,
// -8192 offset, as TComInterpolationFilter's two-stage path, .cpp:94-257); chroma likewise with
// the 4-tap filters.  Descriptors are built one per lane and stored as 16-byte vectors.
// what the residual pass reads and writes
struct CtuMc {
  CtuLayout L;
  hvx_ctu_params P;
  const uint8_t *cur;
  const uint8_t *const *refs;
  int stride;
  const hvx_me_result *res;
  int16_t *resid;
  uint8_t *pred_out;
  hvx_tu_desc *descs;
  int64_t *offs;
  int32_t *est_idx;
  hvx_cu_result *out;
  CtuChroma C;
};

// TU descriptor `kind` (0 luma, 1 Cb, 2 Cr, 3 / 4 the Cb / Cr transform-skip twins at depth 3)
// of luma TU position t of CU (ctu, j) of size S (hvxo_ctu_tu_desc semantics), stored as 16-byte
// vectors, with the TU's residual offset and estBits table index
template <int S>
__device__ __forceinline__ void ctu_desc(const CtuMc &M, int ctu, int j, bool valid, int t, int kind) {
  const CtuLayout &L = M.L;
  const hvx_ctu_params &P = M.P;
  hvx_tu_desc *__restrict__ descs = M.descs;
  int64_t *__restrict__ offs = M.offs;
  int32_t *__restrict__ est_idx = M.est_idx;
  constexpr int d = S == 64 ? 0 : S == 32 ? 1 : S == 16 ? 2 : 3;
  constexpr int T = S < 32 ? S : 32, log2 = T == 8 ? 3 : T == 16 ? 4 : 5, Tc = T / 2;
  const int c = kind == 0 ? 0 : 1 + (kind - 1) % 2;
  hvx_tu_desc td;
  memset(&td, 0, sizeof(td));
  td.slice_type = P.slice_type;
  td.sign_hiding = 1; td.use_rdoq = 1; td.use_rdoq_ts = 1;
  td.pps_tskip = 1;  // TransformSkip=1: 4x4 TUs code transform_skip_flag
  td.max_log2_tr_range = 15; td.bit_depth = 8;
  td.tr_idx = S > 32 ? 1 : 0;
  int tu, ei;
  if (c == 0) {
    tu = ctu_tu_index(L, ctu, d, j, t);
    td.width = td.height = valid ? T : 0;  // width 0: no size class picks it up
    td.log2_size = log2;
    td.qp_per = P.qp / 6; td.qp_rem = P.qp % 6;
    td.lambda = P.lambda;
    ei = log2 - 2;
  } else {  // half size, chroma QP and RDOQ lambda, chroma cbf context = transform depth
    tu = ctu_tu_index(L, ctu, d, j, t, c);
    td.comp = c;
    td.width = td.height = valid ? Tc : 0;
    td.log2_size = log2 - 1;
    td.ctx_qt_cbf = S > 32 ? 1 : 0;
    td.qp_per = P.qp_chroma / 6; td.qp_rem = P.qp_chroma % 6;
    td.lambda = P.lambda_chroma;
    ei = 4 + log2 - 3;
    if (kind >= 3) { tu = ctu_tu_ts(L, tu); td.transform_skip = 1; ei = 4; }
  }
  static_assert(sizeof(hvx_tu_desc) % 16 == 0, "descriptor stored as 16-byte vectors");
  const uint4 *src = reinterpret_cast<const uint4 *>(&td);
  uint4 *dst = reinterpret_cast<uint4 *>(descs + tu);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(hvx_tu_desc) / 16); q++) dst[q] = src[q];
  offs[tu] = ctu_tu_offset(L, tu);
  est_idx[tu] = ei;
}

// one CU of size S: the body of k_ctu_pred_resid<S> (win / hs: its LDS)
template <int S>
__device__ void ctu_pred_resid_cu(const CtuMc &M, int ctu, int j, uint8_t *win, int16_t *hs) {
  const CtuLayout &L = M.L;
  const hvx_ctu_params &P = M.P;
  const uint8_t *__restrict__ cur = M.cur;
  const uint8_t *const *__restrict__ refs = M.refs;
  const int stride = M.stride;
  int16_t *__restrict__ resid = M.resid;
  uint8_t *__restrict__ pred_out = M.pred_out;
  hvx_tu_desc *__restrict__ descs = M.descs;
  int64_t *__restrict__ offs = M.offs;
  int32_t *__restrict__ est_idx = M.est_idx;
  const CtuChroma &C = M.C;
  constexpr int d = S == 64 ? 0 : S == 32 ? 1 : S == 16 ? 2 : 3, g = 1 << d;
  constexpr int T = S < 32 ? S : 32, log2 = T == 8 ? 3 : T == 16 ? 4 : 5, ntu = (S / T) * (S / T);
  constexpr int WP = S + 8, WR = S + 7;                    // luma window pitch / rows
  constexpr int Sc = S / 2, Tc = T / 2, CWP = Sc + 4, CWR = Sc + 3;
  static_assert(2 * CWR * CWP <= WR * WP && 2 * CWR * Sc <= WR * S, "chroma windows fit the luma buffers");
  const int lane = lane_id();
  const int cuid = ctu * HVX_CUS_PER_CTU + depth_base(d) + j;
  const int x = (ctu % L.nctu_x) * 64 + (j % g) * S, y = (ctu / L.nctu_x) * 64 + (j / g) * S;
  const bool valid = x + S <= P.pic_w && y + S <= P.pic_h;
  int best = 0;
  uint32_t best_cost = 0;
  const hvx_me_result *r = M.res + (size_t)cuid * L.nref;
  if (valid) {
    for (int k = 0; k < L.nref; k++) {
      const uint32_t ck = r[k].cost;
      if (k == 0 || ck < best_cost) { best_cost = ck; best = k; }
    }
  }
  const int mvx = valid ? r[best].mv_x : 0, mvy = valid ? r[best].mv_y : 0;
  if (lane == 0) {
    hvx_cu_result o;
    o.valid = valid; o.ref = valid ? best : 0;
    o.mv_x = mvx; o.mv_y = mvy;
    o.me_cost = valid ? best_cost : 0; o.sse = 0; o.abs_sum = 0; o.n_tu = valid ? ntu : 0;
    M.out[cuid] = o;
  }
  // descriptors: per luma TU position the luma TU, then (4:2:0) Cb, Cr and, at depth 3, the
  // transform-skip twins of the 4x4 Cb / Cr TUs (xEstimateInterResidualQT's second mode)
  const int nper = C.on ? (d == 3 ? 5 : 3) : 1;
  for (int k = lane; k < ntu * nper; k += HVX_WAVE) ctu_desc<S>(M, ctu, j, valid, k / nper, k % nper);
  if (!valid) return;
  {  // luma
    const int fx = mvx & 3, fy = mvy & 3;
    const uint8_t *rp = refs[best] + (y + (mvy >> 2) - 3) * stride + x + (mvx >> 2) - 3;
    for (int k = lane; k < WR * WR; k += HVX_WAVE) {
      const int rr = k / WR, cc = k % WR;
      win[rr * WP + cc] = rp[rr * stride + cc];
    }
    __syncthreads();
    if (fx) {
      const int r0 = fy ? 0 : 3, nr = fy ? WR : S;
      for (int k = lane; k < nr * S; k += HVX_WAVE) {
        const int rr = r0 + k / S, cc = k % S;
        int s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) s += kLumaFilter[fx][i] * win[rr * WP + cc + i];
        hs[rr * S + cc] = (int16_t)(s - 8192);
      }
      __syncthreads();
    }
    for (int k = lane; k < S * S; k += HVX_WAVE) {
      const int yy = k / S, xx = k % S;
      int pred;
      if (!fy) {
        pred = fx ? clip_pel((hs[(yy + 3) * S + xx] + 8192 + 32) >> 6) : win[(yy + 3) * WP + xx + 3];
      } else if (!fx) {
        int s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) s += kLumaFilter[fy][i] * win[(yy + i) * WP + xx + 3];
        pred = clip_pel((s + 32) >> 6);
      } else {
        int s = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) s += kLumaFilter[fy][i] * hs[(yy + i) * S + xx];
        pred = clip_pel((s + (1 << 11) + (8192 << 6)) >> 12);
      }
      const int t = (yy / T) * (S / T) + (xx / T);
      const int tu = ctu_tu_index(L, ctu, d, j, t);
      const int64_t o = ctu_tu_offset(L, tu) + (yy % T) * T + (xx % T);
      resid[o] = (int16_t)((int)cur[(y + yy) * stride + x + xx] - pred);
      pred_out[o] = (uint8_t)pred;
    }
  }
  if (!C.on) return;
  __syncthreads();  // the luma stages are done with win / hs
  {  // Cb and Cr together: window c at win + (c-1)*CWR*CWP, first stage at hs + (c-1)*CWR*Sc
    const int fx = mvx & 7, fy = mvy & 7, xc = x / 2, yc = y / 2;
    const int wo = (yc + (mvy >> 3) - 1) * C.stride + xc + (mvx >> 3) - 1;
    for (int k = lane; k < 2 * CWR * CWR; k += HVX_WAVE) {
      const int c = k / (CWR * CWR), kk = k % (CWR * CWR), rr = kk / CWR, cc = kk % CWR;
      win[c * CWR * CWP + rr * CWP + cc] = C.refs[c * L.nref + best][wo + rr * C.stride + cc];
    }
    __syncthreads();
    if (fx) {
      const int r0 = fy ? 0 : 1, nr = fy ? CWR : Sc;
      for (int k = lane; k < 2 * nr * Sc; k += HVX_WAVE) {
        const int c = k / (nr * Sc), kk = k % (nr * Sc), rr = r0 + kk / Sc, cc = kk % Sc;
        const uint8_t *w = win + c * CWR * CWP + rr * CWP + cc;
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) s += kChromaFilter[fx][i] * w[i];
        hs[c * CWR * Sc + rr * Sc + cc] = (int16_t)(s - 8192);
      }
      __syncthreads();
    }
    for (int k = lane; k < 2 * Sc * Sc; k += HVX_WAVE) {
      const int c = k / (Sc * Sc), kk = k % (Sc * Sc), yy = kk / Sc, xx = kk % Sc;
      const uint8_t *w = win + c * CWR * CWP;
      const int16_t *h = hs + c * CWR * Sc;
      int pred;
      if (!fy) {
        pred = fx ? clip_pel((h[(yy + 1) * Sc + xx] + 8192 + 32) >> 6) : w[(yy + 1) * CWP + xx + 1];
      } else if (!fx) {
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) s += kChromaFilter[fy][i] * w[(yy + i) * CWP + xx + 1];
        pred = clip_pel((s + 32) >> 6);
      } else {
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) s += kChromaFilter[fy][i] * h[(yy + i) * Sc + xx];
        pred = clip_pel((s + (1 << 11) + (8192 << 6)) >> 12);
      }
      const int t = (yy / Tc) * (Sc / Tc) + (xx / Tc);
      const int tu = ctu_tu_index(L, ctu, d, j, t, c + 1);
      const int16_t rv = (int16_t)((int)C.cur[c][(yc + yy) * C.stride + xc + xx] - pred);
      const int64_t o = ctu_tu_offset(L, tu) + (yy % Tc) * Tc + (xx % Tc);
      resid[o] = rv;
      pred_out[o] = (uint8_t)pred;
      if (d == 3) {
        const int64_t ot = ctu_tu_offset(L, ctu_tu_ts(L, tu)) + yy * 4 + xx;
        resid[ot] = rv;
        pred_out[ot] = (uint8_t)pred;
      }
    }
  }
}

template <int S>
static __global__ __launch_bounds__(64) void k_ctu_pred_resid(CtuMc M, int ctu0) {
  constexpr int d = S == 64 ? 0 : S == 32 ? 1 : S == 16 ? 2 : 3, ncu = 1 << (2 * d);
  __shared__ uint8_t win[(S + 7) * (S + 8)];
  __shared__ int16_t hs[(S + 7) * S];
  ctu_pred_resid_cu<S>(M, ctu0 + (int)(blockIdx.x / ncu), (int)(blockIdx.x % ncu), win, hs);
}

// Depth 3 (8x8 CUs), NC CUs per wave (one wave per CU left most of the launch waiting on
// dependent memory round trips with little work).  The originals are fetched first (they do not
// depend on the search), the luma and chroma reference windows of all NC CUs in one round trip
// once the references and MVs are known.  The MC is branch-free: the two-stage form with the
// phase-0 filters ({0,0,0,64,0,0,0,0} / {0,64,0,0}) gives exactly the reference's one-stage and
// copy cases ((64X + 2048) >> 12 == (X + 32) >> 6, (4096b + 2048) >> 12 == b), the first stage is
// v_dot4_i32_i8 on sign-biased window bytes (b - 128: the -8192 offset), the second
// v_dot2_i32_i16 on int16 tap pairs.
template <int NC>
static __global__ __launch_bounds__(64) void k_ctu_pred_resid8q(CtuMc M) {
  static_assert(NC % 2 == 0 && NC * 5 <= 64 && 64 % NC == 0, "CUs per wave");
  __shared__ uint32_t winY[NC][15 * 4];      // 15 rows x 16 bytes (15 used), biased
  __shared__ int16_t hsY[NC][15 * 8];
  __shared__ uint32_t winC[2 * NC][7 * 2];   // 7 rows x 8 bytes (7 used), biased
  __shared__ int16_t hsC[2 * NC][7 * 4];
  const CtuLayout &L = M.L;
  const hvx_ctu_params &P = M.P;
  const CtuChroma &C = M.C;
  constexpr int PER = 64 / NC;  // waves per CTU
  const int lane = lane_id(), ctu = (int)(blockIdx.x / PER), j0 = (int)(blockIdx.x % PER) * NC;
  const int stride = M.stride;
  const int bx = (ctu % L.nctu_x) * 64, by = (ctu / L.nctu_x) * 64;
  int x[NC], y[NC];
  uint32_t vmask = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    const int j = j0 + c;
    x[c] = bx + (j % 8) * 8;
    y[c] = by + (j / 8) * 8;
    vmask |= (x[c] + 8 <= P.pic_w && y[c] + 8 <= P.pic_h) ? 1u << c : 0u;
  }
  // the originals: luma sample (lane >> 3, lane & 7) of every CU; chroma sample
  // ((lane >> 2) & 3, lane & 3) of component (lane >> 4) & 1 of CU 2p + (lane >> 5)
  const int ly = lane >> 3, lx = lane & 7;
  const int cyy = (lane >> 2) & 3, cxx = lane & 3, ccomp = (lane >> 4) & 1, cq = lane >> 5;
  int curY[NC], curC[NC / 2];
#pragma unroll
  for (int c = 0; c < NC; c++) curY[c] = (vmask >> c) & 1 ? M.cur[(y[c] + ly) * stride + x[c] + lx] : 0;
  if (C.on) {
#pragma unroll
    for (int p = 0; p < NC / 2; p++) {
      const int c = 2 * p + cq;
      const int cx0 = bx + ((j0 + c) % 8) * 8, cy0 = by + ((j0 + c) / 8) * 8;
      curC[p] = (vmask >> c) & 1 ? C.cur[ccomp][(cy0 / 2 + cyy) * C.stride + cx0 / 2 + cxx] : 0;
    }
  }
  int bref[NC], mvx[NC], mvy[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) {  // wave-uniform: first-minimum reference
    const int j = j0 + c;
    const bool v = (vmask >> c) & 1;
    const hvx_me_result *r = M.res + ((size_t)ctu * HVX_CUS_PER_CTU + 21 + j) * L.nref;
    int best = 0;
    uint32_t bc = 0;
    if (v)
      for (int k = 0; k < L.nref; k++) {
        const uint32_t ck = r[k].cost;
        if (k == 0 || ck < bc) { bc = ck; best = k; }
      }
    bref[c] = best;
    mvx[c] = v ? r[best].mv_x : 0;
    mvy[c] = v ? r[best].mv_y : 0;
    if (lane == c) {
      hvx_cu_result o;
      o.valid = v; o.ref = best; o.mv_x = mvx[c]; o.mv_y = mvy[c];
      o.me_cost = v ? bc : 0; o.sse = 0; o.abs_sum = 0; o.n_tu = v ? 1 : 0;
      M.out[(size_t)ctu * HVX_CUS_PER_CTU + 21 + j] = o;
    }
  }
  const int nper = C.on ? 5 : 1;
  if (lane < NC * nper) {
    const int c = lane / nper;
    ctu_desc<8>(M, ctu, j0 + c, (vmask >> c) & 1, 0, lane % nper);
  }
  // reference windows: luma rows y-3 .. y+11, columns x-3 .. x+11; chroma rows yc-1 .. yc+5,
  // columns xc-1 .. xc+5 at the 1/8-sample MV
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!((vmask >> c) & 1)) continue;
    const uint8_t *rp = M.refs[bref[c]] + (y[c] + (mvy[c] >> 2) - 3) * stride + x[c] + (mvx[c] >> 2) - 3;
    uint8_t *w = reinterpret_cast<uint8_t *>(winY[c]);
    for (int k = lane; k < 225; k += HVX_WAVE) {
      const int rr = k / 15, cc = k - rr * 15;
      w[rr * 16 + cc] = rp[rr * stride + cc] ^ 0x80;
    }
    if (C.on) {
      const int xc = x[c] / 2, yc = y[c] / 2, wo = (yc + (mvy[c] >> 3) - 1) * C.stride + xc + (mvx[c] >> 3) - 1;
      if (lane < 49) {
        const int rr = lane / 7, cc = lane - rr * 7;
#pragma unroll
        for (int comp = 0; comp < 2; comp++)
          reinterpret_cast<uint8_t *>(winC[2 * c + comp])[rr * 8 + cc] = C.refs[comp * L.nref + bref[c]][wo + rr * C.stride + cc] ^ 0x80;
      }
    }
  }
  __syncthreads();
  // first stages
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!((vmask >> c) & 1)) continue;
    const int fx = mvx[c] & 3;
    const int clo = (int)kLumaTap4[fx][0], chi = (int)kLumaTap4[fx][1];
    for (int k = lane; k < 120; k += HVX_WAVE) {
      const int rr = k >> 3, xx = k & 7;
      const uint32_t *w = winY[c] + rr * 4 + (xx >> 2);
      const uint32_t sh = xx & 3, lo = __builtin_amdgcn_alignbyte(w[1], w[0], sh), hi = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
      hsY[c][rr * 8 + xx] = (int16_t)__builtin_amdgcn_sdot4((int)lo, clo, __builtin_amdgcn_sdot4((int)hi, chi, 0, false), false);
    }
    if (C.on) {
      const int cw = (int)kChromaTap4[mvx[c] & 7];
#pragma unroll
      for (int comp = 0; comp < 2; comp++)
        if (lane < 28) {
          const int rr = lane >> 2, xx = lane & 3;
          const uint32_t *w = winC[2 * c + comp] + rr * 2;
          hsC[2 * c + comp][rr * 4 + xx] = (int16_t)__builtin_amdgcn_sdot4((int)__builtin_amdgcn_alignbyte(w[1], w[0], xx), cw, 0, false);
        }
    }
  }
  __syncthreads();
  typedef short s2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int c = 0; c < NC; c++) {  // luma second stage, residual, prediction
    if (!((vmask >> c) & 1)) continue;
    const int fy = mvy[c] & 3;
    int s = (1 << 11) + (8192 << 6);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const s2 pr = {hsY[c][(ly + 2 * u) * 8 + lx], hsY[c][(ly + 2 * u + 1) * 8 + lx]};
      s = __builtin_amdgcn_sdot2(pr, __builtin_bit_cast(s2, kLumaPairs[fy][u]), s, false);
    }
    const int pred = clip_pel(s >> 12);
    const int64_t o = ctu_tu_offset(L, ctu_tu_index(L, ctu, 3, j0 + c, 0)) + lane;
    M.resid[o] = (int16_t)(curY[c] - pred);
    M.pred_out[o] = (uint8_t)pred;
  }
  if (!C.on) return;
#pragma unroll
  for (int p = 0; p < NC / 2; p++) {  // chroma second stage, two CUs per pass (lanes 32.. the odd one)
    int c = 2 * p, cmy = mvy[2 * p];
    bool v = (vmask >> (2 * p)) & 1;
    if (cq) { c = 2 * p + 1; cmy = mvy[2 * p + 1]; v = (vmask >> (2 * p + 1)) & 1; }
    if (!v) continue;
    const int fy = cmy & 7;
    const int16_t *h = hsC[2 * c + ccomp];
    int s = (1 << 11) + (8192 << 6);
    const s2 p0 = {h[cyy * 4 + cxx], h[(cyy + 1) * 4 + cxx]}, p1 = {h[(cyy + 2) * 4 + cxx], h[(cyy + 3) * 4 + cxx]};
    s = __builtin_amdgcn_sdot2(p0, __builtin_bit_cast(s2, kChromaPairs[fy][0]), s, false);
    s = __builtin_amdgcn_sdot2(p1, __builtin_bit_cast(s2, kChromaPairs[fy][1]), s, false);
    const int pred = clip_pel(s >> 12);
    const int tu = ctu_tu_index(L, ctu, 3, j0 + c, 0, ccomp + 1);
    const int16_t rv = (int16_t)(curC[p] - pred);
    const int64_t o = ctu_tu_offset(L, tu) + cyy * 4 + cxx, ot = ctu_tu_offset(L, ctu_tu_ts(L, tu)) + cyy * 4 + cxx;
    M.resid[o] = rv;
    M.pred_out[o] = (uint8_t)pred;
    M.resid[ot] = rv;
    M.pred_out[ot] = (uint8_t)pred;
  }
}

static __global__ __launch_bounds__(256) void k_ctu_finalize(CtuLayout L, const int32_t *__restrict__ abs_sum,
                                                      const uint32_t *__restrict__ sse, hvx_cu_result *__restrict__ out) {
  const int cuid = blockIdx.x * blockDim.x + threadIdx.x;
  if (cuid >= L.nctu * HVX_CUS_PER_CTU) return;
  hvx_cu_result o = out[cuid];
  if (!o.valid) return;
  const int ctu = cuid / HVX_CUS_PER_CTU, ci = cuid % HVX_CUS_PER_CTU;
  int d, j, S, g;
  cu_geom(ci, d, j, S, g);
  uint32_t s = 0;
  int a = 0;
  for (int t = 0; t < o.n_tu; t++) {
    const int tu = ctu_tu_index(L, ctu, d, j, t);
    s += sse[tu];
    a += abs_sum[tu];
  }
  o.sse = s;
  o.abs_sum = a;
  out[cuid] = o;
}

// ------------------------------------------------------------------------------------------
// CU decision (hvx_ctu_decide; restated by hvxo_ctu_decide).  TEncCu::xCompressCU's depth
// recursion (TEncCu.cpp:349-877): a CU's leaf cost (ME ruiBits + counted coefficient rate +
// split_cu_flag=0, TEncCu.cpp:681) against its four children's best trees + split_cu_flag=1
// (:797), costs by calcRdCost (TComRdCost.cpp:57), the split taken only on a strictly smaller
// cost (xCheckBestMode :1166).  One THREAD per CTU walks the 85-node tree in z-order (the
// recursion is compile-time unrolled), so each split flag's context sees the final depths of
// its left/above neighbours inside the CTU exactly as getCtxSplitFlag (TComDataCU.cpp:1487) does;
// the CTU's final depth map lives in two 64-bit planes (2 bits per 8x8).
struct DecideArgs {
  CtuLayout L;
  int pic_w, pic_h;
  double lambda;
  const hvx_cu_result *cu;
  const hvx_me_result *res;
  const hvx_coeff_bits *cb;
  const uint8_t *st;          // the context snapshot (split flag 0..2, luma qt_cbf 28.., qt_root_cbf 41)
  const int32_t *eb;
  hvx_cu_decision *dec;
  int metric;                 // HVX_RD_SSE / HVX_RD_SSIM
  double lambda_ssim;
  CtuChroma C;                // 4:2:0 planes (C.on), else luma only
  double cw;                  // TComRdCost::m_distortionWeight of Cb / Cr
};

// TComRdCost::getDistPart of a chroma block: weight * SSE, truncated (TComRdCost.cpp:443-446)
__device__ __forceinline__ uint32_t dec_wdist(double w, uint32_t sse) { return (uint32_t)__dmul_rn(w, (double)sse); }

// the CU-level RD cost (hvxo's cu_cost): calcRdCost, or D_ssim + lambda_ssim * R
__device__ __forceinline__ double dec_cu_cost(const DecideArgs &A, uint32_t bits, uint32_t dist, float sdist) {
  if (A.metric == HVX_RD_SSIM) return __dadd_rn((double)sdist, __dmul_rn(A.lambda_ssim, (double)bits));
  return floor((double)dist + (double)bits * A.lambda + 0.5);
}

__device__ __forceinline__ double dec_rd_cost(uint32_t bits, uint32_t dist, double lambda) {
  return floor((double)dist + (double)bits * lambda + 0.5);
}

struct DepthMap {
  uint64_t lo = 0, hi = 0;
  __device__ __forceinline__ int at(int x8, int y8) const {
    const int i = y8 * 8 + x8;
    return (int)((lo >> i) & 1) | ((int)((hi >> i) & 1) << 1);
  }
  __device__ __forceinline__ void fill(int x8, int y8, int n8, int d) {
    uint64_t m = 0;
    const uint64_t row = (n8 == 8) ? 0xffull : ((1ull << n8) - 1);
    for (int y = 0; y < n8; y++) m |= row << ((y8 + y) * 8 + x8);
    lo = (d & 1) ? (lo | m) : (lo & ~m);
    hi = (d & 2) ? (hi | m) : (hi & ~m);
  }
};

// the CTU's leaf records held in lanes: CU ci in lane ci % 64 of register ci / 64
struct DecLanes {
  uint32_t valid[2], bits[2], dist[2], ssim[2];
};
// the walk's results, written back into the same lanes
struct DecOuts {
  uint32_t bb[2], bd[2], bs[2];
  uint64_t split[2];  // bit ci % 64 of word ci / 64 (wave-uniform)
};

// TEncCu::xCompressCU's depth recursion for CU (D, CX, CY) of a CTU as wave-uniform code: the
// node's leaf record comes from its lane by v_readlane (constant lane: the recursion is unrolled
// at compile time), so the chain of decisions has no memory access on it.  rf[ctx][f] =
// split_cu_flag f's rate under context ctx.
template <int D, int CX, int CY>
__device__ __forceinline__ bool dec_walk(const DecideArgs &A, const uint32_t (&rf)[3][2], int ctu, DepthMap &dm,
                                         const DecLanes &V, DecOuts &O, uint32_t &bits, uint32_t &dist, float &sdist) {
  constexpr int g = 1 << D, S = 64 >> D, n8 = S / 8;
  constexpr int CI = (D == 0 ? 0 : D == 1 ? 1 : D == 2 ? 5 : 21) + CY * g + CX, H = CI / 64, LN = CI % 64;
  const int x = (ctu % A.L.nctu_x) * 64 + CX * S, y = (ctu / A.L.nctu_x) * 64 + CY * S;
  if (x >= A.pic_w || y >= A.pic_h) return false;
  constexpr int x8 = CX * n8, y8 = CY * n8;
  const bool valid = __builtin_amdgcn_readlane((int)V.valid[H], LN) != 0;
  const int ctx = (x8 > 0 && dm.at(x8 - 1, y8) > D) + (y8 > 0 && dm.at(x8, y8 - 1) > D);
  uint32_t lb = 0, ld = 0;
  float ls = 0.0f;
  if (valid) {
    lb = (uint32_t)__builtin_amdgcn_readlane((int)V.bits[H], LN) + (D < 3 ? rf[ctx][0] : 0u);
    ld = (uint32_t)__builtin_amdgcn_readlane((int)V.dist[H], LN);
    ls = __int_as_float(__builtin_amdgcn_readlane((int)V.ssim[H], LN));
  }
  bool split = !valid;
  uint32_t sb = 0, sd = 0;
  float ss = 0.0f;
  if constexpr (D < 3) {
    uint32_t b, dd;
    float sv;
    if (dec_walk<D + 1, 2 * CX, 2 * CY>(A, rf, ctu, dm, V, O, b, dd, sv)) { sb += b; sd += dd; ss += sv; }
    if (dec_walk<D + 1, 2 * CX + 1, 2 * CY>(A, rf, ctu, dm, V, O, b, dd, sv)) { sb += b; sd += dd; ss += sv; }
    if (dec_walk<D + 1, 2 * CX, 2 * CY + 1>(A, rf, ctu, dm, V, O, b, dd, sv)) { sb += b; sd += dd; ss += sv; }
    if (dec_walk<D + 1, 2 * CX + 1, 2 * CY + 1>(A, rf, ctu, dm, V, O, b, dd, sv)) { sb += b; sd += dd; ss += sv; }
    if (valid) {
      sb += rf[ctx][1];
      if (dec_cu_cost(A, sb, sd, ss) < dec_cu_cost(A, lb, ld, ls)) split = true;
    }
  }
  bits = split ? sb : lb;
  dist = split ? sd : ld;
  sdist = split ? ss : ls;
  if (split) O.split[H] |= 1ull << LN;
  const bool me = lane_id() == LN;  // this node's lane takes its results
  O.bb[H] = me ? bits : O.bb[H];
  O.bd[H] = me ? dist : O.bd[H];
  O.bs[H] = me ? __float_as_uint(sdist) : O.bs[H];
  if (!split) dm.fill(x8, y8, n8, D);
  return true;
}

// Leaf evaluation of every CU (hvxo_ctu_decide's leaf_eval: encodeResAndCalcRdInterCU's residual
// decisions, TEncSearch.cpp:4341-4421): one THREAD per CU over its TUs' per-TU records -- counted
// rate, uiAbsSum, coded SSE, zero-residual and clipped-reconstruction distortions (k_tu_fin) --
// per TU and component the forced-zero test (and at 4x4 chroma the transform-skip mode), the
// qt_root_cbf test and the leaf distortion as the sum of the chosen TU distortions (chroma
// weighted per component).  Writes coef_frac, bits, dist and cbf.
static __global__ __launch_bounds__(64) void k_ctu_leaf(DecideArgs A, const int32_t *__restrict__ abs_sum,
                                                 const uint32_t *__restrict__ sse, const uint32_t *__restrict__ zd,
                                                 const uint32_t *__restrict__ csse) {
  const int cuid = blockIdx.x * 64 + threadIdx.x;
  if (cuid >= A.L.nctu * HVX_CUS_PER_CTU) return;
  const int ctu = cuid / HVX_CUS_PER_CTU, ci = cuid % HVX_CUS_PER_CTU;
  const hvx_cu_result cu = A.cu[cuid];
  if (!cu.valid) return;
  int d, j, S, g;
  cu_geom(ci, d, j, S, g);
  const int T = S < 32 ? S : 32, ntu = (S / T) * (S / T), ncomp = A.C.on ? 3 : 1;
  const double lam = A.lambda;
  uint64_t tree = 0, cf = 0;
  uint32_t nz_dist = 0, zero_dist = 0;
  int cbf = 0;
  for (int t = 0; t < ntu; t++) {
    for (int comp = 0; comp < ncomp; comp++) {  // per TU Y, Cb, Cr (xEstimateInterResidualQT's component loop)
      const int m_cbf = comp ? 33 + (S > 32 ? 1 : 0) : 28 + (S > 32 ? 0 : 1);
      const uint32_t c0 = (uint32_t)A.eb[A.st[m_cbf] ^ 0], c1 = (uint32_t)A.eb[A.st[m_cbf] ^ 1];
      const int tu = ctu_tu_index(A.L, ctu, d, j, t, comp);
      uint32_t td = comp ? dec_wdist(A.cw, zd[tu]) : zd[tu];
      const uint64_t fr = A.cb[tu].frac_bits;
      uint64_t tf = c0;
      zero_dist += td;
      cf += fr;
      if (abs_sum[tu] > 0) {
        const uint64_t f1 = c1 + fr;
        const uint32_t sd = comp ? dec_wdist(A.cw, sse[tu]) : sse[tu];
        if (!(dec_rd_cost(c0 >> 15, td, lam) < dec_rd_cost((uint32_t)(f1 >> 15), sd, lam))) {
          tf = f1;
          td = sd;
          cbf |= 1 << (4 * comp + t);
        }
      }
      if (comp && T == 8) {  // the transform-skip mode of a 4x4 TU: chosen when its coded cost <= mode 0's best
        const int tt = ctu_tu_ts(A.L, tu);
        if (abs_sum[tt] > 0) {
          const uint64_t f2 = c1 + A.cb[tt].frac_bits;
          const uint32_t sd = dec_wdist(A.cw, sse[tt]);
          if (dec_rd_cost((uint32_t)(f2 >> 15), sd, lam) <= dec_rd_cost((uint32_t)(tf >> 15), td, lam)) {
            tf = f2;
            td = sd;
            cbf |= (1 << (4 * comp + t)) | (1 << (8 + 4 * comp + t));
          }
        }
      }
      tree += tf;
      nz_dist += td;
    }
  }
  const uint32_t r0 = (uint32_t)A.eb[A.st[41] ^ 0], r1 = (uint32_t)A.eb[A.st[41] ^ 1];
  if (dec_rd_cost(r0 >> 15, zero_dist, lam) < dec_rd_cost((uint32_t)(tree >> 15), nz_dist, lam)) cbf = 0;
  // the clipped reconstruction's distortion: coded TUs' csse, prediction-only TUs' zero-residual sum
  uint32_t dist = 0;
  for (int comp = 0; comp < ncomp; comp++) {
    uint32_t cd = 0;
    for (int t = 0; t < ntu; t++) {
      const int tu = ctu_tu_index(A.L, ctu, d, j, t, comp);
      const bool coded = (cbf >> (4 * comp + t)) & 1, ts = comp && ((cbf >> (8 + 4 * comp + t)) & 1);
      cd += coded ? csse[ts ? ctu_tu_ts(A.L, tu) : tu] : zd[tu];
    }
    dist += comp ? dec_wdist(A.cw, cd) : cd;
  }
  hvx_cu_decision &r = A.dec[cuid];
  r.coef_frac = cf;
  r.cbf = cbf;
  r.dist = dist;
  r.bits = A.res[(size_t)cuid * A.L.nref + cu.ref].bits + (uint32_t)((cbf ? r1 + tree : r0) >> 15);
  r.ssim_dist = 0.0f;
}

// HVX_RD_SSIM (after k_ctu_leaf): D_ssim = sum over the CU's luma 8x8 blocks (raster order) of
// 1 - SSIM(org, rec), one block per lane with compute_SSIM's float operations in its order
// (stvssim.c:506-545); one wave per CU.
static __global__ __launch_bounds__(64) void k_ctu_leaf_ssim(DecideArgs A, const uint8_t *__restrict__ cur, int stride,
                                                      const int16_t *__restrict__ resid,
                                                      const int16_t *__restrict__ res_out) {
  const int cuid = blockIdx.x, ctu = cuid / HVX_CUS_PER_CTU, ci = cuid % HVX_CUS_PER_CTU;
  const hvx_cu_result cu = A.cu[cuid];
  if (!cu.valid) return;
  int d, j, S, g;
  cu_geom(ci, d, j, S, g);
  const int x = (ctu % A.L.nctu_x) * 64 + (j % g) * S, y = (ctu / A.L.nctu_x) * 64 + (j / g) * S;
  const int T = S < 32 ? S : 32, lane = lane_id();
  const int cbf = A.dec[cuid].cbf;
  __shared__ float sdist[64];
  const int nb8 = S / 8;
  if (lane < nb8 * nb8) {
    const int by = lane / nb8, bx = lane - by * nb8;
    const float C1 = 0.01f * 0.01f * (float)(255 * 255), C2 = 0.03f * 0.03f * (float)(255 * 255);
    const float wgt = 1.0f / (float)(8 * 8);
    float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
    for (int n = 0; n < 8; n++)
      for (int m = 0; m < 8; m++) {
        const int yy = by * 8 + n, xx = bx * 8 + m, t = (yy / T) * (S / T) + xx / T;
        const int64_t o = ctu_tu_offset(A.L, ctu_tu_index(A.L, ctu, d, j, t)) + (yy % T) * T + (xx % T);
        const int po = cur[(y + yy) * stride + x + xx];
        const int pe = clip_pel(po - resid[o] + (((cbf >> t) & 1) ? res_out[o] : 0));
        mo += wgt * po; me += wgt * pe;
        vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
      }
    const float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
    float sv = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
    sv /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
    sv /= 1.0f;  // one window (compute_SSIM's dist /= cnt)
    if (sv >= 1.0 && sv < 1.01) sv = 1.0f;
    sdist[lane] = 1.0f - sv;
  }
  __syncthreads();
  if (lane == 0) {
    float dsum = 0.0f;
    for (int b = 0; b < nb8 * nb8; b++) dsum += sdist[b];
    A.dec[cuid].ssim_dist = dsum;
  }
}

// One WAVE per CTU: the 85 leaf records (k_ctu_leaf) and CU results are loaded lane-parallel, the
// depth recursion (dec_walk) runs wave-uniform on them, and the decisions are stored lane-parallel.
static __global__ __launch_bounds__(64) void k_ctu_decide(DecideArgs A) {
  const int ctu = blockIdx.x, lane = lane_id();
  DecLanes V;
  hvx_cu_decision lf[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int ci = lane + 64 * h;
    const size_t cuid = (size_t)ctu * HVX_CUS_PER_CTU + ci;
    lf[h] = hvx_cu_decision{0, 0, 0, 0, 0, 0, 0, 0, 0.0f, 0.0f, 0};
    V.valid[h] = 0;
    if (ci < HVX_CUS_PER_CTU && A.cu[cuid].valid) {
      lf[h] = A.dec[cuid];
      V.valid[h] = 1;
    }
    V.bits[h] = lf[h].bits; V.dist[h] = lf[h].dist; V.ssim[h] = __float_as_uint(lf[h].ssim_dist);
  }
  uint32_t rf[3][2];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int st = A.st[c];
    rf[c][0] = (uint32_t)A.eb[st ^ 0] >> 15;
    rf[c][1] = (uint32_t)A.eb[st ^ 1] >> 15;
  }
  DepthMap dm;
  DecOuts O = {};
  uint32_t b, d;
  float sd;
  dec_walk<0, 0, 0>(A, rf, ctu, dm, V, O, b, d, sd);
  // store: leaf = in the picture, not splitting, and every ancestor splits
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int ci = lane + 64 * h;
    if (ci >= HVX_CUS_PER_CTU) continue;
    int dd, j, S, g;
    cu_geom(ci, dd, j, S, g);
    const int x = (ctu % A.L.nctu_x) * 64 + (j % g) * S, y = (ctu / A.L.nctu_x) * 64 + (j / g) * S;
    hvx_cu_decision o = hvx_cu_decision{0, 0, 0, 0, 0, 0, 0, 0, 0.0f, 0.0f, 0};
    if (x < A.pic_w && y < A.pic_h) {
      const bool sp = (O.split[h] >> (ci % 64)) & 1;
      bool reached = true;
      int pj = j, pg = g;
      for (int pd = dd - 1; pd >= 0; pd--) {  // the ancestors, parent first
        pj = ((pj / pg) >> 1) * (pg >> 1) + ((pj % pg) >> 1);
        pg >>= 1;
        const int pci = depth_base(pd) + pj;
        reached = reached && ((O.split[pci / 64] >> (pci % 64)) & 1);
      }
      o = lf[h];
      o.split = sp;
      o.leaf = reached && !sp;
      o.best_bits = O.bb[h];
      o.best_dist = O.bd[h];
      o.best_ssim_dist = __uint_as_float(O.bs[h]);
    }
    A.dec[(size_t)ctu * HVX_CUS_PER_CTU + ci] = o;
  }
}

// reconstruction of the leaves: recon = clip(org - residual + coded reconstructed residual)
// (= pred + the residual the leaf keeps, TComYuv::addClip) into the 8-bit picture plane; one
// 256-thread block per CTU, each thread 16 samples of a 64x64 CTU
__device__ __forceinline__ void ctu_bs_unit(const hvx_cu_result *__restrict__ cu, const hvx_cu_decision *__restrict__ dec,
                                            int pic_w, int pic_h, int qp, int ux, int uy, uint8_t *__restrict__ bs_ver,
                                            uint8_t *__restrict__ bs_hor, int8_t *__restrict__ qpm);
struct CtuBsArgs {
  const hvx_cu_result *cu;
  uint8_t *bsv, *bsh;  // nullptr: no boundary strengths
  int8_t *qpm;
  int qp;
};
static __global__ __launch_bounds__(256) void k_ctu_recon(CtuLayout L, int pic_w, int pic_h, const uint8_t *__restrict__ cur,
                                                   int stride, const hvx_cu_decision *__restrict__ dec,
                                                   const int16_t *__restrict__ resid, const int16_t *__restrict__ res_out,
                                                   uint8_t *__restrict__ recon, CtuChroma C, uint8_t *__restrict__ rp_y,
                                                   uint8_t *__restrict__ rp_cb, uint8_t *__restrict__ rp_cr, CtuBsArgs B) {
  // rp_*: the reference picture's planes (nullable), written with the same samples before deblocking;
  // B.bsv: also the boundary strengths of the CTU's 16x16 units of 4x4 samples (k_ctu_bs)
  const int ctu = blockIdx.x;
  if (B.bsv) {
    const int ux = (ctu % L.nctu_x) * 16 + (int)(threadIdx.x & 15), uy = (ctu / L.nctu_x) * 16 + (int)(threadIdx.x >> 4);
    if (ux < (pic_w >> 2) && uy < (pic_h >> 2)) ctu_bs_unit(B.cu, dec, pic_w, pic_h, B.qp, ux, uy, B.bsv, B.bsh, B.qpm);
  }
  const int x0 = (ctu % L.nctu_x) * 64, y0 = (ctu / L.nctu_x) * 64;
  const hvx_cu_decision *dc = dec + (size_t)ctu * HVX_CUS_PER_CTU;
  // the CTU's leaf CU of every 8x8 block (-1: none) and the CUs' cbf words, staged in LDS once
  __shared__ int cbfm[HVX_CUS_PER_CTU];
  __shared__ int8_t leafm[HVX_CUS_PER_CTU], blk[64];
  if (threadIdx.x < HVX_CUS_PER_CTU) {
    leafm[threadIdx.x] = (int8_t)dc[threadIdx.x].leaf;
    cbfm[threadIdx.x] = dc[threadIdx.x].cbf;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int bx = threadIdx.x & 7, by = threadIdx.x >> 3;
    int ci = -1;
    for (int d = 0; d < 4 && ci < 0; d++) {
      const int c = depth_base(d) + (by >> (3 - d)) * (1 << d) + (bx >> (3 - d));
      if (leafm[c]) ci = c;
    }
    blk[threadIdx.x] = (int8_t)ci;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * 64; k += 256) {
    const int yy = k >> 6, xx = k & 63, x = x0 + xx, y = y0 + yy;
    if (x >= pic_w || y >= pic_h) continue;
    const int ci = blk[(yy >> 3) * 8 + (xx >> 3)];
    if (ci < 0) continue;  // not reached for a decided CTU
    int d, j, S0, g0;
    cu_geom(ci, d, j, S0, g0);
    const int S = 64 >> d, T = S < 32 ? S : 32, cx = xx % S, cy = yy % S, t = (cy / T) * (S / T) + (cx / T);
    const int tu = ctu_tu_index(L, ctu, d, j, t);
    const int64_t o = ctu_tu_offset(L, tu) + (cy % T) * T + (cx % T);
    const int v = (int)cur[y * stride + x] - resid[o] + (((cbfm[ci] >> t) & 1) ? res_out[o] : 0);
    const uint8_t rv = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    recon[y * stride + x] = rv;
    if (rp_y) rp_y[y * stride + x] = rv;
  }
  if (!C.on) return;
  for (int k = threadIdx.x; k < 2 * 32 * 32; k += 256) {  // Cb then Cr, 32x32 chroma samples per CTU
    const int c = 1 + (k >> 10), yy = (k >> 5) & 31, xx = k & 31, x = x0 / 2 + xx, y = y0 / 2 + yy;
    if (2 * x >= pic_w || 2 * y >= pic_h) continue;
    const int ci = blk[(yy >> 2) * 8 + (xx >> 2)];
    if (ci < 0) continue;
    int d, j, S0, g0;
    cu_geom(ci, d, j, S0, g0);
    const int Sc = 32 >> d, Tc = (Sc < 16 ? Sc : 16), cx = xx % Sc, cy = yy % Sc, t = (cy / Tc) * (Sc / Tc) + (cx / Tc);
    const int tu = ctu_tu_index(L, ctu, d, j, t, c), cbf = cbfm[ci];
    const int64_t o = ctu_tu_offset(L, tu) + (cy % Tc) * Tc + (cx % Tc);
    const int64_t orr = ((cbf >> (8 + 4 * c + t)) & 1) ? ctu_tu_offset(L, ctu_tu_ts(L, tu)) + cy * 4 + cx : o;
    const int v = (int)C.cur[c - 1][y * C.stride + x] - resid[o] + (((cbf >> (4 * c + t)) & 1) ? res_out[orr] : 0);
    const uint8_t rv = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    C.recon[c - 1][y * C.stride + x] = rv;
    uint8_t *rp = c == 1 ? rp_cb : rp_cr;
    if (rp) rp[y * C.stride + x] = rv;
  }

}

// Boundary strengths of the decided CU trees (restated by hvxo_ctu_bs): TComLoopFilter's
// xSetEdgefilterTU/PU (TComLoopFilter.cpp:274-359) + xGetBoundaryStrengthSingle (:417-557) for
// 2Nx2N inter CUs of a P slice with luma TUs of min(CU, 32).  One thread per 4x4 luma unit writes
// the BS of its left and top edges (0 off the 8x8 grid / at the picture border) and its QP.
__device__ __forceinline__ void unit_block(const hvx_cu_decision *dec, int nctu_x, int ux, int uy, int &ctu, int &ci,
                                           int &t) {
  ctu = (uy >> 4) * nctu_x + (ux >> 4);
  const int lx = ux & 15, ly = uy & 15;
  for (int d = 0; d < 4; d++) {
    const int su = 16 >> d, j = (ly / su) * (1 << d) + lx / su, k = depth_base(d) + j;
    if (d == 3 || dec[(size_t)ctu * HVX_CUS_PER_CTU + k].leaf) {
      const int tu = su < 8 ? su : 8;
      ci = k;
      t = ((ly % su) / tu) * (su / tu) + (lx % su) / tu;
      return;
    }
  }
}

__device__ __forceinline__ void ctu_bs_unit(const hvx_cu_result *__restrict__ cu, const hvx_cu_decision *__restrict__ dec,
                                            int pic_w, int pic_h, int qp, int ux, int uy, uint8_t *__restrict__ bs_ver,
                                            uint8_t *__restrict__ bs_hor, int8_t *__restrict__ qpm) {
  const int uw = pic_w >> 2, nctu_x = (pic_w + 63) >> 6, u = uy * uw + ux;
  qpm[u] = (int8_t)qp;
  int cq, kq, tq;
  unit_block(dec, nctu_x, ux, uy, cq, kq, tq);
  const hvx_cu_decision &dq = dec[(size_t)cq * HVX_CUS_PER_CTU + kq];
  const hvx_cu_result &rq = cu[(size_t)cq * HVX_CUS_PER_CTU + kq];
#pragma unroll
  for (int dir = 0; dir < 2; dir++) {
    uint8_t bs = 0;
    if (dir == 0 ? ((ux & 1) == 0 && ux > 0) : ((uy & 1) == 0 && uy > 0)) {
      int cp, kp, tp;
      unit_block(dec, nctu_x, dir ? ux : ux - 1, dir ? uy - 1 : uy, cp, kp, tp);
      if (cq != cp || kq != kp || tq != tp) {
        const hvx_cu_decision &dp = dec[(size_t)cp * HVX_CUS_PER_CTU + kp];
        const hvx_cu_result &rp = cu[(size_t)cp * HVX_CUS_PER_CTU + kp];
        if (((dq.cbf >> tq) & 1) || ((dp.cbf >> tp) & 1)) bs = 1;
        else bs = (rq.ref != rp.ref || abs(rq.mv_x - rp.mv_x) >= 4 || abs(rq.mv_y - rp.mv_y) >= 4) ? 1 : 0;
      }
    }
    (dir ? bs_hor : bs_ver)[u] = bs;
  }
}
static __global__ __launch_bounds__(256) void k_ctu_bs(const hvx_cu_result *__restrict__ cu,
                                                const hvx_cu_decision *__restrict__ dec, int pic_w, int pic_h, int qp,
                                                uint8_t *__restrict__ bs_ver, uint8_t *__restrict__ bs_hor,
                                                int8_t *__restrict__ qpm) {
  const int uw = pic_w >> 2, uh = pic_h >> 2;
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= uw * uh) return;
  ctu_bs_unit(cu, dec, pic_w, pic_h, qp, u % uw, u / uw, bs_ver, bs_hor, qpm);
}
