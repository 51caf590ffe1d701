// hvx_ctu.hpp -- the CTU analysis pass on the device (the bench workload; hvx_types.h,
// DESIGN.md).  All CTUs of a picture are independent here (no neighbour-dependent
// predictors), so the pass is a fixed sequence of wide launches:
//   for depth 0..3: k_ctu_me_jobs (one thread per CU x reference) -> k_me
//   k_ctu_pred_resid (one wave per CU: best reference, luma MC, residual, TU descriptors)
//   k_tu<L,pipeline> per TU size class over contiguous class ranges
//   k_ctu_finalize (per-CU sums)
// The composition is restated on the CPU by hvxo_ctu_analyze (oracle/hvx_oracle.c).
#pragma once
#include "hvx_dev.hpp"
#include "hvx_me.hpp"

struct CtuLayout {
  int nctu_x, nctu_y, nctu, nref;
  // TU classes, contiguous: [0,8n) 32x32 | [8n,24n) 16x16 | [24n,88n) 8x8
  __host__ __device__ int ntu() const { return 88 * nctu; }
  __host__ __device__ int64_t nres() const { return (int64_t)16384 * nctu; }
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

// TU index and residual offset of TU t of CU (ctu, d, j)
__device__ __forceinline__ int ctu_tu_index(const CtuLayout &L, int ctu, int d, int j, int t) {
  const int n = L.nctu;
  if (d == 0) return ctu * 8 + t;
  if (d == 1) return ctu * 8 + 4 + j;
  if (d == 2) return 8 * n + ctu * 16 + j;
  return 24 * n + ctu * 64 + j;
}
__device__ __forceinline__ int64_t ctu_tu_offset(const CtuLayout &L, int tu) {
  const int64_t n = L.nctu;
  if (tu < 8 * n) return (int64_t)tu * 1024;
  if (tu < 24 * n) return 8 * n * 1024 + (int64_t)(tu - 8 * n) * 256;
  return 8 * n * 1024 + 16 * n * 256 + (int64_t)(tu - 24 * n) * 64;
}

__global__ void k_set_ptr(const uint8_t **slot, const uint8_t *p) { *slot = p; }

// one thread per (ctu, cu of this depth, ref)
__global__ __launch_bounds__(256) void k_ctu_me_jobs(CtuLayout L, hvx_ctu_params P, int depth,
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

// one wave per CU: best reference, luma MC (standard two-stage quarter-pel), residual into the
// TU-class layout, TU descriptors (hvxo_ctu_tu_desc semantics).
__global__ __launch_bounds__(64) void k_ctu_pred_resid(CtuLayout L, hvx_ctu_params P, const uint8_t *__restrict__ cur,
                                                       const uint8_t *const *__restrict__ refs, int stride,
                                                       const hvx_me_result *__restrict__ res, int16_t *__restrict__ resid,
                                                       hvx_tu_desc *__restrict__ descs, int64_t *__restrict__ offs,
                                                       int32_t *__restrict__ est_idx, hvx_cu_result *__restrict__ out,
                                                       int first, int ncu) {
  // blocks cover CUs [first, first + ncu) of every CTU (one depth range per launch)
  const int ctu = blockIdx.x / ncu, ci = first + (int)(blockIdx.x % ncu);
  const int cuid = ctu * HVX_CUS_PER_CTU + ci;
  int d, j, S, g;
  cu_geom(ci, d, j, S, g);
  const int x = (ctu % L.nctu_x) * 64 + (j % g) * S, y = (ctu / L.nctu_x) * 64 + (j / g) * S;
  const bool valid = x + S <= P.pic_w && y + S <= P.pic_h;
  const int T = S < 32 ? S : 32, log2 = T == 8 ? 3 : T == 16 ? 4 : 5, ntu = (S / T) * (S / T);
  int best = 0;
  uint32_t best_cost = 0;
  const hvx_me_result *r = res + (size_t)cuid * L.nref;
  if (valid) {
    for (int k = 0; k < L.nref; k++)
      if (k == 0 || r[k].cost < best_cost) { best_cost = r[k].cost; best = k; }
  }
  if (lane_id() == 0) {
    hvx_cu_result o;
    o.valid = valid; o.ref = valid ? best : 0;
    o.mv_x = valid ? r[best].mv_x : 0; o.mv_y = valid ? r[best].mv_y : 0;
    o.me_cost = valid ? best_cost : 0; o.sse = 0; o.abs_sum = 0; o.n_tu = valid ? ntu : 0;
    out[cuid] = o;
  }
  for (int t = lane_id(); t < ntu; t += HVX_WAVE) {
    const int tu = ctu_tu_index(L, ctu, d, j, t);
    hvx_tu_desc td;
    memset(&td, 0, sizeof(td));
    td.width = td.height = valid ? T : 0;  // width 0: no size class picks it up
    td.log2_size = log2;
    td.tr_idx = S > 32 ? 1 : 0;
    td.slice_type = P.slice_type;
    td.qp_per = P.qp / 6; td.qp_rem = P.qp % 6;
    td.sign_hiding = 1; td.use_rdoq = 1; td.use_rdoq_ts = 1;
    td.max_log2_tr_range = 15; td.bit_depth = 8;
    td.lambda = P.lambda;
    descs[tu] = td;
    offs[tu] = ctu_tu_offset(L, tu);
    est_idx[tu] = log2 - 2;
  }
  if (!valid) return;
  const uint8_t *rp = refs[best];
  const int mvx = r[best].mv_x, mvy = r[best].mv_y;
  for (int k = lane_id(); k < S * S; k += HVX_WAVE) {
    const int yy = k / S, xx = k % S;
    const int pred = me_qpel_sample(rp + y * stride + x, stride, xx, yy, mvx, mvy);
    const int t = (yy / T) * (S / T) + (xx / T);
    const int tu = ctu_tu_index(L, ctu, d, j, t);
    resid[ctu_tu_offset(L, tu) + (yy % T) * T + (xx % T)] = (int16_t)((int)cur[(y + yy) * stride + x + xx] - pred);
  }
}

__global__ __launch_bounds__(256) void k_ctu_finalize(CtuLayout L, const int32_t *__restrict__ abs_sum,
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
