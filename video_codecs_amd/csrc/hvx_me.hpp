// hvx_me.hpp -- uni-prediction motion estimation (gfx950): TZ integer search + half/quarter
// SATD refinement, i.e. TEncSearch::xMotionEstimation with bBi=false
// (TEncSearch.cpp:3663-3760; xTZSearch :3881 with TZ_SEARCH_CONFIGURATION :297-313,
// xTZSearchHelp :332, xTZ8PointDiamondSearch :629, xTZ2PointSearch :438,
// xSetSearchRange :3765, xPatternSearchFracDIF :4240, xPatternRefinement :808;
// TComDataCU::clipMv TComDataCU.cpp:2788; TComRdCost::getCost TComRdCost.h:172).
//
// Mapping: one 64-lane wave per (PU, reference) search job.  The PU's original block is
// staged once into LDS (8-bit); reference pixels stream from the 8-bit padded plane through
// L1/L2 (a 2160p plane is 9.4 MB: the 4 references of an LDP slice stay resident in the
// 256 MB Infinity Cache).  Every candidate SAD is a wave-wide sum (samples over lanes,
// shuffle all-reduce) so the TZ control flow stays wave-uniform and the candidates are
// visited in exactly the reference's order with its strict '<' tie-break -> identical MVs.
// Fractional refinement interpolates each candidate block into LDS with the reference's
// 16-bit two-stage arithmetic and takes an 8x8/4x4 Hadamard SATD across lanes.
#pragma once
#include "hvx_dev.hpp"

struct MeState {
  const uint8_t *org;  // LDS, stride 64
  const uint8_t *ref;  // PU origin at MV (0,0) in the reference plane
  int sr, w, h, sub;
  uint32_t lam;
  int px, py, cost_scale;
  int best_x, best_y, best_dist, best_round, point_nr;
  uint32_t best_sad;
};

struct MeRange { int l, r, t, b; };

__device__ __forceinline__ uint32_t me_mv_cost(const MeState &m, int x, int y) {
  const uint32_t bits = eg_bits((x << m.cost_scale) - m.px) + eg_bits((y << m.cost_scale) - m.py);
  return (m.lam * bits) >> 16;
}

__device__ __forceinline__ uint32_t me_sad(const MeState &m, int x, int y) {
  const uint8_t *r = m.ref + y * m.sr + x;
  const int w = m.w, rows = (m.h + (1 << m.sub) - 1) >> m.sub;
  uint32_t s = 0;
  for (int i = lane_id(); i < rows * w; i += HVX_WAVE) {
    const int yy = (i / w) << m.sub, xx = i - (i / w) * w;
    s += (uint32_t)abs((int)m.org[yy * 64 + xx] - (int)r[yy * m.sr + xx]);
  }
  return wave_sum_u32(s) << m.sub;
}

// xTZSearchHelp (:332), non-SELECTIVE branch
__device__ __forceinline__ void me_help(MeState &m, int x, int y, int pnr, int dist) {
  const uint32_t sad = me_sad(m, x, y) + me_mv_cost(m, x, y);
  if (sad < m.best_sad) { m.best_sad = sad; m.best_x = x; m.best_y = y; m.best_dist = dist; m.best_round = 0; m.point_nr = pnr; }
}

// xTZ2PointSearch (:438)
__device__ void me_2point(MeState &m, const MeRange &g) {
  const int sx = m.best_x, sy = m.best_y;
  switch (m.point_nr) {
    case 1: if (sx - 1 >= g.l) me_help(m, sx - 1, sy, 0, 2); if (sy - 1 >= g.t) me_help(m, sx, sy - 1, 0, 2); break;
    case 2: if (sy - 1 >= g.t) { if (sx - 1 >= g.l) me_help(m, sx - 1, sy - 1, 0, 2); if (sx + 1 <= g.r) me_help(m, sx + 1, sy - 1, 0, 2); } break;
    case 3: if (sy - 1 >= g.t) me_help(m, sx, sy - 1, 0, 2); if (sx + 1 <= g.r) me_help(m, sx + 1, sy, 0, 2); break;
    case 4: if (sx - 1 >= g.l) { if (sy + 1 <= g.b) me_help(m, sx - 1, sy + 1, 0, 2); if (sy - 1 >= g.t) me_help(m, sx - 1, sy - 1, 0, 2); } break;
    case 5: if (sx + 1 <= g.r) { if (sy - 1 >= g.t) me_help(m, sx + 1, sy - 1, 0, 2); if (sy + 1 <= g.b) me_help(m, sx + 1, sy + 1, 0, 2); } break;
    case 6: if (sx - 1 >= g.l) me_help(m, sx - 1, sy, 0, 2); if (sy + 1 <= g.b) me_help(m, sx, sy + 1, 0, 2); break;
    case 7: if (sy + 1 <= g.b) { if (sx - 1 >= g.l) me_help(m, sx - 1, sy + 1, 0, 2); if (sx + 1 <= g.r) me_help(m, sx + 1, sy + 1, 0, 2); } break;
    case 8: if (sx + 1 <= g.r) me_help(m, sx + 1, sy, 0, 2); if (sy + 1 <= g.b) me_help(m, sx, sy + 1, 0, 2); break;
    default: break;  // unreachable: the reference asserts here
  }
}

// xTZ8PointDiamondSearch (:629)
__device__ void me_diamond(MeState &m, const MeRange &g, int sx, int sy, int d) {
  const int top = sy - d, bottom = sy + d, left = sx - d, right = sx + d;
  m.best_round += 1;
  if (d == 1) {
    if (top >= g.t) me_help(m, sx, top, 2, d);
    if (left >= g.l) me_help(m, left, sy, 4, d);
    if (right <= g.r) me_help(m, right, sy, 5, d);
    if (bottom <= g.b) me_help(m, sx, bottom, 7, d);
    return;
  }
  const bool inside = top >= g.t && left >= g.l && right <= g.r && bottom <= g.b;
  if (d <= 8) {
    const int t2 = sy - (d >> 1), b2 = sy + (d >> 1), l2 = sx - (d >> 1), r2 = sx + (d >> 1);
    if (inside) {
      me_help(m, sx, top, 2, d);
      me_help(m, l2, t2, 1, d >> 1);
      me_help(m, r2, t2, 3, d >> 1);
      me_help(m, left, sy, 4, d);
      me_help(m, right, sy, 5, d);
      me_help(m, l2, b2, 6, d >> 1);
      me_help(m, r2, b2, 8, d >> 1);
      me_help(m, sx, bottom, 7, d);
    } else {
      if (top >= g.t) me_help(m, sx, top, 2, d);
      if (t2 >= g.t) { if (l2 >= g.l) me_help(m, l2, t2, 1, d >> 1); if (r2 <= g.r) me_help(m, r2, t2, 3, d >> 1); }
      if (left >= g.l) me_help(m, left, sy, 4, d);
      if (right <= g.r) me_help(m, right, sy, 5, d);
      if (b2 <= g.b) { if (l2 >= g.l) me_help(m, l2, b2, 6, d >> 1); if (r2 <= g.r) me_help(m, r2, b2, 8, d >> 1); }
      if (bottom <= g.b) me_help(m, sx, bottom, 7, d);
    }
  } else {
    const int q = d >> 2;
    if (inside) {
      me_help(m, sx, top, 0, d);
      me_help(m, left, sy, 0, d);
      me_help(m, right, sy, 0, d);
      me_help(m, sx, bottom, 0, d);
      for (int i = 1; i < 4; i++) {
        const int yt = top + q * i, yb = bottom - q * i, xl = sx - q * i, xr = sx + q * i;
        me_help(m, xl, yt, 0, d);
        me_help(m, xr, yt, 0, d);
        me_help(m, xl, yb, 0, d);
        me_help(m, xr, yb, 0, d);
      }
    } else {
      if (top >= g.t) me_help(m, sx, top, 0, d);
      if (left >= g.l) me_help(m, left, sy, 0, d);
      if (right <= g.r) me_help(m, right, sy, 0, d);
      if (bottom <= g.b) me_help(m, sx, bottom, 0, d);
      for (int i = 1; i < 4; i++) {
        const int yt = top + q * i, yb = bottom - q * i, xl = sx - q * i, xr = sx + q * i;
        if (yt >= g.t) { if (xl >= g.l) me_help(m, xl, yt, 0, d); if (xr <= g.r) me_help(m, xr, yt, 0, d); }
        if (yb <= g.b) { if (xl >= g.l) me_help(m, xl, yb, 0, d); if (xr <= g.r) me_help(m, xr, yb, 0, d); }
      }
    }
  }
}

// TComDataCU::clipMv: quarter-pel, result stored as Short
__device__ __forceinline__ void me_clip(const hvx_me_job &j, int &mx, int &my) {
  const int hmax = (j.pic_w + 8 - j.cu_x - 1) << 2, hmin = (-j.max_cu - 8 - j.cu_x + 1) << 2;
  const int vmax = (j.pic_h + 8 - j.cu_y - 1) << 2, vmin = (-j.max_cu - 8 - j.cu_y + 1) << 2;
  mx = (int16_t)(mx < hmin ? hmin : mx > hmax ? hmax : mx);
  my = (int16_t)(my < vmin ? vmin : my > vmax ? vmax : my);
}

__device__ __forceinline__ MeRange me_search_range(const hvx_me_job &j, int px, int py, int sr) {
  int cx = px, cy = py;
  me_clip(j, cx, cy);
  int lx = cx - (sr << 2), ly = cy - (sr << 2), rx = cx + (sr << 2), ry = cy + (sr << 2);
  me_clip(j, lx, ly);
  me_clip(j, rx, ry);
  MeRange g;
  g.l = lx >> 2; g.t = ly >> 2; g.r = rx >> 2; g.b = ry >> 2;
  return g;
}

// Quarter-sample luma sample at (x,y) + quarter-pel (qx,qy); standard two-stage 8-bit path.
__device__ __forceinline__ int me_qpel_sample(const uint8_t *ref, int sr, int x, int y, int qx, int qy) {
  const int fx = qx & 3, fy = qy & 3;
  const uint8_t *p = ref + (y + (qy >> 2)) * sr + x + (qx >> 2);
  if (!fx && !fy) return p[0];
  if (!fy) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += kLumaFilter[fx][k] * p[k - 3];
    return clip_pel((s + 32) >> 6);
  }
  if (!fx) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += kLumaFilter[fy][k] * p[(k - 3) * sr];
    return clip_pel((s + 32) >> 6);
  }
  int s2 = 0;
#pragma unroll
  for (int t = 0; t < 8; t++) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += kLumaFilter[fx][k] * p[(t - 3) * sr + k - 3];
    s2 += kLumaFilter[fy][t] * (int16_t)(s - 8192);
  }
  return clip_pel((s2 + (1 << 11) + (8192 << 6)) >> 12);
}

// xPatternRefinement (:808): 9 candidates around base (quarter-pel, relative to MV 0)
// s_acMvRefineH / s_acMvRefineQ (TEncSearch.cpp:51-75)
__constant__ int8_t kRefH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
__constant__ int8_t kRefQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

__device__ uint32_t me_refine(MeState &m, int16_t *blk, bool had, int bqx, int bqy, int frac, int &fx, int &fy) {
  uint32_t best = 0xFFFFFFFFu;
  int bi = 0;
  for (int i = 0; i < 9; i++) {
    const int dx = frac == 2 ? kRefH[i][0] : kRefQ[i][0], dy = frac == 2 ? kRefH[i][1] : kRefQ[i][1];
    const int qx = bqx + dx * frac, qy = bqy + dy * frac;
    __syncthreads();
    for (int k = lane_id(); k < m.w * m.h; k += HVX_WAVE) {
      const int y = k / m.w, x = k - y * m.w;
      blk[y * 64 + x] = (int16_t)me_qpel_sample(m.ref, m.sr, x, y, qx, qy);
    }
    __syncthreads();
    uint32_t d;
    if (had) {
      d = wave_satd(m.org, 64, blk, 64, m.w, m.h);
    } else {
      uint32_t s = 0;
      for (int k = lane_id(); k < m.w * m.h; k += HVX_WAVE) {
        const int y = k / m.w, x = k - y * m.w;
        s += (uint32_t)abs((int)m.org[y * 64 + x] - (int)blk[y * 64 + x]);
      }
      d = wave_sum_u32(s);
    }
    d += me_mv_cost(m, dx + fx, dy + fy);
    if (d < best) { best = d; bi = i; }
  }
  fx = frac == 2 ? kRefH[bi][0] : kRefQ[bi][0];
  fy = frac == 2 ? kRefH[bi][1] : kRefQ[bi][1];
  return best;
}

// one whole xMotionEstimation for job j by the calling wave; writes *out (lane 0)
__device__ void me_run(const hvx_me_job &j, const uint8_t *const *__restrict__ cur_planes,
                       const uint8_t *const *__restrict__ ref_planes, int stride, uint8_t *org, int16_t *blk,
                       hvx_me_result *out) {
  if (j.w <= 0 || j.h <= 0) {  // empty slot (e.g. a CU outside the picture): defined zero result
    if (lane_id() == 0) { hvx_me_result z; memset(&z, 0, sizeof(z)); *out = z; }
    return;
  }
  const uint8_t *cur = cur_planes[j.cur_idx] + j.pu_y * stride + j.pu_x;
  for (int k = lane_id(); k < j.w * j.h; k += HVX_WAVE) {
    const int y = k / j.w, x = k - y * j.w;
    org[y * 64 + x] = cur[y * stride + x];
  }
  __syncthreads();
  MeState m;
  m.org = org;
  m.ref = ref_planes[j.ref_idx] + j.pu_y * stride + j.pu_x;
  m.sr = stride; m.w = j.w; m.h = j.h;
  m.sub = ((j.flags & HVX_ME_FEN) && j.h > 8) ? 1 : 0;
  {
    const int w = j.w;
    const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
    if (!spec) m.sub = 0;
  }
  m.lam = j.lambda_motion;
  m.px = j.pred_x; m.py = j.pred_y;
  m.cost_scale = 2;
  const int sr = j.search_range;
  const MeRange g0 = me_search_range(j, j.pred_x, j.pred_y, sr);

  // ---- xTZSearch ----
  int mx = j.pred_x, my = j.pred_y;
  me_clip(j, mx, my);
  mx >>= 2; my >>= 2;
  m.best_sad = 0xFFFFFFFFu;
  m.best_x = m.best_y = 0; m.best_dist = 0; m.best_round = 0; m.point_nr = 0;
  me_help(m, mx, my, 0, 0);
  me_help(m, 0, 0, 0, 0);
  MeRange g = g0;
  if (j.use_int2nx2n) {
    int ix = j.i2_x << 2, iy = j.i2_y << 2;
    me_clip(j, ix, iy);
    me_help(m, ix >> 2, iy >> 2, 0, 0);
    g = me_search_range(j, m.best_x << 2, m.best_y << 2, sr);
  }
  int sx = m.best_x, sy = m.best_y;
  for (int d = 1; d <= sr; d *= 2) {
    me_diamond(m, g0, sx, sy, d);
    if ((j.flags & HVX_ME_SMOOTHMV) && m.best_round >= 3) break;
  }
  if (m.best_dist == 1) { m.best_dist = 0; me_2point(m, g0); }
  if (m.best_dist > 5) {
    m.best_dist = 5;
    for (sy = g.t; sy <= g.b; sy += 5)
      for (sx = g.l; sx <= g.r; sx += 5) me_help(m, sx, sy, 0, 5);
  }
  while (m.best_dist > 0) {
    sx = m.best_x; sy = m.best_y;
    m.best_dist = 0; m.point_nr = 0;
    for (int d = 1; d < sr + 1; d *= 2) me_diamond(m, g0, sx, sy, d);
    if (m.best_dist == 1) {
      m.best_dist = 0;
      if (m.point_nr != 0) me_2point(m, g0);
    }
  }
  const int ix = m.best_x, iy = m.best_y;
  const uint32_t sad_int = m.best_sad - me_mv_cost(m, ix, iy);

  // ---- xPatternSearchFracDIF ----
  const bool had = (j.flags & HVX_ME_HADME) != 0;
  m.cost_scale = 1;
  int hx = ix << 1, hy = iy << 1;
  me_refine(m, blk, had, ix << 2, iy << 2, 2, hx, hy);
  m.cost_scale = 0;
  int qx = ((ix << 1) + hx) << 1, qy = ((iy << 1) + hy) << 1;
  const uint32_t cost = me_refine(m, blk, had, (ix << 2) + (hx << 1), (iy << 2) + (hy << 1), 1, qx, qy);
  const int fmx = (ix << 2) + (hx << 1) + qx, fmy = (iy << 2) + (hy << 1) + qy;
  const uint32_t mv_bits = eg_bits(fmx - m.px) + eg_bits(fmy - m.py);
  const uint32_t bits = (uint32_t)j.bits_in + mv_bits;
  if (lane_id() == 0) {
    hvx_me_result r;
    r.mv_int_x = ix; r.mv_int_y = iy; r.sad_int = sad_int;
    r.half_x = hx; r.half_y = hy; r.qtr_x = qx; r.qtr_y = qy; r.cost_frac = cost;
    r.mv_x = fmx; r.mv_y = fmy; r.bits = bits;
    r.cost = (uint32_t)(floor(1.0 * ((double)cost - (double)((m.lam * mv_bits) >> 16))) + (double)((m.lam * bits) >> 16));
    *out = r;
  }
}

__global__ __launch_bounds__(64) void k_me(const uint8_t *const *__restrict__ cur_planes,
                                          const uint8_t *const *__restrict__ ref_planes, int stride,
                                          const hvx_me_job *__restrict__ jobs, int n, hvx_me_result *__restrict__ out) {
  __shared__ uint8_t org[64 * 64];
  __shared__ int16_t blk[64 * 64];
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_me_job j = jobs[jid];
  me_run(j, cur_planes, ref_planes, stride, org, blk, out + jid);
}

// CTU-pass view: block b = (ctu * ncu + cu) * nref + ref of one depth -> job slot
// ((ctu * 85 + first + cu) * nref + ref)
__global__ __launch_bounds__(64) void k_me_ctu_depth(const uint8_t *const *__restrict__ cur_planes,
                                                    const uint8_t *const *__restrict__ ref_planes, int stride,
                                                    const hvx_me_job *__restrict__ jobs, hvx_me_result *__restrict__ out,
                                                    int nref, int ncu, int first) {
  __shared__ uint8_t org[64 * 64];
  __shared__ int16_t blk[64 * 64];
  const int b = blockIdx.x;
  const int ref = b % nref, cu = (b / nref) % ncu, ctu = b / (nref * ncu);
  const size_t slot = ((size_t)ctu * HVX_CUS_PER_CTU + first + cu) * nref + ref;
  const hvx_me_job j = jobs[slot];
  me_run(j, cur_planes, ref_planes, stride, org, blk, out + slot);
}
