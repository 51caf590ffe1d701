// hvx_deblock.hpp -- deblocking of a reconstructed picture (gfx950); SURVEY.md 8(f) item 3.
// Restated by oracle/hvx_oracle.c ("Deblocking"); TComLoopFilter::loopFilterPic
// (TComLoopFilter.cpp:130) on given boundary-strength / QP maps (hvx_types.h hvx_deblock_params).
//
// Two launches, exactly the reference's two sweeps: every vertical edge of the picture, then every
// horizontal edge of that result.  Inside a sweep the edges are 8 samples apart and a filter
// reads 4 and writes at most 3 samples on each side, so all edge segments of a sweep are
// independent: one THREAD per 4-line luma segment (plus, on the 16-sample grid with bs 2, the 2
// chroma lines of Cb and Cr it covers).  Lanes walk along the edge direction's perpendicular
// (vertical edges: consecutive edges of one row band; horizontal edges: consecutive 4-column
// groups), so a wave's row accesses are contiguous.
#pragma once
#include "hvx_dev.hpp"

namespace dbk {
static __constant__ uint8_t kTc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};
static __constant__ uint8_t kBeta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                  34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static __constant__ uint8_t kCScale[58] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19,
                                    20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33, 34, 34, 35, 35,
                                    36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51};

// xEdgeFilterLuma's 4-line segment (TComLoopFilter.cpp:605-675): s = q0 of line 0
__device__ __forceinline__ void luma_seg(uint8_t *s, int step, int off, int bs, int qp, int beta_off, int tc_off) {
  const int tc = kTc[clip3(0, 53, qp + 2 * (bs - 1) + 2 * tc_off)];
  const int beta = kBeta[clip3(0, 51, qp + 2 * beta_off)];
  const int side = (beta + (beta >> 1)) >> 3, thr_cut = tc * 10;
  int m[4][8];  // lines 0..3, samples p3..q3
#pragma unroll
  for (int l = 0; l < 4; l++)
#pragma unroll
    for (int i = 0; i < 8; i++) m[l][i] = s[l * step + (i - 4) * off];
  const int dp0 = abs(m[0][1] - 2 * m[0][2] + m[0][3]), dq0 = abs(m[0][4] - 2 * m[0][5] + m[0][6]);
  const int dp3 = abs(m[3][1] - 2 * m[3][2] + m[3][3]), dq3 = abs(m[3][4] - 2 * m[3][5] + m[3][6]);
  const int d0 = dp0 + dq0, d3 = dp3 + dq3, d = d0 + d3;
  if (d >= beta) return;
  const bool fp = dp0 + dp3 < side, fq = dq0 + dq3 < side;
  const bool sw = (abs(m[0][0] - m[0][3]) + abs(m[0][7] - m[0][4]) < (beta >> 3)) && (2 * d0 < (beta >> 2)) &&
                  (abs(m[0][3] - m[0][4]) < ((tc * 5 + 1) >> 1)) &&
                  (abs(m[3][0] - m[3][3]) + abs(m[3][7] - m[3][4]) < (beta >> 3)) && (2 * d3 < (beta >> 2)) &&
                  (abs(m[3][3] - m[3][4]) < ((tc * 5 + 1) >> 1));
#pragma unroll
  for (int l = 0; l < 4; l++) {
    const int m0 = m[l][0], m1 = m[l][1], m2 = m[l][2], m3 = m[l][3], m4 = m[l][4], m5 = m[l][5], m6 = m[l][6],
              m7 = m[l][7];
    uint8_t *q = s + l * step;
    if (sw) {  // xPelFilterLuma (:833-854)
      q[-off] = (uint8_t)clip3(m3 - 2 * tc, m3 + 2 * tc, (m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3);
      q[0] = (uint8_t)clip3(m4 - 2 * tc, m4 + 2 * tc, (m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3);
      q[-2 * off] = (uint8_t)clip3(m2 - 2 * tc, m2 + 2 * tc, (m1 + m2 + m3 + m4 + 2) >> 2);
      q[off] = (uint8_t)clip3(m5 - 2 * tc, m5 + 2 * tc, (m3 + m4 + m5 + m6 + 2) >> 2);
      q[-3 * off] = (uint8_t)clip3(m1 - 2 * tc, m1 + 2 * tc, (2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3);
      q[2 * off] = (uint8_t)clip3(m6 - 2 * tc, m6 + 2 * tc, (m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3);
    } else {  // weak filter (:855-877)
      int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
      if (abs(delta) < thr_cut) {
        delta = clip3(-tc, tc, delta);
        q[-off] = (uint8_t)clip_pel(m3 + delta);
        q[0] = (uint8_t)clip_pel(m4 - delta);
        const int tc2 = tc >> 1;
        if (fp) q[-2 * off] = (uint8_t)clip_pel(m2 + clip3(-tc2, tc2, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
        if (fq) q[off] = (uint8_t)clip_pel(m5 + clip3(-tc2, tc2, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
      }
    }
  }
}

// xEdgeFilterChroma's part of one luma unit (:750-815): 2 lines of one chroma plane, bs 2
__device__ __forceinline__ void chroma_seg(uint8_t *s, int step, int off, int bs, int qp_avg, int qp_offset,
                                           int tc_off) {
  int qp = qp_avg + qp_offset;
  if (qp >= 58) qp -= 6;
  else if (qp >= 0) qp = kCScale[qp];
  const int tc = kTc[clip3(0, 53, qp + 2 * (bs - 1) + 2 * tc_off)];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    uint8_t *q = s + l * step;
    const int m2 = q[-2 * off], m3 = q[-off], m4 = q[0], m5 = q[off];
    const int delta = clip3(-tc, tc, ((((m4 - m3) << 2) + m2 - m5 + 4) >> 3));
    q[-off] = (uint8_t)clip_pel(m3 + delta);
    q[0] = (uint8_t)clip_pel(m4 - delta);
  }
}
}  // namespace dbk

// DIR 0: vertical edges x = 8, 16, ..; thread (uy, e).  DIR 1: horizontal edges y = 8, 16, ..; thread (e, ux).
template <int DIR>
static __global__ __launch_bounds__(256) void k_deblock(uint8_t *__restrict__ y, int ys, uint8_t *__restrict__ cb,
                                                 uint8_t *__restrict__ cr, int cs, const uint8_t *__restrict__ bsm,
                                                 const int8_t *__restrict__ qp, hvx_deblock_params p) {
  using namespace dbk;
  const int uw = p.pic_w >> 2, uh = p.pic_h >> 2;
  const int ne = (DIR == 0 ? p.pic_w : p.pic_h) / 8 - 1;  // interior edges (the picture border is never filtered)
  const int along = DIR == 0 ? uh : uw;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ne * along) return;
  const int e = DIR == 0 ? t % ne + 1 : t / along + 1, a = DIR == 0 ? t / ne : t % along;
  const int ux = DIR == 0 ? 2 * e : a, uy = DIR == 0 ? a : 2 * e;
  const int bs = bsm[uy * uw + ux];
  if (!bs) return;
  const int qq = qp[uy * uw + ux], qpp = DIR == 0 ? qp[uy * uw + ux - 1] : qp[(uy - 1) * uw + ux];
  const int avg = (qpp + qq + 1) >> 1;
  const int x = ux * 4, yy = uy * 4;
  if (DIR == 0) luma_seg(y + (int64_t)yy * ys + x, ys, 1, bs, avg, p.beta_offset_div2, p.tc_offset_div2);
  else luma_seg(y + (int64_t)yy * ys + x, 1, ys, bs, avg, p.beta_offset_div2, p.tc_offset_div2);
  if (cb && bs == 2 && (e & 1) == 0) {  // the 16-sample luma grid = the 8-sample chroma grid (cb NULL: luma only)
    const int64_t o = (int64_t)(yy / 2) * cs + x / 2;
    if (DIR == 0) {
      chroma_seg(cb + o, cs, 1, bs, avg, p.cb_qp_offset, p.tc_offset_div2);
      chroma_seg(cr + o, cs, 1, bs, avg, p.cr_qp_offset, p.tc_offset_div2);
    } else {
      chroma_seg(cb + o, 1, cs, bs, avg, p.cb_qp_offset, p.tc_offset_div2);
      chroma_seg(cr + o, 1, cs, bs, avg, p.cr_qp_offset, p.tc_offset_div2);
    }
  }
}
