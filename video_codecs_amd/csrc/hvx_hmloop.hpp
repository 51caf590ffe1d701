// hvx_hmloop.hpp -- the picture-level steps after TEncSlice::compressSlice on a picture the
// HM-exact engine decided (hvx_hm_finish_picture, include/hvx.h): the deblocking filter's inputs
// derived from the CTU data on the device, TComPic::compressMotion's collocated field, and the
// reference planes with extended borders the next pictures' searches read.
//
// Every kernel here is one thread per output element (a 4x4 unit, a 16x16 block, a sample): the
// work is a gather over the picture's CTU records / samples, HBM-bound and a few microseconds at
// 2160p -- no LDS staging, no wave-level cooperation.
#pragma once
#include "hvx_dev.hpp"

namespace hvxi {

// the slice facts the boundary strength needs (hvx_hm_picture subset)
struct LfPic {
  int w, h, wc, is_b;
  int ref_poc[2][4];
};

// g_auiRasterToZscan of the 4x4 unit (ux, uy) of a CTU: x bits interleaved below y bits
__device__ __forceinline__ int lf_unit_z(int ux, int uy) {
  int z = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) z |= (((ux >> b) & 1) << (2 * b)) | (((uy >> b) & 1) << (2 * b + 1));
  return z;
}
__device__ __forceinline__ const hvx_hm_part *lf_part(const hvx_hm_ctu *ctus, int wc, int x, int y) {
  return &ctus[(y >> 6) * wc + (x >> 6)].p[lf_unit_z((x & 63) >> 2, (y & 63) >> 2)];
}
// TComSlice::getRefPic of list l as the picture's identity (its POC); INT_MIN = NULL
__device__ __forceinline__ int lf_ref(const hvx_hm_part *q, const LfPic &P, int l) {
  const int r = q->ref[l];
  return r < 0 ? INT_MIN : P.ref_poc[l][r & 3];
}
__device__ __forceinline__ bool lf_far(int ax, int ay, int bx, int by) { return abs(ax - bx) >= 4 || abs(ay - by) >= 4; }

// The boundary strength loopFilterPic gives the left (dir 0) / top (dir 1) edge of the unit at luma
// (x, y): xDeblockCU's edge marking (TComLoopFilter.cpp:170-218) -- xSetEdgefilterTU (:274) marks
// every TU's left / top edge as a transform edge, xSetEdgefilterPU (:299) the CU's own edge
// (bLeftEdge / bTopEdge of xSetLoopfilterParam :362: inside the picture, LFCrossSliceBoundaryFlag
// on) and the partition's internal PU edges -- then xGetBoundaryStrengthSingle (:417).  Only the
// 8x8 grid is filtered (xEdgeFilterLuma's iEdge step, :220): 0 elsewhere.
__device__ int lf_bs(const hvx_hm_ctu *ctus, const LfPic &P, int x, int y, int dir) {
  if (dir == 0 ? (x & 7) || x == 0 : (y & 7) || y == 0) return 0;
  const hvx_hm_part *q = lf_part(ctus, P.wc, x, y);
  const int cs = 64 >> q->depth;
  const int r = (dir == 0 ? (x & 63) : (y & 63)) & (cs - 1);  // offset inside the CU across the edge
  const bool tu_edge = (r & ((cs >> q->tr_idx) - 1)) == 0;
  bool pu_edge = false;
  switch (q->part) {
    case 1: pu_edge = dir == 1 && r == cs / 2; break;       // SIZE_2NxN
    case 2: pu_edge = dir == 0 && r == cs / 2; break;       // SIZE_Nx2N
    case 3: pu_edge = r == cs / 2; break;                   // SIZE_NxN
    case 4: pu_edge = dir == 1 && r == cs / 4; break;       // SIZE_2NxnU
    case 5: pu_edge = dir == 1 && r == cs - cs / 4; break;  // SIZE_2NxnD
    case 6: pu_edge = dir == 0 && r == cs / 4; break;       // SIZE_nLx2N
    case 7: pu_edge = dir == 0 && r == cs - cs / 4; break;  // SIZE_nRx2N
    default: break;
  }
  if (!tu_edge && !pu_edge) return 0;
  const hvx_hm_part *p = dir == 0 ? lf_part(ctus, P.wc, x - 4, y) : lf_part(ctus, P.wc, x, y - 4);
  if (p->pred == 1 || q->pred == 1) return 2;  // MODE_INTRA
  if (tu_edge && (((q->cbf[0] >> q->tr_idx) & 1) || ((p->cbf[0] >> p->tr_idx) & 1))) return 1;
  int rp[2], rq[2], mp[2][2], mq[2][2];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    rp[l] = lf_ref(p, P, l);
    rq[l] = lf_ref(q, P, l);
#pragma unroll
    for (int c = 0; c < 2; c++) {
      mp[l][c] = rp[l] == INT_MIN ? 0 : p->mv[l][c];
      mq[l][c] = rq[l] == INT_MIN ? 0 : q->mv[l][c];
    }
  }
  if (!P.is_b) return (rp[0] != rq[0] || lf_far(mq[0][0], mq[0][1], mp[0][0], mp[0][1])) ? 1 : 0;
  const bool s00 = lf_far(mq[0][0], mq[0][1], mp[0][0], mp[0][1]) || lf_far(mq[1][0], mq[1][1], mp[1][0], mp[1][1]);
  const bool s10 = lf_far(mq[1][0], mq[1][1], mp[0][0], mp[0][1]) || lf_far(mq[0][0], mq[0][1], mp[1][0], mp[1][1]);
  if ((rp[0] == rq[0] && rp[1] == rq[1]) || (rp[0] == rq[1] && rp[1] == rq[0])) {
    if (rp[0] != rp[1]) return (rp[0] == rq[0] ? s00 : s10) ? 1 : 0;
    return (s00 && s10) ? 1 : 0;
  }
  return 1;
}

// one thread per 4x4 luma unit: bs_ver, bs_hor, QpY ((w/4) x (h/4) raster maps of hvx_deblock)
__global__ void k_hm_lf_params(const hvx_hm_ctu *ctus, LfPic P, uint8_t *bs_ver, uint8_t *bs_hor, int8_t *qp) {
  const int uw = P.w >> 2, n = uw * (P.h >> 2);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int x = (i % uw) * 4, y = (i / uw) * 4;
  bs_ver[i] = (uint8_t)lf_bs(ctus, P, x, y, 0);
  bs_hor[i] = (uint8_t)lf_bs(ctus, P, x, y, 1);
  qp[i] = lf_part(ctus, P.wc, x, y)->qp;
}

// TComPic::compressMotion (TComDataCU::compressMV): per CTU and 16x16 block (z-order) the motion of
// its first 4x4 unit -- the hvx_hm_picture.col_field rows {pred mode (-1 outside the picture), ref
// idx L0, L1, MV L0 x, y, L1 x, y, 0}
__global__ void k_hm_col_field(const hvx_hm_ctu *ctus, int w, int h, int wc, int nctu, int16_t *col) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nctu * 16) return;
  const int a = i >> 4, b = i & 15;
  const int bx = (b & 1) | ((b >> 1) & 2), by = ((b >> 1) & 1) | ((b >> 2) & 2);
  const int x = (a % wc) * 64 + bx * 16, y = (a / wc) * 64 + by * 16;
  const hvx_hm_part &q = ctus[a].p[b * 16];
  int16_t *o = col + (size_t)i * 8;
  o[0] = (x >= w || y >= h) ? (int16_t)-1 : (int16_t)q.pred;
  o[1] = q.ref[0];
  o[2] = q.ref[1];
  o[3] = q.mv[0][0];
  o[4] = q.mv[0][1];
  o[5] = q.mv[1][0];
  o[6] = q.mv[1][1];
  o[7] = 0;
}

// TComPicYuv::extendPicBorder of a reconstructed plane into a reference plane: every sample of the
// w x h plane plus `m` on each side, sample (x, y) = rec(clamp(x), clamp(y)), widened to T.
// blockIdx.y = output row (-m .. h+m-1), x across threads.
template <typename T>
__global__ void k_ref_plane(const uint8_t *rec, int rec_stride, int w, int h, int m, T *dst, int dst_stride) {
  const int ox = blockIdx.x * blockDim.x + threadIdx.x - m, oy = (int)blockIdx.y - m;
  if (ox >= w + m) return;
  const int sx = ox < 0 ? 0 : ox >= w ? w - 1 : ox, sy = oy < 0 ? 0 : oy >= h ? h - 1 : oy;
  dst[(ptrdiff_t)oy * dst_stride + ox] = (T)rec[(size_t)sy * rec_stride + sx];
}

}  // namespace hvxi
