// hvx_sao.hpp -- sample adaptive offset on a deblocked picture (gfx950); SURVEY.md 8(f) item 3.
// Restated by oracle/hvx_oracle.c ("SAO"); TEncSampleAdaptiveOffset::getStatistics/getBlkStats
// (TEncSampleAdaptiveOffset.cpp:285, 892) and TComSampleAdaptiveOffset::offsetCTU/offsetBlock
// (TComSampleAdaptiveOffset.cpp:313, 554), single slice and tile, 8-bit 4:2:0.
//
// Statistics: one workgroup per (CTU, component).  A thread takes 4 horizontally adjacent
// samples per step (one dword of the reconstruction row plus the row above and below), finds
// the edge class of every type and the band, and adds (org - rec, 1) into per-type LDS
// histograms with LDS atomics (int32: at most 64*64 samples of |d| <= 255 per CTU); the
// workgroup then widens them to the int64 SAOStatData layout.  Application: one thread per
// 4 output samples, reading the unmodified input picture (src != dst) so that CTUs are
// independent -- the reference's copy of the deblocked picture (SAOProcess :246-249).
#pragma once
#include "hvx_dev.hpp"

namespace sao {
__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// edge class (edge type + 2) of type t at p: the two neighbours of EO_0/90/135/45
__device__ __forceinline__ int edge(const uint8_t *p, int s, int t) {
  const int c = p[0];
  int a, b;
  if (t == 0) { a = p[-1]; b = p[1]; }
  else if (t == 1) { a = p[-s]; b = p[s]; }
  else if (t == 2) { a = p[-s - 1]; b = p[s + 1]; }
  else { a = p[-s + 1]; b = p[s - 1]; }
  return sgn(c - a) + sgn(c - b) + 2;
}

struct Blk {
  int x0, y0, bw, bh, L, A, R, B;
};
__device__ __forceinline__ Blk block(int ctu, int ncx, int w, int h, int cs) {
  Blk b;
  const int cx = ctu % ncx, cy = ctu / ncx;
  b.x0 = cx * cs; b.y0 = cy * cs;
  b.bw = min(cs, w - b.x0); b.bh = min(cs, h - b.y0);
  b.L = cx > 0; b.A = cy > 0; b.R = b.x0 + cs < w; b.B = b.y0 + cs < h;
  return b;
}
}  // namespace sao

// grid (nctu, ncomp); 256 threads.  out: [ctu][3][5] hvx_sao_stat
__global__ __launch_bounds__(256) void k_sao_stats(const uint8_t *__restrict__ org_y, const uint8_t *__restrict__ org_cb,
                                                  const uint8_t *__restrict__ org_cr, int os_y, int os_c,
                                                  const uint8_t *__restrict__ rec_y, const uint8_t *__restrict__ rec_cb,
                                                  const uint8_t *__restrict__ rec_cr, int rs_y, int rs_c, int pic_w,
                                                  int pic_h, hvx_sao_stat *__restrict__ out) {
  using namespace sao;
  __shared__ int hist[HVX_SAO_TYPES][2][HVX_SAO_CLASSES];
  const int comp = blockIdx.y, ctu = blockIdx.x;
  const int cs = comp ? 32 : 64, w = comp ? pic_w >> 1 : pic_w, h = comp ? pic_h >> 1 : pic_h;
  const int skr = comp ? 3 : 5, skb = comp ? 2 : 4;  // m_skipLinesR/B (createEncData :125-131)
  const uint8_t *org = comp == 0 ? org_y : comp == 1 ? org_cb : org_cr;
  const uint8_t *rec = comp == 0 ? rec_y : comp == 1 ? rec_cb : rec_cr;
  const int os = comp ? os_c : os_y, rs = comp ? rs_c : rs_y;
  const int ncx = (pic_w + 63) >> 6;
  for (int i = threadIdx.x; i < HVX_SAO_TYPES * 2 * HVX_SAO_CLASSES; i += 256) (&hist[0][0][0])[i] = 0;
  __syncthreads();
  const Blk b = block(ctu, ncx, w, h, cs);
  // per type: [xs, xe) x [ys, ye) (getBlkStats :941, 989, 1051, 1140, 1229)
  int xs[5], xe[5], ys[5], ye[5];
  xs[4] = 0; xe[4] = b.R ? b.bw - skr : b.bw; ys[4] = 0; ye[4] = b.B ? b.bh - skb : b.bh;
  xs[0] = b.L ? 0 : 1; xe[0] = b.R ? b.bw - skr : b.bw - 1; ys[0] = 0; ye[0] = ye[4];
  xs[1] = 0; xe[1] = xe[4]; ys[1] = b.A ? 0 : 1; ye[1] = b.B ? b.bh - skb : b.bh - 1;
  xs[2] = xs[3] = xs[0]; xe[2] = xe[3] = xe[0]; ys[2] = ys[3] = ys[1]; ye[2] = ye[3] = ye[1];
  const int nq = (b.bw + 3) >> 2;  // 4-sample groups per row
  for (int q = threadIdx.x; q < nq * b.bh; q += 256) {
    const int y = q / nq, xg = (q - y * nq) * 4;
    const uint8_t *rr = rec + (size_t)(b.y0 + y) * rs + b.x0;
    const uint8_t *orow = org + (size_t)(b.y0 + y) * os + b.x0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int x = xg + i;
      if (x >= b.bw) break;
      const uint8_t *p = rr + x;
      const int d = (int)orow[x] - (int)p[0];
#pragma unroll
      for (int t = 0; t < 5; t++) {
        if (x >= xs[t] && x < xe[t] && y >= ys[t] && y < ye[t]) {
          const int k = t == 4 ? p[0] >> 3 : edge(p, rs, t);
          atomicAdd(&hist[t][0][k], d);
          atomicAdd(&hist[t][1][k], 1);
        }
      }
    }
  }
  __syncthreads();
  hvx_sao_stat *st = out + ((size_t)ctu * 3 + comp) * HVX_SAO_TYPES;
  for (int i = threadIdx.x; i < HVX_SAO_TYPES * 2 * HVX_SAO_CLASSES; i += 256) {
    const int t = i / (2 * HVX_SAO_CLASSES), r = i % (2 * HVX_SAO_CLASSES);
    const int64_t v = (&hist[0][0][0])[i];
    if (r < HVX_SAO_CLASSES) st[t].diff[r] = v;
    else st[t].count[r - HVX_SAO_CLASSES] = v;
  }
}

// grid-stride over every 4-sample group of the plane comp = blockIdx.y; dst = src with offsets
__global__ __launch_bounds__(256) void k_sao_apply(const uint8_t *__restrict__ src_y, const uint8_t *__restrict__ src_cb,
                                                  const uint8_t *__restrict__ src_cr, int ss_y, int ss_c,
                                                  uint8_t *__restrict__ dst_y, uint8_t *__restrict__ dst_cb,
                                                  uint8_t *__restrict__ dst_cr, int ds_y, int ds_c, int pic_w, int pic_h,
                                                  const hvx_sao_ctu *__restrict__ params) {
  using namespace sao;
  const int comp = blockIdx.y;
  const int cs = comp ? 32 : 64, w = comp ? pic_w >> 1 : pic_w, h = comp ? pic_h >> 1 : pic_h;
  const uint8_t *src = comp == 0 ? src_y : comp == 1 ? src_cb : src_cr;
  uint8_t *dst = comp == 0 ? dst_y : comp == 1 ? dst_cb : dst_cr;
  const int ss = comp ? ss_c : ss_y, ds = comp ? ds_c : ds_y;
  const int ncx = (pic_w + 63) >> 6, nq = (w + 3) >> 2;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq * h; q += gridDim.x * blockDim.x) {
    const int y = q / nq, xg = (q - y * nq) * 4;
    const int ctu = (y / cs) * ncx + xg / cs;  // 4-sample groups never straddle a CTU (cs % 4 == 0)
    const hvx_sao_offset o = params[ctu].comp[comp];
    const Blk b = block(ctu, ncx, w, h, cs);
    const uint8_t *row = src + (size_t)y * ss;
    uint8_t *drow = dst + (size_t)y * ds;
    const int t = o.type, ly = y - b.y0;
    // offsetBlock's regions (:337-553): EO drops the columns / rows whose neighbour is outside the picture
    const int xs = (t == 0 || t == 2 || t == 3) && !b.L ? 1 : 0, xe = (t == 0 || t == 2 || t == 3) && !b.R ? b.bw - 1 : b.bw;
    const bool row_in = !(t >= 1 && t <= 3) || ((b.A || ly > 0) && (b.B || ly < b.bh - 1));
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int x = xg + i;
      if (x >= w) break;
      const int lx = x - b.x0;
      int v = row[x];
      if (t >= 0 && row_in && lx >= xs && lx < xe) {
        int off;
        if (t == HVX_SAO_BO) {
          const int k = ((v >> 3) - o.band) & 31;
          off = k < 4 ? o.offset[k] : 0;
        } else {
          const int e = edge(row + x, ss, t);
          off = e == 2 ? 0 : o.offset[e < 2 ? e : e - 1];
        }
        v = clip3(0, 255, v + off);
      }
      drow[x] = (uint8_t)v;
    }
  }
}
