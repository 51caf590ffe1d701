// hvx_sao.hpp -- sample adaptive offset on a deblocked picture (gfx950); SURVEY.md 8(f) item 3.
// Restated by oracle/hvx_oracle.c ("SAO"); TEncSampleAdaptiveOffset::getStatistics/getBlkStats
// (TEncSampleAdaptiveOffset.cpp:285, 892) and TComSampleAdaptiveOffset::offsetCTU/offsetBlock
// (TComSampleAdaptiveOffset.cpp:313, 554), single slice and tile, 8-bit 4:2:0.
//
// Statistics: one workgroup per (CTU, component), the block staged in LDS; edge-offset sums in
// registers, band histograms in LDS (int32: at most 64*64 samples of |d| <= 255 per CTU),
// widened to the int64 SAOStatData layout at the end.  Application: one thread per
// 4 output samples, reading the unmodified input picture (src != dst) so that CTUs are
// independent -- the reference's copy of the deblocked picture (SAOProcess :246-249).
#pragma once
#include "hvx_dev.hpp"
#include "hvx_me.hpp"  // wave_sum_dpp

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
// The CTU block and its 1-sample ring (where inside the picture) are staged in LDS; each thread
// keeps the edge-offset sums of its samples in registers (4 types x 5 classes, diff and count)
// and adds band-offset samples to LDS histograms; the register sums are reduced per wave with
// DPP adds and once per wave into LDS.
static __global__ __launch_bounds__(256) void k_sao_stats(const uint8_t *__restrict__ org_y, const uint8_t *__restrict__ org_cb,
                                                  const uint8_t *__restrict__ org_cr, int os_y, int os_c,
                                                  const uint8_t *__restrict__ rec_y, const uint8_t *__restrict__ rec_cb,
                                                  const uint8_t *__restrict__ rec_cr, int rs_y, int rs_c, int pic_w,
                                                  int pic_h, hvx_sao_stat *__restrict__ out) {
  using namespace sao;
  constexpr int TS = 68;  // tile stride: 64 + ring, dword-aligned rows
  __shared__ uint8_t tile[66 * TS];
  __shared__ uint8_t otile[64 * 64];
  constexpr int NC = 16;  // band-histogram copies (lane & 15): same-band lanes of one instruction spread over banks
  __shared__ int bo[2][HVX_SAO_CLASSES][NC];
  __shared__ int eo[4][2][5];
  const int comp = blockIdx.y, ctu = blockIdx.x;
  const int cs = comp ? 32 : 64, w = comp ? pic_w >> 1 : pic_w, h = comp ? pic_h >> 1 : pic_h;
  const int skr = comp ? 3 : 5, skb = comp ? 2 : 4;  // m_skipLinesR/B (createEncData :125-131)
  const uint8_t *org = comp == 0 ? org_y : comp == 1 ? org_cb : org_cr;
  const uint8_t *rec = comp == 0 ? rec_y : comp == 1 ? rec_cb : rec_cr;
  const int os = comp ? os_c : os_y, rs = comp ? rs_c : rs_y;
  const int ncx = (pic_w + 63) >> 6;
  const Blk b = block(ctu, ncx, w, h, cs);
  for (int i = threadIdx.x; i < 2 * HVX_SAO_CLASSES * NC + 40; i += 256) {
    if (i < 2 * HVX_SAO_CLASSES * NC) (&bo[0][0][0])[i] = 0;
    else (&eo[0][0][0])[i - 2 * HVX_SAO_CLASSES * NC] = 0;
  }
  // staging: every load of the block issued before the first LDS store of a batch (latency overlap)
  const int tw = b.bw + 2, th = b.bh + 2;
  for (int i0 = threadIdx.x; i0 < tw * th; i0 += 256 * 8) {
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = i0 + u * 256, ty = i / tw, tx = i - ty * tw, gy = b.y0 + ty - 1, gx = b.x0 + tx - 1;
      v[u] = (i < tw * th && gy >= 0 && gy < h && gx >= 0 && gx < w) ? rec[(size_t)gy * rs + gx] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = i0 + u * 256, ty = i / tw, tx = i - ty * tw;
      if (i < tw * th) tile[ty * TS + tx] = v[u];
    }
  }
  for (int i0 = threadIdx.x; i0 < b.bw * b.bh; i0 += 256 * 8) {
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = i0 + u * 256, y = i / b.bw, x = i - y * b.bw;
      v[u] = i < b.bw * b.bh ? org[(size_t)(b.y0 + y) * os + b.x0 + x] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (i0 + u * 256 < b.bw * b.bh) otile[i0 + u * 256] = v[u];
  }
  __syncthreads();
  // per type: [xs, xe) x [ys, ye) (getBlkStats :941, 989, 1051, 1140, 1229)
  const int bxe = b.R ? b.bw - skr : b.bw, bye = b.B ? b.bh - skb : b.bh;
  const int exs = b.L ? 0 : 1, exe = b.R ? b.bw - skr : b.bw - 1;
  const int vys = b.A ? 0 : 1, vye = b.B ? b.bh - skb : b.bh - 1;
  int ad[4][5], ac[4][5];
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int k = 0; k < 5; k++) ad[t][k] = ac[t][k] = 0;
  for (int i = threadIdx.x; i < b.bw * b.bh; i += 256) {
    const int y = i / b.bw, x = i - y * b.bw;
    const uint8_t *p = tile + (y + 1) * TS + x + 1;
    const int c = p[0];
    const int d = (int)otile[i] - c;
    if (x < bxe && y < bye) {
      atomicAdd(&bo[0][c >> 3][threadIdx.x & (NC - 1)], d);
      atomicAdd(&bo[1][c >> 3][threadIdx.x & (NC - 1)], 1);
    }
    const bool in_x = x >= exs && x < exe, in_yv = y >= vys && y < vye;
    const bool in[4] = {in_x && y < bye, x < bxe && in_yv, in_x && in_yv, in_x && in_yv};
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int k = in[t] ? edge(p, TS, t) : -1;
#pragma unroll
      for (int j = 0; j < 5; j++) {
        ad[t][j] += k == j ? d : 0;
        ac[t][j] += k == j ? 1 : 0;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const int vd = (int)wave_sum_dpp((uint32_t)ad[t][j]), vc = (int)wave_sum_dpp((uint32_t)ac[t][j]);
      if (lane_id() == 0) {
        atomicAdd(&eo[t][0][j], vd);
        atomicAdd(&eo[t][1][j], vc);
      }
    }
  __syncthreads();
  hvx_sao_stat *st = out + ((size_t)ctu * 3 + comp) * HVX_SAO_TYPES;
  for (int i = threadIdx.x; i < HVX_SAO_TYPES * 2 * HVX_SAO_CLASSES; i += 256) {
    const int t = i / (2 * HVX_SAO_CLASSES), r = i % (2 * HVX_SAO_CLASSES), k = r % HVX_SAO_CLASSES, dc = r / HVX_SAO_CLASSES;
    int64_t v = 0;
    if (t == 4) {
#pragma unroll
      for (int j = 0; j < NC; j++) v += bo[dc][k][j];
    } else if (k < 5) {
      v = eo[t][dc][k];
    }
    if (dc == 0) st[t].diff[k] = v;
    else st[t].count[k] = v;
  }
}

// grid-stride over every 4-sample group of the plane comp = blockIdx.y; dst = src with offsets
static __global__ __launch_bounds__(256) void k_sao_apply(const uint8_t *__restrict__ src_y, const uint8_t *__restrict__ src_cb,
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
