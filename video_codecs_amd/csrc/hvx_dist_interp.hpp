// hvx_dist_interp.hpp -- distortion, interpolation and picture-plane kernels (gfx950).
//
// Distortion: TComRdCost.cpp:294-1593.  One 64-lane wave per job, 4 jobs per 256-thread
// workgroup; samples spread over lanes, DPP/shuffle all-reduce.
// Interpolation: TComInterpolationFilter.cpp:94-394.  One workgroup per filter call,
// one output sample per lane-iteration, 16-bit intermediates exactly as the reference.
#pragma once
#include "hvx_dev.hpp"

static __global__ __launch_bounds__(256) void k_dist(const int16_t *__restrict__ org, const int16_t *__restrict__ cur,
                                              const hvx_dist_job *__restrict__ jobs, int n, uint32_t *__restrict__ out) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const hvx_dist_job jb = jobs[j];
  const int16_t *o = org + jb.org_off, *c = cur + jb.cur_off;
  const int w = jb.w, h = jb.h, so = jb.org_stride, sc = jb.cur_stride;
  uint32_t r;
  if (jb.kind == HVX_DIST_SATD) {
    r = wave_satd(o, so, c, sc, w, h);
  } else {
    int sub = 0;
    if (jb.kind == HVX_DIST_SAD_ME) {
      const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
      sub = spec ? jb.sub_shift : 0;
    }
    const int rows = (h + (1 << sub) - 1) >> sub;
    const bool sq = jb.kind == HVX_DIST_SSE || jb.kind == HVX_DIST_SSE_W;
    uint32_t s = 0;
    for (int i = lane_id(); i < rows * w; i += HVX_WAVE) {
      const int y = (i / w) << sub, x = i % w;
      const int d = (int)o[y * so + x] - (int)c[y * sc + x];
      s += sq ? (uint32_t)(d * d) : (uint32_t)abs(d);
    }
    r = wave_sum_u32(s) << sub;
    if (jb.kind == HVX_DIST_SSE_W) r = (uint32_t)(jb.weight * (double)r);
  }
  if (lane_id() == 0) out[j] = r;
}

// filter<N,isVertical,isFirst,isLast> (TComInterpolationFilter.cpp:172) + filterCopy (:94)
static __global__ __launch_bounds__(256) void k_interp(const int16_t *__restrict__ src, int16_t *__restrict__ dst,
                                                const hvx_interp_job *__restrict__ jobs) {
  const hvx_interp_job jb = jobs[blockIdx.x];
  const int16_t *s = src + jb.src_off;
  int16_t *d = dst + jb.dst_off;
  const int w = jb.w, h = jb.h, ss = jb.src_stride, ds = jb.dst_stride;
  const int first = jb.vertical ? jb.is_first : 1, last = jb.is_last;
  if (jb.frac == 0) {
    for (int i = threadIdx.x; i < w * h; i += blockDim.x) {
      const int y = i / w, x = i % w;
      const int v = s[y * ss + x];
      int16_t r;
      if (first == last) r = (int16_t)v;
      else if (first) r = (int16_t)((int16_t)(v << 6) - 8192);
      else r = (int16_t)clip_pel((v + 8192 + 32) >> 6);
      d[y * ds + x] = r;
    }
    return;
  }
  const int ntaps = jb.is_luma ? 8 : 4;
  const int cs = jb.vertical ? ss : 1;
  int shift = 6, offset;
  if (last) {
    shift += first ? 0 : 6;
    offset = (1 << (shift - 1)) + (first ? 0 : 8192 << 6);
  } else {
    shift -= first ? 6 : 0;
    offset = first ? -8192 << shift : 0;
  }
  const int8_t *cf = jb.is_luma ? kLumaFilter[jb.frac] : kChromaFilter[jb.frac];
  const int16_t *base = s - (ntaps / 2 - 1) * cs;
  for (int i = threadIdx.x; i < w * h; i += blockDim.x) {
    const int y = i / w, x = i % w;
    const int16_t *p = base + y * ss + x;
    int sum = 0;
    for (int k = 0; k < ntaps; k++) sum += p[k * cs] * cf[k];
    int16_t v = (int16_t)((sum + offset) >> shift);
    if (last) v = (int16_t)clip_pel(v);
    d[y * ds + x] = v;
  }
}

// TComPicYuv int16 plane -> 8-bit padded plane interior
static __global__ __launch_bounds__(256) void k_plane_from_pel(const int16_t *__restrict__ pel, int pel_stride, int w, int h,
                                                        uint8_t *__restrict__ plane, int stride) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x < w && y < h) plane[y * stride + x] = (uint8_t)clip_pel(pel[y * pel_stride + x]);
}

// TComPicYuv::extendPicBorder (TComPicYuv.cpp:197): replicate edges into the margin.
// pass 0: left/right margins of every interior row; pass 1: top/bottom rows (full width).
static __global__ __launch_bounds__(256) void k_plane_extend(uint8_t *__restrict__ plane, int stride, int w, int h, int margin, int pass) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;  // column incl. margin: [-margin, w+margin)
  const int y = blockIdx.y;
  if (pass == 0) {
    if (y >= h || x >= 2 * margin) return;
    uint8_t *row = plane + y * stride;
    if (x < margin) row[x - margin] = row[0];
    else row[w + (x - margin)] = row[w - 1];
  } else {
    const int cx = x - margin;
    if (cx >= w + margin || y >= 2 * margin) return;
    if (y < margin) plane[(y - margin) * stride + cx] = plane[cx];
    else plane[(h + y - margin) * stride + cx] = plane[(h - 1) * stride + cx];
  }
}

// extendPicBorder of up to three planes in one launch (blockIdx.y = plane): every margin sample
// takes the picture sample at the clamped position, which is what the two passes above (left /
// right columns, then whole top / bottom rows) produce
struct PlaneSet {
  uint8_t *p[3];
  int s[3], w[3], h[3], m[3];
};
static __global__ __launch_bounds__(256) void k_planes_extend(PlaneSet E) {
  const int pi = blockIdx.y;
  uint8_t *pl = E.p[pi];
  const int s = E.s[pi], w = E.w[pi], h = E.h[pi], m = E.m[pi];
  const int k = blockIdx.x * blockDim.x + threadIdx.x, nside = 2 * m * h, nrow = w + 2 * m;
  int x, y;
  if (k < nside) {
    const int c = k % (2 * m);
    y = k / (2 * m);
    x = c < m ? c - m : w + c - m;
  } else if (k < nside + 2 * m * nrow) {
    const int k2 = k - nside, rr = k2 / nrow;
    y = rr < m ? rr - m : h + rr - m;
    x = k2 % nrow - m;
  } else {
    return;
  }
  const int cy = y < 0 ? 0 : y >= h ? h - 1 : y, cx = x < 0 ? 0 : x >= w ? w - 1 : x;
  pl[(int64_t)y * s + x] = pl[(int64_t)cy * s + cx];
}
