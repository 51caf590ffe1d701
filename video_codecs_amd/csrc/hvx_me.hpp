// hvx_me.hpp -- uni-prediction motion estimation (gfx950): TZ integer search + half/quarter
// SATD refinement, i.e. TEncSearch::xMotionEstimation with bBi=false
// (TEncSearch.cpp:3663-3760; xTZSearch :3881 with TZ_SEARCH_CONFIGURATION :297-313,
// xTZSearchHelp :332, xTZ8PointDiamondSearch :629, xTZ2PointSearch :438,
// xSetSearchRange :3765, xPatternSearchFracDIF :4240, xPatternRefinement :808;
// TComDataCU::clipMv TComDataCU.cpp:2788; TComRdCost::getCost TComRdCost.h:172).
//
// Two kernels, one 64-lane wave per (PU, reference) job each:
//
//  k_me_int  -- the TZ integer search.  The reference visits candidates one at a time
//     (xTZSearchHelp, strict '<').  Each search step here evaluates its whole candidate
//     LIST at once: all diamonds of a stage around their common start, the 2-point pair,
//     64 raster points per pass.  Lanes split over candidates (64/2^ceil(log2 n) lanes per
//     candidate, one 4-pixel row group per lane-iteration, v_sad_u8 on dword loads) and the
//     list is then reduced to its FIRST minimum with a wave-wide (cost, index) key-min --
//     exactly the point a sequence of strict '<' updates would keep.  The smooth-MV early
//     stop of the first stage replays the diamonds' minima in order.  Low register use
//     (no interpolation state) keeps 8 waves per SIMD resident.
//
//  k_me_frac -- xPatternSearchFracDIF from the integer result.  Per stage (half, quarter)
//     the 3 horizontal sub-pel phases the 9 candidates need are filtered once into LDS
//     planes (the reference's first-stage 16-bit intermediates), each candidate is one
//     vertical pass over a plane, and its SATD is an 8x8 Hadamard done ACROSS lanes (one
//     sample per lane, butterflies on xor-shuffles) for blocks of <= 16 tiles; larger or
//     4x4-tiled blocks go through an LDS block + per-lane tiles.  Templated on the largest
//     block size so a depth's launch only reserves the LDS its blocks need.
#pragma once
#include "hvx_dev.hpp"

struct MeRange { int l, r, t, b; };

// The reference's per-point range tests (xTZ8PointDiamondSearch, xTZ2PointSearch) check only
// the bound in each direction the point moved from the start -- a start outside the range
// (the zero MV, a far predictor) still has its axis points searched.
__device__ __forceinline__ bool me_in(const MeRange &g, int dx, int dy, int x, int y) {
  return ((dx >= 0) | (x >= g.l)) & ((dx <= 0) | (x <= g.r)) & ((dy >= 0) | (y >= g.t)) & ((dy <= 0) | (y <= g.b));
}

// TComDataCU::clipMv: quarter-pel, result stored as Short
__device__ __forceinline__ void me_clip(const hvx_me_job &j, int &mx, int &my) {
  const int hmax = (j.pic_w + 8 - j.cu_x - 1) << 2, hmin = (-j.max_cu - 8 - j.cu_x + 1) << 2;
  const int vmax = (j.pic_h + 8 - j.cu_y - 1) << 2, vmin = (-j.max_cu - 8 - j.cu_y + 1) << 2;
  mx = (int16_t)(mx < hmin ? hmin : mx > hmax ? hmax : mx);
  my = (int16_t)(my < vmin ? vmin : my > vmax ? vmax : my);
}

// xSetSearchRange (:3765)
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

// TComRdCost::getCost(x, y) with the predictor at quarter-pel and the candidate at 1<<scale units
__device__ __forceinline__ uint32_t me_mv_cost(uint32_t lam, int px, int py, int scale, int x, int y) {
  const uint32_t bits = eg_bits((x << scale) - px) + eg_bits((y << scale) - py);
  return (lam * bits) >> 16;
}

// 4 bytes at any address from two aligned dword loads (plane margins cover the over-read)
__device__ __forceinline__ uint32_t ld4_any(const uint8_t *p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(v, o, HVX_WAVE);
    v = t < v ? t : v;
  }
  return v;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// A job of NW waves owns its workgroup when NW > 1; an NW == 1 job may share a workgroup with
// other single-wave jobs (k_me_ctu8_cu), so its thread index is the lane and its LDS hand-offs
// are wave-level (no workgroup barrier other waves would have to meet).
template <int NW>
__device__ __forceinline__ int me_tid() { return NW > 1 ? (int)threadIdx.x : lane_id(); }
template <int NW>
__device__ __forceinline__ void me_sync() {
  if constexpr (NW > 1) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

#define ME_DPP(v, ctrl) ((uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)(v), (ctrl), 0xf, 0xf, false))

// Wave-wide minimum (every lane active): v_min_u32_dpp inside rows of 16 lanes (quad swaps,
// half-row and row mirrors), then the 4 row minima on the SALU.  Result is wave-uniform.
__device__ __forceinline__ uint32_t wave_min_key(uint32_t v) {
  v = min(v, ME_DPP(v, 0xB1));   // quad_perm [1,0,3,2]
  v = min(v, ME_DPP(v, 0x4E));   // quad_perm [2,3,0,1]
  v = min(v, ME_DPP(v, 0x141));  // row_half_mirror
  v = min(v, ME_DPP(v, 0x140));  // row_mirror
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return min(min(a, b), min(c, d));
}

// Sum over aligned groups of 1<<sh lanes, every lane of a group ends with its sum (every lane
// active; sh wave-uniform).
__device__ __forceinline__ uint32_t seg_sum(uint32_t v, int sh) {
  if (sh >= 1) v += ME_DPP(v, 0xB1);
  if (sh >= 2) v += ME_DPP(v, 0x4E);
  if (sh >= 3) v += ME_DPP(v, 0x141);
  if (sh >= 4) v += ME_DPP(v, 0x140);
  if (sh >= 5) v += __shfl_xor(v, 16, HVX_WAVE);
  if (sh >= 6) v += __shfl_xor(v, 32, HVX_WAVE);
  return v;
}

// (cost, list index) key of one candidate of a list of <= 256 points.  Costs stay below 2^24
// (SAD <= 64*64*255, MV costs of a few thousand), so key order == cost order, ties broken by
// the lower index: the first minimum, i.e. the point a chain of strict '<' updates keeps.
constexpr uint32_t kMeKeyNone = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t me_key(uint32_t cost, int idx) { return (cost << 8) | (uint32_t)idx; }

typedef uint32_t me_v2u __attribute__((ext_vector_type(2)));
typedef uint32_t me_v3u __attribute__((ext_vector_type(3)));
typedef uint32_t me_v4u __attribute__((ext_vector_type(4)));

// N consecutive dwords at byte offset voff + soff of a buffer (dwordx4 pieces + remainder)
template <int N>
__device__ __forceinline__ void me_ldw(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff, uint32_t *w) {
#pragma unroll
  for (int i = 0; i + 4 <= N; i += 4) {
    const me_v4u t = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 4 * i, soff, 0);
    w[i] = t.x; w[i + 1] = t.y; w[i + 2] = t.z; w[i + 3] = t.w;
  }
  constexpr int B = N & ~3;
  if constexpr (N % 4 == 1) {
    w[B] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 4 * B, soff, 0);
  } else if constexpr (N % 4 == 2) {
    const me_v2u t = __builtin_amdgcn_raw_buffer_load_b64(rs, voff + 4 * B, soff, 0);
    w[B] = t.x; w[B + 1] = t.y;
  } else if constexpr (N % 4 == 3) {
    const me_v3u t = __builtin_amdgcn_raw_buffer_load_b96(rs, voff + 4 * B, soff, 0);
    w[B] = t.x; w[B + 1] = t.y; w[B + 2] = t.z;
  }
}

// buffer resource over a whole padded 8-bit plane given its sample-(0,0) pointer (ME plane
// contract: margin HVX_PLANE_MARGIN on every side); built from wave-uniform values
__device__ __forceinline__ __amdgpu_buffer_rsrc_t me_plane_rsrc(const uint8_t *origin, int stride, int pic_h) {
  const uint8_t *base = origin - (size_t)HVX_PLANE_MARGIN * stride - HVX_PLANE_MARGIN;
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int bytes = __builtin_amdgcn_readfirstlane(stride * (pic_h + 2 * HVX_PLANE_MARGIN));
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

// ======================================================================================
// integer TZ search
// ======================================================================================
constexpr int kMeMaxList = 256;  // diamonds d = 1..256: 4 + 3*8 + 5*16 = 108 points; raster passes <= 256

struct MeInt {
  const uint8_t *org;  // LDS, stride os (64 for the generic kernel, S for the CTU kernels)
  const uint8_t *ref;  // PU origin at MV (0,0) in the reference plane
  uint32_t *red;       // LDS, [2][kMeMaxRanges][NW] per-wave range minima (ping-pong), NW > 1 only
  int par;             // ping-pong parity of red
  __amdgpu_buffer_rsrc_t rs;  // the reference plane as a buffer (compile-time-shape kernels)
  uint32_t roff;              // byte offset of the PU origin at MV (0,0) in rs
  int sr, sub, rows, gw, os;
  uint32_t lam;
  int px, py;
  int best_x, best_y, best_dist, best_round, point_nr;
  uint32_t best_sad;
};

struct MeCand { int x, y, pnr, dist; bool ok; };

// SAD (before the FEN scale) of the block at (x,y) over row groups s, s+L, s+2L, ...
// (group = 4 pixels of one sampled row).  Runtime geometry (generic PU shapes).
__device__ __forceinline__ uint32_t me_sad_part(const MeInt &m, int x, int y, int s, int L) {
  const int n = m.rows * m.gw;
  int r = s / m.gw, g = s - r * m.gw;
  const int dr = L / m.gw, dg = L - dr * m.gw;
  const uint8_t *base = m.ref + y * m.sr + x;
  const int rs = m.sr << m.sub, os = m.os << m.sub;
  uint32_t acc = 0;
  for (int i = s; i < n; i += L) {
    const uint32_t o = *(const uint32_t *)(m.org + r * os + 4 * g);
    acc = __builtin_amdgcn_sad_u8(o, ld4_any(base + r * rs + 4 * g), acc);
    g += dg;
    r += dr;
    if (g >= m.gw) { g -= m.gw; r++; }
  }
  return acc;
}

// Same for a square SxS block with compile-time FEN shift and lanes-per-point 1<<SH: lane s
// takes sampled rows s, s+L, ...  Rows come from buffer loads at the point's dword-aligned
// offset + an SGPR row offset (plane strides are multiples of 4, so one alignbyte shift serves
// every row); the row loop unrolls so that up to ~24 dwords per lane are in flight at once.
template <int S, int SUB, int SH>
__device__ __forceinline__ uint32_t me_sad_part_ct(const MeInt &m, int x, int y, int s) {
  constexpr int ROWS = S >> SUB, L = 1 << SH, PER = (ROWS + L - 1) / L, GW = S / 4;
  constexpr int BUDGET = S == 8 ? 12 : 24;  // dwords in flight per lane (8x8: keep occupancy)
  constexpr int RUN = (GW + 1) * PER <= BUDGET ? PER : (BUDGET / (GW + 1) > 0 ? BUDGET / (GW + 1) : 1);
  constexpr int UNR = RUN < 1 ? 1 : RUN;
  const uint32_t a = m.roff + (uint32_t)(y * m.sr + x) + (uint32_t)((s << SUB) * m.sr);
  const uint32_t va = a & ~3u, sh = a & 3u;
  const uint8_t *o = m.org + (s << SUB) * S;
  uint32_t acc = 0;
#pragma unroll UNR
  for (int k = 0; k < PER; k++) {
    if (ROWS % L == 0 || s + k * L < ROWS) {
      uint32_t w[GW + 1];
      me_ldw<GW + 1>(m.rs, va, ((k * L) << SUB) * m.sr, w);
      const uint32_t *ow = (const uint32_t *)(o + ((k * L) << SUB) * S);
#pragma unroll
      for (int i = 0; i < GW; i++) acc = __builtin_amdgcn_sad_u8(ow[i], __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh), acc);
    }
  }
  return acc;
}

// S == 0: runtime geometry
template <int S, int SUB>
__device__ __forceinline__ uint32_t me_sad_any(const MeInt &m, int x, int y, int s, int sh) {
  if constexpr (S == 0) {
    return me_sad_part(m, x, y, s, 1 << sh);
  } else {
    switch (sh) {
      case 0: return me_sad_part_ct<S, SUB, 0>(m, x, y, s);
      case 1: return me_sad_part_ct<S, SUB, 1>(m, x, y, s);
      case 2: return me_sad_part_ct<S, SUB, 2>(m, x, y, s);
      case 3: return me_sad_part_ct<S, SUB, 3>(m, x, y, s);
      case 4: return me_sad_part_ct<S, SUB, 4>(m, x, y, s);
      case 5: return me_sad_part_ct<S, SUB, 5>(m, x, y, s);
      default: return me_sad_part_ct<S, SUB, 6>(m, x, y, s);
    }
  }
}

constexpr int kMeMaxRanges = 9;  // first-stage diamonds d = 1 .. 256

// Costs (SAD + MV cost; points outside the search range excluded) of list points [0, n),
// n <= kMeMaxList, reduced to the FIRST-minimum key of each range r < nr -- range r being the
// points p with rng(p) == r -- identical in every wave of the job on return.  The NW waves take
// equal contiguous shares of the list; inside a wave, 64/2^ceil(log2 share) lanes work on each
// point of a pass; each lane keeps its points' per-range minima in registers, reduced once per
// list (DPP + SALU; across waves through a ping-pong LDS slot, one barrier).
template <int S, int SUB, int NW, int NR, typename F, typename R>
__device__ __forceinline__ void me_eval_min(MeInt &m, int n, int nr, F cand, R rng, uint32_t (&key)[NR]) {
  const int lane = lane_id(), wave = NW > 1 ? uni((int)(threadIdx.x >> 6)) : 0;
  const int per = (n + NW - 1) / NW, lo = wave * per, hi = min(n, lo + per);
  uint32_t part[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) part[r] = kMeKeyNone;
  for (int base = lo; base < hi; base += HVX_WAVE) {
    const int cnt = min(HVX_WAVE, hi - base);
    const int sh = 6 - (cnt <= 1 ? 0 : 32 - __clz(cnt - 1)), L = 1 << sh;
    const int q = lane >> sh, s = lane & (L - 1);
    MeCand c;
    c.ok = false; c.x = c.y = 0;
    if (q < cnt) c = cand(base + q);
    uint32_t acc = c.ok ? me_sad_any<S, SUB>(m, c.x, c.y, s, sh) : 0u;
    acc = seg_sum(acc, sh);  // every lane of the point's group holds its SAD
    if (c.ok) {
      const int p = base + q;
      const uint32_t k = me_key((acc << m.sub) + me_mv_cost(m.lam, m.px, m.py, 2, c.x, c.y), p);
      const int r = NR == 1 ? 0 : rng(p);
#pragma unroll
      for (int i = 0; i < NR; i++)
        if (i == r) part[i] = min(part[i], k);
    }
  }
#pragma unroll
  for (int r = 0; r < NR; r++) {
    key[r] = kMeKeyNone;
    if (r < nr) {
      const uint32_t w = wave_min_key(part[r]);
      if constexpr (NW == 1) key[r] = w;
      else if (lane == 0) m.red[(m.par * kMeMaxRanges + r) * NW + wave] = w;
    }
  }
  if constexpr (NW > 1) {
    __syncthreads();  // the other parity slot is rewritten only after the NEXT list's barrier
#pragma unroll
    for (int r = 0; r < NR; r++) {
      if (r < nr) {
        uint32_t v = kMeKeyNone;
#pragma unroll
        for (int w = 0; w < NW; w++) v = min(v, m.red[(m.par * kMeMaxRanges + r) * NW + w]);
        key[r] = (uint32_t)uni((int)v);
      }
    }
    m.par ^= 1;
  }
}

// diamonds d = 1, 2, 4, ... around (sx,sy), concatenated in xTZ8PointDiamondSearch order
__device__ __forceinline__ int me_dia_start(int k) { return k == 0 ? 0 : k <= 3 ? 4 + 8 * (k - 1) : 28 + 16 * (k - 4); }

// xTZSearchHelp applied to a list's first minimum (strict '<' against the running best)
template <typename F>
__device__ __forceinline__ void me_take(MeInt &m, uint32_t key, F cand) {
  if (key != kMeKeyNone && (key >> 8) < m.best_sad) {
    const MeCand w = cand((int)(key & 255u));
    m.best_sad = key >> 8; m.best_x = w.x; m.best_y = w.y; m.best_dist = w.dist; m.best_round = 0; m.point_nr = w.pnr;
  }
}

__device__ __forceinline__ int me_rng0(int) { return 0; }

__device__ __forceinline__ int me_dia_k(int p) { return p < 4 ? 0 : p < 28 ? 1 + ((p - 4) >> 3) : 4 + ((p - 28) >> 4); }

// Point p of that list as an offset from the start (xTZ8PointDiamondSearch :629-800: d = 1 is
// the 4-point cross; d = 2..8 the 8-point diamond with half-distance diagonals; d >= 16 the
// 4 axis points + 3 rows of 4 points per quadrant edge), packed into one table word:
// dx | dy << 10 (10-bit two's complement) | point_nr << 20 | log2(distance) << 24.
struct MeDiaTab { uint32_t v[108]; };
constexpr uint32_t me_dia_pack(int dx, int dy, int pnr, int dist) {
  int dl = 0;
  while ((1 << dl) < dist) dl++;
  return ((uint32_t)dx & 0x3FFu) | (((uint32_t)dy & 0x3FFu) << 10) | ((uint32_t)pnr << 20) | ((uint32_t)dl << 24);
}
constexpr MeDiaTab me_dia_build() {
  MeDiaTab t{};
  for (int p = 0; p < 108; p++) {
    int k = 0, q = 0;
    if (p < 4) { k = 0; q = p; }
    else if (p < 28) { k = 1 + ((p - 4) >> 3); q = (p - 4) & 7; }
    else { k = 4 + ((p - 28) >> 4); q = (p - 28) & 15; }
    const int d = 1 << k, h = d >> 1;
    int dx = 0, dy = 0, pnr = 0, dist = d;
    if (k == 0) {
      const int tab[4][3] = {{0, -1, 2}, {-1, 0, 4}, {1, 0, 5}, {0, 1, 7}};
      dx = tab[q][0]; dy = tab[q][1]; pnr = tab[q][2];
    } else if (k <= 3) {
      const int tab[8][4] = {{0, -2, 2, 2}, {-1, -1, 1, 1}, {1, -1, 3, 1}, {-2, 0, 4, 2},
                             {2, 0, 5, 2},  {-1, 1, 6, 1},  {1, 1, 8, 1},  {0, 2, 7, 2}};  // units of h
      dx = tab[q][0] * h; dy = tab[q][1] * h; pnr = tab[q][2]; dist = tab[q][3] * h;
    } else if (q < 4) {
      dx = q == 1 ? -d : q == 2 ? d : 0;
      dy = q == 0 ? -d : q == 3 ? d : 0;
    } else {
      const int i = 1 + ((q - 4) >> 2), kk = (q - 4) & 3, o = (d >> 2) * i;
      dx = (kk & 1) ? o : -o;
      dy = (kk & 2) ? d - o : o - d;
    }
    t.v[p] = me_dia_pack(dx, dy, pnr, dist);
  }
  return t;
}
static __constant__ MeDiaTab kDiaTab = me_dia_build();

__device__ __forceinline__ MeCand me_dia_cand(const MeRange &g, int sx, int sy, int p) {
  const uint32_t v = kDiaTab.v[p];
  const int dx = (int)(v << 22) >> 22, dy = (int)(v << 12) >> 22;
  MeCand c;
  c.x = sx + dx; c.y = sy + dy; c.pnr = (int)((v >> 20) & 15u); c.dist = 1 << ((v >> 24) & 15u);
  c.ok = me_in(g, dx, dy, c.x, c.y);  // == the reference's tests, whether the diamond is inside or not
  return c;
}

// xTZ2PointSearch (:438): the two points completing the diamond around point_nr
static __constant__ int8_t kTwoPoint[8][2][2] = {{{-1, 0}, {0, -1}}, {{-1, -1}, {1, -1}}, {{0, -1}, {1, 0}},
                                          {{-1, 1}, {-1, -1}}, {{1, -1}, {1, 1}}, {{-1, 0}, {0, 1}},
                                          {{-1, 1}, {1, 1}}, {{1, 0}, {0, 1}}};

template <int S, int SUB, int NW>
__device__ __forceinline__ void me_2point(MeInt &m, const MeRange &g) {
  const int pn = m.point_nr, bx = m.best_x, by = m.best_y;
  if (pn < 1 || pn > 8) return;  // unreachable: the reference asserts here
  auto cand = [=](int p) {
    MeCand c;
    const int dx = kTwoPoint[pn - 1][p][0], dy = kTwoPoint[pn - 1][p][1];
    c.x = bx + dx; c.y = by + dy;
    c.pnr = 0; c.dist = 2; c.ok = me_in(g, dx, dy, c.x, c.y);
    return c;
  };
  uint32_t key[1];
  me_eval_min<S, SUB, NW, 1>(m, 2, 1, cand, me_rng0, key);
  me_take(m, key[0], cand);
}

// xTZSearch (:3881) for job j; returns with m.best_* = the integer result
template <int S, int SUB, int NW>
__device__ void me_tz(const hvx_me_job &j, MeInt &m) {
  const int sr = j.search_range;
  const MeRange g0 = me_search_range(j, j.pred_x, j.pred_y, sr);
  int mx = j.pred_x, my = j.pred_y;
  me_clip(j, mx, my);
  mx >>= 2; my >>= 2;
  int ix = 0, iy = 0;
  if (j.use_int2nx2n) {
    ix = j.i2_x << 2; iy = j.i2_y << 2;
    me_clip(j, ix, iy);
    ix >>= 2; iy >>= 2;
  }
  m.best_sad = 0xFFFFFFFFu;
  m.best_x = m.best_y = 0; m.best_dist = 0; m.best_round = 0; m.point_nr = 0;
  // predictor, zero MV, then the 2Nx2N integer MV
  {
    auto cand = [=](int p) {
      MeCand c;
      c.x = p == 0 ? mx : p == 1 ? 0 : ix; c.y = p == 0 ? my : p == 1 ? 0 : iy;
      c.pnr = 0; c.dist = 0; c.ok = true;
      return c;
    };
    uint32_t key[1];
    me_eval_min<S, SUB, NW, 1>(m, j.use_int2nx2n ? 3 : 2, 1, cand, me_rng0, key);
    me_take(m, key[0], cand);
  }
  const MeRange g = j.use_int2nx2n ? me_search_range(j, m.best_x << 2, m.best_y << 2, sr) : g0;
  int nd = 0;
  while ((1 << nd) <= sr) nd++;
  const int ndp = me_dia_start(nd);
  // first stage: the diamonds around the start (one list, one minimum per diamond), replayed
  // in order and stopped after 3 rounds without a gain
  {
    const int sx = m.best_x, sy = m.best_y;
    auto cand = [=](int p) { return me_dia_cand(g0, sx, sy, p); };
    uint32_t key[kMeMaxRanges];
    me_eval_min<S, SUB, NW, kMeMaxRanges>(m, ndp, nd, cand, me_dia_k, key);
    bool stop = false;
#pragma unroll
    for (int k = 0; k < kMeMaxRanges; k++) {
      if (k < nd && !stop) {
        m.best_round += 1;
        me_take(m, key[k], cand);
        if ((j.flags & HVX_ME_SMOOTHMV) && m.best_round >= 3) stop = true;
      }
    }
  }
  if (m.best_dist == 1) { m.best_dist = 0; me_2point<S, SUB, NW>(m, g0); }
  // raster (step 5) over the re-centred range, lists of kMeMaxList points
  if (m.best_dist > 5) {
    m.best_dist = 5;
    const int nx = (g.r - g.l) / 5 + 1, ny = (g.b - g.t) / 5 + 1, n = nx * ny;
    const float rnx = 1.0f / (float)nx;
    for (int base = 0; base < n; base += kMeMaxList) {
      const int cnt = min(kMeMaxList, n - base);
      auto cand = [=](int p) {
        const int q = base + p;
        int ry = (int)((float)q * rnx), rx = q - ry * nx;  // float quotient, exact after one correction
        if (rx < 0) { ry--; rx += nx; } else if (rx >= nx) { ry++; rx -= nx; }
        MeCand c;
        c.x = g.l + 5 * rx; c.y = g.t + 5 * ry; c.pnr = 0; c.dist = 5; c.ok = true;
        return c;
      };
      uint32_t key[1];
      me_eval_min<S, SUB, NW, 1>(m, cnt, 1, cand, me_rng0, key);
      me_take(m, key[0], cand);
    }
  }
  // star refinement: every round's diamonds share their start -> one list, one minimum
  while (m.best_dist > 0) {
    const int sx = m.best_x, sy = m.best_y;
    m.best_dist = 0; m.point_nr = 0;
    auto cand = [=](int p) { return me_dia_cand(g0, sx, sy, p); };
    uint32_t key[1];
    me_eval_min<S, SUB, NW, 1>(m, ndp, 1, cand, me_rng0, key);
    me_take(m, key[0], cand);
    if (m.best_dist == 1) {
      m.best_dist = 0;
      if (m.point_nr != 0) me_2point<S, SUB, NW>(m, g0);
    }
  }
}

// the job's reference: PU-origin pointer (generic SAD, fractional stage) and buffer view
__device__ __forceinline__ void me_ref_setup(MeInt &m, const hvx_me_job &j, const uint8_t *ref_origin, int stride) {
  m.ref = ref_origin + j.pu_y * stride + j.pu_x;
  m.sr = stride;
  m.rs = me_plane_rsrc(ref_origin, stride, j.pic_h);
  m.roff = (uint32_t)((HVX_PLANE_MARGIN + j.pu_y) * stride + HVX_PLANE_MARGIN + j.pu_x);
}

// S == 0: any PU shape (org stride 64, runtime FEN); otherwise square SxS with FEN shift SUB.
template <int S, int SUB, int NW>
__device__ __forceinline__ void me_int_job(const hvx_me_job &j, const uint8_t *const *__restrict__ cur_planes,
                                           const uint8_t *const *__restrict__ ref_planes, int stride, uint8_t *org,
                                           uint32_t *red, hvx_me_result *out) {
  if (j.w <= 0 || j.h <= 0) {  // empty slot (e.g. a CU outside the picture): defined zero result
    if (threadIdx.x == 0) { hvx_me_result z; memset(&z, 0, sizeof(z)); *out = z; }
    return;
  }
  constexpr int OS = S ? S : 64;
  const uint8_t *cur = cur_planes[j.cur_idx] + j.pu_y * stride + j.pu_x;
  for (int k = threadIdx.x; k < j.w * j.h; k += HVX_WAVE * NW) {
    const int y = k / j.w, x = k - y * j.w;
    org[y * OS + x] = cur[y * stride + x];
  }
  __syncthreads();
  MeInt m;
  m.org = org; m.red = red; m.par = 0; m.os = OS;
  me_ref_setup(m, j, ref_planes[j.ref_idx], stride);
  const int w = j.w;
  if (S) {
    m.sub = SUB;
  } else {
    const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
    m.sub = ((j.flags & HVX_ME_FEN) && j.h > 8 && spec) ? 1 : 0;
  }
  m.rows = (j.h + (1 << m.sub) - 1) >> m.sub;
  m.gw = w >> 2;
  m.lam = j.lambda_motion;
  m.px = j.pred_x; m.py = j.pred_y;
  me_tz<S, SUB, NW>(j, m);
  if (threadIdx.x == 0) {
    out->mv_int_x = m.best_x; out->mv_int_y = m.best_y;
    out->sad_int = m.best_sad - me_mv_cost(m.lam, m.px, m.py, 2, m.best_x, m.best_y);
  }
}

static __global__ __launch_bounds__(64) void k_me_int(const uint8_t *const *__restrict__ cur_planes,
                                              const uint8_t *const *__restrict__ ref_planes, int stride,
                                              const hvx_me_job *__restrict__ jobs, int n, hvx_me_result *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t org[64 * 64];
  __shared__ uint32_t red[2 * kMeMaxRanges];
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_me_job j = jobs[jid];
  me_int_job<0, 0, 1>(j, cur_planes, ref_planes, stride, org, red, out + jid);
}

// ======================================================================================
// fractional refinement
// ======================================================================================

// Quarter-sample luma sample at (x,y) + quarter-pel (qx,qy); standard two-stage 8-bit path
// (TComInterpolationFilter::filterHor/filterVer, isFirst/isLast offsets).  Used by the CTU
// pass's motion compensation.
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

// xPatternRefinement (:808) candidate offsets: s_acMvRefineH / s_acMvRefineQ (TEncSearch.cpp:51-75)
static __constant__ int8_t kRefH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
static __constant__ int8_t kRefQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};

// Fractional-search LDS image for blocks up to SxS, NW waves per job.  The phase planes use
// a row stride of S+8 int16: an 8x8 tile row of 8 samples then covers 4 banks and the 8
// rows of a tile land on disjoint banks (conflict-free cross-lane tiles).
template <int S, int NW, typename TO = uint8_t>
struct MeFracSmem {
  static constexpr int HS = S + 8;
  int16_t hp[3][(S + 8) * HS];  // first-stage intermediates of the 3 horizontal phases, rows iy-4 ..
  // per-wave candidate block of the per-lane-tile SATD path: only shapes that are not multiples
  // of 8 (<= 16 rows) take it, so 16 rows of the S stride suffice above S = 32
  uint8_t blk[NW][S <= 32 ? S * S : 16 * S];
  alignas(16) TO org[S * S];    // the search pattern: the original (8-bit) or a bi target (int16)
  uint32_t cost[9];
  uint32_t part[NW][3][4];      // per-wave SATD partial sums of the 9 candidates (me_sum9 slots)
  uint32_t sat[NW][9];          // per-wave SATD partial sums by candidate slot (MFMA path)
};

typedef short me_s2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int me_sel3(const int (&v)[3], int i) { return i == 0 ? v[0] : i == 1 ? v[1] : v[2]; }

// first filter stage of two adjacent outputs: sum_t c[fx][t] * (b[t], b[t+1]) - 8192 on int16
// pairs (P[t] = (b[t], b[t+1])), one v_pk_mad per tap
__device__ __forceinline__ me_s2 me_fir_pk(int fx, const uint32_t *P) {
  me_s2 acc = {-8192, -8192};
#pragma unroll
  for (int t = 0; t < 8; t++) acc = acc + (short)kLumaFilter[fx][t] * __builtin_bit_cast(me_s2, P[t]);
  return acc;
}

// one prediction sample of a candidate column phase (its plane at element offset po of hp) at
// vertical quarter position qy (relative to the integer MV row iy): the reference's second
// filter stage
template <int S, int NW, typename TO>
__device__ __forceinline__ int me_frac_sample(const MeFracSmem<S, NW, TO> &sm, int po, int ry, int fy, int x, int y) {
  constexpr int HS = MeFracSmem<S, NW, TO>::HS;
  const int16_t *h = &sm.hp[0][0] + po + x;
  if (!fy) return clip_pel((h[(ry + 4 + y) * HS] + 8192 + 32) >> 6);
  int s = 0;
  const int r0 = ry + 1 + y;
#pragma unroll
  for (int t = 0; t < 8; t++) s += kLumaFilter[fy][t] * h[(r0 + t) * HS];
  return clip_pel((s + (1 << 11) + (8192 << 6)) >> 12);
}

// 8x8 Hadamard across the wave on VALU partner fetches only (every lane active): the stages
// pair lane L with L^1, L^2 (quad swaps), L^7 (row_half_mirror), L^15 (row_mirror), L^16,
// L^32 (gfx950 permlane16/32 swaps).  Over GF(2) the masks {1,2,7,15,16,32} are a basis of
// the lane index; in its coordinates c(L) every stage is the standard xor butterfly, so lane L
// holds the sample at x = c & 7, y = c >> 3 (me_had_xy) and takes the butterfly role of
// coordinate bit k (low: a + b, high: b - a).  The result is the reference's 8x8 Hadamard up
// to coefficient order (TComRdCost::xCalcHADs8x8 sums magnitudes, so the SATD is identical).
__device__ __forceinline__ int me_had_c(int lane) {
  const int b2 = (lane >> 2) & 1, b3 = (lane >> 3) & 1;
  return lane ^ (b2 * 3) ^ (b3 * 4);
}
__device__ __forceinline__ void me_had_xy(int lane, int &x, int &y) {
  const int c = me_had_c(lane);
  x = c & 7; y = c >> 3;
}
// The same transform on int16 pairs: p[i] holds two candidates' values (lo, hi) and every
// butterfly is one partner fetch + one v_pk_mad_i16 (sign * own + partner) for both.  8-bit
// inputs: |values| <= 64 * 510 after the 6 stages, inside int16.
template <int NP>
__device__ __forceinline__ void had8_xlane_pk(uint32_t (&p)[NP]) {
  const int c = me_had_c(lane_id());
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const short sg1 = (short)(1 - (((c >> k) & 1) << 1));
    const me_s2 sg = {sg1, sg1};
#pragma unroll
    for (int i = 0; i < NP; i++) {
      if (k < 4) {
        uint32_t t;
        if (k == 0) t = (uint32_t)__builtin_amdgcn_mov_dpp((int)p[i], 0xB1, 0xf, 0xf, false);
        else if (k == 1) t = (uint32_t)__builtin_amdgcn_mov_dpp((int)p[i], 0x4E, 0xf, 0xf, false);
        else if (k == 2) t = (uint32_t)__builtin_amdgcn_mov_dpp((int)p[i], 0x141, 0xf, 0xf, false);
        else t = (uint32_t)__builtin_amdgcn_mov_dpp((int)p[i], 0x140, 0xf, 0xf, false);
        p[i] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(me_s2, t) + sg * __builtin_bit_cast(me_s2, p[i]));
      } else {
        const auto pr = k == 4 ? __builtin_amdgcn_permlane16_swap(p[i], p[i], false, false)
                               : __builtin_amdgcn_permlane32_swap(p[i], p[i], false, false);
        p[i] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(me_s2, (uint32_t)pr[0]) +
                                                sg * __builtin_bit_cast(me_s2, (uint32_t)pr[1]));
      }
    }
  }
}

// wave-wide sum (every lane active): DPP adds inside rows of 16, the 4 row sums on the SALU
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
  v += ME_DPP(v, 0xB1);
  v += ME_DPP(v, 0x4E);
  v += ME_DPP(v, 0x141);
  v += ME_DPP(v, 0x140);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

// second filter stage of one candidate sample from a column window hw[t] = hp[c] row
// (ryb + 1 + y + t), t = 0..8; off = ry - ryb (0 or 1) and fy are wave-uniform
__device__ __forceinline__ int me_vsample(const int *hw, int off, int fy) {
  if (!fy) return clip_pel(((off ? hw[4] : hw[3]) + 8192 + 32) >> 6);
  int s = 0;
  if (off) {
#pragma unroll
    for (int t = 0; t < 8; t++) s += kLumaFilter[fy][t] * hw[t + 1];
  } else {
#pragma unroll
    for (int t = 0; t < 8; t++) s += kLumaFilter[fy][t] * hw[t];
  }
  return clip_pel((s + (1 << 11) + (8192 << 6)) >> 12);
}

// The same second stage read straight from the phase plane: h points at the first tap's row
// (row stride HS).  Each tap pair is loaded as an int16 pair (ds_read_u16 + _d16_hi) and
// accumulated by one v_dot2_i32_i16, so the per-tap multiplies and the per-lane window
// selection of me_vsample disappear.
template <int HS>
__device__ __forceinline__ int me_vsample_pk(const int16_t *h, int fy) {
  if (!fy) return clip_pel((h[3 * HS] + 8192 + 32) >> 6);
  int s = (1 << 11) + (8192 << 6);
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const me_s2 pr = {h[(2 * u) * HS], h[(2 * u + 1) * HS]};
    s = __builtin_amdgcn_sdot2(pr, __builtin_bit_cast(me_s2, kLumaPairs[fy][u]), s, false);
  }
  return clip_pel(s >> 12);
}

// Sums over the wave of the 9 candidates' |coefficient| vectors at once: permlane32 swaps
// fold candidate pairs (2k, 2k+1) into the two wave halves, permlane16 swaps fold those pairs
// into rows, DPP adds finish inside rows.  Every lane of row r of u[k] then holds the sum of
// candidate 4k + {0,2,1,3}[r] (u[2]: row 0 = candidate 8, other rows 0).
template <int NC = 9>  // NC = 8: a[8] unused, u[2] = 0
__device__ __forceinline__ void me_sum9(const int (&a)[9], uint32_t (&u)[3]) {
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const auto p = __builtin_amdgcn_permlane32_swap((unsigned)a[2 * k], (unsigned)a[2 * k + 1], false, false);
    w[k] = p[0] + p[1];
  }
  if constexpr (NC == 9) {
    const auto p = __builtin_amdgcn_permlane32_swap((unsigned)a[8], 0u, false, false);
    w[4] = p[0] + p[1];
  } else {
    w[4] = 0;
  }
  {
    const auto p = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
    u[0] = p[0] + p[1];
  }
  {
    const auto p = __builtin_amdgcn_permlane16_swap(w[2], w[3], false, false);
    u[1] = p[0] + p[1];
  }
  if constexpr (NC == 9) {
    const auto p = __builtin_amdgcn_permlane16_swap(w[4], 0u, false, false);
    u[2] = p[0] + p[1];
  } else {
    u[2] = 0;
  }
#pragma unroll
  for (int k = 0; k < (NC == 9 ? 3 : 2); k++) {
    u[k] += ME_DPP(u[k], 0xB1);
    u[k] += ME_DPP(u[k], 0x4E);
    u[k] += ME_DPP(u[k], 0x141);
    u[k] += ME_DPP(u[k], 0x140);
  }
}

typedef _Float16 me_h4 __attribute__((ext_vector_type(4)));
typedef float me_f4 __attribute__((ext_vector_type(4)));

// The block-diagonal diag(H8, H8) (Sylvester order, symmetric) as a v_mfma_f32_16x16x16_f16
// operand fragment: lane l holds element [l & 15][4 (l >> 4) + j] -- the A fragment, and by
// symmetry also the B fragment.
__device__ __forceinline__ me_h4 me_hb_frag(int lane) {
  const int r = lane & 15;
  me_h4 h;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = 4 * (lane >> 4) + j;
    h[j] = (r >> 3) != (k >> 3) ? (_Float16)0.0f : (__popc(r & k & 7) & 1) ? (_Float16)-1.0f : (_Float16)1.0f;
  }
  return h;
}

// xCalcHADs8x8 (TComRdCost.cpp) of the four 8x8 tiles of a 16x16 difference block D on two
// MFMAs.  (a0, a1) is the lane's A fragment -- row lane & 15, columns 4 (lane >> 4) .. +3 -- as
// f16 bit patterns 0x6600 + d, i.e. exactly 1536 + d for |d| <= 255; cb holds -12288 in columns
// 0 and 8, which cancels the bias through the H8 column sums.  X = D diag(H8,H8) (|X| <= 2040,
// exact in f16), Z = diag(H8,H8) X = H8 D H8 per tile (|Z| <= 16320); all sums are integers
// below 2^24, so f32 accumulation is exact in any order.  Returns in every lane (sum |Z| + 2) >> 2
// of the tile at (row half lane >> 5, column half (lane >> 3) & 1) of Z's layout.
__device__ __forceinline__ uint32_t me_satd4_mfma(uint32_t a0, uint32_t a1, me_h4 hb, me_f4 cb) {
  const me_h4 a = __builtin_bit_cast(me_h4, me_v2u{a0, a1});
  const me_f4 x = __builtin_amdgcn_mfma_f32_16x16x16f16(a, hb, cb, 0, 0, 0);
  const uint32_t p0 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x[0], x[1]));
  const uint32_t p1 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x[2], x[3]));
  const me_h4 xb = __builtin_bit_cast(me_h4, me_v2u{p0, p1});
  const me_f4 z = __builtin_amdgcn_mfma_f32_16x16x16f16(hb, xb, me_f4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
  uint32_t v = (uint32_t)(fabsf(z[0]) + fabsf(z[1]) + fabsf(z[2]) + fabsf(z[3]));
  v += ME_DPP(v, 0xB1);   // lanes ^1
  v += ME_DPP(v, 0x4E);   // ^2
  v += ME_DPP(v, 0x141);  // the other quad of the half row
  const auto pr = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // lanes ^16
  v = (uint32_t)pr[0] + (uint32_t)pr[1];
  return (v + 2) >> 2;
}

// candidate index (s_acMvRefineH / s_acMvRefineQ order) of slot c*3 + d, (dx, dy) = (c-1, d-1),
// as 4-bit fields
constexpr uint64_t kRefSlotH = 0x846201735ull, kRefSlotQ = 0x864201753ull;


// xPatternRefinement (:808): the 9 candidates of one stage.  (qx0,qy0) = stage centre in
// quarter-pel relative to the PU, step 2 (half) or 1 (quarter); (ix,iy) the integer MV.
// The NW waves of the job share the phase planes and take candidates i = wave, wave+NW, ...
// GENERIC: any block shape up to SxS; otherwise square SxS blocks only (the CTU pass).
// QC (quarter stage): the centre candidate is the half stage's best, whose cost (ccost) the half
// stage already computed from the same samples and MV; the tile work covers the other 8 only.
template <int S, int NW, bool GENERIC, typename TO, bool QC = false>
__device__ uint32_t me_frac_stage(MeFracSmem<S, NW, TO> &sm, const hvx_me_job &j, const uint8_t *ref, int stride, int ix,
                                  int iy, int qx0, int qy0, int step, int scale, int mvx0, int mvy0, int &bi,
                                  uint32_t ccost = 0) {
  constexpr int HS = MeFracSmem<S, NW, TO>::HS;
  // the stage geometry is wave-uniform: held in SGPRs, the phase / offset selections below are
  // scalar branches instead of per-tap v_cndmask
  ix = uni(ix); iy = uni(iy); qx0 = uni(qx0); qy0 = uni(qy0);
  const int w = GENERIC ? j.w : S, h = GENERIC ? j.h : S, lane = lane_id(), wave = NW > 1 ? (int)(threadIdx.x >> 6) : 0;
  const bool had = (j.flags & HVX_ME_HADME) != 0;
  // 1. horizontal phases: column c at quarter x = qx0 + (c-1)*step, integer offset ix-1 or ix
  // (oxo 0/1), phase fx.  In the half stage columns 0 and 2 are the same half-sample filter one
  // pixel apart: one plane of S+1 columns serves both (po[2] = po[0] + 1).  An item (row r,
  // columns x0..x0+3) loads the 12 bytes at columns x0+ix-4 .. x0+ix+7 (one buffer load),
  // forms the byte pairs and filters two outputs per v_pk_mad (8-bit taps and samples, 16-bit
  // intermediates: the reference's first stage, offset -8192, fits int16 exactly).
  me_sync<NW>();
  int po[3];
  {
    int oxo[3], fxs[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const int qx = qx0 + (c - 1) * step;
      oxo[c] = (qx >> 2) - ix + 1;  // 0 or 1
      fxs[c] = qx & 3;
    }
    constexpr int PL = (S + 8) * HS;  // elements per plane
    const bool shared = fxs[0] == fxs[2] && oxo[2] == oxo[0] + 1;
    po[0] = 0; po[1] = PL; po[2] = shared ? 1 : 2 * PL;
    const int gw = w >> 2, gwp = gw + (shared ? 1 : 0);
    const __amdgpu_buffer_rsrc_t rs = me_plane_rsrc(ref - (j.pu_y * stride + j.pu_x), stride, j.pic_h);
    const uint32_t base = (uint32_t)((HVX_PLANE_MARGIN + j.pu_y + iy - 4) * stride + HVX_PLANE_MARGIN + j.pu_x + ix - 4);
    for (int k = me_tid<NW>(); k < (h + 8) * gwp; k += 64 * NW) {
      const int r = k / gwp, x0 = (k - r * gwp) << 2;
      const uint32_t a = base + (uint32_t)(r * stride + x0);
      const me_v4u q = __builtin_amdgcn_raw_buffer_load_b128(rs, a & ~3u, 0, 0);
      const uint32_t sh = a & 3u;
      // the 12 bytes as signed bytes b - 128: then sum_t c_t * (b_t - 128) = sum_t c_t * b_t - 64 * 128,
      // which is the reference's first-stage value with its -8192 offset, one v_dot4_i32_i8 per 4 taps
      const uint32_t wv[3] = {__builtin_amdgcn_alignbyte(q.y, q.x, sh) ^ 0x80808080u,
                              __builtin_amdgcn_alignbyte(q.z, q.y, sh) ^ 0x80808080u,
                              __builtin_amdgcn_alignbyte(q.w, q.z, sh) ^ 0x80808080u};
      uint32_t W[9];  // W[s] = bytes s .. s+3
#pragma unroll
      for (int t = 0; t < 9; t++) W[t] = (t & 3) ? __builtin_amdgcn_alignbyte(wv[(t >> 2) + 1], wv[t >> 2], t & 3) : wv[t >> 2];
#pragma unroll
      for (int c = 0; c < 3; c++) {
        if (c == 2 && shared) continue;
        if (c != 0 && x0 >= w) continue;  // the extra column item only feeds the shared plane
        const int fx = fxs[c], o0 = oxo[c];
        int ov[4];
        if (!fx) {
#pragma unroll
          for (int i = 0; i < 4; i++) {  // (b - 128) * 64 of byte 3 + o0 + i
            const int bi = 3 + o0 + i;
            ov[i] = (int)(int8_t)(W[bi & ~3] >> (8 * (bi & 3))) * 64;
          }
        } else {
          const int clo = (int)kLumaTap4[fx][0], chi = (int)kLumaTap4[fx][1];
          if (o0) {
#pragma unroll
            for (int i = 0; i < 4; i++) ov[i] = __builtin_amdgcn_sdot4((int)W[i + 5], chi, __builtin_amdgcn_sdot4((int)W[i + 1], clo, 0, false), false);
          } else {
#pragma unroll
            for (int i = 0; i < 4; i++) ov[i] = __builtin_amdgcn_sdot4((int)W[i + 4], chi, __builtin_amdgcn_sdot4((int)W[i], clo, 0, false), false);
          }
        }
        uint32_t *dst = (uint32_t *)(&sm.hp[0][0] + po[c] + r * HS + x0);  // 8-byte aligned
        dst[0] = __builtin_amdgcn_perm((uint32_t)ov[1], (uint32_t)ov[0], 0x05040100u);
        dst[1] = __builtin_amdgcn_perm((uint32_t)ov[3], (uint32_t)ov[2], 0x05040100u);
      }
    }
  }
  me_sync<NW>();
  // 2. the 9 candidates' costs (SATD or SAD + MV cost)
  const bool xl = had && (!GENERIC || ((w % 8 == 0) && (h % 8 == 0)));
  const int tw = w >> 3, nt = (w * h) >> 6;
  if constexpr (!GENERIC && sizeof(TO) == 1) {
    if (xl) {
      // Square blocks of the CTU pass: the Hadamards on MFMA (me_satd4_mfma), four 8x8 tiles per
      // pair of MFMAs.  S == 8: one pair per vertical phase d, its tiles the candidates
      // (c, d), c = 0..2, of the three column phases (the fourth tile repeats c = 2); S >= 16: one
      // pair per 16x16 region and candidate, the regions spread over the job's waves.
      const me_h4 hb = me_hb_frag(lane);
      const float cbv = (lane & 7) == 0 ? -12288.0f : 0.0f;
      const me_f4 cb = {cbv, cbv, cbv, cbv};
      int offs[3], fys[3];
      int ryb = 0;
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const int qy = qy0 + (d - 1) * step, ry = (qy >> 2) - iy;
        if (d == 0) ryb = ry;
        offs[d] = ry - ryb; fys[d] = qy & 3;
      }
      // A-fragment geometry: tile (row half b3, column half b5), tile row lane & 7, columns 4 b4 .. +3
      const int b3 = (lane >> 3) & 1, b4 = (lane >> 4) & 1, b5 = lane >> 5;
      if constexpr (S == 8) {
        const int y = lane & 7, x = 4 * b4, qa = 2 * b3 + b5, qz = 2 * b5 + b3;
        const int pol = qa == 0 ? po[0] : qa == 1 ? po[1] : po[2];
        const uint32_t ow = *(const uint32_t *)&sm.org[y * S + x];
        const uint32_t ob0 = __builtin_amdgcn_perm(0u, ow, 0x0c010c00u) + 0x66006600u;
        const uint32_t ob1 = __builtin_amdgcn_perm(0u, ow, 0x0c030c02u) + 0x66006600u;
        const bool rep = (lane & 0x17) == 0 && qz < 3;  // lanes 0, 8, 32: the sums of tiles 0, 1, 2
#pragma unroll
        for (int d = 0; d < 3; d++) {
          const int16_t *h = &sm.hp[0][0] + pol + (ryb + 1 + y + offs[d]) * HS + x;
          uint32_t pv[4];
#pragma unroll
          for (int k = 0; k < 4; k++) pv[k] = (uint32_t)me_vsample_pk<HS>(h + k, fys[d]);
          const uint32_t t = me_satd4_mfma(ob0 - (pv[0] | (pv[1] << 16)), ob1 - (pv[2] | (pv[3] << 16)), hb, cb);
          if (rep) sm.sat[0][3 * qz + d] = t;
        }
      } else {
        constexpr int RW = S / 16, NRG = RW * RW;
        uint32_t acc[9];
#pragma unroll
        for (int k = 0; k < 9; k++) acc[k] = 0;
        for (int rg = wave; rg < NRG; rg += NW) {
          const int y = (rg / RW) * 16 + 8 * b3 + (lane & 7), x = (rg % RW) * 16 + 8 * b5 + 4 * b4;
          const uint32_t ow = *(const uint32_t *)&sm.org[y * S + x];
          const uint32_t ob0 = __builtin_amdgcn_perm(0u, ow, 0x0c010c00u) + 0x66006600u;
          const uint32_t ob1 = __builtin_amdgcn_perm(0u, ow, 0x0c030c02u) + 0x66006600u;
#pragma unroll
          for (int sl = 0; sl < 9; sl++) {
            if (QC && sl == 4) continue;
            const int c = sl / 3, d = sl % 3;
            const int16_t *h = &sm.hp[0][0] + po[c] + (ryb + 1 + y + offs[d]) * HS + x;
            uint32_t pv[4];
#pragma unroll
            for (int k = 0; k < 4; k++) pv[k] = (uint32_t)me_vsample_pk<HS>(h + k, fys[d]);
            acc[sl] += me_satd4_mfma(ob0 - (pv[0] | (pv[1] << 16)), ob1 - (pv[2] | (pv[3] << 16)), hb, cb);
          }
        }
#pragma unroll
        for (int sl = 0; sl < 9; sl++) {
          if (QC && sl == 4) continue;
          uint32_t v = acc[sl] + ME_DPP(acc[sl], 0x140);  // the other column half (row_mirror)
          const auto pr = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // the other row half
          v = (uint32_t)pr[0] + (uint32_t)pr[1];
          if (lane == 0) sm.sat[wave][sl] = v;
        }
      }
      me_sync<NW>();
      // lane-parallel costs: lane sl < 9 takes slot sl; first minimum in the reference's order
      const bool valid = lane < 9;
      const int sl = valid ? lane : 0;
      uint32_t dsum = 0;
#pragma unroll
      for (int ww = 0; ww < NW; ww++) dsum += sm.sat[ww][sl];
      const int c = (sl * 11) >> 5, dx = c - 1, dy = sl - 3 * c - 1;
      const uint64_t idx = step == 2 ? kRefSlotH : kRefSlotQ;
      const int ci = (int)((idx >> (4 * sl)) & 15);
      const uint32_t cost = (QC && sl == 4) ? ccost
                                            : dsum + me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, scale, mvx0 + dx, mvy0 + dy);
      const uint32_t key = wave_min_key(valid ? (cost << 4) | (uint32_t)ci : kMeKeyNone);
      bi = (int)(key & 15u);
      return key >> 4;
    }
  }
  int hx, hy;
  me_had_xy(lane, hx, hy);
  if (xl) {
    // all 9 candidates per 8x8 tile, the tiles spread over the job's waves: per column phase c
    // the 9-row window of hp[c] the 3 vertical phases need is read once; the 9 tiles' Hadamards
    // run side by side on DPP butterflies and are summed together (me_sum9)
    int offs[3], fys[3];
    int ryb = 0;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int qy = qy0 + (d - 1) * step, ry = (qy >> 2) - iy;
      if (d == 0) ryb = ry;
      offs[d] = ry - ryb; fys[d] = qy & 3;
    }
    uint32_t acc[3] = {0u, 0u, 0u};
    for (int t = wave; t < nt; t += NW) {
      const int x = ((t % tw) << 3) + hx, y = ((t / tw) << 3) + hy;
      const int o = sm.org[y * S + x];
      int v[9] = {};
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int16_t *h = &sm.hp[0][0] + po[c] + (ryb + 1 + y) * HS + x;
#pragma unroll
        for (int d = 0; d < 3; d++)
          if (!QC || c * 3 + d != 4) v[c * 3 + d] = o - me_vsample_pk<HS>(h + offs[d] * HS, fys[d]);
      }
      // candidate pairs as int16 halves: (0,1) (2,3) (4,5) (6,7) (8,-); QC: (0,1) (2,3) (5,6) (7,8)
      constexpr int NP = QC ? 4 : 5;
      int w[9];
#pragma unroll
      for (int k = 0; k < 9; k++) w[k] = QC ? v[k < 4 ? k : (k < 8 ? k + 1 : 0)] : v[k];
      uint32_t pk[NP];
#pragma unroll
      for (int k = 0; k < 4; k++) pk[k] = __builtin_amdgcn_perm((uint32_t)w[2 * k + 1], (uint32_t)w[2 * k], 0x05040100u);
      if constexpr (!QC) pk[NP - 1] = (uint32_t)w[8] & 0xffffu;
      had8_xlane_pk<NP>(pk);
#pragma unroll
      for (int k = 0; k < NP; k++) {
        const me_s2 x = __builtin_bit_cast(me_s2, pk[k]);
        pk[k] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, -x));
      }
#pragma unroll
      for (int k = 0; k < 4; k++) { w[2 * k] = (int)(pk[k] & 0xffffu); w[2 * k + 1] = (int)(pk[k] >> 16); }
      w[8] = QC ? 0 : (int)(pk[NP - 1] & 0xffffu);
      uint32_t u[3];
      me_sum9<QC ? 8 : 9>(w, u);
#pragma unroll
      for (int k = 0; k < (QC ? 2 : 3); k++) acc[k] += (u[k] + 2) >> 2;  // xCalcHADs8x8 rounding per tile
    }
    // lane-parallel costs: lane (row r, kk = lane & 15 < 3) takes the slot s = c*3 + d me_sum9
    // put there; the first minimum in the reference's candidate order is a (cost, index) key-min
    const int kk = lane & 15, r = lane >> 4;
    const bool valid = kk < 2 || (kk == 2 && r == 0);
    uint32_t dsum = kk == 0 ? acc[0] : kk == 1 ? acc[1] : acc[2];
    if constexpr (NW > 1) {  // the waves' partial sums, added in wave order through LDS
      if (kk == 0) {
#pragma unroll
        for (int k = 0; k < 3; k++) sm.part[wave][k][r] = acc[k];
      }
      __syncthreads();
      dsum = 0;
      if (valid) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) dsum += sm.part[ww][kk < 3 ? kk : 0][r];
      }
    }
    const int wi = 4 * kk + ((0xD8 >> (2 * r)) & 3);  // the me_sum9 slot of this lane (kk < 2)
    const int sl = QC ? (kk >= 2 ? 4 : wi + (wi >= 4)) : (kk >= 2 ? 8 : wi);
    const int c = (sl * 11) >> 5, dx = c - 1, dy = sl - 3 * c - 1;  // sl / 3, sl % 3 for sl < 9
    const uint64_t idx = step == 2 ? kRefSlotH : kRefSlotQ;
    const int ci = (int)((idx >> (4 * sl)) & 15);
    const uint32_t cost = (QC && kk >= 2) ? ccost
                                           : dsum + me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, scale, mvx0 + dx, mvy0 + dy);
    const uint32_t key = wave_min_key(valid ? (cost << 4) | (uint32_t)ci : kMeKeyNone);
    bi = (int)(key & 15u);
    return key >> 4;
  }
  for (int i = wave; i < 9 && !xl; i += NW) {
    const int dx = step == 2 ? kRefH[i][0] : kRefQ[i][0], dy = step == 2 ? kRefH[i][1] : kRefQ[i][1];
    const int qy = qy0 + dy * step, ry = (qy >> 2) - iy, fy = qy & 3, c = dx + 1;
    uint32_t d = 0;
    if (had) {
      if (GENERIC) {
        uint8_t *blk = sm.blk[wave];
        for (int k = lane; k < w * h; k += HVX_WAVE) {
          const int y = k / w, x = k - y * w;
          blk[y * S + x] = (uint8_t)me_frac_sample(sm, me_sel3(po, c), ry, fy, x, y);
        }
        // the wave's lanes read each other's samples: release, wave barrier, acquire (the barrier
        // alone does not order memory -- with the fences after it the reads could be hoisted)
        me_sync<1>();
        d = wave_satd(sm.org, S, (const uint8_t *)blk, S, w, h);
      }
    } else {
      uint32_t sacc = 0;
      for (int k = lane; k < w * h; k += HVX_WAVE) {
        const int y = k / w, x = k - y * w;
        sacc += (uint32_t)abs((int)sm.org[y * S + x] - me_frac_sample(sm, me_sel3(po, c), ry, fy, x, y));
      }
      d = wave_sum_u32(sacc);
    }
    d += me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, scale, mvx0 + dx, mvy0 + dy);
    if (lane == 0) sm.cost[i] = d;
  }
  me_sync<NW>();
  // 3. reference order, strict '<'
  uint32_t best = 0xFFFFFFFFu;
  bi = 0;
  for (int i = 0; i < 9; i++) {
    const uint32_t d = sm.cost[i];
    if (d < best) { best = d; bi = i; }
  }
  return best;
}

template <int S, int NW, bool GENERIC, typename TO>
__device__ void me_frac_refine(const hvx_me_job &j, const uint8_t *ref, int stride, int ix, int iy, uint32_t sad_int,
                               MeFracSmem<S, NW, TO> &sm, hvx_me_result *out);

template <int S, int NW, bool GENERIC>
__device__ void me_frac_job(const hvx_me_job &j, const uint8_t *const *__restrict__ cur_planes,
                            const uint8_t *const *__restrict__ ref_planes, int stride, MeFracSmem<S, NW> &sm,
                            hvx_me_result *out) {
  if (j.w <= 0 || j.h <= 0 || j.w > S || j.h > S) return;  // k_me_int wrote the empty result
  if (!GENERIC && (j.w != S || j.h != S)) return;
  const int ix = out->mv_int_x, iy = out->mv_int_y;
  const uint32_t sad_int = out->sad_int;
  const uint8_t *cur = cur_planes[j.cur_idx] + j.pu_y * stride + j.pu_x;
  for (int k = threadIdx.x; k < j.w * j.h; k += 64 * NW) {
    const int y = k / j.w, x = k - y * j.w;
    sm.org[y * S + x] = cur[y * stride + x];
  }
  const uint8_t *ref = ref_planes[j.ref_idx] + j.pu_y * stride + j.pu_x;
  me_frac_refine<S, NW, GENERIC, uint8_t>(j, ref, stride, ix, iy, sad_int, sm, out);
}

// xPatternSearchFracDIF (:4240) from the integer result (ix, iy, sad_int), the original block
// already in sm.org; writes the complete hvx_me_result.
template <int S, int NW, bool GENERIC, typename TO>
__device__ void me_frac_refine(const hvx_me_job &j, const uint8_t *ref, int stride, int ix, int iy, uint32_t sad_int,
                               MeFracSmem<S, NW, TO> &sm, hvx_me_result *out) {
  // half-pel around the integer MV, then quarter-pel
  int bh, bq;
  const uint32_t hcost =
      me_frac_stage<S, NW, GENERIC, TO>(sm, j, ref, stride, ix, iy, ix << 2, iy << 2, 2, 1, ix << 1, iy << 1, bh);
  const int hx = kRefH[bh][0], hy = kRefH[bh][1];
  const int cqx = (ix << 2) + (hx << 1), cqy = (iy << 2) + (hy << 1);
  const uint32_t cost =
      me_frac_stage<S, NW, GENERIC, TO, true>(sm, j, ref, stride, ix, iy, cqx, cqy, 1, 0, cqx, cqy, bq, hcost);
  const int qx = kRefQ[bq][0], qy = kRefQ[bq][1];
  const int fmx = cqx + qx, fmy = cqy + qy;
  const uint32_t mv_bits = eg_bits(fmx - j.pred_x) + eg_bits(fmy - j.pred_y);
  const uint32_t bits = (uint32_t)j.bits_in + mv_bits;
  const uint32_t lam = j.lambda_motion;
  if (me_tid<NW>() == 0) {
    hvx_me_result r;
    r.mv_int_x = ix; r.mv_int_y = iy; r.sad_int = sad_int;
    r.half_x = hx; r.half_y = hy; r.qtr_x = qx; r.qtr_y = qy; r.cost_frac = cost;
    r.mv_x = fmx; r.mv_y = fmy; r.bits = bits;
    const double wgt = (j.flags & HVX_ME_BI) ? 0.5 : 1.0;  // fWeight (TEncSearch.cpp:3696, :3759)
    r.cost = (uint32_t)(floor(wgt * ((double)cost - (double)((lam * mv_bits) >> 16))) + (double)((lam * bits) >> 16));
    *out = r;
  }
}

// generic jobs (any PU shape up to 64x64), 4 waves per job
static __global__ __launch_bounds__(256) void k_me_frac(const uint8_t *const *__restrict__ cur_planes,
                                                const uint8_t *const *__restrict__ ref_planes, int stride,
                                                const hvx_me_job *__restrict__ jobs, int n, hvx_me_result *__restrict__ out) {
  __shared__ MeFracSmem<64, 4> sm;
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_me_job j = jobs[jid];
  me_frac_job<64, 4, true>(j, cur_planes, ref_planes, stride, sm, out + jid);
}

// ======================================================================================
// integer full search: xMotionEstimation with FastSearch=0 or bBi (TEncSearch.cpp:3728-3730)
// ======================================================================================
// xPatternSearch (:3786): every integer position of the (clipped) range around the centre in
// raster order, strict '<' -> the first minimum of SAD + MV cost.  One 256-thread workgroup
// per job: thread t takes points t, t+256, ... and keeps its first minimum as a
// (cost, raster index) key; a workgroup key-min picks the reference's point.  The pattern is
// int16 (a bi target 2*org - other spans [-255, 510]), so SADs are plain |a - b| sums.
static __global__ __launch_bounds__(256) void k_me_full(const int16_t *const *__restrict__ tgt_planes, int tstride,
                                                const uint8_t *const *__restrict__ ref_planes, int stride,
                                                const hvx_me_job *__restrict__ jobs, int n, hvx_me_result *__restrict__ out) {
  __shared__ MeFracSmem<64, 4, int16_t> sm;
  __shared__ uint64_t wkey[4];
  const int jid = blockIdx.x;
  if (jid >= n) return;
  const hvx_me_job j = jobs[jid];
  if (j.w <= 0 || j.h <= 0 || j.w > 64 || j.h > 64) {
    if (threadIdx.x == 0) { hvx_me_result z; memset(&z, 0, sizeof(z)); out[jid] = z; }
    return;
  }
  const int16_t *tg = tgt_planes[j.cur_idx] + (size_t)j.pu_y * tstride + j.pu_x;
  for (int k = threadIdx.x; k < j.w * j.h; k += 256) {
    const int y = k / j.w, x = k - y * j.w;
    sm.org[y * 64 + x] = tg[y * tstride + x];
  }
  __syncthreads();
  const uint8_t *ref = ref_planes[j.ref_idx] + j.pu_y * stride + j.pu_x;
  const MeRange g = me_search_range(j, j.center_x, j.center_y, j.search_range);
  // FEN (m_bUseFastEnc) subsamples rows when iRows > 8 (:3810); the reference's specialised
  // SAD widths honour iSubShift, the generic one does not (TComRdCost.cpp:461-950)
  const int w = j.w;
  const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  const int sub = ((j.flags & HVX_ME_FEN) && j.h > 8 && spec) ? 1 : 0;
  const int nx = g.r - g.l + 1, np = nx * (g.b - g.t + 1);
  uint64_t best = ~0ull;
  for (int p = threadIdx.x; p < np; p += 256) {
    const int py = p / nx, x = g.l + (p - py * nx), y = g.t + py;
    const uint8_t *r = ref + y * stride + x;
    uint32_t s = 0;
    for (int row = 0; row < j.h; row += 1 << sub)
      for (int c = 0; c < w; c++) s += (uint32_t)abs((int)sm.org[row * 64 + c] - (int)r[row * stride + c]);
    const uint32_t cost = (s << sub) + me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, 2, x, y);
    const uint64_t key = ((uint64_t)cost << 32) | (uint32_t)p;
    best = key < best ? key : best;
  }
  best = wave_min_u64(best);
  if (lane_id() == 0) wkey[threadIdx.x >> 6] = best;
  __syncthreads();
  best = wkey[0];
  for (int k = 1; k < 4; k++) best = wkey[k] < best ? wkey[k] : best;
  const int bp = (int)(uint32_t)best, by = bp / nx;
  const int ix = g.l + (bp - by * nx), iy = g.t + by;
  const uint32_t sad_int = (uint32_t)(best >> 32) - me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, 2, ix, iy);
  // the fractional refinement reads the same pattern (stride 64 = S)
  me_frac_refine<64, 4, true, int16_t>(j, ref, stride, ix, iy, sad_int, sm, out + jid);
}
