// hvx_intra.hpp -- intra reference samples, prediction and the first-pass mode search (gfx950).
// Restated by oracle/hvx_oracle.c ("Intra prediction"); SURVEY.md 8(f) item 2.
//
// One wave per block.  The reference border (HM's m_piYuvExt row 0 / column 0: B[0] = above-left,
// B[1..2N] = above + above-right, B[2N+1..4N] = left + below-left top-down) is built straight from
// the 8-bit plane into LDS: every lane resolves its own border positions, including HM's
// substitution of unavailable units (fillReferenceSamples, TComPattern.cpp:364-540) -- a gap
// takes the last sample of the nearest available unit below it in HM's line order, or, with none
// below, the first sample of the nearest one above -- by bit scans over the 65-bit availability
// mask, so there is no serial walk.  The [1 2 1] / strong-bilinear smoothing (TComPattern.cpp:
// 190-330) is one more lane-parallel pass over LDS.
//
// The first-pass search (estIntraPredLumaQT, TEncSearch.cpp:2244-2323) maps (mode, Hadamard tile)
// pairs onto lanes: 35 modes x (N/8)^2 8x8 tiles (4x4 tiles for N = 4), so a 4x4/8x8 PU keeps 35
// lanes busy and a 64x64 PU 2240 tile jobs; each lane predicts its tile sample by sample from the
// LDS border, differences against the LDS original, transforms in registers and adds its SATD to
// the mode's LDS sum.  The mode rates, the cost ranking (xUpdateCandList :5254, strict '<') and
// the MPM append are 35 scalar steps on lane 0.
#pragma once
#include "hvx_dev.hpp"

namespace intra {
constexpr int kB = 257;  // border samples of a 64x64 block
static __constant__ int8_t kAng[9] = {0, 2, 5, 9, 13, 17, 21, 26, 32};                    // TComPrediction.cpp:287
static __constant__ int16_t kInvAng[9] = {0, 4096, 1638, 910, 630, 482, 390, 315, 256};  // :288
static __constant__ int8_t kFilterThr[5] = {10, 7, 1, 0, 10};                             // m_aucIntraFilter (:50)
static __constant__ int8_t kNumRdMpm[6] = {3, 8, 8, 3, 3, 3}, kNumRdNoMpm[6] = {3, 9, 9, 4, 4, 5};  // TComRom.cpp:545-562

struct Border {
  int16_t unf[kB + 3];
  int16_t filt[kB + 3];
};

__device__ __forceinline__ bool job_ok(const hvx_intra_job &j) {
  return j.ch_type >= 0 && j.ch_type <= 1 && j.log2_size >= 2 && j.log2_size <= (j.ch_type ? 5 : 6) &&
         j.unit_log2 >= 1 && j.unit_log2 <= 2 && j.mode >= 0 && j.mode <= 34;
}

// HM's reference line L (bottom-left upwards, the above-left unit, then the above row): line
// index l -> sample of the plane (p = block origin)
__device__ __forceinline__ int line_raw(const uint8_t *p, int stride, int n, int u, int l) {
  if (l < 2 * n) return p[(2 * n - 1 - l) * stride - 1];
  if (l < 2 * n + u) return p[-stride - 1];
  return p[-stride + (l - 2 * n - u)];
}

__device__ __forceinline__ int highest_below(const uint32_t *a, int uu) {  // available unit < uu, or -1
  for (int w = uu >> 5; w >= 0; w--) {
    uint32_t m = a[w];
    if (w == (uu >> 5)) m &= (1u << (uu & 31)) - 1u;
    if (m) return w * 32 + 31 - __clz(m);
  }
  return -1;
}
__device__ __forceinline__ int lowest_above(const uint32_t *a, int uu) {  // available unit > uu
  for (int w = uu >> 5; w < 3; w++) {
    uint32_t m = a[w];
    if (w == (uu >> 5)) m &= ~((2u << (uu & 31)) - 1u);
    if (m) return w * 32 + __ffs(m) - 1;
  }
  return 0;  // unreachable when any unit is available
}

// fillReferenceSamples (TComPattern.cpp:364-540), 8-bit, into B (whole wave)
__device__ __forceinline__ void build_border(const uint8_t *p, int stride, int n, int ulog2, const uint32_t *avail,
                                             int16_t *B) {
  const int u = 1 << ulog2, nunits = ((4 * n) >> ulog2) + 1;
  uint32_t a[3];
  int navail = 0;
#pragma unroll
  for (int w = 0; w < 3; w++) {
    const int lo = w * 32;
    a[w] = nunits >= lo + 32 ? avail[w] : nunits > lo ? avail[w] & ((1u << (nunits - lo)) - 1u) : 0u;
    navail += __popc(a[w]);
  }
  for (int k = lane_id(); k <= 4 * n; k += HVX_WAVE) {
    const int l = k == 0 ? 2 * n + u - 1 : k <= 2 * n ? 2 * n + u + k - 1 : 4 * n - k;
    int v = 128;  // no neighbour at all: 1 << (bitDepth - 1) (:384-395)
    if (navail) {
      const int uu = l >> ulog2;
      if ((a[uu >> 5] >> (uu & 31)) & 1) {
        v = line_raw(p, stride, n, u, l);
      } else {
        const int j = highest_below(a, uu);
        v = j >= 0 ? line_raw(p, stride, n, u, j * u + u - 1) : line_raw(p, stride, n, u, lowest_above(a, uu) * u);
      }
    }
    B[k] = (int16_t)v;
  }
}

// F order (bottom-left .. above-left .. above-right) -> B index
__device__ __forceinline__ int f_index(int n, int k) { return k < 2 * n ? 4 * n - k : k == 2 * n ? 0 : k - 2 * n; }

// initIntraPatternChType's smoothing (TComPattern.cpp:190-330) B -> out (whole wave)
__device__ __forceinline__ void filter_border(const int16_t *B, int n, int log2n, bool luma, bool strong_en,
                                              int16_t *out) {
  const int bl = B[4 * n], tl = B[0], tr = B[2 * n];
  const bool strong = luma && strong_en && n >= 32 && abs(bl + tl - 2 * B[3 * n]) < 8 && abs(tl + tr - 2 * B[n]) < 8;
  const int shift = log2n + 1;
  for (int k = lane_id(); k <= 4 * n; k += HVX_WAVE) {
    int v;
    if (k == 0 || k == 4 * n) v = B[f_index(n, k)];
    else if (strong && k == 2 * n) v = tl;
    else if (strong && k < 2 * n) v = ((2 * n - k) * bl + k * tl + n) >> shift;
    else if (strong) v = ((4 * n - k) * tl + (k - 2 * n) * tr + n) >> shift;
    else v = (B[f_index(n, k - 1)] + 2 * B[f_index(n, k)] + B[f_index(n, k + 1)] + 2) >> 2;
    out[f_index(n, k)] = (int16_t)v;
  }
}

// filteringIntraReferenceSamples (TComPattern.cpp:544-569), 4:2:0
__device__ __forceinline__ bool use_filter(int mode, int log2n, bool luma) {
  if (!luma || mode == 1) return false;
  const int d10 = abs(mode - 10), d26 = abs(mode - 26);
  return (d10 < d26 ? d10 : d26) > kFilterThr[log2n - 2];
}

// the per-mode constants of predIntraAng
struct Mode {
  int mode, ver, angle, inv;
  __device__ __forceinline__ explicit Mode(int m) : mode(m), ver(m >= 18), angle(0), inv(0) {
    if (m >= 2) {
      const int am = ver ? m - 26 : 10 - m, aa = abs(am);
      angle = (am < 0 ? -kAng[aa] : kAng[aa]);
      inv = kInvAng[aa];
    }
  }
};

// one sample of predIntraAng (TComPrediction.cpp:455-516) with bAbove = bLeft = true and edge
// filters enabled: planar (:756), DC + xDCPredFiltering (:183, :816), xPredIntraAng (:247);
// B(k) = border sample k
template <class F>
__device__ __forceinline__ int pred_sample_f(const F &B, int n, int log2n, const Mode &md, bool edge, int dc, int r,
                                             int c) {
  if (md.mode == 0)
    return ((n - 1 - c) * B(2 * n + 1 + r) + (c + 1) * B(1 + n) + (n - 1 - r) * B(1 + c) + (r + 1) * B(3 * n + 1) + n) >>
           (log2n + 1);
  if (md.mode == 1) {
    if (edge && r == 0 && c == 0) return (B(1) + B(2 * n + 1) + 2 * dc + 2) >> 2;
    if (edge && r == 0) return (B(1 + c) + 3 * dc + 2) >> 2;
    if (edge && c == 0) return (B(2 * n + 1 + r) + 3 * dc + 2) >> 2;
    return dc;
  }
  const int y = md.ver ? r : c, x = md.ver ? c : r;
  // refMain[k] / refSide[k]: the above row (B[k]) or the left column (B[0], B[2n+k])
  auto above = [&](int k) { return B(k); };
  auto left = [&](int k) { return k ? B(2 * n + k) : B(0); };
  auto mainr = [&](int k) {
    if (k >= 0) return md.ver ? above(k) : left(k);
    const int s = (128 - k * md.inv) >> 8;  // the projected side (:321-329)
    return md.ver ? left(s) : above(s);
  };
  if (md.angle == 0) {
    int v = mainr(x + 1);
    if (edge && x == 0) {
      const int s1 = md.ver ? left(y + 1) : above(y + 1), s0 = B(0);
      v = clip_pel(v + ((s1 - s0) >> 1));
    }
    return v;
  }
  const int dp = (y + 1) * md.angle, di = dp >> 5, f = dp & 31;
  if (f) return ((32 - f) * mainr(x + di + 1) + f * mainr(x + di + 2) + 16) >> 5;
  return mainr(x + di + 1);
}

__device__ __forceinline__ int pred_sample(const int16_t *B, int n, int log2n, const Mode &md, bool edge, int dc, int r,
                                           int c) {
  return pred_sample_f([&](int k) { return (int)B[k]; }, n, log2n, md, edge, dc, r, c);
}

__device__ __forceinline__ int dc_value(const int16_t *B, int n, int log2n) {
  int s = 0;
  for (int i = lane_id(); i < n; i += HVX_WAVE) s += B[1 + i] + B[2 * n + 1 + i];
  return (wave_sum_i32(s) + n) >> (log2n + 1);
}

// the block's borders (unfiltered, and filtered for luma) in LDS; returns the DC value
__device__ __forceinline__ int prepare(const hvx_intra_job &j, const uint8_t *rec, int stride, Border &s) {
  const int n = 1 << j.log2_size;
  const bool luma = j.ch_type == 0;
  build_border(rec + (int64_t)j.y * stride + j.x, stride, n, j.unit_log2, j.avail, s.unf);
  __syncthreads();
  if (luma) filter_border(s.unf, n, j.log2_size, true, (j.flags & HVX_INTRA_STRONG) != 0, s.filt);
  const int dc = dc_value(s.unf, n, j.log2_size);
  __syncthreads();
  return dc;
}
}  // namespace intra

// hvx_intra_pred_batch: one wave per job
static __global__ __launch_bounds__(64) void k_intra_pred(const uint8_t *__restrict__ rec, int stride,
                                                   const hvx_intra_job *__restrict__ jobs, int n_jobs,
                                                   uint8_t *__restrict__ pred, const int64_t *__restrict__ off,
                                                   int16_t *__restrict__ ref_out) {
  using namespace intra;
  __shared__ Border s;
  const int i = blockIdx.x;
  if (i >= n_jobs) return;
  const hvx_intra_job j = jobs[i];
  if (!job_ok(j)) return;
  const int n = 1 << j.log2_size, lane = lane_id();
  const bool luma = j.ch_type == 0;
  const int dc = prepare(j, rec, stride, s);
  if (ref_out) {
    int16_t *o = ref_out + (size_t)i * 2 * kB;
    for (int k = lane; k < kB; k += HVX_WAVE) {
      o[k] = k <= 4 * n ? s.unf[k] : 0;
      o[kB + k] = (luma && k <= 4 * n) ? s.filt[k] : 0;
    }
  }
  const Mode md(j.mode);
  const int16_t *B = use_filter(j.mode, j.log2_size, luma) ? s.filt : s.unf;
  const bool edge = luma && n <= 16;
  uint8_t *dst = pred + off[i];
  for (int k = lane; k < n * n; k += HVX_WAVE)
    dst[k] = (uint8_t)pred_sample(B, n, j.log2_size, md, edge, dc, k >> j.log2_size, k & (n - 1));
}

// hvx_intra_search_batch: one wave per luma PU
__device__ __forceinline__ void intra_search_pu(const uint8_t *__restrict__ org, const uint8_t *__restrict__ rec,
                                                int stride, const hvx_intra_job *__restrict__ jobs, int n_jobs,
                                                const int32_t *__restrict__ eb,
                                                hvx_intra_search_result *__restrict__ out, int skip_small, int i) {
  using namespace intra;
  __shared__ Border s;
  __shared__ uint8_t so[64 * 64];
  __shared__ uint32_t satd[36];
  __shared__ int s_list[12], s_mpm[3];   // lane 0's candidate list in LDS (no dynamically indexed
  __shared__ double s_cc[10];            // private arrays -> no scratch)
  const hvx_intra_job j = jobs[i];
  if (!job_ok(j) || j.ch_type != 0 || (skip_small && j.log2_size <= 3)) return;  // 4x4/8x8: k_intra_search_lane
  const int log2n = j.log2_size, n = 1 << log2n, lane = lane_id();
  const uint8_t *po = org + (int64_t)j.y * stride + j.x;
  for (int k = lane; k < n * n; k += HVX_WAVE) so[k] = po[(k >> log2n) * stride + (k & (n - 1))];
  if (lane < 36) satd[lane] = 0;
  const int dc = prepare(j, rec, stride, s);
  const bool edge = n <= 16;
  // (mode, tile) jobs over lanes
  const int lt = n == 4 ? 2 : 3, t = 1 << lt, tps = n >> lt, ntile = tps * tps;
  for (int idx = lane; idx < 35 * ntile; idx += HVX_WAVE) {
    const int m = idx / ntile, ti = idx - m * ntile, r0 = (ti / tps) << lt, c0 = (ti % tps) << lt;
    const Mode md(m);
    const int16_t *B = use_filter(m, log2n, true) ? s.filt : s.unf;
    uint32_t sum = 0;
    if (t == 8) {
      int d[8][8];
#pragma unroll
      for (int y = 0; y < 8; y++) {
        int row[8];
#pragma unroll
        for (int x = 0; x < 8; x++)
          row[x] = (int)so[(r0 + y) * n + c0 + x] - pred_sample(B, n, log2n, md, edge, dc, r0 + y, c0 + x);
        hadamard8(row, d[y]);
      }
#pragma unroll
      for (int x = 0; x < 8; x++) {
        int col[8], rr[8];
#pragma unroll
        for (int y = 0; y < 8; y++) col[y] = d[y][x];
        hadamard8(col, rr);
#pragma unroll
        for (int k = 0; k < 8; k++) sum += (uint32_t)abs(rr[k]);
      }
      sum = (sum + 2) >> 2;  // xCalcHADs8x8 (TComRdCost.cpp:1428)
    } else {
      int d[4][4];
#pragma unroll
      for (int y = 0; y < 4; y++) {
        int row[4];
#pragma unroll
        for (int x = 0; x < 4; x++) row[x] = (int)so[y * 4 + x] - pred_sample(B, 4, 2, md, edge, dc, y, x);
        hadamard4(row, d[y]);
      }
#pragma unroll
      for (int x = 0; x < 4; x++) {
        int col[4] = {d[0][x], d[1][x], d[2][x], d[3][x]}, rr[4];
        hadamard4(col, rr);
#pragma unroll
        for (int k = 0; k < 4; k++) sum += (uint32_t)abs(rr[k]);
      }
      sum = (sum + 1) >> 1;  // xCalcHADs4x4 (:1374)
    }
    atomicAdd(&satd[m], sum);
  }
  __syncthreads();
  if (lane != 0) return;
  // rates, costs, ranking, MPM append: 35 scalar steps
  int imode;
  int *mpm = s_mpm, *list = s_list;
  double *cc = s_cc;
  const int ld = j.left_dir, ad = j.above_dir;  // getIntraDirPredictor (TComDataCU.cpp:1441-1478)
  if (ld == ad) {
    imode = 1;
    if (ld > 1) { mpm[0] = ld; mpm[1] = ((ld + 29) % 32) + 2; mpm[2] = ((ld - 1) % 32) + 2; }
    else { mpm[0] = 0; mpm[1] = 1; mpm[2] = 26; }
  } else {
    imode = 2;
    mpm[0] = ld; mpm[1] = ad;
    mpm[2] = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  }
  const int mp0 = mpm[0], mp1 = mpm[1], mp2 = mpm[2];
  const bool fast = (j.flags & HVX_INTRA_FAST_MPM) != 0;
  int num = fast ? kNumRdMpm[log2n - 1] : kNumRdNoMpm[log2n - 1];
  for (int k = 0; k < 10; k++) { list[k] = 0; cc[k] = 1.7976931348623157e308; }
  list[10] = list[11] = 0;
  hvx_intra_search_result &r = out[i];  // written in place (a private copy would live in scratch)
  const uint64_t frac = (uint64_t)(uint32_t)j.frac_bits;
  const int st = j.ctx_state & 127;
  const uint64_t eb_mpm = (uint64_t)(uint32_t)eb[st ^ 1], eb_no = (uint64_t)(uint32_t)eb[st];
  for (int m = 0; m < 35; m++) {
    const int idx = m == mp0 ? 0 : m == mp1 ? 1 : m == mp2 ? 2 : -1;
    // xModeBitsIntra (TEncSearch.cpp:5222): flag bin + 1/2 (MPM index) or 5 bypass bins
    const uint64_t total = frac + (idx >= 0 ? eb_mpm : eb_no) + 32768ull * (uint64_t)(idx < 0 ? 5 : idx ? 2 : 1);
    const uint32_t bits = (uint32_t)(total >> 15);
    const uint32_t sd = satd[m];
    r.satd[m] = sd;
    r.mode_bits[m] = (uint8_t)bits;
    const double cost = __dadd_rn((double)sd, __dmul_rn((double)bits, j.sqrt_lambda));
    int sh = 0;  // xUpdateCandList (:5254)
    while (sh < num && cost < cc[num - 1 - sh]) sh++;
    if (sh) {
      for (int k = 1; k < sh; k++) { list[num - k] = list[num - 1 - k]; cc[num - k] = cc[num - 1 - k]; }
      list[num - sh] = m;
      cc[num - sh] = cost;
    }
  }
  r.num_rd = (uint8_t)num;
  for (int k = 0; k < 8; k++) r.cand_cost[k] = k < num ? cc[k] : 0.0;
  if (fast)  // :2299-2321
    for (int q = 0; q < imode; q++) {
      bool inc = false;
      for (int k = 0; k < num; k++) inc |= mpm[q] == list[k];
      if (!inc) list[num++] = mpm[q];
    }
  r.n_cand = (uint8_t)num;
  for (int k = 0; k < 11; k++) r.cand[k] = (uint8_t)(k < num ? list[k] : 0);
  for (int k = 0; k < 4; k++) r.pad_[k] = 0;
}

// one wave per PU, grid-stride over the jobs (so that the 4x4/8x8 jobs it skips cost a load each)
static __global__ __launch_bounds__(64) void k_intra_search(const uint8_t *__restrict__ org, const uint8_t *__restrict__ rec,
                                                     int stride, const hvx_intra_job *__restrict__ jobs, int n_jobs,
                                                     const int32_t *__restrict__ eb,
                                                     hvx_intra_search_result *__restrict__ out, int skip_small) {
  for (int i = blockIdx.x; i < n_jobs; i += gridDim.x) {
    intra_search_pu(org, rec, stride, jobs, n_jobs, eb, out, skip_small, i);
    __syncthreads();  // the LDS of this PU is rewritten by the next
  }
}

// hvx_intra_search_batch for 4x4 and 8x8 luma PUs (75% of a picture's PUs): one PU per LANE.
// The 35-mode loop is uniform across the wave (mode constants and the filtered/unfiltered choice
// are per size), each lane predicts its own PU from its own border column in LDS ([k][lane]:
// conflict-free), transforms in registers and ranks its candidates in registers: xUpdateCandList's
// insertion as a fixed 9-slot network with static indices, so nothing is dynamically indexed.
template <int LOG2N>
static __global__ __launch_bounds__(64) void k_intra_search_lane(const uint8_t *__restrict__ org, const uint8_t *__restrict__ rec,
                                                          int stride, const hvx_intra_job *__restrict__ jobs, int n_jobs,
                                                          const int32_t *__restrict__ eb,
                                                          hvx_intra_search_result *__restrict__ out) {
  using namespace intra;
  constexpr int N = 1 << LOG2N, NB = 4 * N + 1, T = N == 4 ? 4 : 8;
  __shared__ int16_t su[NB * 64], sf[NB * 64];
  const int lane = lane_id(), i = blockIdx.x * 64 + lane;
  const bool active = i < n_jobs;
  const hvx_intra_job j = jobs[active ? i : n_jobs - 1];
  const bool ok = active && job_ok(j) && j.ch_type == 0 && j.log2_size == LOG2N;
  if (__ballot(ok) == 0) return;  // no job of this size in the wave (a mixed batch)
  {  // the border (fillReferenceSamples, TComPattern.cpp:364-540) of this lane's PU, position by position
    const uint8_t *p = rec + (int64_t)j.y * stride + j.x;
    const int ulog2 = j.unit_log2, u = 1 << ulog2, nunits = ((4 * N) >> ulog2) + 1;
    uint32_t a[3];
    int navail = 0;
#pragma unroll
    for (int w = 0; w < 3; w++) {
      const int lo = w * 32;
      a[w] = nunits >= lo + 32 ? j.avail[w] : nunits > lo ? j.avail[w] & ((1u << (nunits - lo)) - 1u) : 0u;
      navail += __popc(a[w]);
    }
    for (int k = 0; k < NB; k++) {
      const int l = k == 0 ? 2 * N + u - 1 : k <= 2 * N ? 2 * N + u + k - 1 : 4 * N - k;
      int v = 128;
      if (navail && ok) {
        const int uu = l >> ulog2;
        if ((a[uu >> 5] >> (uu & 31)) & 1) v = line_raw(p, stride, N, u, l);
        else {
          const int jj = highest_below(a, uu);
          v = jj >= 0 ? line_raw(p, stride, N, u, jj * u + u - 1) : line_raw(p, stride, N, u, lowest_above(a, uu) * u);
        }
      }
      su[k * 64 + lane] = (int16_t)v;
    }
    for (int k = 0; k <= 4 * N; k++) {  // [1 2 1] smoothing (strong smoothing needs 32x32)
      const int fk = f_index(N, k);
      int v;
      if (k == 0 || k == 4 * N) v = su[fk * 64 + lane];
      else v = (su[f_index(N, k - 1) * 64 + lane] + 2 * su[fk * 64 + lane] + su[f_index(N, k + 1) * 64 + lane] + 2) >> 2;
      sf[fk * 64 + lane] = (int16_t)v;
    }
  }
  auto bu = [&](int k) { return (int)su[k * 64 + lane]; };
  int dcs = 0;
#pragma unroll
  for (int k = 0; k < N; k++) dcs += bu(1 + k) + bu(2 * N + 1 + k);
  const int dc = (dcs + N) >> (LOG2N + 1);
  __shared__ uint8_t so[N * N * 64];  // the original block, [sample][lane]
  {
    const uint8_t *po = org + (int64_t)j.y * stride + j.x;
    for (int y = 0; y < N; y++)
      for (int x = 0; x < N; x++) so[(y * N + x) * 64 + lane] = ok ? po[y * stride + x] : 0;
  }
  // MPMs (getIntraDirPredictor, TComDataCU.cpp:1441-1478) and the rate constants
  const int ld = j.left_dir, ad = j.above_dir;
  int mp0, mp1, mp2, imode;
  if (ld == ad) {
    imode = 1;
    if (ld > 1) { mp0 = ld; mp1 = ((ld + 29) % 32) + 2; mp2 = ((ld - 1) % 32) + 2; }
    else { mp0 = 0; mp1 = 1; mp2 = 26; }
  } else {
    imode = 2;
    mp0 = ld; mp1 = ad;
    mp2 = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  }
  const bool fast = (j.flags & HVX_INTRA_FAST_MPM) != 0;
  const int num = fast ? kNumRdMpm[LOG2N - 1] : kNumRdNoMpm[LOG2N - 1];  // 8 or 9
  const uint64_t frac = (uint64_t)(uint32_t)j.frac_bits;
  const int st = j.ctx_state & 127;
  const uint64_t eb_mpm = (uint64_t)(uint32_t)eb[st ^ 1], eb_no = (uint64_t)(uint32_t)eb[st];
  hvx_intra_search_result *r = out + (active ? i : 0);
  double cc[9];
  int cl[9];
#pragma unroll
  for (int k = 0; k < 9; k++) { cc[k] = 1.7976931348623157e308; cl[k] = 0; }
  for (int m = 0; m < 35; m++) {  // uniform across the wave
    const Mode md(m);
    const int16_t *bp = use_filter(m, LOG2N, true) ? sf : su;
    auto bb = [&](int k) { return (int)bp[k * 64 + lane]; };
    uint32_t sum = 0;
    int d[T][T];
#pragma unroll
    for (int y = 0; y < T; y++) {
      int row[T];
#pragma unroll
      for (int x = 0; x < T; x++) {
        const int pv = pred_sample_f(bb, N, LOG2N, md, true, dc, y, x);
        row[x] = (int)so[(y * N + x) * 64 + lane] - pv;
      }
      if constexpr (T == 8) hadamard8(row, d[y]);
      else hadamard4(row, d[y]);
    }
#pragma unroll
    for (int x = 0; x < T; x++) {
      int col[T], rr[T];
#pragma unroll
      for (int y = 0; y < T; y++) col[y] = d[y][x];
      if constexpr (T == 8) hadamard8(col, rr);
      else hadamard4(col, rr);
#pragma unroll
      for (int k = 0; k < T; k++) sum += (uint32_t)abs(rr[k]);
    }
    sum = T == 8 ? (sum + 2) >> 2 : (sum + 1) >> 1;  // xCalcHADs8x8 / xCalcHADs4x4
    const int idx = m == mp0 ? 0 : m == mp1 ? 1 : m == mp2 ? 2 : -1;
    const uint64_t total = frac + (idx >= 0 ? eb_mpm : eb_no) + 32768ull * (uint64_t)(idx < 0 ? 5 : idx ? 2 : 1);
    const uint32_t bits = (uint32_t)(total >> 15);
    const double cost = __dadd_rn((double)sum, __dmul_rn((double)bits, j.sqrt_lambda));
      if (ok) { r->satd[m] = sum; r->mode_bits[m] = (uint8_t)bits; }
    // xUpdateCandList (:5254) on the sorted `num` slots: the new entry goes after every entry it
    // does not beat (strict '<'), the last one drops out
    bool c[9];
#pragma unroll
    for (int k = 0; k < 9; k++) c[k] = k < num && cost < cc[k];
#pragma unroll
    for (int k = 8; k >= 0; k--)
      if (c[k]) {
        const bool from_prev = k > 0 && c[k - 1];
        cc[k] = from_prev ? cc[k - 1] : cost;
        cl[k] = from_prev ? cl[k - 1] : m;
      }
  }
  if (!ok) return;  // inactive lanes and jobs of other sizes (another launch serves them)
  r->num_rd = (uint8_t)num;
#pragma unroll
  for (int k = 0; k < 8; k++) r->cand_cost[k] = k < num ? cc[k] : 0.0;
#pragma unroll
  for (int k = 0; k < 9; k++) r->cand[k] = (uint8_t)(k < num ? cl[k] : 0);
  r->cand[9] = r->cand[10] = 0;
  int n2 = num;
  if (fast) {  // :2299-2321 (the MPMs are distinct, so an appended one never matches another)
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int mq = q == 0 ? mp0 : q == 1 ? mp1 : mp2;
      bool inc = q >= imode;
#pragma unroll
      for (int k = 0; k < 9; k++) inc |= k < num && mq == cl[k];
      if (!inc) r->cand[n2++] = (uint8_t)mq;
    }
  }
  r->n_cand = (uint8_t)n2;
#pragma unroll
  for (int k = 0; k < 4; k++) r->pad_[k] = 0;
}
