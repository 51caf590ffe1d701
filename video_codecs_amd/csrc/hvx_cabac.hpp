// hvx_cabac.hpp -- coefficient rate on the device (gfx950): TEncSbac::codeCoeffNxN
// (TEncSbac.cpp:1181-1540, with codeTransformSkipFlags :997, codeLastSignificantXY :1115 and
// xWriteCoefRemainExGolomb :337) as counted by TEncBinCABACCounter
// (TEncBinCoderCABACCounter.cpp:74-120): every context-coded bin adds
// ContextModel::m_entropyBits[state ^ bin] and advances that context's state
// (ContextModel.h:79-85), every bypass bin adds 32768.
//
// Mapping: one TU per LANE, 64 TUs per wave.  The count is a serial walk over the TU's
// reverse scan whose context states evolve bin by bin, so the parallelism is across TUs.
// Each lane keeps the 143 context states it can touch (models 42..184: significant-CG, sig,
// last X/Y, greater-1, greater-2, transform-skip) in its own LDS byte column
// (state r of lane l at [r*64 + l]: the 64 lanes of an access hit 16 consecutive dwords,
// conflict-free); the entropy table (128 int) and the state-transition table (256 bytes)
// are shared LDS.  The significant-CG map of a TU (<= 64 groups) is a 64-bit register mask.
// Levels are read through an accessor (raster int32 for the ABI batch, the CTU pass's
// interleaved scan-order arrays there), so no per-lane private arrays spill to scratch.
#pragma once
#include "hvx_dev.hpp"

namespace cab {
constexpr int kCtxLo = 42;          // first model the coefficient syntax uses (sig CG)
constexpr int kRows = 185 - kCtxLo; // ..184 (transform-skip chroma)
constexpr int kSigCG = 42 - kCtxLo, kSig = 46 - kCtxLo, kLastX = 90 - kCtxLo, kLastY = 120 - kCtxLo;
constexpr int kOne = 150 - kCtxLo, kAbs = 174 - kCtxLo, kTskip = 183 - kCtxLo;

__constant__ uint8_t kTransIdxLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                         13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                         24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                         33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

struct Shared {
  uint8_t st[kRows * 64];   // per-lane state columns
  uint8_t next[256];        // next[state*2 + bin]
  int32_t eb[128];          // ContextModel::m_entropyBits
};

// fill the shared tables (whole wave)
__device__ __forceinline__ void init_tables(Shared &s, const int32_t *entropy_bits) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 128; i += 64) {
    s.eb[i] = entropy_bits[i];
    const int p = i >> 1, mps = i & 1;
    s.next[i * 2 + mps] = (uint8_t)(((p < 62 ? p + 1 : p) << 1) | mps);                      // MPS
    s.next[i * 2 + (mps ^ 1)] = (uint8_t)((kTransIdxLps[p] << 1) | (p == 0 ? mps ^ 1 : mps)); // LPS
  }
}

struct Lane {
  uint8_t *col;  // &s.st[lane]
  const Shared *s;
  uint64_t frac;
  __device__ __forceinline__ void bin(int row, int v) {
    uint8_t &st = col[row * 64];
    const int q = st;
    frac += (uint32_t)s->eb[q ^ v];
    st = s->next[q * 2 + v];
  }
  __device__ __forceinline__ void ep(int n) { frac += 32768ull * (uint32_t)n; }
};

// xWriteCoefRemainExGolomb (:337): bypass bins of one escape code
__device__ __forceinline__ int remain_bins(uint32_t symbol, int r, bool limited, int max_log2) {
  if (symbol < (3u << r)) return (int)(symbol >> r) + 1 + r;
  if (limited) {
    const uint32_t maxp = 32 - (3 + max_log2);
    uint32_t prefix = 0, suffix_len;
    const uint32_t v = (symbol >> r) - 3;
    if (v >= ((1u << maxp) - 1)) {
      prefix = maxp;
      suffix_len = (uint32_t)(max_log2 - r);
    } else {
      while (v > ((2u << prefix) - 2)) prefix++;
      suffix_len = prefix + 1;
    }
    return (int)(prefix + 3 + suffix_len + r);
  }
  int len = r;
  uint32_t cn = symbol - (3u << r);
  while (cn >= (1u << len)) cn -= (1u << (len++));
  return 3 + len + 1 - r + len;
}

__device__ __forceinline__ int log2_tu(int n) { return n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : 5; }

// getSigCtxInc (TComTrQuant.cpp:2717), square TU of log2 size lw
__device__ __forceinline__ int sig_ctx(int pattern, int first_sig, int single, int raster, int lw, int ch) {
  if (first_sig == single) return single;
  const int py = raster >> lw, px = raster - (py << lw);
  if (px + py == 0) return 0;
  int offset;
  if (lw == 2) {
    offset = kCtxIndMap4x4[4 * py + px];
  } else {
    int cnt;
    if (pattern == 0) { const int t = (px & 3) + (py & 3); cnt = t >= 3 ? 0 : t >= 1 ? 1 : 2; }
    else if (pattern == 1) { const int y = py & 3; cnt = y >= 2 ? 0 : y >= 1 ? 1 : 2; }
    else if (pattern == 2) { const int x = px & 3; cnt = x >= 2 ? 0 : x >= 1 ? 1 : 2; }
    else cnt = 2;
    const int nf = ((px >> 2) + (py >> 2)) > 0;
    offset = (nf ? (ch ? 0 : 3) : 0) + cnt;
  }
  return first_sig + offset;
}

// codeCoeffNxN for one square TU.  lev(sp) returns the level at GROUPED SCAN position sp
// (scan = kScan[scan_type] at the TU's size).  Returns num_sig; frac accumulates in L.
// Coefficient groups are the unit of work: each group's 16 levels are fetched by 16
// independent loads into registers (fully unrolled, static indices), so a group costs one
// memory latency, and every later pass over the group reads registers.
template <class LevAt>
__device__ int coeff_bits(const hvx_tu_desc &d, LevAt lev, Lane &L, uint32_t &rice_stat) {
  const int n = d.width, lw = log2_tu(n), l = lw - 2, wg = n >> 2, ncg = wg * wg;
  const int ch = d.comp ? 1 : 0;
  const uint8_t *scan_cg = kScanCG[d.scan_type] + cg_base(l);
  const uint16_t *scan = kScan[d.scan_type] + scan_base(l);
  // significant-CG map (raster CG index), the last significant scan position, the count
  uint64_t cgm = 0;
  int num_sig = 0, scan_last = -1;
  for (int sub = 0; sub < ncg; sub++) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) m |= (uint32_t)(lev(sub * 16 + k) != 0) << k;
    if (m) {
      cgm |= 1ull << scan_cg[sub];
      num_sig += __popc(m);
      scan_last = sub * 16 + 31 - __clz(m);
    }
  }
  if (num_sig == 0) return 0;  // the reference exits here (empty TU); nothing is coded
  const bool be_valid = d.transquant_bypass ? false : (d.sign_hiding != 0);
  if (d.pps_tskip && !d.transquant_bypass && n <= 4) L.bin(kTskip + ch, d.transform_skip ? 1 : 0);
  // firstSignificanceMapContext (getTUEntropyCodingParameters, TComChromaFormat.cpp:96)
  const int single = ch ? 15 : 27;
  int first_sig;
  if (d.ts_context && (d.transquant_bypass || d.transform_skip)) first_sig = single;
  else if (n == 4) first_sig = 0;
  else if (n == 8) first_sig = 9 + ((d.scan_type != 0 && !ch) ? 6 : 0);
  else first_sig = ch ? 12 : 21;
  // codeLastSignificantXY (:1115)
  {
    const int r = scan[scan_last];
    int py = r >> lw, px = r - (py << lw);
    if (d.scan_type == 2) { const int t = px; px = py; py = t; }
    const int gx = kGroupIdx[px], gy = kGroupIdx[py], gmax = kGroupIdx[n - 1];
    const int cw = lw - 2;  // square: width and height contexts coincide
    const int off = ch ? 0 : cw * 3 + ((cw + 1) >> 2), sh = ch ? cw : (cw + 3) >> 2;
    const int bx = kLastX + ch * 15 + off, by = kLastY + ch * 15 + off;
    int k;
    for (k = 0; k < gx; k++) L.bin(bx + (k >> sh), 1);
    if (gx < gmax) L.bin(bx + (k >> sh), 0);
    for (k = 0; k < gy; k++) L.bin(by + (k >> sh), 1);
    if (gy < gmax) L.bin(by + (k >> sh), 0);
    if (gx > 3) L.ep((gx - 2) >> 1);
    if (gy > 3) L.ep((gy - 2) >> 1);
  }
  const int base_cg = kSigCG + ch * 2, base_sig = kSig + (ch ? 28 : 0);
  const int last_set = scan_last >> 4, last_pin = scan_last & 15;
  int c1 = 1;
  for (int sub = last_set; sub >= 0; sub--) {
    const int sub_pos = sub << 4;
    const int cg = scan_cg[sub], cgy = cg / wg, cgx = cg - cgy * wg;
    int a[16];
#pragma unroll
    for (int k = 0; k < 16; k++) a[k] = lev(sub_pos + k);
    if (sub == last_set || sub == 0) cgm |= 1ull << cg;
    else {
      const int rr = cgx < wg - 1 ? (int)((cgm >> (cg + 1)) & 1) : 0;
      const int bb = cgy < wg - 1 ? (int)((cgm >> (cg + wg)) & 1) : 0;
      L.bin(base_cg + ((rr + bb) != 0), (int)((cgm >> cg) & 1));
    }
    // significance flags (reverse scan inside the group); non-zero count, first/last positions
    const bool is_last_set = sub == last_set;
    int nnz = is_last_set ? 1 : 0, last_nz = is_last_set ? last_pin : -1, first_nz = is_last_set ? last_pin : 16;
    if ((cgm >> cg) & 1) {
      int pattern = 0;
      if (wg > 1) {
        const int rr = cgx < wg - 1 ? (int)((cgm >> (cg + 1)) & 1) : 0;
        const int bb = cgy < wg - 1 ? (int)((cgm >> (cg + wg)) & 1) : 0;
        pattern = rr + (bb << 1);
      }
#pragma unroll
      for (int pin = 15; pin >= 0; pin--) {
        if (is_last_set && pin >= last_pin) continue;
        const int sig = a[pin] != 0;
        if (pin > 0 || sub == 0 || nnz) L.bin(base_sig + sig_ctx(pattern, first_sig, single, scan[sub_pos + pin], lw, ch), sig);
        if (sig) {
          nnz++;
          if (last_nz == -1) last_nz = pin;
          first_nz = pin;
        }
      }
    }
    if (nnz == 0) continue;
    // greater-1 / greater-2 flags over the group's non-zero levels in reverse scan order
    const bool hidden = (last_nz - first_nz) >= 4;  // SBH_THRESHOLD
    const int set = (ch ? 4 : 0) + ((!ch && sub > 0) ? 2 : 0) + (c1 == 0 ? 1 : 0);
    c1 = 1;
    const int base_one = kOne + 4 * set;
    bool escape = nnz > 8;
    int idx = 0, first_c2_abs = 0;
    bool have_c2 = false;
#pragma unroll
    for (int pin = 15; pin >= 0; pin--) {
      const int av = abs(a[pin]);
      if (!av || idx >= 8) continue;
      const int gt1 = av > 1;
      L.bin(base_one + c1, gt1);
      if (gt1) {
        c1 = 0;
        if (!have_c2) { have_c2 = true; first_c2_abs = av; }
        else escape = true;
      } else if (c1 < 3 && c1 > 0) {
        c1++;
      }
      idx++;
    }
    if (c1 == 0 && have_c2) {
      const int gt2 = first_c2_abs > 2;
      L.bin(kAbs + set, gt2);
      if (gt2) escape = true;
    }
    L.ep((be_valid && hidden) ? nnz - 1 : nnz);
    if (escape) {
      int rice = (int)(rice_stat / 4);
      bool upd = d.persistent_rice != 0;
      int first2 = 1;
      idx = 0;
#pragma unroll
      for (int pin = 15; pin >= 0; pin--) {
        const int av = abs(a[pin]);
        if (!av) continue;
        const int base = idx < 8 ? 2 + first2 : 1;
        if (av >= base) {
          const uint32_t esc = (uint32_t)(av - base);
          L.ep(remain_bins(esc, rice, d.extended_precision != 0, d.max_log2_tr_range));
          if (av > (3 << rice)) rice = d.persistent_rice ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
          if (upd) {
            const uint32_t init = rice_stat / 4;
            if (esc >= (3u << init)) rice_stat++;
            else if (esc * 2 < (1u << init) && rice_stat > 0) rice_stat--;
            upd = false;
          }
        }
        if (av >= 2) first2 = 0;
        idx++;
      }
    }
  }
  return num_sig;
}

// copy the lanes' states between global (`stride` bytes per TU; stride 0 = one snapshot shared
// by every TU) and the LDS columns, coalesced across the wave; tu0 = first TU of the wave,
// cnt = TUs in the wave
__device__ __forceinline__ void states_load(Shared &s, const uint8_t *g, size_t stride, int tu0, int cnt) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < cnt * kRows; i += 64) {
    const int t = i / kRows, r = i - t * kRows;
    s.st[r * 64 + t] = g[(size_t)(tu0 + t) * stride + kCtxLo + r];
  }
}
__device__ __forceinline__ void states_store(const Shared &s, uint8_t *g, int tu0, int cnt) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < cnt * kRows; i += 64) {
    const int t = i / kRows, r = i - t * kRows;
    g[(size_t)(tu0 + t) * HVX_NUM_CTX + kCtxLo + r] = s.st[r * 64 + t];
  }
}
}  // namespace cab

// hvx_coeff_bits_batch: TU i = lane (i % 64) of block i / 64; raster int32 levels at d_off[i].
// states_stride HVX_NUM_CTX: per-TU states, advanced in place; 0: one shared snapshot (read only:
// the CTU decision counts every TU from the same state)
__global__ __launch_bounds__(64) void k_coeff_bits(const hvx_tu_desc *__restrict__ descs, const int64_t *__restrict__ offs,
                                                   int n, const int32_t *__restrict__ levels,
                                                   const int32_t *__restrict__ entropy_bits, uint8_t *__restrict__ states,
                                                   int states_stride, hvx_coeff_bits *__restrict__ out) {
  __shared__ cab::Shared s;
  const int lane = threadIdx.x, tu0 = blockIdx.x * 64, cnt = min(64, n - tu0), t = tu0 + lane;
  cab::init_tables(s, entropy_bits);
  cab::states_load(s, states, (size_t)states_stride, tu0, cnt);
  __syncthreads();
  if (lane < cnt) {
    const hvx_tu_desc d = descs[t];
    hvx_coeff_bits r{0, (uint32_t)d.golomb_rice_stat, 0xffffffffu};  // num_sig ~0: unsupported geometry
    if ((d.width == 4 || d.width == 8 || d.width == 16 || d.width == 32) && d.height == d.width &&
        (unsigned)d.scan_type <= 2u) {
      const int32_t *lv = levels + offs[t];
      const uint16_t *scan = kScan[d.scan_type] + scan_base(cab::log2_tu(d.width) - 2);
      cab::Lane L{&s.st[lane], &s, 0};
      uint32_t rice = (uint32_t)d.golomb_rice_stat;
      const int ns = cab::coeff_bits(d, [&](int sp) { return lv[scan[sp]]; }, L, rice);
      r.frac_bits = L.frac;
      r.rice_stat = rice;
      r.num_sig = (uint32_t)ns;
    }
    out[t] = r;
  }
  if (states_stride) {
    __syncthreads();
    cab::states_store(s, states, tu0, cnt);
  }
}

// The CTU decision's variant (hvx_ctu_decide): one size class of the CTU pass, levels read from
// the RDOQ's interleaved scan-order array (G = 64 TUs per group: lane l of block b counts TU
// b*64 + l, whose element sp sits at ((b*NN + sp)*64 + l) -- the 64 lanes of every level load
// touch 64 consecutive words), every TU from the same snapshot.
template <int L>
__global__ __launch_bounds__(64) void k_coeff_bits_il(const hvx_tu_desc *__restrict__ descs, int n,
                                                      const int32_t *__restrict__ levI,
                                                      const int32_t *__restrict__ entropy_bits,
                                                      const uint8_t *__restrict__ snapshot,
                                                      hvx_coeff_bits *__restrict__ out) {
  constexpr int N = 4 << L, NN = N * N;
  __shared__ cab::Shared s;
  const int lane = threadIdx.x, tu0 = blockIdx.x * 64, cnt = min(64, n - tu0), t = tu0 + lane;
  cab::init_tables(s, entropy_bits);
  cab::states_load(s, snapshot, 0, tu0, cnt);
  __syncthreads();
  if (lane >= cnt) return;
  const hvx_tu_desc d = descs[t];
  hvx_coeff_bits r{0, (uint32_t)d.golomb_rice_stat, 0xffffffffu};
  if (d.width == N && d.height == N && (unsigned)d.scan_type <= 2u) {
    const int32_t *lv = levI + tu_il(t, 0, NN, 64);
    cab::Lane Lc{&s.st[lane], &s, 0};
    uint32_t rice = (uint32_t)d.golomb_rice_stat;
    const int ns = cab::coeff_bits(d, [&](int sp) { return lv[(size_t)sp * 64]; }, Lc, rice);
    r.frac_bits = Lc.frac;
    r.rice_stat = rice;
    r.num_sig = (uint32_t)ns;
  }
  out[t] = r;
}
