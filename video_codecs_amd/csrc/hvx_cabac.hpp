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

static __constant__ uint8_t kTransIdxLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                         13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                         24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                         33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

static __constant__ uint8_t kMinInGroup[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};  // g_uiMinInGroup (TComRom.cpp)

struct Shared {
  uint8_t st[kRows * 64];   // per-lane state columns
  uint8_t next[256];        // next[state*2 + bin]
  int32_t eb[128];          // ContextModel::m_entropyBits
};

// fill the shared tables (whole wave)
__device__ __forceinline__ void init_tables(Shared &s, const int32_t *entropy_bits) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < 128; i += 64) {
    s.eb[i] = entropy_bits ? entropy_bits[i] : 0;  // the writer has no rate table
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
  // the bypass forms the writer needs values for; the counter only counts them
  __device__ __forceinline__ void ep_bits(uint32_t, int n) { ep(n); }
  __device__ __forceinline__ void eps(uint32_t, int n) { ep(n); }
  __device__ __forceinline__ void esc(uint32_t symbol, int r, bool limited, int max_log2);
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
  // the reference's loop `while (cn >= (1 << len)) cn -= 1 << len++` from len = r runs
  // floor(log2(((symbol - (3 << r)) >> r) + 1)) times (the closed form of rd_ic_rate, hvx_tu.hpp)
  const uint32_t v = ((symbol - (3u << r)) >> r) + 1;
  const int len = r + (31 - __clz(v));
  return 3 + len + 1 - r + len;
}

__device__ __forceinline__ void Lane::esc(uint32_t symbol, int r, bool limited, int max_log2) {
  ep(remain_bins(symbol, r, limited, max_log2));
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

// firstSignificanceMapContext (getTUEntropyCodingParameters, TComChromaFormat.cpp:96)
__device__ __forceinline__ int first_sig_ctx(const hvx_tu_desc &d, int n, int ch) {
  const int single = ch ? 15 : 27;
  if (d.ts_context && (d.transquant_bypass || d.transform_skip)) return single;
  if (n == 4) return 0;
  if (n == 8) return 9 + ((d.scan_type != 0 && !ch) ? 6 : 0);
  return ch ? 12 : 21;
}

// The scan geometry coeff_bits reads, from the constant tables: the CG scan (scan_cg[sub]),
// the grouped scan (raster of scan position sp) and the significance context of a position
// under a neighbour-CG pattern.  The HM engine substitutes a view of the same values staged in
// LDS (hvx_hm.hpp code_coeff_nxn), so its serial syntax walk issues no global-memory loads.
struct ScanTables {
  const uint8_t *scan_cg;
  const uint16_t *scan;
  int lw, ch, first_sig, single;
  __device__ __forceinline__ ScanTables(const hvx_tu_desc &d) {
    const int n = d.width, l = log2_tu(n) - 2;
    lw = l + 2;
    ch = d.comp ? 1 : 0;
    scan_cg = kScanCG[d.scan_type] + cg_base(l);
    scan = kScan[d.scan_type] + scan_base(l);
    first_sig = first_sig_ctx(d, n, ch);
    single = ch ? 15 : 27;
  }
  __device__ __forceinline__ int cg(int sub) const { return scan_cg[sub]; }
  __device__ __forceinline__ int raster(int sp) const { return scan[sp]; }
  __device__ __forceinline__ int sigc(int pattern, int sp) const;
};

template <class LevAt, class C, class Env>
__device__ __forceinline__ int coeff_bits_env(const hvx_tu_desc &d, const Env &env, LevAt lev, C &L, uint32_t &rice_stat);

__device__ __forceinline__ int ScanTables::sigc(int pattern, int sp) const {
  return sig_ctx(pattern, first_sig, single, scan[sp], lw, ch);
}

// codeCoeffNxN for one square TU.  lev(sp) returns the level at GROUPED SCAN position sp
// (scan = kScan[scan_type] at the TU's size).  Returns num_sig; frac accumulates in L.
template <class LevAt, class C>
__device__ __forceinline__ int coeff_bits(const hvx_tu_desc &d, LevAt lev, C &L, uint32_t &rice_stat) {
  return coeff_bits_env(d, ScanTables(d), lev, L, rice_stat);
}

// Coefficient groups are the unit of work: each group's 16 levels are fetched by 16
// independent loads into registers (fully unrolled, static indices), so a group costs one
// memory latency, and every later pass over the group reads registers.
template <class LevAt, class C, class Env>
__device__ __forceinline__ int coeff_bits_env(const hvx_tu_desc &d, const Env &env, LevAt lev, C &L, uint32_t &rice_stat) {
  const int n = d.width, lw = log2_tu(n), wg = n >> 2, ncg = wg * wg;
  const int ch = d.comp ? 1 : 0;
  // significant-CG map (raster CG index), the last significant scan position, the count
  uint64_t cgm = 0;
  int num_sig = 0, scan_last = -1;
  for (int sub = 0; sub < ncg; sub++) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) m |= (uint32_t)(lev(sub * 16 + k) != 0) << k;
    if (m) {
      cgm |= 1ull << env.cg(sub);
      num_sig += __popc(m);
      scan_last = sub * 16 + 31 - __clz(m);
    }
  }
  if (num_sig == 0) return 0;  // the reference exits here (empty TU); nothing is coded
  const bool be_valid = d.transquant_bypass ? false : (d.sign_hiding != 0);
  if (d.pps_tskip && !d.transquant_bypass && n <= 4) L.bin(kTskip + ch, d.transform_skip ? 1 : 0);
  // codeLastSignificantXY (:1115)
  {
    const int r = env.raster(scan_last);
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
    // the fixed-length suffixes: one encodeBinEP per bit, most significant first
    if (gx > 3) L.ep_bits((uint32_t)(px - kMinInGroup[gx]), (gx - 2) >> 1);
    if (gy > 3) L.ep_bits((uint32_t)(py - kMinInGroup[gy]), (gy - 2) >> 1);
  }
  const int base_cg = kSigCG + ch * 2, base_sig = kSig + (ch ? 28 : 0);
  const int last_set = scan_last >> 4, last_pin = scan_last & 15;
  int c1 = 1;
  for (int sub = last_set; sub >= 0; sub--) {
    const int sub_pos = sub << 4;
    const int cg = env.cg(sub), cgy = cg / wg, cgx = cg - cgy * wg;
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
    uint32_t signs = 0;  // coeffSigns, in coding order (the last position's sign first)
#pragma unroll
    for (int pin = 0; pin < 16; pin++)
      if (is_last_set && pin == last_pin) signs = (uint32_t)(a[pin] < 0);  // static indices: no scratch
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
        if (pin > 0 || sub == 0 || nnz) L.bin(base_sig + env.sigc(pattern, sub_pos + pin), sig);
        if (sig) {
          nnz++;
          signs = 2 * signs + (uint32_t)(a[pin] < 0);
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
    if (be_valid && hidden) L.eps(signs >> 1, nnz - 1);  // the first coefficient's sign is hidden
    else L.eps(signs, nnz);
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
          L.esc(esc, rice, d.extended_precision != 0, d.max_log2_tr_range);
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

// ---------------------------------------------------------------------------------------------
// The slice writer's arithmetic coder, TEncBinCABAC (TEncBinCoderCABAC.cpp:60-460), as a second
// bin sink for coeff_bits: the same context evolution as the counter, the bins driving the
// lane's registers, completed bytes appended to the lane's output run.  rangeTabLps
// (TComCABACTables.cpp:44, the specification's Table 9-52) is staged in LDS; renormalisation
// shifts are the reference's table (:113).
// ---------------------------------------------------------------------------------------------
static __constant__ uint8_t kLpsTable[64 * 4] = {
    128, 176, 208, 240, 128, 167, 197, 227, 128, 158, 187, 216, 123, 150, 178, 205, 116, 142, 169, 195,
    111, 135, 160, 185, 105, 128, 152, 175, 100, 122, 144, 166, 95,  116, 137, 158, 90,  110, 130, 150,
    85,  104, 123, 142, 81,  99,  117, 135, 77,  94,  111, 128, 73,  89,  105, 122, 69,  85,  100, 116,
    66,  80,  95,  110, 62,  76,  90,  104, 59,  72,  86,  99,  56,  69,  81,  94,  53,  65,  77,  89,
    51,  62,  73,  85,  48,  59,  69,  80,  46,  56,  66,  76,  43,  53,  63,  72,  41,  50,  59,  69,
    39,  48,  56,  65,  37,  45,  54,  62,  35,  43,  51,  59,  33,  41,  48,  56,  32,  39,  46,  53,
    30,  37,  43,  50,  29,  35,  41,  48,  27,  33,  39,  45,  26,  31,  37,  43,  24,  30,  35,  41,
    23,  28,  33,  39,  22,  27,  32,  37,  21,  26,  30,  35,  20,  24,  29,  33,  19,  23,  27,  31,
    18,  22,  26,  30,  17,  21,  25,  28,  16,  20,  23,  27,  15,  19,  22,  25,  14,  18,  21,  24,
    14,  17,  20,  23,  13,  16,  19,  22,  12,  15,  18,  21,  12,  14,  17,  20,  11,  14,  16,  19,
    11,  13,  15,  18,  10,  12,  15,  17,  10,  12,  14,  16,  9,   11,  13,  15,  9,   11,  12,  14,
    8,   10,  12,  14,  8,   9,   11,  13,  7,   9,   11,  12,  7,   9,   10,  12,  7,   8,   10,  11,
    6,   8,   9,   11,  6,   7,   9,   10,  6,   7,   8,   9,   2,   2,   2,   2};
static __constant__ uint8_t kRenormTable[32] = {6, 5, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

struct Writer {
  uint8_t *col;          // &s.st[lane]
  const Shared *s;
  const uint8_t *lps;    // LDS copy of kLpsTable
  uint32_t low, range;   // m_uiLow, m_uiRange
  int bits_left, nbuf;   // m_bitsLeft, m_numBufferedBytes
  uint32_t buffered;     // m_bufferedByte
  uint8_t *out;
  int nout, cap;
  uint32_t bins;         // bins coded (m_uiBinsCoded with m_binCountIncrement 1)
  uint64_t cd0, cd1;     // contexts coded (setBinsCoded(1)): rows 0..63, 64..127
  uint32_t cd2;          //   rows 128..142
  __device__ __forceinline__ void put(uint32_t b) {
    if (nout < cap) out[nout] = (uint8_t)b;
    nout++;
  }
  // writeOut (:425): the lead byte; 0xff bytes are held back until a carry can no longer reach them
  __device__ __forceinline__ void write_out() {
    const uint32_t lead = low >> (24 - bits_left);
    bits_left += 8;
    low &= 0xffffffffu >> bits_left;
    if (lead == 0xff) {
      nbuf++;
    } else if (nbuf > 0) {
      const uint32_t carry = lead >> 8;
      put(buffered + carry);
      buffered = lead & 0xff;
      const uint32_t fill = (0xff + carry) & 0xff;
      for (; nbuf > 1; nbuf--) put(fill);
    } else {
      nbuf = 1;
      buffered = lead;
    }
  }
  __device__ __forceinline__ void test() {
    if (bits_left < 12) write_out();
  }
  // encodeBin (:200) + ContextModel::update
  __device__ __forceinline__ void bin(int row, int v) {
    bins++;
    if (row < 64) cd0 |= 1ull << row;
    else if (row < 128) cd1 |= 1ull << (row - 64);
    else cd2 |= 1u << (row - 128);
    uint8_t &st = col[row * 64];
    const int q = st, mps = q & 1;
    const uint32_t l = lps[(q >> 1) * 4 + ((range >> 6) & 3)];
    range -= l;
    if (v != mps) {
      const int nb = kRenormTable[l >> 3];
      low = (low + range) << nb;
      range = l << nb;
      bits_left -= nb;
      test();
    } else if (range < 256) {
      low <<= 1;
      range <<= 1;
      bits_left--;
      test();
    }
    st = s->next[q * 2 + v];
  }
  // encodeAlignedBinsEP (:334): reached only with range == 256 (cabac_bypass_alignment)
  __device__ __forceinline__ void aligned(uint32_t vals, int n) {
    while (n > 0) {
      const int k = n < 8 ? n : 8;
      low = (low << k) + (((vals >> (n - k)) & ((1u << k) - 1)) << 8);
      n -= k;
      bits_left -= k;
      test();
    }
  }
  // encodeBinEP (:262)
  __device__ __forceinline__ void ep1(uint32_t b) {
    bins++;
    if (range == 256) { aligned(b, 1); return; }
    low <<= 1;
    if (b) low += range;
    bits_left--;
    test();
  }
  // codeLastSignificantXY's suffix (TEncSbac.cpp:1163-1180): one encodeBinEP per bit, msb first
  __device__ __forceinline__ void ep_bits(uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) ep1((v >> i) & 1u);
  }
  // encodeBinsEP (:290): most significant first, in pieces of 8
  __device__ __forceinline__ void eps(uint32_t vals, int n) {
    bins += (uint32_t)n;
    if (range == 256) { aligned(vals, n); return; }
    while (n > 8) {
      n -= 8;
      const uint32_t pat = vals >> n;
      low = (low << 8) + range * pat;
      vals -= pat << n;
      bits_left -= 8;
      test();
    }
    low = (low << n) + range * vals;
    bits_left -= n;
    test();
  }
  // xWriteCoefRemainExGolomb (TEncSbac.cpp:337), COEF_REMAIN_BIN_REDUCTION 3
  __device__ __forceinline__ void esc(uint32_t symbol, int r, bool limited, int max_log2) {
    if (symbol < (3u << r)) {
      const uint32_t len = symbol >> r;
      eps((1u << (len + 1)) - 2, (int)len + 1);
      eps(symbol & ((1u << r) - 1), r);
    } else if (limited) {
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
      const uint32_t suffix = v - ((1u << prefix) - 1), tot = prefix + 3;
      eps((1u << tot) - 1, (int)tot);
      eps((suffix << r) | (symbol & ((1u << r) - 1)), (int)(suffix_len + r));
    } else {
      int len = r;
      uint32_t cn = symbol - (3u << r);
      while (cn >= (1u << len)) cn -= (1u << (len++));
      eps((1u << (3 + len + 1 - r)) - 2, 3 + len + 1 - r);
      eps(cn, len);
    }
  }
};

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
static __global__ __launch_bounds__(64) void k_coeff_bits(const hvx_tu_desc *__restrict__ descs, const int64_t *__restrict__ offs,
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

// Runs per wave: the runs of a wave take different branches bin by bin (MPS / LPS, bypass lengths,
// renormalisation, writeOut), and the wave executes the union; fewer runs per wave spread the
// runs over more SIMDs, each wave still alone on its SIMD for a picture's worth of runs.
constexpr int kWriteRuns = 16;

// hvx_coeff_write_batch: stream k = lane (k % kWriteRuns) of block k / kWriteRuns writes TUs
// [stream_first[k], stream_first[k + 1]) through one TEncBinCABAC, from its own context states
// (states + k * HVX_NUM_CTX, advanced in place) and registers (regs[k], advanced in place); the
// completed bytes go to out + out_off[k] (at most out_cap), their count to out_len[k] (-1: past
// out_cap, -2: a TU geometry the coder does not take).  Raster int32 levels at levels + offs[t].
static __global__ __launch_bounds__(64) void k_coeff_write(const hvx_tu_desc *__restrict__ descs, const int64_t *__restrict__ offs,
                                                    const int32_t *__restrict__ levels,
                                                    const int32_t *__restrict__ stream_first, int n_streams,
                                                    uint8_t *__restrict__ states, hvx_cabac_regs *__restrict__ regs,
                                                    uint8_t *__restrict__ out, const int64_t *__restrict__ out_off,
                                                    int out_cap, int32_t *__restrict__ out_len) {
  __shared__ cab::Shared s;
  __shared__ uint8_t lps[256];
  const int lane = threadIdx.x, k0 = blockIdx.x * kWriteRuns, cnt = min(kWriteRuns, n_streams - k0), k = k0 + lane;
  cab::init_tables(s, nullptr);
  for (int i = lane; i < 256; i += 64) lps[i] = cab::kLpsTable[i];
  cab::states_load(s, states, (size_t)HVX_NUM_CTX, k0, cnt);
  __syncthreads();
  if (lane < cnt) {
    // every descriptor of the run is validated before anything is coded, so a run refused with
    // -2 leaves its registers and states untouched (the caller can fall back from a consistent
    // point).  Unsupported: non-square or non-4..32 TUs, scan types > 2, and persistent Rice
    // adaptation (its statistic would have to carry across the TUs of a run).
    bool ok = true;
    for (int t = stream_first[k]; t < stream_first[k + 1]; t++) {
      const hvx_tu_desc &d = descs[t];
      ok = ok && (d.width == 4 || d.width == 8 || d.width == 16 || d.width == 32) && d.height == d.width &&
           (unsigned)d.scan_type <= 2u && d.persistent_rice == 0;
    }
    const hvx_cabac_regs r0 = regs[k];
    cab::Writer W{&s.st[lane], &s, lps, r0.low, r0.range, r0.bits_left, r0.num_buffered, r0.buffered_byte,
                  out + out_off[k], 0, out_cap, r0.bins,
                  (uint64_t)r0.coded[0] | ((uint64_t)r0.coded[1] << 32), (uint64_t)r0.coded[2] | ((uint64_t)r0.coded[3] << 32),
                  r0.coded[4]};
    for (int t = stream_first[k]; t < stream_first[k + 1] && ok; t++) {
      const hvx_tu_desc d = descs[t];
      const int32_t *lv = levels + offs[t];
      const uint16_t *scan = kScan[d.scan_type] + scan_base(cab::log2_tu(d.width) - 2);
      uint32_t rice = (uint32_t)d.golomb_rice_stat;
      cab::coeff_bits(d, [&](int sp) { return lv[scan[sp]]; }, W, rice);
    }
    if (ok) {
      hvx_cabac_regs r1;
      r1.low = W.low; r1.range = W.range; r1.bits_left = W.bits_left; r1.num_buffered = W.nbuf;
      r1.buffered_byte = W.buffered; r1.bins = W.bins;
      r1.coded[0] = (uint32_t)W.cd0; r1.coded[1] = (uint32_t)(W.cd0 >> 32);
      r1.coded[2] = (uint32_t)W.cd1; r1.coded[3] = (uint32_t)(W.cd1 >> 32); r1.coded[4] = W.cd2;
      regs[k] = r1;
    }
    out_len[k] = !ok ? -2 : W.nout <= out_cap ? W.nout : -1;
  }
  __syncthreads();
  cab::states_store(s, states, k0, cnt);
}
