/* hvx_oracle.c -- CPU restatement of the HM-16.5rc1 CU mode-decision kernels.
 *
 * TEST INFRASTRUCTURE ONLY (see hvx_oracle.h).  Plain C, scalar, written from
 * the reference's behaviour; every function cites the reference file:line it
 * restates (paths relative to /root/reference/hm-16.5rc1/source/Lib unless noted).
 * Floating point follows the reference's operation order exactly; build with
 * -ffp-contract=off (x86-64 SSE2 semantics, as the reference was compiled).
 * Parity is pinned by tests/test_oracle_golden.py against tests/golden/.
 */
#include "hvx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ============================================================================================
 * Tables.  Values are HEVC-specification constants (the reference stores the same numbers in
 * TComRom.cpp:354-362, 489-515, 598 and TComTrQuant.cpp ctxIndMap4x4); generated or listed here.
 * ========================================================================================== */
static const int kQuantScales[6] = {26214, 23302, 20560, 18396, 16384, 14564};
static const int kInvQuantScales[6] = {40, 45, 51, 57, 64, 72};
static const int kGroupIdx[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                  8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
static const int kCtxIndMap4x4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
static const int kDst4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
/* |cos| samples of the 32-point HEVC core transform: c[j] ~ 64*sqrt(2)*cos(pi*j/64) */
static const int kCos[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                             61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
static const int kLumaFilter[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                      {-1, 4, -10, 58, 17, -5, 1, 0},
                                      {-1, 4, -11, 40, 40, -11, 4, -1},
                                      {0, 1, -5, 17, 58, -10, 4, -1}};
static const int kChromaFilter[8][4] = {{0, 64, 0, 0},   {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                        {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

/* T32[k][n] = sign * kCos[fold(k*(2n+1) mod 128)]; smaller sizes are row subsets (T_N[k] = T32[k*32/N]). */
static int dct32(int k, int n) {
  if (k == 0) return 64;
  int j = (k * (2 * n + 1)) % 128;
  int sign = 1;
  if (j > 64) j = 128 - j;           /* cos(2pi - a) = cos(a) */
  if (j > 32) { j = 64 - j; sign = -1; } /* cos(pi - a) = -cos(a) */
  return sign * kCos[j];
}

void hvxo_dct_matrix(int n, int16_t *m) {
  for (int k = 0; k < n; k++)
    for (int x = 0; x < n; x++) m[k * n + x] = (int16_t)dct32(k * (32 / n), x);
}

static int16_t g_mat[4][32 * 32];
static int g_tables_ready = 0;
/* scans: [grouped][type][log2w][log2h] (TComRom.cpp:192-262 generation rules; diag = up-right) */
static uint32_t *g_scan[2][3][6][6];

static void gen_scan(uint32_t *out, int w, int h, int stride, int type, int offx, int offy) {
  int i = 0;
  if (type == 0) {
    for (int d = 0; d < w + h - 1; d++) {
      int y = d < h - 1 ? d : h - 1;
      int x = d - y;
      while (y >= 0 && x < w) out[i++] = (uint32_t)((y + offy) * stride + x + offx), y--, x++;
    }
  } else if (type == 1) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) out[i++] = (uint32_t)((y + offy) * stride + x + offx);
  } else {
    for (int x = 0; x < w; x++)
      for (int y = 0; y < h; y++) out[i++] = (uint32_t)((y + offy) * stride + x + offx);
  }
}

static void init_tables(void) {
  if (g_tables_ready) return;
  for (int l = 0; l < 4; l++) hvxo_dct_matrix(4 << l, g_mat[l]);
  for (int lw = 0; lw < 6; lw++)
    for (int lh = 0; lh < 6; lh++)
      for (int t = 0; t < 3; t++) {
        int w = 1 << lw, h = 1 << lh;
        g_scan[0][t][lw][lh] = (uint32_t *)malloc(sizeof(uint32_t) * w * h);
        gen_scan(g_scan[0][t][lw][lh], w, h, w, t, 0, 0);
        g_scan[1][t][lw][lh] = (uint32_t *)malloc(sizeof(uint32_t) * w * h);
        if (lw >= 2 && lh >= 2) {
          int gw = w >> 2, gh = h >> 2;
          uint32_t cg[256];
          gen_scan(cg, gw, gh, gw, t, 0, 0);
          for (int g = 0; g < gw * gh; g++) {
            int gx = cg[g] % gw, gy = cg[g] / gw;
            gen_scan(g_scan[1][t][lw][lh] + g * 16, 4, 4, w, t, gx * 4, gy * 4);
          }
        } else {
          gen_scan(g_scan[1][t][lw][lh], w, h, w, t, 0, 0);
        }
      }
  g_tables_ready = 1;
}
/* the lazily built scan tables, once, before threads share the oracle */
void hvxo_init_tables(void) { init_tables(); }

const uint32_t *hvxo_scan(int grouped, int scan_type, int log2w, int log2h) {
  init_tables();
  return g_scan[grouped ? 1 : 0][scan_type][log2w][log2h];
}

/* ============================================================================================
 * Distortion: TComRdCost.cpp
 * ========================================================================================== */
/* xGetSAD4..64/12/24/48/16N (:489-950): every 2^s-th row, result << s.  xGetSAD (:461) = s 0. */
uint32_t hvxo_sad(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, int sub_shift) {
  uint32_t sum = 0;
  int step = 1 << sub_shift;
  for (int y = 0; y < h; y += step)
    for (int x = 0; x < w; x++) sum += (uint32_t)abs(org[y * so + x] - cur[y * sc + x]);
  return sum << sub_shift;
}

/* ME dispatch (setDistParam(pattern) :306-335): widths 4/8/16/32/64/12/24/48 honour the row
 * subsampling; any other width goes to the generic xGetSAD, which ignores it. */
uint32_t hvxo_sad_me(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, int sub_shift) {
  int specialised = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  return hvxo_sad(org, so, cur, sc, w, h, specialised ? sub_shift : 0);
}

/* xCalcHADs2x2 (:1310) */
static uint32_t had2(const int16_t *o, int so, const int16_t *c, int sc) {
  int d0 = o[0] - c[0], d1 = o[1] - c[1], d2 = o[so] - c[sc], d3 = o[so + 1] - c[sc + 1];
  int m0 = d0 + d2, m1 = d1 + d3, m2 = d0 - d2, m3 = d1 - d3;
  return (uint32_t)(abs(m0 + m1) + abs(m0 - m1) + abs(m2 + m3) + abs(m2 - m3));
}

/* 1-D 4-point Hadamard in the reference's butterfly order */
static void hadamard4(const int *in, int *out) {
  int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[0] - in[2], a3 = in[1] - in[3];
  out[0] = a0 + a1; out[1] = a0 - a1; out[2] = a2 + a3; out[3] = a2 - a3;
}

/* xCalcHADs4x4 (:1332): 2-D Hadamard of the 4x4 difference, (sum|.|+1)>>1.  The absolute sum
 * of a full 2-D Hadamard is independent of the row/column order of the butterflies. */
static uint32_t had4(const int16_t *o, int so, const int16_t *c, int sc) {
  int d[4][4], t[4][4];
  for (int y = 0; y < 4; y++)
    for (int x = 0; x < 4; x++) d[y][x] = o[y * so + x] - c[y * sc + x];
  for (int y = 0; y < 4; y++) hadamard4(d[y], t[y]);
  uint32_t s = 0;
  for (int x = 0; x < 4; x++) {
    int col[4] = {t[0][x], t[1][x], t[2][x], t[3][x]}, r[4];
    hadamard4(col, r);
    for (int k = 0; k < 4; k++) s += (uint32_t)abs(r[k]);
  }
  return (s + 1) >> 1;
}

static void hadamard8(const int *in, int *out) {
  int a[8], b[8];
  for (int i = 0; i < 4; i++) { a[i] = in[i] + in[i + 4]; a[i + 4] = in[i] - in[i + 4]; }
  b[0] = a[0] + a[2]; b[1] = a[1] + a[3]; b[2] = a[0] - a[2]; b[3] = a[1] - a[3];
  b[4] = a[4] + a[6]; b[5] = a[5] + a[7]; b[6] = a[4] - a[6]; b[7] = a[5] - a[7];
  for (int i = 0; i < 4; i++) { out[2 * i] = b[2 * i] + b[2 * i + 1]; out[2 * i + 1] = b[2 * i] - b[2 * i + 1]; }
}

/* xCalcHADs8x8 (:1428): (sum|.|+2)>>2 */
static uint32_t had8(const int16_t *o, int so, const int16_t *c, int sc) {
  int d[8][8], t[8][8];
  for (int y = 0; y < 8; y++)
    for (int x = 0; x < 8; x++) d[y][x] = o[y * so + x] - c[y * sc + x];
  for (int y = 0; y < 8; y++) hadamard8(d[y], t[y]);
  uint32_t s = 0;
  for (int x = 0; x < 8; x++) {
    int col[8], r[8];
    for (int y = 0; y < 8; y++) col[y] = t[y][x];
    hadamard8(col, r);
    for (int k = 0; k < 8; k++) s += (uint32_t)abs(r[k]);
  }
  return (s + 2) >> 2;
}

/* xGetHADs (:1526): tile by 8x8 if both dims % 8 == 0, else 4x4, else 2x2 */
uint32_t hvxo_satd(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h) {
  uint32_t sum = 0;
  int t = (w % 8 == 0 && h % 8 == 0) ? 8 : (w % 4 == 0 && h % 4 == 0) ? 4 : 2;
  for (int y = 0; y < h; y += t)
    for (int x = 0; x < w; x += t) {
      const int16_t *o = org + y * so + x, *c = cur + y * sc + x;
      sum += t == 8 ? had8(o, so, c, sc) : t == 4 ? had4(o, so, c, sc) : had2(o, so, c, sc);
    }
  return sum;
}

/* xGetSSE* (:959-1300) */
uint32_t hvxo_sse(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h) {
  uint32_t sum = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int d = org[y * so + x] - cur[y * sc + x];
      sum += (uint32_t)(d * d);
    }
  return sum;
}

/* getDistPart for a chroma component (:443-446): (Distortion)(weight * sse) */
uint32_t hvxo_sse_weighted(const int16_t *org, int so, const int16_t *cur, int sc, int w, int h, double weight) {
  return (uint32_t)(weight * (double)hvxo_sse(org, so, cur, sc, w, h));
}

/* xGetExpGolombNumberOfBits (:279) */
uint32_t hvxo_eg_bits(int v) {
  uint32_t len = 1;
  uint32_t t = (v <= 0) ? ((uint32_t)(-v) << 1) + 1 : (uint32_t)v << 1;
  while (t != 1) { t >>= 1; len += 2; }
  return len;
}

/* ============================================================================================
 * Interpolation: TComInterpolationFilter.cpp (8-bit: IF_INTERNAL_PREC 14, IF_FILTER_PREC 6)
 * ========================================================================================== */
#define IF_OFFS 8192
static inline int16_t clip_pel(int v) { return (int16_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* filterCopy (:94) */
static void filter_copy(const int16_t *src, int ss, int16_t *dst, int ds, int w, int h, int is_first, int is_last) {
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int v = src[y * ss + x];
      if (is_first == is_last) dst[y * ds + x] = (int16_t)v;
      else if (is_first) dst[y * ds + x] = (int16_t)((int16_t)(v << 6) - IF_OFFS);
      else dst[y * ds + x] = clip_pel((v + IF_OFFS + 32) >> 6);
    }
}

/* filter<N,isVertical,isFirst,isLast> (:172-257) */
static void filter_n(int ntaps, const int *c, int vertical, const int16_t *src, int ss, int16_t *dst, int ds,
                     int w, int h, int is_first, int is_last) {
  int cstride = vertical ? ss : 1;
  src -= (ntaps / 2 - 1) * cstride;
  int head = 6, shift = 6, offset;
  if (is_last) {
    shift += is_first ? 0 : head;
    offset = 1 << (shift - 1);
    offset += is_first ? 0 : IF_OFFS << 6;
  } else {
    shift -= is_first ? head : 0;
    offset = is_first ? -IF_OFFS << shift : 0;
  }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int sum = 0;
      for (int k = 0; k < ntaps; k++) sum += src[y * ss + x + k * cstride] * c[k];
      int16_t v = (int16_t)((sum + offset) >> shift);
      if (is_last) v = clip_pel(v);
      dst[y * ds + x] = v;
    }
}

/* filterHor (:341); chroma frac is the 1/8-pel index at 4:2:0 (frac << (1 - csx), csx = 1) */
void hvxo_filter_hor(int is_luma, const int16_t *src, int ss, int16_t *dst, int ds, int w, int h, int frac, int is_last) {
  if (frac == 0) filter_copy(src, ss, dst, ds, w, h, 1, is_last);
  else if (is_luma) filter_n(8, kLumaFilter[frac], 0, src, ss, dst, ds, w, h, 1, is_last);
  else filter_n(4, kChromaFilter[frac], 0, src, ss, dst, ds, w, h, 1, is_last);
}

/* filterVer (:377) */
void hvxo_filter_ver(int is_luma, const int16_t *src, int ss, int16_t *dst, int ds, int w, int h, int frac,
                     int is_first, int is_last) {
  if (frac == 0) filter_copy(src, ss, dst, ds, w, h, is_first, is_last);
  else if (is_luma) filter_n(8, kLumaFilter[frac], 1, src, ss, dst, ds, w, h, is_first, is_last);
  else filter_n(4, kChromaFilter[frac], 1, src, ss, dst, ds, w, h, is_first, is_last);
}

/* Quarter-sample luma block at quarter-pel MV, standard two-stage (TComPrediction::xPredInterBlk
 * TComPrediction.cpp:668-706 order: horizontal non-last into 16-bit, then vertical last). */
void hvxo_luma_block_qpel(const uint8_t *ref, int stride, int x, int y, int mvx, int mvy, int w, int h, int16_t *out, int os) {
  int fx = mvx & 3, fy = mvy & 3, ix = x + (mvx >> 2), iy = y + (mvy >> 2);
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      const uint8_t *p = ref + (iy + r) * stride + ix + c;
      int v;
      if (!fx && !fy) v = p[0];
      else if (!fy) {
        int s = 0;
        for (int k = 0; k < 8; k++) s += kLumaFilter[fx][k] * p[k - 3];
        v = clip_pel((s + 32) >> 6);
      } else if (!fx) {
        int s = 0;
        for (int k = 0; k < 8; k++) s += kLumaFilter[fy][k] * p[(k - 3) * stride];
        v = clip_pel((s + 32) >> 6);
      } else {
        int s2 = 0;
        for (int t = 0; t < 8; t++) {
          int s = 0;
          for (int k = 0; k < 8; k++) s += kLumaFilter[fx][k] * p[(t - 3) * stride + k - 3];
          s2 += kLumaFilter[fy][t] * (int16_t)(s - IF_OFFS);
        }
        v = clip_pel((s2 + (1 << 11) + (IF_OFFS << 6)) >> 12);
      }
      out[r * os + c] = (int16_t)v;
    }
}

/* ============================================================================================
 * Transforms: xTrMxN / xITrMxN (TComTrQuant.cpp:860-987).  Partial butterflies (:388-848) are
 * exact integer matrix products; written here as the products they compute.
 * 8-bit: forward shift_1st = log2 - 1, shift_2nd = log2 + 6; inverse 7 and 12, clip to 16 bits.
 * ========================================================================================== */
static int mat(int n, int use_dst, int k, int x) {
  if (use_dst) return kDst4[k][x];
  init_tables();
  int l = n == 4 ? 0 : n == 8 ? 1 : n == 16 ? 2 : 3;
  return g_mat[l][k * n + x];
}

void hvxo_fwd_transform(const int32_t *block, int32_t *coeff, int n, int use_dst) {
  int log2 = n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : 5;
  int s1 = log2 - 1, s2 = log2 + 6;
  int a1 = s1 > 0 ? 1 << (s1 - 1) : 0, a2 = 1 << (s2 - 1);
  int32_t tmp[32 * 32];
  for (int y = 0; y < n; y++)
    for (int u = 0; u < n; u++) {
      int s = 0;
      for (int x = 0; x < n; x++) s += mat(n, use_dst, u, x) * block[y * n + x];
      tmp[u * n + y] = (s + a1) >> s1;
    }
  for (int u = 0; u < n; u++)
    for (int v = 0; v < n; v++) {
      int s = 0;
      for (int y = 0; y < n; y++) s += mat(n, use_dst, v, y) * tmp[u * n + y];
      coeff[v * n + u] = (s + a2) >> s2;
    }
}

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }

void hvxo_inv_transform(const int32_t *coeff, int32_t *block, int n, int use_dst) {
  int32_t tmp[32 * 32];
  for (int u = 0; u < n; u++)
    for (int y = 0; y < n; y++) {
      int s = 0;
      for (int v = 0; v < n; v++) s += mat(n, use_dst, v, y) * coeff[v * n + u];
      tmp[u * n + y] = clip3(-32768, 32767, (s + 64) >> 7);
    }
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++) {
      int s = 0;
      for (int u = 0; u < n; u++) s += mat(n, use_dst, u, x) * tmp[u * n + y];
      block[y * n + x] = clip3(-32768, 32767, (s + 2048) >> 12);
    }
}

/* ============================================================================================
 * Quantisation.  TComTrQuant.cpp:991-1430, 2129-3052; context selection from
 * TComChromaFormat.h:203-262 / TComChromaFormat.cpp:96-150 and ContextTables.h.
 * ========================================================================================== */
typedef struct {
  const uint32_t *scan, *scan_cg;
  int wg, hg;          /* width/height in 4x4 groups */
  int scan_type;
  int first_sig_ctx;   /* firstSignificanceMapContext */
} coding_params;

static const int kSigCtxSetStart[2][4] = {{0, 9, 21, 27}, {0, 9, 12, 15}};

static void get_coding_params(const hvx_tu_desc *tu, coding_params *cp) {
  int lw = tu->width == 4 ? 2 : tu->width == 8 ? 3 : tu->width == 16 ? 4 : 5;
  int lh = tu->height == 4 ? 2 : tu->height == 8 ? 3 : tu->height == 16 ? 4 : 5;
  int ch = tu->comp ? 1 : 0;
  cp->scan_type = tu->scan_type;
  cp->wg = tu->width >> 2;
  cp->hg = tu->height >> 2;
  cp->scan = hvxo_scan(1, tu->scan_type, lw, lh);
  cp->scan_cg = hvxo_scan(0, tu->scan_type, lw - 2, lh - 2);
  if (tu->ts_context && (tu->transquant_bypass || tu->transform_skip)) cp->first_sig_ctx = kSigCtxSetStart[ch][3];
  else if (tu->width == 4 && tu->height == 4) cp->first_sig_ctx = kSigCtxSetStart[ch][0];
  else if (tu->width == 8 && tu->height == 8) cp->first_sig_ctx = kSigCtxSetStart[ch][1] + (tu->scan_type != 0 ? (ch ? 0 : 6) : 0);
  else cp->first_sig_ctx = kSigCtxSetStart[ch][2];
}

static int transform_shift(const hvx_tu_desc *tu) {
  int s = tu->max_log2_tr_range - tu->bit_depth - tu->log2_size;
  if (tu->transform_skip && tu->extended_precision && s < 0) s = 0;
  return s;
}

/* calcPatternSigCtx (:2682) */
static int pattern_sig_ctx(const uint32_t *flags, int cx, int cy, int wg, int hg) {
  if (wg <= 1 && hg <= 1) return 0;
  int r = cx < wg - 1 ? (flags[cy * wg + cx + 1] != 0) : 0;
  int b = cy < hg - 1 ? (flags[(cy + 1) * wg + cx] != 0) : 0;
  return r + (b << 1);
}

/* getSigCtxInc (:2717) */
static int sig_ctx_inc(int pattern, const coding_params *cp, int scan_pos, int lw, int lh, int ch) {
  if (cp->first_sig_ctx == kSigCtxSetStart[ch][3]) return kSigCtxSetStart[ch][3];
  int raster = (int)cp->scan[scan_pos];
  int py = raster >> lw, px = raster - (py << lw);
  if (px + py == 0) return 0;
  int offset;
  if (lw == 2 && lh == 2) offset = kCtxIndMap4x4[4 * py + px];
  else {
    int cnt;
    switch (pattern) {
      case 0: { int t = (px & 3) + (py & 3); cnt = t >= 3 ? 0 : t >= 1 ? 1 : 2; } break;
      case 1: { int y = py & 3; cnt = y >= 2 ? 0 : y >= 1 ? 1 : 2; } break;
      case 2: { int x = px & 3; cnt = x >= 2 ? 0 : x >= 1 ? 1 : 2; } break;
      default: cnt = 2; break;
    }
    int not_first = ((px >> 2) + (py >> 2)) > 0;
    offset = (not_first ? (ch ? 0 : 3) : 0) + cnt;
  }
  return cp->first_sig_ctx + offset;
}

/* getSigCoeffGroupCtxInc (:3033) */
static int sig_cg_ctx(const uint32_t *flags, int cx, int cy, int wg, int hg) {
  int r = cx < wg - 1 ? (flags[cy * wg + cx + 1] != 0) : 0;
  int b = cy < hg - 1 ? (flags[(cy + 1) * wg + cx] != 0) : 0;
  return (r + b) != 0;
}

/* getContextSetIndex (TComChromaFormat.h:243) */
static int ctx_set_index(int comp, int subset, int found_gt1) {
  return (comp ? 4 : 0) + ((comp == 0 && subset > 0) ? 2 : 0) + (found_gt1 ? 1 : 0);
}

typedef struct {
  const hvx_estbits *est;
  double lambda;
} rd_ctx;

static inline double icost(const rd_ctx *r, double rate) { return r->lambda * rate; }  /* xGetICost :3012 */

/* xGetICRate (:2891) */
static int ic_rate(const rd_ctx *r, uint32_t level, int ctx_one, int ctx_abs, int rice, uint32_t c1_idx, uint32_t c2_idx,
                   int limited_prefix, int max_log2) {
  int rate = 32768;
  uint32_t base = (c1_idx < 8) ? (2 + (c2_idx < 1)) : 1;
  if (level >= base) {
    uint32_t symbol = level - base;
    if (symbol < (3u << rice)) {
      uint32_t len = symbol >> rice;
      rate += (int)((len + 1 + rice) << 15);
    } else if (limited_prefix) {
      uint32_t maxp = 32 - (3 + max_log2), prefix = 0, suffix = (symbol >> rice) - 3;
      while (prefix < maxp && suffix > ((2u << prefix) - 2)) prefix++;
      uint32_t suffix_len = prefix == maxp ? (uint32_t)(max_log2 - rice) : prefix + 1;
      rate += (int)((3 + prefix + suffix_len + rice) << 15);
    } else {
      uint32_t len = rice;
      symbol = symbol - (3u << rice);
      while (symbol >= (1u << len)) { symbol -= (1u << (len++)); }
      rate += (int)((3 + len + 1 - rice + len) << 15);
    }
    if (c1_idx < 8) {
      rate += r->est->greaterOneBits[ctx_one][1];
      if (c2_idx < 1) rate += r->est->levelAbsBits[ctx_abs][1];
    }
  } else if (level == 1) {
    rate += r->est->greaterOneBits[ctx_one][0];
  } else if (level == 2) {
    rate += r->est->greaterOneBits[ctx_one][1];
    rate += r->est->levelAbsBits[ctx_abs][0];
  } else {
    rate = 0;
  }
  return rate;
}

static inline double rate_sig(const rd_ctx *r, int v, int ctx) { return icost(r, (double)r->est->significantBits[ctx][v]); }
static inline double rate_sig_cg(const rd_ctx *r, int v, int ctx) { return icost(r, (double)r->est->significantCoeffGroupBits[ctx][v]); }

/* xGetRateLast (:2982) */
static double rate_last(const rd_ctx *r, int px, int py, int ch) {
  int cx = kGroupIdx[px], cy = kGroupIdx[py];
  double c = (double)(r->est->lastXBits[ch][cx] + r->est->lastYBits[ch][cy]);
  if (cx > 3) c += 32768.0 * ((cx - 2) >> 1);
  if (cy > 3) c += 32768.0 * ((cy - 2) >> 1);
  return icost(r, c);
}

/* wrapping int32 helpers (Intermediate_Int is 32-bit in the reference Main build) */
static inline int32_t shl32(int32_t v, int s) { return (int32_t)((uint32_t)v << s); }
static inline int32_t sub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

/* xGetCodedLevel (:2822) */
static uint32_t coded_level(const rd_ctx *r, double *cost, double *cost0, double *cost_sig, int32_t level_double,
                            uint32_t max_abs, int ctx_sig, int ctx_one, int ctx_abs, int rice, uint32_t c1_idx,
                            uint32_t c2_idx, int qbits, double err_scale, int last, int limited, int max_log2) {
  double cur_sig = 0;
  uint32_t best = 0;
  if (!last && max_abs < 3) {
    *cost_sig = rate_sig(r, 0, ctx_sig);
    *cost = *cost0 + *cost_sig;
    if (max_abs == 0) return best;
  } else {
    *cost = 1.7e+308;  /* MAX_DOUBLE (CommonDef.h) */
  }
  if (!last) cur_sig = rate_sig(r, 1, ctx_sig);
  uint32_t min_abs = max_abs > 1 ? max_abs - 1 : 1;
  for (int lv = (int)max_abs; lv >= (int)min_abs; lv--) {
    double err = (double)sub32(level_double, shl32(lv, qbits));
    double c = err * err * err_scale + icost(r, (double)ic_rate(r, (uint32_t)lv, ctx_one, ctx_abs, rice, c1_idx, c2_idx, limited, max_log2));
    c += cur_sig;
    if (c < *cost) { best = (uint32_t)lv; *cost = c; *cost_sig = cur_sig; }
  }
  return best;
}

/* setErrScaleCoeff (:3106-3129), flat scaling list */
static double err_scale(const hvx_tu_desc *tu) {
  int ts = tu->max_log2_tr_range - tu->bit_depth - tu->log2_size;
  double e = (double)(1 << 15);
  e = e * pow(2.0, (-2.0 * ts));
  int q = kQuantScales[tu->qp_rem];
  return e / q / q / (1 << 0);
}

/* xRateDistOptQuant (:2129-2671) */
#ifdef HVXO_RDOQ_STATS
long long hvxo_rdoq_stat[4][3]; /* per log2 size - 2: calls, calls with every rounded level 0, calls with absSum 0 */
long long hvxo_rdoq_spec[4][3]; /* per log2 size - 2: decided positions, positions after a speculation miss, groups with a miss */
#endif
static void rdoq(const hvx_tu_desc *tu, const hvx_estbits *est, const int32_t *src, int32_t *dst, int32_t *arl, int32_t *abs_sum) {
  const int w = tu->width, h = tu->height, ch = tu->comp ? 1 : 0, comp = tu->comp;
#ifdef HVXO_RDOQ_STATS
  {
    const int qb = 14 + tu->qp_per + transform_shift(tu), qc = kQuantScales[tu->qp_rem];
    int anyq = 0;
    for (int i = 0; i < w * h; i++) {
      int64_t t = (int64_t)abs(src[i]) * qc;
      int64_t lim = (int64_t)INT32_MAX - ((int64_t)1 << (qb - 1));
      int32_t ld = (int32_t)(t < lim ? t : lim);
      if (((ld + (1 << (qb - 1))) >> qb) > 0) anyq = 1;
    }
    const int l = (w == 4 ? 0 : w == 8 ? 1 : w == 16 ? 2 : 3);
    __atomic_add_fetch(&hvxo_rdoq_stat[l][0], 1, __ATOMIC_RELAXED);
    if (!anyq) __atomic_add_fetch(&hvxo_rdoq_stat[l][1], 1, __ATOMIC_RELAXED);
  }
#endif
  const int lw = w == 4 ? 2 : w == 8 ? 3 : w == 16 ? 4 : 5, lh = h == 4 ? 2 : h == 8 ? 3 : h == 16 ? 4 : 5;
  const int n = w * h, ext = tu->extended_precision, max_log2 = tu->max_log2_tr_range;
  const int ts = transform_shift(tu);
  rd_ctx rc = {est, tu->lambda};
  const uint32_t rice0 = (uint32_t)tu->golomb_rice_stat / 4;
  uint32_t rice = rice0;
  double block_uncoded = 0;
  double cost_coeff[1024], cost_sig[1024], cost_coeff0[1024];
  int rate_up[1024], rate_down[1024], sig_delta[1024];
  int32_t delta_u[1024];
  memset(cost_coeff, 0, sizeof(double) * n);
  memset(cost_sig, 0, sizeof(double) * n);
  memset(rate_up, 0, sizeof(int) * n);
  memset(rate_down, 0, sizeof(int) * n);
  memset(sig_delta, 0, sizeof(int) * n);
  memset(delta_u, 0, sizeof(int32_t) * n);
  if (arl) memset(arl, 0, sizeof(int32_t) * n);
  const int qbits = 14 + tu->qp_per + ts;
  const double escale = err_scale(tu);
  const int qcoef = kQuantScales[tu->qp_rem];
  const int32_t ecmax = (1 << max_log2) - 1, ecmin = -(1 << max_log2);
  const int qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
  coding_params cp;
  get_coding_params(tu, &cp);
  double cost_cg_sig[64];
  uint32_t sig_cg[64];
  memset(cost_cg_sig, 0, sizeof(cost_cg_sig));
  memset(sig_cg, 0, sizeof(sig_cg));
  int cg_last = -1, last = -1;
  uint32_t ctx_set = 0, c1_idx = 0, c2_idx = 0;
  int c1 = 1, c2 = 0;
  double base_cost = 0;
  const int ncg = n >> 4;
  const int sig_off = ch ? 28 : 0;

#ifdef HVXO_RDOQ_STATS
  const int sl = (w == 4 ? 0 : w == 8 ? 1 : w == 16 ? 2 : 3);
#endif
  for (int cgp = ncg - 1; cgp >= 0; cgp--) {
#ifdef HVXO_RDOQ_STATS
    int spec_missed = 0;
#endif
    int cgblk = (int)cp.scan_cg[cgp];
    int cy = cgblk / cp.wg, cx = cgblk - cy * cp.wg;
    int nnz_before0 = 0;
    double coded_level_dist = 0, uncoded_dist = 0, sig_cost = 0, sig_cost0 = 0;
    int pattern = pattern_sig_ctx(sig_cg, cx, cy, cp.wg, cp.hg);
    for (int pin = 15; pin >= 0; pin--) {
      int sp = cgp * 16 + pin;
      int blk = (int)cp.scan[sp];
      int64_t tmp = (int64_t)abs(src[blk]) * qcoef;
      int64_t lim = (int64_t)INT32_MAX - ((int64_t)1 << (qbits - 1));
      int32_t ld = (int32_t)(tmp < lim ? tmp : lim);
      if (tu->adaptive_qp_select && arl) arl[blk] = (ld + add_c) >> qbits_c;
      uint32_t q = (uint32_t)((ld + (1 << (qbits - 1))) >> qbits);
      uint32_t max_abs = (uint32_t)ecmax < q ? (uint32_t)ecmax : q;
      double err = (double)ld;
      cost_coeff0[sp] = err * err * escale;
      block_uncoded += cost_coeff0[sp];
      dst[blk] = (int32_t)max_abs;
      if (max_abs > 0 && last < 0) {
        last = sp;
        ctx_set = (uint32_t)ctx_set_index(comp, sp >> 4, 0);
        cg_last = cgp;
      }
      if (last >= 0) {
        uint32_t level;
        int ctx_one = 4 * (int)ctx_set + c1, ctx_abs = (int)ctx_set + c2;
        if (sp == last) {
          level = coded_level(&rc, &cost_coeff[sp], &cost_coeff0[sp], &cost_sig[sp], ld, max_abs, sig_off, ctx_one,
                              ctx_abs, (int)rice, c1_idx, c2_idx, qbits, escale, 1, ext, max_log2);
        } else {
          int ctx_sig = sig_off + sig_ctx_inc(pattern, &cp, sp, lw, lh, ch);
          level = coded_level(&rc, &cost_coeff[sp], &cost_coeff0[sp], &cost_sig[sp], ld, max_abs, ctx_sig, ctx_one,
                              ctx_abs, (int)rice, c1_idx, c2_idx, qbits, escale, 0, ext, max_log2);
          sig_delta[blk] = est->significantBits[ctx_sig][1] - est->significantBits[ctx_sig][0];
        }
        delta_u[blk] = sub32(ld, shl32((int32_t)level, qbits)) >> (qbits - 8);
        if (level > 0) {
          int now = ic_rate(&rc, level, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2);
          rate_up[blk] = ic_rate(&rc, level + 1, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2) - now;
          rate_down[blk] = ic_rate(&rc, level - 1, ctx_one, ctx_abs, (int)rice, c1_idx, c2_idx, ext, max_log2) - now;
        } else {
          rate_up[blk] = est->greaterOneBits[ctx_one][0];
        }
        dst[blk] = (int32_t)level;
        base_cost += cost_coeff[sp];
#ifdef HVXO_RDOQ_STATS
        {  /* would the state update with max_abs have matched the one with the decided level? */
          uint32_t b0 = (c1_idx < 8) ? (2 + (c2_idx < 1)) : 1;
          int r_a = level >= b0 && level > 3u * (1u << rice), r_b = max_abs >= b0 && max_abs > 3u * (1u << rice);
          int same = r_a == r_b && (level >= 1) == (max_abs >= 1) && (level > 1) == (max_abs > 1) &&
                     (level == 1) == (max_abs == 1);
          __atomic_add_fetch(&hvxo_rdoq_spec[sl][0], 1, __ATOMIC_RELAXED);
          if (spec_missed) __atomic_add_fetch(&hvxo_rdoq_spec[sl][1], 1, __ATOMIC_RELAXED);
          if (!same && !spec_missed) { spec_missed = 1; __atomic_add_fetch(&hvxo_rdoq_spec[sl][2], 1, __ATOMIC_RELAXED); }
        }
#endif
        uint32_t base = (c1_idx < 8) ? (2 + (c2_idx < 1)) : 1;
        if (level >= base && level > 3u * (1u << rice)) rice = tu->persistent_rice ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
        if (level >= 1) c1_idx++;
        if (level > 1) { c1 = 0; c2 += (c2 < 2); c2_idx++; }
        else if (c1 < 3 && c1 > 0 && level) c1++;
        if ((sp % 16 == 0) && sp > 0) {
          ctx_set = (uint32_t)ctx_set_index(comp, (sp - 1) >> 4, c1 == 0);
          c1 = 1; c2 = 0; c1_idx = 0; c2_idx = 0;
          rice = rice0;
        }
      } else {
        base_cost += cost_coeff0[sp];
      }
      sig_cost += cost_sig[sp];
      if (pin == 0) sig_cost0 = cost_sig[sp];
      if (dst[blk]) {
        sig_cg[cgblk] = 1;
        coded_level_dist += cost_coeff[sp] - cost_sig[sp];
        uncoded_dist += cost_coeff0[sp];
        if (pin != 0) nnz_before0++;
      }
    }
    if (cg_last >= 0) {
      if (cgp) {
        if (sig_cg[cgblk] == 0) {
          int ctx = sig_cg_ctx(sig_cg, cx, cy, cp.wg, cp.hg);
          base_cost += rate_sig_cg(&rc, 0, ctx) - sig_cost;
          cost_cg_sig[cgp] = rate_sig_cg(&rc, 0, ctx);
        } else if (cgp < cg_last) {
          if (nnz_before0 == 0) { base_cost -= sig_cost0; sig_cost -= sig_cost0; }
          double cost_zero_cg = base_cost;
          int ctx = sig_cg_ctx(sig_cg, cx, cy, cp.wg, cp.hg);
          base_cost += rate_sig_cg(&rc, 1, ctx);
          cost_zero_cg += rate_sig_cg(&rc, 0, ctx);
          cost_cg_sig[cgp] = rate_sig_cg(&rc, 1, ctx);
          cost_zero_cg += uncoded_dist;
          cost_zero_cg -= coded_level_dist;
          cost_zero_cg -= sig_cost;
          if (cost_zero_cg < base_cost) {
            sig_cg[cgblk] = 0;
            base_cost = cost_zero_cg;
            cost_cg_sig[cgp] = rate_sig_cg(&rc, 0, ctx);
            for (int pin = 15; pin >= 0; pin--) {
              int sp = cgp * 16 + pin;
              int blk = (int)cp.scan[sp];
              if (dst[blk]) { dst[blk] = 0; cost_coeff[sp] = cost_coeff0[sp]; cost_sig[sp] = 0; }
            }
          }
        }
      } else {
        sig_cg[cgblk] = 1;
      }
    }
  }

  if (last < 0) return;

  double best_cost;
  int best_last_p1 = 0;
  if (!tu->is_intra && ch == 0 && tu->tr_idx == 0) {
    best_cost = block_uncoded + icost(&rc, (double)est->blockRootCbpBits[0][0]);
    base_cost += icost(&rc, (double)est->blockRootCbpBits[0][1]);
  } else {
    int ctx = tu->ctx_qt_cbf + (ch ? 5 : 0);
    best_cost = block_uncoded + icost(&rc, (double)est->blockCbpBits[ctx][0]);
    base_cost += icost(&rc, (double)est->blockCbpBits[ctx][1]);
  }
  int found = 0;
  for (int cgp = cg_last; cgp >= 0; cgp--) {
    int cgblk = (int)cp.scan_cg[cgp];
    base_cost -= cost_cg_sig[cgp];
    if (sig_cg[cgblk]) {
      for (int pin = 15; pin >= 0; pin--) {
        int sp = cgp * 16 + pin;
        if (sp > last) continue;
        int blk = (int)cp.scan[sp];
        if (dst[blk]) {
          int py = blk >> lw, px = blk - (py << lw);
          double cl = cp.scan_type == 2 ? rate_last(&rc, py, px, ch) : rate_last(&rc, px, py, ch);
          double total = base_cost + cl - cost_sig[sp];
          if (total < best_cost) { best_last_p1 = sp + 1; best_cost = total; }
          if (dst[blk] > 1) { found = 1; break; }
          base_cost -= cost_coeff[sp];
          base_cost += cost_coeff0[sp];
        } else {
          base_cost -= cost_sig[sp];
        }
      }
      if (found) break;
    }
  }
  for (int sp = 0; sp < best_last_p1; sp++) {
    int blk = (int)cp.scan[sp];
    int32_t lv = dst[blk];
    *abs_sum += lv;
    dst[blk] = src[blk] < 0 ? -lv : lv;
  }
  for (int sp = best_last_p1; sp <= last; sp++) dst[cp.scan[sp]] = 0;

  if (tu->sign_hiding && *abs_sum >= 2) {
    const double iq = (double)kInvQuantScales[tu->qp_rem];
    int64_t rd_factor = (int64_t)(iq * iq * (1 << (2 * tu->qp_per)) / tu->lambda / 16 / (1 << 0) + 0.5);
    int last_cg = -1;
    for (int sub = (n - 1) >> 4; sub >= 0; sub--) {
      int pos = sub << 4, first_nz = 16, last_nz = -1, abs_in = 0, k;
      for (k = 15; k >= 0; k--) if (dst[cp.scan[k + pos]]) { last_nz = k; break; }
      for (k = 0; k < 16; k++) if (dst[cp.scan[k + pos]]) { first_nz = k; break; }
      for (k = first_nz; k <= last_nz; k++) abs_in += dst[cp.scan[k + pos]];
      if (last_nz >= 0 && last_cg == -1) last_cg = 1;
      if (last_nz - first_nz >= 4) {
        uint32_t signbit = dst[cp.scan[pos + first_nz]] > 0 ? 0 : 1;
        if (signbit != (uint32_t)(abs_in & 1)) {
          int64_t min_inc = INT64_MAX, cur = INT64_MAX;
          int min_pos = -1, final_change = 0, cur_change = 0;
          for (k = (last_cg == 1 ? last_nz : 15); k >= 0; k--) {
            int blk = (int)cp.scan[k + pos];
            if (dst[blk] != 0) {
              int64_t up = rd_factor * (-delta_u[blk]) + rate_up[blk];
              int64_t down = rd_factor * (delta_u[blk]) + rate_down[blk] - ((abs(dst[blk]) == 1) ? sig_delta[blk] : 0);
              if (last_cg == 1 && last_nz == k && abs(dst[blk]) == 1) down -= (4 << 15);
              if (up < down) { cur = up; cur_change = 1; }
              else {
                cur_change = -1;
                cur = (k == first_nz && abs(dst[blk]) == 1) ? INT64_MAX : down;
              }
            } else {
              cur = rd_factor * (-(abs(delta_u[blk]))) + (1 << 15) + rate_up[blk] + sig_delta[blk];
              cur_change = 1;
              if (k < first_nz) {
                uint32_t ts_bit = src[blk] >= 0 ? 0 : 1;
                if (ts_bit != signbit) cur = INT64_MAX;
              }
            }
            if (cur < min_inc) { min_inc = cur; final_change = cur_change; min_pos = blk; }
          }
          if (dst[min_pos] == ecmax || dst[min_pos] == ecmin) final_change = -1;
          if (src[min_pos] >= 0) dst[min_pos] += final_change;
          else dst[min_pos] -= final_change;
        }
      }
      if (last_cg == 1) last_cg = 0;
    }
  }
}

/* signBitHidingHDQ (:991) */
static void sbh_hdq(int32_t *q, const int32_t *coef, const int32_t *delta_u, const coding_params *cp, int n, int max_log2) {
  const int32_t ecmax = (1 << max_log2) - 1, ecmin = -(1 << max_log2);
  int last_cg = -1;
  for (int sub = (n - 1) >> 4; sub >= 0; sub--) {
    int pos = sub << 4, first_nz = 16, last_nz = -1, abs_in = 0, k;
    for (k = 15; k >= 0; k--) if (q[cp->scan[k + pos]]) { last_nz = k; break; }
    for (k = 0; k < 16; k++) if (q[cp->scan[k + pos]]) { first_nz = k; break; }
    for (k = first_nz; k <= last_nz; k++) abs_in += q[cp->scan[k + pos]];
    if (last_nz >= 0 && last_cg == -1) last_cg = 1;
    if (last_nz - first_nz >= 4) {
      uint32_t signbit = q[cp->scan[pos + first_nz]] > 0 ? 0 : 1;
      if (signbit != (uint32_t)(abs_in & 1)) {
        int32_t cur = INT32_MAX, min_inc = INT32_MAX;
        int min_pos = -1, final_change = 0, cur_change = 0;
        for (k = (last_cg == 1 ? last_nz : 15); k >= 0; k--) {
          int blk = (int)cp->scan[k + pos];
          if (q[blk] != 0) {
            if (delta_u[blk] > 0) { cur = -delta_u[blk]; cur_change = 1; }
            else if (k == first_nz && abs(q[blk]) == 1) cur = INT32_MAX;
            else { cur = delta_u[blk]; cur_change = -1; }
          } else if (k < first_nz) {
            uint32_t tsb = coef[blk] >= 0 ? 0 : 1;
            if (tsb != signbit) cur = INT32_MAX;
            else { cur = -delta_u[blk]; cur_change = 1; }
          } else {
            cur = -delta_u[blk]; cur_change = 1;
          }
          if (cur < min_inc) { min_inc = cur; final_change = cur_change; min_pos = blk; }
        }
        if (q[min_pos] == ecmax || q[min_pos] == ecmin) final_change = -1;
        if (coef[min_pos] >= 0) q[min_pos] += final_change;
        else q[min_pos] -= final_change;
      }
    }
    if (last_cg == 1) last_cg = 0;
  }
}

/* xQuant (:1126) incl. T0196 selective RDOQ (xNeedRDOQ :1257) */
void hvxo_quant(const hvx_tu_desc *tu, const hvx_estbits *est, const int32_t *coef, int32_t *levels, int32_t *arl, int32_t *abs_sum) {
  const int n = tu->width * tu->height;
  const int ts = transform_shift(tu);
  const int qbits = 14 + tu->qp_per + ts;
  const int qc = kQuantScales[tu->qp_rem];
  *abs_sum = 0;
  int use_rdoq = tu->transform_skip ? tu->use_rdoq_ts : tu->use_rdoq;
  if (use_rdoq) {
    int need = 1;
    if (tu->selective_rdoq) {
      int add = (tu->comp == 0 ? 171 : 256) << (qbits - 9);
      need = 0;
      for (int i = 0; i < n && !need; i++) {
        int64_t t = (int64_t)abs(coef[i]) * qc;
        if ((int32_t)((t + add) >> qbits) != 0) need = 1;
      }
    }
    if (need) rdoq(tu, est, coef, levels, arl, abs_sum);
    else { memset(levels, 0, sizeof(int32_t) * n); *abs_sum = 0; }
    return;
  }
  coding_params cp;
  get_coding_params(tu, &cp);
  const int32_t ecmax = (1 << tu->max_log2_tr_range) - 1, ecmin = -(1 << tu->max_log2_tr_range);
  int32_t delta_u[1024];
  const int add = (tu->slice_type == 2 ? 171 : 85) << (qbits - 9);
  const int qbits8 = qbits - 8;
  const int qbits_c = qbits - 7, add_c = 1 << (qbits_c - 1);
  for (int i = 0; i < n; i++) {
    int32_t lv = coef[i];
    int sign = lv < 0 ? -1 : 1;
    int64_t t = (int64_t)abs(lv) * qc;
    if (tu->adaptive_qp_select && arl) arl[i] = (int32_t)((t + add_c) >> qbits_c);
    int32_t qm = (int32_t)((t + add) >> qbits);
    delta_u[i] = (int32_t)((t - (int64_t)shl32(qm, qbits)) >> qbits8);
    *abs_sum += qm;
    levels[i] = clip3(ecmin, ecmax, qm * sign);
  }
  if (tu->sign_hiding && *abs_sum >= 2) sbh_hdq(levels, coef, delta_u, &cp, n, tu->max_log2_tr_range);
}

/* transformNxN (:1460): bypass / transform-skip (:2021) / xT, then xQuant */
void hvxo_transform_nxn(const hvx_tu_desc *tu, const hvx_estbits *est, const int16_t *residual, int stride,
                        int32_t *temp, int32_t *levels, int32_t *arl, int32_t *abs_sum) {
  const int w = tu->width, h = tu->height;
  *abs_sum = 0;
  if (tu->transquant_bypass) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) { levels[y * w + x] = residual[y * stride + x]; *abs_sum += abs(residual[y * stride + x]); }
    return;
  }
  if (tu->transform_skip) {
    int ts = transform_shift(tu);
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        int32_t v = residual[y * stride + x];
        temp[y * w + x] = ts >= 0 ? shl32(v, ts) : (v + (1 << (-ts - 1))) >> -ts;
      }
  } else {
    int32_t blk[1024];
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) blk[y * w + x] = residual[y * stride + x];
    hvxo_fwd_transform(blk, temp, w, tu->use_dst && w == 4 && h == 4);  /* xTrMxN :876 */
  }
  hvxo_quant(tu, est, temp, levels, arl, abs_sum);
}

/* invTransformNxN (:1547) = xDeQuant (:1314, flat list) + xITransformSkip (:2070) / xIT (:1988) */
void hvxo_inv_transform_nxn(const hvx_tu_desc *tu, const int32_t *levels, int16_t *residual, int stride) {
  const int w = tu->width, h = tu->height, n = w * h;
  if (tu->transquant_bypass) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) residual[y * stride + x] = (int16_t)levels[y * w + x];
    return;
  }
  const int ts = transform_shift(tu);
  const int max_log2 = tu->max_log2_tr_range;
  const int32_t tmin = -(1 << max_log2), tmax = (1 << max_log2) - 1;
  const int right = 6 - (ts + tu->qp_per);
  const int scale = kInvQuantScales[tu->qp_rem];
  int tib = 32 + right - 7;
  if (max_log2 + 1 < tib) tib = max_log2 + 1;
  const int32_t imin = -(1 << (tib - 1)), imax = (1 << (tib - 1)) - 1;
  int32_t deq[1024];
  for (int i = 0; i < n; i++) {
    int32_t c = clip3(imin, imax, levels[i]);
    int32_t v = right > 0 ? (c * scale + (1 << (right - 1))) >> right : shl32(c * scale, -right);
    deq[i] = clip3(tmin, tmax, v);
  }
  if (tu->transform_skip) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        int32_t v = deq[y * w + x];
        residual[y * stride + x] = (int16_t)(ts >= 0 ? (v + (ts == 0 ? 0 : 1 << (ts - 1))) >> ts : shl32(v, -ts));
      }
  } else {
    int32_t blk[1024];
    hvxo_inv_transform(deq, blk, w, tu->use_dst && w == 4 && h == 4);  /* xITrMxN :945 */
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) residual[y * stride + x] = (int16_t)blk[y * w + x];
  }
}

/* ============================================================================================
 * Motion estimation: TEncSearch.cpp (uni-prediction xMotionEstimation, TZ search config :297)
 * ========================================================================================== */
typedef struct {
  const uint8_t *org; int so;  /* PU origin in the current plane */
  const int16_t *org16;        /* or an int16 pattern (full search / bi target), stride so */
  const uint8_t *ref; int sr;  /* PU origin in the reference plane (MV 0) */
  int w, h, sub;
  uint32_t lam;                /* m_uiCost */
  int px, py, cost_scale;      /* m_mvPredictor, m_iCostScale */
  int best_x, best_y, best_dist, best_round, point_nr;
  uint32_t best_sad;
} tz_state;

/* TComRdCost::getCost(x, y) (TComRdCost.h:172) */
static inline uint32_t mv_cost(const tz_state *t, int x, int y) {
  uint32_t bits = hvxo_eg_bits((x << t->cost_scale) - t->px) + hvxo_eg_bits((y << t->cost_scale) - t->py);
  return (t->lam * bits) >> 16;
}

static uint32_t sad_u8(const uint8_t *o, int so, const uint8_t *c, int sc, int w, int h, int sub) {
  int specialised = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  if (!specialised) sub = 0;
  uint32_t s = 0;
  for (int y = 0; y < h; y += 1 << sub)
    for (int x = 0; x < w; x++) s += (uint32_t)abs((int)o[y * so + x] - (int)c[y * sc + x]);
  return s << sub;
}

/* xTZSearchHelp (:332), non-SELECTIVE branch */
static void tz_help(tz_state *t, int x, int y, int point_nr, int dist) {
  uint32_t sad = sad_u8(t->org, t->so, t->ref + y * t->sr + x, t->sr, t->w, t->h, t->sub);
  sad += mv_cost(t, x, y);
  if (sad < t->best_sad) {
    t->best_sad = sad; t->best_x = x; t->best_y = y; t->best_dist = dist; t->best_round = 0; t->point_nr = point_nr;
  }
}

typedef struct { int l, r, t, b; } srch_rng;

/* xTZ2PointSearch (:438) */
static void tz_2point(tz_state *t, const srch_rng *g) {
  int sx = t->best_x, sy = t->best_y;
  switch (t->point_nr) {
    case 1:
      if (sx - 1 >= g->l) tz_help(t, sx - 1, sy, 0, 2);
      if (sy - 1 >= g->t) tz_help(t, sx, sy - 1, 0, 2);
      break;
    case 2:
      if (sy - 1 >= g->t) {
        if (sx - 1 >= g->l) tz_help(t, sx - 1, sy - 1, 0, 2);
        if (sx + 1 <= g->r) tz_help(t, sx + 1, sy - 1, 0, 2);
      }
      break;
    case 3:
      if (sy - 1 >= g->t) tz_help(t, sx, sy - 1, 0, 2);
      if (sx + 1 <= g->r) tz_help(t, sx + 1, sy, 0, 2);
      break;
    case 4:
      if (sx - 1 >= g->l) {
        if (sy + 1 <= g->b) tz_help(t, sx - 1, sy + 1, 0, 2);
        if (sy - 1 >= g->t) tz_help(t, sx - 1, sy - 1, 0, 2);
      }
      break;
    case 5:
      if (sx + 1 <= g->r) {
        if (sy - 1 >= g->t) tz_help(t, sx + 1, sy - 1, 0, 2);
        if (sy + 1 <= g->b) tz_help(t, sx + 1, sy + 1, 0, 2);
      }
      break;
    case 6:
      if (sx - 1 >= g->l) tz_help(t, sx - 1, sy, 0, 2);
      if (sy + 1 <= g->b) tz_help(t, sx, sy + 1, 0, 2);
      break;
    case 7:
      if (sy + 1 <= g->b) {
        if (sx - 1 >= g->l) tz_help(t, sx - 1, sy + 1, 0, 2);
        if (sx + 1 <= g->r) tz_help(t, sx + 1, sy + 1, 0, 2);
      }
      break;
    case 8:
      if (sx + 1 <= g->r) tz_help(t, sx + 1, sy, 0, 2);
      if (sy + 1 <= g->b) tz_help(t, sx, sy + 1, 0, 2);
      break;
    default: abort();
  }
}

/* xTZ8PointDiamondSearch (:629) */
static void tz_diamond(tz_state *t, const srch_rng *g, int sx, int sy, int d) {
  const int top = sy - d, bottom = sy + d, left = sx - d, right = sx + d;
  t->best_round += 1;
  if (d == 1) {
    if (top >= g->t) tz_help(t, sx, top, 2, d);
    if (left >= g->l) tz_help(t, left, sy, 4, d);
    if (right <= g->r) tz_help(t, right, sy, 5, d);
    if (bottom <= g->b) tz_help(t, sx, bottom, 7, d);
    return;
  }
  const int inside = top >= g->t && left >= g->l && right <= g->r && bottom <= g->b;
  if (d <= 8) {
    const int t2 = sy - (d >> 1), b2 = sy + (d >> 1), l2 = sx - (d >> 1), r2 = sx + (d >> 1);
    if (inside) {
      tz_help(t, sx, top, 2, d);
      tz_help(t, l2, t2, 1, d >> 1);
      tz_help(t, r2, t2, 3, d >> 1);
      tz_help(t, left, sy, 4, d);
      tz_help(t, right, sy, 5, d);
      tz_help(t, l2, b2, 6, d >> 1);
      tz_help(t, r2, b2, 8, d >> 1);
      tz_help(t, sx, bottom, 7, d);
    } else {
      if (top >= g->t) tz_help(t, sx, top, 2, d);
      if (t2 >= g->t) {
        if (l2 >= g->l) tz_help(t, l2, t2, 1, d >> 1);
        if (r2 <= g->r) tz_help(t, r2, t2, 3, d >> 1);
      }
      if (left >= g->l) tz_help(t, left, sy, 4, d);
      if (right <= g->r) tz_help(t, right, sy, 5, d);
      if (b2 <= g->b) {
        if (l2 >= g->l) tz_help(t, l2, b2, 6, d >> 1);
        if (r2 <= g->r) tz_help(t, r2, b2, 8, d >> 1);
      }
      if (bottom <= g->b) tz_help(t, sx, bottom, 7, d);
    }
  } else {
    if (inside) {
      tz_help(t, sx, top, 0, d);
      tz_help(t, left, sy, 0, d);
      tz_help(t, right, sy, 0, d);
      tz_help(t, sx, bottom, 0, d);
      for (int i = 1; i < 4; i++) {
        int yt = top + ((d >> 2) * i), yb = bottom - ((d >> 2) * i);
        int xl = sx - ((d >> 2) * i), xr = sx + ((d >> 2) * i);
        tz_help(t, xl, yt, 0, d);
        tz_help(t, xr, yt, 0, d);
        tz_help(t, xl, yb, 0, d);
        tz_help(t, xr, yb, 0, d);
      }
    } else {
      if (top >= g->t) tz_help(t, sx, top, 0, d);
      if (left >= g->l) tz_help(t, left, sy, 0, d);
      if (right <= g->r) tz_help(t, right, sy, 0, d);
      if (bottom <= g->b) tz_help(t, sx, bottom, 0, d);
      for (int i = 1; i < 4; i++) {
        int yt = top + ((d >> 2) * i), yb = bottom - ((d >> 2) * i);
        int xl = sx - ((d >> 2) * i), xr = sx + ((d >> 2) * i);
        if (yt >= g->t) {
          if (xl >= g->l) tz_help(t, xl, yt, 0, d);
          if (xr <= g->r) tz_help(t, xr, yt, 0, d);
        }
        if (yb <= g->b) {
          if (xl >= g->l) tz_help(t, xl, yb, 0, d);
          if (xr <= g->r) tz_help(t, xr, yb, 0, d);
        }
      }
    }
  }
}

/* TComDataCU::clipMv (TComDataCU.cpp:2788), MV in quarter-pel, stored as Short */
static void clip_mv(const hvx_me_job *j, int *mx, int *my) {
  int hmax = (j->pic_w + 8 - j->cu_x - 1) << 2, hmin = (-j->max_cu - 8 - j->cu_x + 1) << 2;
  int vmax = (j->pic_h + 8 - j->cu_y - 1) << 2, vmin = (-j->max_cu - 8 - j->cu_y + 1) << 2;
  *mx = (int16_t)(*mx < hmin ? hmin : *mx > hmax ? hmax : *mx);
  *my = (int16_t)(*my < vmin ? vmin : *my > vmax ? vmax : *my);
}

/* xSetSearchRange (:3765); returns integer-pel bounds */
static void set_search_range(const hvx_me_job *j, int px, int py, int sr, srch_rng *g) {
  int cx = px, cy = py;
  clip_mv(j, &cx, &cy);
  int lx = cx - (sr << 2), ly = cy - (sr << 2), rx = cx + (sr << 2), ry = cy + (sr << 2);
  clip_mv(j, &lx, &ly);
  clip_mv(j, &rx, &ry);
  g->l = lx >> 2; g->t = ly >> 2; g->r = rx >> 2; g->b = ry >> 2;
}

/* xTZSearch (:3881) with TZ_SEARCH_CONFIGURATION (:297-313) */
static void tz_search(tz_state *t, const hvx_me_job *j, const srch_rng *g0, int *mvx, int *mvy, uint32_t *sad) {
  const int sr = j->search_range;
  srch_rng g = *g0;          /* raster range (re-centred when a 2Nx2N integer MV is given) */
  int mx = *mvx, my = *mvy;
  clip_mv(j, &mx, &my);
  mx >>= 2; my >>= 2;
  t->best_sad = 0xFFFFFFFFu;
  t->best_x = t->best_y = 0; t->best_dist = 0; t->best_round = 0; t->point_nr = 0;
  tz_help(t, mx, my, 0, 0);
  tz_help(t, 0, 0, 0, 0);    /* bTestZeroVector */
  if (j->use_int2nx2n) {
    int ix = j->i2_x << 2, iy = j->i2_y << 2;
    clip_mv(j, &ix, &iy);
    ix >>= 2; iy >>= 2;
    tz_help(t, ix, iy, 0, 0);
    set_search_range(j, t->best_x << 2, t->best_y << 2, sr, &g);
  }
  int sx = t->best_x, sy = t->best_y;
  for (int d = 1; d <= sr; d *= 2) {
    tz_diamond(t, g0, sx, sy, d);
    if ((j->flags & HVX_ME_SMOOTHMV) && t->best_round >= 3) break;
  }
  if (t->best_dist == 1) { t->best_dist = 0; tz_2point(t, g0); }
  if (t->best_dist > 5) {
    t->best_dist = 5;
    for (sy = g.t; sy <= g.b; sy += 5)
      for (sx = g.l; sx <= g.r; sx += 5) tz_help(t, sx, sy, 0, 5);
  }
  while (t->best_dist > 0) {  /* star refinement */
    sx = t->best_x; sy = t->best_y;
    t->best_dist = 0; t->point_nr = 0;
    for (int d = 1; d < sr + 1; d *= 2) tz_diamond(t, g0, sx, sy, d);
    if (t->best_dist == 1) {
      t->best_dist = 0;
      if (t->point_nr != 0) tz_2point(t, g0);
    }
  }
  *mvx = t->best_x; *mvy = t->best_y;
  *sad = t->best_sad - mv_cost(t, t->best_x, t->best_y);
}

/* xPatternRefinement (:808) over interpolated candidates: iFrac 2 (half) or 1 (quarter).
 * base_q: quarter-pel position of the refinement centre relative to the PU at MV 0. */
static uint32_t pattern_refine(tz_state *t, int use_had, int base_qx, int base_qy, int frac, int *fx, int *fy) {
  static const int kRefH[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, 0}, {1, 0}, {-1, -1}, {1, -1}, {-1, 1}, {1, 1}};
  static const int kRefQ[9][2] = {{0, 0}, {0, -1}, {0, 1}, {-1, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {1, 1}};
  const int (*ref)[2] = frac == 2 ? kRefH : kRefQ;
  uint32_t best = 0xFFFFFFFFu;
  int bi = 0;
  int16_t org[64 * 64], blk[64 * 64];
  for (int y = 0; y < t->h; y++)
    for (int x = 0; x < t->w; x++) org[y * 64 + x] = t->org16 ? t->org16[y * t->so + x] : t->org[y * t->so + x];
  for (int i = 0; i < 9; i++) {
    int qx = base_qx + ref[i][0] * frac, qy = base_qy + ref[i][1] * frac;
    hvxo_luma_block_qpel(t->ref, t->sr, 0, 0, qx, qy, t->w, t->h, blk, 64);
    uint32_t d = use_had ? hvxo_satd(org, 64, blk, 64, t->w, t->h) : hvxo_sad_me(org, 64, blk, 64, t->w, t->h, 0);
    d += mv_cost(t, ref[i][0] + *fx, ref[i][1] + *fy);
    if (d < best) { best = d; bi = i; }
  }
  *fx = ref[bi][0];
  *fy = ref[bi][1];
  return best;
}

void hvxo_motion_estimation(const uint8_t *cur, int cur_stride, const uint8_t *refp, int ref_stride,
                            const hvx_me_job *j, hvx_me_result *r) {
  tz_state t;
  t.org16 = NULL;
  t.org = cur + j->pu_y * cur_stride + j->pu_x; t.so = cur_stride;
  t.ref = refp + j->pu_y * ref_stride + j->pu_x; t.sr = ref_stride;
  t.w = j->w; t.h = j->h;
  t.sub = ((j->flags & HVX_ME_FEN) && j->h > 8) ? 1 : 0;
  t.lam = j->lambda_motion;
  t.px = j->pred_x; t.py = j->pred_y;
  srch_rng g;
  set_search_range(j, j->pred_x, j->pred_y, j->search_range, &g);
  t.cost_scale = 2;
  int mvx = j->pred_x, mvy = j->pred_y;
  uint32_t sad;
  tz_search(&t, j, &g, &mvx, &mvy, &sad);
  r->mv_int_x = mvx; r->mv_int_y = mvy; r->sad_int = sad;
  /* xPatternSearchFracDIF (:4240) */
  const int had = (j->flags & HVX_ME_HADME) != 0;
  t.cost_scale = 1;
  int hx = mvx << 1, hy = mvy << 1;
  uint32_t cost = pattern_refine(&t, had, mvx << 2, mvy << 2, 2, &hx, &hy);
  t.cost_scale = 0;
  int qx = ((mvx << 1) + hx) << 1, qy = ((mvy << 1) + hy) << 1;
  cost = pattern_refine(&t, had, (mvx << 2) + (hx << 1), (mvy << 2) + (hy << 1), 1, &qx, &qy);
  r->half_x = hx; r->half_y = hy; r->qtr_x = qx; r->qtr_y = qy; r->cost_frac = cost;
  int fmx = (mvx << 2) + (hx << 1) + qx, fmy = (mvy << 2) + (hy << 1) + qy;
  uint32_t mv_bits = hvxo_eg_bits(fmx - t.px) + hvxo_eg_bits(fmy - t.py);
  uint32_t bits = (uint32_t)j->bits_in + mv_bits;
  r->mv_x = fmx; r->mv_y = fmy; r->bits = bits;
  r->cost = (uint32_t)(floor(1.0 * ((double)cost - (double)((t.lam * mv_bits) >> 16))) + (double)((t.lam * bits) >> 16));
}

/* ============================================================================================
 * SSIM metric: stvssim_src/stvssimrdo2_att/lencod/src/stvssim.c
 * ========================================================================================== */
/* compute_SSIM (:491-566), _SSIM_WEIGHTED_ 0: uniform weights 1/wint^2 */
float hvxo_ssim(const uint8_t *org, int so, const uint8_t *rec, int sr, int w, int h, int wint, int overlap) {
  const float K1 = 0.01f, K2 = 0.03f;
  float maxsq = (float)(255 * 255);
  float C1 = K1 * K1 * maxsq, C2 = K2 * K2 * maxsq;
  float win_pixels = (float)(wint * wint);
  float dist = 0.0f;
  int cnt = 0;
  for (int j = 0; j <= h - wint; j += overlap)
    for (int i = 0; i <= w - wint; i += overlap) {
      float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
      for (int n = j; n < j + wint; n++)
        for (int m = i; m < i + wint; m++) {
          float wgt = 1.0f / win_pixels;
          int po = org[n * so + m], pe = rec[n * sr + m];
          mo += wgt * po; me += wgt * pe;
          vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
        }
      float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
      float s = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
      s /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
      dist += s;
      cnt++;
    }
  dist /= (float)cnt;
  if (dist >= 1.0 && dist < 1.01) dist = 1.0f;
  return dist;
}

/* orientation filters (:116-334): weight wa on the oriented line, wb elsewhere */
static float orient_w(int k, int beta, int y, int x, float wa, float wb) {
  if (wa < 0) wa = 1.0f;
  if (wb < 0) wb = 1.0f;
  if (wa < wb) { float c = wb; wb = wa; wa = c; }
  int on;
  if (beta == 4) {
    switch (k) {
      case 0: on = x == beta / 2 - 1; break;          /* hFilter_4 */
      case 1: on = x + y == beta - 1; break;          /* rFilter_4 */
      case 2: on = y == beta / 2 - 1; break;          /* vFilter_4 */
      default: on = x == y; break;                    /* lFilter_4 */
    }
  } else {
    switch (k) {
      case 0: on = x >= beta / 2 - 1 && x <= beta / 2 + 1; break;        /* hFilter */
      case 1: on = x + y - beta >= -2 && x + y - beta <= 0; break;       /* rFilter */
      case 2: on = y >= beta / 2 - 1 && y <= beta / 2 + 1; break;        /* vFilter */
      default: on = abs(x - y) <= 1; break;                              /* lFilter */
    }
  }
  return on ? wa : wb;
}

/* calOrit (:336) */
static void cal_orit(float o, short *orit) {
  static const float orient[4] = {0, 3.1415926f / 4, 3.1415926f / 2, 3.1415926f * 3 / 4};
  float dn[4], dx = 10000.0f;
  for (int k = 0; k < 4; k++) {
    dn[k] = (float)fabs(o - orient[k]);
    if (dn[k] < dx) dx = dn[k];
  }
  for (int k = 0; k < 4; k++)
    if (fabs(dx - dn[k]) < 0.01f) orit[k]++;
}

/* compute_stVSSIM (:587-830).  org_hist[o] / rec_hist[o] for o < frameused-1 are the history
 * frames (refPicsData / srcPicsData); the current frame is org_hist[frameused-1]. */
float hvxo_stvssim(const uint8_t *const *org_hist, const uint8_t *const *rec_hist, int hs, const float *dirs,
                   int ds, int w, int h, int wint, int overlap, int gama, int comp, float *ssim, float *ssim3d,
                   float *stvssim) {
  const float K1 = 0.01f, K2 = 0.03f;
  const int used = gama < 26 ? gama : 26;
  const int uv = comp > 0 ? 2 : 1;
  float wa = 0.6f, wb = 1.0f - wa, wgta[4], wgtb[4];
  if (wint == 4) {
    wgta[0] = wgta[2] = wgta[1] = wgta[3] = wa / (wint * (used));
    wgtb[0] = wgtb[2] = wgtb[1] = wgtb[3] = wb / ((wint * wint - wint) * (used));
  } else {
    wgta[0] = wgta[2] = wa / (3 * wint * (used));
    wgta[1] = wgta[3] = wa / ((3 * wint - 2) * (used));
    wgtb[0] = wgtb[2] = wb / ((wint * wint - 3 * wint) * (used));
    wgtb[1] = wgtb[3] = wb / ((wint * wint - 3 * wint + 2) * (used));
  }
  float maxsq = (float)(255 * 255);
  float C1 = K1 * K1 * maxsq, C2 = K2 * K2 * maxsq;
  float s3x = 0, sx = 0, stx = 0;
  int cnt = 0;
  for (int j = 0; j <= h - wint; j += overlap)
    for (int i = 0; i <= w - wint; i += overlap) {
      float s3[4];
      for (int k = 0; k < 4; k++) {
        float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
        for (int o = 0; o < used; o++) {
          const uint8_t *ro = o != used - 1 ? org_hist[o] : org_hist[used - 1];
          const uint8_t *re = o != used - 1 ? rec_hist[o] : rec_hist[used - 1];
          for (int n = j; n < j + wint; n++)
            for (int m = i; m < i + wint; m++) {
              float wgt = orient_w(k, wint, n - j, m - i, wgta[k], wgtb[k]);
              int po = ro[n * hs + m], pe = re[n * hs + m];
              mo += wgt * po; me += wgt * pe;
              vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
            }
        }
        float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
        float s = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
        s /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
        s3[k] = s;
        if (s3[k] >= 1.0 && s3[k] < 1.01) s3[k] = 1.0f;
      }
      short orit[4] = {0, 0, 0, 0};
      for (int n = j; n < j + wint; n++)
        for (int m = i; m < i + wint; m++) cal_orit(dirs[(n * uv) * ds + m * uv], orit);
      short tmp = 0, inx = 0;
      for (int n = 0; n < 4; n++)
        if (orit[n] > tmp) { tmp = orit[n]; inx = (short)n; }
      int n;
      for (n = 0; n < 4; ++n)
        if ((tmp - orit[n]) < 10 && inx != n) break;
      float t3;
      if (n == 4) { s3x += s3[inx]; t3 = s3[inx]; }
      else { s3x += (s3[inx] + s3[n]) / 2; t3 = (s3[inx] + s3[n]) / 2; }
      /* plain SSIM on the current frame */
      const uint8_t *ro = org_hist[used - 1], *re = rec_hist[used - 1];
      float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
      float wgt = 1.0f / (wint * wint);
      for (int nn = j; nn < j + wint; nn++)
        for (int m = i; m < i + wint; m++) {
          int po = ro[nn * hs + m], pe = re[nn * hs + m];
          mo += wgt * po; me += wgt * pe;
          vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
        }
      float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
      float s = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
      s /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
      sx += s;
      stx += s * t3;
      cnt++;
    }
  s3x /= (float)cnt;
  sx /= (float)cnt;
  stx /= (float)cnt;
  float ret = sx * s3x;
  if (stx >= 1.0 && stx < 1.01) stx = 1.0f;
  *ssim = sx; *ssim3d = s3x; *stvssim = stx;
  return ret;
}

/* lambda_2 (:1782-1806, active expression :1805) */
double hvxo_lambda_2(int qp) {
  double a1 = 5.883060266548170e-03, b2 = -2.229472265847692e-02, b1 = 9.279543980380707e-02;
  return -a1 * b2 * exp(b1 * (qp - 15));
}

/* adjust_lambda (:1565, active _ADJUST_L2_ body :1707) */
double hvxo_adjust_lambda(double lambda, double eta) { return lambda * pow(eta, 0.85); }

/* ============================================================================================
 * estBit: TLibEncoder/TEncSbac.cpp:1726-1950 (estCBFBit :1751, estSignificantCoeffGroupMapBit
 * :1778, estSignificantMapBit :1797, estLastSignificantPositionBit :1860,
 * estSignificantCoefficientsBit :1920); context buffer order = the TEncSbac constructor;
 * significanceMapContextSetStart/Size ContextTables.h:85-86;
 * getLastSignificantContextParameters TComChromaFormat.h:211.
 * ========================================================================================== */
static int ctx_bits(const uint8_t *states, const int32_t *eb, int ctx, int val) {
  return eb[states[ctx] ^ val]; /* ContextModel::getEntropyBits, ContextModel.h:79 */
}

void hvxo_estbits_update(const uint8_t *states, const int32_t *eb, const uint32_t *rice, int w, int h, int ch,
                         hvx_estbits *e) {
  /* context buffer offsets: split 3, skip 3, merge flag 1, merge idx 1, part size 4, pred mode 1,
   * intra 1, chroma 2, dqp 3, inter dir 5, ref 2, mvd 2 -> qt cbf at 28 (10), subdiv 3, root cbf
   * at 41 (1), sig CG at 42 (2x2), sig at 46 (44), last X at 90 (2x15), last Y at 120, one at
   * 150 (24), abs at 174 (6) */
  static const int start[2][4] = {{0, 9, 21, 27}, {0, 9, 12, 15}};
  static const int size[2][4] = {{9, 12, 6, 1}, {9, 3, 3, 1}};
  int i, b, k;
  for (i = 0; i < 10; i++)
    for (b = 0; b < 2; b++) e->blockCbpBits[i][b] = ctx_bits(states, eb, 28 + i, b);
  for (i = 0; i < 4; i++) /* the reference's loop runs to 4 over a 1-model buffer: models 41..44 */
    for (b = 0; b < 2; b++) e->blockRootCbpBits[i][b] = ctx_bits(states, eb, 41 + i, b);
  for (i = 0; i < 2; i++)
    for (b = 0; b < 2; b++) e->significantCoeffGroupBits[i][b] = ctx_bits(states, eb, 42 + ch * 2 + i, b);
  {
    const int type = (w == 4 && h == 4) ? 0 : (w == 8 && h == 8) ? 1 : 2;
    const int first = start[ch][type], num = size[ch][type], off = ch ? 28 : 0;
    if (first > 0)
      for (b = 0; b < 2; b++) e->significantBits[off][b] = ctx_bits(states, eb, 46 + off, b);
    for (b = 0; b < 2; b++) e->significantBits[off + start[ch][3]][b] = ctx_bits(states, eb, 46 + off + start[ch][3], b);
    for (k = first; k < first + num; k++)
      for (b = 0; b < 2; b++) e->significantBits[off + k][b] = ctx_bits(states, eb, 46 + off + k, b);
  }
  {
    static const int group[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                  8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9}; /* g_uiGroupIdx */
    const int cw = (w == 4 ? 0 : w == 8 ? 1 : w == 16 ? 2 : 3), chh = (h == 4 ? 0 : h == 8 ? 1 : h == 16 ? 2 : 3);
    const int ox = ch ? 0 : cw * 3 + ((cw + 1) >> 2), oy = ch ? 0 : chh * 3 + ((chh + 1) >> 2);
    const int sx = ch ? cw : (cw + 3) >> 2, sy = ch ? chh : (chh + 3) >> 2;
    int bits = 0, c;
    for (c = 0; c < group[w - 1]; c++) {
      const int m = 90 + ch * 15 + ox + (c >> sx);
      e->lastXBits[ch][c] = bits + ctx_bits(states, eb, m, 0);
      bits += ctx_bits(states, eb, m, 1);
    }
    e->lastXBits[ch][c] = bits;
    bits = 0;
    for (c = 0; c < group[h - 1]; c++) {
      const int m = 120 + ch * 15 + oy + (c >> sy);
      e->lastYBits[ch][c] = bits + ctx_bits(states, eb, m, 0);
      bits += ctx_bits(states, eb, m, 1);
    }
    e->lastYBits[ch][c] = bits;
  }
  for (i = (ch ? 16 : 0); i < (ch ? 24 : 16); i++)
    for (b = 0; b < 2; b++) e->greaterOneBits[i][b] = ctx_bits(states, eb, 150 + i, b);
  for (i = (ch ? 4 : 0); i < (ch ? 6 : 4); i++)
    for (b = 0; b < 2; b++) e->levelAbsBits[i][b] = ctx_bits(states, eb, 174 + i, b);
  for (i = 0; i < 4; i++) e->golombRiceAdaptationStatistics[i] = (int32_t)rice[i];
}


/* ============================================================================================
 * Coefficient rate: TEncSbac::codeCoeffNxN (TEncSbac.cpp:1181-1540) with codeTransformSkipFlags
 * (:997), codeLastSignificantXY (:1115), xWriteCoefRemainExGolomb (:337), counted by
 * TEncBinCABACCounter (TEncBinCoderCABACCounter.cpp:74-120): encodeBin adds
 * m_entropyBits[state ^ bin] and advances the state (ContextModel.h:79-85), bypass bins add
 * 32768 each.  State transitions are the specification's (transIdxLps; MPS: +1 up to 62).
 * Main-profile scope: no RDPCM, no CABAC bypass alignment.
 * ========================================================================================== */
static const uint8_t kTransIdxLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                         13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                         24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                         33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};
static const int kMinInGroup[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};

/* Arithmetic coder of the slice writer, TEncBinCABAC (TEncBinCoderCABAC.cpp:60-460): rangeTabLps
 * (TComCABACTables.cpp:44, the specification's Table 9-52) and the renormalisation shift table
 * (:113). */
static const uint8_t kLpsTable[64][4] = {
  {128, 176, 208, 240},
  {128, 167, 197, 227},
  {128, 158, 187, 216},
  {123, 150, 178, 205},
  {116, 142, 169, 195},
  {111, 135, 160, 185},
  {105, 128, 152, 175},
  {100, 122, 144, 166},
  { 95, 116, 137, 158},
  { 90, 110, 130, 150},
  { 85, 104, 123, 142},
  { 81,  99, 117, 135},
  { 77,  94, 111, 128},
  { 73,  89, 105, 122},
  { 69,  85, 100, 116},
  { 66,  80,  95, 110},
  { 62,  76,  90, 104},
  { 59,  72,  86,  99},
  { 56,  69,  81,  94},
  { 53,  65,  77,  89},
  { 51,  62,  73,  85},
  { 48,  59,  69,  80},
  { 46,  56,  66,  76},
  { 43,  53,  63,  72},
  { 41,  50,  59,  69},
  { 39,  48,  56,  65},
  { 37,  45,  54,  62},
  { 35,  43,  51,  59},
  { 33,  41,  48,  56},
  { 32,  39,  46,  53},
  { 30,  37,  43,  50},
  { 29,  35,  41,  48},
  { 27,  33,  39,  45},
  { 26,  31,  37,  43},
  { 24,  30,  35,  41},
  { 23,  28,  33,  39},
  { 22,  27,  32,  37},
  { 21,  26,  30,  35},
  { 20,  24,  29,  33},
  { 19,  23,  27,  31},
  { 18,  22,  26,  30},
  { 17,  21,  25,  28},
  { 16,  20,  23,  27},
  { 15,  19,  22,  25},
  { 14,  18,  21,  24},
  { 14,  17,  20,  23},
  { 13,  16,  19,  22},
  { 12,  15,  18,  21},
  { 12,  14,  17,  20},
  { 11,  14,  16,  19},
  { 11,  13,  15,  18},
  { 10,  12,  15,  17},
  { 10,  12,  14,  16},
  {  9,  11,  13,  15},
  {  9,  11,  12,  14},
  {  8,  10,  12,  14},
  {  8,   9,  11,  13},
  {  7,   9,  11,  12},
  {  7,   9,  10,  12},
  {  7,   8,  10,  11},
  {  6,   8,   9,  11},
  {  6,   7,   9,  10},
  {  6,   7,   8,   9},
  {  2,   2,   2,   2}};
static const uint8_t kRenormTable[32] = {6, 5, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

/* One coder for both bin sinks: w == NULL counts like TEncBinCABACCounter, otherwise the bins
 * drive TEncBinCABAC's registers *w and the bytes go to out[0..cap) (nout counts every byte,
 * also past cap). */
typedef struct {
  uint8_t *st;
  const int32_t *eb;
  uint64_t frac;
  hvx_cabac_regs *w;
  uint8_t *out;
  int nout, cap;
} cab_counter;

static void cab_put(cab_counter *c, uint32_t byte) {
  if (c->nout < c->cap) c->out[c->nout] = (uint8_t)byte;
  c->nout++;
}
/* TEncBinCABAC::writeOut (:425) / testAndWriteOut (:417) */
static void cab_write_out(cab_counter *c) {
  hvx_cabac_regs *r = c->w;
  const uint32_t lead = r->low >> (24 - r->bits_left);
  r->bits_left += 8;
  r->low &= 0xffffffffu >> r->bits_left;
  if (lead == 0xff) {
    r->num_buffered++;
  } else if (r->num_buffered > 0) {
    const uint32_t carry = lead >> 8;
    cab_put(c, r->buffered_byte + carry);
    r->buffered_byte = lead & 0xff;
    const uint32_t fill = (0xff + carry) & 0xff;
    while (r->num_buffered > 1) {
      cab_put(c, fill);
      r->num_buffered--;
    }
  } else {
    r->num_buffered = 1;
    r->buffered_byte = lead;
  }
}
static void cab_test(cab_counter *c) {
  if (c->w->bits_left < 12) cab_write_out(c);
}

/* encodeBin (:200) or TEncBinCABACCounter::encodeBin, then ContextModel::update */
static void cab_bin(cab_counter *c, int ctx, int v) {
  const int s = c->st[ctx], p = s >> 1, mps = s & 1;
  if (c->w) {
    hvx_cabac_regs *r = c->w;
    r->bins++;
    if (ctx >= 42 && ctx < 202) r->coded[(ctx - 42) >> 5] |= 1u << ((ctx - 42) & 31);
    const uint32_t lps = kLpsTable[p][(r->range >> 6) & 3];
    r->range -= lps;
    if (v != mps) {
      const int nb = kRenormTable[lps >> 3];
      r->low = (r->low + r->range) << nb;
      r->range = lps << nb;
      r->bits_left -= nb;
      cab_test(c);
    } else if (r->range < 256) {
      r->low <<= 1;
      r->range <<= 1;
      r->bits_left--;
      cab_test(c);
    }
  } else {
    c->frac += (uint32_t)c->eb[s ^ v];
  }
  if (v == mps) c->st[ctx] = (uint8_t)(((p < 62 ? p + 1 : p) << 1) | mps);
  else c->st[ctx] = (uint8_t)((kTransIdxLps[p] << 1) | (p == 0 ? mps ^ 1 : mps));
}
/* encodeAlignedBinsEP (:334): only reachable with range == 256 (cabac_bypass_alignment) */
static void cab_aligned_eps(cab_counter *c, uint32_t vals, int n) {
  hvx_cabac_regs *r = c->w;
  while (n > 0) {
    const int k = n < 8 ? n : 8;
    const uint32_t bins = (vals >> (n - k)) & ((1u << k) - 1);
    r->low = (r->low << k) + (bins << 8);
    n -= k;
    r->bits_left -= k;
    cab_test(c);
  }
}
/* encodeBinEP (:262): one bypass bin */
static void cab_ep1(cab_counter *c, uint32_t bin) {
  if (!c->w) { c->frac += 32768u; return; }
  hvx_cabac_regs *r = c->w;
  r->bins++;
  if (r->range == 256) { cab_aligned_eps(c, bin, 1); return; }
  r->low <<= 1;
  if (bin) r->low += r->range;
  r->bits_left--;
  cab_test(c);
}
/* encodeBinsEP (:290): n bypass bins, most significant first, in pieces of 8 */
static void cab_eps(cab_counter *c, uint32_t vals, int n) {
  if (!c->w) { c->frac += 32768u * (uint32_t)n; return; }
  hvx_cabac_regs *r = c->w;
  r->bins += (uint32_t)n;
  if (r->range == 256) { cab_aligned_eps(c, vals, n); return; }
  while (n > 8) {
    n -= 8;
    const uint32_t pat = vals >> n;
    r->low <<= 8;
    r->low += r->range * pat;
    vals -= pat << n;
    r->bits_left -= 8;
    cab_test(c);
  }
  r->low <<= n;
  r->low += r->range * vals;
  r->bits_left -= n;
  cab_test(c);
}

/* xWriteCoefRemainExGolomb (TEncSbac.cpp:337): the escape code of one level (COEF_REMAIN_BIN_REDUCTION 3) */
static void cab_escape(cab_counter *c, uint32_t symbol, int r, int limited, int max_log2) {
  if (symbol < (3u << r)) {
    const uint32_t len = symbol >> r;
    cab_eps(c, (1u << (len + 1)) - 2, (int)len + 1);
    cab_eps(c, symbol % (1u << r), r);
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
    cab_eps(c, (1u << tot) - 1, (int)tot);
    cab_eps(c, (suffix << r) | (symbol & ((1u << r) - 1)), (int)(suffix_len + r));
  } else {
    int len = r;
    uint32_t cn = symbol - (3u << r);
    while (cn >= (1u << len)) cn -= (1u << (len++));
    cab_eps(c, (1u << (3 + len + 1 - r)) - 2, 3 + len + 1 - r);
    cab_eps(c, cn, len);
  }
}

static int log2_4_32(int n) { return n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : 5; }

static void coeff_code(const hvx_tu_desc *tu, const int32_t *coef, cab_counter *cc, hvx_coeff_bits *out) {
  const int w = tu->width, h = tu->height, lw = log2_4_32(w), lh = log2_4_32(h), n = w * h;
  const int ch = tu->comp ? 1 : 0;
  cab_counter c = *cc;
  uint32_t rice_stat = (uint32_t)tu->golomb_rice_stat;
  int num_sig = 0, i;
  for (i = 0; i < n; i++) num_sig += coef[i] != 0;
  out->num_sig = (uint32_t)num_sig;
  if (num_sig == 0) { /* the reference exits (1) here; nothing is coded */
    out->frac_bits = 0;
    out->rice_stat = rice_stat;
    return;
  }
  const int be_valid = tu->transquant_bypass ? 0 : tu->sign_hiding;
  /* codeTransformSkipFlags (:997): TUCompRectHasAssociatedTransformSkipFlag, log2 max 2 */
  if (tu->pps_tskip && !tu->transquant_bypass && w <= 4) cab_bin(&c, 183 + ch, tu->transform_skip ? 1 : 0);
  coding_params cp;
  get_coding_params(tu, &cp);
  uint32_t cg_flags[64];
  memset(cg_flags, 0, sizeof(cg_flags));
  int scan_last = -1, pos_last = 0, left = num_sig;
  do {
    pos_last = (int)cp.scan[++scan_last];
    if (coef[pos_last]) {
      const int py = pos_last >> lw, px = pos_last - (py << lw);
      cg_flags[cp.wg * (py >> 2) + (px >> 2)] = 1;
      left--;
    }
  } while (left > 0);
  /* codeLastSignificantXY (:1115) */
  {
    int py = pos_last >> lw, px = pos_last - (py << lw), bw = w, bh = h;
    if (cp.scan_type == 2) { int t = px; px = py; py = t; t = bw; bw = bh; bh = t; }
    const int gx = kGroupIdx[px], gy = kGroupIdx[py];
    const int cw = log2_4_32(bw) - 2, chh = log2_4_32(bh) - 2; /* getLastSignificantContextParameters */
    const int ox = ch ? 0 : cw * 3 + ((cw + 1) >> 2), oy = ch ? 0 : chh * 3 + ((chh + 1) >> 2);
    const int sx = ch ? cw : (cw + 3) >> 2, sy = ch ? chh : (chh + 3) >> 2;
    const int bx = 90 + ch * 15 + ox, by = 120 + ch * 15 + oy;
    int k;
    for (k = 0; k < gx; k++) cab_bin(&c, bx + (k >> sx), 1);
    if (gx < kGroupIdx[bw - 1]) cab_bin(&c, bx + (k >> sx), 0);
    for (k = 0; k < gy; k++) cab_bin(&c, by + (k >> sy), 1);
    if (gy < kGroupIdx[bh - 1]) cab_bin(&c, by + (k >> sy), 0);
    /* the fixed-length suffixes, one encodeBinEP per bit, most significant first */
    for (k = gx > 3 ? ((gx - 2) >> 1) - 1 : -1; k >= 0; k--) cab_ep1(&c, ((uint32_t)(px - kMinInGroup[gx]) >> k) & 1);
    for (k = gy > 3 ? ((gy - 2) >> 1) - 1 : -1; k >= 0; k--) cab_ep1(&c, ((uint32_t)(py - kMinInGroup[gy]) >> k) & 1);
  }
  const int base_cg = 42 + ch * 2, base_sig = 46 + (ch ? 28 : 0);
  const int last_set = scan_last >> 4;
  int c1 = 1, scan_sig = scan_last;
  for (int sub = last_set; sub >= 0; sub--) {
    int nnz = 0, sub_pos = sub << 4, last_nz = -1, first_nz = 16, escape = 0;
    int rice = (int)(rice_stat / 4);
    int upd_rice = tu->persistent_rice;
    uint32_t signs = 0;
    int absc[16];
    if (scan_sig == scan_last) {
      absc[0] = abs(coef[pos_last]);
      signs = coef[pos_last] < 0;
      nnz = 1;
      last_nz = first_nz = scan_sig;
      scan_sig--;
    }
    const int cg = (int)cp.scan_cg[sub], cgy = cg / cp.wg, cgx = cg - cgy * cp.wg;
    if (sub == last_set || sub == 0) cg_flags[cg] = 1;
    else cab_bin(&c, base_cg + sig_cg_ctx(cg_flags, cgx, cgy, cp.wg, cp.hg), cg_flags[cg] != 0);
    if (cg_flags[cg]) {
      const int pattern = pattern_sig_ctx(cg_flags, cgx, cgy, cp.wg, cp.hg);
      for (; scan_sig >= sub_pos; scan_sig--) {
        const int blk = (int)cp.scan[scan_sig], sig = coef[blk] != 0;
        if (scan_sig > sub_pos || sub == 0 || nnz) cab_bin(&c, base_sig + sig_ctx_inc(pattern, &cp, scan_sig, lw, lh, ch), sig);
        if (sig) {
          absc[nnz] = abs(coef[blk]);
          signs = 2 * signs + (coef[blk] < 0);
          nnz++;
          if (last_nz == -1) last_nz = scan_sig;
          first_nz = scan_sig;
        }
      }
    } else {
      scan_sig = sub_pos - 1;
    }
    if (nnz > 0) {
      const int hidden = (last_nz - first_nz) >= 4; /* SBH_THRESHOLD */
      const int set = ctx_set_index(tu->comp, sub, c1 == 0);
      c1 = 1;
      const int base_one = 150 + 4 * set;
      const int nc1 = nnz < 8 ? nnz : 8;
      int first_c2 = -1;
      for (int k = 0; k < nc1; k++) {
        const int gt1 = absc[k] > 1;
        cab_bin(&c, base_one + c1, gt1);
        if (gt1) {
          c1 = 0;
          if (first_c2 == -1) first_c2 = k;
          else escape = 1;
        } else if (c1 < 3 && c1 > 0) {
          c1++;
        }
      }
      if (c1 == 0 && first_c2 != -1) {
        const int gt2 = absc[first_c2] > 2;
        cab_bin(&c, 174 + set, gt2);
        if (gt2) escape = 1;
      }
      escape = escape || nnz > 8;
      if (be_valid && hidden) cab_eps(&c, signs >> 1, nnz - 1); /* the first coefficient's sign is hidden */
      else cab_eps(&c, signs, nnz);
      if (escape) {
        int first2 = 1;
        for (int k = 0; k < nnz; k++) {
          const int base = k < 8 ? 2 + first2 : 1;
          if (absc[k] >= base) {
            const uint32_t esc = (uint32_t)(absc[k] - base);
            cab_escape(&c, esc, rice, tu->extended_precision, tu->max_log2_tr_range);
            if (absc[k] > (3 << rice)) rice = tu->persistent_rice ? rice + 1 : (rice + 1 < 4 ? rice + 1 : 4);
            if (upd_rice) {
              const uint32_t init = rice_stat / 4;
              if (esc >= (3u << init)) rice_stat++;
              else if (esc * 2 < (1u << init) && rice_stat > 0) rice_stat--;
              upd_rice = 0;
            }
          }
          if (absc[k] >= 2) first2 = 0;
        }
      }
    }
  }
  out->frac_bits = c.frac;
  out->rice_stat = rice_stat;
  *cc = c;
}

void hvxo_coeff_bits(const hvx_tu_desc *tu, const int32_t *coef, uint8_t *states, const int32_t *eb, hvx_coeff_bits *out) {
  cab_counter c = {states, eb, 0, NULL, NULL, 0, 0};
  coeff_code(tu, coef, &c, out);
}

/* TEncSbac::codeCoeffNxN through the real arithmetic coder TEncBinCABAC: the same syntax and
 * context evolution as hvxo_coeff_bits, the bins driving the registers *regs; the bytes the call
 * completes go to out.  Returns the byte count (-1 past cap).  Main-profile scope as above (no
 * cabac_bypass_alignment: the aligned path is restated but only reached with range 256). */
int hvxo_coeff_write(const hvx_tu_desc *tu, const int32_t *coef, uint8_t *states, hvx_cabac_regs *regs, uint8_t *out,
                     int cap) {
  cab_counter c = {states, NULL, 0, regs, out, 0, cap};
  hvx_coeff_bits o;
  coeff_code(tu, coef, &c, &o);
  return c.nout <= cap ? c.nout : -1;
}

/* ============================================================================================
 * Motion compensation: TComPrediction.cpp:517-722, TComYuv.cpp:352 (8-bit, 4:2:0, no WP)
 * ========================================================================================== */
/* TComYuv::addAvg: shiftNum = max(2, IF_INTERNAL_PREC - 8) + 1 = 7,
 * offset = (1 << 6) + 2 * IF_INTERNAL_OFFS, ClipBD */
void hvxo_add_avg(const int16_t *a, const int16_t *b, int16_t *dst, int n) {
  for (int i = 0; i < n; i++) dst[i] = clip_pel((a[i] + b[i] + (1 << 6) + 2 * IF_OFFS) >> 7);
}

/* xPredInterBlk (:668-706) for one component of the PU at component position (x, y) */
static void mc_pred_blk(int is_luma, const int16_t *plane, int stride, int x, int y, int mvx, int mvy, int w, int h,
                        int bi, int16_t *dst) {
  const int sh = is_luma ? 2 : 3; /* shiftHor/Ver = 2 + component scale (4:2:0 chroma: 1) */
  const int xf = mvx & ((1 << sh) - 1), yf = mvy & ((1 << sh) - 1);
  const int16_t *ref = plane + (y + (mvy >> sh)) * stride + x + (mvx >> sh);
  if (yf == 0) {
    hvxo_filter_hor(is_luma, ref, stride, dst, w, w, h, xf, !bi);
  } else if (xf == 0) {
    hvxo_filter_ver(is_luma, ref, stride, dst, w, w, h, yf, 1, !bi);
  } else {
    static _Thread_local int16_t tmp[(64 + 7) * 64]; /* per thread: bench.py's cpu_baseline runs CTUs on threads */
    const int n = is_luma ? 8 : 4;
    hvxo_filter_hor(is_luma, ref - (n / 2 - 1) * stride, stride, tmp, w, w, h + n - 1, xf, 0);
    hvxo_filter_ver(is_luma, tmp + (n / 2 - 1) * w, w, dst, w, w, h, yf, 0, !bi);
  }
}

static void mc_clip(const hvx_mc_job *j, int *mx, int *my) { /* TComDataCU::clipMv (TComDataCU.cpp:2788) */
  const int hmax = (j->pic_w + 8 - j->cu_x - 1) << 2, hmin = (-j->max_cu - 8 - j->cu_x + 1) << 2;
  const int vmax = (j->pic_h + 8 - j->cu_y - 1) << 2, vmin = (-j->max_cu - 8 - j->cu_y + 1) << 2;
  *mx = (int16_t)(*mx < hmin ? hmin : *mx > hmax ? hmax : *mx);
  *my = (int16_t)(*my < vmin ? vmin : *my > vmax ? vmax : *my);
}

void hvxo_mc(const int16_t *const *planes, int ls, int cs, const hvx_mc_job *j, int16_t *out) {
  const int v0 = j->ref[0] >= 0, v1 = j->ref[1] >= 0;
  /* xCheckIdenticalMotion (:500): B slice without WP, same POC and same (unclipped) MV */
  const int identical = (j->flags & HVX_MC_B_SLICE) && v0 && v1 && j->poc[0] == j->poc[1] &&
                        j->mv_x[0] == j->mv_x[1] && j->mv_y[0] == j->mv_y[1];
  const int bi = v0 && v1 && !identical;
  const int lu = v0 ? 0 : 1;
  int mx[2] = {j->mv_x[0], j->mv_x[1]}, my[2] = {j->mv_y[0], j->mv_y[1]};
  mc_clip(j, &mx[0], &my[0]); /* xPredInterUni clips its list's MV */
  mc_clip(j, &mx[1], &my[1]);
  static _Thread_local int16_t pa[64 * 64], pb[64 * 64];
  for (int comp = 0; comp < 3; comp++) {
    const int luma = comp == 0;
    const int w = luma ? j->w : j->w >> 1, h = luma ? j->h : j->h >> 1;
    const int x = luma ? j->pu_x : j->pu_x >> 1, y = luma ? j->pu_y : j->pu_y >> 1;
    const int stride = luma ? ls : cs;
    int16_t *o = out + (comp == 0 ? 0 : comp == 1 ? j->w * j->h : j->w * j->h + w * h);
    if (bi) { /* xPredInterBi: both lists as 14-bit intermediates, then xWeightedAverage -> addAvg */
      mc_pred_blk(luma, planes[3 * j->ref[0] + comp], stride, x, y, mx[0], my[0], w, h, 1, pa);
      mc_pred_blk(luma, planes[3 * j->ref[1] + comp], stride, x, y, mx[1], my[1], w, h, 1, pb);
      hvxo_add_avg(pa, pb, o, w * h);
    } else {
      mc_pred_blk(luma, planes[3 * j->ref[lu] + comp], stride, x, y, mx[lu], my[lu], w, h, 0, o);
    }
  }
}


/* xMotionEstimation with the integer full search (TEncSearch.cpp:3663-3760, FastSearch=0 or
 * bBi): xSetSearchRange around (center_x, center_y) (:3765), xPatternSearch (:3786; FEN
 * subsampling when rows > 8 :3810, strict '<' in raster order), xPatternSearchFracDIF, and the
 * final cost with fWeight 0.5 for bBi (:3696, :3759).  tgt: int16 pattern plane (sample 0,0). */
void hvxo_me_full(const int16_t *tgt, int tstride, const uint8_t *refp, int ref_stride, const hvx_me_job *j,
                  hvx_me_result *r) {
  hvxo_me_full_pat(tgt + j->pu_y * tstride + j->pu_x, tstride, refp, ref_stride, j, r);
}
/* the same with the pattern given at the PU's first sample (TComPattern over a TComYuv, e.g. the
 * bi-prediction target m_cYuvPredTemp at uiPartAddr, stride 64) */
void hvxo_me_full_pat(const int16_t *pat, int pstride, const uint8_t *refp, int ref_stride, const hvx_me_job *j,
                      hvx_me_result *r) {
  tz_state t;
  memset(&t, 0, sizeof(t));
  t.org = NULL;
  t.org16 = pat; t.so = pstride;
  t.ref = refp + j->pu_y * ref_stride + j->pu_x; t.sr = ref_stride;
  t.w = j->w; t.h = j->h;
  const int w = j->w;
  const int spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  const int sub = ((j->flags & HVX_ME_FEN) && j->h > 8 && spec) ? 1 : 0;
  t.lam = j->lambda_motion;
  t.px = j->pred_x; t.py = j->pred_y;
  srch_rng g;
  set_search_range(j, j->center_x, j->center_y, j->search_range, &g);
  t.cost_scale = 2;
  uint32_t best = 0xFFFFFFFFu;
  int bx = 0, by = 0;
  for (int y = g.t; y <= g.b; y++)
    for (int x = g.l; x <= g.r; x++) {
      const uint8_t *c = t.ref + y * ref_stride + x;
      uint32_t s = 0;
      for (int row = 0; row < t.h; row += 1 << sub)
        for (int col = 0; col < w; col++) s += (uint32_t)abs((int)t.org16[row * pstride + col] - (int)c[row * ref_stride + col]);
      s = (s << sub) + mv_cost(&t, x, y);
      if (s < best) { best = s; bx = x; by = y; }
    }
  r->mv_int_x = bx; r->mv_int_y = by; r->sad_int = best - mv_cost(&t, bx, by);
  const int had = (j->flags & HVX_ME_HADME) != 0;
  t.cost_scale = 1;
  int hx = bx << 1, hy = by << 1;
  uint32_t cost = pattern_refine(&t, had, bx << 2, by << 2, 2, &hx, &hy);
  t.cost_scale = 0;
  int qx = ((bx << 1) + hx) << 1, qy = ((by << 1) + hy) << 1;
  cost = pattern_refine(&t, had, (bx << 2) + (hx << 1), (by << 2) + (hy << 1), 1, &qx, &qy);
  r->half_x = hx; r->half_y = hy; r->qtr_x = qx; r->qtr_y = qy; r->cost_frac = cost;
  const int fmx = (bx << 2) + (hx << 1) + qx, fmy = (by << 2) + (hy << 1) + qy;
  const uint32_t mv_bits = hvxo_eg_bits(fmx - t.px) + hvxo_eg_bits(fmy - t.py);
  const uint32_t bits = (uint32_t)j->bits_in + mv_bits;
  const double wgt = (j->flags & HVX_ME_BI) ? 0.5 : 1.0;
  r->mv_x = fmx; r->mv_y = fmy; r->bits = bits;
  r->cost = (uint32_t)(floor(wgt * ((double)cost - (double)((t.lam * mv_bits) >> 16))) + (double)((t.lam * bits) >> 16));
}

/* ============================================================================================
 * Intra prediction.  Border layout B (4N+1 samples): B[0] = above-left,
 * B[1..2N] = above + above-right row left to right, B[2N+1..4N] = left + below-left column top
 * to bottom -- the row 0 / column 0 of HM's (2N+1)x(2N+1) m_piYuvExt buffer.
 * ========================================================================================== */
static int avail_bit(const uint32_t *a, int i) { return (int)((a[i >> 5] >> (i & 31)) & 1); }

/* fillReferenceSamples (TComPattern.cpp:364-540), 8-bit.  raw = reconstructed samples at the
 * border positions (read whatever their availability); the line of the reference is
 * L[0..2N) = left column bottom-up, L[2N..2N+u) = the above-left unit, L[2N+u..) = above row. */
static int line_raw(const int16_t *raw, int n, int u, int l) {
  if (l < 2 * n) return raw[2 * n + 1 + (2 * n - 1 - l)];
  if (l < 2 * n + u) return raw[0];
  return raw[1 + (l - 2 * n - u)];
}

void hvxo_intra_fill(const int16_t *raw, const uint32_t *avail, int n, int unit_log2, int16_t *B) {
  const int u = 1 << unit_log2, lu = (2 * n) >> unit_log2, nunits = 2 * lu + 1, nl = 4 * n + u;
  int16_t L[4 * 64 + 8];
  int navail = 0;
  for (int i = 0; i < nunits; i++) navail += avail_bit(avail, i);
  if (navail == 0) { /* :384-395 DC fill */
    for (int k = 0; k <= 4 * n; k++) B[k] = 128;
    return;
  }
  for (int l = 0; l < nl; l++) L[l] = 128; /* :425-429 */
  for (int i = 0; i < nunits; i++)
    if (avail_bit(avail, i))
      for (int k = 0; k < u; k++) L[i * u + k] = (int16_t)line_raw(raw, n, u, i * u + k);
  int cur = 0;
  if (!avail_bit(avail, 0)) { /* :476-506: pad the bottom run with the first available sample */
    int next = 1;
    while (next < nunits && !avail_bit(avail, next)) next++;
    const int16_t ref = L[next * u];
    for (; cur < next; cur++)
      for (int k = 0; k < u; k++) L[cur * u + k] = ref;
  }
  for (; cur < nunits; cur++) /* :508-526: every other gap takes the sample just below it */
    if (!avail_bit(avail, cur))
      for (int k = 0; k < u; k++) L[cur * u + k] = L[cur * u - 1];
  B[0] = L[2 * n + u - 1]; /* :530-539 */
  for (int i = 0; i < 2 * n; i++) B[1 + i] = L[2 * n + u + i];
  for (int j = 0; j < 2 * n; j++) B[2 * n + 1 + j] = L[2 * n - 1 - j];
}

/* the smoothing of initIntraPatternChType (TComPattern.cpp:190-330) over F = B in the order
 * bottom-left .. above-left .. above-right */
static int f_index(int n, int k) { return k < 2 * n ? 4 * n - k : k == 2 * n ? 0 : k - 2 * n; }

void hvxo_intra_filter(const int16_t *B, int n, int is_luma, int strong_enabled, int16_t *out) {
  const int bl = B[4 * n], tl = B[0], tr = B[2 * n];
  int strong = is_luma && strong_enabled;
  if (strong) { /* :214-226, threshold 1 << (8 - 5) */
    const int bil_left = abs(bl + tl - 2 * B[3 * n]) < 8, bil_above = abs(tl + tr - 2 * B[n]) < 8;
    if (n < 32 || !bil_left || !bil_above) strong = 0;
  }
  const int shift = strong ? (n == 64 ? 7 : n == 32 ? 6 : n == 16 ? 5 : n == 8 ? 4 : 3) : 0;
  for (int k = 0; k <= 4 * n; k++) {
    int v;
    if (k == 0 || k == 4 * n) v = B[f_index(n, k)];                  /* ends unfiltered */
    else if (strong && k == 2 * n) v = tl;                             /* :262 */
    else if (strong && k < 2 * n) v = ((2 * n - k) * bl + k * tl + n) >> shift;  /* :236-243 */
    else if (strong) v = ((4 * n - k) * tl + (k - 2 * n) * tr + n) >> shift;     /* :281-288 */
    else v = (B[f_index(n, k - 1)] + 2 * B[f_index(n, k)] + B[f_index(n, k + 1)] + 2) >> 2;
    out[f_index(n, k)] = (int16_t)v;
  }
}

/* TComPrediction::filteringIntraReferenceSamples (TComPattern.cpp:544-569), 4:2:0 */
int hvxo_intra_use_filter(int mode, int n, int is_luma) {
  static const int thr[5] = {10, 7, 1, 0, 10}; /* m_aucIntraFilter (TComPrediction.cpp:50) */
  if (!is_luma || mode == 1) return 0;
  int l = 0;
  while ((4 << l) < n) l++;
  const int d10 = abs(mode - 10), d26 = abs(mode - 26);
  return (d10 < d26 ? d10 : d26) > thr[l];
}

/* predIntraAng (TComPrediction.cpp:455-516) with bAbove = bLeft = true (initIntraPatternChType
 * always reports both, TComPattern.cpp:152-153) and the edge filters enabled (no RDPCM). */
void hvxo_intra_pred(const int16_t *B, int n, int is_luma, int mode, uint8_t *pred) {
  int log2n = 0;
  while ((1 << log2n) < n) log2n++;
  const int edge = is_luma && n <= 16;
#define A(i) ((int)B[1 + (i)])
#define LF(j) ((int)B[2 * n + 1 + (j)])
  if (mode == 0) { /* xPredIntraPlanar (:756) */
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++)
        pred[r * n + c] = (uint8_t)(((n - 1 - c) * LF(r) + (c + 1) * A(n) + (n - 1 - r) * A(c) + (r + 1) * LF(n) + n) >>
                                    (log2n + 1));
    return;
  }
  if (mode == 1) { /* predIntraGetPredValDC (:183) + xDCPredFiltering (:816) */
    int sum = 0;
    for (int i = 0; i < n; i++) sum += A(i) + LF(i);
    const int dc = (sum + n) / (2 * n);
    for (int r = 0; r < n; r++)
      for (int c = 0; c < n; c++) {
        int v = dc;
        if (edge && r == 0 && c == 0) v = (A(0) + LF(0) + 2 * dc + 2) >> 2;
        else if (edge && r == 0) v = (A(c) + 3 * dc + 2) >> 2;
        else if (edge && c == 0) v = (LF(r) + 3 * dc + 2) >> 2;
        pred[r * n + c] = (uint8_t)v;
      }
    return;
  }
  /* xPredIntraAng (:247-452) */
  static const int ang_table[9] = {0, 2, 5, 9, 13, 17, 21, 26, 32};
  static const int inv_table[9] = {0, 4096, 1638, 910, 630, 482, 390, 315, 256};
  const int ver = mode >= 18, am = ver ? mode - 26 : 10 - mode, aa = abs(am);
  const int angle = (am < 0 ? -1 : 1) * ang_table[aa], inv = inv_table[aa];
  int ref_above[2 * 64 + 1 + 64], ref_left[2 * 64 + 1 + 64];
  int *above = ref_above + 64, *left = ref_left + 64; /* index -64..2n */
  for (int k = 0; k <= 2 * n; k++) { above[k] = B[k]; left[k] = k ? LF(k - 1) : B[0]; }
  int *mainr = ver ? above : left, *side = ver ? left : above;
  if (angle < 0) { /* :321-329 extend the main reference with the projected side */
    int sum = 128;
    for (int k = -1; k > (n * angle) >> 5; k--) { sum += inv; mainr[k] = side[sum >> 8]; }
  }
  int tmp[64 * 64];
  for (int y = 0; y < n; y++) {
    const int dp = (y + 1) * angle, di = dp >> 5, f = dp & 31;
    for (int x = 0; x < n; x++) {
      int v;
      if (angle == 0) v = mainr[x + 1];
      else if (f) v = ((32 - f) * mainr[x + di + 1] + f * mainr[x + di + 2] + 16) >> 5;
      else v = mainr[x + di + 1];
      tmp[y * n + x] = v;
    }
    if (angle == 0 && edge) { /* :375-381 */
      int v = tmp[y * n] + ((side[y + 1] - side[0]) >> 1);
      tmp[y * n] = v < 0 ? 0 : v > 255 ? 255 : v;
    }
  }
  for (int r = 0; r < n; r++)
    for (int c = 0; c < n; c++) pred[r * n + c] = (uint8_t)(ver ? tmp[r * n + c] : tmp[c * n + r]);
#undef A
#undef LF
}

/* TComDataCU::getIntraDirPredictor (TComDataCU.cpp:1441-1478) from the two neighbour dirs;
 * returns iMode (1: left == above, 2 otherwise) */
static int intra_mpm(int ld, int ad, int *p) {
  if (ld == ad) {
    if (ld > 1) { p[0] = ld; p[1] = ((ld + 29) % 32) + 2; p[2] = ((ld - 1) % 32) + 2; }
    else { p[0] = 0; p[1] = 1; p[2] = 26; }
    return 1;
  }
  p[0] = ld; p[1] = ad;
  p[2] = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  return 2;
}

/* estIntraPredLumaQT's first pass (TEncSearch.cpp:2244-2323) for one luma PU: org = n*n
 * original samples, raw = reconstructed samples at the border positions. */
void hvxo_intra_search(const uint8_t *org, const int16_t *raw, const hvx_intra_job *j, const int32_t *eb,
                       hvx_intra_search_result *r) {
  const int n = 1 << j->log2_size;
  int16_t unf[257], filt[257];
  hvxo_intra_fill(raw, j->avail, n, j->unit_log2, unf);
  hvxo_intra_filter(unf, n, 1, (j->flags & HVX_INTRA_STRONG) != 0, filt); /* bFilterRefSamples = true (:2256) */
  memset(r, 0, sizeof(*r));
  int mpm[3];
  const int imode = intra_mpm(j->left_dir, j->above_dir, mpm);
  const int fast = (j->flags & HVX_INTRA_FAST_MPM) != 0;
  static const int num_mpm[6] = {3, 8, 8, 3, 3, 3}, num_nompm[6] = {3, 9, 9, 4, 4, 5}; /* TComRom.cpp:545-562 */
  const int widx = j->log2_size - 1; /* getIntraSizeIdx (TComDataCU.cpp:2804) */
  int num = fast ? num_mpm[widx] : num_nompm[widx];
  uint32_t list[35];
  double ccost[35];
  for (int i = 0; i < 35; i++) { list[i] = 0; ccost[i] = 1.7e308; }
  uint8_t pred[64 * 64];
  int16_t org16[64 * 64], pred16[64 * 64];
  for (int i = 0; i < n * n; i++) org16[i] = org[i];
  /* xModeBitsIntra: loadIntraDirMode copies the source coder's bin state, m_fracBits included
   * (TEncSbac.cpp:403), and resetBits keeps its low 15 bits (TEncBinCoderCABAC.cpp:172): every
   * mode counts from the same fraction */
  const uint64_t frac = (uint64_t)j->frac_bits;
  for (int m = 0; m < 35; m++) {
    hvxo_intra_pred(hvxo_intra_use_filter(m, n, 1) ? filt : unf, n, 1, m, pred);
    for (int i = 0; i < n * n; i++) pred16[i] = pred[i];
    const uint32_t satd = hvxo_satd(org16, n, pred16, n, n, n);
    /* xModeBitsIntra (:5222): TEncSbac::codeIntraDirLumaAng (TEncSbac.cpp:643) counted by
     * TEncBinCABACCounter: flag bin + 1/2 (MPM idx) or 5 bypass bins */
    int idx = -1;
    for (int i = 0; i < 3; i++)
      if (m == mpm[i]) idx = i;
    const uint64_t total = frac + (uint64_t)eb[j->ctx_state ^ (idx >= 0 ? 1 : 0)] +
                           32768ull * (uint64_t)(idx < 0 ? 5 : idx ? 2 : 1);
    const uint32_t bits = (uint32_t)(total >> 15);
    r->satd[m] = satd;
    r->mode_bits[m] = (uint8_t)bits;
    const double cost = (double)satd + (double)bits * j->sqrt_lambda;
    /* xUpdateCandList (:5254) */
    int shift = 0;
    while (shift < num && cost < ccost[num - 1 - shift]) shift++;
    if (shift) {
      for (int i = 1; i < shift; i++) { list[num - i] = list[num - 1 - i]; ccost[num - i] = ccost[num - 1 - i]; }
      list[num - shift] = (uint32_t)m;
      ccost[num - shift] = cost;
    }
  }
  r->num_rd = (uint8_t)num;
  for (int i = 0; i < num && i < 8; i++) r->cand_cost[i] = ccost[i];
  if (fast) { /* :2299-2321 */
    const int ncand = imode >= 0 ? imode : 3;
    for (int jj = 0; jj < ncand; jj++) {
      int inc = 0;
      for (int i = 0; i < num; i++) inc |= mpm[jj] == (int)list[i];
      if (!inc) list[num++] = (uint32_t)mpm[jj];
    }
  }
  r->n_cand = (uint8_t)num;
  for (int i = 0; i < num; i++) r->cand[i] = (uint8_t)list[i];
}

/* ============================================================================================
 * Deblocking: TComLoopFilter::loopFilterPic (TComLoopFilter.cpp:130) on
 * given boundary strengths.  Vertical edges of the whole picture first (luma + chroma), then
 * horizontal edges on that result -- the reference's two CTU sweeps (:132-154); inside one sweep
 * the edges are 8 samples apart and touch at most 4 samples on each side, so their order is free.
 * ========================================================================================== */
static const uint8_t dbk_tc[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};
static const uint8_t dbk_beta[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                     8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                     34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
/* g_aucChromaScale[CHROMA_420] (TComRom.cpp:536) */
static const uint8_t dbk_cscale[58] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19,
                                       20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33, 34, 34, 35, 35,
                                       36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51};
static int clip3i(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }

/* xEdgeFilterLuma's 4-line segment (:605-675) with xCalcDP/DQ (:948), xUseStrongFiltering (:936)
 * and xPelFilterLuma (:833); s = sample q0 of line 0, step = to the next line, off = across */
static void dbk_luma_seg(uint8_t *s, int step, int off, int bs, int qp, const hvx_deblock_params *p) {
  const int tc = dbk_tc[clip3i(0, 53, qp + 2 * (bs - 1) + 2 * p->tc_offset_div2)];
  const int beta = dbk_beta[clip3i(0, 51, qp + 2 * p->beta_offset_div2)];
  const int side = (beta + (beta >> 1)) >> 3, thr_cut = tc * 10;
#define PX(l, i) ((int)s[(l) * step + (i) * off])
  const int dp0 = abs(PX(0, -3) - 2 * PX(0, -2) + PX(0, -1)), dq0 = abs(PX(0, 0) - 2 * PX(0, 1) + PX(0, 2));
  const int dp3 = abs(PX(3, -3) - 2 * PX(3, -2) + PX(3, -1)), dq3 = abs(PX(3, 0) - 2 * PX(3, 1) + PX(3, 2));
  const int d0 = dp0 + dq0, d3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3, d = d0 + d3;
  if (d >= beta) return;
  const int fp = dp < side, fq = dq < side;
  int sw = 1;
  for (int l = 0; l < 4; l += 3) {
    const int dl = 2 * (l ? d3 : d0);
    const int ds = abs(PX(l, -4) - PX(l, -1)) + abs(PX(l, 3) - PX(l, 0));
    sw &= ds < (beta >> 3) && dl < (beta >> 2) && abs(PX(l, -1) - PX(l, 0)) < ((tc * 5 + 1) >> 1);
  }
  for (int l = 0; l < 4; l++) {
    uint8_t *q = s + l * step;
    const int m0 = q[-4 * off], m1 = q[-3 * off], m2 = q[-2 * off], m3 = q[-off], m4 = q[0], m5 = q[off],
              m6 = q[2 * off], m7 = q[3 * off];
    if (sw) {
      q[-off] = (uint8_t)clip3i(m3 - 2 * tc, m3 + 2 * tc, (m1 + 2 * m2 + 2 * m3 + 2 * m4 + m5 + 4) >> 3);
      q[0] = (uint8_t)clip3i(m4 - 2 * tc, m4 + 2 * tc, (m2 + 2 * m3 + 2 * m4 + 2 * m5 + m6 + 4) >> 3);
      q[-2 * off] = (uint8_t)clip3i(m2 - 2 * tc, m2 + 2 * tc, (m1 + m2 + m3 + m4 + 2) >> 2);
      q[off] = (uint8_t)clip3i(m5 - 2 * tc, m5 + 2 * tc, (m3 + m4 + m5 + m6 + 2) >> 2);
      q[-3 * off] = (uint8_t)clip3i(m1 - 2 * tc, m1 + 2 * tc, (2 * m0 + 3 * m1 + m2 + m3 + m4 + 4) >> 3);
      q[2 * off] = (uint8_t)clip3i(m6 - 2 * tc, m6 + 2 * tc, (m3 + m4 + m5 + 3 * m6 + 2 * m7 + 4) >> 3);
    } else {
      int delta = (9 * (m4 - m3) - 3 * (m5 - m2) + 8) >> 4;
      if (abs(delta) < thr_cut) {
        delta = clip3i(-tc, tc, delta);
        q[-off] = (uint8_t)clip3i(0, 255, m3 + delta);
        q[0] = (uint8_t)clip3i(0, 255, m4 - delta);
        const int tc2 = tc >> 1;
        if (fp) q[-2 * off] = (uint8_t)clip3i(0, 255, m2 + clip3i(-tc2, tc2, (((m1 + m3 + 1) >> 1) - m2 + delta) >> 1));
        if (fq) q[off] = (uint8_t)clip3i(0, 255, m5 + clip3i(-tc2, tc2, (((m6 + m4 + 1) >> 1) - m5 - delta) >> 1));
      }
    }
  }
#undef PX
}

/* xEdgeFilterChroma's per-unit part (:750-815) with xPelFilterChroma (:904): 2 lines, bs 2 */
static void dbk_chroma_seg(uint8_t *s, int step, int off, int bs, int qp_avg, int qp_offset,
                           const hvx_deblock_params *p) {
  int qp = qp_avg + qp_offset;
  if (qp >= 58) qp -= 6;                  /* :791-796, 4:2:0 */
  else if (qp >= 0) qp = dbk_cscale[qp];  /* getScaledChromaQP */
  const int tc = dbk_tc[clip3i(0, 53, qp + 2 * (bs - 1) + 2 * p->tc_offset_div2)];
  for (int l = 0; l < 2; l++) {
    uint8_t *q = s + l * step;
    const int m2 = q[-2 * off], m3 = q[-off], m4 = q[0], m5 = q[off];
    const int delta = clip3i(-tc, tc, ((((m4 - m3) << 2) + m2 - m5 + 4) >> 3));
    q[-off] = (uint8_t)clip3i(0, 255, m3 + delta);
    q[0] = (uint8_t)clip3i(0, 255, m4 - delta);
  }
}

void hvxo_deblock(uint8_t *y, int ys, uint8_t *cb, uint8_t *cr, int cs, const uint8_t *bs_ver, const uint8_t *bs_hor,
                  const int8_t *qp, const hvx_deblock_params *p) {
  const int uw = p->pic_w / 4, uh = p->pic_h / 4;
  for (int dir = 0; dir < 2; dir++) {
    const uint8_t *bsm = dir ? bs_hor : bs_ver;
    for (int uy = 0; uy < uh; uy++)
      for (int ux = 0; ux < uw; ux++) {
        const int x = ux * 4, yy = uy * 4;
        if ((dir ? yy : x) % 8 != 0 || (dir ? yy : x) == 0) continue;
        const int bs = bsm[uy * uw + ux];
        if (!bs) continue;
        const int qq = qp[uy * uw + ux], qpp = dir ? qp[(uy - 1) * uw + ux] : qp[uy * uw + ux - 1];
        const int avg = (qpp + qq + 1) >> 1;
        if (dir == 0) dbk_luma_seg(y + yy * ys + x, ys, 1, bs, avg, p);
        else dbk_luma_seg(y + yy * ys + x, 1, ys, bs, avg, p);
        if (bs == 2 && (dir ? yy : x) % 16 == 0) {
          const int cx = x / 2, cy = yy / 2;
          for (int c = 0; c < 2; c++) {
            uint8_t *pl = c ? cr : cb;
            const int off = c ? p->cr_qp_offset : p->cb_qp_offset;
            if (dir == 0) dbk_chroma_seg(pl + cy * cs + cx, cs, 1, bs, avg, off, p);
            else dbk_chroma_seg(pl + cy * cs + cx, 1, cs, bs, avg, off, p);
          }
        }
      }
  }
}

/* =====================================================================================
 * SAO: statistics and application on one plane, single slice and tile
 * (deriveLoopFilterBoundaryAvailibility, TComPicSym.cpp:368: a neighbour CTU is available
 * when it exists).  The reference walks each row with running sign buffers; each buffered
 * sign equals the sign against the neighbour of the class, so the edge class is computed
 * directly here: sgn(c - a) + sgn(c - b) + 2 over the class's two neighbours a, b.
 * ===================================================================================== */
static int sao_sgn(int v) { return (v > 0) - (v < 0); }
/* the two neighbours of edge-offset type t (SAO_TYPE_EO_0/90/135/45) */
static const int kSaoNb[4][2][2] = {{{-1, 0}, {1, 0}}, {{0, -1}, {0, 1}}, {{-1, -1}, {1, 1}}, {{1, -1}, {-1, 1}}};

static int sao_edge(const uint8_t *p, int s, int t) {
  const int c = p[0];
  return sao_sgn(c - p[kSaoNb[t][0][1] * s + kSaoNb[t][0][0]]) + sao_sgn(c - p[kSaoNb[t][1][1] * s + kSaoNb[t][1][0]]) + 2;
}

/* getBlkStats (TEncSampleAdaptiveOffset.cpp:892-1282), isCalculatePreDeblockSamples = false;
 * skipped right columns / bottom rows m_skipLinesR/B (createEncData :125-131: 5/4 luma, 3/2 chroma) */
void hvxo_sao_stats(const uint8_t *org, int os, const uint8_t *rec, int rs, int w, int h, int comp, hvx_sao_stat *out) {
  const int cs = comp ? 32 : 64, skr = comp ? 3 : 5, skb = comp ? 2 : 4;
  const int ncx = (w + cs - 1) / cs, ncy = (h + cs - 1) / cs;
  for (int cy = 0; cy < ncy; cy++)
    for (int cx = 0; cx < ncx; cx++) {
      const int x0 = cx * cs, y0 = cy * cs, bw = w - x0 < cs ? w - x0 : cs, bh = h - y0 < cs ? h - y0 : cs;
      /* getStatistics :303-307: right / below from the picture boundary */
      const int L = cx > 0, A = cy > 0, R = x0 + cs < w, B = y0 + cs < h;
      hvx_sao_stat *st = out + (size_t)(cy * ncx + cx) * HVX_SAO_TYPES;
      memset(st, 0, sizeof(hvx_sao_stat) * HVX_SAO_TYPES);
      for (int t = 0; t < HVX_SAO_TYPES; t++) {
        int xs, xe, ys, ye;
        if (t == 4) { xs = 0; xe = R ? bw - skr : bw; ys = 0; ye = B ? bh - skb : bh; }       /* BO :1229 */
        else if (t == 0) { xs = L ? 0 : 1; xe = R ? bw - skr : bw - 1; ys = 0; ye = B ? bh - skb : bh; } /* :941 */
        else if (t == 1) { xs = 0; xe = R ? bw - skr : bw; ys = A ? 0 : 1; ye = B ? bh - skb : bh - 1; } /* :989 */
        else { xs = L ? 0 : 1; xe = R ? bw - skr : bw - 1; ys = A ? 0 : 1; ye = B ? bh - skb : bh - 1; } /* :1051, :1140 */
        /* EO_135 / EO_45 first row: nothing without the above CTU (:1069-1070, :1157-1161) */
        for (int y = ys; y < ye; y++)
          for (int x = xs; x < xe; x++) {
            const uint8_t *p = rec + (size_t)(y0 + y) * rs + x0 + x;
            const int d = (int)org[(size_t)(y0 + y) * os + x0 + x] - (int)p[0];
            const int k = t == 4 ? p[0] >> 3 : sao_edge(p, rs, t);
            st[t].diff[k] += d;
            st[t].count[k]++;
          }
      }
    }
}

/* offsetCTU / offsetBlock (TComSampleAdaptiveOffset.cpp:313-612): every class's region is the
 * block minus the columns/rows whose neighbour lies outside the picture */
void hvxo_sao_apply(const uint8_t *src, int ss, uint8_t *dst, int ds, int w, int h, int comp,
                    const hvx_sao_ctu *params) {
  const int cs = comp ? 32 : 64;
  const int ncx = (w + cs - 1) / cs, ncy = (h + cs - 1) / cs;
  for (int y = 0; y < h; y++) memcpy(dst + (size_t)y * ds, src + (size_t)y * ss, (size_t)w);
  for (int cy = 0; cy < ncy; cy++)
    for (int cx = 0; cx < ncx; cx++) {
      const hvx_sao_offset *o = &params[cy * ncx + cx].comp[comp];
      if (o->type < 0) continue;
      const int x0 = cx * cs, y0 = cy * cs, bw = w - x0 < cs ? w - x0 : cs, bh = h - y0 < cs ? h - y0 : cs;
      const int L = cx > 0, A = cy > 0, R = cx + 1 < ncx, B = cy + 1 < ncy;
      const int t = o->type;
      const int xs = (t == 0 || t >= 2) && t != 4 && !L ? 1 : 0, xe = (t == 0 || t == 2 || t == 3) && !R ? bw - 1 : bw;
      const int ys = t >= 1 && t <= 3 && !A ? 1 : 0, ye = t >= 1 && t <= 3 && !B ? bh - 1 : bh;
      for (int y = ys; y < ye; y++)
        for (int x = xs; x < xe; x++) {
          const uint8_t *p = src + (size_t)(y0 + y) * ss + x0 + x;
          int off;
          if (t == 4) {
            const int k = ((p[0] >> 3) - o->band) & 31;
            off = k < 4 ? o->offset[k] : 0;
          } else {
            const int e = sao_edge(p, ss, t);
            off = e == 2 ? 0 : o->offset[e < 2 ? e : e - 1];
          }
          const int v = p[0] + off;
          dst[(size_t)(y0 + y) * ds + x0 + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
}

/* ============================================================================================
 * SAO RD decision (TEncSampleAdaptiveOffset.cpp:332-889), 8-bit: DISTORTION_PRECISION_ADJUSTMENT(0)
 * = 0, offset step log2 0, max offset 7 (getMaxOffsetQVal)
 * ========================================================================================== */
typedef struct { int mode, type, aux, offset[32]; } sao_offset_t; /* SAOOffset (modeIdc, typeIdc, typeAuxInfo) */
typedef struct { sao_offset_t c[3]; } sao_blk_t;                  /* SAOBlkParam */
typedef struct { uint8_t st[2]; uint64_t frac; } sao_coder_t;      /* the RD counter: sao_merge, sao_type_idx */
typedef struct { const int32_t *eb; const double *lambda; const int *en; } sao_env_t;

static void sao_bin(const sao_env_t *e, sao_coder_t *c, int ctx, int v) { /* TEncBinCABACCounter::encodeBin */
  const int s = c->st[ctx], p = s >> 1, mps = s & 1;
  c->frac += (uint64_t)(uint32_t)e->eb[s ^ v];
  if (v == mps) c->st[ctx] = (uint8_t)(((p < 62 ? p + 1 : p) << 1) | mps);
  else c->st[ctx] = (uint8_t)((kTransIdxLps[p] << 1) | (p == 0 ? mps ^ 1 : mps));
}
static void sao_ep(sao_coder_t *c, int n) { c->frac += 32768ull * (uint64_t)n; }
static uint32_t sao_written(const sao_coder_t *c) { return (uint32_t)(c->frac >> 15); }
static void sao_reset_bits(sao_coder_t *c) { c->frac &= 32767; }

/* codeSaoMaxUvlc (TEncSbac.cpp:1548) with maxSymbol 7 */
static void sao_max_uvlc(sao_coder_t *c, int code) { sao_ep(c, code == 0 ? 1 : code + (code < 7 ? 1 : 0)); }
/* codeSAOOffsetParam (:1605) */
static void sao_code_offset(const sao_env_t *e, sao_coder_t *c, int comp, const sao_offset_t *p) {
  if (!e->en[comp]) return;
  const int first = comp != 2;  /* first component of its channel type */
  if (first) {
    const int sym = p->mode == 0 ? 0 : p->type == 4 ? 1 : 2;
    sao_bin(e, c, 1, sym != 0); /* codeSaoTypeIdx */
    if (sym) sao_ep(c, 1);
  }
  if (p->mode == 1) {
    int off[4], k = 0;
    const int ncls = p->type == 4 ? 4 : 5;
    for (int i = 0; i < ncls; i++) {
      if (p->type != 4 && i == 2) continue; /* SAO_CLASS_EO_PLAIN */
      off[k++] = p->offset[p->type == 4 ? (p->aux + i) % 32 : i];
    }
    for (int i = 0; i < 4; i++) sao_max_uvlc(c, off[i] < 0 ? -off[i] : off[i]);
    if (p->type == 4) {
      for (int i = 0; i < 4; i++)
        if (off[i]) sao_ep(c, 1);
      sao_ep(c, 5); /* sao_band_position */
    } else if (first) {
      sao_ep(c, 2); /* sao_eo_class */
    }
  }
}
/* codeSAOBlkParam (:1683) */
static void sao_code_blk(const sao_env_t *e, sao_coder_t *c, const sao_blk_t *b, int left, int above, int only_merge) {
  int is_left = 0, is_above = 0;
  if (left) {
    is_left = b->c[0].mode == 2 && b->c[0].type == 0;
    sao_bin(e, c, 0, is_left);
  }
  if (above && !is_left) {
    is_above = b->c[0].mode == 2 && b->c[0].type == 1;
    sao_bin(e, c, 0, is_above);
  }
  if (only_merge) return;
  if (!is_left && !is_above)
    for (int k = 0; k < 3; k++) sao_code_offset(e, c, k, &b->c[k]);
}

static int64_t sao_est_dist(int64_t count, int64_t offset, int64_t diff) { return (count * offset * offset - diff * offset * 2) >> 0; }
/* estIterOffset (:414) */
static int sao_iter_offset(int type, double lambda, int in, int64_t count, int64_t diff, int64_t *best_dist, double *best_cost) {
  int it = in, out = 0;
  double min_cost = lambda;
  while (it != 0) {
    int64_t rate = type == 4 ? (abs(it) + 2) : (abs(it) + 1);
    if (abs(it) == 7) rate--;
    const int64_t dist = sao_est_dist(count, (int64_t)it, diff);
    const double cost = ((double)dist + lambda * (double)rate);
    if (cost < min_cost) {
      min_cost = cost;
      out = it;
      *best_dist = dist;
      *best_cost = cost;
    }
    it = it > 0 ? it - 1 : it + 1;
  }
  return out;
}
/* deriveOffsets (:447) */
static void sao_derive_offsets(double lambda, int type, const int64_t *diff, const int64_t *count, int *q, int *aux) {
  memset(q, 0, 32 * sizeof(int));
  const int ncls = type == 4 ? 32 : 5;
  for (int i = 0; i < ncls; i++) {
    if (type != 4 && i == 2) continue;
    if (count[i] == 0) continue;
    const double x = (double)diff[i] / (double)count[i];
    int v = (int)(x >= 0 ? (double)(int)(x + 0.5) : (double)(int)(x - 0.5)); /* xRoundIbdi, 8-bit */
    q[i] = v < -7 ? -7 : v > 7 ? 7 : v;
  }
  if (type != 4) {
    for (int i = 0; i < 5; i++) {
      if ((i == 0 || i == 1) && q[i] < 0) q[i] = 0;
      if ((i == 3 || i == 4) && q[i] > 0) q[i] = 0;
      if (q[i] != 0) {
        int64_t d = 0;
        double cst = 0;
        q[i] = sao_iter_offset(type, lambda, q[i], count[i], diff[i], &d, &cst);
      }
    }
    *aux = 0;
  } else {
    int64_t dist_bo[32];
    double cost_bo[32];
    memset(dist_bo, 0, sizeof(dist_bo));
    for (int i = 0; i < 32; i++) {
      cost_bo[i] = lambda;
      if (q[i] != 0) q[i] = sao_iter_offset(type, lambda, q[i], count[i], diff[i], &dist_bo[i], &cost_bo[i]);
    }
    double min_cost = 1.7e308;
    for (int b = 0; b < 32 - 4 + 1; b++) {
      double cst = cost_bo[b];
      cst += cost_bo[b + 1];
      cst += cost_bo[b + 2];
      cst += cost_bo[b + 3];
      if (cst < min_cost) { min_cost = cst; *aux = b; }
    }
    int keep[32];
    memset(keep, 0, sizeof(keep));
    for (int i = 0; i < 4; i++) keep[(*aux + i) % 32] = q[(*aux + i) % 32];
    memcpy(q, keep, sizeof(keep));
  }
}
/* getDistortion (:370) on de-quantised offsets */
static int64_t sao_distortion(int type, int aux, const int *inv, const int64_t *diff, const int64_t *count) {
  int64_t d = 0;
  if (type != 4) {
    for (int i = 0; i < 5; i++) d += sao_est_dist(count[i], inv[i], diff[i]);
  } else {
    for (int i = aux; i < aux + 4; i++) {
      const int b = i % 32;
      d += sao_est_dist(count[b], inv[b], diff[b]);
    }
  }
  return d;
}
/* TComSampleAdaptiveOffset::invertQuantOffsets (TComSampleAdaptiveOffset.cpp:167), step 1 */
static void sao_invert(int type, int aux, int *dst, const int *src) {
  int coded[32];
  memcpy(coded, src, sizeof(coded));
  memset(dst, 0, 32 * sizeof(int));
  if (type == 4) {
    for (int i = 0; i < 4; i++) dst[(aux + i) % 32] = coded[(aux + i) % 32];
  } else {
    for (int i = 0; i < 5; i++) dst[i] = coded[i];
  }
}

/* deriveModeNewRDO (:566) */
static void sao_mode_new(const sao_env_t *e, const int64_t *st, sao_blk_t *merge[2], sao_coder_t *coders, int in_label,
                         sao_blk_t *mode, double *norm_cost) {
  enum { CUR = 1, NEXT = 2, MID = 3, TEMP = 4 };
  sao_coder_t go;
  int64_t dist[3], mdist[3] = {0, 0, 0};
  sao_offset_t test[3];
  int inv[32];
  double min_cost, cost;
  memset(test, 0, sizeof(test));
  mode->c[0].mode = 0;
  go = coders[in_label];
  sao_code_blk(e, &go, mode, merge[0] != NULL, merge[1] != NULL, 1);
  coders[MID] = go;
  { /* luma */
    mode->c[0].mode = 0;
    sao_reset_bits(&go);
    sao_code_offset(e, &go, 0, &mode->c[0]);
    mdist[0] = 0;
    min_cost = e->lambda[0] * ((double)sao_written(&go));
    coders[TEMP] = go;
    if (e->en[0]) {
      for (int t = 0; t < 5; t++) {
        test[0].mode = 1;
        test[0].type = t;
        const int64_t *s = st + (size_t)(0 * 5 + t) * 64;
        sao_derive_offsets(e->lambda[0], t, s, s + 32, test[0].offset, &test[0].aux);
        sao_invert(t, test[0].aux, inv, test[0].offset);
        dist[0] = sao_distortion(t, test[0].aux, inv, s, s + 32);
        go = coders[MID];
        sao_reset_bits(&go);
        sao_code_offset(e, &go, 0, &test[0]);
        const int rate = (int)sao_written(&go);
        cost = (double)dist[0] + e->lambda[0] * ((double)rate);
        if (cost < min_cost) {
          min_cost = cost;
          mdist[0] = dist[0];
          mode->c[0] = test[0];
          coders[TEMP] = go;
        }
      }
    }
    go = coders[TEMP];
    coders[MID] = go;
  }
  /* chroma: "off" as the initial cost */
  cost = 0;
  uint32_t prev = 0;
  sao_reset_bits(&go);
  for (int k = 1; k < 3; k++) {
    mode->c[k].mode = 0;
    mdist[k] = 0;
    sao_code_offset(e, &go, k, &mode->c[k]);
    const uint32_t now = sao_written(&go);
    cost += e->lambda[k] * (now - prev);
    prev = now;
  }
  min_cost = cost;
  for (int t = 0; t < 5; t++) {
    go = coders[MID];
    sao_reset_bits(&go);
    prev = 0;
    cost = 0;
    for (int k = 1; k < 3; k++) {
      if (!e->en[k]) {
        test[k].mode = 0;
        dist[k] = 0;
        continue;
      }
      test[k].mode = 1;
      test[k].type = t;
      const int64_t *s = st + (size_t)(k * 5 + t) * 64;
      sao_derive_offsets(e->lambda[k], t, s, s + 32, test[k].offset, &test[k].aux);
      sao_invert(t, test[k].aux, inv, test[k].offset);
      dist[k] = sao_distortion(t, test[k].aux, inv, s, s + 32);
      sao_code_offset(e, &go, k, &test[k]);
      const uint32_t now = sao_written(&go);
      cost += dist[k] + (e->lambda[k] * (now - prev));
      prev = now;
    }
    if (cost < min_cost) {
      min_cost = cost;
      for (int k = 1; k < 3; k++) {
        mdist[k] = dist[k];
        mode->c[k] = test[k];
      }
    }
  }
  /* re-generated rate and normalised cost */
  *norm_cost = 0;
  for (int k = 0; k < 3; k++) *norm_cost += (double)mdist[k] / e->lambda[k];
  go = coders[in_label];
  sao_reset_bits(&go);
  sao_code_blk(e, &go, mode, merge[0] != NULL, merge[1] != NULL, 0);
  *norm_cost += (double)sao_written(&go);
  coders[5] = go; /* the go-on coder after the mode's final coding (m_pcRDGoOnSbacCoder) */
}

/* deriveModeMergeRDO (:709) */
static void sao_mode_merge(const sao_env_t *e, const int64_t *st, sao_blk_t *merge[2], sao_coder_t *coders, int in_label,
                           sao_blk_t *mode, double *norm_cost) {
  enum { TEMP = 4 };
  *norm_cost = 1.7e308;
  for (int mt = 0; mt < 2; mt++) {
    if (!merge[mt]) continue;
    sao_blk_t test = *merge[mt];
    double nd = 0;
    for (int k = 0; k < 3; k++) {
      test.c[k].mode = 2;
      test.c[k].type = mt;
      const sao_offset_t *m = &merge[mt]->c[k];
      if (m->mode != 0) {
        const int64_t *s = st + (size_t)(k * 5 + m->type) * 64;
        nd += (((double)sao_distortion(m->type, m->aux, m->offset, s, s + 32)) / e->lambda[k]);
      }
    }
    sao_coder_t go = coders[in_label];
    sao_reset_bits(&go);
    sao_code_blk(e, &go, &test, merge[0] != NULL, merge[1] != NULL, 0);
    const int rate = (int)sao_written(&go);
    const double cost = nd + (double)rate;
    if (cost < *norm_cost) {
      *norm_cost = cost;
      *mode = test;
      coders[TEMP] = go;
    }
  }
  coders[5] = coders[TEMP];
}

double hvxo_sao_decide(int w, int h, const int64_t *stats, const double *lambdas, int *slice_enabled,
                       const uint8_t *sao_states, int frac_lo, const int32_t *entropy_bits, int slice_ctus, int test_off,
                       int32_t *out, hvx_sao_ctu *recon_out) {
  enum { PIC_INIT = 0, CUR = 1, NEXT = 2, GO = 5 };
  const int wc = (w + 63) / 64, hc = (h + 63) / 64, n = wc * hc;
  const sao_env_t e = {entropy_bits, lambdas, slice_enabled};
  sao_coder_t coders[6];
  memset(coders, 0, sizeof(coders));
  coders[PIC_INIT].st[0] = sao_states[0];
  coders[PIC_INIT].st[1] = sao_states[1];
  coders[PIC_INIT].frac = (uint64_t)frac_lo;
  const int all_off = !slice_enabled[0] && !slice_enabled[1] && !slice_enabled[2];
  sao_blk_t *coded = (sao_blk_t *)calloc((size_t)n, sizeof(sao_blk_t));
  sao_blk_t *recon = (sao_blk_t *)calloc((size_t)n, sizeof(sao_blk_t));
  coders[GO] = coders[PIC_INIT];
  double total = 0;
  for (int a = 0; a < n; a++) {
    if (all_off) continue; /* codedParams reset: every component off */
    coders[CUR] = coders[GO];
    sao_blk_t *merge[2] = {NULL, NULL};
    const int x = a % wc, y = a / wc, s0 = slice_ctus > 0 ? a - a % slice_ctus : 0;
    if (x > 0 && a - 1 >= s0) merge[0] = &recon[a - 1];   /* getMergeList: left, same slice */
    if (y > 0 && a - wc >= s0) merge[1] = &recon[a - wc]; /* above */
    const int64_t *st = stats + (size_t)a * 960;
    double min_cost = 1.7e308, cost;
    sao_blk_t mode;
    memset(&mode, 0, sizeof(mode));
    for (int m = 1; m < 3; m++) { /* SAO_MODE_OFF is covered by the NEW mode's comparisons */
      if (m == 1) sao_mode_new(&e, st, merge, coders, CUR, &mode, &cost);
      else sao_mode_merge(&e, st, merge, coders, CUR, &mode, &cost);
      if (cost < min_cost) {
        min_cost = cost;
        coded[a] = mode;
        coders[NEXT] = coders[GO];
      }
    }
    total += min_cost;
    coders[GO] = coders[NEXT];
    /* reconstructBlkSAOParam */
    recon[a] = coded[a];
    for (int k = 0; k < 3; k++) {
      sao_offset_t *o = &recon[a].c[k];
      if (o->mode == 1) sao_invert(o->type, o->aux, o->offset, o->offset);
      else if (o->mode == 2) *o = merge[o->type]->c[k];
    }
  }
  if (!all_off && total >= 0 && test_off) { /* the coded parameters only: offsetCTU has run (:840-859) */
    memset(coded, 0, (size_t)n * sizeof(sao_blk_t));
    slice_enabled[0] = slice_enabled[1] = slice_enabled[2] = 0;
  }
  for (int a = 0; a < n; a++)
    for (int k = 0; k < 3; k++) {
      const sao_offset_t *o = &coded[a].c[k];
      int32_t *r = out + ((size_t)a * 3 + k) * 8;
      memset(r, 0, 8 * sizeof(int32_t));
      r[0] = o->mode;
      if (o->mode != 0) {
        r[1] = o->type;
        if (o->mode == 1) {
          r[2] = o->aux;
          if (o->type == 4)
            for (int i = 0; i < 4; i++) r[3 + i] = o->offset[(o->aux + i) % 32];
          else
            for (int i = 0; i < 5; i++) r[3 + i] = o->offset[i];
        }
      }
      if (recon_out) {
        const sao_offset_t *q = &recon[a].c[k];
        hvx_sao_offset *d = &recon_out[a].comp[k];
        memset(d, 0, sizeof(*d));
        d->type = (int8_t)(q->mode == 0 ? -1 : q->type);
        if (q->mode != 0) {
          if (q->type == 4) {
            d->band = (uint8_t)q->aux;
            for (int i = 0; i < 4; i++) d->offset[i] = (int8_t)q->offset[(q->aux + i) % 32];
          } else {
            d->offset[0] = (int8_t)q->offset[0];
            d->offset[1] = (int8_t)q->offset[1];
            d->offset[2] = (int8_t)q->offset[3];
            d->offset[3] = (int8_t)q->offset[4];
          }
        }
      }
    }
  free(coded);
  free(recon);
  return total;
}

void hvxo_sao_pic_params(int layer, const double *disabled_rate, double rate, double rate_chroma, int *slice_enabled) {
  for (int k = 0; k < 3; k++) {
    slice_enabled[k] = 1;
    if (rate > 0.0) {
      if (rate_chroma > 0.0) {
        if (layer > 0 && disabled_rate[k * 7 + layer - 1] > (k == 0 ? rate : rate_chroma)) slice_enabled[k] = 0;
      } else {
        if (layer > 0 && disabled_rate[0] > rate) slice_enabled[k] = 0;
      }
    }
  }
}

void hvxo_sao_update_rates(int layer, const hvx_sao_ctu *recon, int nctu, double rate, double rate_chroma,
                           double *disabled_rate) {
  if (!(rate > 0.0)) return;
  int off[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++)
    for (int a = 0; a < nctu; a++)
      if (recon[a].comp[k].type < 0) off[k]++;
  if (rate_chroma > 0.0) {
    for (int k = 0; k < 3; k++) disabled_rate[k * 7 + layer] = (double)off[k] / (double)nctu;
  } else if (layer == 0) {
    disabled_rate[0] = (double)(off[0] + off[1] + off[2]) / (double)(nctu * 3);
  }
}
