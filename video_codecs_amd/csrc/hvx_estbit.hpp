// hvx_estbit.hpp -- TEncSbac::estBit (TEncSbac.cpp:1726-1950): CABAC context states ->
// the estBits rate tables RDOQ reads.  One implementation for the host entry point and the
// batched kernel (one thread per table: ~200 table reads, no reuse across jobs).
#pragma once
#include "hvx_dev.hpp"

// significanceMapContextSetStart / Size (ContextTables.h:85-86), [chType][4x4, 8x8, NxN, single]
__host__ __device__ __forceinline__ int estbit_sig_start(int ch, int t) {
  return ch ? (t == 0 ? 0 : t == 1 ? 9 : t == 2 ? 12 : 15) : (t == 0 ? 0 : t == 1 ? 9 : t == 2 ? 21 : 27);
}
__host__ __device__ __forceinline__ int estbit_sig_size(int ch, int t) {
  return ch ? (t == 0 ? 9 : t == 1 ? 3 : t == 2 ? 3 : 1) : (t == 0 ? 9 : t == 1 ? 12 : t == 2 ? 6 : 1);
}
// g_uiGroupIdx (TComRom.cpp) for the last-position prefix: the group of coordinate v < 32
__host__ __device__ __forceinline__ int estbit_group_idx(int v) {
  if (v < 4) return v;
  int g = 4, lo = 4, len = 2;  // groups of 2, 2, 4, 4, 8, 8 starting at 4
  while (v >= lo + len * 2) { lo += len * 2; g += 2; len <<= 1; }
  return g + (v >= lo + len ? 1 : 0);
}
__host__ __device__ __forceinline__ int estbit_log2(int v) {
  int l = 0;
  while ((1 << (l + 1)) <= v) l++;
  return l;
}

__host__ __device__ inline void estbit_update(const uint8_t *st, const int32_t *eb, const uint32_t *rice, int w, int h,
                                              int ch, hvx_estbits *e) {
  // ContextModel::getEntropyBits(val) = m_entropyBits[m_ucState ^ val] (ContextModel.h:79)
#define EB(ctx, v) eb[st[(ctx)] ^ (v)]
  // estCBFBit
  for (int i = 0; i < 10; i++)
    for (int b = 0; b < 2; b++) e->blockCbpBits[i][b] = EB(HVX_CTX_QT_CBF + i, b);
  for (int i = 0; i < 4; i++)
    for (int b = 0; b < 2; b++) e->blockRootCbpBits[i][b] = EB(HVX_CTX_QT_ROOT_CBF + i, b);
  // estSignificantCoeffGroupMapBit
  for (int i = 0; i < 2; i++)
    for (int b = 0; b < 2; b++) e->significantCoeffGroupBits[i][b] = EB(HVX_CTX_SIG_CG + ch * 2 + i, b);
  // estSignificantMapBit
  const int type = (w == 4 && h == 4) ? 0 : (w == 8 && h == 8) ? 1 : 2;
  const int first = estbit_sig_start(ch, type), num = estbit_sig_size(ch, type), off = ch ? 28 : 0;
  if (first > 0)
    for (int b = 0; b < 2; b++) e->significantBits[off][b] = EB(HVX_CTX_SIG + off, b);
  {
    const int single = estbit_sig_start(ch, 3);
    for (int b = 0; b < 2; b++) e->significantBits[off + single][b] = EB(HVX_CTX_SIG + off + single, b);
  }
  for (int k = first; k < first + num; k++)
    for (int b = 0; b < 2; b++) e->significantBits[off + k][b] = EB(HVX_CTX_SIG + off + k, b);
  // estLastSignificantPositionBit (getLastSignificantContextParameters, TComChromaFormat.h:211)
  {
    const int cw = estbit_log2(w) - 2, chh = estbit_log2(h) - 2;
    const int ox = ch ? 0 : cw * 3 + ((cw + 1) >> 2), oy = ch ? 0 : chh * 3 + ((chh + 1) >> 2);
    const int sx = ch ? cw : (cw + 3) >> 2, sy = ch ? chh : (chh + 3) >> 2;
    const int bx = HVX_CTX_LAST_X + ch * 15, by = HVX_CTX_LAST_Y + ch * 15;
    int bits = 0, c;
    for (c = 0; c < estbit_group_idx(w - 1); c++) {
      const int o = ox + (c >> sx);
      e->lastXBits[ch][c] = bits + EB(bx + o, 0);
      bits += EB(bx + o, 1);
    }
    e->lastXBits[ch][c] = bits;
    bits = 0;
    for (c = 0; c < estbit_group_idx(h - 1); c++) {
      const int o = oy + (c >> sy);
      e->lastYBits[ch][c] = bits + EB(by + o, 0);
      bits += EB(by + o, 1);
    }
    e->lastYBits[ch][c] = bits;
  }
  // estSignificantCoefficientsBit
  for (int i = ch ? 16 : 0; i < (ch ? 24 : 16); i++)
    for (int b = 0; b < 2; b++) e->greaterOneBits[i][b] = EB(HVX_CTX_ONE + i, b);
  for (int i = ch ? 4 : 0; i < (ch ? 6 : 4); i++)
    for (int b = 0; b < 2; b++) e->levelAbsBits[i][b] = EB(HVX_CTX_ABS + i, b);
#undef EB
  for (int i = 0; i < 4; i++) e->golombRiceAdaptationStatistics[i] = (int32_t)rice[i];
}

static __global__ __launch_bounds__(64) void k_estbits(const uint8_t *__restrict__ states, const int32_t *__restrict__ eb,
                                                const uint32_t *__restrict__ rice, const hvx_estbit_job *__restrict__ jobs,
                                                int n, hvx_estbits *__restrict__ inout) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const hvx_estbit_job j = jobs[i];
  estbit_update(states + (size_t)i * HVX_NUM_CTX, eb, rice + (size_t)i * 4, j.width, j.height, j.ch_type, inout + i);
}
