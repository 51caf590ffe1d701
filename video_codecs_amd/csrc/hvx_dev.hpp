// hvx_dev.hpp -- shared device helpers and constant tables for the gfx950 (CDNA4) kernels.
// Included once, by hvx_lib.hip (single translation unit: the __constant__ tables below
// are uploaded once per context by hvx_create).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hvx.h"

#define HVX_WAVE 64

// ---------------------------------------------------------------------------------------
// Constant tables (HEVC spec values; host-generated, uploaded in hvx_create).
//   kScan[type][l]   : grouped 4x4 scan of a (4<<l)x(4<<l) TU, raster positions (l = log2-2)
//   kScanCG[type][l] : scan of the (1<<l)x(1<<l) coefficient-group grid
//   kMat[l]          : DCT matrix of size 4<<l, [k][x]
// ---------------------------------------------------------------------------------------
static __constant__ uint16_t kScan[3][1360];
static __constant__ uint8_t kScanCG[3][85];
static __constant__ int16_t kMat[1360];
static __constant__ int16_t kMatT[1360];  // each size's matrix transposed: kMatT[x][k] = kMat[k][x]
static __constant__ int8_t kDst4[16] = {29, 55, 74, 84, 74, 74, 0, -74, 84, -29, -74, 55, 55, -84, 74, -29};
static __constant__ int32_t kQuantScales[6] = {26214, 23302, 20560, 18396, 16384, 14564};
static __constant__ int32_t kInvQuantScales[6] = {40, 45, 51, 57, 64, 72};
static __constant__ uint8_t kGroupIdx[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                      8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
static __constant__ uint8_t kCtxIndMap4x4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
static __constant__ int8_t kLumaFilter[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                         {-1, 4, -10, 58, 17, -5, 1, 0},
                                         {-1, 4, -11, 40, 40, -11, 4, -1},
                                         {0, 1, -5, 17, 58, -10, 4, -1}};
// the luma taps as int16 pairs (t = 2u, 2u + 1) for v_dot2_i32_i16
constexpr uint32_t luma_pair(int a, int b) { return ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16); }
static __constant__ uint32_t kLumaPairs[4][4] = {
    {luma_pair(0, 0), luma_pair(0, 64), luma_pair(0, 0), luma_pair(0, 0)},
    {luma_pair(-1, 4), luma_pair(-10, 58), luma_pair(17, -5), luma_pair(1, 0)},
    {luma_pair(-1, 4), luma_pair(-11, 40), luma_pair(40, -11), luma_pair(4, -1)},
    {luma_pair(0, 1), luma_pair(-5, 17), luma_pair(58, -10), luma_pair(4, -1)}};
// the luma taps as packed int8: [fx][0] = taps 0..3, [fx][1] = taps 4..7 (byte k = tap k) for v_dot4_i32_i8
constexpr uint32_t tap4(int a, int b, int c, int d) {
  return ((uint32_t)a & 0xffu) | (((uint32_t)b & 0xffu) << 8) | (((uint32_t)c & 0xffu) << 16) | ((uint32_t)d << 24);
}
static __constant__ uint32_t kLumaTap4[4][2] = {{tap4(0, 0, 0, 64), tap4(0, 0, 0, 0)},
                                         {tap4(-1, 4, -10, 58), tap4(17, -5, 1, 0)},
                                         {tap4(-1, 4, -11, 40), tap4(40, -11, 4, -1)},
                                         {tap4(0, 1, -5, 17), tap4(58, -10, 4, -1)}};
// the chroma taps packed for v_dot4_i32_i8 (byte k = tap k) and as int16 pairs (taps 0,1 | 2,3)
static __constant__ uint32_t kChromaTap4[8] = {tap4(0, 64, 0, 0),   tap4(-2, 58, 10, -2), tap4(-4, 54, 16, -2), tap4(-6, 46, 28, -4),
                                        tap4(-4, 36, 36, -4), tap4(-4, 28, 46, -6), tap4(-2, 16, 54, -4), tap4(-2, 10, 58, -2)};
static __constant__ uint32_t kChromaPairs[8][2] = {
    {luma_pair(0, 64), luma_pair(0, 0)},   {luma_pair(-2, 58), luma_pair(10, -2)}, {luma_pair(-4, 54), luma_pair(16, -2)},
    {luma_pair(-6, 46), luma_pair(28, -4)}, {luma_pair(-4, 36), luma_pair(36, -4)}, {luma_pair(-4, 28), luma_pair(46, -6)},
    {luma_pair(-2, 16), luma_pair(54, -4)}, {luma_pair(-2, 10), luma_pair(58, -2)}};
static __constant__ int8_t kChromaFilter[8][4] = {{0, 64, 0, 0},   {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-6, 46, 28, -4},
                                           {-4, 36, 36, -4}, {-4, 28, 46, -6}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

__device__ __forceinline__ int scan_base(int l) { return l == 0 ? 0 : l == 1 ? 16 : l == 2 ? 80 : 336; }
__device__ __forceinline__ int cg_base(int l) { return l == 0 ? 0 : l == 1 ? 1 : l == 2 ? 5 : 21; }
__device__ __forceinline__ int mat_base(int l) { return scan_base(l); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & (HVX_WAVE - 1); }

// all-lanes sum over the 64-lane wave (every lane receives the total)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, HVX_WAVE);
  return v;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, HVX_WAVE);
  return v;
}

__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }
__device__ __forceinline__ int clip_pel(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
__device__ __forceinline__ int32_t shl32(int32_t v, int s) { return (int32_t)((uint32_t)v << s); }
__device__ __forceinline__ int32_t sub32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

// TComRdCost::xGetExpGolombNumberOfBits (TComRdCost.cpp:279), closed form of the loop
__device__ __forceinline__ uint32_t eg_bits(int v) {
  // t = 2|v| + (v <= 0) >= 1, branch-free (lanes are different candidates)
  const uint32_t t = ((uint32_t)abs(v) << 1) | (v <= 0 ? 1u : 0u);
  return 63u - 2u * (uint32_t)__builtin_clz(t);
}

// ---------------------------------------------------------------------------------------
// Hadamard tiles (TComRdCost.cpp:1310-1523) on int differences held in registers.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void hadamard4(const int *in, int *out) {
  int a0 = in[0] + in[2], a1 = in[1] + in[3], a2 = in[0] - in[2], a3 = in[1] - in[3];
  out[0] = a0 + a1; out[1] = a0 - a1; out[2] = a2 + a3; out[3] = a2 - a3;
}
__device__ __forceinline__ void hadamard8(const int *in, int *out) {
  int a[8], b[8];
#pragma unroll
  for (int i = 0; i < 4; i++) { a[i] = in[i] + in[i + 4]; a[i + 4] = in[i] - in[i + 4]; }
  b[0] = a[0] + a[2]; b[1] = a[1] + a[3]; b[2] = a[0] - a[2]; b[3] = a[1] - a[3];
  b[4] = a[4] + a[6]; b[5] = a[5] + a[7]; b[6] = a[4] - a[6]; b[7] = a[5] - a[7];
#pragma unroll
  for (int i = 0; i < 4; i++) { out[2 * i] = b[2 * i] + b[2 * i + 1]; out[2 * i + 1] = b[2 * i] - b[2 * i + 1]; }
}

template <typename TO, typename TC>
__device__ __forceinline__ uint32_t had8_tile(const TO *o, int so, const TC *c, int sc) {
  int d[8][8];
#pragma unroll
  for (int y = 0; y < 8; y++) {
    int row[8];
#pragma unroll
    for (int x = 0; x < 8; x++) row[x] = (int)o[y * so + x] - (int)c[y * sc + x];
    hadamard8(row, d[y]);
  }
  uint32_t s = 0;
#pragma unroll
  for (int x = 0; x < 8; x++) {
    int col[8], r[8];
#pragma unroll
    for (int y = 0; y < 8; y++) col[y] = d[y][x];
    hadamard8(col, r);
#pragma unroll
    for (int k = 0; k < 8; k++) s += (uint32_t)abs(r[k]);
  }
  return (s + 2) >> 2;
}

template <typename TO, typename TC>
__device__ __forceinline__ uint32_t had4_tile(const TO *o, int so, const TC *c, int sc) {
  int d[4][4];
#pragma unroll
  for (int y = 0; y < 4; y++) {
    int row[4];
#pragma unroll
    for (int x = 0; x < 4; x++) row[x] = (int)o[y * so + x] - (int)c[y * sc + x];
    hadamard4(row, d[y]);
  }
  uint32_t s = 0;
#pragma unroll
  for (int x = 0; x < 4; x++) {
    int col[4] = {d[0][x], d[1][x], d[2][x], d[3][x]}, r[4];
    hadamard4(col, r);
#pragma unroll
    for (int k = 0; k < 4; k++) s += (uint32_t)abs(r[k]);
  }
  return (s + 1) >> 1;
}

template <typename TO, typename TC>
__device__ __forceinline__ uint32_t had2_tile(const TO *o, int so, const TC *c, int sc) {
  int d0 = (int)o[0] - (int)c[0], d1 = (int)o[1] - (int)c[1];
  int d2 = (int)o[so] - (int)c[sc], d3 = (int)o[so + 1] - (int)c[sc + 1];
  int m0 = d0 + d2, m1 = d1 + d3, m2 = d0 - d2, m3 = d1 - d3;
  return (uint32_t)(abs(m0 + m1) + abs(m0 - m1) + abs(m2 + m3) + abs(m2 - m3));
}

// xGetHADs (TComRdCost.cpp:1526) computed by one wave: tiles spread over lanes, total to all lanes.
template <typename TO, typename TC>
__device__ __forceinline__ uint32_t wave_satd(const TO *org, int so, const TC *cur, int sc, int w, int h) {
  const int t = (w % 8 == 0 && h % 8 == 0) ? 8 : (w % 4 == 0 && h % 4 == 0) ? 4 : 2;
  const int tw = w / t, nt = tw * (h / t);
  uint32_t s = 0;
  for (int i = lane_id(); i < nt; i += HVX_WAVE) {
    int ty = i / tw, tx = i - ty * tw;
    const TO *o = org + ty * t * so + tx * t;
    const TC *c = cur + ty * t * sc + tx * t;
    s += t == 8 ? had8_tile(o, so, c, sc) : t == 4 ? had4_tile(o, so, c, sc) : had2_tile(o, so, c, sc);
  }
  return wave_sum_u32(s);
}
