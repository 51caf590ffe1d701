// hvx_tables.hpp -- host generation + upload of the device constant tables (scan orders, DCT
// matrices; TComRom.cpp:192-262).  Included by every translation unit after hvx_dev.hpp: the
// tables have internal linkage, so each unit uploads its own copies.
#pragma once
#include <vector>

#include "hvx_host.hpp"

namespace {
// ---- host generation of the constant tables (HEVC spec rules; TComRom.cpp:192-262) ----
const int kCosH[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4, 0};
int dct32(int k, int n) {
  if (k == 0) return 64;
  int j = (k * (2 * n + 1)) % 128, sign = 1;
  if (j > 64) j = 128 - j;
  if (j > 32) { j = 64 - j; sign = -1; }
  return sign * kCosH[j];
}

void gen_scan(std::vector<int> &out, int w, int h, int stride, int type, int offx, int offy) {
  if (type == 0) {
    for (int d = 0; d < w + h - 1; d++) {
      int y = d < h - 1 ? d : h - 1, x = d - y;
      while (y >= 0 && x < w) out.push_back((y + offy) * stride + x + offx), y--, x++;
    }
  } else if (type == 1) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) out.push_back((y + offy) * stride + x + offx);
  } else {
    for (int x = 0; x < w; x++)
      for (int y = 0; y < h; y++) out.push_back((y + offy) * stride + x + offx);
  }
}

int upload_tables() {
  uint16_t scan[3][1360];
  uint8_t scan_cg[3][85];
  int16_t mat[1360];
  for (int t = 0; t < 3; t++) {
    int sb = 0, cb = 0;
    for (int l = 0; l < 4; l++) {
      const int n = 4 << l, g = 1 << l;
      std::vector<int> cg, full;
      gen_scan(cg, g, g, g, t, 0, 0);
      for (int i = 0; i < g * g; i++) {
        const int gx = cg[i] % g, gy = cg[i] / g;
        gen_scan(full, 4, 4, n, t, gx * 4, gy * 4);
      }
      for (int i = 0; i < n * n; i++) scan[t][sb + i] = (uint16_t)full[i];
      for (int i = 0; i < g * g; i++) scan_cg[t][cb + i] = (uint8_t)cg[i];
      sb += n * n;
      cb += g * g;
    }
  }
  int mb = 0;
  for (int l = 0; l < 4; l++) {
    const int n = 4 << l;
    for (int k = 0; k < n; k++)
      for (int x = 0; x < n; x++) mat[mb + k * n + x] = (int16_t)dct32(k * (32 / n), x);
    mb += n * n;
  }
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kScan), scan, sizeof(scan)));
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kScanCG), scan_cg, sizeof(scan_cg)));
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kMat), mat, sizeof(mat)));
  int16_t matT[1360];
  mb = 0;
  for (int l = 0; l < 4; l++) {
    const int n = 4 << l;
    for (int k = 0; k < n; k++)
      for (int x = 0; x < n; x++) matT[mb + x * n + k] = mat[mb + k * n + x];
    mb += n * n;
  }
  HVX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kMatT), matT, sizeof(matT)));
  return HVX_OK;
}
}  // namespace
