// hvx_ssimw.hpp -- the stVSSIM orientation filters (stvssim.c hFilter / rFilter / vFilter / lFilter
// :116-334 and their 4x4 forms), shared by the metric kernels (hvx_ssim.hpp) and the CU decision's
// stVSSIM cost (hvx_hm.hpp).
#pragma once
#include <hip/hip_runtime.h>

// the weight of window sample (y, x) under directional filter k (0 h, 1 r, 2 v, 3 l) of a beta x beta
// window: wa on the filter's line (3 samples wide for 8x8 windows, 1 for 4x4), wb elsewhere
__device__ __forceinline__ float orient_weight(int k, int beta, int y, int x, float wa, float wb) {
  if (wa < 0) wa = 1.0f;
  if (wb < 0) wb = 1.0f;
  if (wa < wb) { const float c = wb; wb = wa; wa = c; }
  bool on;
  if (beta == 4) {
    on = k == 0 ? x == beta / 2 - 1 : k == 1 ? x + y == beta - 1 : k == 2 ? y == beta / 2 - 1 : x == y;
  } else {
    on = k == 0 ? (x >= beta / 2 - 1 && x <= beta / 2 + 1)
       : k == 1 ? (x + y - beta >= -2 && x + y - beta <= 0)
       : k == 2 ? (y >= beta / 2 - 1 && y <= beta / 2 + 1)
       : abs(x - y) <= 1;
  }
  return on ? wa : wb;
}

