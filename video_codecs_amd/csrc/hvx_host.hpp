// hvx_host.hpp -- host-side internals shared by the translation units of libhvx.so
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/hvx.h"

struct hvx_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  // staging for the host-memory single-TU forms
  char *scratch = nullptr;
  char *pinned = nullptr;
  // interleaved per-TU scratch of the batched TU pipeline (grown on demand)
  char *tu_scr = nullptr;
  size_t tu_scr_bytes = 0;
};

namespace hvxi {
int fail(int code, const char *what);
int hip_fail(hipError_t e, const char *what);
int launched(const char *what);
}  // namespace hvxi

#define HVX_HIP(call)                                          \
  do {                                                         \
    hipError_t e_ = (call);                                    \
    if (e_ != hipSuccess) return hvxi::hip_fail(e_, #call);    \
  } while (0)

// hvx_hm.hip: uploads that translation unit's copies of the constant tables
int hvx_hm_module_init();
