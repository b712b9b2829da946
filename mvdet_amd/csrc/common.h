// Shared helpers for the libmvbev HIP sources (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/mvbev.h"

#define MVBEV_CHECK_LAUNCH()                         \
  do {                                               \
    hipError_t _e = hipGetLastError();               \
    if (_e != hipSuccess) return MVBEV_ERR_HIP;      \
  } while (0)

namespace mvbev {

constexpr int kWave = 64;

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so give each
// XCD group a contiguous range of logical tiles.  Speed only, never correctness.
__device__ inline int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8, k = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <typename T> __device__ inline float to_f32(T v);
template <> __device__ inline float to_f32<float>(float v) { return v; }
template <> __device__ inline float to_f32<__half>(__half v) { return __half2float(v); }
template <typename T> __device__ inline T from_f32(float v);
template <> __device__ inline float from_f32<float>(float v) { return v; }
template <> __device__ inline __half from_f32<__half>(float v) { return __float2half(v); }

}  // namespace mvbev
