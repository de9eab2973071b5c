// Shared helpers for the gfx950 (CDNA4 / MI355X) kernels of torchpruner_amd.
// Wave size is 64 on CDNA: every wave-level idiom below is written for 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#define TP_WAVE 64

#define TP_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      return _e;                                                                  \
    }                                                                             \
  } while (0)

namespace tp {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Reduce over groups of G consecutive lanes (G power of two <= 64).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = G / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// NaN-propagating max / relu: fmaxf(NaN, x) returns x, which would silently erase the
// NaN marks the pruner's cascade probe relies on (SURVEY.md §7.3 hard part 2).
__device__ __forceinline__ float nan_max(float a, float b) {
  return (a > b || a != a) ? a : b;
}
__device__ __forceinline__ float nan_relu(float x) { return (x > 0.f || x != x) ? x : 0.f; }

inline unsigned ceil_div(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace tp
