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
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Raw buffer loads (offset >= num_records returns 0 in hardware). Declared against the LLVM
// intrinsics directly: the clang __builtin_amdgcn_raw_buffer_load_b128 of ROCm 7.2 lowers to a
// single-dword load on gfx950.
__device__ f32x4 buf_load_f32x4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ unsigned buf_load_u32(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");

// Buffer descriptor for a flat range of ``bytes`` (stride 0, raw addressing). Build it only
// from wave-uniform values (kernel arguments) so it lives in SGPRs.
__device__ __forceinline__ i32x4 make_rsrc(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  i32x4 r;
  r.x = (int)(unsigned)a;
  r.y = (int)((a >> 32) & 0xffffu);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}

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

// Per-element score partial of a data-gradient epilogue (g = dL/da, a = the activation):
// tay_mode 0 Taylor -(g * a); 1 Sensitivity |g|; 2 Sensitivity of a ReLU-masked gradient
// |g| where a > 0 (the evaluation module is the BN before the ReLU: ResNet bn1 / bn2).
// v + v[lane ^ 8] / ^ 16 / ^ 32 without the LDS: DPP row_ror:8 (xor 8 inside a 16-lane row) and
// gfx950's v_permlane16_swap / v_permlane32_swap (the two swapped halves summed); each lane gets
// the same float sum as `v + __shfl_xor(v, m)` (one add of the same two values), bit for bit
__device__ __forceinline__ float xsum8(float v) {
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xf, 0xf, false));
}
__device__ __forceinline__ float xsum16(float v) {
  const auto s = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)s[0]) + __builtin_bit_cast(float, (unsigned)s[1]);
}
__device__ __forceinline__ float xsum32(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)s[0]) + __builtin_bit_cast(float, (unsigned)s[1]);
}

__device__ __forceinline__ float tay_term(int mode, float g, float a) {
  return mode == 1 ? fabsf(g) : mode == 2 ? (a > 0.f ? fabsf(g) : 0.f) : -(g * a);
}
// NaN-propagating ReLU (slope 0) / LeakyReLU (slope > 0): NaN passes through (pruner NaN probe)
__device__ __forceinline__ float nan_act(float x, float slope) {
  return (x > 0.f || x != x) ? x : (slope != 0.f ? x * slope : 0.f);
}
// backward of nan_act given its OUTPUT a (sign(a) == sign(x) for slope >= 0)
__device__ __forceinline__ float act_grad(float a, float g, float slope) {
  return a > 0.f ? g : (slope != 0.f ? g * slope : 0.f);
}

// Division by a runtime-invariant divisor as mul-hi + add + shift (Granlund-Montgomery; valid
// for 0 <= n < 2^31): a 32-bit integer division is otherwise ~25 VALU instructions.
struct FastDiv {
  unsigned d = 1, m = 1, l = 0;
  FastDiv() = default;
  explicit FastDiv(unsigned dv) : d(dv) {
    l = 0;
    while ((1ull << l) < dv) ++l;
    m = (unsigned)(((1ull << 32) * ((1ull << l) - dv)) / dv + 1);
  }
  __device__ __forceinline__ int div(int n) const { return (int)((__umulhi((unsigned)n, m) + (unsigned)n) >> l); }
};

inline unsigned ceil_div(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace tp
