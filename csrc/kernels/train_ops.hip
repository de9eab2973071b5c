// Training-mode elementwise ops of the finetune step: inverted dropout with
// a counter-based Philox4x32-10 generator. The keep mask is a pure function of (seed, element
// index), so the backward regenerates it instead of storing a mask tensor, and the result does
// not depend on the launch geometry. y = x * (keep ? 1/(1-p) : 0) as a multiplication, so NaN
// inputs stay NaN even in dropped positions (the pruner's NaN probe relies on NaN propagation).
#include "tp_common.h"

namespace tp {

struct Philox {
  static constexpr unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  __device__ static uint4 round(uint4 c, uint2 k) {
    const unsigned long long p0 = (unsigned long long)M0 * c.x, p1 = (unsigned long long)M1 * c.z;
    return make_uint4((unsigned)(p1 >> 32) ^ c.y ^ k.x, (unsigned)p1, (unsigned)(p0 >> 32) ^ c.w ^ k.y, (unsigned)p0);
  }
  // 10 rounds on counter (ctr_lo, ctr_hi, 0, 0) with a 64-bit key
  __device__ static uint4 gen(unsigned long long ctr, unsigned long long key) {
    uint4 c = make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), 0u, 0u);
    uint2 k = make_uint2((unsigned)key, (unsigned)(key >> 32));
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      c = round(c, k);
      k.x += W0;
      k.y += W1;
    }
    return round(c, k);
  }
};

// element e uses word (e & 3) of Philox(counter = e >> 2): 4 elements per generator call
__global__ __launch_bounds__(256) void dropout_fb(const float4* __restrict__ x, float4* __restrict__ y, long long n4,
                                                  unsigned long long seed, unsigned threshold, float scale) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < n4;
       t += (long long)gridDim.x * blockDim.x) {
    const uint4 r = Philox::gen((unsigned long long)t, seed);
    const float4 v = x[t];
    float4 o;
    o.x = v.x * (r.x >= threshold ? scale : 0.f);
    o.y = v.y * (r.y >= threshold ? scale : 0.f);
    o.z = v.z * (r.z >= threshold ? scale : 0.f);
    o.w = v.w * (r.w >= threshold ? scale : 0.f);
    y[t] = o;
  }
}

__global__ void dropout_tail(const float* __restrict__ x, float* __restrict__ y, long long n, long long n4,
                             unsigned long long seed, unsigned threshold, float scale) {
  const long long e = n4 * 4 + threadIdx.x;
  if (e >= n) return;
  const uint4 r = Philox::gen((unsigned long long)n4, seed);
  const unsigned w = threadIdx.x == 0 ? r.x : threadIdx.x == 1 ? r.y : r.z;
  y[e] = x[e] * (w >= threshold ? scale : 0.f);
}

}  // namespace tp

// y = dropout(x) (forward) or dx = dropout'(g) (backward: same seed, same call): the keep
// decision is uint32 >= threshold with threshold = round(p * 2^32).
extern "C" hipError_t tp_dropout(const float* x, float* y, long long n, unsigned long long seed, double p,
                                 hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (!(p >= 0.0 && p < 1.0) || ((uintptr_t)x | (uintptr_t)y) % 16) return hipErrorInvalidValue;
  const double th = p * 4294967296.0;
  const unsigned threshold = th >= 4294967295.0 ? 0xFFFFFFFFu : (unsigned)th;
  const float scale = (float)(1.0 / (1.0 - p));
  const long long n4 = n / 4;
  if (n4 > 0) {
    const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(n4, 256), 8192);
    tp::dropout_fb<<<grid, 256, 0, st>>>(reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), n4, seed,
                                         threshold, scale);
  }
  if (n % 4) tp::dropout_tail<<<1, 4, 0, st>>>(x, y, n, n4, seed, threshold, scale);
  return hipGetLastError();
}
