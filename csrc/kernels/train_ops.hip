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

// ---- max-pool (k x k, stride s, padding p) with a window-local argmax byte, and its backward
// as a gather (each input pixel sums the gradients of the windows whose argmax it is, in a fixed
// window order: deterministic, no atomics). Tie / NaN rule of PyTorch's max_pool2d: a later tap
// wins only if it is greater or NaN; the index starts at the first in-image tap.
namespace tp {

__global__ __launch_bounds__(256) void maxpool_fwd_arg(const float* __restrict__ x, float* __restrict__ y,
                                                       uint8_t* __restrict__ am, int B, int H, int W, int C, int k,
                                                       int s, int pad, int Ho, int Wo) {
  const long long total = (long long)B * Ho * Wo * (C / 4);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % (C / 4));
    const long long r = t / (C / 4);
    const int ow = (int)(r % Wo), oh = (int)((r / Wo) % Ho);
    const long long b = r / ((long long)Wo * Ho);
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int arg[4] = {-1, -1, -1, -1};
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - pad + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - pad + kw;
        if (iw < 0 || iw >= W) continue;
        const float4 v4 = *reinterpret_cast<const float4*>(x + ((b * H + ih) * W + iw) * C + c4 * 4);
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (arg[q] < 0) arg[q] = kh * k + kw;  // initial index: the first in-image tap
          if (v[q] > best[q] || v[q] != v[q]) {
            best[q] = v[q];
            arg[q] = kh * k + kw;
          }
        }
      }
    }
    *reinterpret_cast<float4*>(y + r * C + c4 * 4) = make_float4(best[0], best[1], best[2], best[3]);
    const unsigned packed = (unsigned)(arg[0] & 0xff) | ((unsigned)(arg[1] & 0xff) << 8) |
                            ((unsigned)(arg[2] & 0xff) << 16) | ((unsigned)(arg[3] & 0xff) << 24);
    *reinterpret_cast<unsigned*>(am + r * C + c4 * 4) = packed;
  }
}

// one block per (input row, 256-wide slice of the row's W x C/4 quads): the row (b, ih) and
// its output-row window range are block-uniform, the per-thread index math is 32-bit (the
// grid-stride version spent its time in 64-bit divisions: 222 us for the ResNet-50 stem at
// B=128, ~2x its HBM time)
__global__ __launch_bounds__(256) void maxpool_bwd_gather(const float* __restrict__ g, const uint8_t* __restrict__ am,
                                                          float* __restrict__ dx, int B, int H, int W, int C, int k,
                                                          int s, int pad, int Ho, int Wo, int cpr) {
  const int C4 = C / 4;
  const int row = blockIdx.x / cpr, chunk = blockIdx.x - row * cpr;  // row = b * H + ih
  const int q = chunk * 256 + threadIdx.x;
  if (q >= W * C4) return;
  const int b = row / H, ih = row - b * H;
  const int iw = q / C4, c4 = q - iw * C4;
  // windows oh with oh*s - pad <= ih <= oh*s - pad + k - 1
  const int oh0 = max(0, (ih + pad - k + s) / s), oh1 = min(Ho - 1, (ih + pad) / s);
  const int ow0 = max(0, (iw + pad - k + s) / s), ow1 = min(Wo - 1, (iw + pad) / s);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int oh = oh0; oh <= oh1; ++oh) {
    const int th = ih - (oh * s - pad);
    const size_t obase = ((size_t)b * Ho + oh) * Wo;
    for (int ow = ow0; ow <= ow1; ++ow) {
      const unsigned want = (unsigned)(th * k + iw - (ow * s - pad));
      const size_t o = (obase + ow) * C + c4 * 4;
      const unsigned a = *reinterpret_cast<const unsigned*>(am + o);
      const float4 gv = *reinterpret_cast<const float4*>(g + o);
      if ((a & 0xffu) == want) acc.x += gv.x;
      if (((a >> 8) & 0xffu) == want) acc.y += gv.y;
      if (((a >> 16) & 0xffu) == want) acc.z += gv.z;
      if ((a >> 24) == want) acc.w += gv.w;
    }
  }
  *reinterpret_cast<float4*>(dx + ((size_t)row * W + iw) * C + c4 * 4) = acc;
}

// global average pool backward: dx[b][p][c] = g[b][c] / HW
__global__ __launch_bounds__(256) void avgpool_bwd(const float* __restrict__ g, float* __restrict__ dx, int B, int HW,
                                                   int C) {
  const long long total = (long long)B * HW * (C / 4);
  const float inv = 1.f / (float)HW;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % (C / 4));
    const long long b = t / ((long long)(C / 4) * HW);
    const float4 v = *reinterpret_cast<const float4*>(g + b * C + c4 * 4);
    reinterpret_cast<float4*>(dx)[t] = make_float4(v.x * inv, v.y * inv, v.z * inv, v.w * inv);
  }
}

}  // namespace tp

extern "C" hipError_t tp_maxpool_fwd_arg(const float* x, float* y, uint8_t* am, int B, int H, int W, int C, int k,
                                         int s, int pad, hipStream_t st) {
  if (C % 4 || k < 1 || k * k > 255 || s < 1 || pad < 0 || 2 * pad > k) return hipErrorInvalidValue;
  const int Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  if (Ho <= 0 || Wo <= 0) return hipErrorInvalidValue;
  const long long total = (long long)B * Ho * Wo * (C / 4);
  if (total == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::maxpool_fwd_arg<<<grid, 256, 0, st>>>(x, y, am, B, H, W, C, k, s, pad, Ho, Wo);
  return hipGetLastError();
}

extern "C" hipError_t tp_maxpool_bwd(const float* g, const uint8_t* am, float* dx, int B, int H, int W, int C, int k,
                                     int s, int pad, hipStream_t st) {
  if (C % 4 || k < 1 || k * k > 255 || s < 1 || pad < 0 || 2 * pad > k) return hipErrorInvalidValue;
  const int Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  const long long total = (long long)B * H * W * (C / 4);
  if (total == 0) return hipSuccess;
  const int cpr = (int)tp::ceil_div((long long)W * (C / 4), 256);  // blocks per input row
  const long long blocks = (long long)B * H * cpr;
  if ((long long)W * (C / 4) >= (1ll << 31) || blocks >= (1ll << 31)) return hipErrorInvalidValue;
  tp::maxpool_bwd_gather<<<(unsigned)blocks, 256, 0, st>>>(g, am, dx, B, H, W, C, k, s, pad, Ho, Wo, cpr);
  return hipGetLastError();
}

extern "C" hipError_t tp_avgpool_bwd(const float* g, float* dx, int B, int HW, int C, hipStream_t st) {
  if (C % 4 || HW <= 0) return hipErrorInvalidValue;
  const long long total = (long long)B * HW * (C / 4);
  if (total == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::avgpool_bwd<<<grid, 256, 0, st>>>(g, dx, B, HW, C);
  return hipGetLastError();
}
