// Pruner kernels.
//
// * channel_fill   — `index_fill_(1, idx, value)` used by the NaN probe (pruner.py:138-142)
//                    and by simulated-pruning ablations (nbVGG:1276).
// * nan_channels   — "which channels of this activation carry a NaN" (pruner.py:158-162),
//                    producing a per-channel flag vector in a single pass.
// * gather_multi   — one launch slicing up to 8 tensors {param, grad, optimizer states}
//                    along an axis with a shared keep-index list (pruner.py:106-112,
//                    opt_pruner.py:17-19 issue one ATen index_select per tensor).
#include "tp_common.h"

namespace tp {

__global__ void channel_fill(float* __restrict__ x, long long B, int C, long long S,
                             const int64_t* __restrict__ idx, int nidx, float value) {
  long long total = B * nidx * S;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    long long s = t % S;
    long long r = t / S;
    int i = (int)(r % nidx);
    long long b = r / nidx;
    x[(b * C + idx[i]) * S + s] = value;
  }
}

// flags[c] = 1 if any x[b, c, s] is NaN. One block per channel.
__global__ __launch_bounds__(256) void nan_channels(const float* __restrict__ x, long long B, int C,
                                                   long long S, uint8_t* __restrict__ flags) {
  const int c = blockIdx.x;
  int found = 0;
  for (long long t = threadIdx.x; t < B * S; t += blockDim.x) {
    long long b = t / S, s = t % S;
    float v = x[(b * C + c) * S + s];
    found |= (v != v);
  }
  found = __syncthreads_or(found);
  if (threadIdx.x == 0) flags[c] = (uint8_t)(found ? 1 : 0);
}

struct GatherDesc {
  const void* src;
  void* dst;
  long long outer;
  long long n;      // source extent along the sliced axis
  long long inner;  // elements after the axis
};

struct GatherBatch {
  GatherDesc d[8];
  int count;
};

template <typename T>
__global__ __launch_bounds__(256) void gather_multi(GatherBatch batch, const int64_t* __restrict__ keep,
                                                    long long nkeep) {
  const GatherDesc g = batch.d[blockIdx.y];
  const T* __restrict__ src = reinterpret_cast<const T*>(g.src);
  T* __restrict__ dst = reinterpret_cast<T*>(g.dst);
  const long long total = g.outer * nkeep * g.inner;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    long long i = t % g.inner;
    long long r = t / g.inner;
    long long j = r % nkeep;
    long long o = r / nkeep;
    dst[t] = src[(o * g.n + keep[j]) * g.inner + i];
  }
}

}  // namespace tp

extern "C" hipError_t tp_channel_fill(float* x, long long B, int C, long long S, const int64_t* idx,
                                      int nidx, float value, hipStream_t st) {
  long long total = B * nidx * S;
  if (total == 0) return hipSuccess;
  unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 4096);
  tp::channel_fill<<<grid, 256, 0, st>>>(x, B, C, S, idx, nidx, value);
  return hipGetLastError();
}

extern "C" hipError_t tp_nan_channels(const float* x, long long B, int C, long long S, uint8_t* flags,
                                      hipStream_t st) {
  if (C == 0) return hipSuccess;
  tp::nan_channels<<<C, 256, 0, st>>>(x, B, C, S, flags);
  return hipGetLastError();
}

// srcs/dsts/outer/n/inner arrays of length count (<= 8); elsize in {1,2,4,8} bytes.
extern "C" hipError_t tp_gather_multi(const void* const* srcs, void* const* dsts, const long long* outer,
                                      const long long* n, const long long* inner, int count, int elsize,
                                      const int64_t* keep, long long nkeep, hipStream_t st) {
  if (count <= 0 || count > 8) return hipErrorInvalidValue;
  tp::GatherBatch b{};
  b.count = count;
  long long maxtot = 0;
  for (int i = 0; i < count; ++i) {
    b.d[i] = tp::GatherDesc{srcs[i], dsts[i], outer[i], n[i], inner[i]};
    maxtot = std::max(maxtot, outer[i] * nkeep * inner[i]);
  }
  if (maxtot == 0) return hipSuccess;
  dim3 grid((unsigned)std::min<long long>(tp::ceil_div(maxtot, 256), 2048), count);
  switch (elsize) {
    case 1: tp::gather_multi<uint8_t><<<grid, 256, 0, st>>>(b, keep, nkeep); break;
    case 2: tp::gather_multi<uint16_t><<<grid, 256, 0, st>>>(b, keep, nkeep); break;
    case 4: tp::gather_multi<uint32_t><<<grid, 256, 0, st>>>(b, keep, nkeep); break;
    case 8: tp::gather_multi<uint64_t><<<grid, 256, 0, st>>>(b, keep, nkeep); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// NHWC 2x2/stride-2 max-pool with argmax bytes (NaN-propagating, first max wins like PyTorch's
// scan order (0,0),(0,1),(1,0),(1,1)) and its inverse scatter (unpool). Used by the fused
// engine when a layer runs as a dense GEMM (2x2 images) instead of a pooling conv kernel.
// ---------------------------------------------------------------------------------------------
namespace tp {
__global__ __launch_bounds__(256) void maxpool2_nhwc(const float* __restrict__ x, float* __restrict__ y,
                                                     uint8_t* __restrict__ am, int B, int H, int W, int C) {
  const int H2 = H / 2, W2 = W / 2;
  const long long total = (long long)B * H2 * W2 * C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long r = t / C;
    const int ow = (int)(r % W2), oh = (int)((r / W2) % H2);
    const long long b = r / ((long long)W2 * H2);
    float best = 0.f;
    int arg = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = x[((b * H + 2 * oh + (q >> 1)) * W + 2 * ow + (q & 1)) * C + c];
      if (q == 0 || v > best || (v != v && best == best)) {
        best = v;
        arg = q;
      }
    }
    y[t] = best;
    am[t] = (uint8_t)arg;
  }
}

__global__ __launch_bounds__(256) void unpool2_nhwc(const float* __restrict__ g, const uint8_t* __restrict__ am,
                                                    float* __restrict__ out, int B, int H, int W, int C) {
  const long long total = (long long)B * H * W * C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long r = t / C;
    const int iw = (int)(r % W), ih = (int)((r / W) % H);
    const long long b = r / ((long long)W * H);
    const long long o = ((b * (H / 2) + ih / 2) * (W / 2) + iw / 2) * C + c;
    out[t] = am[o] == (uint8_t)((ih & 1) * 2 + (iw & 1)) ? g[o] : 0.f;
  }
}

// C % 4 == 0: one thread per (pooled pixel, 4-channel group) reads a float4 of the pooled grad
// and its 4 argmax bytes once and writes the 2x2 window as four float4 rows (16-B stores,
// consecutive lanes on consecutive channel groups). Feeds the staged Winograd dgrad a dense
// full-resolution operand instead of rebuilding it per MFMA chunk.
__global__ __launch_bounds__(256) void unpool2_nhwc_v4(const float4* __restrict__ g, const uint32_t* __restrict__ am,
                                                       float4* __restrict__ out, int W2, int C4, long long total) {
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % C4);
    const long long p = t / C4;  // pooled pixel (b, ph, pw) = b * H2 * W2 + ph * W2 + pw
    const long long row = p / W2;  // b * H2 + ph
    const int pw = (int)(p - row * W2);
    const float4 v = g[t];
    const uint32_t a = am[t];
    const long long o00 = ((row * 2) * (2 * W2) + 2 * pw) * C4 + c4;  // full-res (2ph, 2pw)
    const long long drow = (long long)(2 * W2) * C4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 r;
      r.x = ((a >> 0) & 0xffu) == (uint32_t)q ? v.x : 0.f;
      r.y = ((a >> 8) & 0xffu) == (uint32_t)q ? v.y : 0.f;
      r.z = ((a >> 16) & 0xffu) == (uint32_t)q ? v.z : 0.f;
      r.w = ((a >> 24) & 0xffu) == (uint32_t)q ? v.w : 0.f;
      out[o00 + (q >> 1) * drow + (q & 1) * C4] = r;
    }
  }
}
}  // namespace tp

extern "C" hipError_t tp_maxpool2_nhwc(const float* x, float* y, uint8_t* am, int B, int H, int W, int C,
                                       hipStream_t st) {
  const long long total = (long long)B * (H / 2) * (W / 2) * C;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::maxpool2_nhwc<<<grid, 256, 0, st>>>(x, y, am, B, H, W, C);
  return hipGetLastError();
}

extern "C" hipError_t tp_unpool2_nhwc(const float* g, const uint8_t* am, float* out, int B, int H, int W, int C,
                                      hipStream_t st) {
  if (C % 4 == 0 && H % 2 == 0 && W % 2 == 0 && (reinterpret_cast<uintptr_t>(g) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (reinterpret_cast<uintptr_t>(am) & 3) == 0) {
    const long long total = (long long)B * (H / 2) * (W / 2) * (C / 4);
    const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
    tp::unpool2_nhwc_v4<<<grid, 256, 0, st>>>(reinterpret_cast<const float4*>(g),
                                              reinterpret_cast<const uint32_t*>(am), reinterpret_cast<float4*>(out),
                                              W / 2, C / 4, total);
    return hipGetLastError();
  }
  const long long total = (long long)B * H * W * C;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::unpool2_nhwc<<<grid, 256, 0, st>>>(g, am, out, B, H, W, C);
  return hipGetLastError();
}

// Generic NHWC max-pool (k x k, stride s, zero-free padding p: padded taps are skipped, as in
// PyTorch) with NaN propagation, and global average pooling NHWC -> (B, C).
namespace tp {
__global__ __launch_bounds__(256) void maxpool_nhwc(const float* __restrict__ x, float* __restrict__ y, int B, int H,
                                                    int W, int C, int k, int s, int pad, int Ho, int Wo) {
  const long long total = (long long)B * Ho * Wo * (C / 4);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % (C / 4));
    const long long r = t / (C / 4);
    const int ow = (int)(r % Wo), oh = (int)((r / Wo) % Ho);
    const long long b = r / ((long long)Wo * Ho);
    float4 best = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - pad + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - pad + kw;
        if (iw < 0 || iw >= W) continue;
        const float4 v = *reinterpret_cast<const float4*>(x + ((b * H + ih) * W + iw) * C + c4 * 4);
        best.x = nan_max(best.x, v.x);
        best.y = nan_max(best.y, v.y);
        best.z = nan_max(best.z, v.z);
        best.w = nan_max(best.w, v.w);
      }
    }
    *reinterpret_cast<float4*>(y + r * C + c4 * 4) = best;
  }
}

__global__ __launch_bounds__(256) void avgpool_nhwc(const float* __restrict__ x, float* __restrict__ y, int B, int HW,
                                                    int C) {
  const long long total = (long long)B * C;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % C);
    const long long b = t / C;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += x[(b * HW + i) * C + c];
    y[t] = s / (float)HW;
  }
}
}  // namespace tp

extern "C" hipError_t tp_maxpool_nhwc(const float* x, float* y, int B, int H, int W, int C, int k, int s, int pad,
                                      hipStream_t st) {
  if (C % 4 != 0) return hipErrorInvalidValue;
  const int Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  const long long total = (long long)B * Ho * Wo * (C / 4);
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::maxpool_nhwc<<<grid, 256, 0, st>>>(x, y, B, H, W, C, k, s, pad, Ho, Wo);
  return hipGetLastError();
}

extern "C" hipError_t tp_avgpool_nhwc(const float* x, float* y, int B, int HW, int C, hipStream_t st) {
  const long long total = (long long)B * C;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::avgpool_nhwc<<<grid, 256, 0, st>>>(x, y, B, HW, C);
  return hipGetLastError();
}
