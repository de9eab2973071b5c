// Batched-prefix Monte-Carlo Shapley kernels and the fused
// cross-entropy used by the attribution engine (K8).
//
// The reference evaluates one permutation prefix at a time: `z.index_fill_(1,[i],0)`,
// one partial forward, then a device->host copy of the loss delta for every unit
// (shapley_values.py:51-61). Prefix losses L_0..L_n of one permutation are independent
// given their masks, so K prefixes are materialised in a single launch as a (K*B)
// batch (prefix_mask) and the K deltas are scattered on device (shapley_accumulate).
#include "tp_common.h"

namespace tp {

// out[k, e] = (rank[channel(e)] < p0 + k) ? 0 : z[e]  for e in [0, N), k in [0, K).
template <bool CL>
__global__ __launch_bounds__(256) void prefix_mask4(const float4* __restrict__ z, float4* __restrict__ out,
                                                    const int* __restrict__ rank, long long N4, int C, int S,
                                                    int p0, int K) {
  const long long total = N4 * K;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e4 = t % N4;
    const int k = (int)(t / N4);
    const int lim = p0 + k;
    float4 v = z[e4];
    const long long e = e4 * 4;
    if (CL) {
      const int c = (int)(e % C);
      if (rank[c] < lim) v.x = 0.f;
      if (rank[c + 1] < lim) v.y = 0.f;
      if (rank[c + 2] < lim) v.z = 0.f;
      if (rank[c + 3] < lim) v.w = 0.f;
    } else {
      const int c = (int)((e / S) % C);
      if (rank[c] < lim) v = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    out[t] = v;
  }
}

template <bool CL>
__global__ __launch_bounds__(256) void prefix_mask1(const float* __restrict__ z, float* __restrict__ out,
                                                    const int* __restrict__ rank, long long N, int C, int S,
                                                    int p0, int K) {
  const long long total = N * K;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long e = t % N;
    const int k = (int)(t / N);
    const int c = CL ? (int)(e % C) : (int)((e / S) % C);
    out[t] = rank[c] < p0 + k ? 0.f : z[e];
  }
}

// Prefix-delta operands (exact alternative to materialising K masked copies when the next layer
// is a Linear): for prefixes p0 .. p0+cnt-1 of permutation `perm`, copy j differs from the base
// prefix p0 by the units perm[p0], .., perm[p0+j-1] being zeroed as well, so its next-layer
// pre-activation is  Y0 - sum_{i<j} z[:, perm[p0+i]] W[:, perm[p0+i]]  = Y0 - (T @ Wsub^T)[j]:
//   T[(j*B + b)*Kc + i] = (i < j) ? z[b*C + perm[p0+i]] : 0     (cnt*B rows, Kc >= cnt columns)
//   Wsub[n*Kc + i]      = (i < cnt - 1) ? W[n*C + perm[p0+i]] : 0   (N rows)
// The K x (C-wide) GEMM of the masked copies becomes one (B x C) GEMM + one K x (Kc-wide) GEMM.
__global__ __launch_bounds__(256) void prefix_tri_operands(const float* __restrict__ z, const float* __restrict__ W,
                                                           const int* __restrict__ perm, int B, int C, int N,
                                                           int p0, int cnt, int Kc, float* __restrict__ T,
                                                           float* __restrict__ Wsub) {
  const long long nt = (long long)cnt * B * Kc, nw = (long long)N * Kc;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < nt + nw;
       t += (long long)gridDim.x * blockDim.x) {
    if (t < nt) {
      const int i = (int)(t % Kc);
      const long long r = t / Kc;
      const int b = (int)(r % B), j = (int)(r / B);
      T[t] = i < j ? z[(long long)b * C + perm[p0 + i]] : 0.f;
    } else {
      const long long u = t - nt;
      const int i = (int)(u % Kc), n = (int)(u / Kc);
      Wsub[u] = i < cnt - 1 ? W[(long long)n * C + perm[p0 + i]] : 0.f;  // column cnt-1 of T is 0
    }
  }
}

// Per-sample form: sv[(row0+b)*n + perm[k0+k]] += (L[k+1][b] - L[k][b]) * scale.
__global__ void shapley_scatter(const float* __restrict__ L, const int* __restrict__ perm,
                                double* __restrict__ sv, int row0, int B, int n, int k0, int K,
                                double scale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= K * B) return;
  const int k = t / B, b = t % B;
  const double d = ((double)L[(k + 1) * B + b] - (double)L[k * B + b]) * scale;
  sv[(long long)(row0 + b) * n + perm[k0 + k]] += d;
}

// Column form (reduction mean/sum): one wave per prefix step, fixed summation order.
__global__ __launch_bounds__(64) void shapley_column(const float* __restrict__ L, const int* __restrict__ perm,
                                                     double* __restrict__ sv_col, int B, int k0,
                                                     double scale) {
  const int k = blockIdx.x;
  double acc = 0.0;
  for (int b = threadIdx.x; b < B; b += 64)
    acc += (double)L[(k + 1) * B + b] - (double)L[k * B + b];
  acc = wave_sum(acc);
  if (threadIdx.x == 0) sv_col[perm[k0 + k]] += acc * scale;
}

// Fused softmax cross-entropy: per-sample loss and (optionally) dL/dlogits * gscale.
__global__ __launch_bounds__(256) void cross_entropy_fb(const float* __restrict__ logits,
                                                        const int64_t* __restrict__ target,
                                                        float* __restrict__ loss, float* __restrict__ grad,
                                                        int B, int NC, float gscale) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= B) return;
  const float* x = logits + (long long)wave * NC;
  float m = -INFINITY;
  for (int j = lane; j < NC; j += 64) m = nan_max(m, x[j]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = nan_max(m, __shfl_xor(m, off, 64));
  float s = 0.f;
  for (int j = lane; j < NC; j += 64) s += __expf(x[j] - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  const int64_t t = target[wave];
  if (lane == 0) loss[wave] = lse - x[t];
  if (grad) {
    float* g = grad + (long long)wave * NC;
    const float inv = 1.f / s;
    for (int j = lane; j < NC; j += 64) {
      float p = __expf(x[j] - m) * inv;
      g[j] = (p - (j == t ? 1.f : 0.f)) * gscale;
    }
  }
}

}  // namespace tp

extern "C" hipError_t tp_prefix_mask(const float* z, float* out, const int* rank, long long N, int C, int S,
                                     int channels_last, int p0, int K, hipStream_t st) {
  const bool vec = (N % 4 == 0) && (channels_last ? (C % 4 == 0) : (S % 4 == 0)) &&
                   (((uintptr_t)z | (uintptr_t)out) % 16 == 0);
  const long long total = (vec ? N / 4 : N) * K;
  if (total == 0) return hipSuccess;
  unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 8192);
  if (vec) {
    if (channels_last)
      tp::prefix_mask4<true><<<grid, 256, 0, st>>>((const float4*)z, (float4*)out, rank, N / 4, C, S, p0, K);
    else
      tp::prefix_mask4<false><<<grid, 256, 0, st>>>((const float4*)z, (float4*)out, rank, N / 4, C, S, p0, K);
  } else {
    if (channels_last) tp::prefix_mask1<true><<<grid, 256, 0, st>>>(z, out, rank, N, C, S, p0, K);
    else tp::prefix_mask1<false><<<grid, 256, 0, st>>>(z, out, rank, N, C, S, p0, K);
  }
  return hipGetLastError();
}

extern "C" hipError_t tp_shapley_scatter(const float* L, const int* perm, double* sv, int row0, int B, int n,
                                         int k0, int K, double scale, hipStream_t st) {
  if (K * B == 0) return hipSuccess;
  tp::shapley_scatter<<<tp::ceil_div((long long)K * B, 256), 256, 0, st>>>(L, perm, sv, row0, B, n, k0, K, scale);
  return hipGetLastError();
}

extern "C" hipError_t tp_shapley_column(const float* L, const int* perm, double* sv_col, int B, int k0, int K,
                                        double scale, hipStream_t st) {
  if (K == 0) return hipSuccess;
  tp::shapley_column<<<K, 64, 0, st>>>(L, perm, sv_col, B, k0, scale);
  return hipGetLastError();
}

extern "C" hipError_t tp_cross_entropy(const float* logits, const int64_t* target, float* loss, float* grad,
                                       int B, int NC, float gscale, hipStream_t st) {
  if (B == 0) return hipSuccess;
  tp::cross_entropy_fb<<<tp::ceil_div((long long)B * 64, 256), 256, 0, st>>>(logits, target, loss, grad, B, NC,
                                                                            gscale);
  return hipGetLastError();
}

extern "C" hipError_t tp_prefix_tri_operands(const float* z, const float* W, const int* perm, int B, int C, int N,
                                             int p0, int cnt, int Kc, float* T, float* Wsub, hipStream_t st) {
  if (cnt <= 0 || cnt > Kc || B <= 0 || N <= 0) return hipErrorInvalidValue;
  const long long total = (long long)cnt * B * Kc + (long long)N * Kc;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 8192);
  tp::prefix_tri_operands<<<grid, 256, 0, st>>>(z, W, perm, B, C, N, p0, cnt, Kc, T, Wsub);
  return hipGetLastError();
}
