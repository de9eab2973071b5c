// Training-mode BatchNorm2d on NHWC activations: batch statistics,
// normalisation and the backward pass of the finetune loop, deterministic (fixed-order
// two-level reductions, no atomics).
//
//   x: P rows (= B*H*W pixels) x C channels. C % 4 == 0: float4 rows (V4); any other C (pruned
//      widths left unpadded): the same kernels with per-element loads (scalar tail per row)
//   Cr <= C: channels carrying parameters (gamma / beta / running statistics); channels c >= Cr
//      are the zero padding of a pruned width carried at the kernels' granule: a = b = 0 there,
//      so they stay exact zeros forward and backward, and no statistic is written for them
//   stats   : partial[g][0|1][c] = sum / sum of squares over row group g  (pass 1)
//             finalize: mean, biased var -> invstd, running-stat update  (pass 2, fp64)
//   forward : y = x * a[c] + b[c],  a = gamma * invstd, b = beta - mean * a
//   backward: partial sums of g and g * xhat (pass 1), finalize -> (sum_g, sum_gxhat),
//             dx = a * (g - sum_g / P - xhat * sum_gxhat / P)
//
// A block owns a 64-wide column quad range (16 threads x float4) x 16 row lanes, and walks
// rows_per_group rows; the 16 row lanes are folded in LDS in a fixed order.
#include "tp_common.h"

namespace tp {

constexpr int BN_T = 256, BN_CQ = 16, BN_RL = BN_T / BN_CQ;  // 16 column quads x 16 row lanes

// MODE 0: (sum x, sum x^2); MODE 1: (sum g, sum g * (x - mean) * invstd)
// ReLU backward through the block's output y (MODE 1, ym non-null): the gradient reaching the BN
// is g where y > 0 and 0 elsewhere (NaN y -> 0, as the ATen threshold backward)
// or, cheaper, by the forward's ReLU bit mask mk (one byte per 4 channels, bit q = y[c+q] > 0:
// 1/16 of the bytes of reading y back)
// The ReLU bit mask: byte i holds flat elements 4i..4i+3 of the (P, C) activation (bit q = element
// 4i + q > 0) — for C % 4 == 0 that is "byte p*C/4 + c/4, bit = c % 4".
__device__ __forceinline__ float4 relu_mask4(float4 d, const float* ym, size_t off, const uint8_t* mk = nullptr) {
  if (mk) {
    const unsigned m = mk[off >> 2];
    return make_float4((m & 1u) ? d.x : 0.f, (m & 2u) ? d.y : 0.f, (m & 4u) ? d.z : 0.f, (m & 8u) ? d.w : 0.f);
  }
  if (!ym) return d;
  const float4 m = *reinterpret_cast<const float4*>(ym + off);
  return make_float4(m.x > 0.f ? d.x : 0.f, m.y > 0.f ? d.y : 0.f, m.z > 0.f ? d.z : 0.f, m.w > 0.f ? d.w : 0.f);
}

// 4 channels c..c+3 of row r: one float4 (V4) or per-element loads guarded by c + q < C
template <bool V4>
__device__ __forceinline__ float4 ld4(const float* __restrict__ t, size_t row_off, int c, int C) {
  if (V4) return *reinterpret_cast<const float4*>(t + row_off + c);
  const float* q = t + row_off + c;
  return make_float4(q[0], c + 1 < C ? q[1] : 0.f, c + 2 < C ? q[2] : 0.f, c + 3 < C ? q[3] : 0.f);
}
// relu_mask4 for any C: element e = off + q reads bit (e & 3) of byte e >> 2
template <bool V4>
__device__ __forceinline__ float4 relu_mask4g(float4 d, const float* ym, size_t off, const uint8_t* mk, int c, int C) {
  if (V4) return relu_mask4(d, ym, off, mk);
  float v[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t e = off + q;
    bool keep = true;
    if (c + q >= C) keep = false;
    else if (mk) keep = (mk[e >> 2] >> (e & 3)) & 1u;
    else if (ym) keep = ym[e] > 0.f;
    v[q] = keep ? v[q] : 0.f;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

template <int MODE, bool V4 = true>
__global__ __launch_bounds__(BN_T) void bn_partial(const float* __restrict__ x, const float* __restrict__ g,
                                                   const float* __restrict__ mean, const float* __restrict__ invstd,
                                                   double* __restrict__ part, int P, int C, int rows_per_group,
                                                   const float* __restrict__ ym = nullptr,
                                                   const uint8_t* __restrict__ mk = nullptr) {
  __shared__ double red[2][BN_RL][BN_CQ * 4];
  const int cq = threadIdx.x % BN_CQ, rl = threadIdx.x / BN_CQ;
  const int c = (blockIdx.x * BN_CQ + cq) * 4;
  const int r0 = blockIdx.y * rows_per_group, r1 = min(P, r0 + rows_per_group);
  float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
  if (c < C) {
    float4 mu = s0, is = s0;
    if (MODE == 1) {
      mu = ld4<V4>(mean, 0, c, C);
      is = ld4<V4>(invstd, 0, c, C);
    }
    // 4 independent rows per iteration: 4 (8 in backward) loads in flight per thread
    constexpr int U = 4;
    int r = r0 + rl;
    for (; r + (U - 1) * BN_RL < r1; r += U * BN_RL) {
      float4 v[U], d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = ld4<V4>(x, (size_t)(r + u * BN_RL) * C, c, C);
        if (MODE == 1)
          d[u] = relu_mask4g<V4>(ld4<V4>(g, (size_t)(r + u * BN_RL) * C, c, C), ym, (size_t)(r + u * BN_RL) * C + c,
                                 mk, c, C);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (MODE == 0) {
          s0.x += v[u].x;
          s0.y += v[u].y;
          s0.z += v[u].z;
          s0.w += v[u].w;
          s1.x += v[u].x * v[u].x;
          s1.y += v[u].y * v[u].y;
          s1.z += v[u].z * v[u].z;
          s1.w += v[u].w * v[u].w;
        } else {
          s0.x += d[u].x;
          s0.y += d[u].y;
          s0.z += d[u].z;
          s0.w += d[u].w;
          s1.x += d[u].x * (v[u].x - mu.x) * is.x;
          s1.y += d[u].y * (v[u].y - mu.y) * is.y;
          s1.z += d[u].z * (v[u].z - mu.z) * is.z;
          s1.w += d[u].w * (v[u].w - mu.w) * is.w;
        }
      }
    }
    for (; r < r1; r += BN_RL) {
      const float4 v = ld4<V4>(x, (size_t)r * C, c, C);
      if (MODE == 0) {
        s0.x += v.x;
        s0.y += v.y;
        s0.z += v.z;
        s0.w += v.w;
        s1.x += v.x * v.x;
        s1.y += v.y * v.y;
        s1.z += v.z * v.z;
        s1.w += v.w * v.w;
      } else {
        const float4 d = relu_mask4g<V4>(ld4<V4>(g, (size_t)r * C, c, C), ym, (size_t)r * C + c, mk, c, C);
        s0.x += d.x;
        s0.y += d.y;
        s0.z += d.z;
        s0.w += d.w;
        s1.x += d.x * (v.x - mu.x) * is.x;
        s1.y += d.y * (v.y - mu.y) * is.y;
        s1.z += d.z * (v.z - mu.z) * is.z;
        s1.w += d.w * (v.w - mu.w) * is.w;
      }
    }
  }
  red[0][rl][cq * 4 + 0] = s0.x;
  red[0][rl][cq * 4 + 1] = s0.y;
  red[0][rl][cq * 4 + 2] = s0.z;
  red[0][rl][cq * 4 + 3] = s0.w;
  red[1][rl][cq * 4 + 0] = s1.x;
  red[1][rl][cq * 4 + 1] = s1.y;
  red[1][rl][cq * 4 + 2] = s1.z;
  red[1][rl][cq * 4 + 3] = s1.w;
  __syncthreads();
  if (threadIdx.x < 2 * BN_CQ * 4) {
    const int which = threadIdx.x / (BN_CQ * 4), col = threadIdx.x % (BN_CQ * 4);
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < BN_RL; ++i) t += red[which][i][col];
    const int cc = blockIdx.x * BN_CQ * 4 + col;
    if (cc < C) part[((size_t)blockIdx.y * 2 + which) * C + cc] = t;
  }
}

// Sum of the row-group partials of 16 channels per block (1024 threads): 64 group lanes stride
// over the groups (coalesced 16-channel rows), then lane 0 folds the 64 lane sums in order
// (deterministic). 64 lanes, not 16: the 64-channel BNs of the 56-px stage have 1024 groups and
// only 4 blocks, and the finalize ran ~22 us there as a chain of 64 dependent load pairs.
// TP_BN_FOLD_LANES=16: the previous 16-lane fold order (bit-identical statistics to round-5
// builds before this change; diagnostic of training-trajectory sensitivity, scripts/probes/)
constexpr int BN_FIN_T = 1024, BN_FIN_GL = BN_FIN_T / 16;
static int bn_fold_lanes() {
  static const int l = [] {
    const char* e = getenv("TP_BN_FOLD_LANES");
    const int v = e ? atoi(e) : BN_FIN_GL;
    return v == 16 ? 16 : BN_FIN_GL;
  }();
  return l;
}
__device__ __forceinline__ void fold_groups(const double* __restrict__ part, int groups, int C, int c, int cl, int gl,
                                            int lanes, double& s, double& q) {
  __shared__ double red[2][BN_FIN_GL][16];
  s = 0.0;
  q = 0.0;
  if (c < C && gl < lanes)
    for (int i = gl; i < groups; i += lanes) {
      s += part[(size_t)(2 * i) * C + c];
      q += part[(size_t)(2 * i + 1) * C + c];
    }
  red[0][gl][cl] = s;
  red[1][gl][cl] = q;
  __syncthreads();
  if (gl != 0) return;
  s = 0.0;
  q = 0.0;
  for (int i = 0; i < lanes; ++i) {
    s += red[0][i][cl];
    q += red[1][i][cl];
  }
}

// Forward finalize: mean / invstd for the apply pass, running statistics (PyTorch semantics:
// running_var takes the unbiased variance), and the affine folded into (a, b).
__global__ __launch_bounds__(BN_FIN_T) void bn_fwd_finalize(const double* __restrict__ part, int groups, int P, int C,
                                                       int Cr,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, float momentum, float* __restrict__ run_mean,
                                                       float* __restrict__ run_var, float* __restrict__ mean,
                                                       float* __restrict__ invstd, float* __restrict__ a,
                                                       float* __restrict__ b, long long* __restrict__ nbt, int lanes) {
  const int cl = threadIdx.x % 16, gl = threadIdx.x / 16, c = blockIdx.x * 16 + cl;
  // the module's num_batches_tracked += 1 (one lane, plain vector store): no separate add launch
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  double s, q;
  fold_groups(part, groups, C, c, cl, gl, lanes, s, q);
  if (gl != 0 || c >= C) return;
  const double m = s / P;
  const double var = fmax(q / P - m * m, 0.0);
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)m;
  invstd[c] = is;
  if (c >= Cr) {  // zero padding of a pruned width: stays zero
    a[c] = 0.f;
    b[c] = 0.f;
    return;
  }
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)m;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)(P > 1 ? var * P / (P - 1) : var);
  }
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  a[c] = ga * is;
  b[c] = be - (float)m * ga * is;
}

// Backward finalize: dgamma = sum(g * xhat), dbeta = sum(g), and the coefficients of
// dx = a * g + k1 + k2 * x  (k1, k2 fold the mean-subtraction terms).
__global__ __launch_bounds__(BN_FIN_T) void bn_bwd_finalize(const double* __restrict__ part, int groups, int P, int C,
                                                       int Cr,
                                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                       float* __restrict__ dbeta, float* __restrict__ a,
                                                       float* __restrict__ k1, float* __restrict__ k2, int lanes) {
  const int cl = threadIdx.x % 16, gl = threadIdx.x / 16, c = blockIdx.x * 16 + cl;
  double sg, sgx;
  fold_groups(part, groups, C, c, cl, gl, lanes, sg, sgx);
  if (gl != 0 || c >= C) return;
  if (c >= Cr) {
    a[c] = 0.f;
    k1[c] = 0.f;
    k2[c] = 0.f;
    return;
  }
  if (dgamma) dgamma[c] = (float)sgx;
  if (dbeta) dbeta[c] = (float)sg;
  const double is = invstd[c], ga = gamma ? gamma[c] : 1.0;
  const double ac = ga * is;
  // dx = ac * (g - sg/P - xhat * sgx/P), xhat = (x - mean) * is
  a[c] = (float)ac;
  k2[c] = (float)(-ac * is * sgx / P);
  k1[c] = (float)(-ac * sg / P - (-ac * is * sgx / P) * mean[c]);
}

// forward: y = act(x*a + b (+ res));  backward: dx = gm*a + k1 + k2*x with gm = g masked by the
// ReLU output ym (when given), and dres = gm (the residual branch's gradient) when requested
template <bool BWD>
__global__ __launch_bounds__(256) void bn_apply(const float* __restrict__ x, const float* __restrict__ g,
                                                const float* __restrict__ a, const float* __restrict__ b,
                                                const float* __restrict__ k2, float* __restrict__ out, unsigned n4,
                                                unsigned C4, const float* __restrict__ res = nullptr, int relu = 0,
                                                const float* __restrict__ ym = nullptr,
                                                float* __restrict__ dres = nullptr,
                                                uint8_t* __restrict__ mk = nullptr);

// bn_apply for C % 4 != 0: thread t owns flat elements 4t..4t+3 (< n) — the ReLU mask byte t —
// each with its own channel (e % C), per-element loads and stores
template <bool BWD>
__global__ __launch_bounds__(256) void bn_apply_any(const float* __restrict__ x, const float* __restrict__ g,
                                                    const float* __restrict__ a, const float* __restrict__ b,
                                                    const float* __restrict__ k2, float* __restrict__ out,
                                                    unsigned long long n, unsigned C,
                                                    const float* __restrict__ res = nullptr, int relu = 0,
                                                    const float* __restrict__ ym = nullptr,
                                                    float* __restrict__ dres = nullptr,
                                                    uint8_t* __restrict__ mk = nullptr) {
  const unsigned long long n4 = (n + 3) / 4;
  for (unsigned long long t = blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += (unsigned long long)gridDim.x * blockDim.x) {
    unsigned bits = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned long long e = 4 * t + q;
      if (e >= n) break;
      const unsigned c = (unsigned)(e % C);
      const float v = x[e];
      if (BWD) {
        float d = g[e];
        if (mk) d = ((mk[t] >> q) & 1u) ? d : 0.f;
        else if (ym) d = ym[e] > 0.f ? d : 0.f;
        if (dres) dres[e] = d;
        if (out) out[e] = d * a[c] + b[c] + k2[c] * v;
      } else {
        float o = v * a[c] + b[c];
        if (res) o += res[e];
        if (relu) {
          o = nan_relu(o);
          bits |= o > 0.f ? (1u << q) : 0u;
        }
        out[e] = o;
      }
    }
    if (!BWD && relu && mk) mk[t] = (uint8_t)bits;
  }
}

template <bool BWD>
__global__ __launch_bounds__(256) void bn_apply(const float* __restrict__ x, const float* __restrict__ g,
                                                const float* __restrict__ a, const float* __restrict__ b,
                                                const float* __restrict__ k2, float* __restrict__ out, unsigned n4,
                                                unsigned C4, const float* __restrict__ res, int relu,
                                                const float* __restrict__ ym, float* __restrict__ dres,
                                                uint8_t* __restrict__ mk) {
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += gridDim.x * blockDim.x) {
    const unsigned c = (t % C4) * 4;
    const float4 v = reinterpret_cast<const float4*>(x)[t];
    const float4 av = *reinterpret_cast<const float4*>(a + c);
    const float4 bv = *reinterpret_cast<const float4*>(b + c);
    float4 o;
    if (BWD) {
      const float4 d = relu_mask4(reinterpret_cast<const float4*>(g)[t], ym, (size_t)t * 4, mk);
      if (dres) reinterpret_cast<float4*>(dres)[t] = d;
      if (!out) continue;
      const float4 kv = *reinterpret_cast<const float4*>(k2 + c);
      o.x = d.x * av.x + bv.x + kv.x * v.x;
      o.y = d.y * av.y + bv.y + kv.y * v.y;
      o.z = d.z * av.z + bv.z + kv.z * v.z;
      o.w = d.w * av.w + bv.w + kv.w * v.w;
    } else {
      o.x = v.x * av.x + bv.x;
      o.y = v.y * av.y + bv.y;
      o.z = v.z * av.z + bv.z;
      o.w = v.w * av.w + bv.w;
      if (res) {
        const float4 rv = reinterpret_cast<const float4*>(res)[t];
        o.x += rv.x;
        o.y += rv.y;
        o.z += rv.z;
        o.w += rv.w;
      }
      if (relu) {
        o.x = nan_relu(o.x);
        o.y = nan_relu(o.y);
        o.z = nan_relu(o.z);
        o.w = nan_relu(o.w);
        if (mk)  // the backward's ReLU mask: bit q = output channel c+q is > 0
          mk[t] = (uint8_t)((o.x > 0.f ? 1u : 0u) | (o.y > 0.f ? 2u : 0u) | (o.z > 0.f ? 4u : 0u) |
                            (o.w > 0.f ? 8u : 0u));
      }
    }
    reinterpret_cast<float4*>(out)[t] = o;
  }
}

// Fold [G][2][C] per-tile statistics (written by a conv epilogue) into [G2][2][C] groups for
// bn_fwd_finalize: block (64-channel slice, output group) sums its tiles with 4 lanes per
// channel and a fixed-order LDS fold (deterministic).
__global__ __launch_bounds__(256) void bn_fold_tiles(const double* __restrict__ in, int G, int C,
                                                     double* __restrict__ out, int per) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
  const int g0 = blockIdx.y * per, g1 = min(G, g0 + per);
  double s = 0.0, q = 0.0;
  if (c < C)
    for (int g = g0 + lane; g < g1; g += 4) {
      s += in[(size_t)(2 * g) * C + c];
      q += in[(size_t)(2 * g + 1) * C + c];
    }
  red[0][lane][cl] = s;
  red[1][lane][cl] = q;
  __syncthreads();
  if (lane < 2 && c < C) {
    const double t = red[lane][0][cl] + red[lane][1][cl] + red[lane][2][cl] + red[lane][3][cl];
    out[((size_t)blockIdx.y * 2 + lane) * C + c] = t;
  }
}

inline int bn_groups(int P, int C) {
  const int col_blocks = (C + BN_CQ * 4 - 1) / (BN_CQ * 4);
  int groups = std::max(1, std::min(1024, 1024 / std::max(1, col_blocks)));
  return std::min(groups, std::max(1, P / 64));
}

}  // namespace tp

// Workspace: ws holds 2 * groups * C doubles (groups = tp_bn_groups(P, C)).
extern "C" int tp_bn_groups(int P, int C) { return tp::bn_groups(P, C); }

namespace tp {
// launch bn_apply (float4 rows) or bn_apply_any (per-element) over the whole (P, C) activation
template <bool BWD>
static void apply_launch(const float* x, const float* g, const float* a, const float* b, const float* k2, float* out,
                         long long P, int C, const float* res, int relu, const float* ym, float* dres, uint8_t* mk,
                         hipStream_t st) {
  const long long n = P * C;
  if (C % 4 == 0) {
    const unsigned n4 = (unsigned)(n / 4);
    bn_apply<BWD><<<(unsigned)std::min<long long>(ceil_div((long long)n4, 256), 8192), 256, 0, st>>>(
        x, g, a, b, k2, out, n4, (unsigned)(C / 4), res, relu, ym, dres, mk);
  } else {
    const long long n4 = (n + 3) / 4;
    bn_apply_any<BWD><<<(unsigned)std::min<long long>(ceil_div(n4, 256), 8192), 256, 0, st>>>(
        x, g, a, b, k2, out, (unsigned long long)n, (unsigned)C, res, relu, ym, dres, mk);
  }
}

template <int MODE>
static void partial_launch(dim3 grid, const float* x, const float* g, const float* mean, const float* invstd,
                           double* ws, int P, int C, int rpg, const float* ym, const uint8_t* mk, hipStream_t st) {
  if (C % 4 == 0) bn_partial<MODE, true><<<grid, BN_T, 0, st>>>(x, g, mean, invstd, ws, P, C, rpg, ym, mk);
  else bn_partial<MODE, false><<<grid, BN_T, 0, st>>>(x, g, mean, invstd, ws, P, C, rpg, ym, mk);
}
}  // namespace tp

// Fused block tail: y = relu?(BN(x) + res?) (res: the residual branch, same shape as x). Any C;
// channels c >= Cr are zero padding (no parameters, outputs 0).
// mko (nullable, relu only): the ReLU bit mask, ceil(P*C/4) bytes (byte i, bit q = flat element 4i+q > 0)
extern "C" hipError_t tp_bn_fwd_train5(const float* x, float* y, int P, int C, int Cr, const float* gamma,
                                       const float* beta, float eps, float momentum, float* run_mean, float* run_var,
                                       float* mean, float* invstd, float* a, float* b, double* ws, const float* res,
                                       int relu, uint8_t* mko, long long* nbt, hipStream_t st) {
  using namespace tp;
  if (C <= 0 || P <= 0 || Cr <= 0 || Cr > C || (long long)P * C >= (1ll << 32)) return hipErrorInvalidValue;
  const int groups = bn_groups(P, C);
  const int rpg = (P + groups - 1) / groups;
  const dim3 grid((C + BN_CQ * 4 - 1) / (BN_CQ * 4), groups);
  partial_launch<0>(grid, x, nullptr, nullptr, nullptr, ws, P, C, rpg, nullptr, nullptr, st);
  bn_fwd_finalize<<<(C + 15) / 16, BN_FIN_T, 0, st>>>(ws, groups, P, C, Cr, gamma, beta, eps, momentum, run_mean,
                                                    run_var, mean, invstd, a, b, nbt, bn_fold_lanes());
  apply_launch<false>(x, nullptr, a, b, nullptr, y, P, C, res, relu, nullptr, nullptr, relu ? mko : nullptr, st);
  return hipGetLastError();
}

extern "C" hipError_t tp_bn_fwd_train4(const float* x, float* y, int P, int C, const float* gamma, const float* beta,
                                       float eps, float momentum, float* run_mean, float* run_var, float* mean,
                                       float* invstd, float* a, float* b, double* ws, const float* res, int relu,
                                       uint8_t* mko, long long* nbt, hipStream_t st) {
  return tp_bn_fwd_train5(x, y, P, C, C, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, a, b, ws, res,
                          relu, mko, nbt, st);
}

// Forward with the batch statistics already reduced per conv tile (``pre``: [G][2][C] sums and
// sums of squares over the tiles' rows, from the producing conv's epilogue): no statistics pass
// over x. ws holds 2 * min(G, 256) * C doubles.
extern "C" hipError_t tp_bn_fwd_train_pre2(const float* x, float* y, int P, int C, int Cr, const float* gamma,
                                           const float* beta, float eps, float momentum, float* run_mean,
                                           float* run_var, float* mean, float* invstd, float* a, float* b,
                                           double* ws, const double* pre, int G, const float* res, int relu,
                                           uint8_t* mko, long long* nbt, hipStream_t st) {
  using namespace tp;
  if (C <= 0 || P <= 0 || Cr <= 0 || Cr > C || G <= 0 || (long long)P * C >= (1ll << 32)) return hipErrorInvalidValue;
  const int G2 = std::min(G, 256), per = (G + G2 - 1) / G2;
  const int groups = (G + per - 1) / per;
  bn_fold_tiles<<<dim3((C + 63) / 64, groups), 256, 0, st>>>(pre, G, C, ws, per);
  bn_fwd_finalize<<<(C + 15) / 16, BN_FIN_T, 0, st>>>(ws, groups, P, C, Cr, gamma, beta, eps, momentum, run_mean,
                                                    run_var, mean, invstd, a, b, nbt, bn_fold_lanes());
  apply_launch<false>(x, nullptr, a, b, nullptr, y, P, C, res, relu, nullptr, nullptr, relu ? mko : nullptr, st);
  return hipGetLastError();
}

extern "C" hipError_t tp_bn_fwd_train_pre(const float* x, float* y, int P, int C, const float* gamma,
                                          const float* beta, float eps, float momentum, float* run_mean,
                                          float* run_var, float* mean, float* invstd, float* a, float* b,
                                          double* ws, const double* pre, int G, const float* res, int relu,
                                          uint8_t* mko, long long* nbt, hipStream_t st) {
  return tp_bn_fwd_train_pre2(x, y, P, C, C, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, a, b, ws,
                              pre, G, res, relu, mko, nbt, st);
}

// num_batches_tracked-free entry (``nbt`` = null)
extern "C" hipError_t tp_bn_fwd_train3(const float* x, float* y, int P, int C, const float* gamma, const float* beta,
                                       float eps, float momentum, float* run_mean, float* run_var, float* mean,
                                       float* invstd, float* a, float* b, double* ws, const float* res, int relu,
                                       uint8_t* mko, hipStream_t st) {
  return tp_bn_fwd_train4(x, y, P, C, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, a, b, ws, res, relu,
                          mko, nullptr, st);
}

extern "C" hipError_t tp_bn_fwd_train2(const float* x, float* y, int P, int C, const float* gamma, const float* beta,
                                       float eps, float momentum, float* run_mean, float* run_var, float* mean,
                                       float* invstd, float* a, float* b, double* ws, const float* res, int relu,
                                       hipStream_t st) {
  return tp_bn_fwd_train3(x, y, P, C, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, a, b, ws, res, relu,
                          nullptr, st);
}

extern "C" hipError_t tp_bn_fwd_train(const float* x, float* y, int P, int C, const float* gamma, const float* beta,
                                      float eps, float momentum, float* run_mean, float* run_var, float* mean,
                                      float* invstd, float* a, float* b, double* ws, hipStream_t st) {
  return tp_bn_fwd_train2(x, y, P, C, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, a, b, ws, nullptr,
                          0, st);
}

// Backward of the fused tail: ym = the block output y (ReLU mask; nullable), dres = gradient of
// the residual input (nullable). dx nullable (dgamma / dbeta only). Channels c >= Cr: padding
// (dx = 0 there, no dgamma / dbeta written).
// mk (nullable): the forward's ReLU bit mask, used instead of ym
extern "C" hipError_t tp_bn_bwd_train4(const float* g, const float* x, float* dx, int P, int C, int Cr,
                                       const float* gamma, const float* mean, const float* invstd, float* dgamma,
                                       float* dbeta, float* a, float* k1, float* k2, double* ws, const float* ym,
                                       float* dres, const uint8_t* mk, hipStream_t st) {
  using namespace tp;
  if (C <= 0 || P <= 0 || Cr <= 0 || Cr > C || (long long)P * C >= (1ll << 32)) return hipErrorInvalidValue;
  const int groups = bn_groups(P, C);
  const int rpg = (P + groups - 1) / groups;
  const dim3 grid((C + BN_CQ * 4 - 1) / (BN_CQ * 4), groups);
  partial_launch<1>(grid, x, g, mean, invstd, ws, P, C, rpg, ym, mk, st);
  bn_bwd_finalize<<<(C + 15) / 16, BN_FIN_T, 0, st>>>(ws, groups, P, C, Cr, gamma, mean, invstd, dgamma, dbeta, a, k1,
                                                      k2, bn_fold_lanes());
  if (dx || dres)
    apply_launch<true>(x, g, a, k1, k2, dx, P, C, nullptr, 0, ym, dres, const_cast<uint8_t*>(mk), st);
  return hipGetLastError();
}

// Backward with the statistics (sum gm, sum gm * xhat) already reduced per conv tile by the GEMM
// epilogue that produced g (``pre``: [G][2][C], tp_conv_gen5's bnb mode): no statistics pass over
// g and x. ws holds 2 * min(G, 256) * C doubles.
extern "C" hipError_t tp_bn_bwd_train_pre(const float* g, const float* x, float* dx, int P, int C, int Cr,
                                          const float* gamma, const float* mean, const float* invstd, float* dgamma,
                                          float* dbeta, float* a, float* k1, float* k2, double* ws, const double* pre,
                                          int G, const float* ym, float* dres, const uint8_t* mk, hipStream_t st) {
  using namespace tp;
  if (C <= 0 || P <= 0 || Cr <= 0 || Cr > C || G <= 0 || (long long)P * C >= (1ll << 32)) return hipErrorInvalidValue;
  const int G2 = std::min(G, 256), per = (G + G2 - 1) / G2;
  const int groups = (G + per - 1) / per;
  bn_fold_tiles<<<dim3((C + 63) / 64, groups), 256, 0, st>>>(pre, G, C, ws, per);
  bn_bwd_finalize<<<(C + 15) / 16, BN_FIN_T, 0, st>>>(ws, groups, P, C, Cr, gamma, mean, invstd, dgamma, dbeta, a, k1,
                                                      k2, bn_fold_lanes());
  if (dx || dres)
    apply_launch<true>(x, g, a, k1, k2, dx, P, C, nullptr, 0, ym, dres, const_cast<uint8_t*>(mk), st);
  return hipGetLastError();
}

extern "C" hipError_t tp_bn_bwd_train3(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                                       const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a,
                                       float* k1, float* k2, double* ws, const float* ym, float* dres,
                                       const uint8_t* mk, hipStream_t st) {
  return tp_bn_bwd_train4(g, x, dx, P, C, C, gamma, mean, invstd, dgamma, dbeta, a, k1, k2, ws, ym, dres, mk, st);
}

extern "C" hipError_t tp_bn_bwd_train2(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                                       const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a,
                                       float* k1, float* k2, double* ws, const float* ym, float* dres,
                                       hipStream_t st) {
  return tp_bn_bwd_train3(g, x, dx, P, C, gamma, mean, invstd, dgamma, dbeta, a, k1, k2, ws, ym, dres, nullptr, st);
}

extern "C" hipError_t tp_bn_bwd_train(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                                      const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a,
                                      float* k1, float* k2, double* ws, hipStream_t st) {
  return tp_bn_bwd_train2(g, x, dx, P, C, gamma, mean, invstd, dgamma, dbeta, a, k1, k2, ws, nullptr, nullptr, st);
}
