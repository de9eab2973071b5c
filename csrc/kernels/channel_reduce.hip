// Per-(sample, channel) attribution reductions and score accumulators.
//
// The reference computes every score in a module hook with a chain of ATen ops
// followed by `.detach().cpu().numpy()` and `np.concatenate` on every batch
// (apoz.py:31-38, sensitivity.py:27-33, taylor.py:40-48). Here a single pass reads the
// activation and/or gradient once, produces the (B, C) per-sample score slab on device,
// and a second deterministic column pass folds it into fp64 running sums. There is no
// host sync per batch and no float atomics (bit-reproducible results).
#include "tp_common.h"

namespace tp {

enum ReduceMode : int { TAYLOR_ABS = 0, TAYLOR_SIGNED = 1, SENS_ABS = 2, APOZ_POS = 3, SUM_GRAD = 4 };

// spatial chunks of the NHWC reduction (>= ~512 positions each, at most 64)
__host__ __device__ inline int nhwc_chunks(int S) { return S <= 1024 ? 1 : (S / 512 > 64 ? 64 : S / 512); }

template <int MODE>
__device__ __forceinline__ float elem(float a, float g) {
  if constexpr (MODE == TAYLOR_ABS || MODE == TAYLOR_SIGNED) return -(g * a);
  else if constexpr (MODE == SENS_ABS) return fabsf(g);
  else if constexpr (MODE == APOZ_POS) return a > 0.f ? 1.f : 0.f;
  else return g;
}

template <int MODE>
__device__ __forceinline__ float finish(float v) {
  if constexpr (MODE == TAYLOR_ABS) return fabsf(v);
  else return v;
}

// NCHW (rows = B*C, each row S contiguous floats). LPR lanes cooperate on one row.
template <int MODE, int LPR, bool VEC>
__global__ __launch_bounds__(256) void channel_reduce_nchw(const float* __restrict__ act,
                                                           const float* __restrict__ grad,
                                                           float* __restrict__ out, long long rows,
                                                           int S) {
  long long gtid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long row = gtid / LPR;
  int lr = (int)(gtid % LPR);
  float acc = 0.f;
  if (row < rows) {
    if constexpr (VEC) {
      const int S4 = S >> 2;
      const float4* a4 = reinterpret_cast<const float4*>(act ? act + row * S : nullptr);
      const float4* g4 = reinterpret_cast<const float4*>(grad ? grad + row * S : nullptr);
      for (int s = lr; s < S4; s += LPR) {
        float4 av = make_float4(0.f, 0.f, 0.f, 0.f), gv = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (MODE != SENS_ABS && MODE != SUM_GRAD) av = a4[s];
        if constexpr (MODE != APOZ_POS) gv = g4[s];
        acc += elem<MODE>(av.x, gv.x) + elem<MODE>(av.y, gv.y) + elem<MODE>(av.z, gv.z) +
               elem<MODE>(av.w, gv.w);
      }
    } else {
      const float* a = act ? act + row * S : nullptr;
      const float* g = grad ? grad + row * S : nullptr;
      for (int s = lr; s < S; s += LPR) {
        float av = 0.f, gv = 0.f;
        if constexpr (MODE != SENS_ABS && MODE != SUM_GRAD) av = a[s];
        if constexpr (MODE != APOZ_POS) gv = g[s];
        acc += elem<MODE>(av, gv);
      }
    }
  }
  if constexpr (LPR > 1) acc = group_sum<LPR>(acc);
  if (row < rows && lr == 0) out[row] = finish<MODE>(acc);
}

// NHWC / channels_last (b, s, c): a block owns (b, 64-channel tile, spatial chunk); 4 waves
// split the chunk. With several chunks (large feature maps: 112x112 = 12,544 positions) each
// block writes a partial to ``ws`` [b][chunk][c] and nhwc_finish sums the chunks in order.
template <int MODE>
__global__ __launch_bounds__(256) void channel_reduce_nhwc(const float* __restrict__ act,
                                                           const float* __restrict__ grad,
                                                           float* __restrict__ out, float* __restrict__ ws,
                                                           int C, int S, int chunk) {
  __shared__ float part[4][64];
  const int b = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sg = threadIdx.x >> 6;
  const int s0 = blockIdx.z * chunk, s1 = min(S, s0 + chunk);
  float acc = 0.f;
  if (c < C) {
    const long long base = (long long)b * S * C + c;
    for (int s = s0 + sg; s < s1; s += 4) {
      float av = 0.f, gv = 0.f;
      if constexpr (MODE != SENS_ABS && MODE != SUM_GRAD) av = act[base + (long long)s * C];
      if constexpr (MODE != APOZ_POS) gv = grad[base + (long long)s * C];
      acc += elem<MODE>(av, gv);
    }
  }
  part[sg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (sg == 0 && c < C) {
    float v = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    if (gridDim.z == 1) out[(long long)b * C + c] = finish<MODE>(v);
    else ws[((long long)b * gridDim.z + blockIdx.z) * C + c] = v;
  }
}

// Vectorised NHWC reduction (C % 32 == 0, 16-B aligned operands): a lane owns one 4-channel
// quad and walks positions with a stride of R = 256 / QB rows, 4 positions in flight
// (float4 loads of both operands, independent accumulators summed in a fixed order); the R row
// groups are reduced through LDS in row order. The spatial map is split into enough chunks that
// the launch has >= 2048 blocks (partials summed in chunk order by nhwc_finish): bandwidth-bound
// ResNet Taylor / Sensitivity scoring ran at ~2.3 TB/s with scalar loads and 256 blocks.
__host__ __device__ inline int nhwc_v4_qb(int C) {
  const int Q = C / 4;
  return Q >= 64 ? 64 : (Q & -Q);
}
__host__ __device__ inline int nhwc_v4_chunks(int B, int C, int S) {
  const int Q = C / 4, qb = nhwc_v4_qb(C);
  const long long blocks = (long long)B * ((Q + qb - 1) / qb);
  int k = 1;
  while (blocks * k < 2048 && S / (2 * k) >= 16 && k < 64) k *= 2;
  return k;
}

template <int MODE>
__global__ __launch_bounds__(256) void channel_reduce_nhwc_v4(const float4* __restrict__ act,
                                                              const float4* __restrict__ grad,
                                                              float* __restrict__ out, float* __restrict__ ws,
                                                              int Q, int S, int chunk, int QB) {
  __shared__ float4 part[256];
  const int b = blockIdx.y;
  const int ql = threadIdx.x % QB, r = threadIdx.x / QB, R = 256 / QB;
  const int q = blockIdx.x * QB + ql;
  const int s0 = blockIdx.z * chunk, s1 = min(S, s0 + chunk);
  constexpr bool NA = MODE == SENS_ABS || MODE == SUM_GRAD, NG = MODE == APOZ_POS;
  auto term = [](const float4& a, const float4& g) {
    return make_float4(elem<MODE>(a.x, g.x), elem<MODE>(a.y, g.y), elem<MODE>(a.z, g.z), elem<MODE>(a.w, g.w));
  };
  float4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < Q) {
    const long long base = (long long)b * S * Q + q;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = s0 + r;
    for (; s + 3 * R < s1; s += 4 * R) {
      float4 av[4], gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = NA ? z : act[base + (long long)(s + u * R) * Q];
        gv[u] = NG ? z : grad[base + (long long)(s + u * R) * Q];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 t = term(av[u], gv[u]);
        acc[u].x += t.x; acc[u].y += t.y; acc[u].z += t.z; acc[u].w += t.w;
      }
    }
    for (; s < s1; s += R) {  // at most 3 tail positions
      const float4 t = term(NA ? z : act[base + (long long)s * Q], NG ? z : grad[base + (long long)s * Q]);
      acc[0].x += t.x; acc[0].y += t.y; acc[0].z += t.z; acc[0].w += t.w;
    }
  }
  float4 v;
  v.x = (acc[0].x + acc[1].x) + (acc[2].x + acc[3].x);
  v.y = (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y);
  v.z = (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z);
  v.w = (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w);
  part[threadIdx.x] = v;
  __syncthreads();
  if (r == 0 && q < Q) {
    for (int k = 1; k < R; ++k) {
      const float4 p = part[k * QB + ql];
      v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
    }
    const long long C = 4ll * Q;
    if (gridDim.z == 1) {
      float* o = out + (long long)b * C + 4 * q;
      o[0] = finish<MODE>(v.x); o[1] = finish<MODE>(v.y); o[2] = finish<MODE>(v.z); o[3] = finish<MODE>(v.w);
    } else {
      *reinterpret_cast<float4*>(ws + ((long long)b * gridDim.z + blockIdx.z) * C + 4 * q) = v;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void nhwc_finish(const float* __restrict__ ws, float* __restrict__ out, int B,
                                                   int C, int chunks) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)B * C) return;
  const long long b = t / C, c = t % C;
  float v = 0.f;
  for (int k = 0; k < chunks; ++k) v += ws[(b * chunks + k) * C + c];
  out[t] = finish<MODE>(v);
}

template <int MODE>
static hipError_t launch_reduce(const float* act, const float* grad, float* out, float* ws, int B, int C, int S,
                                int channels_last, hipStream_t st) {
  const bool al = ((((uintptr_t)act) | ((uintptr_t)grad)) % 16) == 0;
  if (channels_last && C % 32 == 0 && al) {
    const int chunks = ws ? nhwc_v4_chunks(B, C, S) : 1;
    const int chunk = (S + chunks - 1) / chunks;
    const int Q = C / 4, qb = nhwc_v4_qb(C);
    dim3 grid(ceil_div(Q, qb), B, chunks);
    channel_reduce_nhwc_v4<MODE><<<grid, 256, 0, st>>>(reinterpret_cast<const float4*>(act),
                                                       reinterpret_cast<const float4*>(grad), out, ws, Q, S, chunk, qb);
    if (chunks > 1) nhwc_finish<MODE><<<ceil_div((long long)B * C, 256), 256, 0, st>>>(ws, out, B, C, chunks);
    return hipGetLastError();
  }
  if (channels_last) {
    const int chunks = ws ? nhwc_chunks(S) : 1;
    const int chunk = (S + chunks - 1) / chunks;
    dim3 grid(ceil_div(C, 64), B, chunks);
    channel_reduce_nhwc<MODE><<<grid, 256, 0, st>>>(act, grad, out, ws, C, S, chunk);
    if (chunks > 1) nhwc_finish<MODE><<<ceil_div((long long)B * C, 256), 256, 0, st>>>(ws, out, B, C, chunks);
    return hipGetLastError();
  }
  long long rows = (long long)B * C;
  const bool vec = (S % 4 == 0) && ((((uintptr_t)act) | ((uintptr_t)grad)) % 16 == 0);
  const int Se = vec ? S / 4 : S;
  int lpr = Se >= 64 ? 64 : (Se >= 16 ? 16 : (Se >= 4 ? 4 : 1));
  long long threads = rows * lpr;
  unsigned grid = ceil_div(threads, 256);
#define TP_L(L)                                                                           \
  if (lpr == L) {                                                                         \
    if (vec) channel_reduce_nchw<MODE, L, true><<<grid, 256, 0, st>>>(act, grad, out, rows, S); \
    else channel_reduce_nchw<MODE, L, false><<<grid, 256, 0, st>>>(act, grad, out, rows, S);   \
  }
  TP_L(64) TP_L(16) TP_L(4) TP_L(1)
#undef TP_L
  return hipGetLastError();
}

// acc_sum[c] += sum_b v[b, c] (and acc_sq[c] += v^2) in fp64, fixed summation order.
__global__ __launch_bounds__(256) void column_accumulate(const float* __restrict__ v,
                                                         double* __restrict__ acc_sum,
                                                         double* __restrict__ acc_sq, int B, int C) {
  __shared__ double ps[4][64];
  __shared__ double pq[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int b = rg; b < B; b += 4) {
      double x = (double)v[(long long)b * C + c];
      s += x;
      q += x * x;
    }
  }
  ps[rg][threadIdx.x & 63] = s;
  pq[rg][threadIdx.x & 63] = q;
  __syncthreads();
  if (rg == 0 && c < C) {
    acc_sum[c] += ps[0][threadIdx.x] + ps[1][threadIdx.x] + ps[2][threadIdx.x] + ps[3][threadIdx.x];
    if (acc_sq)
      acc_sq[c] += pq[0][threadIdx.x] + pq[1][threadIdx.x] + pq[2][threadIdx.x] + pq[3][threadIdx.x];
  }
}

// Multi-layer score fold used by the fused engine after each backward: for every layer l,
// v = |T_l[b,c]| (or signed); acc_l[c] += sum_b v; then T_l[b,c] <- v (keep per-sample slab)
// or 0 (persistent arena ready for the next batch). One launch for all layers.
struct ScoreDesc {
  float* T;     // (R, B, C): R partial slots per score (summed in slot order: deterministic)
  double* acc;
  int B;
  int C;
  int R;
};
struct ScoreBatch {
  ScoreDesc d[16];
};

// Pass 1: one block per (score tensor, 256-column chunk, chunk of FOLD_ROWS rows); threads =
// (row group, column unit: a float4 quad when C % 4 == 0, else a scalar). Each block writes its
// fp64 column partials to ws[tensor][row chunk][C]. Pass 2 adds the row-chunk partials in
// order into acc. Both passes use fixed summation orders: deterministic.
constexpr int FOLD_ROWS = 32;

__global__ __launch_bounds__(1024) void score_fold_rows(ScoreBatch batch, int take_abs, int after, double* ws,
                                                         int ldc, int n_rchunks) {
  __shared__ double ps[4096];
  const ScoreDesc s = batch.d[blockIdx.y];
  const int c_base = blockIdx.x * 256;
  const int r0 = blockIdx.z * FOLD_ROWS;
  if (c_base >= s.C || r0 >= s.B) return;  // uniform per block
  const int r1 = min(s.B, r0 + FOLD_ROWS);
  const bool vec = (s.C & 3) == 0;
  const int cols = min(256, s.C - c_base);
  const int nq = vec ? (cols + 3) / 4 : min(cols, 256);
  const int RG = min(1024 / nq, FOLD_ROWS);
  const int rg = threadIdx.x / nq, cu = threadIdx.x % nq;
  const int w = vec ? 4 : 1;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  const long long slot = (long long)s.B * s.C;
  if (rg < RG) {
    const int c = c_base + cu * w;
    for (int b = r0 + rg; b < r1; b += RG) {
      float* p = s.T + (long long)b * s.C + c;
      if (vec) {
        float4 v = *reinterpret_cast<float4*>(p);
        for (int r = 1; r < s.R; ++r) {
          const float4 u = *reinterpret_cast<const float4*>(p + r * slot);
          v.x += u.x;
          v.y += u.y;
          v.z += u.z;
          v.w += u.w;
        }
        if (take_abs) {
          v.x = fabsf(v.x);
          v.y = fabsf(v.y);
          v.z = fabsf(v.z);
          v.w = fabsf(v.w);
        }
        a[0] += (double)v.x;
        a[1] += (double)v.y;
        a[2] += (double)v.z;
        a[3] += (double)v.w;
        if (after == 1) {  // keep the processed per-sample value (in slot 0)
          *reinterpret_cast<float4*>(p) = v;
          for (int r = 1; r < s.R; ++r) *reinterpret_cast<float4*>(p + r * slot) = make_float4(0.f, 0.f, 0.f, 0.f);
        } else if (after == 2) {  // zero for the next batch
          for (int r = 0; r < s.R; ++r) *reinterpret_cast<float4*>(p + r * slot) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      } else {
        float v = *p;
        for (int r = 1; r < s.R; ++r) v += p[r * slot];
        if (take_abs) v = fabsf(v);
        a[0] += (double)v;
        if (after == 1) {
          *p = v;
          for (int r = 1; r < s.R; ++r) p[r * slot] = 0.f;
        } else if (after == 2) {
          for (int r = 0; r < s.R; ++r) p[r * slot] = 0.f;
        }
      }
    }
    for (int i = 0; i < w; ++i) ps[rg * (nq * w) + cu * w + i] = a[i];
  }
  __syncthreads();
  if (s.acc) {
    for (int col = threadIdx.x; col < cols; col += blockDim.x) {
      double t = 0.0;
      for (int g = 0; g < RG; ++g) t += ps[g * (nq * w) + col];
      ws[((long long)blockIdx.y * n_rchunks + blockIdx.z) * ldc + c_base + col] = t;
    }
  }
}

__global__ __launch_bounds__(256) void score_fold_final(ScoreBatch batch, const double* ws, int ldc, int n_rchunks) {
  const ScoreDesc s = batch.d[blockIdx.y];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (!s.acc || c >= s.C) return;
  const int nr = (s.B + FOLD_ROWS - 1) / FOLD_ROWS;
  double t = 0.0;
  for (int z = 0; z < nr; ++z) t += ws[((long long)blockIdx.y * n_rchunks + z) * ldc + c];
  s.acc[c] += t;
}

}  // namespace tp

extern "C" int tp_score_fold_ws_elems(const int* B, const int* C, int count) {
  int maxc = 0, maxb = 0;
  for (int i = 0; i < count; ++i) {
    maxc = std::max(maxc, C[i]);
    maxb = std::max(maxb, B[i]);
  }
  return count * tp::ceil_div(maxb, tp::FOLD_ROWS) * maxc;
}

// ws: tp_score_fold_ws_elems doubles
extern "C" hipError_t tp_score_fold_multi(float* const* T, double* const* acc, const int* B, const int* C,
                                          const int* R, int count, int take_abs, int after, double* ws,
                                          hipStream_t st) {
  if (count <= 0 || count > 16) return hipErrorInvalidValue;
  tp::ScoreBatch b{};
  int maxc = 0, maxb = 0;
  bool any_acc = false;
  for (int i = 0; i < count; ++i) {
    b.d[i] = tp::ScoreDesc{T[i], acc[i], B[i], C[i], R[i]};
    maxc = std::max(maxc, C[i]);
    maxb = std::max(maxb, B[i]);
    any_acc |= acc[i] != nullptr;
  }
  if (any_acc && !ws) return hipErrorInvalidValue;
  const int nr = tp::ceil_div(maxb, tp::FOLD_ROWS);
  tp::score_fold_rows<<<dim3(tp::ceil_div(maxc, 256), count, nr), 1024, 0, st>>>(b, take_abs, after, ws, maxc, nr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !any_acc) return e;
  tp::score_fold_final<<<dim3(tp::ceil_div(maxc, 256), count), 256, 0, st>>>(b, ws, maxc, nr);
  return hipGetLastError();
}

extern "C" int tp_channel_reduce_ws_elems(int B, int C, int S, int channels_last) {
  int k = channels_last ? tp::nhwc_chunks(S) : 1;
  if (channels_last && C % 32 == 0) k = std::max(k, tp::nhwc_v4_chunks(B, C, S));  // either kernel may run
  return k > 1 ? B * C * k : 0;
}

extern "C" hipError_t tp_channel_reduce(const float* act, const float* grad, float* out, float* ws, int B, int C,
                                        int S, int mode, int channels_last, hipStream_t st) {
  using namespace tp;
  switch (mode) {
    case TAYLOR_ABS: return launch_reduce<TAYLOR_ABS>(act, grad, out, ws, B, C, S, channels_last, st);
    case TAYLOR_SIGNED: return launch_reduce<TAYLOR_SIGNED>(act, grad, out, ws, B, C, S, channels_last, st);
    case SENS_ABS: return launch_reduce<SENS_ABS>(act, grad, out, ws, B, C, S, channels_last, st);
    case APOZ_POS: return launch_reduce<APOZ_POS>(act, grad, out, ws, B, C, S, channels_last, st);
    case SUM_GRAD: return launch_reduce<SUM_GRAD>(act, grad, out, ws, B, C, S, channels_last, st);
  }
  return hipErrorInvalidValue;
}

extern "C" hipError_t tp_column_accumulate(const float* v, double* acc_sum, double* acc_sq, int B, int C,
                                           hipStream_t st) {
  tp::column_accumulate<<<tp::ceil_div(C, 64), 256, 0, st>>>(v, acc_sum, acc_sq, B, C);
  return hipGetLastError();
}
