// Winograd F(2x2, 3x3) weight gradient of a stride-1, pad-1 3x3 convolution (the training half of
// config #5): 16 multiplies per (2x2 output tile, in, out channel) instead of 36.
//
// The forward computes Y = A^T [(G w G^T) .* (B^T d B)] A per output tile (d = its 4x4 input
// patch), so by the chain rule
//   dU[xi][co][ci] = sum over tiles of  dM[xi][tile][co] * V[xi][tile][ci],
//   dM = A dY A^T (4x4 from the tile's 2x2 output gradient),  V = B^T d B,
//   dW[co][ci] = G^T dU G (3x3).
// Three steps: (1) transform kernels write V and dM to HBM in transform-point-major layout
// (16, T, C) — plain pixel-major GEMM operands; (2) the 16 GEMMs run as ONE batched launch of the
// pixel-split wgrad MFMA kernel (conv_wgrad.hip, 1x1 "direct" mode, deterministic split combine);
// (3) the output transform writes dW straight into the parameter layout (real channels only).
// Pays off where the GEMM dominates the extra transform traffic (C >= 128); the training conv's
// tuner times it against the direct wgrad per shape.
#include "tp_common.h"

namespace tp {

// V = B^T d B, B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]; one thread per (tile, 4 channels)
__global__ __launch_bounds__(256) void wgrad_x_transform(const float* __restrict__ x, float* __restrict__ v, int B,
                                                         int H, int W, int C, long long T, FastDiv fd_timg,
                                                         FastDiv fd_w2) {
  const int C4 = C / 4, W2 = W / 2, T_img = (H / 2) * W2;
  const long long total = T * C4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const int t = (int)(i / C4);
    const int b = fd_timg.div(t), r = t - b * T_img;
    const int th = fd_w2.div(r), tw = r - th * W2;
    float4 d[16];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ih = 2 * th - 1 + rr, iw = 2 * tw - 1 + q;
        d[rr * 4 + q] = (ih >= 0 && ih < H && iw >= 0 && iw < W)
                            ? *reinterpret_cast<const float4*>(x + (((long long)b * H + ih) * W + iw) * C + c4 * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    float4 tt[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tt[0 * 4 + j] = d[0 * 4 + j] - d[2 * 4 + j];
      tt[1 * 4 + j] = d[1 * 4 + j] + d[2 * 4 + j];
      tt[2 * 4 + j] = d[2 * 4 + j] - d[1 * 4 + j];
      tt[3 * 4 + j] = d[1 * 4 + j] - d[3 * 4 + j];
    }
    const long long stride = T * C;
    float* o = v + (long long)t * C + c4 * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      *reinterpret_cast<float4*>(o + (k * 4 + 0) * stride) = tt[k * 4 + 0] - tt[k * 4 + 2];
      *reinterpret_cast<float4*>(o + (k * 4 + 1) * stride) = tt[k * 4 + 1] + tt[k * 4 + 2];
      *reinterpret_cast<float4*>(o + (k * 4 + 2) * stride) = tt[k * 4 + 2] - tt[k * 4 + 1];
      *reinterpret_cast<float4*>(o + (k * 4 + 3) * stride) = tt[k * 4 + 1] - tt[k * 4 + 3];
    }
  }
}

// dM = A dY A^T, A = [[1,0],[1,1],[1,-1],[0,-1]]; one thread per (tile, 4 output channels)
__global__ __launch_bounds__(256) void wgrad_g_transform(const float* __restrict__ g, float* __restrict__ m, int B,
                                                         int H, int W, int K, long long T, FastDiv fd_timg,
                                                         FastDiv fd_w2) {
  const int K4 = K / 4, W2 = W / 2, T_img = (H / 2) * W2;
  const long long total = T * K4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int k4 = (int)(i % K4);
    const int t = (int)(i / K4);
    const int b = fd_timg.div(t), r = t - b * T_img;
    const int th = fd_w2.div(r), tw = r - th * W2;
    const float* src = g + (((long long)b * H + 2 * th) * W + 2 * tw) * K + k4 * 4;
    const float4 y00 = *reinterpret_cast<const float4*>(src);
    const float4 y01 = *reinterpret_cast<const float4*>(src + K);
    const float4 y10 = *reinterpret_cast<const float4*>(src + (long long)W * K);
    const float4 y11 = *reinterpret_cast<const float4*>(src + (long long)W * K + K);
    // rows: t[i][b] = sum_a A[i][a] dY[a][b]
    const float4 t0[2] = {y00, y01};
    const float4 t1[2] = {y00 + y10, y01 + y11};
    const float4 t2[2] = {y00 - y10, y01 - y11};
    const float4 t3[2] = {-y10, -y11};
    const float4* tr[4] = {t0, t1, t2, t3};
    const long long stride = T * K;
    float* o = m + (long long)t * K + k4 * 4;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const float4 a = tr[ii][0], c = tr[ii][1];
      *reinterpret_cast<float4*>(o + (ii * 4 + 0) * stride) = a;
      *reinterpret_cast<float4*>(o + (ii * 4 + 1) * stride) = a + c;
      *reinterpret_cast<float4*>(o + (ii * 4 + 2) * stride) = a - c;
      *reinterpret_cast<float4*>(o + (ii * 4 + 3) * stride) = -c;
    }
  }
}

// dW[co][ci][a][b] = sum_ij G[i][a] dU[i][j][co][ci] G[j][b] into the parameter layout
// (fin_co x fin_ci real channels, element strides fs). dU: [16][Cout][Kpad] (Kpad >= Cin).
__global__ __launch_bounds__(256) void wgrad_out_transform(const float* __restrict__ du, float* __restrict__ fin,
                                                           int Cout, int Kpad, int fin_co, int fin_ci, long long fs0,
                                                           long long fs1, long long fs2, long long fs3) {
  const float G[4][3] = {{1.f, 0.f, 0.f}, {0.5f, 0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0.f, 0.f, 1.f}};
  const long long total = (long long)fin_co * fin_ci;
  const long long plane = (long long)Cout * Kpad;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % fin_ci), co = (int)(i / fin_ci);
    float u[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) u[xi] = du[xi * plane + (long long)co * Kpad + ci];
    float h[4][3];  // h[i][b] = sum_j u[i][j] G[j][b]
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int bb = 0; bb < 3; ++bb)
        h[ii][bb] = u[ii * 4 + 0] * G[0][bb] + u[ii * 4 + 1] * G[1][bb] + u[ii * 4 + 2] * G[2][bb] +
                    u[ii * 4 + 3] * G[3][bb];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int bb = 0; bb < 3; ++bb)
        fin[co * fs0 + ci * fs1 + a * fs2 + bb * fs3] =
            G[0][a] * h[0][bb] + G[1][a] * h[1][bb] + G[2][a] * h[2][bb] + G[3][a] * h[3][bb];
  }
}

}  // namespace tp

extern "C" hipError_t tp_conv_wgrad3(const float* g, const float* x, float* dw, float* ws, int B, int H, int W,
                                     int Cin, int Cout, int ks, int stride, int pad, int Kpad, int cfg, int splits,
                                     float* fin, int fin_co, int fin_ci, const long long* fs, int batch,
                                     long long g_bstride, long long x_bstride, hipStream_t st);

// Workspace (floats) of tp_wino_wgrad: V (16*T*Cin) + dM (16*T*Cout) + dU (16*Cout*Kp) + the
// split slabs of the batched GEMM (splits*16*Cout*Kp); Kp = Cin rounded up to the GEMM's 32-wide
// K granule (pruned widths: the padded columns of dU are zeros nobody reads).
extern "C" long long tp_wino_wgrad_ws_elems(int B, int H, int W, int Cin, int Cout, int splits) {
  const long long T = (long long)B * (H / 2) * (W / 2);
  const long long Kp = (Cin + 31) / 32 * 32;
  return 16 * T * Cin + 16 * T * Cout + 16ll * Cout * Kp * (1 + (splits > 1 ? splits : 0));
}

// g (B, H, W, Cout), x (B, H, W, Cin) NHWC; H, W even; Cin % 4 == 0 (any pruned width carried at
// a multiple of 4), Cout % 4 == 0. Writes the (fin_co, fin_ci, 3, 3) parameter-layout gradient with
// element strides fs.
extern "C" hipError_t tp_wino_wgrad(const float* g, const float* x, float* ws, int B, int H, int W, int Cin, int Cout,
                                    int cfg, int splits, float* fin, int fin_co, int fin_ci, const long long* fs,
                                    hipStream_t st) {
  using namespace tp;
  if ((H & 1) || (W & 1) || Cin % 4 || Cin < 8 || Cout % 4 || !fin || !fs || fin_co > Cout || fin_ci > Cin ||
      splits < 1)
    return hipErrorInvalidValue;
  const int Kp = (Cin + 31) / 32 * 32;
  const long long T = (long long)B * (H / 2) * (W / 2);
  if (T <= 0) return hipErrorInvalidValue;
  if (T * Cin * 4 >= (1ll << 31) || T * Cout * 4 >= (1ll << 31) || T >= (1ll << 31)) return hipErrorInvalidValue;
  float* v = ws;
  float* m = v + 16 * T * Cin;
  float* du = m + 16 * T * Cout;
  float* slabs = du + 16ll * Cout * Kp;
  const FastDiv fd_timg((unsigned)((H / 2) * (W / 2))), fd_w2((unsigned)(W / 2));
  unsigned grid = (unsigned)std::min<long long>(ceil_div(T * (Cin / 4), 256), 16384);
  wgrad_x_transform<<<grid, 256, 0, st>>>(x, v, B, H, W, Cin, T, fd_timg, fd_w2);
  grid = (unsigned)std::min<long long>(ceil_div(T * (Cout / 4), 256), 16384);
  wgrad_g_transform<<<grid, 256, 0, st>>>(g, m, B, H, W, Cout, T, fd_timg, fd_w2);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // 16 GEMMs dU[xi] = dM[xi]^T V[xi] over the T tiles: "1x1 conv" weight gradients of (1, T, 1, C)
  e = tp_conv_wgrad3(m, v, du, splits > 1 ? slabs : nullptr, 1, (int)T, 1, Cin, Cout, 1, 1, 0, Kp, cfg, splits,
                     nullptr, 0, 0, nullptr, 16, T * Cout, T * Cin, st);
  if (e != hipSuccess) return e;
  grid = (unsigned)std::min<long long>(ceil_div((long long)fin_co * fin_ci, 256), 16384);
  wgrad_out_transform<<<grid, 256, 0, st>>>(du, fin, Cout, Kp, fin_co, fin_ci, fs[0], fs[1], fs[2], fs[3]);
  return hipGetLastError();
}
