// Probe: fused Winograd F(4x4, 3x3) forward on fp32 MFMA (v_mfma_f32_16x16x4_f32).
// 36 transform points per 4x4 output tile (2.25 multiplies per output vs 4 for F(2x2,3x3)).
// A wave owns 16 output tiles x 16 output channels x 36 points (144 accumulator registers);
// per 4-channel chunk each lane loads the 6x6 patch of tile (lane&15), channel (lane>>4), forms
// V = B^T d B and feeds the 36 values as MFMA A operands; U = G g G^T images of one (4-channel
// chunk, 16-output-channel block) are DMA'd into LDS (double-buffered) and shared by the 4 waves.
#include <hip/hip_runtime.h>

#include "tp_common.h"

namespace tp {
namespace probe {

__device__ float buf_load_f32(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");

constexpr int TK = 16;              // output channels per block
constexpr int UIMG = 36 * 4 * TK;   // floats of one U image (2304 = 576 16-B slots)

struct Args {
  const float* x;  // NHWC (B,H,W,C)
  const float* u;  // [C/4][K/16][36][4][16]
  int B, H, W, C, K, P;
  long long x_elems;
  const float* scale;
  const float* shift;
  int relu;
  float* out;      // NHWC (B,H,W,K)
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int xcd_remap4(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// 1-D B^T transform of 6 values
__device__ __forceinline__ void bt6(float d0, float d1, float d2, float d3, float d4, float d5, float* r) {
  const float a = fmaf(-4.f, d2, d4), b = fmaf(-4.f, d1, d3);
  const float c = d4 - d2, e = d3 - d1;
  r[0] = fmaf(4.f, d0, fmaf(-5.f, d2, d4));
  r[1] = a + b;
  r[2] = a - b;
  r[3] = fmaf(2.f, e, c);
  r[4] = fmaf(-2.f, e, c);
  r[5] = fmaf(4.f, d1, fmaf(-5.f, d3, d5));
}

// 1-D A^T transform: 6 -> 4
__device__ __forceinline__ void at6(float m0, float m1, float m2, float m3, float m4, float m5, float* y) {
  const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
  y[0] = m0 + s12 + s34;
  y[1] = fmaf(2.f, d34, d12);
  y[2] = fmaf(4.f, s34, s12);
  y[3] = fmaf(8.f, d34, d12) + m5;
}

__global__ __launch_bounds__(256, 2) void wino_f4x3_fwd(Args p) {
  __shared__ __attribute__((aligned(16))) float us0[UIMG];
  __shared__ __attribute__((aligned(16))) float us1[UIMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int n_k = p.K / TK;
  const int tile = xcd_remap4(blockIdx.x, gridDim.x);
  const int kb = tile % n_k, k0 = kb * TK;
  const int blk_p = tile / n_k;
  const int H4 = p.H >> 2, W4 = p.W >> 2, T_img = H4 * W4;
  constexpr unsigned OOB = 0x80000000u;

  const __amdgpu_buffer_rsrc_t urs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.u, (short)0, (int)(36u * p.C * p.K * 4u), 0x00020000);
  // the descriptor starts (W+1)*C floats before x so every tile's patch origin (row and col -1)
  // is a non-negative per-lane voffset; taps outside the image are masked to OOB
  const int xpad = (p.W + 1) * p.C;
  const i32x4 xr = make_rsrc(p.x - xpad, (unsigned)((p.x_elems + xpad) * 4));

  const int pin = blk_p * 64 + wave * 16 + j;
  const bool tok = pin < p.P;
  int b = 0, th = 0, tw = 0;
  if (tok) {
    b = pin / T_img;
    const int r = pin - b * T_img;
    th = r / W4;
    tw = r - th * W4;
  }
  const int ih0 = 4 * th - 1, iw0 = 4 * tw - 1;
  unsigned rmask = 0, cmask = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    rmask |= (tok && ih0 + r >= 0 && ih0 + r < p.H ? 1u : 0u) << r;
    cmask |= (iw0 + r >= 0 && iw0 + r < p.W ? 1u : 0u) << r;
  }
  const int base = ((b * p.H + ih0) * p.W + iw0) * p.C + g + xpad;  // >= 0
  const int WC = p.W * p.C;

  auto stage = [&](int c0, float* ud) {
    const unsigned ubase = (unsigned)(((c0 >> 2) * n_k + kb) * UIMG) * 4u;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(urs, (lds_ptr_t)(ud + (i * 256 + wave * 64) * 4), 16,
                                               (unsigned)(i * 256 + tid) * 16u, ubase, 0, 0);
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(urs, (lds_ptr_t)(ud + 512 * 4), 16, (unsigned)(512 + tid) * 16u,
                                               ubase, 0, 0);
  };

  float xin[36];
  auto issue_x = [&](int c0) {
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const bool ok = (rmask >> r) & (cmask >> q) & 1u;
        // per-lane part in voffset (one VGPR), the wave-uniform tap/channel part in soffset
        xin[r * 6 + q] = buf_load_f32(xr, (int)(ok ? (unsigned)base * 4u : OOB), (r * WC + q * p.C + c0) * 4, 0);
      }
  };

  f32x4 acc[36];
#pragma unroll
  for (int x = 0; x < 36; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = p.C >> 2;
  stage(0, us0);
  issue_x(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const float* ub = (ch & 1) ? us1 : us0;
    float* un = (ch & 1) ? us0 : us1;
    float v[36];
    {
      float t[36];
#pragma unroll
      for (int q = 0; q < 6; ++q) {  // columns: t[:, q] = B^T d[:, q]
        float r6[6];
        bt6(xin[0 * 6 + q], xin[1 * 6 + q], xin[2 * 6 + q], xin[3 * 6 + q], xin[4 * 6 + q], xin[5 * 6 + q], r6);
#pragma unroll
        for (int r = 0; r < 6; ++r) t[r * 6 + q] = r6[r];
      }
#pragma unroll
      for (int r = 0; r < 6; ++r)  // rows: v[r, :] = t[r, :] B
        bt6(t[r * 6 + 0], t[r * 6 + 1], t[r * 6 + 2], t[r * 6 + 3], t[r * 6 + 4], t[r * 6 + 5], v + r * 6);
    }
    const bool more = ch + 1 < nch;
    if (more) {
      stage((ch + 1) * 4, un);
      issue_x((ch + 1) * 4);
    }
    const float* ul = ub + lane;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int x = 0; x < 36; ++x) acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[x], ul[x * 64], acc[x], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();
  }

  // epilogue: lane holds tiles 4g + i (i = 0..3) of the wave, channel k0 + j
  const int k = k0 + j;
  const float sc = p.scale ? p.scale[k] : 1.f, sh = p.shift ? p.shift[k] : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pe = blk_p * 64 + wave * 16 + 4 * g + i;
    if (pe >= p.P) continue;
    const int be = pe / T_img, re = pe - be * T_img;
    const int the = re / W4, twe = re - the * W4;
    float t[24];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      float y4[4];
      at6(acc[0 * 6 + q][i], acc[1 * 6 + q][i], acc[2 * 6 + q][i], acc[3 * 6 + q][i], acc[4 * 6 + q][i],
          acc[5 * 6 + q][i], y4);
#pragma unroll
      for (int a = 0; a < 4; ++a) t[a * 6 + q] = y4[a];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float y4[4];
      at6(t[a * 6 + 0], t[a * 6 + 1], t[a * 6 + 2], t[a * 6 + 3], t[a * 6 + 4], t[a * 6 + 5], y4);
      float* o = p.out + (((long long)be * p.H + 4 * the + a) * p.W + 4 * twe) * p.K + k;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float y = fmaf(y4[c], sc, sh);
        if (p.relu) y = y > 0.f ? y : (y != y ? y : 0.f);
        o[c * p.K] = y;
      }
    }
  }
}

}  // namespace probe
}  // namespace tp

extern "C" int tp_probe_wino4_fwd(const float* x, const float* u, const float* scale, const float* shift,
                                  float* out, int B, int H, int W, int C, int K, int relu, void* stream) {
  if (H % 4 || W % 4 || C % 4 || K % 16) return 1;
  tp::probe::Args a{};
  a.x = x;
  a.u = u;
  a.B = B;
  a.H = H;
  a.W = W;
  a.C = C;
  a.K = K;
  a.P = B * (H / 4) * (W / 4);
  a.x_elems = (long long)B * H * W * C;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.out = out;
  const int grid = (a.P + 63) / 64 * (K / 16);
  tp::probe::wino_f4x3_fwd<<<grid, 256, 0, (hipStream_t)stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
