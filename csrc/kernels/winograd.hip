// Fused Winograd F(2x2, 3x3) convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32), the
// 2.25x-fewer-multiplies algorithm MIOpen uses for fp32 3x3 convs, re-designed so that
// NOTHING but the input, the pre-transformed weights and the final output touch memory:
//
//   * a wave owns 16 output tiles (2x2 pixels each) x 32 output channels x all 16 transform
//     points xi; its 16*2 accumulator tiles (16x16, 4 regs) live in registers;
//   * per 8-channel chunk each lane loads the 4x4 input patch of "its" tile (MFMA A-row =
//     lane&15) for 2 channels (A-k = lane>>4), forms V = B^T d B in registers (32 adds per
//     channel) and feeds the 16 V values straight into 16 MFMAs as the A operand;
//   * the transformed weights U = G g G^T ([16][C][K], K interleaved per 32-block) are staged
//     in LDS per block (shared by its 4 waves) and read as the B operand;
//   * the epilogue applies Y = A^T m A in registers. A 2x2 Winograd output tile IS a 2x2
//     max-pool window, so pooling is 3 max ops on values the lane already holds; BN affine,
//     ReLU, Taylor partials and the masked gradient are fused exactly as in conv_mfma.hip.
//   * UNPOOL: the dgrad input is rebuilt on the fly from the pooled gradient + argmax bytes
//     (a 4x4 full-resolution patch spans 3x3 pooled cells).
#include "tp_common.h"

namespace tp {

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ f32x2 buf_load_f32x2(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2f32");
__device__ unsigned short buf_load_u16(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i16");

enum WEpi : int { W_FWD = 0, W_FWD_POOL = 1, W_BWD = 2, W_PARTIAL = 3 };

struct WinoArgs {
  const float* x;           // NHWC (B,H,W,C), or pooled grad (B,H/2,W/2,C) when UNPOOL
  const uint8_t* x_argmax;  // UNPOOL: argmax bytes of the pooled grad
  const float* u;           // [16][C][K] transformed weights, K interleaved per 32-block
  int B, H, W, C, K;
  int P;                    // output tiles = B*(H/2)*(W/2)
  int c_per_split;
  long long x_elems;
  const float* scale;
  const float* shift;
  int relu;
  float* out;
  uint8_t* out_argmax;
  const float* act;
  float* taylor;
  int pooled_m;             // W_PARTIAL: write the slab in pooled M order (b, th, tw, q)
};

__device__ __forceinline__ int xcd_remap_w(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// V = B^T d B for one channel (d row-major 4x4), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
__device__ __forceinline__ void input_transform(const float d[16], float v[16]) {
  float t[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0 * 4 + j] = d[0 * 4 + j] - d[2 * 4 + j];
    t[1 * 4 + j] = d[1 * 4 + j] + d[2 * 4 + j];
    t[2 * 4 + j] = d[2 * 4 + j] - d[1 * 4 + j];
    t[3 * 4 + j] = d[1 * 4 + j] - d[3 * 4 + j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i * 4 + 0] = t[i * 4 + 0] - t[i * 4 + 2];
    v[i * 4 + 1] = t[i * 4 + 1] + t[i * 4 + 2];
    v[i * 4 + 2] = t[i * 4 + 2] - t[i * 4 + 1];
    v[i * 4 + 3] = t[i * 4 + 1] - t[i * 4 + 3];
  }
}

// Y = A^T m A, A^T = [[1,1,1,0],[0,1,-1,-1]]  ->  y[a*2+b]
__device__ __forceinline__ void output_transform(const float m[16], float y[4]) {
  float t[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0 * 4 + j] = m[0 * 4 + j] + m[1 * 4 + j] + m[2 * 4 + j];
    t[1 * 4 + j] = m[1 * 4 + j] - m[2 * 4 + j] - m[3 * 4 + j];
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    y[a * 2 + 0] = t[a * 4 + 0] + t[a * 4 + 1] + t[a * 4 + 2];
    y[a * 2 + 1] = t[a * 4 + 1] - t[a * 4 + 2] - t[a * 4 + 3];
  }
}

template <int EPI, bool UNPOOL>
__global__ __launch_bounds__(256, 2) void wino_f2x3(WinoArgs p) {
  constexpr int TK = 32, CH = 8, LDU = 48;       // LDU: 2*48 = 32 mod 64 -> conflict-free b64 reads
  constexpr int STAGE = 16 * CH * LDU;           // floats per U stage
  __shared__ __attribute__((aligned(16))) float us[2 * STAGE];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int n_k = (p.K + TK - 1) / TK;
  const int tile = xcd_remap_w(blockIdx.x, gridDim.x);
  const int k0 = (tile % n_k) * TK;
  const int pw0 = (tile / n_k) * 64 + wave * 16;  // first tile of this wave
  const int H2 = p.H >> 1, W2 = p.W >> 1, T_img = H2 * W2;
  const int c_begin = blockIdx.y * p.c_per_split;
  const int c_end = min(p.C, c_begin + p.c_per_split);

  const i32x4 xr = make_rsrc(p.x, (unsigned)(p.x_elems * 4));
  const i32x4 ar = make_rsrc(p.x_argmax, UNPOOL ? (unsigned)p.x_elems : 0u);
  const i32x4 ur = make_rsrc(p.u, (unsigned)(16u * p.C * p.K * 4u));
  constexpr unsigned OOB = 0x80000000u;

  // ---- the input tile of this lane (A row j) ------------------------------------------
  const int pin = pw0 + j;
  int b = 0, th = 0, tw = 0;
  const bool tok = pin < p.P;
  if (tok) {
    b = pin / T_img;
    const int r = pin - b * T_img;
    th = r / W2;
    tw = r - th * W2;
  }
  // offsets (elements, channel 0) and validity of the 16 patch pixels (or 9 pooled cells)
  int poff[16];
  unsigned pmask = 0;
  if constexpr (!UNPOOL) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ih = 2 * th - 1 + r, iw = 2 * tw - 1 + q;
        const bool ok = tok && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        poff[r * 4 + q] = ((b * p.H + ih) * p.W + iw) * p.C;
        pmask |= (ok ? 1u : 0u) << (r * 4 + q);
      }
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ph = th - 1 + r, pq = tw - 1 + q;
        const bool ok = tok && ph >= 0 && ph < H2 && pq >= 0 && pq < W2;
        poff[r * 3 + q] = ((b * H2 + ph) * W2 + pq) * p.C;
        pmask |= (ok ? 1u : 0u) << (r * 3 + q);
      }
  }

  // ---- U staging: thread -> (row = xi*CH + c, half of the 32 k's) ---------------------
  const int srow = threadIdx.x >> 1, shalf = threadIdx.x & 1;
  const int s_xi = srow / CH, s_c = srow % CH;
  float4 ru[4];
  auto load_u = [&](int c0) {
    const unsigned base = (unsigned)((s_xi * p.C + c0 + s_c) * p.K + k0 + shalf * 16) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 v = buf_load_f32x4(ur, (int)(base + 16u * i), 0, 0);
      ru[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_u = [&](int buf) {
    float* dst = us + buf * STAGE + srow * LDU + shalf * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(dst + 4 * i) = ru[i];
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[x][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (c_begin < c_end) {
    load_u(c_begin);
    store_u(0);
    __syncthreads();
    int buf = 0;
    for (int c0 = c_begin; c0 < c_end; c0 += CH) {
      const bool more = c0 + CH < c_end;
      if (more) load_u(c0 + CH);
      // patch values for channels c0+2g, c0+2g+1
      float d0[16], d1[16];
      const int cc = c0 + 2 * g;
      if constexpr (!UNPOOL) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const unsigned vo = ((pmask >> t) & 1u) ? (unsigned)(poff[t] + cc) * 4u : OOB;
          const f32x2 v = buf_load_f32x2(xr, (int)vo, 0, 0);
          d0[t] = v[0];
          d1[t] = v[1];
        }
      } else {
        float g0[9], g1[9];
        unsigned am[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const bool ok = (pmask >> t) & 1u;
          const f32x2 v = buf_load_f32x2(xr, (int)(ok ? (unsigned)(poff[t] + cc) * 4u : OOB), 0, 0);
          g0[t] = v[0];
          g1[t] = v[1];
          am[t] = buf_load_u16(ar, (int)(ok ? (unsigned)(poff[t] + cc) : OOB), 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cell = ((r + 1) >> 1) * 3 + ((q + 1) >> 1);
            const unsigned want = (unsigned)((((r + 1) & 1) << 1) | ((q + 1) & 1));
            d0[r * 4 + q] = (am[cell] & 0xffu) == want ? g0[cell] : 0.f;
            d1[r * 4 + q] = ((am[cell] >> 8) & 0xffu) == want ? g1[cell] : 0.f;
          }
      }
      const float* ub = us + buf * STAGE;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v[16];
        input_transform(e == 0 ? d0 : d1, v);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int x = 0; x < 16; ++x) {
          const float2 w2 = *reinterpret_cast<const float2*>(ub + (x * CH + 2 * g + e) * LDU + 2 * j);
          acc[x][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[x], w2.x, acc[x][0], 0, 0, 0);
          acc[x][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[x], w2.y, acc[x][1], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
      if (more) store_u(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- epilogue: output tiles pw0 + 4g + r, channels k0 + j + 16n ----------------------
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int k = k0 + j + 16 * n;
    const bool kok = k < p.K;
    float sc = 1.f, sh = 0.f;
    if (kok && EPI != W_PARTIAL) {
      sc = p.scale ? p.scale[k] : 1.f;
      if (EPI != W_BWD) sh = p.shift ? p.shift[k] : 0.f;
    }
    int cur_b = -1;
    float tsum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pt = pw0 + 4 * g + r;
      if (!kok || pt >= p.P) continue;
      float m[16], y[4];
#pragma unroll
      for (int x = 0; x < 16; ++x) m[x] = acc[x][n][r];
      output_transform(m, y);
      const int bb = pt / T_img;
      const int rr = pt - bb * T_img;
      const int oh2 = rr / W2, ow2 = rr - oh2 * W2;
      if constexpr (EPI == W_FWD_POOL) {
        float best = 0.f;
        int arg = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = y[q] * sc + sh;
          if (p.relu) v = nan_relu(v);
          if (q == 0 || v > best || (v != v && best == best)) {
            best = v;
            arg = q;
          }
        }
        const long long o = (long long)pt * p.K + k;
        p.out[o] = best;
        p.out_argmax[o] = (uint8_t)arg;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int oh = 2 * oh2 + (q >> 1), ow = 2 * ow2 + (q & 1);
          const long long pix = ((long long)bb * p.H + oh) * p.W + ow;
          if constexpr (EPI == W_FWD) {
            float v = y[q] * sc + sh;
            if (p.relu) v = nan_relu(v);
            p.out[pix * p.K + k] = v;
          } else if constexpr (EPI == W_PARTIAL) {
            const long long mrow = p.pooled_m ? (long long)pt * 4 + q : pix;
            p.out[((long long)blockIdx.y * p.B * p.H * p.W + mrow) * p.K + k] = y[q];
          } else {  // W_BWD
            const float a = p.act[pix * p.K + k];
            if (p.taylor) {
              if (bb != cur_b) {
                if (cur_b >= 0) atomicAdd(p.taylor + (long long)cur_b * p.K + k, tsum);
                cur_b = bb;
                tsum = 0.f;
              }
              tsum += -(y[q] * a);
            }
            if (p.out) p.out[pix * p.K + k] = a > 0.f ? y[q] * sc : 0.f;
          }
        }
      }
    }
    if constexpr (EPI == W_BWD) {
      if (p.taylor && cur_b >= 0) atomicAdd(p.taylor + (long long)cur_b * p.K + k, tsum);
    }
  }
}

}  // namespace tp

// Winograd conv: same operand/epilogue contract as tp_conv_igemm (3x3, stride 1, pad 1),
// ``u`` = transformed weights. epi: 0 fwd, 1 fwd+pool, 2 bwd (dgrad epilogue). H, W even,
// C % 8 == 0, K % 32 == 0. splits > 1 -> partial slabs in ``ws`` + conv_epilogue combine.
extern "C" hipError_t tp_conv_epilogue_slabs(const float* ws, int splits, int B, int H, int W, int K, int epi,
                                              const float* scale, const float* shift, int relu, float* out,
                                              uint8_t* out_argmax, const float* act, float* taylor,
                                              hipStream_t st);

extern "C" hipError_t tp_conv_wino(const float* x, const uint8_t* x_argmax, const float* u, int B, int H, int W,
                                   int C, int K, int unpool, int epi, int splits, const float* scale,
                                   const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act,
                                   float* taylor, float* ws, hipStream_t st) {
  using namespace tp;
  if ((H & 1) || (W & 1) || C % 8 != 0 || K % 32 != 0) return hipErrorInvalidValue;
  WinoArgs a{};
  a.x = x;
  a.x_argmax = x_argmax;
  a.u = u;
  a.B = B;
  a.H = H;
  a.W = W;
  a.C = C;
  a.K = K;
  a.P = B * (H / 2) * (W / 2);
  a.x_elems = unpool ? (long long)B * (H / 2) * (W / 2) * C : (long long)B * H * W * C;
  if (a.x_elems * 4 >= (1ll << 31) || 16ll * C * K * 4 >= (1ll << 31)) return hipErrorInvalidValue;
  const int chunks = C / 8;
  splits = std::max(1, std::min(splits, chunks));
  a.c_per_split = ((chunks + splits - 1) / splits) * 8;
  splits = (C + a.c_per_split - 1) / a.c_per_split;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.out = out;
  a.out_argmax = out_argmax;
  a.act = act;
  a.taylor = taylor;
  const int n_p = (a.P + 63) / 64, n_k = K / 32;
  dim3 grid(n_p * n_k, splits);
  if (splits > 1) {
    if (!ws) return hipErrorInvalidValue;
    WinoArgs pa = a;
    pa.out = ws;
    pa.pooled_m = epi == W_FWD_POOL ? 1 : 0;
    if (unpool) wino_f2x3<W_PARTIAL, true><<<grid, 256, 0, st>>>(pa);
    else wino_f2x3<W_PARTIAL, false><<<grid, 256, 0, st>>>(pa);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return tp_conv_epilogue_slabs(ws, splits, B, H, W, K, epi, scale, shift, relu, out, out_argmax, act, taylor, st);
  }
#define TP_W(E, U) wino_f2x3<E, U><<<grid, 256, 0, st>>>(a)
  if (epi == W_FWD) { if (unpool) TP_W(W_FWD, true); else TP_W(W_FWD, false); }
  else if (epi == W_FWD_POOL) { if (unpool) return hipErrorInvalidValue; TP_W(W_FWD_POOL, false); }
  else if (epi == W_BWD) { if (unpool) TP_W(W_BWD, true); else TP_W(W_BWD, false); }
  else return hipErrorInvalidValue;
#undef TP_W
  return hipGetLastError();
}
