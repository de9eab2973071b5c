// Weight gradient of a convolution on fp32 MFMA: the finetune half of the
// prune -> finetune loop (BASELINE config #5), so pruned shapes never wait for a JIT'd library
// kernel.
//
//   dW[co][k] = sum_p g[p][co] * x_im2col[p][k],   k = (kh*KS + kw)*Cin + ci,  p = (b, oh, ow)
//
// GEMM with M = Cout, N = K columns and the reduction over all B*Ho*Wo output pixels. Both
// operands are pixel-major in memory (NHWC rows), so slices of 32 pixels are staged into LDS
// exactly as they sit in HBM (float4 copies, no transposes): sA[p][co], sB[p][k]. An MFMA
// 32x32x2 step takes the two pixel rows 2s, 2s+1: lane (li, lh) reads sA[2s+lh][col li] and
// sB[2s+lh][col li] — ds_read_b32 with consecutive lanes on consecutive words, and row pitch
// = 32 (mod 64) words so the two lane halves hit disjoint banks.
//
// The pixel range is split over grid.y (split-K): partial slabs [split][Cout][Kpad] are summed
// in a fixed order by wgrad_combine_par (deterministic, no atomics).
#include "tp_common.h"

namespace tp {

struct WgradArgs {
  const float* g;  // (B, Ho, Wo, Cout) NHWC
  const float* x;  // (B, H, W, Cin) NHWC
  float* out;      // [splits][Cout][Kpad]
  int B, H, W, Cin, Ho, Wo, Cout, ks, stride, pad;
  int Kc;    // ks*ks*Cin valid columns
  int Kpad;  // columns of the output (multiple of 32)
  int P;     // B*Ho*Wo
  int slices_per_split;
  long long g_elems, x_elems;
  FastDiv fd_hwo, fd_wo;  // pixel -> (image, oh, ow) decode without integer divisions
  // optional final layout: the parameter gradient (fin_co, fin_ci, ks, ks) with element strides
  // fs[4], written straight from the GEMM tile (no split) or the split combine
  float* fin;
  int fin_co, fin_ci;
  long long fs[4];
  // batched GEMMs (blockIdx.z): operand z at g + z*g_bstride, x + z*x_bstride, result [z][Cout][Kpad]
  int batch;
  long long g_bstride, x_bstride;
};

// column k = (kh*ks + kw)*Cin + ci of the (Cout, Kpad) GEMM -> offset in the final layout, or -1
__device__ __forceinline__ long long wgrad_fin_off(const WgradArgs& p, int co, int k) {
  if (co >= p.fin_co || k >= p.Kc) return -1;
  const int tap = k / p.Cin, ci = k - tap * p.Cin;
  if (ci >= p.fin_ci) return -1;
  const int kh = tap / p.ks, kw = tap - kh * p.ks;
  return co * p.fs[0] + ci * p.fs[1] + kh * p.fs[2] + kw * p.fs[3];
}

template <int BM, int BN, int WM, int WN>
struct WTile {
  static constexpr int NW = (BM / WM) * (BN / WN);
  static constexpr int NT = 64 * NW;
  static constexpr int LDA = BM + 32, LDB = BN + 32;  // row pitch == 32 (mod 64) words
  static constexpr int STAGE = 32 * (LDA + LDB);
  static constexpr int A_CH = 32 * BM / 4 / NT;
  static constexpr int B_CH = 32 * BN / 4 / NT;
  static constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(A_CH >= 1 && B_CH >= 1 && (NT % (BM / 4)) == 0 && (NT % (BN / 4)) == 0, "tile/thread mapping");
};

// DIRECT: 1x1 / stride 1 / no padding — the im2col operand is x itself (no pixel decode).
template <int BM, int BN, int WM, int WN, bool DIRECT>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void conv_wgrad(WgradArgs p) {
  using T = WTile<BM, BN, WM, WN>;
  __shared__ __attribute__((aligned(16))) float smem[2 * T::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k_tiles = (p.Kpad + BN - 1) / BN;
  const int co0 = (blockIdx.x / k_tiles) * BM, k0 = (blockIdx.x % k_tiles) * BN;
  const int s_begin = blockIdx.y * p.slices_per_split;
  const int s_end = min((p.P + 31) / 32, s_begin + p.slices_per_split);
  constexpr unsigned OOB = 0x80000000u;
  const int z = blockIdx.z;
  const i32x4 gr = make_rsrc(p.g + z * p.g_bstride, (unsigned)(p.g_elems * 4));
  const i32x4 xr = make_rsrc(p.x + z * p.x_bstride, (unsigned)(p.x_elems * 4));

  // per-thread column decode of the im2col operand (fixed for the whole pixel loop)
  const int b_c4 = tid % (BN / 4), b_r0 = tid / (BN / 4);
  const int kcol = k0 + 4 * b_c4;
  const int tap = kcol / p.Cin, ci = kcol - tap * p.Cin;
  const int kh = tap / p.ks, kw = tap - kh * p.ks;
  const bool col_ok = kcol < p.Kc;
  const int a_c4 = tid % (BM / 4), a_r0 = tid / (BM / 4);
  const bool co_ok = co0 + 4 * a_c4 < p.Cout;
  const int HWo = p.Ho * p.Wo;

  float4 ra[T::A_CH], rb[T::B_CH];
  auto load = [&](int sl) {
    const int p0 = sl * 32;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) {
      const int pix = p0 + a_r0 + i * (T::NT / (BM / 4));
      const bool ok = co_ok && pix < p.P;
      const unsigned vo = ok ? (unsigned)(pix * p.Cout + co0 + 4 * a_c4) * 4u : OOB;
      const f32x4 v = buf_load_f32x4(gr, (int)vo, 0, 0);
      ra[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i) {
      const int pix = p0 + b_r0 + i * (T::NT / (BN / 4));
      bool ok = col_ok && pix < p.P;
      int off = pix * p.Cin + ci;
      if (!DIRECT && ok) {
        const int b = p.fd_hwo.div(pix), r = pix - b * HWo;
        const int oh = p.fd_wo.div(r), ow = r - oh * p.Wo;
        const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
        ok = ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        off = ((b * p.H + ih) * p.W + iw) * p.Cin + ci;
      }
      const f32x4 v = buf_load_f32x4(xr, (int)(ok ? (unsigned)off * 4u : OOB), 0, 0);
      rb[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store = [&](int buf) {
    float* sA = smem + buf * T::STAGE;
    float* sB = sA + 32 * T::LDA;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i)
      *reinterpret_cast<float4*>(sA + (a_r0 + i * (T::NT / (BM / 4))) * T::LDA + 4 * a_c4) = ra[i];
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i)
      *reinterpret_cast<float4*>(sB + (b_r0 + i * (T::NT / (BN / 4))) * T::LDB + 4 * b_c4) = rb[i];
  };

  f32x16 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int wm0 = (wave / (BN / WN)) * WM, wn0 = (wave % (BN / WN)) * WN;
  const int li = lane & 31, lh = lane >> 5;

  if (s_begin < s_end) {
    load(s_begin);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int sl = s_begin; sl < s_end; ++sl) {
      const bool more = sl + 1 < s_end;
      if (more) load(sl + 1);
      const float* sA = smem + buf * T::STAGE + lh * T::LDA + wm0 + li;
      const float* sB = smem + buf * T::STAGE + 32 * T::LDA + lh * T::LDB + wn0 + li;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        float af[T::TM], bf[T::TN];
#pragma unroll
        for (int i = 0; i < T::TM; ++i) af[i] = sA[(2 * s) * T::LDA + i * 32];
#pragma unroll
        for (int j = 0; j < T::TN; ++j) bf[j] = sB[(2 * s) * T::LDB + j * 32];
#pragma unroll
        for (int i = 0; i < T::TM; ++i)
#pragma unroll
          for (int j = 0; j < T::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if (more) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  float* out = p.out + ((long long)blockIdx.y * p.batch + z) * p.Cout * p.Kpad;
  const bool fin = p.fin && gridDim.y == 1 && gridDim.z == 1;
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) {
      const int k = k0 + wn0 + j * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (fin) {
          const long long o = wgrad_fin_off(p, co, k);
          if (o >= 0) p.fin[o] = acc[i][j][r];
        } else if (co < p.Cout && k < p.Kpad) {
          out[(long long)co * p.Kpad + k] = acc[i][j][r];
        }
      }
    }
}

// Split combine, deterministic: a block owns 64 consecutive GEMM elements; its SL waves
// (SL = min(8, splits), blockDim = 64 * SL) each sum the splits q = wave, wave + SL, ... in
// increasing order (4 loads in flight), then wave 0 adds the SL lane sums in wave order. The
// old one-thread-per-element walk over the 64-256 split slabs of the big-map wgrads left ~2
// waves per CU with one dependent load at a time (~200 GB/s). FIN: write straight into the
// final weight layout (wgrad_fin_off); otherwise dw[t].
template <bool FIN>
__global__ __launch_bounds__(512) void wgrad_combine_par(const float* __restrict__ slabs, WgradArgs p,
                                                         float* __restrict__ dw, int splits, long long n) {
  __shared__ float red[8][64];
  const int tl = threadIdx.x & 63, sl = threadIdx.x >> 6, SL = blockDim.x >> 6;
  for (long long base = (long long)blockIdx.x * 64; base < n; base += (long long)gridDim.x * 64) {
    const long long t = base + tl;
    float s = 0.f;
    if (t < n) {
      int q = sl;
      for (; q + 3 * SL < splits; q += 4 * SL) {
        const float v0 = slabs[(long long)q * n + t], v1 = slabs[(long long)(q + SL) * n + t];
        const float v2 = slabs[(long long)(q + 2 * SL) * n + t], v3 = slabs[(long long)(q + 3 * SL) * n + t];
        s += v0;
        s += v1;
        s += v2;
        s += v3;
      }
      for (; q < splits; q += SL) s += slabs[(long long)q * n + t];
    }
    red[sl][tl] = s;
    __syncthreads();
    if (sl == 0 && t < n) {
      for (int i = 1; i < SL; ++i) s += red[i][tl];
      if constexpr (FIN) {
        const int co = (int)(t / p.Kpad), k = (int)(t - (long long)co * p.Kpad);
        const long long o = wgrad_fin_off(p, co, k);
        if (o >= 0) p.fin[o] = s;
      } else {
        dw[t] = s;
      }
    }
    __syncthreads();
  }
}

}  // namespace tp

namespace {
template <int BM, int BN, int WM, int WN>
hipError_t launch_wgrad(const tp::WgradArgs& a, int splits, hipStream_t st) {
  const int tiles = ((a.Cout + BM - 1) / BM) * ((a.Kpad + BN - 1) / BN);
  const dim3 grid(tiles, splits, a.batch);
  if (a.ks == 1 && a.stride == 1 && a.pad == 0)
    tp::conv_wgrad<BM, BN, WM, WN, true><<<grid, tp::WTile<BM, BN, WM, WN>::NT, 0, st>>>(a);
  else
    tp::conv_wgrad<BM, BN, WM, WN, false><<<grid, tp::WTile<BM, BN, WM, WN>::NT, 0, st>>>(a);
  return hipGetLastError();
}
}  // namespace

// Tile configs: 0 = 128x128 (4 waves of 64x64), 1 = 64x64 (4 waves of 32x32), 2 = 128x64
// (4 waves of 64x32). ``ws`` holds splits*Cout*Kpad floats (may alias dw when splits == 1).
// x (B, H, W, Cin) NHWC with Cin % 4 == 0; g (B, Ho, Wo, Cout) NHWC with Cout % 4 == 0;
// dw (Cout, Kpad), Kpad % 32 == 0 and >= ks*ks*Cin.
// fin (nullable): also/instead write the parameter-layout gradient (fin_co <= Cout, fin_ci <= Cin,
// ks, ks) with element strides fs[4]; dw is then not written (may be null).
// batch > 1: ``batch`` independent GEMMs (operands g + z*g_bstride, x + z*x_bstride) -> dw
// [batch][Cout][Kpad]; no ``fin`` (the Winograd weight gradient's 16 transform-point GEMMs).
extern "C" hipError_t tp_conv_wgrad3(const float* g, const float* x, float* dw, float* ws, int B, int H, int W,
                                     int Cin, int Cout, int ks, int stride, int pad, int Kpad, int cfg, int splits,
                                     float* fin, int fin_co, int fin_ci, const long long* fs, int batch,
                                     long long g_bstride, long long x_bstride, hipStream_t st) {
  using namespace tp;
  if (Cin % 4 || Cout % 4 || Kpad % 32 || Kpad < ks * ks * Cin || splits < 1) return hipErrorInvalidValue;
  if (batch < 1 || batch > 65535 || (batch > 1 && fin)) return hipErrorInvalidValue;
  if (fin && (fin_co > Cout || fin_ci > Cin || fin_co <= 0 || fin_ci <= 0 || !fs)) return hipErrorInvalidValue;
  if (!fin && !dw) return hipErrorInvalidValue;
  WgradArgs a{};
  a.batch = batch;
  a.g_bstride = g_bstride;
  a.x_bstride = x_bstride;
  a.fin = fin;
  a.fin_co = fin_co;
  a.fin_ci = fin_ci;
  if (fin)
    for (int i = 0; i < 4; ++i) a.fs[i] = fs[i];
  a.g = g;
  a.x = x;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.Cout = Cout;
  a.ks = ks;
  a.stride = stride;
  a.pad = pad;
  a.Ho = (H + 2 * pad - ks) / stride + 1;
  a.Wo = (W + 2 * pad - ks) / stride + 1;
  a.Kc = ks * ks * Cin;
  a.Kpad = Kpad;
  a.P = B * a.Ho * a.Wo;
  a.fd_hwo = FastDiv((unsigned)std::max(1, a.Ho * a.Wo));
  a.fd_wo = FastDiv((unsigned)std::max(1, a.Wo));
  a.g_elems = (long long)a.P * Cout;
  a.x_elems = (long long)B * H * W * Cin;
  if (a.g_elems * 4 >= (1ll << 31) || a.x_elems * 4 >= (1ll << 31)) return hipErrorInvalidValue;
  const int slices = (a.P + 31) / 32;
  splits = std::min(splits, slices);
  a.slices_per_split = (slices + splits - 1) / splits;
  splits = (slices + a.slices_per_split - 1) / a.slices_per_split;
  a.out = splits > 1 ? ws : dw;
  if (splits > 1 && !ws) return hipErrorInvalidValue;
  hipError_t e;
  switch (cfg) {
    case 0: e = launch_wgrad<128, 128, 64, 64>(a, splits, st); break;
    case 1: e = launch_wgrad<64, 64, 32, 32>(a, splits, st); break;
    case 2: e = launch_wgrad<128, 64, 64, 32>(a, splits, st); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess || splits == 1) return e;
  const long long n = fin ? (long long)Cout * Kpad : (long long)batch * Cout * Kpad;
  // lanes per element: only as many as it takes to put ~16 waves on every CU (n * lanes >= 256K
  // threads). Big weights keep one lane per element, i.e. the splits summed strictly in order —
  // the summation order of earlier builds: a training recipe on a knife edge (the bench's seed-0
  // VGG teacher) follows it bit for bit. TP_WGRAD_COMBINE_LANES=1 forces one lane everywhere.
  static const int lanes_max = [] {
    const char* e = getenv("TP_WGRAD_COMBINE_LANES");
    return e && atoi(e) == 1 ? 1 : 8;
  }();
  const int sl = (int)std::max<long long>(1, std::min<long long>({(long long)lanes_max, (long long)splits,
                                                                  ceil_div(262144ll, n)}));
  const unsigned grid = (unsigned)std::min<long long>(ceil_div(n, 64), 16384);
  if (fin)
    wgrad_combine_par<true><<<grid, 64 * sl, 0, st>>>(ws, a, nullptr, splits, n);
  else
    wgrad_combine_par<false><<<grid, 64 * sl, 0, st>>>(ws, a, dw, splits, n);
  return hipGetLastError();
}

extern "C" hipError_t tp_conv_wgrad2(const float* g, const float* x, float* dw, float* ws, int B, int H, int W,
                                     int Cin, int Cout, int ks, int stride, int pad, int Kpad, int cfg, int splits,
                                     float* fin, int fin_co, int fin_ci, const long long* fs, hipStream_t st) {
  return tp_conv_wgrad3(g, x, dw, ws, B, H, W, Cin, Cout, ks, stride, pad, Kpad, cfg, splits, fin, fin_co, fin_ci, fs,
                        1, 0, 0, st);
}

extern "C" hipError_t tp_conv_wgrad(const float* g, const float* x, float* dw, float* ws, int B, int H, int W,
                                    int Cin, int Cout, int ks, int stride, int pad, int Kpad, int cfg, int splits,
                                    hipStream_t st) {
  return tp_conv_wgrad2(g, x, dw, ws, B, H, W, Cin, Cout, ks, stride, pad, Kpad, cfg, splits, nullptr, 0, 0, nullptr,
                        st);
}
