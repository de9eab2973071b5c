// Persistent, warp-specialised fp32 MFMA GEMM for 1x1 convolutions (ResNet bottleneck / downsample
// convs and their data gradients) with the engine's fused epilogues: BN affine, residual add,
// ReLU-backward mask, NaN-propagating (Leaky)ReLU, APoZ counts.
//
// Why a second 1x1 kernel (conv_mfma.hip's conv_igemm GEN 1 serves every shape): ResNet-50's 1x1
// convs have short K (64-512 channels) and wide outputs, so a tile's epilogue (store the 128x128
// output, read the 128x128 residual / mask: 128 KB of HBM traffic) takes as long as its MFMA
// loop (K = 128: 4 slices). conv_igemm runs the two phases back to back in every block, and its
// blocks start in lockstep, so the CU alternates between MFMA-bound and HBM-bound phases
// (profiles/resnet/resnet50_fwd_conv_roofline_b256.txt: 53-76% of the per-shape roofline).
//
// Here one workgroup per CU loops over output tiles (persistent; grid = CUs, XCD-contiguous tile
// order) with two wave roles that run concurrently:
//   * 8 MFMA waves: the double-buffered LDS K loop of conv_igemm (v_mfma_f32_32x32x2f32, BK = 32,
//     36-float padded rows, ds_read_b128 fragments), then the accumulators go to an LDS output
//     tile and the next tile starts at once (its first global loads are issued before that);
//   * MEMW memory waves: the epilogue of the PREVIOUS tile out of the LDS output tile, spread
//     over the S barrier intervals of the current tile's K loop (S = K / 32), so its HBM
//     traffic runs under the MFMAs.
// The MFMA waves run one flat stream of K slices over their tiles with the global loads two
// slices ahead (one workgroup per CU: two MFMA waves per SIMD have to hide the load latency).
// Every wave executes the same barrier sequence (S + 1 per tile, one drain tile, one final), the
// barriers are raw s_barrier after an LDS-only wait: the memory waves' global stores stay in
// flight across them (a __syncthreads() would drain vmcnt at every interval).
// APoZ counts: per-thread runs -> LDS counters per (image, column) of the tile (double-buffered
// by tile parity) -> one global atomic per (image, column) per tile, flushed one tile later
// (exact integer counts: order-free).
#include "tp_common.h"

namespace tp {
namespace ws {

constexpr int BM = 128, BK = 32, LDK = BK + 4;
constexpr int MFMA_WAVES = 8;
constexpr int CB_IMG = 8;  // images per tile whose APoZ counts are reduced in LDS

struct Args {
  const float* x;  // A: NHWC (B, H, W, Cin)
  const float* w;  // B: (N, Cin)
  int B, H, W, Cin, N, Ho, Wo, stride, M, HWo;
  const float* scale;  // (N) or null
  const float* shift;  // (N) or null
  int relu;
  float slope;
  const float* res;   // (M, N) or null
  const float* mask;  // (M, N) or null: out = mask > 0 ? v : 0
  float* apoz;        // (B, N) or null
  float* out;         // (M, N)
  int m_tiles, n_tiles, tiles;
};

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ int xcd_tile(int t, int tiles) {  // XCD-contiguous ranges (bijective)
  const int q = tiles / 8, r = tiles % 8;
  const int xcd = t % 8, idx = t / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <int BN, int MEMW>
__global__ __launch_bounds__(64 * (MFMA_WAVES + MEMW), 1) void gemm1x1_ws(Args p) {
  constexpr int WN = 32, WM = BN == 128 ? 64 : 32;
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * WAVES_N == MFMA_WAVES, "8 MFMA waves");
  constexpr int TM = WM / 32, TN = 1;
  constexpr int MT_THREADS = 64 * MFMA_WAVES;
  constexpr int A_CH = BM * BK / 4 / MT_THREADS, B_CH = BN * BK / 4 / MT_THREADS;
  static_assert(A_CH >= 1 && B_CH >= 1, "load mapping");
  constexpr int LDT = BN + 4;
  constexpr int STAGE = (BM + BN) * LDK;
  // epilogue mapping: memory thread -> (row lane, column quad)
  constexpr int MEM_THREADS = 64 * MEMW, C4 = BN / 4, RSTEP = MEM_THREADS / C4, NP = BM / RSTEP;
  static_assert(MEM_THREADS % C4 == 0 && BM % RSTEP == 0, "epilogue mapping");

  __shared__ __attribute__((aligned(16))) float stage[2 * STAGE];
  __shared__ __attribute__((aligned(16))) float outb[BM * LDT];
  __shared__ float cb[2][CB_IMG * BN];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const bool is_mfma = wave < MFMA_WAVES;  // wave-uniform role
  const int G = gridDim.x;
  const int my_tiles = p.tiles > (int)blockIdx.x ? (p.tiles - (int)blockIdx.x + G - 1) / G : 0;
  const int S = p.Cin / BK;  // K slices per tile
  const bool cb_ok = p.apoz && (BM - 1) / p.HWo + 2 <= CB_IMG;

  auto tile_mn = [&](int it, int& m0, int& n0) {
    const int t = xcd_tile((int)blockIdx.x + it * G, p.tiles);
    m0 = (t / p.n_tiles) * BM;
    n0 = (t % p.n_tiles) * BN;
  };

  if (is_mfma) {
    // ======================================================================== MFMA waves
    const i32x4 xr = make_rsrc(p.x, (unsigned)((long long)p.B * p.H * p.W * p.Cin * 4));
    const i32x4 wr = make_rsrc(p.w, (unsigned)((long long)p.N * p.Cin * 4));
    constexpr unsigned OOB = 0x80000000u;
    int a_row[A_CH], a_c4[A_CH], b_row[B_CH], b_c4[B_CH];
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      a_row[i] = (tid + i * MT_THREADS) / (BK / 4);
      a_c4[i] = (tid + i * MT_THREADS) % (BK / 4);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      b_row[i] = (tid + i * MT_THREADS) / (BK / 4);
      b_c4[i] = (tid + i * MT_THREADS) % (BK / 4);
    }
    unsigned a_off[A_CH], b_off[B_CH];
    f32x4 ra[A_CH], rb[B_CH];
    auto setup = [&](int it) {  // per-tile operand byte offsets (slice 0)
      int m0, n0;
      tile_mn(it, m0, n0);
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const int m = m0 + a_row[i];
        unsigned o = OOB;
        if (m < p.M) {
          const int b = m / p.HWo, r = m - b * p.HWo;
          const int oh = r / p.Wo, ow = r - oh * p.Wo;
          o = (unsigned)((((long long)b * p.H + oh * p.stride) * p.W + ow * p.stride) * p.Cin + a_c4[i] * 4) * 4u;
        }
        a_off[i] = o;
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + b_row[i];
        b_off[i] = n < p.N ? (unsigned)(n * p.Cin + b_c4[i] * 4) * 4u : OOB;
      }
    };
    const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
    const int li = lane & 31, lh = lane >> 5;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // One flat stream of K slices over this workgroup's tiles, global loads two slices ahead
    // (register sets R0 / R1 by slice parity: the loop is unrolled by 2 so the parity is static)
    // and LDS double-buffered: a slice's loads have two slices of MFMAs to land.
    const int total = my_tiles * S;
    int ld_tile = 0, ld_kt = 0;  // next slice to load
    f32x4 ra1[A_CH], rb1[B_CH];
    auto issue = [&](f32x4* xa, f32x4* xb) {
      if (ld_kt == 0) setup(ld_tile);
      const unsigned ko = (unsigned)(ld_kt * BK) * 4u;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) xa[i] = buf_load_f32x4(xr, (int)(a_off[i] != OOB ? a_off[i] + ko : OOB), 0, 0);
#pragma unroll
      for (int i = 0; i < B_CH; ++i) xb[i] = buf_load_f32x4(wr, (int)(b_off[i] != OOB ? b_off[i] + ko : OOB), 0, 0);
      if (++ld_kt == S) {
        ld_kt = 0;
        ++ld_tile;
      }
    };
    auto put = [&](const f32x4* xa, const f32x4* xb, int buf) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) *reinterpret_cast<f32x4*>(stage + buf * STAGE + a_row[i] * LDK + a_c4[i] * 4) = xa[i];
#pragma unroll
      for (int i = 0; i < B_CH; ++i)
        *reinterpret_cast<f32x4*>(stage + buf * STAGE + (BM + b_row[i]) * LDK + b_c4[i] * 4) = xb[i];
    };
    int kt = 0;  // slice of the current tile being multiplied
    // slice g: multiply LDS buffer g&1; slice g+1's registers go to the other buffer; slice g+2's
    // loads are issued into the register set slice g used
    auto step = [&](int g, int buf, f32x4* xa_next, f32x4* xb_next, f32x4* xa_load, f32x4* xb_load) {
      if (g + 2 < total) issue(xa_load, xb_load);
      const float* a_base = stage + buf * STAGE + (wm0 + li) * LDK + lh * 16;
      const float* b_base = stage + buf * STAGE + (BM + wn0 + li) * LDK + lh * 16;
      float4 af[2][TM], bf[2][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[0][i] = *reinterpret_cast<const float4*>(a_base + i * 32 * LDK);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[0][j] = *reinterpret_cast<const float4*>(b_base + j * 32 * LDK);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < 3) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            af[(c + 1) & 1][i] = *reinterpret_cast<const float4*>(a_base + i * 32 * LDK + (c + 1) * 4);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            bf[(c + 1) & 1][j] = *reinterpret_cast<const float4*>(b_base + j * 32 * LDK + (c + 1) * 4);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c & 1][i][s], bf[c & 1][j][s], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      if (g + 1 < total) put(xa_next, xb_next, buf ^ 1);
      lds_sync();  // K_kt
      if (++kt == S) {  // tile done: hand the accumulators to the memory waves
        kt = 0;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              outb[(wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * LDT + wn0 + j * 32 + li] = acc[i][j][r];
              acc[i][j][r] = 0.f;
            }
        lds_sync();  // R: the output tile is complete
      }
    };
    if (total > 0) {
      issue(ra, rb);
      if (total > 1) issue(ra1, rb1);
      put(ra, rb, 0);
    }
    lds_sync();  // P0
    for (int g = 0; g < total; g += 2) {
      step(g, 0, ra1, rb1, ra, rb);
      if (g + 1 < total) step(g + 1, 1, ra, rb, ra1, rb1);
    }
    for (int i = 0; i <= S; ++i) lds_sync();  // drain: the memory waves finish the last tile
    lds_sync();  // final (matches the memory waves' flush barrier)
    return;
  }

  // ========================================================================== memory waves
  const int mt = tid - MT_THREADS;
  const int c4 = mt % C4, row0 = mt / C4;
  for (int t = mt; t < 2 * CB_IMG * BN; t += MEM_THREADS) (&cb[0][0])[t] = 0.f;

  auto flush_cb = [&](int it) {  // global atomics of tile it's LDS counts; clears them
    int m0, n0;
    tile_mn(it, m0, n0);
    float* c = cb[it & 1];
    const int b_first = m0 / p.HWo;
    const int n_img = (min(m0 + BM, p.M) - 1) / p.HWo - b_first + 1;
    for (int t = mt; t < n_img * BN; t += MEM_THREADS) {
      const int col = n0 + t % BN;
      const float v = c[t];
      if (v > 0.f && col < p.N) atomicAdd(p.apoz + (long long)(b_first + t / BN) * p.N + col, v);
      c[t] = 0.f;
    }
  };

  int cur_b = -1;
  float4 cnt = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sc4 = make_float4(1.f, 1.f, 1.f, 1.f), sh4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool want_rm = p.res || p.mask;
  // Interval iv (0..S-1) of tile j's epilogue covers passes [iv*NP/S, (iv+1)*NP/S), processed in
  // chunks of PC; the residual / mask quads of an interval's first chunk are loaded one interval
  // ahead (they land while the previous interval's stores drain: vmcnt retires in order).
  constexpr int PC = 4;
  auto load_chunk = [&](int j, int q0, int q1, float4* r, float4* mk) {
    int tm0, tn0;
    tile_mn(j, tm0, tn0);
    const int n = tn0 + c4 * 4;
#pragma unroll
    for (int u = 0; u < PC; ++u) {
      const int m = tm0 + row0 + (q0 + u) * RSTEP;
      const bool ok = q0 + u < q1 && n < p.N && m < p.M;
      r[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      mk[u] = make_float4(1.f, 1.f, 1.f, 1.f);
      if (ok && p.res) r[u] = *reinterpret_cast<const float4*>(p.res + (long long)m * p.N + n);
      if (ok && p.mask) mk[u] = *reinterpret_cast<const float4*>(p.mask + (long long)m * p.N + n);
    }
  };
  float4 rq[PC], mq[PC];
#pragma unroll
  for (int u = 0; u < PC; ++u) {
    rq[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    mq[u] = make_float4(1.f, 1.f, 1.f, 1.f);
  }

  lds_sync();  // P0
  for (int i = 0; i <= S; ++i) lds_sync();  // tile 0's K loop and hand-over: nothing to do yet
  if (my_tiles > 0 && want_rm) load_chunk(0, 0, min(NP / S, PC), rq, mq);
  for (int j = 0; j < my_tiles; ++j) {
    int m0, n0;
    tile_mn(j, m0, n0);
    const int b_first = m0 / p.HWo;
    const int n = n0 + c4 * 4;
    const bool nok = n < p.N;
    if (nok) {
      if (p.scale) sc4 = *reinterpret_cast<const float4*>(p.scale + n);
      if (p.shift) sh4 = *reinterpret_cast<const float4*>(p.shift + n);
    }
    if (cb_ok && j >= 1) flush_cb(j - 1);
    float* cbj = cb[j & 1];
    auto count_out = [&]() {  // the open run of counts -> LDS (or global) counters
      float* ap = cb_ok ? cbj + (cur_b - b_first) * BN + c4 * 4 : p.apoz + (long long)cur_b * p.N + n;
      if (cnt.x > 0.f) atomicAdd(ap, cnt.x);
      if (cnt.y > 0.f) atomicAdd(ap + 1, cnt.y);
      if (cnt.z > 0.f) atomicAdd(ap + 2, cnt.z);
      if (cnt.w > 0.f) atomicAdd(ap + 3, cnt.w);
    };
    for (int iv = 0; iv < S; ++iv) {
      const int p0 = iv * NP / S, p1 = (iv + 1) * NP / S;
      float4 nrq[PC], nmq[PC];
      if (want_rm) {
        const int jn = iv + 1 < S ? j : j + 1, ivn = iv + 1 < S ? iv + 1 : 0;
        const int q0 = ivn * NP / S, q1 = (ivn + 1) * NP / S;
        if (jn < my_tiles) load_chunk(jn, q0, min(q1, q0 + PC), nrq, nmq);
      }
      for (int c0 = p0; c0 < p1; c0 += PC) {
        if (c0 != p0 && want_rm) load_chunk(j, c0, min(p1, c0 + PC), rq, mq);
#pragma unroll
        for (int u = 0; u < PC; ++u) {
          const int pass = c0 + u;
          const int row = row0 + pass * RSTEP;
          const int m = m0 + row;
          if (pass >= p1 || !nok || m >= p.M) continue;
          float4 v = *reinterpret_cast<const float4*>(outb + row * LDT + c4 * 4);
          v.x = v.x * sc4.x + sh4.x + rq[u].x;
          v.y = v.y * sc4.y + sh4.y + rq[u].y;
          v.z = v.z * sc4.z + sh4.z + rq[u].z;
          v.w = v.w * sc4.w + sh4.w + rq[u].w;
          if (p.mask) {
            v.x = mq[u].x > 0.f ? v.x : 0.f;
            v.y = mq[u].y > 0.f ? v.y : 0.f;
            v.z = mq[u].z > 0.f ? v.z : 0.f;
            v.w = mq[u].w > 0.f ? v.w : 0.f;
          }
          if (p.relu) {
            v.x = nan_act(v.x, p.slope);
            v.y = nan_act(v.y, p.slope);
            v.z = nan_act(v.z, p.slope);
            v.w = nan_act(v.w, p.slope);
          }
          *reinterpret_cast<float4*>(p.out + (long long)m * p.N + n) = v;
          if (p.apoz) {
            const int b = m / p.HWo;
            if (b != cur_b) {
              if (cur_b >= 0) count_out();
              cur_b = b;
              cnt = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            cnt.x += v.x > 0.f ? 1.f : 0.f;
            cnt.y += v.y > 0.f ? 1.f : 0.f;
            cnt.z += v.z > 0.f ? 1.f : 0.f;
            cnt.w += v.w > 0.f ? 1.f : 0.f;
          }
        }
      }
      if (iv == S - 1 && p.apoz && cur_b >= 0) {  // end of this tile's rows: flush the open run
        count_out();
        cur_b = -1;
        cnt = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (want_rm) {
#pragma unroll
        for (int u = 0; u < PC; ++u) {
          rq[u] = nrq[u];
          mq[u] = nmq[u];
        }
      }
      lds_sync();  // K_iv of the next tile (or a drain barrier)
    }
    lds_sync();  // R of the next tile (or the drain's)
  }
  lds_sync();  // final: every count of the last tile is in LDS
  if (cb_ok && my_tiles > 0) flush_cb(my_tiles - 1);
}

}  // namespace ws
}  // namespace tp

namespace {
int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int BN, int MEMW>
hipError_t launch_ws(const tp::ws::Args& a, hipStream_t st) {
  const int grid = std::max(8, std::min(a.tiles, cu_count()) / 8 * 8);
  tp::ws::gemm1x1_ws<BN, MEMW><<<grid, 64 * (tp::ws::MFMA_WAVES + MEMW), 0, st>>>(a);
  return hipGetLastError();
}
}  // namespace

// 1x1 convolution (stride s, no padding) / dense GEMM out = epi(x @ w^T), x NHWC (B, H, W, Cin),
// w (N, Cin), out (B, Ho, Wo, N) with Ho = (H - 1) / s + 1. variant: 0 = 128x128 tiles + 4 memory
// waves, 1 = 128x128 + 8, 2 = 128x64 + 4. res / mask: (B, Ho, Wo, N) (nullable).
extern "C" hipError_t tp_gemm1x1_ws(const float* x, const float* w, int B, int H, int W, int Cin, int N, int stride,
                                    const float* scale, const float* shift, int relu, float slope, const float* res,
                                    const float* mask, float* apoz, float* out, int variant, hipStream_t st) {
  using tp::ws::Args;
  if (Cin % 32 != 0 || Cin < 32 || N % 4 != 0 || stride < 1 || !(slope >= 0.f)) return hipErrorInvalidValue;
  Args a{};
  a.x = x;
  a.w = w;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.N = N;
  a.stride = stride;
  a.Ho = (H - 1) / stride + 1;
  a.Wo = (W - 1) / stride + 1;
  a.HWo = a.Ho * a.Wo;
  a.M = B * a.HWo;
  if ((long long)B * H * W * Cin * 4 >= (1ll << 31) || (long long)N * Cin * 4 >= (1ll << 31) ||
      (long long)a.M * N * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.slope = slope;
  a.res = res;
  a.mask = mask;
  a.apoz = apoz;
  a.out = out;
  const int bn = variant == 2 ? 64 : 128;
  a.m_tiles = (a.M + tp::ws::BM - 1) / tp::ws::BM;
  a.n_tiles = (N + bn - 1) / bn;
  a.tiles = a.m_tiles * a.n_tiles;
  switch (variant) {
    case 0: return launch_ws<128, 4>(a, st);
    case 1: return launch_ws<128, 8>(a, st);
    case 2: return launch_ws<64, 4>(a, st);
  }
  return hipErrorInvalidValue;
}
