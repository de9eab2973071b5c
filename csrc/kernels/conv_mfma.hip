// Implicit-GEMM 3x3 / 1x1 convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32) with
// fused epilogues — the compute core of the fused attribution engine (SURVEY.md §2.5 K1/K2/K4,
// K5 eval-mode BN folded, K6 NaN-propagating ReLU, K7 2x2 max-pool, K9c Taylor reduction).
//
// Layout: activations NHWC (channels contiguous), weights [Cout][KS][KS][Cin] = [n][k] with
// k = (kh*KS + kw)*Cin + ci. GEMM view: M = B*H*W output pixels, N = Cout, K = KS*KS*Cin.
// stride 1, padding (KS-1)/2 (the VGG / classifier shapes). dgrad of such a conv is the same
// conv of dL/dy with flipped, transposed weights, so one kernel serves forward and backward.
//
// Tiling: 256 threads = 4 waves; block tile BM x BN, wave tile WM x WN made of 32x32 MFMA
// tiles; K staged through double-buffered LDS in BK=32 slices (one conv tap, 32 channels).
// Inside a K-slice lane (i, h) feeds k = h*16 + s at MFMA step s (any bijection works as long
// as A and B agree), so each lane reads its 16 operands with 4 ds_read_b128 per fragment from
// rows padded to 36 floats (144 B = 9 bank slots: conflict-free for ds_read_b128 groups).
//
// M ordering: plain (b, oh, ow) or POOLED_M (b, oh/2, ow/2, dy, dx). With POOLED_M the four
// pixels of every 2x2 pooling window are rows 4g..4g+3 of a 32x32 MFMA tile, which the
// accumulator layout (row = (r&3) + 8(r>>2) + 4(lane>>5)) places in ONE lane's registers
// r = 4g..4g+3 — the max-pool is four in-register max operations.
#include "tp_common.h"

#include <cstdlib>

namespace tp {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// 4 fp32 -> 4 bf16 (round to nearest even: v_cvt_pk_bf16_f32), packed in 2 dwords
__device__ __forceinline__ uint2 bf16x4_of(const f32x4 v) {
  return __builtin_bit_cast(uint2, __builtin_convertvector(v, bf16x4));
}

constexpr int CFG_BF16 = 256;  // tile-config flag: bf16 operands (conv_igemm BF), fp32 accumulation
constexpr int CFG_SK = 32;     // tile-config flag: stream-K split of the tiles x k-slices space (GEN 1, one K pass)
constexpr int CFG_SB = 64;     // tile-config flag: single-buffered LDS stage (GEN 1 1x1 forward, one K pass): half the
                               // LDS, twice the co-resident blocks for the short-K convs (profiles/train/lowk_*)

enum Epi : int {
  EPI_FWD = 0,       // y = relu?(acc*scale[n] + shift[n]) stored NHWC
  EPI_FWD_POOL = 1,  // + 2x2 max-pool: pooled value + argmax byte
  EPI_BWD = 2,       // dgrad epilogue: Taylor partial of the consumer's activation, masked/scaled grad
  EPI_PARTIAL = 3,   // raw split-K partial slab (epilogue applied by conv_epilogue)
  EPI_FWD_TAY = 4,   // GEN 1x1 / GEN 3 3x3 stride-2 data gradient: EPI_FWD's LDS epilogue + Taylor partials (tay_part); a
                     // separate instantiation so the partials' registers never burden EPI_FWD
};

struct ConvArgs {
  // operands
  const float* x;           // A source: NHWC [B][H][W][Cin] (or pooled grad [B][H/2][W/2][Cin] if UNPOOL)
  const uint8_t* x_argmax;  // UNPOOL: argmax bytes of the pooled grad
  const float* w;           // [N][K]
  // shape
  int B, H, W, Cin, N, K;   // K = KS*KS*Cin
  int M;                    // B*H*W
  int k_tiles_per_split;
  long long x_elems;        // elements of the A source tensor (buffer-descriptor bound)
  // epilogue
  const float* scale;       // [N] (EPI_FWD*) or BN scale of the consumer layer (EPI_BWD)
  const float* shift;       // [N]
  int relu;                 // EPI_FWD*: apply ReLU
  float* out;               // EPI_FWD: [M][N]; POOL: [M/4][N]; BWD: masked grad [M][N] (nullable); PARTIAL: slab
  uint8_t* out_argmax;      // POOL: [M/4][N]
  const float* act;         // EPI_BWD: activation [M][N] the grad refers to
  float* taylor;            // EPI_BWD: [B][N] fp32 per-sample sums (atomic), nullable
  int HWo;                  // EPI_BWD/EPI_FWD apoz: pixels per image at the output's resolution
  // GEN (general strided conv) geometry: output Ho x Wo, stride, zero padding
  int Ho, Wo, stride, pad;
  const float* res;         // EPI_FWD: residual [M][N] added before the ReLU (nullable)
  float* apoz;              // EPI_FWD: [B][N] counts of positive outputs (exact integers), nullable
  int epi_lds;              // GEN: 1 -> two-phase LDS-transposed forward epilogue (TP_GEN_EPI=0 disables)
  int sb;                   // GEN 1 1x1 EPI_FWD: 1 -> the single-buffered (SB) instantiation (CFG_SB)
  int tay_group;            // EPI_BWD: >0 -> N = P pixel groups x tay_group channels (a dense-GEMM conv);
                            // Taylor of column n goes to slot n / tay_group of a (P, B, tay_group) slab
  // GEN dgrad epilogue (ResNet backward engine)
  const float* mask;        // [M][N] activation: out = mask > 0 ? v : 0 (ReLU backward), nullable
  int res_stride;           // res is (B, ceil(Ho/s), ceil(Wo/s), N) added at pixels with oh, ow % s == 0
                            // (gradient of a strided 1x1 downsample conv scattered back), 1 = dense
  int tay_mode;             // EPI_BWD partials: 0 Taylor -(g*a), 1 Sensitivity |g|, 2 |g| where a > 0
  int parity;               // GEN 3: rows ordered (oh%2, ow%2, b, oh/2, ow/2) so a tile sees few taps
  float slope;              // activation: 0 = ReLU, > 0 = LeakyReLU negative slope (fwd relu flag /
                            // EPI_BWD mask of the consumer activation)
  int res_rows;             // > 0: residual row = output row % res_rows (one (res_rows, N) residual
                            // broadcast over row blocks: Shapley prefix-delta GEMM)
  double* bnpart;           // GEN EPI_FWD LDS epilogue, no split: per M tile the column sums and sums of
                            // squares of the stored outputs, [m_tile][2][N] (training BN statistics)
  float* tay_part;          // GEN EPI_FWD LDS epilogue with a mask (data gradient), no split: Taylor
                            // partials -(v * mask) (tay_mode 1: |v|) per (image, column) of every M
                            // tile, slot r = m_tile - first tile of the image: [R][B][N], one writer each
  // stream-K (GEN 1, one K pass; see tp_conv_gen4): sk_blocks = P > 0 blocks share the tiles x
  // k-slices iteration space in equal contiguous ranges; a tile cut by a range boundary f has its
  // two raw partial accumulator sets in sk_ws[f][0 / 1] (BM * BN floats each) and gets its
  // epilogue from the fixup launch (sk_fixup = 1, block f): slot 0 + slot 1 in that fixed order
  int sk_blocks;
  int sk_fixup;
  long long sk_iters;
  float* sk_ws;
  // training data gradient of a residual block's conv1 (GEN 1, res_stride 1; see tp_conv_gen5):
  const uint8_t* res_bits;  // the residual is the raw gradient of the block's ReLU output: masked here by
                            // that ReLU's bit mask (byte (pix*N + n) / 4, bit n % 4), so the BN
                            // backward never writes the masked copy
  const float* bnb_y;       // with bnpart: the BatchNorm whose output this gradient reaches — its input
  const float* bnb_mean;    // [M][N], batch mean / invstd [N] and its ReLU bit mask (nullable: no
  const float* bnb_invstd;  // ReLU); the tile sums become (sum gm, sum gm * xhat), gm = the masked
  const uint8_t* bnb_bits;  // gradient, xhat = (y - mean) * invstd: that BN's backward statistics
};

// one ReLU bit-mask nibble (channels n..n+3 of pixel pix, N % 4 == 0) applied to a quad
__device__ __forceinline__ float4 bits_mask(const uint8_t* bits, long long pix, int N, int n, float4 v) {
  const unsigned b = bits[(pix * N + n) >> 2];
  return make_float4(b & 1u ? v.x : 0.f, b & 2u ? v.y : 0.f, b & 4u ? v.z : 0.f, b & 8u ? v.w : 0.f);
}

// Taylor slots R of the GEN epilogue partials for tile height bm: the M tiles an image can touch
__host__ __device__ constexpr int gen_tay_slots(int bm, int HWo) { return (HWo + bm - 2) / bm + 1; }
constexpr int GEN_TAY_IMG = 4;  // images per tile the epilogue partials support (host-checked)

// GEN 3 output row m -> (image, oh, ow). Parity order makes each stride-2 phase class one
// contiguous range of B*Ho*Wo/4 rows: all but the (at most 3) boundary tiles see ONE class and
// iterate exactly the taps it uses (1, 2, 2 or 4 of the 9 for a 3x3/s2 dgrad). Classes are laid
// out heaviest first (longest-job-first dispatch: no tail of 4-tap tiles at the end).
__device__ __forceinline__ void gen3_pix(const ConvArgs& p, int m, int& b, int& oh, int& ow) {
  if (p.parity) {
    const int W2 = p.Wo >> 1, Q = (p.Ho >> 1) * W2, BQ = p.B * Q;
    const int cq = m / BQ, r = m - cq * BQ;
    const int cls = 3 - cq;  // heaviest phase (4 taps) first: its tiles are dispatched first
    b = r / Q;
    const int q = r - b * Q;
    const int qy = q / W2;
    oh = qy * 2 + (cls >> 1);
    ow = (q - qy * W2) * 2 + (cls & 1);
  } else {
    const int HW = p.Ho * p.Wo;
    b = m / HW;
    const int r = m - b * HW;
    oh = r / p.Wo;
    ow = r - oh * p.Wo;
  }
}

// Taylor slab index of (image b, GEMM column n)
__device__ __forceinline__ long long tay_index(const ConvArgs& p, long long b, int n) {
  if (p.tay_group <= 0) return b * p.N + n;
  const int B = p.M / p.HWo;
  return ((long long)(n / p.tay_group) * B + b) * p.tay_group + n % p.tay_group;
}

template <int BM, int BN, int WM, int WN>
struct Tile {
  static constexpr int BK = 32;
  static constexpr int LDK = BK + 4;  // padded row (floats)
  static constexpr int WAVES_N = BN / WN;
  static constexpr int TM = WM / 32, TN = WN / 32;
  static constexpr int NW = (BM / WM) * (BN / WN);  // waves per block
  static constexpr int NT = 64 * NW;                 // threads per block
  static constexpr int A_CHUNKS = BM * BK / 4 / NT;  // float4 per thread per slice
  static constexpr int B_CHUNKS = BN * BK / 4 / NT;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block");
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small");
};

constexpr int tile_threads(int bm, int bn, int wm, int wn) { return 64 * (bm / wm) * (bn / wn); }

__device__ __forceinline__ void pix_of(int m, int H, int W, bool pooled, int& b, int& oh, int& ow) {
  const int HW = H * W;
  b = m / HW;
  const int r = m - b * HW;
  if (pooled) {
    const int w2 = W >> 1;
    const int j = r >> 2, q = r & 3;
    oh = (j / w2) * 2 + (q >> 1);
    ow = (j % w2) * 2 + (q & 1);
  } else {
    oh = r / W;
    ow = r - oh * W;
  }
}

// Bijective XCD-aware remap: consecutive logical tiles share an XCD (blocks b, b+8 share one).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Residual quad at output pixel ``pix`` (linear NHWC pixel index), columns n..n+3; res_stride
// > 1 reads a strided-conv gradient that lives at the even-phase pixels only.
__device__ __forceinline__ float4 res_quad(const ConvArgs& p, long long pix, int n) {
  if (p.res_rows > 0) pix %= p.res_rows;
  if (p.res_stride <= 1) return *reinterpret_cast<const float4*>(p.res + pix * p.N + n);
  const int s = p.res_stride;
  const long long HW = (long long)p.Ho * p.Wo;
  const long long b = pix / HW;
  const int r = (int)(pix - b * HW);
  const int oh = r / p.Wo, ow = r - oh * p.Wo;
  if (oh % s || ow % s) return make_float4(0.f, 0.f, 0.f, 0.f);
  const int Hr = (p.Ho + s - 1) / s, Wr = (p.Wo + s - 1) / s;
  return *reinterpret_cast<const float4*>(p.res + ((b * Hr + oh / s) * Wr + ow / s) * p.N + n);
}

// GEN = 0: stride-1 "same" convs (VGG path, precomputed tap masks); GEN = 1: general strided /
// padded conv (ResNet; 1x1 / 3x3 / 5x5), Cin % 32 == 0; GEN = 2: the same with a 4-channel
// (padded NHWC) input, where one 32-wide K slice holds 8 taps x 4 channels (7x7 stems, tiny-Cin
// 3x3 / 5x5 first layers); GEN = 3: transposed strided
// conv = data gradient of a strided conv. x is dL/dy (B, H, W, Cin = forward Cout) and output
// pixel (oh, ow) gathers y pixel ((oh + pad - kh) / s, (ow + pad - kw) / s) through tap (kh, kw)
// when the division is exact; w[n = forward ci][k = (kh, kw, co)]. With parity row order a
// tile only iterates the taps its stride phases use (1/4 of the 3x3 taps on average).
// BF (opt-in, compute_dtype=bfloat16; GEN 0 only): operands rounded to bf16 (RNE) as they are
// staged into LDS (rows of 32 bf16 = 16 dwords, padded to 20: 80-B rows keep the 16-B fragment
// reads conflict-free), products on v_mfma_f32_32x32x16_bf16 with fp32 accumulation; loads,
// epilogues and every output stay fp32. 16x the fp32 MFMA rate: the K slice is 2 MFMAs, not 16.
// SB: one LDS stage instead of two (the next K slice still loads into registers under the
// MFMAs; an extra barrier per slice before it is stored): for short-K GEMMs (K = 64-128, two to
// four slices) whose blocks are load -> MFMA -> epilogue back to back, twice the co-resident
// blocks overlap one block's epilogue / loads with another's MFMAs.
template <int BM, int BN, int WM, int WN, int KS, bool POOLED_M, bool UNPOOL, int EPI, int GEN = 0, bool BF = false,
          bool SK = false, bool SB = false>
__global__ __launch_bounds__(tile_threads(BM, BN, WM, WN), tile_threads(BM, BN, WM, WN) / 128) void conv_igemm(ConvArgs p) {
  using T = Tile<BM, BN, WM, WN>;
  constexpr int BK = T::BK, LDK = T::LDK;
  static_assert(!SB || (GEN == 1 && !BF && !SK && (EPI == EPI_FWD || EPI == EPI_FWD_TAY)),
                "single-buffered LDS: GEN 1 forward / Taylor-partial data gradient only");
  constexpr int SMEM_SB = (BM + BN) * LDK > BM * (BN + 4) + 8 * BN ? (BM + BN) * LDK : BM * (BN + 4) + 8 * BN;
  constexpr int SMEM = SB ? SMEM_SB : 2 * (BM + BN) * LDK;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  constexpr int STAGE = (BM + BN) * LDK;  // floats per pipeline stage: A rows then B rows
  constexpr int LDKB = 20;                // BF: dwords per LDS row (32 bf16 + pad)
  constexpr int STAGEB = (BM + BN) * LDKB;
  static_assert(!BF || GEN == 0, "bf16 operands: GEN 0 only");
  unsigned* smu = reinterpret_cast<unsigned*>(smem);

  constexpr int SK_PART = 2, SK_FIX = 3;  // stream-K segment modes (0: the tile's whole K range)
  constexpr int TILEF = BM * BN;          // floats of one partial accumulator set

  // one output tile (or, stream-K, a K range of it); returns early for empty tiles. ``tid``: the
  // stream-K loop passes an opaque copy of threadIdx.x so the lane-derived addressing is not
  // hoisted out of the segment loop and kept live across it.
  auto run_tile = [&](const int tid, const int tile, const int split, const int sk_kb, const int sk_ke,
                      const int sk_mode, float* sk_slab) __attribute__((always_inline)) {
  const int lane = tid & 63, wave = tid >> 6;
  const int n_tiles = (p.N + BN - 1) / BN;
  const int m_tiles = (p.M + BM - 1) / BM;
  const int m0 = (tile / n_tiles) * BM;
  const int n0 = (tile % n_tiles) * BN;
  if (m0 >= m_tiles * BM) return;
  // K slices per tap: GEN 1 / 3 take any Cin % 4 == 0 (pruned widths); the last slice of a tap is
  // zero-filled past Cin in the loads (the weight operand is 32-padded per tap), so activations
  // keep their real width in HBM
  const int cin_tiles = (p.Cin + BK - 1) / BK;
  unsigned tmask = (1u << (KS * KS)) - 1u;  // GEN 3: taps any row of this tile can use
  if constexpr (GEN == 3) {
    if (p.parity) {
      const int BQ = p.B * (p.Ho >> 1) * (p.Wo >> 1);
      const int c0 = 3 - (min(m0 + BM, p.M) - 1) / BQ, c1 = 3 - m0 / BQ;
      tmask = 0;
      for (int c = c0; c <= c1; ++c) {
        for (int t = 0; t < KS * KS; ++t)
          if ((((c >> 1) + p.pad - t / KS) & 1) == 0 && (((c & 1) + p.pad - t % KS) & 1) == 0) tmask |= 1u << t;
      }
    }
  }
  const int kt_total = GEN == 3 ? __builtin_popcount(tmask) * cin_tiles : p.K / BK;
  const int kt_begin = sk_mode ? sk_kb : GEN == 3 ? 0 : split * p.k_tiles_per_split;
  const int kt_end = sk_mode ? sk_ke : GEN == 3 ? kt_total : min(kt_total, kt_begin + p.k_tiles_per_split);

  // ---- per-thread A rows: loop-invariant offsets + a bitmask of in-bounds taps ----------
  // Loads go through buffer descriptors: an out-of-range offset returns zeros in hardware,
  // so conv padding and ragged M/N edges cost one v_cndmask instead of a branch per load.
  constexpr unsigned OOB = 0x80000000u;
  const i32x4 xr = make_rsrc(p.x, (unsigned)(p.x_elems * 4));
  const i32x4 wr = make_rsrc(p.w, (unsigned)(p.N * p.K * 4));
  const i32x4 amr = make_rsrc(p.x_argmax, UNPOOL ? (unsigned)p.x_elems : 0u);

  int a_off[T::A_CHUNKS], a_row[T::A_CHUNKS], a_c4[T::A_CHUNKS];
  unsigned a_mask[T::A_CHUNKS];
  int a_oh[T::A_CHUNKS], a_ow[T::A_CHUNKS];
#pragma unroll
  for (int i = 0; i < T::A_CHUNKS; ++i) {
    const int id = tid + i * T::NT;
    a_row[i] = id / (BK / 4);
    a_c4[i] = id % (BK / 4);
    const int m = m0 + a_row[i];
    if constexpr (GEN == 3) {
      int b = 0, oh = 0, ow = 0;
      if (m < p.M) gen3_pix(p, m, b, oh, ow);
      a_mask[i] = m < p.M ? 1u : 0u;
      a_oh[i] = oh + p.pad;
      a_ow[i] = ow + p.pad;
      a_off[i] = b * p.H * p.W * p.Cin;
      continue;
    } else if constexpr (GEN != 0) {
      // a_off = image base offset, a_oh/a_ow = top-left input pixel of the receptive field,
      // a_mask = row valid
      int b = 0, oh = 0, ow = 0;
      if (m < p.M) pix_of(m, p.Ho, p.Wo, false, b, oh, ow);
      a_mask[i] = m < p.M ? 1u : 0u;
      a_oh[i] = oh * p.stride - p.pad;
      a_ow[i] = ow * p.stride - p.pad;
      a_off[i] = b * p.H * p.W * p.Cin;
      continue;
    }
    int b = 0, oh = 0, ow = 0;
    unsigned mask = 0;
    if (m < p.M) {
      pix_of(m, p.H, p.W, POOLED_M, b, oh, ow);
#pragma unroll
      for (int t = 0; t < KS * KS; ++t) {
        const int ih = oh + t / KS - (KS - 1) / 2, iw = ow + t % KS - (KS - 1) / 2;
        if (ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) mask |= 1u << t;
      }
    }
    a_mask[i] = mask;
    a_oh[i] = oh;
    a_ow[i] = ow;
    if constexpr (UNPOOL) a_off[i] = b * (p.H >> 1) * (p.W >> 1) * p.Cin + a_c4[i] * 4;
    else a_off[i] = ((b * p.H + oh) * p.W + ow) * p.Cin + a_c4[i] * 4;
  }
  int b_off[T::B_CHUNKS], b_row[T::B_CHUNKS], b_c4[T::B_CHUNKS];
#pragma unroll
  for (int i = 0; i < T::B_CHUNKS; ++i) {
    const int id = tid + i * T::NT;
    b_row[i] = id / (BK / 4);
    b_c4[i] = id % (BK / 4);
    const int n = n0 + b_row[i];
    b_off[i] = n < p.N ? (n * p.K + b_c4[i] * 4) * 4 : -1;
  }

  f32x4 ra[T::A_CHUNKS], rb[T::B_CHUNKS];  // the buffer-load results as they are (no repacking moves)

  // GEN 1: the K slice's (tap, channel block) advance incrementally with the (strictly
  // sequential) load_tile calls instead of a runtime division per slice; a 1x1 conv's operand
  // address is loop-invariant up to the channel offset, so it is formed once (a_k1).
  int ld_tap = 0, ld_cs = 0;
  unsigned a_k1[GEN == 1 && KS == 1 ? T::A_CHUNKS : 1];
  if constexpr (GEN == 3) {
    ld_tap = tmask ? __builtin_ctz(tmask) : KS * KS;  // kt_begin == 0 (GEN 3 never splits K)
  }
  if constexpr (GEN == 1) {
    ld_tap = kt_begin / cin_tiles;
    ld_cs = kt_begin - ld_tap * cin_tiles;
    if constexpr (KS == 1) {
#pragma unroll
      for (int i = 0; i < T::A_CHUNKS; ++i) {
        const int ih = a_oh[i], iw = a_ow[i];
        const bool ok = a_mask[i] && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
        a_k1[i] = ok ? (unsigned)(a_off[i] + (ih * p.W + iw) * p.Cin + a_c4[i] * 4) * 4u : OOB;
      }
    }
  }

  auto load_tile = [&](int kt) {
    int kb = kt;  // K slice of the weight operand
    if constexpr (GEN == 3) {
      // (tap, channel block) advance with the sequential calls: the next tap is the next set
      // bit of the tile's tap mask (no division / bit search per slice)
      const int tap = ld_tap, cs = ld_cs;
      kb = tap * cin_tiles + cs;
      const int kh = tap / KS, kw = tap % KS, s = p.stride;
      const bool s2 = s == 2;  // the common stride: shifts instead of integer divisions
#pragma unroll
      for (int i = 0; i < T::A_CHUNKS; ++i) {
        const int th = a_oh[i] - kh, tw = a_ow[i] - kw;
        const int yh = s2 ? th >> 1 : th / s, yw = s2 ? tw >> 1 : tw / s;
        const bool ok = a_mask[i] && th >= 0 && tw >= 0 && yh * s == th && yw * s == tw && yh < p.H && yw < p.W &&
                        cs * BK + a_c4[i] * 4 < p.Cin;
        const unsigned vo = ok ? (unsigned)(a_off[i] + (yh * p.W + yw) * p.Cin + cs * BK + a_c4[i] * 4) * 4u : OOB;
        const f32x4 g = buf_load_f32x4(xr, (int)vo, 0, 0);
        ra[i] = g;
      }
      if (++ld_cs == cin_tiles) {
        ld_cs = 0;
        const unsigned rest = tmask & ~((2u << tap) - 1u);
        ld_tap = rest ? __builtin_ctz(rest) : KS * KS;
      }
    } else if constexpr (GEN == 1 && KS == 1) {
      const unsigned coff = (unsigned)(ld_cs * BK) * 4u;
#pragma unroll
      for (int i = 0; i < T::A_CHUNKS; ++i) {
        const bool cok = ld_cs * BK + a_c4[i] * 4 < p.Cin;  // past a pruned width: zeros
        const f32x4 g = buf_load_f32x4(xr, (int)(a_k1[i] != OOB && cok ? a_k1[i] + coff : OOB), 0, 0);
        ra[i] = g;
      }
      ++ld_cs;
    } else if constexpr (GEN != 0) {
#pragma unroll
      for (int i = 0; i < T::A_CHUNKS; ++i) {
        int tap, c;
        if constexpr (GEN == 2) {
          tap = kt * 8 + a_c4[i];
          c = 0;
        } else {
          tap = ld_tap;
          c = ld_cs * BK + a_c4[i] * 4;
        }
        const int ih = a_oh[i] + tap / KS, iw = a_ow[i] + tap % KS;
        const bool ok = a_mask[i] && tap < KS * KS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W &&
                        (GEN == 2 || c < p.Cin);
        const unsigned vo = ok ? (unsigned)(a_off[i] + (ih * p.W + iw) * p.Cin + c) * 4u : OOB;
        const f32x4 g = buf_load_f32x4(xr, (int)vo, 0, 0);
        ra[i] = g;
      }
      if constexpr (GEN == 1) {
        if (++ld_cs == cin_tiles) {
          ld_cs = 0;
          ++ld_tap;
        }
      }
    } else {
    const int tap = kt / cin_tiles;
    const int c0 = (kt - tap * cin_tiles) * BK;
    const int dh = tap / KS - (KS - 1) / 2, dw = tap % KS - (KS - 1) / 2;
#pragma unroll
    for (int i = 0; i < T::A_CHUNKS; ++i) {
      const bool ok = (a_mask[i] >> tap) & 1u;
      if constexpr (UNPOOL) {
        const int ih = a_oh[i] + dh, iw = a_ow[i] + dw;
        const int off = a_off[i] + ((ih >> 1) * (p.W >> 1) + (iw >> 1)) * p.Cin + c0;
        const unsigned vo = ok ? (unsigned)off * 4u : OOB;
        const f32x4 g = buf_load_f32x4(xr, (int)vo, 0, 0);
        const unsigned am = buf_load_u32(amr, (int)(ok ? (unsigned)off : OOB), 0, 0);
        const unsigned q = (unsigned)(((ih & 1) << 1) | (iw & 1));
        float4 v;
        v.x = ((am >> 0) & 0xffu) == q ? g[0] : 0.f;
        v.y = ((am >> 8) & 0xffu) == q ? g[1] : 0.f;
        v.z = ((am >> 16) & 0xffu) == q ? g[2] : 0.f;
        v.w = ((am >> 24) & 0xffu) == q ? g[3] : 0.f;
        ra[i] = f32x4{v.x, v.y, v.z, v.w};
      } else {
        const int delta = (dh * p.W + dw) * p.Cin + c0;  // wave-uniform
        const unsigned vo = ok ? (unsigned)(a_off[i] + delta) * 4u : OOB;
        const f32x4 g = buf_load_f32x4(xr, (int)vo, 0, 0);
        ra[i] = g;
      }
    }
    }
#pragma unroll
    for (int i = 0; i < T::B_CHUNKS; ++i) {
      const unsigned vo = b_off[i] >= 0 ? (unsigned)(b_off[i] + kb * BK * 4) : OOB;
      const f32x4 g = buf_load_f32x4(wr, (int)vo, 0, 0);
      rb[i] = g;
    }
  };
  auto store_tile = [&](int buf) {
    if constexpr (BF) {  // round to bf16 (RNE) on the way into LDS: 4 fp32 -> 2 dwords
#pragma unroll
      for (int i = 0; i < T::A_CHUNKS; ++i)
        *reinterpret_cast<uint2*>(smu + buf * STAGEB + a_row[i] * LDKB + a_c4[i] * 2) = bf16x4_of(ra[i]);
#pragma unroll
      for (int i = 0; i < T::B_CHUNKS; ++i)
        *reinterpret_cast<uint2*>(smu + buf * STAGEB + (BM + b_row[i]) * LDKB + b_c4[i] * 2) = bf16x4_of(rb[i]);
      return;
    }
#pragma unroll
    for (int i = 0; i < T::A_CHUNKS; ++i)
      *reinterpret_cast<f32x4*>(smem + buf * STAGE + a_row[i] * LDK + a_c4[i] * 4) = ra[i];
#pragma unroll
    for (int i = 0; i < T::B_CHUNKS; ++i)
      *reinterpret_cast<f32x4*>(smem + buf * STAGE + (BM + b_row[i]) * LDK + b_c4[i] * 4) = rb[i];
  };

  f32x16 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm0 = (wave / T::WAVES_N) * WM;
  const int wn0 = (wave % T::WAVES_N) * WN;
  const int li = lane & 31, lh = lane >> 5;

  if (sk_mode == SK_FIX) {  // stream-K fixup: the tile's two partial sets, slot 0 + slot 1 (fixed order)
    const float* s0 = sk_slab + (size_t)wave * (T::TM * T::TN * 1024);
    const float* s1 = s0 + TILEF;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = ((i * T::TN + j) * 16 + r) * 64 + lane;
          acc[i][j][r] = s0[o] + s1[o];
        }
  } else if (kt_begin < kt_end) {
    load_tile(kt_begin);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt_begin; kt < kt_end; ++kt) {
      const bool more = kt + 1 < kt_end;
      if (more) load_tile(kt + 1);  // global loads in flight under the MFMAs below
      if constexpr (BF) {
        // lane (li, lh) feeds k = 16 s2 + 8 lh + e of the slice (A and B agree): one 16-B read
        // per fragment per MFMA
        const unsigned* a_bb = smu + buf * STAGEB + (wm0 + li) * LDKB + lh * 4;
        const unsigned* b_bb = smu + buf * STAGEB + (BM + wn0 + li) * LDKB + lh * 4;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u32x4 afb[T::TM], bfb[T::TN];
#pragma unroll
          for (int i = 0; i < T::TM; ++i) afb[i] = *reinterpret_cast<const u32x4*>(a_bb + i * 32 * LDKB + s2 * 8);
#pragma unroll
          for (int j = 0; j < T::TN; ++j) bfb[j] = *reinterpret_cast<const u32x4*>(b_bb + j * 32 * LDKB + s2 * 8);
#pragma unroll
          for (int i = 0; i < T::TM; ++i)
#pragma unroll
            for (int j = 0; j < T::TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, afb[i]),
                                                                  __builtin_bit_cast(bf16x8, bfb[j]), acc[i][j], 0, 0, 0);
        }
        if (more) store_tile(buf ^ 1);
        __syncthreads();
        buf ^= 1;
        continue;
      }
      const float* a_base = smem + buf * STAGE + (wm0 + li) * LDK + lh * 16;
      const float* b_base = smem + buf * STAGE + (BM + wn0 + li) * LDK + lh * 16;
      // software-pipelined fragment reads: chunk c+1 is read while chunk c feeds the MFMAs
      float4 af[2][T::TM], bf[2][T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i) af[0][i] = *reinterpret_cast<const float4*>(a_base + i * 32 * LDK);
#pragma unroll
      for (int j = 0; j < T::TN; ++j) bf[0][j] = *reinterpret_cast<const float4*>(b_base + j * 32 * LDK);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < 3) {
#pragma unroll
          for (int i = 0; i < T::TM; ++i)
            af[(c + 1) & 1][i] = *reinterpret_cast<const float4*>(a_base + i * 32 * LDK + (c + 1) * 4);
#pragma unroll
          for (int j = 0; j < T::TN; ++j)
            bf[(c + 1) & 1][j] = *reinterpret_cast<const float4*>(b_base + j * 32 * LDK + (c + 1) * 4);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int i = 0; i < T::TM; ++i)
#pragma unroll
            for (int j = 0; j < T::TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c & 1][i][s], bf[c & 1][j][s], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
      if constexpr (SB) {  // one stage: every wave is done reading it before the next slice lands
        if (more) {
          __syncthreads();
          store_tile(0);
        }
        __syncthreads();
      } else {
        if (more) store_tile(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
  }
  if (sk_mode == SK_PART) {  // stream-K: this block's K range of the tile, raw, one 256-B row per store
    float* d = sk_slab + (size_t)wave * (T::TM * T::TN * 1024);
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) d[((i * T::TN + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    return;
  }

  // ---- GEN forward / partial epilogue: transpose through LDS, float4 rows ---------------
  // (memory-bound 1x1 convs: scalar per-lane stores + residual loads ran at ~2 TB/s)
  if constexpr (GEN != 0 && (EPI == EPI_FWD || EPI == EPI_FWD_TAY || EPI == EPI_PARTIAL)) {
   if (p.epi_lds) {
    constexpr int LDT = BN + 4;
    constexpr int CB_IMG = 8;  // images per block whose counts are reduced in LDS
    static_assert(BM * LDT + CB_IMG * BN <= SMEM, "output tile must fit in the staging LDS");
    float* ts = smem;  // the main loop ended with a barrier
    float* cb = smem + BM * LDT;  // APoZ counts [image in block][column]
    const int b_first = m0 / p.HWo;
    // Taylor partial row groups: one image (GEN 1), or one (stride phase, image) of the parity
    // row order (GEN 3: Ho / 2 x Wo / 2 contiguous rows each)
    const int tgs = (GEN == 3 && p.parity) ? (p.Ho >> 1) * (p.Wo >> 1) : p.HWo;
    const int g_first = m0 / tgs;
    const bool cb_lds = (EPI == EPI_FWD || EPI == EPI_FWD_TAY) && p.apoz && (min(m0 + BM, p.M) - 1) / p.HWo - b_first < CB_IMG;
    if (cb_lds)
      for (int t = tid; t < CB_IMG * BN; t += T::NT) cb[t] = 0.f;
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ts[(wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * LDT + wn0 + j * 32 + li] = acc[i][j][r];
    __syncthreads();
    constexpr int C4 = BN / 4;
    static_assert(T::NT % C4 == 0, "thread -> column-quad mapping");
    const int c4 = tid % C4;
    const int n = n0 + c4 * 4;
    const bool ncol_ok = n < p.N;
    float4 sc4 = make_float4(1.f, 1.f, 1.f, 1.f), sh4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bm4 = make_float4(0.f, 0.f, 0.f, 0.f), bi4 = bm4;  // bnb: that BN's mean / invstd
    if constexpr (EPI == EPI_FWD || EPI == EPI_FWD_TAY) {
      if (ncol_ok && p.scale) sc4 = *reinterpret_cast<const float4*>(p.scale + n);
      if (ncol_ok && p.shift) sh4 = *reinterpret_cast<const float4*>(p.shift + n);
    }
    if constexpr (GEN == 1 && EPI == EPI_FWD) {
      if (ncol_ok && p.bnb_y) {
        bm4 = *reinterpret_cast<const float4*>(p.bnb_mean + n);
        bi4 = *reinterpret_cast<const float4*>(p.bnb_invstd + n);
      }
    }
    int cur_b = -1;
    float4 cnt = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bs = make_float4(0.f, 0.f, 0.f, 0.f), bq = bs;  // bnpart: this thread's column-quad sums
    constexpr int NTQ = EPI == EPI_FWD_TAY ? GEN_TAY_IMG : 1;
    float4 tq[NTQ];  // tay_part: this thread's column-quad partial per image slot of the tile
#pragma unroll
    for (int i = 0; i < NTQ; ++i) tq[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    // rows are visited in passes of RSTEP; the residual / mask quads of PF passes are loaded
    // together first (PF global loads in flight per thread instead of one round trip per row)
    constexpr int RSTEP = T::NT / C4, RPT = BM / RSTEP, PF = RPT < 4 ? RPT : 4;
    static_assert(BM % RSTEP == 0 && RPT % PF == 0, "epilogue row passes");
    const int row0 = tid / C4;
    for (int it0 = 0; it0 < RPT; it0 += PF) {
      float4 rq[PF], mq[PF], yq[PF];
      long long pq[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int m = m0 + row0 + (it0 + u) * RSTEP;
        const bool ok = ncol_ok && m < p.M;
        long long pix = m;
        if constexpr (GEN == 3) {
          if (ok) {
            int b, oh, ow;
            gen3_pix(p, m, b, oh, ow);
            pix = ((long long)b * p.Ho + oh) * p.Wo + ow;
          }
        }
        pq[u] = pix;
        rq[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        mq[u] = make_float4(1.f, 1.f, 1.f, 1.f);
        yq[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (EPI != EPI_PARTIAL) {
          if (ok && p.res) rq[u] = res_quad(p, pix, n);
          if (ok && p.mask) mq[u] = *reinterpret_cast<const float4*>(p.mask + pix * p.N + n);
        }
        if constexpr (GEN == 1 && EPI == EPI_FWD) {
          if (ok && p.res_bits) rq[u] = bits_mask(p.res_bits, pix, p.N, n, rq[u]);
          if (ok && p.bnb_y) yq[u] = *reinterpret_cast<const float4*>(p.bnb_y + pix * p.N + n);
        }
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
      const int row = row0 + (it0 + u) * RSTEP;
      const int m = m0 + row;
      if (!ncol_ok || m >= p.M) continue;
      float4 v = *reinterpret_cast<const float4*>(ts + row * LDT + c4 * 4);
      if constexpr (EPI == EPI_PARTIAL) {
        *reinterpret_cast<float4*>(p.out + ((long long)split * p.M + m) * p.N + n) = v;
      } else {
        const long long o = pq[u] * p.N + n;
        v.x = v.x * sc4.x + sh4.x;
        v.y = v.y * sc4.y + sh4.y;
        v.z = v.z * sc4.z + sh4.z;
        v.w = v.w * sc4.w + sh4.w;
        v.x += rq[u].x;
        v.y += rq[u].y;
        v.z += rq[u].z;
        v.w += rq[u].w;
        if (p.mask) {  // ReLU backward by the forward activation
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
        *reinterpret_cast<float4*>(p.out + o) = v;
        if constexpr (EPI == EPI_FWD_TAY) {
          if (p.tay_part) {  // slot by image (static selects: no dynamic register indexing)
            const int sl = m / tgs - g_first;
            float4 t;
            if (p.tay_mode) {
              t = make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w));
            } else {
              t = make_float4(-(v.x * mq[u].x), -(v.y * mq[u].y), -(v.z * mq[u].z), -(v.w * mq[u].w));
            }
#pragma unroll
            for (int i = 0; i < NTQ; ++i)
              if (sl == i) {
                tq[i].x += t.x;
                tq[i].y += t.y;
                tq[i].z += t.z;
                tq[i].w += t.w;
              }
          }
        }
        if (p.bnpart) {
          bool bwd_stats = false;
          if constexpr (GEN == 1 && EPI == EPI_FWD) bwd_stats = p.bnb_y != nullptr;
          if (bwd_stats) {  // that BN's backward statistics: (sum gm, sum gm * xhat)
            const float4 gm = p.bnb_bits ? bits_mask(p.bnb_bits, pq[u], p.N, n, v) : v;
            bs.x += gm.x;
            bs.y += gm.y;
            bs.z += gm.z;
            bs.w += gm.w;
            bq.x += gm.x * ((yq[u].x - bm4.x) * bi4.x);
            bq.y += gm.y * ((yq[u].y - bm4.y) * bi4.y);
            bq.z += gm.z * ((yq[u].z - bm4.z) * bi4.z);
            bq.w += gm.w * ((yq[u].w - bm4.w) * bi4.w);
          } else {
            bs.x += v.x;
            bs.y += v.y;
            bs.z += v.z;
            bs.w += v.w;
            bq.x += v.x * v.x;
            bq.y += v.y * v.y;
            bq.z += v.z * v.z;
            bq.w += v.w * v.w;
          }
        }
        if (p.apoz) {  // exact integer counts: atomics are order-free
          const int b = m / p.HWo;
          if (b != cur_b) {
            if (cur_b >= 0) {
              float* ap = cb_lds ? cb + (cur_b - b_first) * BN + c4 * 4 : p.apoz + (long long)cur_b * p.N + n;
              if (cnt.x > 0.f) atomicAdd(ap, cnt.x);
              if (cnt.y > 0.f) atomicAdd(ap + 1, cnt.y);
              if (cnt.z > 0.f) atomicAdd(ap + 2, cnt.z);
              if (cnt.w > 0.f) atomicAdd(ap + 3, cnt.w);
            }
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
    }
    if constexpr (EPI == EPI_FWD || EPI == EPI_FWD_TAY) {
      if (p.apoz && cur_b >= 0) {
        float* ap = cb_lds ? cb + (cur_b - b_first) * BN + c4 * 4 : p.apoz + (long long)cur_b * p.N + n;
        if (cnt.x > 0.f) atomicAdd(ap, cnt.x);
        if (cnt.y > 0.f) atomicAdd(ap + 1, cnt.y);
        if (cnt.z > 0.f) atomicAdd(ap + 2, cnt.z);
        if (cnt.w > 0.f) atomicAdd(ap + 3, cnt.w);
      }
      if (cb_lds) {  // one global atomic per (image, column) of this block
        __syncthreads();
        const int n_img = (min(m0 + BM, p.M) - 1) / p.HWo - b_first + 1;
        for (int t = tid; t < n_img * BN; t += T::NT) {
          const int col = n0 + t % BN;
          if (cb[t] > 0.f && col < p.N) atomicAdd(p.apoz + (long long)(b_first + t / BN) * p.N + col, cb[t]);
        }
      }
      if (p.bnpart) {  // fold the RSTEP row lanes of every column in a fixed order (deterministic)
        __syncthreads();  // the tile in ts is no longer read
        float* red = ts;  // [2][RSTEP][BN]
        *reinterpret_cast<float4*>(red + row0 * BN + c4 * 4) = bs;
        *reinterpret_cast<float4*>(red + (RSTEP + row0) * BN + c4 * 4) = bq;
        __syncthreads();
        for (int t = tid; t < 2 * BN; t += T::NT) {
          const int which = t / BN, col = t - which * BN;
          double acc = 0.0;
#pragma unroll 4
          for (int r = 0; r < RSTEP; ++r) acc += (double)red[(which * RSTEP + r) * BN + col];
          if (n0 + col < p.N) p.bnpart[((long long)(m0 / BM) * 2 + which) * p.N + n0 + col] = acc;
        }
      }
      if (EPI == EPI_FWD_TAY && p.tay_part) {  // fold the RSTEP row lanes per (image slot, column), fixed order
        static_assert(GEN_TAY_IMG * RSTEP * BN <= BM * LDT, "Taylor partial staging must fit in the tile");
        __syncthreads();  // the tile in ts (and any bnpart staging) is no longer read
        float* red = ts;  // [slot][RSTEP][BN]
#pragma unroll
        for (int i = 0; i < NTQ; ++i) *reinterpret_cast<float4*>(red + (i * RSTEP + row0) * BN + c4 * 4) = tq[i];
        __syncthreads();
        const int n_grp = min((min(m0 + BM, p.M) - 1) / tgs - g_first + 1, NTQ);
        const int B = p.M / p.HWo, R = gen_tay_slots(BM, tgs);
        for (int t = tid; t < n_grp * BN; t += T::NT) {
          const int sl = t / BN, col = t - sl * BN;
          float acc = 0.f;
#pragma unroll 4
          for (int r = 0; r < RSTEP; ++r) acc += red[(sl * RSTEP + r) * BN + col];
          const int grp = g_first + sl, cq = grp / B, b = grp - cq * B;  // cq: stride phase (GEN 3)
          const int slot = m0 / BM - (grp * tgs) / BM;
          if (n0 + col < p.N && slot < R)
            p.tay_part[((long long)(cq * R + slot) * B + b) * p.N + n0 + col] = acc;
        }
      }
    }
    return;
   }
  }

  // ---- epilogue --------------------------------------------------------------------------
#pragma unroll
  for (int j = 0; j < T::TN; ++j) {
    const int n = n0 + wn0 + j * 32 + li;
    const bool nok = n < p.N;
    float sc = 1.f, sh = 0.f;
    if constexpr (EPI == EPI_FWD || EPI == EPI_FWD_POOL || EPI == EPI_BWD) {
      if (nok) {
        sc = p.scale ? p.scale[n] : 1.f;
        if constexpr (EPI != EPI_BWD) sh = p.shift ? p.shift[n] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < T::TM; ++i) {
      const int mt = m0 + wm0 + i * 32;
      if constexpr (EPI == EPI_FWD_POOL) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int m = mt + 8 * g + 4 * lh;  // first row of this pooling window
          float best = 0.f;
          int arg = 0, cnt = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float v = acc[i][j][4 * g + q] * sc + sh;
            if (p.relu) v = nan_act(v, p.slope);
            cnt += v > 0.f ? 1 : 0;
            if (q == 0 || v > best || (v != v && best == best)) {
              best = v;
              arg = q;
            }
          }
          if (nok && m < p.M) {
            const long long o = (long long)(m >> 2) * p.N + n;
            p.out[o] = best;
            p.out_argmax[o] = (uint8_t)arg;
            if (p.apoz && cnt) atomicAdd(p.apoz + (long long)(m / p.HWo) * p.N + n, (float)cnt);
          }
        }
      } else if constexpr (EPI == EPI_BWD) {
        int cur_b = -1;
        float tsum = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = mt + 8 * g + 4 * lh + q;
            if (nok && m < p.M) {
              const long long o = (long long)m * p.N + n;
              const float gval = acc[i][j][4 * g + q];
              const float a = p.act[o];
              if (p.taylor) {
                const int b = m / p.HWo;
                if (b != cur_b) {
                  if (cur_b >= 0) atomicAdd(p.taylor + tay_index(p, cur_b, n), tsum);
                  cur_b = b;
                  tsum = 0.f;
                }
                tsum += tay_term(p.tay_mode, gval, a);
              }
              if (p.out) p.out[o] = act_grad(a, gval * sc, p.slope);
            }
          }
        }
        if (p.taylor && cur_b >= 0) atomicAdd(p.taylor + tay_index(p, cur_b, n), tsum);
      } else {
        int cur_b = -1;
        float cnt = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mt + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (nok && m < p.M) {
            float v = acc[i][j][r];
            if constexpr (EPI == EPI_FWD) {
              v = v * sc + sh;
              if (p.res) v += p.res[(long long)(p.res_rows > 0 ? m % p.res_rows : m) * p.N + n];
              if (p.relu) v = nan_act(v, p.slope);
              p.out[(long long)m * p.N + n] = v;
              if (p.apoz) {  // counts are exact integers: atomics are order-independent here
                const int b = m / p.HWo;
                if (b != cur_b) {
                  if (cur_b >= 0 && cnt > 0.f) atomicAdd(p.apoz + (long long)cur_b * p.N + n, cnt);
                  cur_b = b;
                  cnt = 0.f;
                }
                cnt += v > 0.f ? 1.f : 0.f;
              }
            } else {  // EPI_PARTIAL
              p.out[((long long)split * p.M + m) * p.N + n] = v;
            }
          }
        }
        if constexpr (EPI == EPI_FWD) {
          if (p.apoz && cur_b >= 0 && cnt > 0.f) atomicAdd(p.apoz + (long long)cur_b * p.N + n, cnt);
        }
      }
    }
  }
  };  // run_tile

  // ---- which tiles this block runs. Default: one tile per block (grid.y = split-K slab).
  // GEN 3 parity order puts the 4-, 2- and 1-tap phase classes in consecutive M ranges: the
  // contiguous XCD remap would hand the two heaviest XCDs all 4-tap tiles and the last two all
  // 1-tap tiles (max/mean work 4/2.25 -> the kernel ran ~1.7x long). Plain round-robin dispatch
  // spreads every class over all XCDs; the A operand here is the small low-resolution gradient.
  // Stream-K (GEN 1, one K pass): block b (XCD-contiguous) owns iterations [b I / P, (b+1) I / P)
  // of the tiles x k-slices space, I / P >= k-slices per tile (host-checked), so a range boundary
  // cuts at most one tile and every cut tile has exactly two contributors: the block before the
  // boundary (slices from 0: slot 0) and the one after (through the last slice: slot 1).
  // SK: a separate instantiation, so the segment loop (whose loop-invariant hoisting costs ~100
  // VGPRs) never touches the data-parallel kernels
  constexpr bool sk = GEN == 1 && SK;
  const int KT = p.K / BK;
  const long long I = p.sk_iters, P = p.sk_blocks > 0 ? p.sk_blocks : 1;
  const int b = sk || !(GEN == 3 && p.parity) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  long long it = sk ? (long long)b * I / P : 0;
  const long long hi = sk ? (long long)(b + 1) * I / P : 0;
  if constexpr (!sk) {
    run_tile(threadIdx.x, b, blockIdx.y, 0, 0, 0, nullptr);
  } else {
    for (int seg = 0;; ++seg) {
      int tile, kb = 0, ke = 0, mode = 0;
      float* slab = nullptr;
      if (p.sk_fixup) {
        if (seg || b == 0 || it % KT == 0) break;  // no tile cut at boundary b
        tile = (int)(it / KT);
        mode = SK_FIX;
        slab = p.sk_ws + (size_t)b * 2 * TILEF;
      } else {
        if (it >= hi) break;
        tile = (int)(it / KT);
        kb = (int)(it % KT);
        ke = (int)min((long long)KT, kb + (hi - it));
        if (kb != 0 || ke != KT) {
          mode = SK_PART;
          slab = kb == 0 ? p.sk_ws + (size_t)(b + 1) * 2 * TILEF  // cut at the range's end
                         : p.sk_ws + ((size_t)b * 2 + 1) * TILEF;  // cut at the range's start
        }
        it += ke - kb;
      }
      if (seg) __syncthreads();  // the previous segment's LDS reads are done
      int tid = threadIdx.x;
      asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"(tid));
      run_tile(tid, tile, 0, kb, ke, mode, slab);
    }
  }
}

// dgrad combines of images with at least this many pixels run one 1024-thread block per
// (image, 64 channels) (conv_epilogue_bwd_img); below it one thread per (image, channel) walks
// the pixels. At 64 pixels the thread-per-channel walk left B=100 batches with 50-100 blocks
// of 64-deep serial load chains (67-101 us per combine, 22% of the step).
constexpr int BWD_IMG_MIN_HW = 16;

// Split-K combine + epilogue (deterministic order over the slabs), one thread per output
// element (or per pooled element).
template <int EPI>
__global__ __launch_bounds__(256) void conv_epilogue(ConvArgs p, const float* __restrict__ slabs, int splits) {
  const long long MN = (long long)p.M * p.N;
  if constexpr (EPI == EPI_FWD_POOL) {
    const unsigned total = (unsigned)(MN / 4), N = (unsigned)p.N;
    for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
      const int n = (int)(t % N);
      const unsigned mp = t / N;
      const float sc = p.scale ? p.scale[n] : 1.f, sh = p.shift ? p.shift[n] : 0.f;
      float best = 0.f;
      int arg = 0, cnt = 0;
      for (int q = 0; q < 4; ++q) {
        const unsigned o = (mp * 4 + q) * N + n;
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += slabs[(size_t)s * MN + o];
        v = v * sc + sh;
        if (p.relu) v = nan_act(v, p.slope);
        cnt += v > 0.f ? 1 : 0;
        if (q == 0 || v > best || (v != v && best == best)) {
          best = v;
          arg = q;
        }
      }
      p.out[t] = best;
      p.out_argmax[t] = (uint8_t)arg;
      if (p.apoz && cnt) atomicAdd(p.apoz + (size_t)(mp * 4 / (unsigned)p.HWo) * N + n, (float)cnt);
    }
  } else if constexpr (EPI == EPI_FWD) {
    // 32-bit index math (host guarantees M*N < 2^31): 64-bit div/mod per element made this
    // combine kernel ~5x slower than its memory traffic
    const unsigned N = (unsigned)p.N;
    if ((N & 3u) == 0) {  // float4 columns
      const unsigned N4 = N >> 2, total = (unsigned)(MN >> 2);
      const float4* S = reinterpret_cast<const float4*>(slabs);
      for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const unsigned row = t / N4;
        const int n = (int)(t - row * N4) * 4;
        float4 v = S[t];
        for (int q = 1; q < splits; ++q) {
          const float4 w = S[(size_t)q * total + t];
          v.x += w.x;
          v.y += w.y;
          v.z += w.z;
          v.w += w.w;
        }
        const float4 sc = p.scale ? *reinterpret_cast<const float4*>(p.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
        const float4 sh = p.shift ? *reinterpret_cast<const float4*>(p.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        v.x = v.x * sc.x + sh.x;
        v.y = v.y * sc.y + sh.y;
        v.z = v.z * sc.z + sh.z;
        v.w = v.w * sc.w + sh.w;
        if (p.res) {
          const float4 r = res_quad(p, row, n);
          v.x += r.x;
          v.y += r.y;
          v.z += r.z;
          v.w += r.w;
        }
        if (p.mask) {
          const float4 a = *reinterpret_cast<const float4*>(p.mask + (size_t)t * 4);
          v.x = a.x > 0.f ? v.x : 0.f;
          v.y = a.y > 0.f ? v.y : 0.f;
          v.z = a.z > 0.f ? v.z : 0.f;
          v.w = a.w > 0.f ? v.w : 0.f;
        }
        if (p.relu) {
          v.x = nan_act(v.x, p.slope);
          v.y = nan_act(v.y, p.slope);
          v.z = nan_act(v.z, p.slope);
          v.w = nan_act(v.w, p.slope);
        }
        *reinterpret_cast<float4*>(p.out + (size_t)t * 4) = v;
        if (p.apoz) {
          float* ap = p.apoz + (size_t)(row / (unsigned)p.HWo) * N + n;
          if (v.x > 0.f) atomicAdd(ap, 1.f);
          if (v.y > 0.f) atomicAdd(ap + 1, 1.f);
          if (v.z > 0.f) atomicAdd(ap + 2, 1.f);
          if (v.w > 0.f) atomicAdd(ap + 3, 1.f);
        }
      }
    } else {  // ragged columns (e.g. a 10-way classifier): scalar, no res / mask / apoz users
      const unsigned total = (unsigned)MN;
      for (unsigned o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
        const unsigned n = o % N;
        float v = 0.f;
        for (int q = 0; q < splits; ++q) v += slabs[(size_t)q * total + o];
        v = v * (p.scale ? p.scale[n] : 1.f) + (p.shift ? p.shift[n] : 0.f);
        if (p.res) v += p.res[p.res_rows > 0 ? (long long)(o / N % (unsigned)p.res_rows) * N + n : (long long)o];
        if (p.mask && !(p.mask[o] > 0.f)) v = 0.f;
        if (p.relu) v = nan_act(v, p.slope);
        p.out[o] = v;
        if (p.apoz && v > 0.f) atomicAdd(p.apoz + (size_t)(o / N / (unsigned)p.HWo) * N + n, 1.f);
      }
    }
  } else if (p.HWo >= BWD_IMG_MIN_HW) {
    // EPI_BWD, images of >= 16 pixels: handled by conv_epilogue_bwd_img (block per image x 64 channels)
  } else {  // EPI_BWD, small images: one thread per (image, channel) walks the image's
            // pixels, so the Taylor sum is a plain deterministic += (no atomics)
    const long long BN = (long long)(p.M / p.HWo) * p.N;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < BN;
         t += (long long)gridDim.x * blockDim.x) {
      const int n = (int)(t % p.N);
      const long long b = t / p.N;
      const float sc = p.scale ? p.scale[n] : 1.f;
      float tsum = 0.f;
      for (int px = 0; px < p.HWo; ++px) {
        const long long o = (b * p.HWo + px) * p.N + n;
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += slabs[s * MN + o];
        const float a = p.act[o];
        tsum += tay_term(p.tay_mode, v, a);
        if (p.out) p.out[o] = act_grad(a, v * sc, p.slope);
      }
      if (p.taylor) p.taylor[tay_index(p, b, n)] += tsum;
    }
  }
}

// Split-combine + dgrad epilogue for large images without atomics: a 1024-thread block owns
// (image b, 64 channels); 16 pixel groups stride over the image, and the Taylor partials are
// combined in LDS in a fixed order (bit-reproducible).
__global__ __launch_bounds__(1024) void conv_epilogue_bwd_img(ConvArgs p, const float* __restrict__ slabs,
                                                               int splits) {
  __shared__ float red[16][64];
  const long long MN = (long long)p.M * p.N;
  const int b = blockIdx.y;
  const int c = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  float tsum = 0.f;
  if (n < p.N) {
    const float sc = p.scale ? p.scale[n] : 1.f;
    for (int px = pg; px < p.HWo; px += 16) {
      const long long o = ((long long)b * p.HWo + px) * p.N + n;
      float v = 0.f;
      for (int s = 0; s < splits; ++s) v += slabs[s * MN + o];
      const float a = p.act[o];
      tsum += tay_term(p.tay_mode, v, a);
      if (p.out) p.out[o] = act_grad(a, v * sc, p.slope);
    }
  }
  red[pg][c] = tsum;
  __syncthreads();
  if (pg == 0 && n < p.N && p.taylor) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    p.taylor[tay_index(p, b, n)] += t;
  }
}

// First layer: direct conv on the VALU (Cin is tiny), NCHW fp32 input -> NHWC output with the
// BN-eval affine and ReLU fused. A thread owns one output pixel x 4 channels, so COUT/4
// consecutive lanes write one pixel's contiguous NHWC row (coalesced 16-B stores); the
// Cin*9 input taps of a pixel are shared through L1 by those lanes.
template <int COUT>
__global__ __launch_bounds__(256) void conv_first_direct(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, float* __restrict__ out,
                                                         int B, int Cin, int H, int W, int relu) {
  // a thread owns one pixel x CPT channels: each loaded input tap feeds CPT FMAs (the
  // 4-channel version was instruction-issue bound: one global + one LDS load per 4 FMAs)
  constexpr int CPT = COUT >= 16 ? 16 : COUT;
  constexpr int G = COUT / CPT;
  extern __shared__ float4 wsh4[];  // [Cin*9][COUT/4] float4
  const int KK = Cin * 9;
  float* wsh = reinterpret_cast<float*>(wsh4);
  for (int t = threadIdx.x; t < KK * COUT; t += blockDim.x) {
    const int n = t % COUT, k = t / COUT;  // w is [COUT][Cin][3][3]
    wsh[t] = w[n * KK + k];
  }
  __syncthreads();
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long pix = gt / G;
  const int grp = (int)(gt % G);
  if (pix >= (long long)B * H * W) return;
  const int b = (int)(pix / (H * W));
  const int r = (int)(pix % (H * W));
  const int oh = r / W, ow = r % W;
  float acc[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) acc[j] = 0.f;
  for (int c = 0; c < Cin; ++c) {
    const float* xc = x + ((long long)b * Cin + c) * H * W;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = oh + kh - 1, iw = ow + kw - 1;
        const float v = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xc[ih * W + iw] : 0.f;
        const float4* wk = wsh4 + ((c * 3 + kh) * 3 + kw) * (COUT / 4) + grp * (CPT / 4);
#pragma unroll
        for (int q = 0; q < CPT / 4; ++q) {
          const float4 ww = wk[q];
          acc[4 * q] = fmaf(v, ww.x, acc[4 * q]);
          acc[4 * q + 1] = fmaf(v, ww.y, acc[4 * q + 1]);
          acc[4 * q + 2] = fmaf(v, ww.z, acc[4 * q + 2]);
          acc[4 * q + 3] = fmaf(v, ww.w, acc[4 * q + 3]);
        }
      }
    }
  }
  const int n0 = grp * CPT;
#pragma unroll
  for (int q = 0; q < CPT / 4; ++q) {
    const int n = n0 + 4 * q;
    float4 v;
    v.x = acc[4 * q] * scale[n] + shift[n];
    v.y = acc[4 * q + 1] * scale[n + 1] + shift[n + 1];
    v.z = acc[4 * q + 2] * scale[n + 2] + shift[n + 2];
    v.w = acc[4 * q + 3] * scale[n + 3] + shift[n + 3];
    if (relu) {
      v.x = nan_relu(v.x);
      v.y = nan_relu(v.y);
      v.z = nan_relu(v.z);
      v.w = nan_relu(v.w);
    }
    *reinterpret_cast<float4*>(out + pix * COUT + n) = v;
  }
}

// First conv layer, wave-uniform channels: a wave owns 64 consecutive output pixels (one per
// lane) x ALL COUT channels, so every weight is the same for the 64 lanes and comes from the
// scalar cache (s_load, an SGPR operand of the FMA) instead of LDS; each input tap is loaded once
// per lane and feeds COUT FMAs. The wave's 64 x COUT output tile is one contiguous NHWC region:
// it is transposed through LDS (rows padded by 4 floats) and written with 1-KB coalesced
// float4 stores. The conv_first_direct version above was LDS-bandwidth bound (every lane read
// its weights from LDS, 4 FMAs per 16-B read).
template <int COUT>
__global__ __launch_bounds__(256) void conv_first_wave(const float* __restrict__ x, const float* __restrict__ wt,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ out,
                                                       int B, int Cin, int H, int W, int relu) {
  constexpr int HC = COUT >= 32 ? 32 : COUT;  // channels per transpose pass
  constexpr int LD = HC + 4;                  // padded LDS row (floats)
  __shared__ __attribute__((aligned(16))) float tile[4][64 * LD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long npix = (long long)B * H * W;
  const long long pix0 = ((long long)blockIdx.x * 4 + wave) * 64;
  if (pix0 >= npix) return;  // whole wave past the end (no block-wide barrier below)
  const long long pix = pix0 + lane;
  const bool valid = pix < npix;
  const int HW = H * W;
  const int b = valid ? (int)(pix / HW) : 0;
  const int r = valid ? (int)(pix - (long long)b * HW) : 0;
  const int oh = r / W, ow = r - (r / W) * W;
  float acc[COUT];
#pragma unroll
  for (int j = 0; j < COUT; ++j) acc[j] = 0.f;
  for (int c = 0; c < Cin; ++c) {
    const float* xc = x + ((long long)b * Cin + c) * HW;
    float v[9];  // the 9 taps' loads in flight together
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh + t / 3 - 1, iw = ow + t % 3 - 1;
      v[t] = (valid && ih >= 0 && ih < H && iw >= 0 && iw < W) ? xc[ih * W + iw] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // compiler fence: one tap's COUT wave-uniform weights (scalar loads) live in SGPRs at a
      // time — hoisting all taps' loads spills SGPRs
      asm volatile("" ::: "memory");
      const float* wr = wt + (c * 9 + t) * COUT;
#pragma unroll
      for (int j = 0; j < COUT; ++j) acc[j] = fmaf(v[t], wr[j], acc[j]);
    }
  }
  float* tw = tile[wave];
  constexpr int Q = HC / 4;  // float4 per pixel row of one pass
#pragma unroll
  for (int h = 0; h < COUT / HC; ++h) {
#pragma unroll
    for (int j = 0; j < HC; j += 4) {
      const int n = h * HC + j;
      float4 y;
      y.x = acc[n] * scale[n] + shift[n];
      y.y = acc[n + 1] * scale[n + 1] + shift[n + 1];
      y.z = acc[n + 2] * scale[n + 2] + shift[n + 2];
      y.w = acc[n + 3] * scale[n + 3] + shift[n + 3];
      if (relu) {
        y.x = nan_relu(y.x);
        y.y = nan_relu(y.y);
        y.z = nan_relu(y.z);
        y.w = nan_relu(y.w);
      }
      *reinterpret_cast<float4*>(tw + lane * LD + j) = y;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      const int idx = i * 64 + lane;  // float4 index in the wave's [64][HC] tile, row-major
      const int px = idx / Q, c4 = idx - px * Q;
      const float4 o = *reinterpret_cast<const float4*>(tw + px * LD + 4 * c4);
      if (pix0 + px < npix) *reinterpret_cast<float4*>(out + (pix0 + px) * COUT + h * HC + 4 * c4) = o;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // reads done before the next pass overwrites the tile
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace tp

// ------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------
namespace {

using tp::ConvArgs;

template <int BM, int BN, int WM, int WN, int KS, bool PM, bool UP, int EPI, bool BF = false>
hipError_t launch_cfg(const ConvArgs& a, int splits, hipStream_t st) {
  const int m_tiles = (a.M + BM - 1) / BM, n_tiles = (a.N + BN - 1) / BN;
  dim3 grid(m_tiles * n_tiles, splits);
  tp::conv_igemm<BM, BN, WM, WN, KS, PM, UP, EPI, 0, BF><<<grid, tp::Tile<BM, BN, WM, WN>::NT, 0, st>>>(a);
  return hipGetLastError();
}

// cfg: 0 = 128x128 (waves 2x2 of 64x64), 1 = 256x64 (4x1 of 64x64), 2 = 64x64 (2x2 of 32x32),
//      4 = 128x128 (8 waves 2x4 of 64x32), 5 = 256x64 (8 waves 4x2 of 64x32), 6 = 128x64 (8 waves 4x2 of 32x32),
//      3 = 128x64 (2x2 of 64x32)
// cfg | CFG_BF16 (3x3 only): the bf16-operand variants of cfgs 0, 2, 3
template <int KS, bool PM, bool UP, int EPI>
hipError_t launch_any(int cfg, const ConvArgs& a, int splits, hipStream_t st) {
  if (cfg & tp::CFG_BF16) {
    if constexpr (KS == 3) {
      switch (cfg & ~tp::CFG_BF16) {
        case 0: return launch_cfg<128, 128, 64, 64, KS, PM, UP, EPI, true>(a, splits, st);
        case 2: return launch_cfg<64, 64, 32, 32, KS, PM, UP, EPI, true>(a, splits, st);
        case 3: return launch_cfg<128, 64, 64, 32, KS, PM, UP, EPI, true>(a, splits, st);
      }
    }
    return hipErrorInvalidValue;
  }
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 64, 64, KS, PM, UP, EPI>(a, splits, st);
    case 1: return launch_cfg<256, 64, 64, 64, KS, PM, UP, EPI>(a, splits, st);
    case 4: return launch_cfg<128, 128, 64, 32, KS, PM, UP, EPI>(a, splits, st);  // 8 waves
    case 5: return launch_cfg<256, 64, 64, 32, KS, PM, UP, EPI>(a, splits, st);   // 8 waves
    case 6: return launch_cfg<128, 64, 32, 32, KS, PM, UP, EPI>(a, splits, st);   // 8 waves
    case 2: return launch_cfg<64, 64, 32, 32, KS, PM, UP, EPI>(a, splits, st);
    case 3: return launch_cfg<128, 64, 64, 32, KS, PM, UP, EPI>(a, splits, st);
  }
  return hipErrorInvalidValue;
}

template <int KS>
hipError_t dispatch_epi(int cfg, int epi, bool pooled_m, bool unpool, const ConvArgs& a, int splits,
                        hipStream_t st) {
  using namespace tp;
  if (epi == EPI_FWD_POOL) {
    if (!pooled_m || unpool) return hipErrorInvalidValue;
    return launch_any<KS, true, false, EPI_FWD_POOL>(cfg, a, splits, st);
  }
  if (epi == EPI_PARTIAL) {
    if (pooled_m) return unpool ? launch_any<KS, true, true, EPI_PARTIAL>(cfg, a, splits, st)
                                : launch_any<KS, true, false, EPI_PARTIAL>(cfg, a, splits, st);
    return unpool ? launch_any<KS, false, true, EPI_PARTIAL>(cfg, a, splits, st)
                  : launch_any<KS, false, false, EPI_PARTIAL>(cfg, a, splits, st);
  }
  if (pooled_m) return hipErrorInvalidValue;
  if (epi == EPI_FWD) return unpool ? launch_any<KS, false, true, EPI_FWD>(cfg, a, splits, st)
                                    : launch_any<KS, false, false, EPI_FWD>(cfg, a, splits, st);
  if (epi == EPI_BWD) return unpool ? launch_any<KS, false, true, EPI_BWD>(cfg, a, splits, st)
                                    : launch_any<KS, false, false, EPI_BWD>(cfg, a, splits, st);
  return hipErrorInvalidValue;
}

}  // namespace

// Main entry. ``ws`` is a workspace of splits*M*N floats when splits > 1.
extern "C" hipError_t tp_conv_igemm(const float* x, const uint8_t* x_argmax, const float* w, int B, int H, int W,
                                    int Cin, int Cout, int ks, int pooled_m, int unpool, int epi, int cfg, int splits,
                                    const float* scale, const float* shift, int relu, float* out,
                                    uint8_t* out_argmax, const float* act, float* taylor, int HWo, int tay_group,
                                    float* ws, int tay_mode, float* apoz, float slope, hipStream_t st) {
  using namespace tp;
  if (Cin % 32 != 0 || !(slope >= 0.f)) return hipErrorInvalidValue;
  ConvArgs a{};
  a.slope = slope;
  a.x = x;
  a.x_argmax = x_argmax;
  a.w = w;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.N = Cout;
  a.K = ks * ks * Cin;
  a.M = B * H * W;
  a.x_elems = unpool ? (long long)B * (H / 2) * (W / 2) * Cin : (long long)B * H * W * Cin;
  // buffer descriptors address 32-bit byte offsets
  if (a.x_elems * 4 >= (1ll << 31) || (long long)Cout * a.K * 4 >= (1ll << 31) ||
      (long long)a.M * a.N >= (1ll << 31))
    return hipErrorInvalidValue;
  const int kt = a.K / 32;
  splits = std::max(1, std::min(splits, kt));
  a.k_tiles_per_split = (kt + splits - 1) / splits;
  splits = (kt + a.k_tiles_per_split - 1) / a.k_tiles_per_split;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.out = out;
  a.out_argmax = out_argmax;
  a.act = act;
  a.taylor = taylor;
  a.HWo = HWo;
  a.tay_group = tay_group;
  a.tay_mode = tay_mode;
  a.apoz = apoz;
  a.Ho = H;
  a.Wo = W;
  a.stride = 1;
  a.pad = (ks - 1) / 2;
  if (splits == 1 || epi == EPI_PARTIAL) {
    ConvArgs b = a;
    if (epi == EPI_PARTIAL) b.out = ws ? ws : out;
    return ks == 3 ? dispatch_epi<3>(cfg, epi, pooled_m, unpool, b, splits, st)
                   : dispatch_epi<1>(cfg, epi, pooled_m, unpool, b, splits, st);
  }
  // split-K: partial slabs then a deterministic combine + epilogue
  ConvArgs b = a;
  b.out = ws;
  hipError_t e = ks == 3 ? dispatch_epi<3>(cfg, EPI_PARTIAL, pooled_m, unpool, b, splits, st)
                         : dispatch_epi<1>(cfg, EPI_PARTIAL, pooled_m, unpool, b, splits, st);
  if (e != hipSuccess) return e;
  const long long MN = (long long)a.M * a.N;
  const long long work = epi == EPI_FWD_POOL ? MN / 4 : (epi == EPI_BWD && a.HWo < BWD_IMG_MIN_HW ? MN / a.HWo : MN);
  unsigned grid = (unsigned)std::min<long long>(ceil_div(work, 256), 4096);
  if (epi == EPI_FWD_POOL) conv_epilogue<EPI_FWD_POOL><<<grid, 256, 0, st>>>(a, ws, splits);
  else if (epi == EPI_FWD) conv_epilogue<EPI_FWD><<<grid, 256, 0, st>>>(a, ws, splits);
  else if (epi == EPI_BWD && a.HWo >= BWD_IMG_MIN_HW)
    conv_epilogue_bwd_img<<<dim3((unsigned)ceil_div(a.N, 64), (unsigned)(a.M / a.HWo)), 1024, 0, st>>>(a, ws, splits);
  else if (epi == EPI_BWD) conv_epilogue<EPI_BWD><<<grid, 256, 0, st>>>(a, ws, splits);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Split combine + epilogue for slabs produced elsewhere (Winograd partials): slab layout
// [splits][M][K], pooled M order for epi == fwd+pool.
extern "C" hipError_t tp_conv_epilogue_slabs(const float* ws, int splits, int B, int H, int W, int K, int epi,
                                              const float* scale, const float* shift, int relu, float* out,
                                              uint8_t* out_argmax, const float* act, float* taylor,
                                              float* apoz, int tay_mode, hipStream_t st) {
  using namespace tp;
  ConvArgs a{};
  a.B = B;
  a.H = H;
  a.W = W;
  a.N = K;
  a.M = B * H * W;
  if ((long long)a.M * K >= (1ll << 31)) return hipErrorInvalidValue;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.out = out;
  a.out_argmax = out_argmax;
  a.act = act;
  a.taylor = taylor;
  a.tay_mode = tay_mode;
  a.apoz = apoz;
  a.HWo = H * W;
  const long long MN = (long long)a.M * a.N;
  const long long work = epi == EPI_FWD_POOL ? MN / 4 : (epi == EPI_BWD && a.HWo < BWD_IMG_MIN_HW ? MN / a.HWo : MN);
  unsigned grid = (unsigned)std::min<long long>(ceil_div(work, 256), 4096);
  if (epi == EPI_FWD_POOL) conv_epilogue<EPI_FWD_POOL><<<grid, 256, 0, st>>>(a, ws, splits);
  else if (epi == EPI_FWD) conv_epilogue<EPI_FWD><<<grid, 256, 0, st>>>(a, ws, splits);
  else if (epi == EPI_BWD && a.HWo >= BWD_IMG_MIN_HW)
    conv_epilogue_bwd_img<<<dim3((unsigned)ceil_div(a.N, 64), (unsigned)(a.M / a.HWo)), 1024, 0, st>>>(a, ws, splits);
  else if (epi == EPI_BWD) conv_epilogue<EPI_BWD><<<grid, 256, 0, st>>>(a, ws, splits);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// ``wt``: the weight as [Cin*9][Cout] (tap-major): the wave-uniform kernel for Cout 16/32/64.
extern "C" hipError_t tp_conv_first_wave(const float* x, const float* wt, const float* scale, const float* shift,
                                         float* out, int B, int Cin, int H, int W, int Cout, int relu,
                                         hipStream_t st) {
  const long long pix = (long long)B * H * W;
  if (pix <= 0 || Cin < 1 || Cin > 16) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)tp::ceil_div(pix, 256);
  if (Cout == 64) tp::conv_first_wave<64><<<grid, 256, 0, st>>>(x, wt, scale, shift, out, B, Cin, H, W, relu);
  else if (Cout == 32) tp::conv_first_wave<32><<<grid, 256, 0, st>>>(x, wt, scale, shift, out, B, Cin, H, W, relu);
  else if (Cout == 16) tp::conv_first_wave<16><<<grid, 256, 0, st>>>(x, wt, scale, shift, out, B, Cin, H, W, relu);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t tp_conv_first_direct(const float* x, const float* w, const float* scale, const float* shift,
                                           float* out, int B, int Cin, int H, int W, int Cout, int relu,
                                           hipStream_t st) {
  const long long pix = (long long)B * H * W;
  const unsigned grid = tp::ceil_div(pix * (Cout >= 16 ? Cout / 16 : 1), 256);
  const size_t lds = (size_t)Cin * 9 * Cout * sizeof(float);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  if (Cout == 64) tp::conv_first_direct<64><<<grid, 256, lds, st>>>(x, w, scale, shift, out, B, Cin, H, W, relu);
  else if (Cout == 32) tp::conv_first_direct<32><<<grid, 256, lds, st>>>(x, w, scale, shift, out, B, Cin, H, W, relu);
  else if (Cout == 16) tp::conv_first_direct<16><<<grid, 256, lds, st>>>(x, w, scale, shift, out, B, Cin, H, W, relu);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// NCHW (B, C, H, W) -> NHWC (B, H, W, Cp) with channels C..Cp-1 zero (Cp % 4 == 0): the
// first layer's input in the layout the Winograd / implicit-GEMM kernels read (float4 stores).
namespace tp {
__global__ __launch_bounds__(256) void nchw_to_nhwc_pad(const float* __restrict__ x, float* __restrict__ y, int B,
                                                        int C, int HW, int Cp) {
  const long long total = (long long)B * HW * (Cp / 4);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % (Cp / 4));
    const long long pix = t / (Cp / 4);
    const long long b = pix / HW, s = pix - b * HW;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c4 * 4 + i;
      v[i] = c < C ? x[(b * C + c) * HW + s] : 0.f;
    }
    *reinterpret_cast<float4*>(y + pix * Cp + c4 * 4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}
}  // namespace tp

extern "C" hipError_t tp_nchw_to_nhwc_pad(const float* x, float* y, int B, int C, int H, int W, int Cp,
                                          hipStream_t st) {
  if (Cp % 4 != 0 || Cp < C) return hipErrorInvalidValue;
  const long long total = (long long)B * H * W * (Cp / 4);
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::nchw_to_nhwc_pad<<<grid, 256, 0, st>>>(x, y, B, C, H * W, Cp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// General strided / padded conv (ResNet): KS in {1, 3} with Cin % 32 == 0, or KS = 7 on a
// 4-channel padded input (stem). Forward epilogue: BN affine, optional residual add, optional
// ReLU, optional APoZ counts of the output (exact integer counts per (image, channel)).
// ---------------------------------------------------------------------------------------------
namespace {
// Stream-K geometry of a GEN kernel instantiation: P = co-resident blocks (CUs x occupancy), the
// number of equal iteration ranges; applicable when the tile count is at least P and not a
// multiple of it (otherwise data-parallel tiles are already balanced).
template <int BM, int BN, int WM, int WN, int KS, int GEN, int EPI>
int sk_blocks() {
  static const int P = [] {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &nb, reinterpret_cast<const void*>(&tp::conv_igemm<BM, BN, WM, WN, KS, false, false, EPI, GEN, false, true>),
            tp::Tile<BM, BN, WM, WN>::NT, 0) != hipSuccess)
      return 0;
    return cus * nb;
  }();
  return P;
}

template <int BM, int BN, int WM, int WN, int KS, int GEN, int EPI>
long long sk_ws_floats(int M, int N) {
  const long long tiles = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if constexpr (GEN != 1) return 0;
  const int P = sk_blocks<BM, BN, WM, WN, KS, GEN, EPI>();
  if (P <= 0 || tiles < P || tiles % P == 0) return 0;
  return (long long)P * 2 * BM * BN;
}

template <int BM, int BN, int WM, int WN, int KS, int GEN, int EPI>
hipError_t launch_gen(const tp::ConvArgs& a, int splits, hipStream_t st) {
  const int m_tiles = (a.M + BM - 1) / BM, n_tiles = (a.N + BN - 1) / BN;
  constexpr int NT = tp::Tile<BM, BN, WM, WN>::NT;
  if constexpr (GEN == 1 && (EPI == tp::EPI_FWD || EPI == tp::EPI_FWD_TAY)) {
  if (a.sk_blocks < 0) {  // stream-K requested (a.sk_ws sized by sk_ws_floats): balanced ranges, then the fixups
    if (splits == 1 && a.sk_ws && sk_ws_floats<BM, BN, WM, WN, KS, GEN, EPI>(a.M, a.N) > 0) {
      tp::ConvArgs b = a;
      b.sk_blocks = sk_blocks<BM, BN, WM, WN, KS, GEN, EPI>();
      b.sk_iters = (long long)m_tiles * n_tiles * (a.K / 32);
      b.sk_fixup = 0;
      tp::conv_igemm<BM, BN, WM, WN, KS, false, false, EPI, GEN, false, true><<<b.sk_blocks, NT, 0, st>>>(b);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      b.sk_fixup = 1;
      tp::conv_igemm<BM, BN, WM, WN, KS, false, false, EPI, GEN, false, true><<<b.sk_blocks, NT, 0, st>>>(b);
      return hipGetLastError();
    }
  }
  }
  dim3 grid(m_tiles * n_tiles, splits);
  if constexpr (GEN == 1 && (EPI == tp::EPI_FWD || EPI == tp::EPI_FWD_TAY) && KS == 1) {
    if (a.sb) {
      if (splits != 1) return hipErrorInvalidValue;
      tp::conv_igemm<BM, BN, WM, WN, KS, false, false, EPI, GEN, false, false, true><<<grid, NT, 0, st>>>(a);
      return hipGetLastError();
    }
  }
  tp::conv_igemm<BM, BN, WM, WN, KS, false, false, EPI, GEN><<<grid, NT, 0, st>>>(a);
  return hipGetLastError();
}

template <int KS, int EPI>
long long sk_ws_cfg(int cfg, int M, int N) {
  switch (cfg) {
    case 0: return sk_ws_floats<128, 128, 64, 64, KS, 1, EPI>(M, N);
    case 1: return sk_ws_floats<256, 64, 64, 64, KS, 1, EPI>(M, N);
    case 2: return sk_ws_floats<64, 64, 32, 32, KS, 1, EPI>(M, N);
    case 3: return sk_ws_floats<128, 64, 64, 32, KS, 1, EPI>(M, N);
    case 4: return sk_ws_floats<128, 128, 64, 32, KS, 1, EPI>(M, N);
    case 5: return sk_ws_floats<256, 64, 64, 32, KS, 1, EPI>(M, N);
    case 6: return sk_ws_floats<128, 64, 32, 32, KS, 1, EPI>(M, N);
  }
  return 0;
}

template <int KS, int GEN, int EPI>
hipError_t gen_cfg(int cfg, const tp::ConvArgs& a, int splits, hipStream_t st) {
  switch (cfg) {
    case 0: return launch_gen<128, 128, 64, 64, KS, GEN, EPI>(a, splits, st);
    case 1: return launch_gen<256, 64, 64, 64, KS, GEN, EPI>(a, splits, st);
    case 2: return launch_gen<64, 64, 32, 32, KS, GEN, EPI>(a, splits, st);
    case 3: return launch_gen<128, 64, 64, 32, KS, GEN, EPI>(a, splits, st);
    case 4: return launch_gen<128, 128, 64, 32, KS, GEN, EPI>(a, splits, st);
    case 5: return launch_gen<256, 64, 64, 32, KS, GEN, EPI>(a, splits, st);
    case 6: return launch_gen<128, 64, 32, 32, KS, GEN, EPI>(a, splits, st);
  }
  return hipErrorInvalidValue;
}

template <int EPI>
hipError_t gen_dispatch(int ks, int gen, int cfg, const tp::ConvArgs& a, int splits, hipStream_t st) {
  if constexpr (EPI == tp::EPI_FWD) {
    if (gen == 3 && ks == 1) return gen_cfg<1, 3, EPI>(cfg, a, 1, st);
    if (gen == 3 && ks == 3) return gen_cfg<3, 3, EPI>(cfg, a, 1, st);
  }
  if (gen == 2 && ks == 7) return gen_cfg<7, 2, EPI>(cfg, a, splits, st);
  if (gen == 2 && ks == 5) return gen_cfg<5, 2, EPI>(cfg, a, splits, st);
  if (gen == 2 && ks == 3) return gen_cfg<3, 2, EPI>(cfg, a, splits, st);
  if (gen == 1 && ks == 1) return gen_cfg<1, 1, EPI>(cfg, a, splits, st);
  if (gen == 1 && ks == 3) return gen_cfg<3, 1, EPI>(cfg, a, splits, st);
  if (gen == 1 && ks == 5) return gen_cfg<5, 1, EPI>(cfg, a, splits, st);
  return hipErrorInvalidValue;
}
}  // namespace

// Workspace floats a stream-K GEN 1 launch of tile config ``cfg`` (without the CFG_SK flag) needs at
// this GEMM shape (0: stream-K does not apply: transposed / strided-gather, 5x5, or the tiles are
// fewer than the co-resident blocks or already a multiple of them). ``tay``: the data-gradient
// Taylor-partials instantiation (EPI_FWD_TAY).
extern "C" long long tp_conv_sk_ws_floats(int cfg, int ks, int transposed, int tay, int M, int N) {
  if (transposed || cfg < 0 || cfg > 6) return 0;
  if (ks == 1) return tay ? sk_ws_cfg<1, tp::EPI_FWD_TAY>(cfg, M, N) : sk_ws_cfg<1, tp::EPI_FWD>(cfg, M, N);
  if (ks == 3 && !tay) return sk_ws_cfg<3, tp::EPI_FWD>(cfg, M, N);
  return 0;
}

// GEMM K of a GEN conv's weight operand: 4-channel packed taps, else every tap's channels padded
// to the 32-wide K slice (Cin % 4 == 0: pruned widths read zeros past Cin)
extern "C" int tp_conv_gen_k(int ks, int Cin) {
  return Cin == 4 ? (ks * ks * 4 + 31) / 32 * 32 : ks * ks * ((Cin + 31) / 32 * 32);
}

extern "C" hipError_t tp_conv_gen2(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   hipStream_t st);

extern "C" hipError_t tp_conv_gen(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                  int stride, int pad, int cfg, int splits, const float* scale, const float* shift,
                                  int relu, const float* res, float* apoz, float* out, float* ws, hipStream_t st) {
  return tp_conv_gen2(x, w, B, H, W, Cin, Cout, ks, stride, pad, 0, 0, 0, cfg, splits, scale, shift, relu, res, 1,
                      nullptr, apoz, out, ws, st);
}

// Shapley prefix-delta GEMM (see prefix_tri_operands in shapley.hip):
//   out[r, n] = act(Y0[r % B0, n] - (T @ Wsub^T)[r, n]),  T (M, Kc), Wsub (N, Kc), Y0 (B0, N)
// on the GEN 1x1 kernel: scale = -1 (a device vector), residual Y0 broadcast by res_rows = B0,
// ReLU / LeakyReLU (slope) in the epilogue.
extern "C" hipError_t tp_prefix_delta_gemm(const float* T, const float* Wsub, const float* neg_one, const float* Y0,
                                           int M, int Kc, int N, int B0, int relu, float slope, int cfg,
                                           float* out, hipStream_t st) {
  using namespace tp;
  if (Kc % 32 != 0 || N % 4 != 0 || B0 <= 0 || M % B0 != 0 || !(slope >= 0.f)) return hipErrorInvalidValue;
  ConvArgs a{};
  a.x = T;
  a.w = Wsub;
  a.B = M;
  a.H = a.W = a.Ho = a.Wo = 1;
  a.HWo = 1;
  a.Cin = Kc;
  a.N = N;
  a.K = Kc;
  a.M = M;
  a.stride = 1;
  a.pad = 0;
  a.x_elems = (long long)M * Kc;
  if (a.x_elems * 4 >= (1ll << 31) || (long long)M * N * 4 >= (1ll << 31)) return hipErrorInvalidValue;
  a.k_tiles_per_split = Kc / 32;
  a.scale = neg_one;
  a.relu = relu;
  a.slope = slope;
  a.res = Y0;
  a.res_stride = 1;
  a.res_rows = B0;
  a.out = out;
  a.epi_lds = 1;
  return gen_dispatch<EPI_FWD>(1, 1, cfg, a, 1, st);
}

// Full entry: ``transposed`` = data gradient of a strided conv (GEN 3) producing Ho_t x Wo_t
// (the forward conv's input size); ``mask`` = ReLU-backward activation; ``res_stride``: see
// ConvArgs. Forward convs pass transposed = 0 (Ho_t/Wo_t ignored), mask = null, res_stride = 1.
extern "C" hipError_t tp_conv_gen3(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, hipStream_t st);

extern "C" hipError_t tp_conv_gen2(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   hipStream_t st) {
  return tp_conv_gen3(x, w, B, H, W, Cin, Cout, ks, stride, pad, transposed, Ho_t, Wo_t, cfg, splits, scale, shift,
                      relu, res, res_stride, mask, apoz, out, ws, nullptr, st);
}

// M tile height of an implicit-GEMM tile config (the row count of a bnpart slab is ceil(M / it))
extern "C" int tp_conv_tile_m(int cfg) {
  switch (cfg & ~(tp::CFG_SK | tp::CFG_SB)) {
    case 1: case 5: return 256;
    case 2: return 64;
    default: return 128;
  }
}

extern "C" hipError_t tp_conv_gen4(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, float* tay_part, int tay_mode, hipStream_t st);

// Taylor partial slots of tp_conv_gen4's ``tay_part`` for tile config cfg at Ho*Wo output pixels
// per image; 0 = the config cannot produce them (a tile would span more than GEN_TAY_IMG images).
extern "C" int tp_conv_gen_tay_slots(int cfg, int HWo) {
  cfg &= ~(tp::CFG_SK | tp::CFG_SB);
  if (cfg == 4) return 0;  // its 8-wave 128x128 EPI_FWD_TAY build spills 29 VGPRs (the others do not)
  const int bm = tp_conv_tile_m(cfg);
  if (HWo <= 0 || (bm - 1) / HWo + 1 > tp::GEN_TAY_IMG) return 0;
  return tp::gen_tay_slots(bm, HWo);
}

extern "C" hipError_t tp_conv_gen3(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, hipStream_t st) {
  return tp_conv_gen4(x, w, B, H, W, Cin, Cout, ks, stride, pad, transposed, Ho_t, Wo_t, cfg, splits, scale, shift,
                      relu, res, res_stride, mask, apoz, out, ws, bnpart, nullptr, 0, st);
}

// ``bnpart`` (nullable): [ceil(M / tile_m(cfg))][2][Cout] doubles receiving the per-tile column
// sums / sums of squares of the output (training BatchNorm statistics); no split-K then.
// ``tay_part`` (nullable, needs ``mask``, no split-K; 1x1 stride 1, or transposed 3x3 stride 2 at
// even Ho / Wo): [R][B][Cout] Taylor partials, R = tp_conv_gen_tay_slots(cfg, Ho * Wo) (transposed:
// 4 x tp_conv_gen_tay_slots(cfg, Ho * Wo / 4), one slot range per stride phase), every slot
// written or left as the caller zeroed it.
extern "C" hipError_t tp_conv_gen5(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, float* tay_part, int tay_mode, const uint8_t* res_bits,
                                   const float* bnb_y, const float* bnb_mean, const float* bnb_invstd,
                                   const uint8_t* bnb_bits, hipStream_t st);

extern "C" hipError_t tp_conv_gen4(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, float* tay_part, int tay_mode, hipStream_t st) {
  return tp_conv_gen5(x, w, B, H, W, Cin, Cout, ks, stride, pad, transposed, Ho_t, Wo_t, cfg, splits, scale, shift,
                      relu, res, res_stride, mask, apoz, out, ws, bnpart, tay_part, tay_mode, nullptr, nullptr,
                      nullptr, nullptr, nullptr, st);
}

// ``res_bits`` (nullable; GEN 1, res at stride 1, no mask, Cout % 4 == 0): res is masked element-wise
// by a ReLU bit mask (byte (pix * Cout + n) / 4, bit n % 4) before the add. ``bnb_y`` (nullable; GEN 1,
// one K pass, with ``bnpart``): ``bnpart`` receives per M tile (sum gm, sum gm * (bnb_y - bnb_mean) *
// bnb_invstd) of the stored gradient gm (masked by ``bnb_bits`` when given) instead of the output's
// (sum, sum of squares): the backward statistics of the BatchNorm that produced the conv's input.
extern "C" hipError_t tp_conv_gen5(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks,
                                   int stride, int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits,
                                   const float* scale, const float* shift, int relu, const float* res,
                                   int res_stride, const float* mask, float* apoz, float* out, float* ws,
                                   double* bnpart, float* tay_part, int tay_mode, const uint8_t* res_bits,
                                   const float* bnb_y, const float* bnb_mean, const float* bnb_invstd,
                                   const uint8_t* bnb_bits, hipStream_t st) {
  using namespace tp;
  const int gen = transposed ? 3 : (Cin == 4 ? 2 : 1);
  if ((gen != 2 && (Cin % 4 != 0 || Cin < 8)) || Cout % 4 != 0 || res_stride < 1) return hipErrorInvalidValue;
  const bool sb = cfg >= 0 && (cfg & CFG_SB);
  if (sb) {  // single-buffered LDS stage: GEN 1 1x1 forward, one K pass, not with stream-K
    cfg &= ~CFG_SB;
    if (gen != 1 || ks != 1 || splits > 1 || (cfg & CFG_SK) || cfg >= 16)
      return hipErrorInvalidValue;
  }
  const bool sk = cfg >= 0 && (cfg & CFG_SK) && (cfg & ~CFG_SK) < 16;
  if (sk) {  // stream-K: GEN 1, one K pass, ``ws`` = the fixup slots (tp_conv_sk_ws_floats)
    cfg &= ~CFG_SK;
    if (gen != 1 || splits > 1 || !ws || (ks != 1 && ks != 3)) return hipErrorInvalidValue;
  }
  if (gen == 3 && (ks != 1 && ks != 3)) return hipErrorInvalidValue;
  ConvArgs a{};
  a.x = x;
  a.w = w;
  a.B = B;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.N = Cout;
  a.K = tp_conv_gen_k(ks, Cin);
  a.Ho = gen == 3 ? Ho_t : (H + 2 * pad - ks) / stride + 1;
  a.Wo = gen == 3 ? Wo_t : (W + 2 * pad - ks) / stride + 1;
  a.parity = gen == 3 && stride == 2 && a.Ho % 2 == 0 && a.Wo % 2 == 0;
  if (gen == 3) splits = 1;
  a.stride = stride;
  a.pad = pad;
  a.M = B * a.Ho * a.Wo;
  a.HWo = a.Ho * a.Wo;
  a.x_elems = (long long)B * H * W * Cin;
  if (a.x_elems * 4 >= (1ll << 31) || (long long)Cout * a.K * 4 >= (1ll << 31) ||
      (long long)a.M * Cout * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  const int kt = a.K / 32;
  splits = std::max(1, std::min(splits, kt));
  a.k_tiles_per_split = (kt + splits - 1) / splits;
  splits = (kt + a.k_tiles_per_split - 1) / a.k_tiles_per_split;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.res = res;
  a.res_stride = res_stride;
  a.mask = mask;
  a.apoz = apoz;
  a.out = out;
  static const int gen_epi = [] {  // TP_GEN_EPI=0: per-lane epilogue stores (experiments); read once
    const char* ge = getenv("TP_GEN_EPI");
    return ge ? atoi(ge) : 1;
  }();
  a.epi_lds = gen_epi;
  if (gen == 3 || mask || res_stride > 1 || bnpart) a.epi_lds = 1;  // only the LDS epilogue implements these
  if (bnpart) {
    if (splits > 1) return hipErrorInvalidValue;
    a.bnpart = bnpart;
  }
  if (res_bits && (gen != 1 || !res || res_stride != 1 || mask || splits > 1 || tay_part || Cout % 4 != 0))
    return hipErrorInvalidValue;
  if (bnb_y && (gen != 1 || !bnpart || !bnb_mean || !bnb_invstd || mask || relu || tay_part || Cout % 4 != 0))
    return hipErrorInvalidValue;
  if (bnb_bits && !bnb_y) return hipErrorInvalidValue;
  a.res_bits = res_bits;
  a.bnb_y = bnb_y;
  a.bnb_mean = bnb_mean;
  a.bnb_invstd = bnb_invstd;
  a.bnb_bits = bnb_bits;
  if (res_bits || bnb_y) a.epi_lds = 1;
  if (tay_part) {  // GEN 1: 1x1; GEN 3: the parity-ordered 3x3 stride-2 data gradient (4 phase groups)
    const bool t3 = gen == 3 && a.parity && ks == 3;
    if (splits > 1 || !mask || !((gen == 1 && ks == 1) || t3) || cfg >= 16 ||
        tp_conv_gen_tay_slots(cfg, t3 ? a.HWo / 4 : a.HWo) == 0)
      return hipErrorInvalidValue;
    a.tay_part = tay_part;
    a.tay_mode = tay_mode;
    a.epi_lds = 1;
  }
  if (sk) {
    a.sk_blocks = -1;
    a.sk_ws = ws;
  }
  a.sb = sb ? 1 : 0;
  if (a.tay_part) return gen == 3 ? gen_cfg<3, 3, EPI_FWD_TAY>(cfg, a, 1, st) : gen_cfg<1, 1, EPI_FWD_TAY>(cfg, a, 1, st);
  if (splits == 1) return gen_dispatch<EPI_FWD>(ks, gen, cfg, a, 1, st);
  if (!ws) return hipErrorInvalidValue;
  ConvArgs b = a;
  b.out = ws;
  hipError_t e = gen_dispatch<EPI_PARTIAL>(ks, gen, cfg, b, splits, st);
  if (e != hipSuccess) return e;
  const long long MN = (long long)a.M * a.N;
  const unsigned grid = (unsigned)std::min<long long>(ceil_div(MN, 256), 4096);
  conv_epilogue<EPI_FWD><<<grid, 256, 0, st>>>(a, ws, splits);
  return hipGetLastError();
}
