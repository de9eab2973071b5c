// Winograd F(4x4, 3x3) convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32) for the stride-1 3x3
// layers of square S x S feature maps, S in {4, 8, 16, 32} (VGG's 32/16/8/4-pixel stages):
// 36 multiplies per 4x4 output tile instead of 144 (direct) or 64 (F(2x2,3x3), winograd.hip),
// i.e. 1.78x fewer MFMAs than F(2x2) at the same LDS bytes per MFMA.
//
//   * a block = 4 waves = 32 output tiles (4x4 pixels) x 32 output channels; wave w owns the 16
//     tiles of half (w & 1) (MFMA rows, lane & 15) x the 16 channels of half (w >> 1) x all 36
//     transform points: 36 accumulator tiles, 144 registers;
//   * input channels advance in chunks of 8: lane (j, g) holds channels 2g, 2g+1 (MFMA k = g) of
//     its tile's 6x6 patch, read as float2 from a 2-plane (channels 0-3 / 4-7) LDS image of the
//     block's input region (halos shared, one 16-B slot per pixel and plane, DMA'd with
//     `buffer_load_dwordx4 ... lds`); the row / image pitches and a pad slot after every 4 columns
//     make the 16 tiles of a wave hit 16 different bank quads (conflict-free ds_read_b64) with
//     compile-time patch offsets; S = 4 stages image interiors only (the border is a constant 0);
//   * the transformed weights U = G g G^T of (8 channels x 32 outputs x 36 points) are one 36-KB
//     pre-arranged LDS image per chunk: one conflict-free ds_read_b64 = the B operands of both
//     channel halves of a point;
//   * software pipeline: the DMA of chunk c+1 is issued at the top of chunk c; after the first
//     half of chunk c's MFMAs the waves wait for it (one barrier), read their next patch and form
//     V = B^T d B for chunk c+1 under the second half of chunk c's MFMAs;
//   * epilogue: Y = A^T m A in registers, parked in LDS, then coalesced 128-B stores with the
//     fused epilogue contract of winograd.hip — BN affine + NaN-propagating ReLU (+ 2x2 max-pool
//     with argmax bytes), APoZ counts, and for the data gradient the ReLU-mask / BN-scale output
//     and the Taylor / Sensitivity partials — summed per (image, channel) in a fixed order with
//     one writer per sum (every image lies in a single block): deterministic, no atomics.
//
// Transform points 0, +-1, +-2, inf (Lavin & Gray); fp32 error ~2e-6 relative (64-channel
// reduction), well inside the engine's fp64-oracle tolerances.
#include "tp_common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace tp {
namespace w4 {

enum Epi : int { FWD = 0, FWD_POOL = 1, BWD = 2, PARTIAL = 3 };  // PARTIAL: raw split-K slab (MODE 2/3)

constexpr int TILES = 32;                 // output tiles per block
constexpr int TK = 32;                    // output channels per block
constexpr int NPT = 36;                   // transform points
constexpr int U_IMG = NPT * 2 * 16 * 8;   // 9216 floats per (8-channel chunk, 32-output) image
constexpr int U_ROUNDS = U_IMG / 1024;    // 9 DMA rounds of 256 16-B slots
constexpr int TPL = 16 * 16 + 4;          // epilogue LDS floats per tile (16 px x 16 ch + bank pad)
constexpr unsigned OOB = 0x80000000u;

// Staged input region per spatial size, per plane: NI images per block (32 tiles), image pitch
// IP slots, row pitch RWP slots, RH rows; for S >= 8 the region carries the 1-pixel halo and a
// pad slot after every 4 columns (col' = x' + x'/4, x' = x + 1); S = 4 holds the 4x4 interiors.
// Conflict rule (ds_read_b64 of 8 B at slot s, bank = 4s + 2(g & 1) mod 64): the 16 slot bases of
// a wave's tiles must be distinct mod 16. XR = DMA rounds of 256 slots for both planes.
template <int S> struct Geo;
template <> struct Geo<32> { static constexpr int NI = 1, RH = 18, RWP = 42, IP = 18 * 42; };
template <> struct Geo<16> { static constexpr int NI = 2, RH = 18, RWP = 23, IP = 18 * 23; };
template <> struct Geo<8> { static constexpr int NI = 8, RH = 10, RWP = 14, IP = 146; };
template <> struct Geo<4> { static constexpr int NI = 32, RH = 4, RWP = 4, IP = 17; };
template <int S> constexpr int plane_slots() { return Geo<S>::NI * Geo<S>::IP; }
// MODE 2 (64-tile blocks): S = 32 holds a whole image (34 rows); otherwise twice the images
// Staged input geometry of a TB-tile block (MODE 2/3). PAD: a pad slot after every 4 columns
// (col' = x' + x'/4) keeps the slot bases of the 16 tiles of a wave distinct mod 16 when a wave
// spans tile rows of one image (S = 32, 16); S = 8 packs its 10 x 10 halo'd images densely
// (IP = 101: 16 tiles = 4 images x 2 x 2 cover all 16 classes). S = 32, TB = 32: half an image.
template <int S, int TB> struct GeoT;
template <int TB> struct GeoT<32, TB> {
  static constexpr int NI = 1, RH = TB / 2 + 2, RWP = 42, IP = (TB / 2 + 2) * 42, PAD = 1;
};
template <int TB> struct GeoT<16, TB> { static constexpr int NI = TB / 16, RH = 18, RWP = 23, IP = 18 * 23, PAD = 1; };
template <int TB> struct GeoT<8, TB> { static constexpr int NI = TB / 4, RH = 10, RWP = 10, IP = 101, PAD = 0; };
template <int TB> struct GeoT<4, TB> { static constexpr int NI = TB, RH = 4, RWP = 4, IP = 17, PAD = 0; };
template <int S> constexpr int x_rounds() { return (2 * plane_slots<S>() + 255) / 256; }
// Band geometry: square maps of any other size (ResNet's 56 / 28 / 14 / 7 pixels). Tile rows hold
// TPR = ceil(S / 4) tiles (the last one partial when S % 4: its out-of-map pixels read zeros and
// are not stored); a block takes BR whole tile rows counted across images (TBR <= 32 real tiles,
// the other MFMA rows are padding); each tile row is staged on its own — 6 pixel rows with the
// halo, columns x' = x + 1 in [0, 4 TPR + 1] with a pad slot after every 4 (col' = x' + x'/4) — so
// a band that straddles two images needs no special case. R: Taylor partial slots per image (the
// most bands one image's TPR tile rows can overlap; one writer per slot).
template <int S> struct Band {
  static constexpr bool ON = !(S == 4 || S == 8 || S == 16 || S == 32);
  static constexpr int TPR = (S + 3) / 4, BR = 32 / TPR, TBR = BR * TPR;
  static constexpr int W = 4 * TPR + 2, RWP = W + (W - 1) / 4, RH = 6 * BR;
  static constexpr int NI = 1, IP = RH * RWP, PAD = 1;
  static constexpr int R = (TPR + BR - 2) / BR + 1;
  static_assert(!ON || (S >= 5 && BR >= 1), "band geometry: 5 <= S <= 128");
};

struct Args {
  const float* x;     // NHWC (B, S, S, C): the input (forward) or the output gradient (dgrad)
  const float* u;     // U images [C/8][K/32][U_IMG]
  int B, C, K, P;     // P = output tiles = B * (S/4)^2
  int ko;             // output channels per pixel (<= K): channels k >= ko are neither read nor stored
  long long x_elems;
  const float* scale; // FWD: BN scale (K); BWD: previous layer's BN scale (K), nullable
  const float* shift; // FWD: BN shift (K), nullable
  int relu;
  float* out;         // FWD: (B,S,S,K) or pooled (B,S/2,S/2,K); BWD: (B,S,S,K) masked grad, nullable
  uint8_t* out_argmax;
  const float* act;   // BWD: the activation the gradient belongs to, (B,S,S,K)
  float* taylor;      // BWD: (R, B, K) slab, slot 0 written (+=), nullable
  float* apoz;        // FWD / FWD_POOL: (B, K) counts of positive outputs (+=), nullable
  int tay_mode;       // BWD partials: 0 Taylor -(g*a), 1 Sensitivity |g|
  long long slab;     // PARTIAL: floats per split slab (M * K); slab s = blockIdx.y
  int pool_order;     // PARTIAL: rows in pooled order (b, y/2, x/2, y&1, x&1) for a pooled combine
  int dbg;            // phase-cost experiments only (TP_W4_DBG; results are WRONG when set): 1 no U DMA,
                      // 2 no X DMA, 16 no epilogue
  const uint8_t* unp; // BWD with out: the argmax bytes (B,S,S,K) of the 2x2 pool that produced the
                      // activation; ``out`` is then written unpooled at (B,2S,2S,K) (the consumer's
                      // full-resolution operand: no separate unpooling pass)
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, float* lds_base, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)lds_base, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// one length-6 column / row of V = B^T d B, B^T rows: [4,0,-5,0,1,0] [0,-4,-4,1,1,0] [0,4,-4,-1,1,0]
// [0,-2,-1,2,1,0] [0,2,-1,-2,1,0] [0,4,0,-5,0,1]
__device__ __forceinline__ void bt6(float& a0, float& a1, float& a2, float& a3, float& a4, float& a5) {
  const float s12 = a1 + a2, s34 = a3 + a4, d12 = a1 - a2, d43 = a4 - a3, d42 = a4 - a2, d31 = a3 - a1;
  const float o0 = fmaf(4.f, a0, fmaf(-5.f, a2, a4));
  const float o5 = fmaf(4.f, a1, fmaf(-5.f, a3, a5));
  a0 = o0;
  a1 = fmaf(-4.f, s12, s34);
  a2 = fmaf(4.f, d12, d43);
  a3 = fmaf(2.f, d31, d42);
  a4 = fmaf(-2.f, d31, d42);
  a5 = o5;
}

__device__ __forceinline__ void input_transform(float (&d)[36]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) bt6(d[c], d[6 + c], d[12 + c], d[18 + c], d[24 + c], d[30 + c]);
#pragma unroll
  for (int r = 0; r < 6; ++r) bt6(d[6 * r], d[6 * r + 1], d[6 * r + 2], d[6 * r + 3], d[6 * r + 4], d[6 * r + 5]);
}

// step k (0..23) of V = B^T d B for two channels: k < 12 column passes (channel k / 6, column
// k % 6), then row passes (channel (k - 12) / 6, row (k - 12) % 6); in this order every row pass
// follows its channel's column passes.
__device__ __forceinline__ void transform_step(float (&d0)[36], float (&d1)[36], int k) {
  float(&d)[36] = (k < 12 ? (k < 6) : (k < 18)) ? d0 : d1;
  if (k < 12) {
    const int c = k % 6;
    bt6(d[c], d[6 + c], d[12 + c], d[18 + c], d[24 + c], d[30 + c]);
  } else {
    const int r = (k - 12) % 6;
    bt6(d[6 * r], d[6 * r + 1], d[6 * r + 2], d[6 * r + 3], d[6 * r + 4], d[6 * r + 5]);
  }
}

// Y = A^T m A, A^T = [[1,1,1,1,1,0],[0,1,-1,2,-2,0],[0,1,1,4,4,0],[0,1,-1,8,-8,1]]
__device__ __forceinline__ void at6(const float m0, const float m1, const float m2, const float m3, const float m4,
                                    const float m5, float& y0, float& y1, float& y2, float& y3) {
  const float a = m1 + m2, b = m1 - m2, c = m3 + m4, d = m3 - m4;
  y0 = m0 + a + c;
  y1 = fmaf(2.f, d, b);
  y2 = fmaf(4.f, c, a);
  y3 = fmaf(8.f, d, b) + m5;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// at6 on two accumulator rows at once (v_pk_add_f32 / v_pk_fma_f32): rows r, r+1 of an f32x4
// accumulator are an aligned register pair, so the epilogue's output transform costs half the
// VALU instructions; same operations and rounding as at6
__device__ __forceinline__ void at6p(const f2v m0, const f2v m1, const f2v m2, const f2v m3, const f2v m4,
                                     const f2v m5, f2v& y0, f2v& y1, f2v& y2, f2v& y3) {
  const f2v a = m1 + m2, b = m1 - m2, c = m3 + m4, d = m3 - m4;
  y0 = m0 + a + c;
  y1 = 2.f * d + b;
  y2 = 4.f * c + a;
  y3 = 8.f * d + b + m5;
}

__device__ __forceinline__ void output_transform2(const f2v (&m)[36], f2v (&y)[16]) {
  f2v t[24];
#pragma unroll
  for (int c = 0; c < 6; ++c)
    at6p(m[c], m[6 + c], m[12 + c], m[18 + c], m[24 + c], m[30 + c], t[c], t[6 + c], t[12 + c], t[18 + c]);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    at6p(t[6 * r], t[6 * r + 1], t[6 * r + 2], t[6 * r + 3], t[6 * r + 4], t[6 * r + 5], y[4 * r], y[4 * r + 1],
         y[4 * r + 2], y[4 * r + 3]);
}

__device__ __forceinline__ void output_transform(const float (&m)[36], float (&y)[16]) {
  float t[24];  // 4 x 6
#pragma unroll
  for (int c = 0; c < 6; ++c)
    at6(m[c], m[6 + c], m[12 + c], m[18 + c], m[24 + c], m[30 + c], t[c], t[6 + c], t[12 + c], t[18 + c]);
#pragma unroll
  for (int r = 0; r < 4; ++r)
    at6(t[6 * r], t[6 * r + 1], t[6 * r + 2], t[6 * r + 3], t[6 * r + 4], t[6 * r + 5], y[4 * r], y[4 * r + 1],
        y[4 * r + 2], y[4 * r + 3]);
}

// Split-points epilogue, phase 1 (32-tile blocks of 4 waves): wave (grp = wave & 1, ph = wave >> 1)
// holds rows 3ph..3ph+2 of the 6x6 transform-point grid (acc[nh * 18 + 6 rr + c]) for its 16
// tiles x both 16-channel halves. Y = A^T M A is linear in M, so each wave forms the partial
// output of its three rows; the ph = 0 waves write it into ya / yb, the ph = 1 waves add theirs
// (read-modify-write; fixed order: one add per output after the write, deterministic). Partial column passes:
//   ph 0 (rows 0-2): t0 = m0 + m1 + m2, t1 = t3 = m1 - m2, t2 = m1 + m2
//   ph 1 (rows 3-5): t0 = s, t1 = 2d, t2 = 4s, t3 = 8d + m5   (s = m3 + m4, d = m3 - m4)
// and for ph 1 the row pass runs on s, d, m5 once each (at6 is linear), the scalings folding
// into the adds.
__device__ __forceinline__ void at6row(const f2v* t, f2v& y0, f2v& y1, f2v& y2, f2v& y3) {
  at6p(t[0], t[1], t[2], t[3], t[4], t[5], y0, y1, y2, y3);
}

// one wave's partial output (its three point rows) for tiles r, r + 1 of the lane: written
// (ph 0) or added (ph 1) into the parked tile image
template <int PH>
__device__ __forceinline__ void sp_partial(const f32x4 (&acc)[NPT], int grp, int lane, float* ya, float* yb) {
  grp &= 1;  // tile group within the parked half of 32 tiles
  const int j = lane & 15, g = lane >> 4;
#pragma unroll
  for (int nh = 0; nh < 2; ++nh) {
    float* ybuf = nh ? yb : ya;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {  // tiles r, r + 1 of this lane: packed pairs
      const int tl = grp * 16 + 4 * g + r;
      f2v m[18];
#pragma unroll
      for (int x = 0; x < 18; ++x) m[x] = f2v{acc[nh * 18 + x][r], acc[nh * 18 + x][r + 1]};
      float* dst = ybuf + tl * TPL + j;
      if constexpr (PH == 0) {
        f2v t0[6], t1[6], t2[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const f2v a = m[6 + c] + m[12 + c];
          t1[c] = m[6 + c] - m[12 + c];
          t2[c] = a;
          t0[c] = m[c] + a;
        }
        f2v y[12];
        at6row(t0, y[0], y[1], y[2], y[3]);
        at6row(t1, y[4], y[5], y[6], y[7]);
        at6row(t2, y[8], y[9], y[10], y[11]);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const f2v v = y[q < 12 ? q : q - 8];  // output row 3 = row 1
          dst[q * 16] = v.x;
          dst[TPL + q * 16] = v.y;
        }
      } else {
        f2v s[6], d[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          s[c] = m[c] + m[6 + c];
          d[c] = m[c] - m[6 + c];
        }
        f2v ys[4], yd[4], y5[4];
        at6row(s, ys[0], ys[1], ys[2], ys[3]);
        at6row(d, yd[0], yd[1], yd[2], yd[3]);
        at6row(m + 12, y5[0], y5[1], y5[2], y5[3]);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = q >> 2, col = q & 3;
          f2v add;
          if (row == 0) add = ys[col];
          else if (row == 1) add = 2.f * yd[col];
          else if (row == 2) add = 4.f * ys[col];
          else add = 8.f * yd[col] + y5[col];
          // plain read-modify-write, one per output after the ph 0 write (fixed order). NOT an LDS
          // float atomic: ds_add_f32 made this epilogue 5x slower on post-ReLU operands than on
          // N(0,1) ones (data-dependent; profiles/wino4/split_points_r5.txt)
          dst[q * 16] += add.x;
          dst[TPL + q * 16] += add.y;
        }
      }
    }
  }
}

// active: the wave's tile group lies in the half of 32 tiles being parked (8-wave blocks park
// their 64 tiles in two halves)
__device__ __forceinline__ void sp_phase1(const f32x4 (&acc)[NPT], int ph, int grp, int lane, float* ya, float* yb,
                                          bool active) {
  if (active && ph == 0) sp_partial<0>(acc, grp, lane, ya, yb);
  __syncthreads();  // ph 1 adds after every ph 0 write has landed
  if (active && ph == 1) sp_partial<1>(acc, grp, lane, ya, yb);
}

// Epilogue of a block of NW waves holding PPW (16-tile group, 16-channel half) accumulator sets
// each: TB = 8 * NW * PPW tiles x 32 output channels. Virtual wave v = wave + NW * pp owns group
// v % (TB/16) and half v / (TB/16) (PPW = 1: MODE 2/3; PPW = 2: the wide kernel, one wave = one
// group x both halves). Outputs are staged in LDS per half of 32 tiles (ya: channels 0-15, yb:
// 16-31), then coalesced 128-B traffic; ``part`` receives per-(tile, channel) partial sums
// (TB x 32 floats). SPP: the split-points kernels (NW = 4 / 8: 32 / 64 tiles): phase 1 is sp_phase1.
template <int EPI, int S, int NW, int PPW = 1, bool SPP = false>
__device__ __forceinline__ void epilogue(const Args& p, f32x4 (&acc)[PPW][NPT], int t0, int k0, float* ya, float* yb,
                                         float* part) {
  constexpr int TPR = (S + 3) / 4, TI = TPR * TPR;
  constexpr int GROUPS = NW * PPW / 2, TB = 16 * GROUPS, HALVES = TB / 32, TPW = 32 / NW;  // tiles per wave (phase 2)
  constexpr bool BAND = Band<S>::ON;
  constexpr int TBR = BAND ? Band<S>::TBR : TB;  // real tiles of the block (t0 = block * TBR)
  constexpr bool PART_TILE = S % 4 != 0;         // the last tile of a row is partial
  static_assert(!BAND || (EPI != FWD_POOL && NW == 4 && PPW == 1), "band geometry: no pooling, 4-wave blocks");
  static_assert(!SPP || PPW == 1, "split-points epilogue: one accumulator set per wave");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const bool want_part = EPI == BWD ? p.taylor != nullptr : p.apoz != nullptr;
  const int c4 = lane & 7;
  const int k = k0 + 4 * c4;
  const int KO = p.ko;          // output row width (pruned widths: K rounded up to 32 in the MFMAs only)
  const bool kok = k < KO;      // this lane's 4 channels are stored (KO % 4 == 0)
  const float* ysrc = (c4 < 4 ? ya : yb) + (c4 & 3) * 4;
  f32x4 sc4 = {1.f, 1.f, 1.f, 1.f}, sh4 = {0.f, 0.f, 0.f, 0.f};
  if (p.scale && kok) sc4 = *reinterpret_cast<const f32x4*>(p.scale + k);
  if (EPI != BWD && p.shift && kok) sh4 = *reinterpret_cast<const f32x4*>(p.shift + k);

#pragma unroll
  for (int hf = 0; hf < HALVES; ++hf) {
    // ---- phase 1: output transform; park this half's 32 tiles x 16 px x (16 + 16) ch -------
    if constexpr (SPP) sp_phase1(acc[0], wave / GROUPS, wave % GROUPS, lane, ya, yb, (wave % GROUPS) / 2 == hf);
#pragma unroll
    for (int pp = 0; pp < (SPP ? 0 : PPW); ++pp) {
      const int vw = wave + NW * pp, grp = vw % GROUPS, nh = vw / GROUPS;
      if (grp / 2 == hf) {
        float* ybuf = nh ? yb : ya;
#pragma unroll
        for (int r = 0; r < 4; r += 2) {  // tiles r, r + 1 of this lane: packed pairs
          const int tl = (grp & 1) * 16 + 4 * g + r;
          f2v m[36], y[16];
#pragma unroll
          for (int x = 0; x < NPT; ++x) m[x] = f2v{acc[pp][x][r], acc[pp][x][r + 1]};
          output_transform2(m, y);
          float* dst = ybuf + tl * TPL + j;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            dst[q * 16] = y[q].x;
            dst[TPL + q * 16] = y[q].y;
          }
        }
      }
    }
    // data gradient: this lane's phase-2 activations, issued before the barrier that ends phase 1
    // (the accumulators are dead, so the registers are free): their global-memory latency runs
    // while the block's other waves finish their output transforms, not inside phase 2
    f32x4 apre[EPI == BWD ? TPW : 1][2];
    if constexpr (EPI == BWD) {
      const int qq = lane >> 3;
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) {
        const int tbv = hf * 32 + wave * TPW + tt;
        const int pt = t0 + tbv;
        const int b = pt / TI, ti = pt - b * TI, tr = ti / TPR, tc = ti - tr * TPR;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int q = qq + 8 * h2;
          const int yy = 4 * tr + (q >> 2), xx = 4 * tc + (q & 3);
          const long long pix = ((long long)b * S + yy) * S + xx;
          const bool ok = kok && pt < p.P && tbv < TBR && (!PART_TILE || (yy < S && xx < S));
          apre[tt][h2] = ok ? *reinterpret_cast<const f32x4*>(p.act + pix * KO + k) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    __syncthreads();
    // ---- phase 2: coalesced traffic; 8 lanes cover one pixel's 32 channels (128 B) ----------
    if constexpr (EPI == FWD_POOL) {
      const int pp = (lane >> 3) & 3;  // pooled pixel (py, px) of the tile
      const int py = pp >> 1, px = pp & 1;
#pragma unroll
      for (int tt = 0; tt < TPW / 2; ++tt) {
        const int tl = wave * TPW + 2 * tt + (lane >> 5);
        const int tb = hf * 32 + tl;
        const int pt = t0 + tb;
        f32x4 cnt = {0.f, 0.f, 0.f, 0.f};
        if (pt < p.P) {
          f32x4 best = {0.f, 0.f, 0.f, 0.f};
          unsigned arg = 0;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int q = (2 * py + (w >> 1)) * 4 + 2 * px + (w & 1);
            const f32x4 yv = *reinterpret_cast<const f32x4*>(ysrc + tl * TPL + q * 16);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float v = yv[e] * sc4[e] + sh4[e];
              if (p.relu) v = nan_relu(v);
              cnt[e] += v > 0.f ? 1.f : 0.f;
              if (w == 0 || v > best[e] || (v != v && best[e] == best[e])) {
                best[e] = v;
                arg = (arg & ~(0xffu << (8 * e))) | ((unsigned)w << (8 * e));
              }
            }
          }
          const int b = pt / TI, ti = pt - b * TI, tr = ti / TPR, tc = ti - tr * TPR;
          const long long o = (((long long)b * (S / 2) + 2 * tr + py) * (S / 2) + 2 * tc + px) * KO + k;
          if (kok) {
            *reinterpret_cast<f32x4*>(p.out + o) = best;
            *reinterpret_cast<unsigned*>(p.out_argmax + o) = arg;
          }
        }
        if (want_part) {  // per-(tile, channel) count over the 4 pooled pixels (lanes ^8, ^16)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cnt[e] = xsum16(xsum8(cnt[e]));
          }
          if (pp == 0) *reinterpret_cast<f32x4*>(part + tb * TK + 4 * c4) = cnt;
        }
      }
    } else {
      const int qq = lane >> 3;  // pixels qq and qq + 8 of the tile
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) {
        const int tl = wave * TPW + tt;
        const int tb = hf * 32 + tl;
        const int pt = t0 + tb;
        f32x4 sum = {0.f, 0.f, 0.f, 0.f};
        if (pt < p.P && tb < TBR) {
          const int b = pt / TI, ti = pt - b * TI, tr = ti / TPR, tc = ti - tr * TPR;
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int q = qq + 8 * h2;
            if (PART_TILE && (4 * tr + (q >> 2) >= S || 4 * tc + (q & 3) >= S)) continue;  // outside the map
            const f32x4 yv = *reinterpret_cast<const f32x4*>(ysrc + tl * TPL + q * 16);
            const long long pix = ((long long)b * S + 4 * tr + (q >> 2)) * S + 4 * tc + (q & 3);
            if constexpr (EPI == PARTIAL) {
              const int yy = 4 * tr + (q >> 2), xx = 4 * tc + (q & 3);
              const long long row = p.pool_order
                                        ? ((((long long)b * (S / 2) + (yy >> 1)) * (S / 2) + (xx >> 1)) * 4 +
                                           (yy & 1) * 2 + (xx & 1))
                                        : pix;
              *reinterpret_cast<f32x4*>(p.out + (long long)blockIdx.y * p.slab + row * p.K + k) = yv;
            } else if constexpr (EPI == FWD) {
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                v[e] = yv[e] * sc4[e] + sh4[e];
                if (p.relu) v[e] = nan_relu(v[e]);
                sum[e] += v[e] > 0.f ? 1.f : 0.f;
              }
              if (kok) *reinterpret_cast<f32x4*>(p.out + pix * KO + k) = v;
            } else {  // BWD
              const f32x4 a = apre[EPI == BWD ? tt : 0][h2];
#pragma unroll
              for (int e = 0; e < 4; ++e) sum[e] += tay_term(p.tay_mode, yv[e], a[e]);
              if (p.out && kok) {
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = a[e] > 0.f ? yv[e] * sc4[e] : 0.f;
                if (p.unp) {  // the 2x2 window of this pooled pixel: v at its argmax, 0 elsewhere
                  const unsigned am4 = *reinterpret_cast<const unsigned*>(p.unp + pix * KO + k);
                  const int yy = 4 * tr + (q >> 2), xx = 4 * tc + (q & 3);
                  const long long o00 = (((long long)b * 2 * S + 2 * yy) * 2 * S + 2 * xx) * KO + k;
#pragma unroll
                  for (int w = 0; w < 4; ++w) {
                    f32x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = ((am4 >> (8 * e)) & 0xffu) == (unsigned)w ? v[e] : 0.f;
                    *reinterpret_cast<f32x4*>(p.out + o00 + ((long long)(w >> 1) * 2 * S + (w & 1)) * KO) = o;
                  }
                } else {
                  *reinterpret_cast<f32x4*>(p.out + pix * KO + k) = v;
                }
              }
            }
          }
        }
        if (want_part) {  // per-(tile, channel) sum over the 16 pixels: lanes ^8, ^16, ^32 (fixed order)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sum[e] = xsum32(xsum16(xsum8(sum[e])));
          }
          if (qq == 0) *reinterpret_cast<f32x4*>(part + tb * TK + 4 * c4) = sum;
        }
      }
    }
    __syncthreads();  // ya / yb are rewritten by the next half
  }
  if (!want_part) return;
  if constexpr (BAND) {
    // a band's tiles cover consecutive images (one writer per (slot, image, channel): slot = this
    // block's index among the bands that overlap the image; APoZ counts are exact, added atomically)
    const int b0 = t0 / TI, nimg = (t0 + TBR - 1) / TI - b0 + 1;
    const int blk = t0 / TBR;
    for (int t = tid; t < nimg * TK; t += 64 * NW) {
      const int il = t / TK, kk = t - il * TK;
      const int b = b0 + il;
      if (b >= p.B || k0 + kk >= KO) continue;
      const int s0 = max(0, b * TI - t0), s1 = min(TBR, (b + 1) * TI - t0);
      float s = 0.f;
      for (int ti = s0; ti < s1; ++ti) s += part[ti * TK + kk];
      if constexpr (EPI == BWD) {
        const int slot = blk - (b * TPR) / Band<S>::BR;
        p.taylor[((long long)slot * p.B + b) * KO + k0 + kk] += s;
      } else {
        if (s > 0.f) atomicAdd(p.apoz + (long long)b * KO + k0 + kk, s);
      }
    }
    return;
  }
  // ---- per-(image, channel) sums over the block's tiles of the image, fixed order ------------
  // Whole images per block: one writer per sum. A block of half an image (S = 32, 32 tiles):
  // Taylor partials go to slot (half) of the (R, B, K) slab (single writer per slot); APoZ counts
  // are exact integers, so their float atomic adds are order-independent.
  constexpr int TIB = TI < TB ? TI : TB;  // tiles of one image in this block
  constexpr int NIB = TB / TIB;           // images in this block
  const int b0 = t0 / TI;
  for (int t = tid; t < NIB * TK; t += 64 * NW) {
    const int il = t / TK, kk = t - il * TK;
    const int b = b0 + il;
    if (b >= p.B || k0 + kk >= KO) continue;
    float s = 0.f;
    for (int ti = 0; ti < TIB; ++ti) s += part[(il * TIB + ti) * TK + kk];
    constexpr bool split_img = TI > TB;
    if constexpr (EPI == BWD) {
      const int slot = split_img ? (t0 / TB) % (TI / TB) : 0;
      p.taylor[((long long)slot * p.B + b) * KO + k0 + kk] += s;
    } else if constexpr (split_img) {
      if (s > 0.f) atomicAdd(p.apoz + (long long)b * KO + k0 + kk, s);
    } else {
      p.apoz[(long long)b * KO + k0 + kk] += s;
    }
  }
}


// LDS DMA issued from inline asm: invisible to the compiler's wait-count tracking, which would
// otherwise wait for every DMA in flight before any LDS read of a buffer it cannot tell apart
// (runtime-selected double buffers). The caller owns the vmcnt waits. rsrc: raw 4-dword buffer
// descriptor (base, stride 0, num_records, raw-buffer flags); lds: wave-uniform LDS byte address.
typedef int i32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4v raw_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  return i32x4v{(int)(unsigned)a, (int)((unsigned)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
}
__device__ __forceinline__ unsigned lds_addr(const float* p) { return (unsigned)(size_t)(lds_ptr_t)p; }
__device__ __forceinline__ void dma16_asm(const i32x4v& rs, unsigned lds, unsigned voff, unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(rs), "s"(soff)
               : "memory", "m0");
}

__device__ __forceinline__ void lds_barrier() {  // LDS reads done + s_barrier, leaving DMA (vmcnt) in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// MODE 2: one block of 8 waves per CU (two per SIMD) = 64 tiles x 32 outputs; wave w owns the 16
// tiles of group (w & 3) x the 16 channels of half (w >> 2).
//
// Cost model (measured, scripts/micro/mfma_valu.hip): on gfx950 fp32 MFMAs and fp32 VALU work
// share the SIMD's issue — VALU between MFMAs does not hide, not even across the two waves of a
// SIMD — so the kernel minimises VALU instructions instead of interleaving them: the input
// transform runs on packed pairs (v_pk_fma_f32 / v_pk_add_f32: both channels of a lane, one
// instruction), the patch of a lane is read as float2 pairs (channels 2g, 2g+1; conflict-free
// ds_read_b64), and the MFMA k of parity e is channel 2g + e. The U image uses layout 1 (one
// float2 = points 2i, 2i+1 of one parity; parity 0 in the first half, parity 1 in the second).
//
// Per chunk c: top barrier (U0(c), X(c) landed) -> issue U1(c) -> read + transform the patch ->
// 36 MFMAs of parity 0 -> barrier (U1(c) landed; U0 and X(c) free) -> issue U0(c+1), X(c+2) ->
// 36 MFMAs of parity 1. X is double-buffered (1.5 chunks of lead), U single-buffered in halves
// (half a chunk of lead). DMA is issued from inline asm; the waits are explicit.
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void bt6p(f2v& a0, f2v& a1, f2v& a2, f2v& a3, f2v& a4, f2v& a5) {
  const f2v s12 = a1 + a2, s34 = a3 + a4, d12 = a1 - a2, d43 = a4 - a3, d42 = a4 - a2, d31 = a3 - a1;
  const f2v o0 = 4.f * a0 + (-5.f * a2 + a4);
  const f2v o5 = 4.f * a1 + (-5.f * a3 + a5);
  a0 = o0;
  a1 = -4.f * s12 + s34;
  a2 = 4.f * d12 + d43;
  a3 = 2.f * d31 + d42;
  a4 = -2.f * d31 + d42;
  a5 = o5;
}

// SPREAD (NW = 4, variant 2): U0(c+1) is issued one 1-KB piece per two MFMA steps over the first
// half of the parity-1 steps instead of in a burst at the mid-chunk barrier, where the burst
// stalled the issuing wave on the TA address FIFO (SQ_VMEM_TA_ADDR_FIFO_FULL) while its MFMAs
// waited; the MFMAs are inline asm with the accumulators pinned to VGPRs, so the branches around
// the pieces cannot make the register allocator copy them (what defeated this schedule with
// builtins). (Spreading X(c+1) over the parity-0 steps as well spilled ~25 VGPRs in the loop: the
// whole transformed patch is still live there.)
#define W4_MFMA2(NOP, c0, c1, a0, a1, w)                                                            \
  asm volatile(NOP                                                                                  \
               "v_mfma_f32_16x16x4_f32 %0, %2, %4, %0\n\t"                                         \
               "v_mfma_f32_16x16x4_f32 %1, %3, %5, %1"                                             \
               : "+v"(c0), "+v"(c1)                                                                 \
               : "v"(a0), "v"(a1), "v"(w.x), "v"(w.y))

// Split points (variant 3): the two waves of a 16-tile group each own three rows of the 6x6
// transform-point grid (18 points) x all 32 output channels instead of all 36 points x 16
// channels. The accumulators stay 36 tiles per wave, the MFMAs 72 per chunk, but each wave forms
// only its half of V = B^T d B: the first (column) pass computes 3 of its 6 outputs, the second
// runs on 3 rows — 72 packed VALU ops per chunk instead of 168 (the 12-op length-6 transform
// below, vs 14). fp32 VALU does not co-issue with fp32 MFMAs on gfx950, so this is the lever.
//   B^T rows: o0 = 4a0 - 5a2 + a4; o1/o2 = p +- q (p = a4 - 4a2, q = a3 - 4a1);
//             o3/o4 = r +- 2s (r = a4 - a2, s = a3 - a1); o5 = 4a1 - 5a3 + a5
__device__ __forceinline__ void bt6q(f2v& a0, f2v& a1, f2v& a2, f2v& a3, f2v& a4, f2v& a5) {
  const f2v p = -4.f * a2 + a4, q = -4.f * a1 + a3, r = a4 - a2, s = a3 - a1;
  const f2v o0 = 4.f * a0 + (-5.f * a2 + a4);
  const f2v o5 = 4.f * a1 + (-5.f * a3 + a5);
  a0 = o0;
  a1 = p + q;
  a2 = p - q;
  a3 = 2.f * s + r;
  a4 = -2.f * s + r;
  a5 = o5;
}

// first (column) pass of one patch column for point half ph: rows 3ph..3ph+2 of V's column c
template <int PH>
__device__ __forceinline__ void sp_col(const f2v (&a)[6], f2v (&w)[18], int c) {
  if constexpr (PH == 0) {
    const f2v p = -4.f * a[2] + a[4], q = -4.f * a[1] + a[3];
    w[c] = 4.f * a[0] + (-5.f * a[2] + a[4]);
    w[6 + c] = p + q;
    w[12 + c] = p - q;
  } else {
    const f2v r = a[4] - a[2], s = a[3] - a[1];
    w[c] = 2.f * s + r;
    w[6 + c] = -2.f * s + r;
    w[12 + c] = 4.f * a[1] + (-5.f * a[3] + a[5]);
  }
}

// w[6 rr + c] = V[3 ph + rr][c] of the lane's two channels. The patch is read column by column
// (one ds_read_b64 each), one column ahead of its pass, so at most two raw columns are live
// (24 VGPRs instead of the whole 72-register patch: no spills beside the 144 accumulators).
template <int S, typename G, int PH>
__device__ __forceinline__ void sp_read_transform(const float* p0, f2v (&w)[18]) {
  f2v col[2][6];
  auto rd = [&](int q, f2v (&d)[6]) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      f2v v = {0.f, 0.f};
      if constexpr (S == 4) {
        if (r >= 1 && r <= 4 && q >= 1 && q <= 4) v = *reinterpret_cast<const f2v*>(p0 + ((r - 1) * 4 + (q - 1)) * 4);
      } else {
        v = *reinterpret_cast<const f2v*>(p0 + (r * G::RWP + q + (G::PAD && q >= 4 ? 1 : 0)) * 4);
      }
      d[r] = v;
      __builtin_amdgcn_sched_barrier(0);  // one ds_read_b64 each (no ds_read2 merging)
    }
  };
  rd(0, col[0]);
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    if (c + 1 < 6) rd(c + 1, col[(c + 1) & 1]);
    sp_col<PH>(col[c & 1], w, c);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int rr = 0; rr < 3; ++rr) bt6q(w[6 * rr], w[6 * rr + 1], w[6 * rr + 2], w[6 * rr + 3], w[6 * rr + 4], w[6 * rr + 5]);
}

// the 72 MFMAs of one chunk for a split-points wave: per parity e (input channel 2g + e) 9 point
// pairs x both channel halves; ``mid`` runs between the parities (U1 wait + barrier + next DMAs)
template <typename Mid>
__device__ __forceinline__ void sp_mfma_chunk(int c, int nc, const f2v (&w)[18], const float* ul, f32x4 (&acc)[NPT],
                                              Mid mid, int ph) {
  (void)c;
  (void)nc;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    if (e == 1) mid();
    const float* ue = ul + (e * 18 + 9 * ph) * 256;
    float2 wq[2][2];  // [pair parity][channel half]
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        wq[s2][h] = *reinterpret_cast<const float2*>(ue + s2 * 256 + h * 128);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const float2 w0 = wq[i & 1][0], w1 = wq[i & 1][1];
      if (i + 2 < 9) {
        wq[i & 1][0] = *reinterpret_cast<const float2*>(ue + (i + 2) * 256);
        __builtin_amdgcn_sched_barrier(0);
        wq[i & 1][1] = *reinterpret_cast<const float2*>(ue + (i + 2) * 256 + 128);
        __builtin_amdgcn_sched_barrier(0);
      }
      const int x = 2 * i;
      const float a0 = e ? w[x].y : w[x].x, a1 = e ? w[x + 1].y : w[x + 1].x;
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, w0.x, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, w0.y, acc[x + 1], 0, 0, 0);
      acc[18 + x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, w1.x, acc[18 + x], 0, 0, 0);
      acc[18 + x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, w1.y, acc[18 + x + 1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <int EPI, int S, int NW, bool SPREAD = false, bool SPLITP = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void wino4_m2(Args p) {
  static_assert(!SPREAD || NW == 4, "SPREAD is the 4-wave (two blocks per CU) schedule");
  // (an 8-wave 64-tile split-points build measured 5-8% slower than the 4-wave one: not built)
  static_assert(!SPLITP || (NW == 4 && !SPREAD), "split points: 4-wave blocks, burst DMA");
  constexpr int TB = 8 * NW, NG = NW / 2;  // tiles per block, 16-tile groups
  constexpr bool XDBL = NW == 8;           // X double-buffered (one block per CU)
  constexpr bool BAND = Band<S>::ON;
  static_assert(!BAND || SPLITP, "band geometry: the split-points kernel");
  using G = std::conditional_t<BAND, Band<S>, GeoT<S, TB>>;
  constexpr int TPR = (S + 3) / 4, TI = TPR * TPR;
  constexpr int TBR = BAND ? Band<S>::TBR : TB;  // real tiles per block
  constexpr int PL = G::NI * G::IP;
  constexpr int NXI = (2 * PL + 63) / 64;  // X DMA wave-instructions (64 16-B slots each)
  constexpr int KX = (NXI + NW - 1) / NW;
  constexpr int XN = (XDBL ? (NXI > 34 ? NXI : 34) : (NXI > 33 ? NXI : 33)) * 256;
  __shared__ __attribute__((aligned(16))) float us[U_IMG];
  __shared__ __attribute__((aligned(16))) float xs0[XN];
  __shared__ __attribute__((aligned(16))) float xs1[XDBL ? XN : TB * TK];  // NW = 4: partial sums
  static_assert(32 * TPL <= XN && TB * TK <= U_IMG && 32 * TPL <= U_IMG, "epilogue buffers");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int n_k = p.K / TK;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = tile % n_k, k0 = kb * TK;
  const int blk_p = tile / n_k;
  const int t0 = blk_p * TBR;
  const int b0 = t0 / TI;
  const int grp = wave % NG, nh = wave / NG;

  const i32x4v urs = raw_rsrc(p.u, (unsigned)((long long)(p.C / 8) * n_k * U_IMG * 4));
  const i32x4v xrs = raw_rsrc(p.x, (unsigned)(p.x_elems * 4));

  const int tib = grp * 16 + j;
  int sbase;
  if constexpr (BAND) {
    const int sl = tib < TBR ? tib : 0;  // padding MFMA rows read tile 0's patch (results dropped)
    sbase = (sl / TPR) * 6 * G::RWP + 5 * (sl % TPR);
  } else {
    const int il = tib / TI, ti = tib - il * TI, tr = ti / TPR, tc = ti - tr * TPR;
    sbase = S == 4 ? il * G::IP : il * G::IP + 4 * tr * G::RWP + (G::PAD ? 5 : 4) * tc;
  }
  const int poff = ((g >> 1) * PL + sbase) * 4 + (g & 1) * 2;  // plane g/2, channels 2g, 2g+1

  // X DMA sources, 16 bits per instruction: pixel index relative to the block's first image (11
  // bits), plane (1), valid (1); the byte offset is rebuilt at issue (3 VALU) — half the registers
  // (band geometry: 32-bit codes — valid bit 31, plane bit 30, pixel index from the block's first
  // image in bits 0-29)
  unsigned xcode[BAND ? KX : (KX + 1) / 2];
#pragma unroll
  for (int i = 0; i < (BAND ? KX : (KX + 1) / 2); ++i) xcode[i] = 0u;
#pragma unroll
  for (int i = 0; i < KX; ++i) {
    const int slot = (wave + NW * i) * 64 + lane;
    const int h = slot / PL, s = slot - h * PL;
    if constexpr (BAND) {
      const int row = s / G::RWP, colp = s - row * G::RWP;
      const int bi = row / 6, rr = row - bi * 6;
      const int blk5 = colp / 5, w5 = colp - blk5 * 5;
      const int xx = 4 * blk5 + w5 - 1;
      const int gr = blk_p * Band<S>::BR + bi;  // global tile row
      const int b = gr / TPR, tr = gr - b * TPR;
      const int yy = 4 * tr - 1 + rr;
      const bool ok = h < 2 && bi < Band<S>::BR && w5 != 4 && xx >= 0 && xx < S && yy >= 0 && yy < S && b < p.B;
      xcode[i] = ok ? 0x80000000u | ((unsigned)h << 30) | (unsigned)(((b - b0) * S + yy) * S + xx) : 0u;
      continue;
    }
    const int im = s / G::IP, rem = s - im * G::IP;
    int xx, yy;
    bool ok;
    if constexpr (S == 4) {
      yy = rem / 4;
      xx = rem - yy * 4;
      ok = rem < 16;
    } else {
      const int row = rem / G::RWP, colp = rem - row * G::RWP;
      int w5 = 0;
      if constexpr (G::PAD) {
        const int blk5 = colp / 5;
        w5 = colp - blk5 * 5;
        xx = 4 * blk5 + w5 - 1;
      } else {
        xx = colp - 1;
      }
      yy = row - 1 + (S == 32 && TB == 32 ? 16 * (blk_p & 1) : 0);
      ok = w5 != 4 && row < G::RH && xx >= 0 && xx < S && yy >= 0 && yy < S;
    }
    ok = ok && h < 2 && im < G::NI && b0 + im < p.B;
    const unsigned code = ok ? (unsigned)((im * S + yy) * S + xx) | ((unsigned)h << 11) | 0x1000u : 0u;
    xcode[i >> 1] |= code << (16 * (i & 1));
  }
  static_assert(BAND || G::NI * S * S <= 2048, "X pixel code");
  const unsigned xbase = (unsigned)b0 * S * S * (unsigned)p.C * 4u;
  const unsigned lane16 = (unsigned)lane * 16u;
  const unsigned c4 = (unsigned)p.C * 4u;

  // U half hf (18 point pairs = 18 wave-instructions) of chunk c0/8
  auto stage_u = [&](int c0, int hf) {
    if (p.dbg & 1) return;
    const unsigned ub = (unsigned)(((c0 >> 3) * n_k + kb) * U_IMG) * 4u;
#pragma unroll
    for (int i = 0; i < (18 + NW - 1) / NW; ++i) {
      const int pt = wave + NW * i;
      if (pt < 18) {
        const int q = hf * 18 + pt;
        dma16_asm(urs, lds_addr(us + q * 256), lane16, ub + (unsigned)q * 1024u);  // point pair q: soffset
      }
    }
  };
  auto stage_x = [&](int c0, float* xd) {
    if (p.dbg & 2) return;
#pragma unroll
    for (int i = 0; i < KX; ++i)
      if (wave + NW * i < NXI) {
        unsigned off;
        if constexpr (BAND) {
          const unsigned code = xcode[i];
          off = (code >> 31) ? xbase + (code & 0x3fffffffu) * c4 + ((code >> 26) & 16u) : OOB;
        } else {
          const unsigned code = xcode[i >> 1] >> (16 * (i & 1));
          off = (code & 0x1000u) ? xbase + (code & 0x7ffu) * c4 + ((code >> 7) & 16u) : OOB;
        }
        dma16_asm(xrs, lds_addr(xd + (wave + NW * i) * 256), off, (unsigned)c0 * 4u);
      }
  };
  auto stage_u_piece = [&](int c0, int hf, int i) {  // piece i of stage_u
    if (p.dbg & 1) return;
    const int pt = wave + NW * i;
    if (pt < 18) {
      const unsigned ub = (unsigned)(((c0 >> 3) * n_k + kb) * U_IMG) * 4u;
      const int q = hf * 18 + pt;
      dma16_asm(urs, lds_addr(us + q * 256), lane16, ub + (unsigned)q * 1024u);
    }
  };

  // split-K over channel chunks: blockIdx.y owns chunks [c_lo, c_hi) (host: no empty split)
  const int nc_all = p.C / 8, cps = (nc_all + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c_lo = (int)blockIdx.y * cps, nc = min(nc_all, c_lo + cps);
  f32x4 acc[NPT];
#pragma unroll
  for (int x = 0; x < NPT; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
  // SPLITP: nh is the wave's point half (rows 3nh..3nh+2 of the 6x6 grid); it reads both channel halves
  const float* ul = us + (SPLITP ? 0 : nh * 128) + j * 8 + 2 * (g ^ ((j >> 3) << 1));
  const bool full_x = (NXI - wave + NW - 1) / NW == KX;  // this wave issues KX (else KX - 1) X DMAs
  // Wait until at most this wave's X DMAs of one chunk (issued last) are in flight
  auto wait_but_x = [&]() {
    if (full_x) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KX) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KX - 1) : "memory");
  };

  // prologue: X(0) (and X(1)), U0(0) in flight
  stage_x(8 * c_lo, xs0);
  if (XDBL && c_lo + 1 < nc) stage_x(8 * (c_lo + 1), xs1);
  stage_u(8 * c_lo, 0);
  for (int c = c_lo; c < nc; ++c) {
    float* xb = (XDBL && ((c - c_lo) & 1)) ? xs1 : xs0;  // X(c)
    // top: U0(c) and X(c) landed everywhere (NW = 8: X(c+1), issued after U0(c), may still be in
    // flight); every wave is done with U1(c-1)
    if (XDBL && c + 1 < nc && c > c_lo) wait_but_x();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    stage_u(8 * c, 1);
    if constexpr (SPLITP) {
      f2v w[18];
      if (nh == 0) sp_read_transform<S, G, 0>(xb + poff, w);  // wave-uniform branch
      else sp_read_transform<S, G, 1>(xb + poff, w);
      if constexpr (!XDBL) {
        lds_barrier();  // every wave has its patch: X(c+1) into the single buffer
        if (c + 1 < nc) stage_x(8 * (c + 1), xs0);
      }
      sp_mfma_chunk(c, nc, w, ul, acc, [&]() {
        if (!XDBL && c + 1 < nc) wait_but_x();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (c + 1 < nc) stage_u(8 * (c + 1), 0);
        if (XDBL && c + 2 < nc) stage_x(8 * (c + 2), xb);
      }, nh);
      continue;
    }
    f2v v[36];
    {
      const float* p0 = xb + poff;
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          f2v d = {0.f, 0.f};
          if constexpr (S == 4) {
            if (r >= 1 && r <= 4 && q >= 1 && q <= 4) d = *reinterpret_cast<const f2v*>(p0 + ((r - 1) * 4 + (q - 1)) * 4);
          } else {
            d = *reinterpret_cast<const f2v*>(p0 + (r * G::RWP + q + (G::PAD && q >= 4 ? 1 : 0)) * 4);
          }
          v[r * 6 + q] = d;
          __builtin_amdgcn_sched_barrier(0);  // one ds_read_b64 each (no ds_read2 merging)
        }
    }
    if constexpr (!XDBL) {  // every wave has its patch: X(c+1) into the single buffer
      lds_barrier();
      if (c + 1 < nc) stage_x(8 * (c + 1), xs0);
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) bt6p(v[q], v[6 + q], v[12 + q], v[18 + q], v[24 + q], v[30 + q]);
#pragma unroll
    for (int r = 0; r < 6; ++r) bt6p(v[6 * r], v[6 * r + 1], v[6 * r + 2], v[6 * r + 3], v[6 * r + 4], v[6 * r + 5]);
    float2 wq[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (e == 1) {
        // U1(c) landed everywhere (NW = 4: X(c+1), issued after it, may still be in flight);
        // every wave is done with U0(c) (and NW = 8: X(c))
        if (!XDBL && c + 1 < nc) wait_but_x();
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (!SPREAD && c + 1 < nc) stage_u(8 * (c + 1), 0);
        if (XDBL && c + 2 < nc) stage_x(8 * (c + 2), xb);
      }
      const float* ue = ul + e * 18 * 256;
      wq[0] = *reinterpret_cast<const float2*>(ue);
      __builtin_amdgcn_sched_barrier(0);
      wq[1] = *reinterpret_cast<const float2*>(ue + 256);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 18; ++i) {
        const float2 w = wq[i & 1];
        if (i + 2 < 18) {
          wq[i & 1] = *reinterpret_cast<const float2*>(ue + (i + 2) * 256);
          __builtin_amdgcn_sched_barrier(0);
        }
        const int x = 2 * i;
        if constexpr (SPREAD) {
          const float a0 = e ? v[x].y : v[x].x, a1 = e ? v[x + 1].y : v[x + 1].x;
          if (i == 0) W4_MFMA2("s_nop 1\n\t", acc[x], acc[x + 1], a0, a1, w);
          else W4_MFMA2("", acc[x], acc[x + 1], a0, a1, w);
          if (e == 1 && c + 1 < nc && (i & 1) == 0 && i / 2 < (18 + NW - 1) / NW)
            stage_u_piece(8 * (c + 1), 0, i / 2);  // U0(c+1), one piece per two parity-1 steps
        } else {
          acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(e ? v[x].y : v[x].x, w.x, acc[x], 0, 0, 0);
          acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(e ? v[x + 1].y : v[x + 1].x, w.y, acc[x + 1], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if constexpr (SPREAD) asm volatile("s_nop 15" ::: "memory");  // inline-asm MFMA results -> epilogue reads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (p.dbg & 16) {
    float t = 0.f;
#pragma unroll
    for (int x = 0; x < NPT; ++x) t += acc[x][0];
    if (t == 1234.5f) p.out[0] = t;
    return;
  }
  if constexpr (XDBL) epilogue<EPI, S, 8>(p, *reinterpret_cast<f32x4(*)[1][NPT]>(&acc), t0, k0, xs0, xs1, us);
  else epilogue<EPI, S, 4, 1, SPLITP>(p, *reinterpret_cast<f32x4(*)[1][NPT]>(&acc), t0, k0, us, xs0, xs1);
}

// U = G g G^T into the LDS images: layout 0 (MODE 0/1): word ((x*2 + nh)*16 + j)*8 + 2*(g ^ 2*(j >> 3)) + e
// of image (cb, kb) holds U[x][c = 8cb + 2g + e][k = 32kb + 16nh + j]; layout 1 (MODE 2): word
// (((e*18 + x/2)*2 + nh)*16 + j)*8 + 2*(g ^ 2*(j >> 3)) + (x & 1) holds U[x][c = 8cb + 2g + e][k]. fp64, rounded once. flip_t: the
// data-gradient operand (w'[k][c] = w[c][k], taps rotated 180 degrees).
__device__ __forceinline__ void weight_transform_one(long long t, const float* __restrict__ w, float* __restrict__ u,
                                                     int K, int C, int flip_t, int S0, int S1, int lay, long long st0,
                                                     long long st1, int st2, int st3) {
  // one thread per (c, k): its 9 taps are read once and all 36 points formed with compile-time G
  // indices (the per-point version re-read the taps 36x and indexed G at run time); same fp64
  // products and summation order per point as before, so the same rounded U
  constexpr double Gm[6][3] = {{0.25, 0.0, 0.0},
                               {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                               {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                               {1.0 / 24, 1.0 / 12, 1.0 / 6},
                               {1.0 / 24, -1.0 / 12, 1.0 / 6},
                               {0.0, 0.0, 1.0}};
  // lanes enumerate (g slot, j) of one (e, nh) so that for each point a wave's 64 stores land in
  // one 128-word span of the image (stride 2) instead of 8 words apart
  const int gs_ = (int)(t & 3), j_ = (int)((t >> 2) & 15), e_ = (int)((t >> 6) & 1), nh_ = (int)((t >> 7) & 1);
  const long long rest = t >> 8;
  const int kb_ = (int)(rest % (K / TK)), cb_ = (int)(rest / (K / TK));
  const int c = 8 * cb_ + 2 * (gs_ ^ ((j_ >> 3) << 1)) + e_, k = TK * kb_ + 16 * nh_ + j_;
  const int r0 = flip_t ? c : k, r1 = flip_t ? k : c;
  const bool ok = r0 < S0 && r1 < S1;
  double wv[9];
  // w's element strides st0..st3 (a channels_last parameter is read in place)
  const float* src = w + (ok ? r0 : 0) * st0 + (ok ? r1 : 0) * st1;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int tt = flip_t ? 8 - tap : tap;
    wv[tap] = ok ? (double)src[(tt / 3) * st2 + (tt % 3) * st3] : 0.0;
  }
  const int cb = c >> 3, cc = c & 7, g = cc >> 1, e = cc & 1;
  const int kb = k / TK, kk = k - kb * TK, nh = kk >> 4, j = kk & 15;
  const int gs = g ^ ((j >> 3) << 1);
  float* dst = u + ((long long)cb * (K / TK) + kb) * U_IMG + (nh << 7) + (j << 3) + (gs << 1);
#pragma unroll
  for (int x = 0; x < NPT; ++x) {
    const int i = x / 6, jj = x % 6;
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) acc += Gm[i][a] * wv[a * 3 + b] * Gm[jj][b];
    const int hi = lay ? e * 18 + x / 2 : x, lo = lay ? (x & 1) : e;
    dst[(hi << 8) + lo] = (float)acc;
  }
}

__global__ __launch_bounds__(256) void weight_transform(const float* __restrict__ w, float* __restrict__ u, int K, int C,
                                                        int flip_t, int S0, int S1, int lay, long long st0,
                                                        long long st1, int st2, int st3) {
  const long long total = (long long)C * K;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x)
    weight_transform_one(t, w, u, K, C, flip_t, S0, S1, lay, st0, st1, st2, st3);
}

// Every U image set of a training step in one launch: descriptor d (W4_DESC int64: w, u, start,
// K, C, flip_t, S0, S1, st0, st1, st2, st3), starts multiples of 256 (C*K is: C % 8, K % 32), so
// a block's 256 (c, k) threads all belong to one operand (block-uniform descriptor search).
constexpr int W4_DESC = 12;
__global__ __launch_bounds__(256) void weight_transform_multi(const long long* __restrict__ desc, int n,
                                                              long long total, int lay) {
  for (long long blk = blockIdx.x; blk * 256 < total; blk += gridDim.x) {
    const long long base = blk * 256;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (desc[mid * W4_DESC + 2] <= base) lo = mid;
      else hi = mid - 1;
    }
    const long long* d = desc + lo * W4_DESC;
    weight_transform_one(base - d[2] + threadIdx.x, reinterpret_cast<const float*>(d[0]), reinterpret_cast<float*>(d[1]),
                         (int)d[3], (int)d[4], (int)d[5], (int)d[6], (int)d[7], lay, d[8], d[9], (int)d[10],
                         (int)d[11]);
  }
}

// TP_W4_MODE (read once): 2 packed transforms, one 8-wave block per CU; 3 (default) packed
// transforms, two 4-wave blocks per CU (the blocks' barriers are independent, so one block's patch
// reads / transform run under the other's MFMAs: 1.3x MODE 2). The round-3 MODE 0/1 prototypes and
// the WIDE kernel were measured slower and removed (profiles/wino4/).
static int kernel_mode() {
  static const int mode = [] {
    const char* m = getenv("TP_W4_MODE");
    return m && atoi(m) == 2 ? 2 : 3;
  }();
  return mode;
}

}  // namespace w4
}  // namespace tp

// U images of a 3x3 weight for wino4: (C/8, K/32, 9216) floats. w: (S0, S1, 3, 3) = the forward
// weight (Cout, Cin, 3, 3), possibly narrower than the padded GEMM; flip_t as tp_wino_weights2.
// strides: w's element strides (st0, st1, st2, st3) — (S1*9, 9, 3, 1) when contiguous
extern "C" hipError_t tp_wino4_weights_strided(const float* w, float* u, int K, int C, int flip_t, int S0, int S1,
                                               long long st0, long long st1, int st2, int st3, hipStream_t st) {
  if (K % 32 || C % 8 || K <= 0 || C <= 0 || S0 <= 0 || S1 <= 0) return hipErrorInvalidValue;
  if (flip_t ? (S0 > C || S1 > K) : (S0 > K || S1 > C)) return hipErrorInvalidValue;
  if (st0 <= 0 || st1 <= 0 || st2 <= 0 || st3 <= 0) return hipErrorInvalidValue;
  const long long total = (long long)C * K;  // one thread per (input, output channel) pair
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 16384);
  tp::w4::weight_transform<<<grid, 256, 0, st>>>(w, u, K, C, flip_t, S0, S1, 1, st0, st1,
                                                 st2, st3);
  return hipGetLastError();
}

// desc: n descriptors of W4_DESC int64 on the device (validated by the binding against live
// tensors), starts ascending in (c, k) threads: start[i+1] = start[i] + C_i * K_i
extern "C" hipError_t tp_wino4_weights_multi(const long long* desc, int n, long long total, hipStream_t st) {
  if (n <= 0 || total <= 0 || total % 256) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)std::min<long long>(total / 256, 16384);
  tp::w4::weight_transform_multi<<<grid, 256, 0, st>>>(desc, n, total, 1);
  return hipGetLastError();
}

extern "C" hipError_t tp_wino4_weights(const float* w, float* u, int K, int C, int flip_t, int S0, int S1,
                                       hipStream_t st) {
  return tp_wino4_weights_strided(w, u, K, C, flip_t, S0, S1, (long long)S1 * 9, 9, 3, 1, st);
}

extern "C" int tp_wino4_u_img() { return tp::w4::U_IMG; }

// square map sizes served by the band geometry (split-points kernel only): ResNet's 3x3 stride-1 maps
static bool wino4_band_size(int S) { return S == 56 || S == 28 || S == 14 || S == 7; }

extern "C" int tp_wino4_ok(int H, int W, int C, int K) {
  return H == W && (H == 4 || H == 8 || H == 16 || H == 32 || wino4_band_size(H)) && C % 8 == 0 && C >= 8 &&
         K % 32 == 0 && K >= 32;
}

// Taylor partial slots (R of the (R, B, K) slab) a wino4 data gradient writes at S x S maps
extern "C" int tp_wino4_taylor_slots(int S) {
  using namespace tp::w4;
  switch (S) {
    case 56: return Band<56>::R;
    case 28: return Band<28>::R;
    case 14: return Band<14>::R;
    case 7: return Band<7>::R;
    case 32: return 2;
    default: return 1;
  }
}

// F(4x4,3x3) conv, S x S maps. epi: 0 fwd (BN affine + ReLU), 1 fwd + 2x2 max-pool (+ argmax),
// 2 dgrad epilogue (x = output gradient, act / scale / taylor as conv_wino). apoz (fwd) and taylor
// (dgrad, slot 0 of the (R, B, K) slab) are summed per (image, channel) with one writer each (+=).
// splits > 1 (MODE 2/3): the channel chunks are split over gridDim.y blocks that write raw slabs
// into ws (splits x M x K floats; pooled row order for epi 1), combined in a fixed order by the
// shared split-K epilogue (conv_mfma.hip) — small batches get enough blocks to fill the chip.
extern "C" hipError_t tp_conv_epilogue_slabs(const float* ws, int splits, int B, int H, int W, int K, int epi,
                                              const float* scale, const float* shift, int relu, float* out,
                                              uint8_t* out_argmax, const float* act, float* taylor,
                                              float* apoz, int tay_mode, hipStream_t st);

// variant 0: the TP_W4_MODE kernel (default MODE 3); variant 2: MODE 3 with spread U DMA;
// variant 3: MODE 3 with split points (each wave 18 points x 32 outputs, half the transform).
// ko (0 = K): output channels stored per pixel (K rounded down to them: ko % 4 == 0, K - 32 < ko <=
// K): the U images and the MFMAs cover K = ko rounded up to 32, the outputs, activations, BN
// scale / shift, Taylor / APoZ slabs have ko channels — pruned widths stay unpadded in HBM.
extern "C" hipError_t tp_conv_wino4_ko(const float* x, const float* u, int B, int S, int C, int K, int epi,
                                       const float* scale, const float* shift, int relu, float* out,
                                       uint8_t* out_argmax, const float* act, float* taylor, float* apoz, int tay_mode,
                                       int splits, float* ws, int variant, hipStream_t st, const uint8_t* unpool_am,
                                       int ko) {
  using namespace tp::w4;
  if (!tp_wino4_ok(S, S, C, K) || B <= 0) return hipErrorInvalidValue;
  if (ko == 0) ko = K;
  if (ko % 4 || ko > K || ko <= K - TK) return hipErrorInvalidValue;
  // band geometry (56 / 28 / 14 / 7-pixel maps): the split-points kernel, no pooling / unpooling
  const bool band = wino4_band_size(S);
  if (band && (variant != 3 || epi == FWD_POOL || unpool_am)) return hipErrorInvalidValue;
  const int nc = C / 8;
  splits = std::max(1, std::min(splits, nc));
  splits = (nc + (nc + splits - 1) / splits - 1) / ((nc + splits - 1) / splits);  // no empty split
  if (variant < 0 || variant > 3 || variant == 1) return hipErrorInvalidValue;
  if (splits > 1 && (!ws || ko != K)) return hipErrorInvalidValue;  // the slab combine writes K-wide rows
  if (epi < 0 || epi > 2 || (epi == BWD && !act) || (epi != BWD && !out) || (epi == FWD_POOL && !out_argmax))
    return hipErrorInvalidValue;
  // fused unpooling: the data gradient's full-resolution output, one K pass (the split-K combine
  // writes pooled rows)
  if (unpool_am && (epi != BWD || !out || splits > 1 || 2ll * B * 2 * S * 2 * S * K >= (1ll << 31)))
    return hipErrorInvalidValue;
  Args a{};
  a.x = x;
  a.u = u;
  a.B = B;
  a.C = C;
  a.K = K;
  a.ko = ko;
  const int tpr = (S + 3) / 4;
  a.P = B * tpr * tpr;
  a.x_elems = (long long)B * S * S * C;
  if (a.x_elems * 4 >= (1ll << 31) || (long long)(C / 8) * (K / 32) * U_IMG * 4 >= (1ll << 31))
    return hipErrorInvalidValue;
  if (epi == BWD && (long long)B * S * S * K * 4 >= (1ll << 31)) return hipErrorInvalidValue;
  a.scale = scale;
  a.shift = shift;
  a.relu = relu;
  a.out = out;
  a.out_argmax = out_argmax;
  a.act = act;
  a.taylor = epi == BWD ? taylor : nullptr;
  a.apoz = epi == BWD ? nullptr : apoz;
  a.tay_mode = tay_mode;
  a.unp = unpool_am;
  static const int dbg = [] {
    const char* d = getenv("TP_W4_DBG");
    const int v = d ? atoi(d) : 0;
    if (v) fprintf(stderr, "[tpamd] WARNING: TP_W4_DBG=%d: F(4x4) results are WRONG (phase-cost experiment)\n", v);
    return v;
  }();
  a.dbg = dbg;
  // 5: MODE 3 with SPREAD DMA; 6: MODE 3 with split points
  const int mode = variant == 2 ? 5 : variant == 3 ? 6 : kernel_mode();
  const int tb = mode == 2 ? 64 : TILES;  // MODE 3: 32-tile blocks
  const int br = band ? 32 / tpr : 0;     // band: whole tile rows per block
  const int n_p = band ? (B * tpr + br - 1) / br : (a.P + tb - 1) / tb, n_k = K / TK;
  const dim3 grid(n_p * n_k, splits);
  if (splits > 1) {
    Args b = a;
    b.out = ws;
    b.out_argmax = nullptr;
    b.act = nullptr;
    b.taylor = nullptr;
    b.apoz = nullptr;
    b.scale = nullptr;
    b.shift = nullptr;
    b.slab = (long long)B * S * S * K;
    b.pool_order = epi == FWD_POOL;
    if (b.slab * splits >= (1ll << 31)) return hipErrorInvalidValue;
    if (band) {
      if (S == 56) wino4_m2<PARTIAL, 56, 4, false, true><<<grid, 256, 0, st>>>(b);
      else if (S == 28) wino4_m2<PARTIAL, 28, 4, false, true><<<grid, 256, 0, st>>>(b);
      else if (S == 14) wino4_m2<PARTIAL, 14, 4, false, true><<<grid, 256, 0, st>>>(b);
      else wino4_m2<PARTIAL, 7, 4, false, true><<<grid, 256, 0, st>>>(b);
    } else {
#define TP_W4P(SS)                                                                      \
  do {                                                                                  \
    if (mode == 6) wino4_m2<PARTIAL, SS, 4, false, true><<<grid, 256, 0, st>>>(b);      \
    else if (mode == 5) wino4_m2<PARTIAL, SS, 4, true><<<grid, 256, 0, st>>>(b);        \
    else if (mode == 2) wino4_m2<PARTIAL, SS, 8><<<grid, 512, 0, st>>>(b);              \
    else wino4_m2<PARTIAL, SS, 4><<<grid, 256, 0, st>>>(b);                             \
  } while (0)
      if (S == 32) TP_W4P(32);
      else if (S == 16) TP_W4P(16);
      else if (S == 8) TP_W4P(8);
      else TP_W4P(4);
#undef TP_W4P
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return tp_conv_epilogue_slabs(ws, splits, B, S, S, K, epi, scale, epi == BWD ? nullptr : shift, relu, out,
                                  out_argmax, act, epi == BWD ? taylor : nullptr, epi == BWD ? nullptr : apoz,
                                  tay_mode, st);
  }
#define TP_W4(E, SS)                                                             \
  do {                                                                           \
    if (mode == 6) wino4_m2<E, SS, 4, false, true><<<grid, 256, 0, st>>>(a);     \
    else if (mode == 5) wino4_m2<E, SS, 4, true><<<grid, 256, 0, st>>>(a);       \
    else if (mode == 2) wino4_m2<E, SS, 8><<<grid, 512, 0, st>>>(a);             \
    else wino4_m2<E, SS, 4><<<grid, 256, 0, st>>>(a);                            \
  } while (0)
#define TP_W4S(E)                   \
  do {                              \
    if (S == 32) TP_W4(E, 32);      \
    else if (S == 16) TP_W4(E, 16); \
    else if (S == 8) TP_W4(E, 8);   \
    else TP_W4(E, 4);               \
  } while (0)
#define TP_W4B(E)                                                                \
  do {                                                                           \
    if (S == 56) wino4_m2<E, 56, 4, false, true><<<grid, 256, 0, st>>>(a);       \
    else if (S == 28) wino4_m2<E, 28, 4, false, true><<<grid, 256, 0, st>>>(a);  \
    else if (S == 14) wino4_m2<E, 14, 4, false, true><<<grid, 256, 0, st>>>(a);  \
    else wino4_m2<E, 7, 4, false, true><<<grid, 256, 0, st>>>(a);                \
  } while (0)
  if (band) {
    if (epi == FWD) TP_W4B(FWD);
    else TP_W4B(BWD);
    return hipGetLastError();
  }
#undef TP_W4B
  if (epi == FWD) TP_W4S(FWD);
  else if (epi == FWD_POOL) TP_W4S(FWD_POOL);
  else TP_W4S(BWD);
#undef TP_W4S
#undef TP_W4
  return hipGetLastError();
}

extern "C" hipError_t tp_conv_wino4(const float* x, const float* u, int B, int S, int C, int K, int epi,
                                    const float* scale, const float* shift, int relu, float* out, uint8_t* out_argmax,
                                    const float* act, float* taylor, float* apoz, int tay_mode, int splits,
                                    float* ws, int variant, hipStream_t st, const uint8_t* unpool_am) {
  return tp_conv_wino4_ko(x, u, B, S, C, K, epi, scale, shift, relu, out, out_argmax, act, taylor, apoz, tay_mode,
                          splits, ws, variant, st, unpool_am, K);
}

// static LDS bytes of a wino4 instantiation (occupancy / budget guard)
extern "C" int tp_wino4_lds_bytes(int S, int variant) {
  using namespace tp::w4;
  const int m = variant >= 2 ? 3 : kernel_mode();
  const void* f = nullptr;
  if (wino4_band_size(S)) {
    f = S == 56 ? (const void*)wino4_m2<BWD, 56, 4, false, true>
        : S == 28 ? (const void*)wino4_m2<BWD, 28, 4, false, true>
        : S == 14 ? (const void*)wino4_m2<BWD, 14, 4, false, true>
                  : (const void*)wino4_m2<BWD, 7, 4, false, true>;
  } else {
#define TP_W4F(SS) f = m == 2 ? (const void*)wino4_m2<BWD, SS, 8> : (const void*)wino4_m2<BWD, SS, 4>
    if (S == 32) TP_W4F(32);
    else if (S == 16) TP_W4F(16);
    else if (S == 8) TP_W4F(8);
    else TP_W4F(4);
#undef TP_W4F
  }
  hipFuncAttributes at{};
  if (hipFuncGetAttributes(&at, f) != hipSuccess) return -1;
  return (int)at.sharedSizeBytes;
}
