// Weight re-layout for the native training convolutions (engine/train.py): one launch per
// operand instead of the pad -> permute -> flip -> contiguous chains ATen needs (4-6 small
// copy kernels per conv and step, ~1.4 ms of a ResNet-50 training step in launch overhead).
//
// Source: the conv parameter w (O, I, KS, KS), contiguous, unpadded.
//   mode 0  forward GEMM operand  out[n < rows][k < cols], n = output channel,
//           k = (kh*KS + kw)*cpad + ci           -> w[n][ci][kh][kw]
//   mode 1  stride-1 data-gradient operand (flipped taps, transposed):
//           out[ci][k], k = (kh*KS + kw)*cpad + co -> w[co][ci][KS-1-kh][KS-1-kw]
//   mode 2  strided (transposed-gather) data-gradient operand, natural taps:
//           out[ci][k], k = (kh*KS + kw)*cpad + co -> w[co][ci][kh][kw]
// Every slot outside the real weight (padded channels, columns past KS*KS*cpad) is zero.
//
// pack_conv_weights_multi: every operand of a training step in ONE launch (engine/train.py
// _PackSet: all packs go stale together at the optimizer step). A descriptor per operand (int64
// x PACK_DESC: w, out, start, O, I, KS, rows, cols, cpad, mode, strides of w in elements — a
// channels_last parameter is read in place, no contiguous copy); a flat element space over the
// operands (start = chunk-aligned prefix offset), one descriptor search per 4096-element chunk.
#include "tp_common.h"

namespace tp {

__global__ __launch_bounds__(256) void pack_conv_weight(const float* __restrict__ w, float* __restrict__ out, int O,
                                                        int I, int KS, int rows, int cols, int cpad, int mode) {
  const long long total = (long long)rows * cols;
  const int taps = KS * KS;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(t / cols), k = (int)(t - (long long)r * cols);
    const int tap = k / cpad, c = k - tap * cpad;
    float v = 0.f;
    if (tap < taps) {
      int kh = tap / KS, kw = tap - kh * KS;
      const int co = mode == 0 ? r : c, ci = mode == 0 ? c : r;
      if (mode == 1) {
        kh = KS - 1 - kh;
        kw = KS - 1 - kw;
      }
      if (co < O && ci < I) v = w[(((long long)co * I + ci) * KS + kh) * KS + kw];
    }
    out[t] = v;
  }
}

constexpr int PACK_DESC = 14, PACK_CHUNK = 4096;  // operands start on PACK_CHUNK-element boundaries

// A block walks whole chunks; every element of a chunk belongs to one operand (aligned starts),
// so the descriptor search runs once per chunk (block-uniform) instead of once per element.
// Mode 0 operands: ceil(rows * cols / PACK_CHUNK) element chunks; modes 1 / 2: one chunk per
// (64-row ci tile, tap, 64-column co tile) — requires cols == KS * KS * cpad (the dgrad operands).
__global__ __launch_bounds__(256) void pack_conv_weights_multi(const long long* __restrict__ desc, int n,
                                                               long long total) {
  const long long chunks = (total + PACK_CHUNK - 1) / PACK_CHUNK;
  for (long long ch = blockIdx.x; ch < chunks; ch += gridDim.x) {
    const long long base = ch * PACK_CHUNK;
    int lo = 0, hi = n - 1;  // last descriptor with start <= base
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (desc[mid * PACK_DESC + 2] <= base) lo = mid;
      else hi = mid - 1;
    }
    const long long* d = desc + lo * PACK_DESC;
    const float* w = reinterpret_cast<const float*>(d[0]);
    float* out = reinterpret_cast<float*>(d[1]);
    const int O = (int)d[3], I = (int)d[4], KS = (int)d[5], rows = (int)d[6], cols = (int)d[7], cpad = (int)d[8];
    const int mode = (int)d[9];
    const long long s0 = d[10], s1 = d[11], s2 = d[12], s3 = d[13];
    const long long off = base - d[2];
    if (mode != 0) {  // data-gradient operands: one 64 (ci) x 64 (co) tile of one tap per chunk, through LDS
      // (out rows are ci, the weight's contiguous dim is co's neighbour ci: a direct per-element
      // copy read one 4-byte word per 64-byte line; the transpose makes both sides coalesced)
      __shared__ float tile[64][65];
      const int q = (int)(off / PACK_CHUNK), ct = (cpad + 63) / 64, taps = KS * KS;
      const int co_t = q % ct, tap = (q / ct) % taps, ci_t = q / (ct * taps);
      int kh = tap / KS, kw = tap - kh * KS;
      if (mode == 1) {
        kh = KS - 1 - kh;
        kw = KS - 1 - kw;
      }
      for (int e = threadIdx.x; e < PACK_CHUNK; e += blockDim.x) {
        const int lco = e >> 6, lci = e & 63, co = co_t * 64 + lco, ci = ci_t * 64 + lci;
        tile[lco][lci] = co < O && ci < I ? w[co * s0 + ci * s1 + kh * s2 + kw * s3] : 0.f;
      }
      __syncthreads();
      for (int e = threadIdx.x; e < PACK_CHUNK; e += blockDim.x) {
        const int lci = e >> 6, lco = e & 63, co = co_t * 64 + lco, ci = ci_t * 64 + lci;
        if (ci < rows && co < cpad) out[(long long)ci * cols + tap * cpad + co] = tile[lco][lci];
      }
      __syncthreads();
      continue;
    }
    const long long size = (long long)rows * cols;
    for (int e = threadIdx.x; e < PACK_CHUNK; e += blockDim.x) {
      const long long i = off + e;
      if (i >= size) break;
      const int r = (int)(i / cols), k = (int)(i - (long long)r * cols);
      const int tap = k / cpad, c = k - tap * cpad;
      float v = 0.f;
      if (tap < KS * KS) {
        int kh = tap / KS, kw = tap - kh * KS;
        const int co = mode == 0 ? r : c, ci = mode == 0 ? c : r;
        if (mode == 1) {
          kh = KS - 1 - kh;
          kw = KS - 1 - kw;
        }
        if (co < O && ci < I) v = w[co * s0 + ci * s1 + kh * s2 + kw * s3];
      }
      out[i] = v;
    }
  }
}

}  // namespace tp

// desc: n descriptors of PACK_DESC int64 on the device (pointers already validated by the
// caller: the binding checks every one against live tensors), starts ascending and multiples of
// PACK_CHUNK; total = the last start + its rows * cols
extern "C" hipError_t tp_pack_conv_weights_multi(const long long* desc, int n, long long total, hipStream_t st) {
  if (n <= 0 || total <= 0) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, (long long)tp::PACK_CHUNK), 8192);
  tp::pack_conv_weights_multi<<<grid, 256, 0, st>>>(desc, n, total);
  return hipGetLastError();
}

extern "C" hipError_t tp_pack_conv_weight(const float* w, float* out, int O, int I, int KS, int rows, int cols,
                                          int cpad, int mode, hipStream_t st) {
  if (O <= 0 || I <= 0 || KS <= 0 || rows <= 0 || cols <= 0 || cpad <= 0 || mode < 0 || mode > 2)
    return hipErrorInvalidValue;
  if ((mode == 0 && (rows < O || cpad < I)) || (mode != 0 && (rows < I || cpad < O))) return hipErrorInvalidValue;
  const long long total = (long long)rows * cols;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 8192);
  tp::pack_conv_weight<<<grid, 256, 0, st>>>(w, out, O, I, KS, rows, cols, cpad, mode);
  return hipGetLastError();
}
