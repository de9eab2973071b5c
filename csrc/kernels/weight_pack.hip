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

}  // namespace tp

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
