// Device-side data pipeline for real datasets (reference experiments/models/cifar10.py:102-161,
// mnist.py:62-82): the whole uint8 dataset lives in HBM (CIFAR-10 train = 150 MB of 288 GB) and
// one kernel per batch gathers the batch's images, applies the training augmentation
// (RandomHorizontalFlip -> RandomCrop(H, padding) with zero fill, torchvision order) and
// ToTensor + Normalize, writing the fp32 NCHW batch the model consumes. The reference runs
// this per image on a host DataLoader worker (num_workers=1).
#include "tp_common.h"

namespace tp {

// out[b, c, h, w] = (pix / 255 - mean[c]) * inv_std[c], pix = src[idx[b], c, r, q] with
//   r = h + aug[b].dy - pad, qf = w + aug[b].dx - pad, q = aug[b].flip ? W - 1 - qf : qf
// and pix = 0 (torchvision's zero padding, before normalisation) outside the image.
__global__ __launch_bounds__(256) void augment_u8(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx,
                                                  const int* __restrict__ aug, int B, int C, int H, int W, int pad,
                                                  const float* __restrict__ mean, const float* __restrict__ inv_std,
                                                  float* __restrict__ out) {
  const long long total = (long long)B * C * H * W;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(t % W);
    long long r_ = t / W;
    const int h = (int)(r_ % H);
    r_ /= H;
    const int c = (int)(r_ % C);
    const int b = (int)(r_ / C);
    int dy = pad, dx = pad, flip = 0;  // no augmentation: the centred (identity) crop
    if (aug) {
      dy = aug[3 * b];
      dx = aug[3 * b + 1];
      flip = aug[3 * b + 2];
    }
    const int r = h + dy - pad, qf = w + dx - pad;
    float v = 0.f;
    if (r >= 0 && r < H && qf >= 0 && qf < W) {
      const int q = flip ? W - 1 - qf : qf;
      v = (float)src[((idx[b] * C + c) * H + r) * (long long)W + q] * (1.f / 255.f);
    }
    out[t] = (v - mean[c]) * inv_std[c];
  }
}

}  // namespace tp

extern "C" hipError_t tp_augment_u8(const uint8_t* src, const int64_t* idx, const int* aug, int B, int C, int H, int W,
                                    int pad, const float* mean, const float* inv_std, float* out, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (pad < 0 || C <= 0 || H <= 0 || W <= 0) return hipErrorInvalidValue;
  const long long total = (long long)B * C * H * W;
  const unsigned grid = (unsigned)std::min<long long>(tp::ceil_div(total, 256), 16384);
  tp::augment_u8<<<grid, 256, 0, st>>>(src, idx, aug, B, C, H, W, pad, mean, inv_std, out);
  return hipGetLastError();
}
