// Micro-benchmark: fp32 MFMA (16x16x4) issue rate with and without interleaved VALU work, 1 or 2
// waves per SIMD, to calibrate the F(4x4) kernel's schedule. Prints TFLOP/s of MFMA work per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV, int NACC>
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, float s) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = s;
  float t[8];
  for (int i = 0; i < 8; ++i) t[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int x = 0; x < NACC; x += 2) {
      acc[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[x], 0, 0, 0);
      acc[x + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc[x + 1], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < NV; ++v) t[v & 7] = fmaf(t[v & 7], 1.0001f, t[(v + 3) & 7]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float r = 0.f;
  for (int i = 0; i < NACC; ++i) r += acc[i][0] + acc[i][3];
  for (int i = 0; i < 8; ++i) r += t[i];
  if (r == 1.2345f) out[threadIdx.x] = r;
}

template <int NV, int NACC>
void run(int threads, const char* name) {
  float* out;
  hipMalloc(&out, 4096);
  const int blocks = 256, iters = 2000;
  hipLaunchKernelGGL((k<NV, NACC>), dim3(blocks), dim3(threads), 0, 0, out, 10, 1.f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<NV, NACC>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2048.0 * NACC * iters * (threads / 64) * blocks;
  printf("%-34s threads=%d  %.3f ms  %.1f TF/s MFMA  (%.1f VALU/MFMA)\n", name, threads, ms, flop / ms / 1e9, NV / 2.0);
  hipFree(out);
}

int main() {
  run<0, 36>(256, "mfma only, 1 wave/SIMD");
  run<0, 36>(512, "mfma only, 2 waves/SIMD");
  run<4, 36>(256, "mfma + 2 valu/mfma, 1 wave/SIMD");
  run<4, 36>(512, "mfma + 2 valu/mfma, 2 waves/SIMD");
  run<8, 36>(256, "mfma + 4 valu/mfma, 1 wave/SIMD");
  run<8, 36>(512, "mfma + 4 valu/mfma, 2 waves/SIMD");
  run<14, 36>(256, "mfma + 7 valu/mfma, 1 wave/SIMD");
  run<14, 36>(512, "mfma + 7 valu/mfma, 2 waves/SIMD");
  run<28, 36>(512, "mfma + 14 valu/mfma, 2 waves/SIMD");
  return 0;
}
