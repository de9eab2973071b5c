// Micro-benchmark: cycles per MFMA of the bf16 shapes the Winograd kernels can use on gfx950 —
// v_mfma_f32_16x16x16_bf16 (4 bf16 per lane) vs v_mfma_f32_16x16x32_bf16 (8 per lane) vs the fp32
// v_mfma_f32_16x16x4_f32 — one wave per SIMD, 8 independent accumulators, back-to-back issue.
// hipcc --offload-arch=gfx950 -O3 scripts/micro/mfma_bf16_rates.hip -o /tmp/mfma_bf16_rates
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters) {
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a = threadIdx.x * 1e-3f;
  s16x4 a4 = {1, 2, 3, 4};
  bf16x8 a8 = {};
  for (int i = 0; i < 8; ++i) a8[i] = (__bf16)(a + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      // inline asm with pinned AGPR accumulators: the builtins let the compiler shuffle the
      // accumulators through v_accvgpr moves inside the loop, which then dominate the timing
      if constexpr (KIND == 0) asm volatile("v_mfma_f32_16x16x16_bf16 %0, %1, %1, %0" : "+a"(acc[x]) : "v"(a4));
      else if constexpr (KIND == 1) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, %0" : "+a"(acc[x]) : "v"(a8));
      else asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %1, %0" : "+a"(acc[x]) : "v"(a));
    }
  }
  asm volatile("s_nop 15" ::: "memory");  // MFMA results readable
  float r = 0.f;
  for (int i = 0; i < 8; ++i) r += acc[i][0];
  if (r == 1.2345f) out[threadIdx.x] = r;
}

template <int KIND>
void run(const char* name) {
  float* out;
  hipMalloc(&out, 4096);
  const int blocks = 256, iters = 200000;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);  // clocks up
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // one wave per SIMD: per SIMD 8 * iters MFMAs; cycles at the measured clock are not known, so
  // report ns per MFMA per SIMD (x 2.4 GHz ~ cycles)
  const double ns = ms * 1e6 / (8.0 * iters);
  printf("%-28s %.2f ns per MFMA per SIMD (~%.1f cycles at 2.4 GHz)\n", name, ns, ns * 2.4);
  hipFree(out);
}

int main() {
  for (int rep = 0; rep < 2; ++rep) {
    run<2>("mfma_f32_16x16x4_f32");
    run<0>("mfma_f32_16x16x16_bf16");
    run<1>("mfma_f32_16x16x32_bf16");
  }
  return 0;
}
