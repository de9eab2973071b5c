// Micro-benchmark: LDS read bandwidth per CU (bytes per shader clock) for ds_read_b32/b64/b128
// with 4 or 8 waves per block (one block per CU), conflict-free contiguous addressing.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int W>
__global__ void k(long long* out, float* sink, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = i;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    f4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int base = ((wave * 16 + r) * 64 * W + lane * W) & 16383;
      if (W == 1) v[r] = f4{lds[base], 0.f, 0.f, 0.f};
      else if (W == 2) { const float2 t = *reinterpret_cast<const float2*>(&lds[base]); v[r] = f4{t.x, t.y, 0.f, 0.f}; }
      else v[r] = *reinterpret_cast<const f4*>(&lds[base]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) acc += v[r][0] + v[r][1] + v[r][2] + v[r][3];
  }
  __syncthreads();
  const long long t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 1.234f) sink[threadIdx.x] = acc;
}

template <int W>
void run(int threads) {
  long long* out;
  float* sink;
  hipMalloc(&out, 8 * 256);
  hipMalloc(&sink, 4096);
  const int iters = 512;
  hipLaunchKernelGGL(k<W>, dim3(256), dim3(threads), 0, 0, out, sink, iters);
  hipDeviceSynchronize();
  long long c;
  hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
  const double bytes = (double)iters * 16 * (threads / 64) * 64 * 4 * W;
  printf("ds_read_b%-3d waves=%d  %.1f B/clk per CU\n", 32 * W, threads / 64, bytes / c);
  hipFree(out);
  hipFree(sink);
}

int main() {
  run<1>(256); run<2>(256); run<4>(256);
  run<1>(512); run<2>(512); run<4>(512);
  run<2>(1024); run<4>(1024);
  return 0;
}
