// Micro-benchmark: cycles per LDS read instruction (one wave per CU) for the F(4x4) patch-read
// address patterns vs conflict-free baselines, to pin down the gfx950 LDS bank model.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ int pattern_addr(int pat, int lane) {  // float index
  const int j = lane & 15, g = lane >> 4;
  // S = 8 dense layout of MODE 2 (IP 101, RWP 10), tiles of wave group 0
  const int il = j >> 2, ti = j & 3, tr = ti >> 1, tc = ti & 1;
  const int s8 = il * 101 + 4 * tr * 10 + 4 * tc;
  // S = 16 padded layout (RWP 23): 16 tiles of one image
  const int tr16 = j >> 2, tc16 = j & 3;
  const int s16 = 4 * tr16 * 23 + 5 * tc16;
  const int PL = 1616;
  switch (pat) {
    case 0: return lane;                              // b32 contiguous
    case 1: return 2 * lane;                          // b64 contiguous
    case 2: return s8 * 4 + g;                        // b32, S=8 slot stride 16 B, channel g
    case 3: return ((g >> 1) * PL + s8) * 4 + (g & 1) * 2;  // b64, plane g/2, pair (g&1)
    case 4: return s16 * 4 + g;                       // b32 S=16
    case 5: return ((g >> 1) * 1656 + s16) * 4 + (g & 1) * 2;  // b64 S=16
    case 6: return j * 4 + g;                         // b32 slots 0..15 (ideal 16 distinct slots)
    case 7: return (j * 4 + g) * 2;                   // b64 lane-linear over 16 slots of 8 floats? (stride 32 B)
    case 8: return j * 8 + 2 * (g ^ ((j >> 3) << 1)); // b64 U-image read
    case 9: return lane * 4;                          // b32 stride 16 B (4-way conflict expected if 64 banks)
    default: return 0;
  }
}

template <int W>  // W = dwords per read (1 or 2)
__global__ __launch_bounds__(256) void k(int pat, long long* out, float* sink) {
  __shared__ float lds[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) lds[i] = i;
  __syncthreads();
  const int a = pattern_addr(pat, threadIdx.x & 63) + (threadIdx.x >> 6) * 4096;
  float acc = 0.f;
  const long long t0 = clock64();
#pragma unroll 1
  for (int it = 0; it < 256; ++it) {
    float v[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (W == 1) v[2 * r] = lds[(a + r * 256) & 16383], v[2 * r + 1] = 0.f;
      else {
        const float2 t = *reinterpret_cast<const float2*>(&lds[(a + r * 256) & 16383]);
        v[2 * r] = t.x;
        v[2 * r + 1] = t.y;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 32; ++r) acc += v[r];
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 1.234f) sink[threadIdx.x] = acc;
}

int main() {
  long long* out;
  float* sink;
  hipMalloc(&out, 8 * 64);
  hipMalloc(&sink, 4096);
  const char* names[] = {"b32 contiguous", "b64 contiguous", "b32 S8 wino4 m2", "b64 S8 planes", "b32 S16", "b64 S16 planes",
                         "b32 16 slots", "b64 stride32B", "b64 U image", "b32 stride16B"};
  for (int pat = 0; pat < 10; ++pat) {
    const bool b64 = pat == 1 || pat == 3 || pat == 5 || pat == 7 || pat == 8;
    if (b64) hipLaunchKernelGGL(k<2>, dim3(1), dim3(256), 0, 0, pat, out, sink);
    else hipLaunchKernelGGL(k<1>, dim3(1), dim3(256), 0, 0, pat, out, sink);
    long long c;
    hipMemcpy(&c, out, 8, hipMemcpyDeviceToHost);
    printf("%-18s %s  %.1f clk per read (4 waves)\n", names[pat], b64 ? "b64" : "b32", c / (256.0 * 16 * 4));
  }
  return 0;
}
