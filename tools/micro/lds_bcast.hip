// LDS read cost by address pattern (gfx950): ds_read_b128 / ds_read_b32 with every lane on one address
// (broadcast), one address per ds_read_b128 lane group, one per contiguous 16 lanes, or 64 distinct
// conflict-free addresses. 8 independent reads between waits; 8 waves per SIMD (the blend's occupancy).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/lds_bcast.hip -o tools/micro/lds_bcast && tools/micro/lds_bcast
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE, int WIDTH>
__global__ __launch_bounds__(256, 8) void lds_kernel(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float s[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) s[i] = (float)i;
  __syncthreads();
  const unsigned lane = threadIdx.x & 63u;
  unsigned a;
  if (MODE == 0) a = 0;                                                        // broadcast
  else if (MODE == 1) a = (((lane >> 5) << 1) | ((0xF00F0FF0u >> (lane & 31u)) & 1u)) * 48u;  // b128 lane groups
  else if (MODE == 2) a = (lane >> 4) * 48u;                                   // contiguous 16 lanes
  else a = lane * 16u;                                                         // 64 distinct
  a = a * 4u + (threadIdx.x >> 6) * 1024u * 0u;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned ad = a + (unsigned)k * 3072u % 8192u;
      if (WIDTH == 16) {
        float4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(ad));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        acc += v.x + v.w;
      } else {
        float v;
        asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(ad));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        acc += v;
      }
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}

template <int MODE, int WIDTH>
float run(float* d, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((lds_kernel<MODE, WIDTH>), dim3(2048), dim3(256), 0, 0, d, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL((lds_kernel<MODE, WIDTH>), dim3(2048), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* d;
  hipMalloc(&d, 16);
  const int it = 2000;
  const double reads = 2048.0 * 4 * it * 8;  // wave-instructions
  const char* names[4] = {"broadcast (1 address)", "4 addresses, one per b128 lane group", "4 addresses, per 16 contiguous lanes",
                          "64 distinct addresses"};
  float t128[4] = {run<0, 16>(d, it), run<1, 16>(d, it), run<2, 16>(d, it), run<3, 16>(d, it)};
  float t32[4] = {run<0, 4>(d, it), run<1, 4>(d, it), run<2, 4>(d, it), run<3, 4>(d, it)};
  for (int m = 0; m < 4; ++m)
    printf("%-40s ds_read_b128 %.3f ms (%.2f ns per wave-instr per CU)  ds_read_b32 %.3f ms (%.2f)\n", names[m], t128[m],
           t128[m] * 1e6 / reads * 256, t32[m], t32[m] * 1e6 / reads * 256);
  return 0;
}
