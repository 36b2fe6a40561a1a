// Workgroup dispatch-rate probe: how long do G workgroups of 256 work-items take when each does
// (almost) nothing, with and without an LDS footprint that limits residency?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFF) out[0] = 1.0f;
}
__global__ __launch_bounds__(256) void k_store(float* out) { out[blockIdx.x * 256 + threadIdx.x] = 1.0f; }
__global__ __launch_bounds__(256) void k_lds21k(float* out) {
  __shared__ float s[21 * 1024 / 4];
  s[threadIdx.x * 5] = (float)threadIdx.x;
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = s[(threadIdx.x * 7) % 5000];
}
__global__ __launch_bounds__(256) void k_chain(const float* in, float* out) {  // two dependent loads
  const int a = (int)in[blockIdx.x];
  out[blockIdx.x * 256 + threadIdx.x] = in[(a + threadIdx.x) & 0xFFFFF];
}

int main() {
  float *out, *in;
  hipMalloc(&out, 64u << 20);
  hipMalloc(&in, 8u << 20);
  hipMemset(in, 0, 8u << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int G : {1024, 4096, 8160, 16320, 32400}) {
    for (int kind = 0; kind < 4; ++kind) {
      float best = 1e9f;
      for (int rep = 0; rep < 20; ++rep) {
        hipEventRecord(a);
        if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, 0, out);
        if (kind == 1) hipLaunchKernelGGL(k_store, dim3(G), dim3(256), 0, 0, out);
        if (kind == 2) hipLaunchKernelGGL(k_lds21k, dim3(G), dim3(256), 0, 0, out);
        if (kind == 3) hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, 0, in, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("G=%6d %-8s %8.2f us\n", G, kind == 0 ? "empty" : kind == 1 ? "store" : kind == 2 ? "lds21k" : "chain",
             best * 1e3f);
    }
  }
  return 0;
}
