// Does a kernel launched with hipExtAnyOrderLaunch (AQL packet without the barrier bit) start beside the
// kernel before it on the SAME stream on gfx950? (The splat's frames in flight would then need no second
// queue and no cross-queue barrier: front end k + 1 any-order behind blend k.) Per frame on one stream:
//   serial    : short(64 WGs, ~2 us), long(2048 WGs, ~20 us), both with the barrier bit
//   any_order : short launched with hipExtAnyOrderLaunch, long with the barrier bit
// Each kernel records its first start and last end (s_memrealtime, 100 MHz) through vector atomics; the
// report gives us per frame and how many short kernels started before the previous long one ended.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/any_order.hip -o tools/micro/any_order && tools/micro/any_order
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin_kernel(unsigned long long ticks, unsigned long long* span) {  // span: [min start, max end]
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicMin(span, t0);
    atomicMax(span + 1, t1);
  }
}

int main() {
  const int N = 200;
  unsigned long long* spans = nullptr;  // [frame][kernel 0 short / 1 long][2]
  const size_t bytes = (size_t)N * 4 * sizeof(unsigned long long);
  CHK(hipMalloc(&spans, bytes));
  hipStream_t A;
  CHK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  std::vector<unsigned long long> h((size_t)N * 4);
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<double> us;
    int overlapped = 0;
    for (int rep = 0; rep < 5; ++rep) {
      for (size_t i = 0; i < h.size(); ++i) h[i] = (i & 1) ? 0ull : ~0ull;
      CHK(hipMemcpy(spans, h.data(), bytes, hipMemcpyHostToDevice));
      CHK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      for (int f = 0; f < N; ++f) {
        unsigned long long* s = spans + (size_t)f * 4;
        hipExtLaunchKernelGGL(spin_kernel, dim3(64), dim3(256), 0, A, nullptr, nullptr, mode ? hipExtAnyOrderLaunch : 0,
                              200ull, s);
        CHK(hipGetLastError());
        hipExtLaunchKernelGGL(spin_kernel, dim3(2048), dim3(256), 0, A, nullptr, nullptr, 0, 2000ull, s + 2);
        CHK(hipGetLastError());
      }
      CHK(hipDeviceSynchronize());
      auto t1 = std::chrono::steady_clock::now();
      CHK(hipMemcpy(h.data(), spans, bytes, hipMemcpyDeviceToHost));
      if (!rep) continue;
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
      for (int f = 1; f < N; ++f)  // short f started before long f - 1 ended
        if (h[(size_t)f * 4] < h[(size_t)(f - 1) * 4 + 3]) ++overlapped;
    }
    std::sort(us.begin(), us.end());
    printf("%-9s: %.2f us per frame (median of %zu); short kernels started beside the previous long one: %d of %d\n",
           mode ? "any_order" : "serial", us[us.size() / 2], us.size(), overlapped, (N - 1) * 4);
  }
  CHK(hipStreamDestroy(A));
  CHK(hipFree(spans));
  return 0;
}
