// What a cross-queue dependency costs on the critical path (the splat's frames in flight): a chain of
// ~20 us kernels on stream A, each made to wait for a short kernel on stream B through events, against the
// same chain alone. Cases (per frame, N frames, median of 5 runs):
//   alone      A: K
//   wait       B: wait(eA) k_short record(eB);  A: record(eA) wait(eB) K   (our pattern: a marker + a barrier per frame on A)
//   wait_only  B: k_short record(eB);            A: wait(eB) K                (no marker on A)
//   marker     A: record(eA) K                                                 (a marker alone)
//   wait_mark  B: k_short record(eB);            A: wait(eB) record(eA) K     (the marker right behind the barrier)
//   waitval    B: k_short writeValue(f);         A: waitValue(f >= frame) K   (stream memory operations)
//   post_mark  B: k_short record(eB);            A: wait(eB) K record(eA)     (the marker behind the kernel)
//   post_mark2 post_mark with the marker every second frame only
//   pingpong   frame f on Q = f odd ? B : A: k_short, wait(done of frame f - 1, the other queue), K, record(done_f)
//              (whole frames alternate queues; the long kernels stay ordered through a pending barrier)
//   pingpong_s pingpong plus the caller's stream S: S records a marker per frame that the frame's k_short
//              waits for (the marker of frame f - 1) and S waits for done_f (the join of each frame)
// each with device-scope (no system fence) and default events; and stream priorities for B.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/queue_sync.hip -o tools/micro/queue_sync && tools/micro/queue_sync
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin_kernel(unsigned long long ticks, unsigned* out) {  // ~ticks of the 100 MHz clock per workgroup
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && out) out[blockIdx.x] = 1u;
}

int main() {
  const int N = 400;
  unsigned* buf = nullptr;
  CHK(hipMalloc(&buf, 1 << 20));
  CHK(hipMemset(buf, 0, 1 << 20));
  int least = 0, greatest = 0;
  CHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  for (int fence = 0; fence < 2; ++fence) {
    const unsigned fl = hipEventDisableTiming | (fence ? 0u : (unsigned)hipEventDisableSystemFence);
    hipStream_t A, B;
    CHK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CHK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, greatest));
    hipEvent_t eA, eB;
    CHK(hipEventCreateWithFlags(&eA, fl));
    CHK(hipEventCreateWithFlags(&eB, fl));
    const char* names[] = {"alone", "wait", "wait_only", "marker", "wait_mark", "waitval", "pingpong", "pingpong_s",
                           "post_mark", "post_mark2"};
    unsigned* flag = buf + 4096;
    hipStream_t S;
    CHK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    hipEvent_t done[2], sm[2];
    for (int q = 0; q < 2; ++q) {
      CHK(hipEventCreateWithFlags(&done[q], fl));
      CHK(hipEventCreateWithFlags(&sm[q], fl));
    }
    for (int mode = 0; mode < 10; ++mode) {
      std::vector<double> us;
      for (int rep = 0; rep < 6; ++rep) {
        CHK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        for (int f = 0; f < N; ++f) {
          if (mode == 1) {
            CHK(hipEventRecord(eA, A));
            CHK(hipStreamWaitEvent(B, eA, 0));
          }
          if (mode == 1 || mode == 2 || mode == 4) {
            hipLaunchKernelGGL(spin_kernel, dim3(64), dim3(256), 0, B, 200ull, buf);  // ~2 us
            CHK(hipEventRecord(eB, B));
            CHK(hipStreamWaitEvent(A, eB, 0));
          }
          if (mode == 3 || mode == 4) CHK(hipEventRecord(eA, A));
          if (mode == 5) {
            const unsigned seq = (unsigned)(rep * N + f + 1);
            hipLaunchKernelGGL(spin_kernel, dim3(64), dim3(256), 0, B, 200ull, buf);
            CHK(hipStreamWriteValue32(B, flag, seq, 0));
            CHK(hipStreamWaitValue32(A, flag, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
          }
          if (mode >= 6) {
            hipStream_t Q = (f & 1) ? B : A;
            if (mode == 7) {
              CHK(hipEventRecord(sm[f & 1], S));
              if (f) CHK(hipStreamWaitEvent(Q, sm[(f - 1) & 1], 0));
            }
            hipLaunchKernelGGL(spin_kernel, dim3(64), dim3(256), 0, Q, 200ull, buf);
            if (f) CHK(hipStreamWaitEvent(Q, done[(f - 1) & 1], 0));
            hipLaunchKernelGGL(spin_kernel, dim3(2048), dim3(256), 0, Q, 2000ull, buf);
            CHK(hipEventRecord(done[f & 1], Q));
            if (mode == 7) CHK(hipStreamWaitEvent(S, done[f & 1], 0));
            continue;
          }
          if (mode >= 8) {
            hipLaunchKernelGGL(spin_kernel, dim3(64), dim3(256), 0, B, 200ull, buf);
            CHK(hipEventRecord(eB, B));
            CHK(hipStreamWaitEvent(A, eB, 0));
            hipLaunchKernelGGL(spin_kernel, dim3(2048), dim3(256), 0, A, 2000ull, buf);
            if (mode == 8 || (f & 1)) CHK(hipEventRecord(eA, A));
            continue;
          }
          hipLaunchKernelGGL(spin_kernel, dim3(2048), dim3(256), 0, A, 2000ull, buf);  // ~20 us
        }
        CHK(hipDeviceSynchronize());
        auto t1 = std::chrono::steady_clock::now();
        if (rep) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
      }
      std::sort(us.begin(), us.end());
      printf("%-10s events %-12s: %.2f us per frame (median of %zu)\n", names[mode],
             fence ? "system-scope" : "device-scope", us[us.size() / 2], us.size());
    }
    for (int q = 0; q < 2; ++q) {
      CHK(hipEventDestroy(done[q]));
      CHK(hipEventDestroy(sm[q]));
    }
    CHK(hipStreamDestroy(S));
    CHK(hipEventDestroy(eA));
    CHK(hipEventDestroy(eB));
    CHK(hipStreamDestroy(A));
    CHK(hipStreamDestroy(B));
  }
  return 0;
}
