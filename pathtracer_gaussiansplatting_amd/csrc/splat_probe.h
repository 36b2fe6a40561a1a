// splat_probe.h — measurement hooks of splat.hip, compiled out of the shipped library.
//
// Stamps (GS_STAMP builds, tools/gs_stamps.py): per-workgroup s_memrealtime (100 MHz) stamps at phase
// boundaries of the fused front end (kind 0) and the blend (kind 1), read back with ptgs_debug_stamps.
// Probes (GS_PROBES = OR of the bits below; tools/gs_probe.py): timing probes that remove one phase of the
// blend (wrong image). Both are plain `if` on compile-time constants inside the kernels: no #if branches,
// and a default build contains neither.
#pragma once

#ifndef GS_PROBES
#define GS_PROBES 0
#endif
#define GS_PROBE_NO_EVAL 1u  // the blend evaluates no list entry (the evaluation's cost)
#define GS_PROBE_NO_REC 2u   // small tiles skip the record gather (its latency)
#define GS_PROBE_NO_RANK 4u  // small tiles rank by identity (the sort's cost)
#define GS_PROBE_NO_EXACT 8u  // small tiles stage with the alpha-box quadrant test only (same image: both are conservative)
#define GS_PROBE_NO_MERGE 16u  // small tiles above GS_MERGE_MIN rank by identity (the wave sort + run searches' cost)
#define GS_PROBE(bit) ((GS_PROBES & (bit)) != 0u)

#ifdef GS_STAMP
#define GS_STAMP_WG 65536
#define GS_STAMP_N 8
namespace ptgs {
__device__ unsigned long long g_gs_stamps[2][GS_STAMP_WG * GS_STAMP_N];
}
#define STAMP(kind, k)                                                                                      \
  do {                                                                                                     \
    const uint32_t wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                              \
    if (threadIdx.x == 0 && wg_ < GS_STAMP_WG)                                                             \
      g_gs_stamps[kind][wg_ * GS_STAMP_N + (k)] = __builtin_amdgcn_s_memrealtime();                       \
  } while (0)
// a stamp once wave 0's outstanding loads have arrived
#define STAMP_WAITED(kind, k)                                                                               \
  do {                                                                                                     \
    if (threadIdx.x == 0) __builtin_amdgcn_s_waitcnt(0);                                                   \
    STAMP(kind, k);                                                                                        \
  } while (0)
#define STAMP_SYNC() __syncthreads()
#define GS_STAMP_EXPORT                                                                                     \
  extern "C" int ptgs_debug_stamps(int kind, unsigned long long* host, unsigned int n) {                   \
    const size_t per = sizeof(ptgs::g_gs_stamps[0]);                                                       \
    if (n * 8ull > per) n = (unsigned int)(per / 8);                                                        \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ptgs::g_gs_stamps), (size_t)n * 8, (size_t)kind * per, \
                                    hipMemcpyDeviceToHost);                                                 \
  }
#else
#define STAMP(kind, k) do { } while (0)
#define STAMP_WAITED(kind, k) do { } while (0)
#define STAMP_SYNC() do { } while (0)
#define GS_STAMP_EXPORT
#endif
