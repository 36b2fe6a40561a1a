// knn.hip — 3DGS initialisation from a point cloud ("PLY (xyz, normal, uchar rgb) is
// the 3DGS initialisation wire format"; the point cloud is what Engine::savePly writes,
// engine.cpp:2849-2895). Kerbl et al. 2023 initialise every Gaussian from one point: mean = xyz,
// isotropic scale = sqrt(mean squared distance to the 3 nearest other points) (clamped below at
// 1e-7 before the sqrt), identity rotation, opacity 0.1, colour = rgb / 255 (the SH DC term's
// value). The 3-NN term is the only non-trivial part and is computed exactly:
//   1. bounds + 30-bit Morton codes (key = code << 32 | index, unique), hipCUB radix sort
//   2. sorted points gathered to float4; boxes of 64 consecutive points (one wave each) and
//      superboxes of 64 boxes (4096 points) with their AABBs
//   3. one work-item per sorted point, a wave = one box: scan the own box, then every superbox
//      whose box distance beats any lane's current 3rd-best, then its qualifying boxes. All loads
//      in the scans are wave-uniform (broadcast); pruning uses the rounded box distance, which
//      lower-bounds the rounded point distance, so the result equals brute force bit for bit.
// dist2 = ((b0 + b1) + b2) / 3 with b0 <= b1 <= b2 the three smallest
// ((dx * dx + dy * dy) + dz * dz) in f32 (no FMA); fewer than 3 other points: mean of those found,
// none: 0.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "knn.h"

namespace ptgs {

namespace {

constexpr uint32_t KNN_BOX = 64;    // points per box (= wave)
constexpr uint32_t KNN_SUPER = 64;  // boxes per superbox

struct KBounds {
  uint32_t lo[3], hi[3];  // order-preserving float encodings
};

__device__ __forceinline__ uint32_t k_f2ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float k_ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

__global__ void knn_bounds_kernel(const float* __restrict__ xyz, uint32_t n, KBounds* __restrict__ b) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (i < n)
    for (int a = 0; a < 3; ++a) lo[a] = hi[a] = xyz[3ull * i + a];
  for (int off = 32; off > 0; off >>= 1)
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
    }
  if ((threadIdx.x & 63u) == 0)
    for (int a = 0; a < 3; ++a) {
      atomicMin(&b->lo[a], k_f2ord(lo[a]));
      atomicMax(&b->hi[a], k_f2ord(hi[a]));
    }
}

__device__ __forceinline__ uint32_t k_expand(uint32_t v) {
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void knn_morton_kernel(const float* __restrict__ xyz, uint32_t n, const KBounds* __restrict__ b,
                                  unsigned long long* __restrict__ keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t q[3];
  for (int a = 0; a < 3; ++a) {
    const float lo = k_ord2f(b->lo[a]), ext = k_ord2f(b->hi[a]) - lo;
    const float u = ext > 0.0f ? (xyz[3ull * i + a] - lo) / ext : 0.0f;
    q[a] = (uint32_t)fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);  // NaN -> 0
  }
  const uint32_t code = (k_expand(q[0]) << 2) | (k_expand(q[1]) << 1) | k_expand(q[2]);
  keys[i] = ((unsigned long long)code << 32) | i;
}

__global__ void knn_gather_kernel(const float* __restrict__ xyz, const unsigned long long* __restrict__ keys,
                                  uint32_t n, float4* __restrict__ pts) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t i = (uint32_t)keys[j];
  pts[j] = make_float4(xyz[3ull * i], xyz[3ull * i + 1], xyz[3ull * i + 2], __uint_as_float(i));
}

struct KBox {
  float lo[3], hi[3];
};

// one wave per box: AABB of 64 consecutive points (or of 64 consecutive boxes for superboxes)
template <bool SUPER>
__global__ void knn_box_kernel(const float4* __restrict__ pts, const KBox* __restrict__ boxes, uint32_t count,
                               KBox* __restrict__ out, uint32_t nout) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
  if (w >= nout) return;
  const uint32_t e = w * 64u + lane;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (e < count) {
    if (SUPER) {
      const KBox b = boxes[e];
      for (int a = 0; a < 3; ++a) { lo[a] = b.lo[a]; hi[a] = b.hi[a]; }
    } else {
      const float4 p = pts[e];
      lo[0] = hi[0] = p.x; lo[1] = hi[1] = p.y; lo[2] = hi[2] = p.z;
    }
  }
  for (int off = 32; off > 0; off >>= 1)
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
    }
  if (lane == 0) {
    KBox b;
    for (int a = 0; a < 3; ++a) { b.lo[a] = lo[a]; b.hi[a] = hi[a]; }
    out[w] = b;
  }
}

__device__ __forceinline__ float box_d2(const KBox& b, float qx, float qy, float qz) {
  const float dx = fmaxf(fmaxf(b.lo[0] - qx, qx - b.hi[0]), 0.0f);
  const float dy = fmaxf(fmaxf(b.lo[1] - qy, qy - b.hi[1]), 0.0f);
  const float dz = fmaxf(fmaxf(b.lo[2] - qz, qz - b.hi[2]), 0.0f);
  return (dx * dx + dy * dy) + dz * dz;
}

struct Best3 {
  float b0 = INFINITY, b1 = INFINITY, b2 = INFINITY;
  uint32_t found = 0;
  __device__ __forceinline__ void insert(float d) {
    ++found;
    if (d < b2) {
      if (d < b1) {
        b2 = b1;
        if (d < b0) { b1 = b0; b0 = d; }
        else b1 = d;
      } else {
        b2 = d;
      }
    }
  }
};

__device__ __forceinline__ void scan_box(const float4* __restrict__ pts, uint32_t n, uint32_t box, uint32_t self,
                                         float qx, float qy, float qz, Best3& best) {
  const uint32_t first = box * KNN_BOX, last = min(first + KNN_BOX, n);
  for (uint32_t t = first; t < last; ++t) {
    const float4 p = pts[t];  // wave-uniform address: one broadcast fetch
    const float dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
    const float d = (dx * dx + dy * dy) + dz * dz;
    if (t != self) best.insert(d);
  }
}

__global__ void __launch_bounds__(256) knn_query_kernel(const float4* __restrict__ pts, uint32_t n,
                                                        const KBox* __restrict__ boxes, uint32_t nb,
                                                        const KBox* __restrict__ sboxes, uint32_t nsb,
                                                        float* __restrict__ dist2) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t own = j / KNN_BOX;  // wave-uniform (blockDim is a multiple of 64)
  if (own >= nb) return;
  const bool live = j < n;
  const float4 q = pts[live ? j : n - 1];
  Best3 best;
  scan_box(pts, n, own, j, q.x, q.y, q.z, best);
  for (uint32_t s = 0; s < nsb; ++s) {
    const KBox sb = sboxes[s];
    if (!__any(live && box_d2(sb, q.x, q.y, q.z) < best.b2)) continue;
    const uint32_t bend = min((s + 1) * KNN_SUPER, nb);
    for (uint32_t b = s * KNN_SUPER; b < bend; ++b) {
      if (b == own) continue;
      const KBox bx = boxes[b];
      if (!__any(live && box_d2(bx, q.x, q.y, q.z) < best.b2)) continue;
      scan_box(pts, n, b, j, q.x, q.y, q.z, best);
    }
  }
  if (!live) return;
  // the count of insert() calls = every other point in the scanned boxes; only min(3, found) are real
  const uint32_t k = min(best.found, 3u);
  float mean = 0.0f;
  if (k == 3) mean = ((best.b0 + best.b1) + best.b2) / 3.0f;
  else if (k == 2) mean = (best.b0 + best.b1) / 2.0f;
  else if (k == 1) mean = best.b0;
  dist2[__float_as_uint(q.w)] = mean;
}

// dist2 may alias opac (each work-item reads its dist2 before writing its opacity)
__global__ void gs_init_kernel(const float* __restrict__ xyz, const uint8_t* __restrict__ rgb, const float* dist2,
                               uint32_t n, float* __restrict__ means, float* __restrict__ scales,
                               float* __restrict__ rots, float* opac, float* __restrict__ colors) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = sqrtf(fmaxf(dist2[i], 1e-7f));
  for (int a = 0; a < 3; ++a) {
    means[3ull * i + a] = xyz[3ull * i + a];
    scales[3ull * i + a] = s;
    colors[3ull * i + a] = rgb ? (float)rgb[3ull * i + a] / 255.0f : 0.0f;
  }
  rots[4ull * i] = 1.0f;
  rots[4ull * i + 1] = 0.0f;
  rots[4ull * i + 2] = 0.0f;
  rots[4ull * i + 3] = 0.0f;
  opac[i] = 0.1f;
}

}  // namespace

hipError_t knn3_mean_dist2(const float* xyz, uint32_t n, float* dist2, hipStream_t s, KnnTimes* times) {
  if (n == 0) return hipSuccess;
  if (n == 1) return hipMemsetAsync(dist2, 0, 4, s);
  hipError_t e;
  const uint32_t nb = (n + KNN_BOX - 1) / KNN_BOX, nsb = (nb + KNN_SUPER - 1) / KNN_SUPER;
  unsigned long long *keys = nullptr, *keys_alt = nullptr;
  float4* pts = nullptr;
  KBox *boxes = nullptr, *sboxes = nullptr;
  KBounds* bnd = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  const dim3 B(256);
  auto G = [](uint64_t cnt) { return dim3((uint32_t)((cnt + 255u) / 256u)); };
#define CK(x) \
  if ((e = (x)) != hipSuccess) goto done
  CK(hipMalloc(&keys, 8ull * n));
  CK(hipMalloc(&keys_alt, 8ull * n));
  CK(hipMalloc(&pts, sizeof(float4) * n));
  CK(hipMalloc(&boxes, sizeof(KBox) * nb));
  CK(hipMalloc(&sboxes, sizeof(KBox) * nsb));
  CK(hipMalloc(&bnd, sizeof(KBounds)));
  CK(hipcub::DeviceRadixSort::SortKeys(nullptr, temp_bytes, keys, keys_alt, (int)n, 0, 62, s));
  CK(hipMalloc(&temp, temp_bytes));
  {
    KBounds init;
    for (int a = 0; a < 3; ++a) { init.lo[a] = 0xFFFFFFFFu; init.hi[a] = 0u; }
    CK(hipMemcpyAsync(bnd, &init, sizeof(init), hipMemcpyHostToDevice, s));
  }
  if (times)
    for (auto& v : ev) CK(hipEventCreate(&v));
  if (times) hipEventRecord(ev[0], s);
  hipLaunchKernelGGL(knn_bounds_kernel, G(n), B, 0, s, xyz, n, bnd);
  hipLaunchKernelGGL(knn_morton_kernel, G(n), B, 0, s, xyz, n, bnd, keys);
  CK(hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, keys_alt, (int)n, 0, 62, s));
  hipLaunchKernelGGL(knn_gather_kernel, G(n), B, 0, s, xyz, keys_alt, n, pts);
  hipLaunchKernelGGL((knn_box_kernel<false>), G(64ull * nb), B, 0, s, pts, nullptr, n, boxes, nb);
  hipLaunchKernelGGL((knn_box_kernel<true>), G(64ull * nsb), B, 0, s, nullptr, boxes, nb, sboxes, nsb);
  if (times) hipEventRecord(ev[1], s);
  hipLaunchKernelGGL(knn_query_kernel, G(64ull * nb), B, 0, s, pts, n, boxes, nb, sboxes, nsb, dist2);
  if (times) hipEventRecord(ev[2], s);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));  // temporaries are freed below
  if (times) {
    hipEventElapsedTime(&times->sort_ms, ev[0], ev[1]);
    hipEventElapsedTime(&times->query_ms, ev[1], ev[2]);
  }
done:
#undef CK
  hipFree(keys);
  hipFree(keys_alt);
  hipFree(pts);
  hipFree(boxes);
  hipFree(sboxes);
  hipFree(bnd);
  hipFree(temp);
  for (auto& v : ev)
    if (v) hipEventDestroy(v);
  return e;
}

hipError_t gaussians_from_points(const float* xyz, const uint8_t* rgb, uint32_t n, float* means, float* scales,
                                 float* rots, float* opac, float* colors, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // dist2 lands in `opac` (n floats) before the init kernel overwrites it with the opacity
  hipError_t e = knn3_mean_dist2(xyz, n, opac, s, nullptr);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gs_init_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, xyz, rgb, opac, n, means, scales, rots,
                     opac, colors);
  return hipGetLastError();
}

}  // namespace ptgs
