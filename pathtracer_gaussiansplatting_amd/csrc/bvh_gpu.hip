// bvh_gpu.hip — GPU BVH builder (the reference relies on the driver's BLAS/TLAS
// builds, engine.cpp:534-655 / :1385-1520; the 1M-triangle C5 scene and scene edits need fast
// rebuilds). A linear BVH (Karras, "Maximizing parallelism in the construction of BVHs, octrees and
// k-d trees", HPG 2012) in the device layout of bvh.h:
//   1. bounds     scene centroid box + coordinate scale (for the conservative box padding)
//   2. morton     30-bit codes of the triangle centroids; key = code << 32 | flattening index (unique)
//   3. sort       keys (hipCUB radix sort)
//   4. hierarchy  n-1 internal nodes from the longest common prefixes of adjacent keys
//   5. boxes      bottom-up, one work-item per leaf, the second arrival at a node continues
//   6. emit       subtrees of <= GS_BVH_LEAF triangles collapse into leaves; the remaining internal
//                 nodes are renumbered by a prefix sum (root stays 0) and written as 64-B nodes
//                 holding both (padded) child boxes; triangle records in leaf (sorted) order
//   7. depth      max depth of the emitted tree (must fit the traversal stack, else the host SAH
//                 builder is used)
// Hits do not depend on the tree (closest hit with the lower-id tie rule, padded boxes), so images
// are identical to the host-built BVH's; only the traversal cost differs (SAH is the default).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>

#include "bvh_gpu.h"

namespace ptgs {

#define GS_BVH_LEAF 4

namespace {

__device__ __forceinline__ uint32_t f2ord(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

struct Bounds {  // ordered-uint encodings
  uint32_t lo[3], hi[3];
  uint32_t maxabs;  // float bits of max |coordinate| (non-negative: bit order = value order)
};

__global__ void bvh_bounds_kernel(const BuildTri* __restrict__ tris, uint32_t n, Bounds* __restrict__ b) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, ma = 0.0f;
  if (i < n) {
    const BuildTri t = tris[i];
    for (int a = 0; a < 3; ++a) {
      const float mn = fminf(t.v0[a], fminf(t.v1[a], t.v2[a])), mx = fmaxf(t.v0[a], fmaxf(t.v1[a], t.v2[a]));
      const float c = 0.5f * (mn + mx);
      lo[a] = c;
      hi[a] = c;
      ma = fmaxf(ma, fmaxf(fabsf(mn), fabsf(mx)));
    }
  }
  for (int off = 32; off > 0; off >>= 1)
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
      if (a == 0) ma = fmaxf(ma, __shfl_xor(ma, off));
    }
  if ((threadIdx.x & 63u) == 0) {
    for (int a = 0; a < 3; ++a) {
      atomicMin(&b->lo[a], f2ord(lo[a]));
      atomicMax(&b->hi[a], f2ord(hi[a]));
    }
    atomicMax(&b->maxabs, __float_as_uint(ma));
  }
}

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {  // 10 bits -> every 3rd bit
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void bvh_morton_kernel(const BuildTri* __restrict__ tris, uint32_t n, const Bounds* __restrict__ b,
                                  unsigned long long* __restrict__ keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const BuildTri t = tris[i];
  uint32_t q[3];
  for (int a = 0; a < 3; ++a) {
    const float mn = fminf(t.v0[a], fminf(t.v1[a], t.v2[a])), mx = fmaxf(t.v0[a], fmaxf(t.v1[a], t.v2[a]));
    const float c = 0.5f * (mn + mx);
    const float lo = ord2f(b->lo[a]), hi = ord2f(b->hi[a]);
    const float ext = hi - lo;
    const float u = ext > 0.0f ? (c - lo) / ext : 0.0f;
    q[a] = (uint32_t)fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
  }
  const uint32_t code = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
  keys[i] = ((unsigned long long)code << 32) | i;
}

__device__ __forceinline__ int lcp(const unsigned long long* k, uint32_t n, int i, int j) {
  if (j < 0 || j >= (int)n) return -1;
  return __clzll(k[i] ^ k[j]);  // keys are unique
}

// internal node i: children encoded >= 0 internal, < 0 leaf ~(sorted triangle index)
__global__ void bvh_karras_kernel(const unsigned long long* __restrict__ k, uint32_t n, int2* __restrict__ child,
                                  uint2* __restrict__ range, int* __restrict__ parent_int,
                                  int* __restrict__ parent_leaf) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= (int)n - 1) return;
  const int d = (lcp(k, n, i, i + 1) - lcp(k, n, i, i - 1)) >= 0 ? 1 : -1;
  const int dmin = lcp(k, n, i, i - d);
  int lmax = 2;
  while (lcp(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (lcp(k, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = lcp(k, n, i, j);
  int s = 0;
  for (int t = (l + 1) >> 1;; t = (t + 1) >> 1) {
    if (lcp(k, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  const int left = (first == gamma) ? ~gamma : gamma;
  const int right = (last == gamma + 1) ? ~(gamma + 1) : gamma + 1;
  child[i] = make_int2(left, right);
  range[i] = make_uint2((uint32_t)first, (uint32_t)last);
  if (left >= 0) parent_int[left] = i; else parent_leaf[~left] = i;
  if (right >= 0) parent_int[right] = i; else parent_leaf[~right] = i;
  if (i == 0) parent_int[0] = -1;
}

struct Box6 {
  float lo[3], hi[3];
};

__device__ __forceinline__ Box6 tri_box(const BuildTri& t) {
  Box6 b;
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = fminf(t.v0[a], fminf(t.v1[a], t.v2[a]));
    b.hi[a] = fmaxf(t.v0[a], fmaxf(t.v1[a], t.v2[a]));
  }
  return b;
}

__global__ void bvh_boxes_kernel(const BuildTri* __restrict__ tris, const unsigned long long* __restrict__ keys,
                                 uint32_t n, const int2* __restrict__ child, const int* __restrict__ parent_int,
                                 const int* __restrict__ parent_leaf, Box6* __restrict__ node_box,
                                 uint32_t* __restrict__ visits) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int node = parent_leaf[k];
  while (node >= 0) {
    __threadfence();
    if (atomicAdd(&visits[node], 1u) == 0) return;  // the sibling's work-item finishes this node
    __threadfence();
    const int2 c = child[node];
    Box6 b;
    for (int s = 0; s < 2; ++s) {
      const int ch = s ? c.y : c.x;
      Box6 cb;
      if (ch < 0) {
        cb = tri_box(tris[(uint32_t)keys[~ch]]);
      } else {
        // written by another work-item (any XCD): agent-scope atomic loads after the acquire fence
        for (int a = 0; a < 3; ++a) {
          cb.lo[a] = __hip_atomic_load(&node_box[ch].lo[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          cb.hi[a] = __hip_atomic_load(&node_box[ch].hi[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      for (int a = 0; a < 3; ++a) {
        b.lo[a] = s ? fminf(b.lo[a], cb.lo[a]) : cb.lo[a];
        b.hi[a] = s ? fmaxf(b.hi[a], cb.hi[a]) : cb.hi[a];
      }
    }
    node_box[node] = b;
    node = parent_int[node];
  }
}

__device__ __forceinline__ bool emitted(const uint2* range, int i) {
  return i == 0 || range[i].y - range[i].x + 1u > GS_BVH_LEAF;
}

__global__ void bvh_flags_kernel(const uint2* __restrict__ range, uint32_t m, uint32_t* __restrict__ flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) flag[i] = emitted(range, (int)i) ? 1u : 0u;
}

// host padding rule (bvh.cpp Builder::padded): relative 1e-5 of the box extent + absolute term
__device__ __forceinline__ void pad_box(const Box6& b, float pad_abs, float* lo, float* hi) {
  const float ext = fmaxf(b.hi[0] - b.lo[0], fmaxf(b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]));
  const float p = ext * 1e-5f + pad_abs;
  for (int a = 0; a < 3; ++a) {
    lo[a] = b.lo[a] - p;
    hi[a] = b.hi[a] + p;
  }
}

__global__ void bvh_emit_kernel(const BuildTri* __restrict__ tris, const unsigned long long* __restrict__ keys,
                                const int2* __restrict__ child, const uint2* __restrict__ range,
                                const Box6* __restrict__ node_box, const uint32_t* __restrict__ newidx,
                                uint32_t m, const Bounds* __restrict__ bnd, float4* __restrict__ nodes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !emitted(range, (int)i)) return;
  const float pad_abs = __uint_as_float(bnd->maxabs) * 4e-7f + 1e-30f;
  const int2 c = child[i];
  float lo[2][3], hi[2][3];
  int link[2];
  for (int s = 0; s < 2; ++s) {
    const int ch = s ? c.y : c.x;
    Box6 b;
    if (ch >= 0 && emitted(range, ch)) {
      link[s] = (int)newidx[ch];
      b = node_box[ch];
    } else {
      uint32_t first, cnt;
      if (ch < 0) {
        first = (uint32_t)~ch;
        cnt = 1;
        b = tri_box(tris[(uint32_t)keys[first]]);
      } else {
        first = range[ch].x;
        cnt = range[ch].y - range[ch].x + 1u;
        b = node_box[ch];
      }
      link[s] = ~(int)(((cnt - 1u) << 27) | first);
    }
    pad_box(b, pad_abs, lo[s], hi[s]);
  }
  float4* o = nodes + 4 * (size_t)newidx[i];
  o[0] = make_float4(lo[0][0], hi[0][0], lo[0][1], hi[0][1]);
  o[1] = make_float4(lo[1][0], hi[1][0], lo[1][1], hi[1][1]);
  o[2] = make_float4(lo[0][2], hi[0][2], lo[1][2], hi[1][2]);
  o[3] = make_float4(__int_as_float(link[0]), __int_as_float(link[1]), 0.0f, 0.0f);
}

__global__ void bvh_tris_kernel(const BuildTri* __restrict__ tris, const unsigned long long* __restrict__ keys,
                                uint32_t n, float4* __restrict__ out, uint32_t* __restrict__ flags) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const BuildTri t = tris[(uint32_t)keys[k]];
  out[3 * k] = make_float4(t.v0[0], t.v0[1], t.v0[2], __uint_as_float(t.mesh));
  out[3 * k + 1] = make_float4(t.v1[0] - t.v0[0], t.v1[1] - t.v0[1], t.v1[2] - t.v0[2], __uint_as_float(t.prim));
  out[3 * k + 2] = make_float4(t.v2[0] - t.v0[0], t.v2[1] - t.v0[1], t.v2[2] - t.v0[2], __uint_as_float(t.gid));
  flags[k] = t.flags;
}

__global__ void bvh_depth_kernel(const uint2* __restrict__ range, const int* __restrict__ parent_int, uint32_t m,
                                 uint32_t* __restrict__ depth) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !emitted(range, (int)i)) return;
  uint32_t d = 0;
  for (int p = parent_int[i]; p >= 0; p = parent_int[p]) ++d;  // ancestors are all emitted
  atomicMax(depth, d + 1u);  // + the leaf level below this node
}

}  // namespace

hipError_t build_bvh_gpu(const std::vector<BuildTri>& tris, uint32_t max_depth, GpuBvh& out, float* build_ms) {
  const uint32_t n = (uint32_t)tris.size(), m = n - 1;
  out = GpuBvh{};
  if (n < 2) return hipErrorInvalidValue;
  hipError_t e;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  BuildTri* d_tris = nullptr;
  unsigned long long *keys = nullptr, *keys_alt = nullptr;
  int2* child = nullptr;
  uint2* range = nullptr;
  int *parent_int = nullptr, *parent_leaf = nullptr;
  Box6* node_box = nullptr;
  uint32_t *visits = nullptr, *flag = nullptr, *newidx = nullptr, *depth = nullptr;
  Bounds* bnd = nullptr;
  void* temp = nullptr;
  size_t temp_bytes = 0, t1 = 0, t2 = 0;
  float4* nodes = nullptr;
  float4* trec = nullptr;
  uint32_t* tflags = nullptr;
  uint32_t n_emit = 0, last_flag = 0, dep = 0;
  const dim3 B(256);
  auto G = [&](uint32_t cnt) { return dim3((cnt + 255u) / 256u); };
#define CK(x) \
  if ((e = (x)) != hipSuccess) goto done
  CK(hipMalloc(&d_tris, sizeof(BuildTri) * n));
  CK(hipMalloc(&keys, 8ull * n));
  CK(hipMalloc(&keys_alt, 8ull * n));
  CK(hipMalloc(&child, sizeof(int2) * m));
  CK(hipMalloc(&range, sizeof(uint2) * m));
  CK(hipMalloc(&parent_int, sizeof(int) * m));
  CK(hipMalloc(&parent_leaf, sizeof(int) * n));
  CK(hipMalloc(&node_box, sizeof(Box6) * m));
  CK(hipMalloc(&visits, 4ull * m));
  CK(hipMalloc(&flag, 4ull * m));
  CK(hipMalloc(&newidx, 4ull * m));
  CK(hipMalloc(&depth, 4));
  CK(hipMalloc(&bnd, sizeof(Bounds)));
  CK(hipMemcpy(d_tris, tris.data(), sizeof(BuildTri) * n, hipMemcpyHostToDevice));
  {
    Bounds init;
    for (int a = 0; a < 3; ++a) {
      init.lo[a] = 0xFFFFFFFFu;
      init.hi[a] = 0u;
    }
    init.maxabs = 0u;
    CK(hipMemcpy(bnd, &init, sizeof(init), hipMemcpyHostToDevice));
  }
  CK(hipMemset(visits, 0, 4ull * m));
  CK(hipMemset(depth, 0, 4));
  CK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, keys, keys_alt, (int)n, 0, 62));
  CK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, flag, newidx, (int)m));
  temp_bytes = t1 > t2 ? t1 : t2;
  CK(hipMalloc(&temp, temp_bytes));
  CK(hipDeviceSynchronize());
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(bvh_bounds_kernel, G(n), B, 0, 0, d_tris, n, bnd);
  hipLaunchKernelGGL(bvh_morton_kernel, G(n), B, 0, 0, d_tris, n, bnd, keys);
  CK(hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, keys_alt, (int)n, 0, 62));
  hipLaunchKernelGGL(bvh_karras_kernel, G(m), B, 0, 0, keys_alt, n, child, range, parent_int, parent_leaf);
  hipLaunchKernelGGL(bvh_boxes_kernel, G(n), B, 0, 0, d_tris, keys_alt, n, child, parent_int, parent_leaf, node_box,
                     visits);
  hipLaunchKernelGGL(bvh_flags_kernel, G(m), B, 0, 0, range, m, flag);
  CK(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, flag, newidx, (int)m));
  CK(hipGetLastError());
  CK(hipMemcpy(&n_emit, newidx + (m - 1), 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&last_flag, flag + (m - 1), 4, hipMemcpyDeviceToHost));
  n_emit += last_flag;
  CK(hipMalloc(&nodes, sizeof(float4) * 4 * n_emit));
  CK(hipMalloc(&trec, sizeof(float4) * 3 * n));
  CK(hipMalloc(&tflags, 4ull * n));
  hipLaunchKernelGGL(bvh_emit_kernel, G(m), B, 0, 0, d_tris, keys_alt, child, range, node_box, newidx, m, bnd, nodes);
  hipLaunchKernelGGL(bvh_tris_kernel, G(n), B, 0, 0, d_tris, keys_alt, n, trec, tflags);
  hipLaunchKernelGGL(bvh_depth_kernel, G(m), B, 0, 0, range, parent_int, m, depth);
  CK(hipGetLastError());
  hipEventRecord(e1, 0);
  CK(hipMemcpy(&dep, depth, 4, hipMemcpyDeviceToHost));
  if (build_ms) hipEventElapsedTime(build_ms, e0, e1);
  out.nodes = nodes;
  out.tris = trec;
  out.tri_flags = tflags;
  out.num_nodes = n_emit;
  out.depth = dep;
  nodes = nullptr;
  trec = nullptr;
  tflags = nullptr;
  if (dep > max_depth) e = hipErrorNotSupported;  // caller falls back to the host builder
done:
#undef CK
  hipFree(d_tris);
  hipFree(keys);
  hipFree(keys_alt);
  hipFree(child);
  hipFree(range);
  hipFree(parent_int);
  hipFree(parent_leaf);
  hipFree(node_box);
  hipFree(visits);
  hipFree(flag);
  hipFree(newidx);
  hipFree(depth);
  hipFree(bnd);
  hipFree(temp);
  hipFree(nodes);
  hipFree(trec);
  hipFree(tflags);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (e != hipSuccess && e != hipErrorNotSupported) {
    hipFree(out.nodes);
    hipFree(out.tris);
    hipFree(out.tri_flags);
    out = GpuBvh{};
  }
  return e;
}

}  // namespace ptgs
