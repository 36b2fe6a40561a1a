// bvh_collapse_gpu.hip — the 4-wide collapse of a device BVH2 (bvh.h layouts) on the GPU, the same
// result as the host's collapse_bvh4 (bvh.cpp) word for word: each 4-wide node takes the children of
// a BVH2 node and repeatedly opens its largest-area interior child (first in list order on ties,
// the opened child's first half in place, its second appended) until it has max_children; 4-wide
// slots are numbered breadth first in (parent, child) order, which a per-level prefix sum over the
// interior-child counts reproduces. Bottom-up per level: the traversal stack need (sum over a path of
// children - 1) and the depth, for the caller's fan-out fallback.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "bvh_gpu.h"

namespace ptgs {

namespace {

struct Ent {
  float lo[3], hi[3];
  int32_t ref;
};

__device__ __forceinline__ void bvh2_children(const float4* n2, int32_t node, Ent e[2]) {
  const float4 a = n2[4 * (size_t)node], b = n2[4 * (size_t)node + 1], c = n2[4 * (size_t)node + 2],
               d = n2[4 * (size_t)node + 3];
  e[0] = Ent{{a.x, a.z, c.x}, {a.y, a.w, c.y}, __float_as_int(d.x)};
  e[1] = Ent{{b.x, b.z, c.z}, {b.y, b.w, c.w}, __float_as_int(d.y)};
}
__device__ __forceinline__ float ent_area(const Ent& e) {  // bvh.cpp ent_area
  float d[3];
  for (int a = 0; a < 3; ++a) d[a] = fmaxf(0.0f, e.hi[a] - e.lo[a]);
  return d[0] * d[1] + d[1] * d[2] + d[2] * d[0];
}
// std::max(0.0f, x) is (0 < x) ? x : 0; fmaxf agrees for every non-NaN x (and -0 vs +0 only feeds a
// product that is compared, never stored)

__device__ __forceinline__ int open_list(const float4* n2, int32_t node, int max_children, Ent list[4]) {
  bvh2_children(n2, node, list);
  int cnt = 2;
  while (cnt < max_children) {
    int best = -1;
    float ba = -1.0f;
    for (int k = 0; k < cnt; ++k)
      if (list[k].ref >= 0 && ent_area(list[k]) > ba) { ba = ent_area(list[k]); best = k; }
    if (best < 0) break;
    Ent sub[2];
    bvh2_children(n2, list[best].ref, sub);
    list[best] = sub[0];
    list[cnt++] = sub[1];
  }
  return cnt;
}

// pass 1 of a level: interior-child count of every node
__global__ void collapse_count_kernel(const float4* __restrict__ n2, const int32_t* __restrict__ level, uint32_t n,
                                      int max_children, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Ent list[4];
  const int c = open_list(n2, level[i], max_children, list);
  uint32_t k = 0;
  for (int j = 0; j < c; ++j) k += list[j].ref >= 0 ? 1u : 0u;
  cnt[i] = k;
}

// pass 2: write the level's 4-wide nodes (slot = first + i) and the next level's BVH2 nodes
__global__ void collapse_emit_kernel(const float4* __restrict__ n2, const int32_t* __restrict__ level, uint32_t n,
                                     uint32_t first, int max_children, const uint32_t* __restrict__ off,
                                     uint32_t next_first, int32_t* __restrict__ next_level, float* __restrict__ n4,
                                     uint32_t* __restrict__ ncount) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Ent list[4];
  const int c = open_list(n2, level[i], max_children, list);
  float* f = n4 + 32 * (size_t)(first + i);
  uint32_t o = off[i];
  for (int j = 0; j < 4; ++j) {
    int32_t child = 0;
    if (j < c) {
      for (int a = 0; a < 3; ++a) {
        f[(2 * a) * 4 + j] = list[j].lo[a];
        f[(2 * a + 1) * 4 + j] = list[j].hi[a];
      }
      if (list[j].ref >= 0) {
        next_level[o] = list[j].ref;
        child = (int32_t)(next_first + o);
        ++o;
      } else {
        child = list[j].ref;
      }
    } else {
      for (int a = 0; a < 6; ++a) f[a * 4 + j] = 1e30f;
    }
    f[24 + j] = __int_as_float(child);
    f[28 + j] = 0.0f;
  }
  ncount[first + i] = (uint32_t)c;
}

// bottom-up: need = (children - 1) + max over interior children, depth = 1 + max
__global__ void collapse_need_kernel(const float* __restrict__ n4, uint32_t first, uint32_t n,
                                     const uint32_t* __restrict__ ncount, uint32_t* __restrict__ need,
                                     uint32_t* __restrict__ dep) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = first + i;
  uint32_t m = 0, d = 0;
  for (int j = 0; j < 4; ++j) {
    const int32_t ch = __float_as_int(n4[32 * (size_t)s + 24 + j]);
    const bool interior = (uint32_t)j < ncount[s] && ch > 0;  // (slot 0 is the root: never a child)
    if (interior) { m = max(m, need[ch]); d = max(d, dep[ch]); }
  }
  need[s] = (ncount[s] - 1u) + m;
  dep[s] = 1u + d;
}

}  // namespace

hipError_t collapse_bvh4_gpu(const float4* nodes2, uint32_t num2, int max_children, float4** nodes4, uint32_t* num4,
                             uint32_t* max_stack, uint32_t* depth4) {
  *nodes4 = nullptr;
  hipError_t e = hipSuccess;
  int32_t *lv[2] = {nullptr, nullptr};
  uint32_t *cnt = nullptr, *off = nullptr, *ncount = nullptr, *need = nullptr, *dep = nullptr;
  float* n4 = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  std::vector<std::pair<uint32_t, uint32_t>> levels;  // (first slot, count)
  uint32_t first = 0, n = 1, total = 1;
  const int32_t root = 0;
  // 4-wide nodes <= BVH2 nodes (each consumes >= 1 BVH2 node)
  const size_t cap = num2 + 1;
#define CK(x) \
  if ((e = (x)) != hipSuccess) goto done
  CK(hipMalloc(&lv[0], 4 * cap));
  CK(hipMalloc(&lv[1], 4 * cap));
  CK(hipMalloc(&cnt, 4 * cap));
  CK(hipMalloc(&off, 4 * cap));
  CK(hipMalloc(&ncount, 4 * cap));
  CK(hipMalloc(&need, 4 * cap));
  CK(hipMalloc(&dep, 4 * cap));
  CK(hipMalloc(&n4, 128 * cap));
  CK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, off, (int)cap));
  CK(hipMalloc(&tmp, tmp_bytes));
  CK(hipMemcpy(lv[0], &root, 4, hipMemcpyHostToDevice));
  {
    int cur = 0;
    while (n > 0) {
      const dim3 G((n + 255) / 256), B(256);
      hipLaunchKernelGGL(collapse_count_kernel, G, B, 0, 0, nodes2, lv[cur], n, max_children, cnt);
      CK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, off, (int)n));
      hipLaunchKernelGGL(collapse_emit_kernel, G, B, 0, 0, nodes2, lv[cur], n, first, max_children, off, first + n,
                         lv[cur ^ 1], n4, ncount);
      CK(hipGetLastError());
      uint32_t last_off = 0, last_cnt = 0;
      CK(hipMemcpy(&last_off, off + (n - 1), 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&last_cnt, cnt + (n - 1), 4, hipMemcpyDeviceToHost));
      levels.push_back({first, n});
      first += n;
      n = last_off + last_cnt;
      total += n;
      if (total > cap) { e = hipErrorUnknown; goto done; }
      cur ^= 1;
    }
  }
  for (size_t k = levels.size(); k-- > 0;) {
    const uint32_t lf = levels[k].first, ln = levels[k].second;
    hipLaunchKernelGGL(collapse_need_kernel, dim3((ln + 255) / 256), dim3(256), 0, 0, n4, lf, ln, ncount, need, dep);
  }
  CK(hipGetLastError());
  CK(hipMemcpy(max_stack, need, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(depth4, dep, 4, hipMemcpyDeviceToHost));
  *num4 = first;
  *nodes4 = reinterpret_cast<float4*>(n4);
  n4 = nullptr;
done:
#undef CK
  for (int k = 0; k < 2; ++k) (void)hipFree(lv[k]);
  (void)hipFree(cnt);
  (void)hipFree(off);
  (void)hipFree(ncount);
  (void)hipFree(need);
  (void)hipFree(dep);
  (void)hipFree(n4);
  (void)hipFree(tmp);
  return e;
}

}  // namespace ptgs
