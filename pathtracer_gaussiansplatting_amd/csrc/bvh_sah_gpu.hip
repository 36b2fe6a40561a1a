// bvh_sah_gpu.hip — GPU binned-SAH BVH builder (the reference relies on the driver's
// ePreferFastTrace BLAS/TLAS builds, engine.cpp:534-655 / :1385-1520). It runs the host builder's
// algorithm (bvh.cpp Builder::build: 32 centroid bins per axis, SAH cost area(L)·nL + area(R)·nR,
// leaf when n <= 4 and area·n <= 0.125·area + best, balanced split past the depth budget) with the
// same float operations, so every split sends the same triangles left / right as the host build:
// the tree, its node boxes and its leaf ranges equal the host tree's (only the order of the
// triangles inside a leaf and the BVH2 node numbering differ; the 4-wide collapse renumbers
// breadth-first, so the BVH4 nodes are identical).
//
//   phase A  (tasks of > GS_SAH_T triangles, level by level over all such tasks at once)
//            bin      one workgroup per 2048-reference chunk of one task: 3 axes x 32 bins of
//                     (box, count) in LDS (ordered-uint atomics), merged into the task's bins with
//                     global atomics; the chunk's bin counts kept for the partition offsets
//            split    one workgroup per task: the three SAH sweeps, the leaf test, the node (its two
//                     child boxes are bin unions), the child tasks (next level or phase B), their
//                     chunks, the link into the parent
//            scatter  one workgroup per chunk: left / right by the split bin, offsets from the
//                     preceding chunks' counts (deterministic), stable within the chunk; child
//                     centroid bounds by block reduction + atomics
//            copy     the task's range back from the scratch buffer
//   phase B  (tasks of <= GS_SAH_T triangles: one workgroup builds the whole subtree depth-first
//            with an LDS stack, the same steps with block reductions / scans)
//   emit     triangle records in leaf order (bvh.h layout)
// The BVH2 nodes are written in the bvh.h layout (padded boxes, links); the host collapses them to
// the 4-wide layout exactly as for its own tree.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "bvh_gpu.h"

#ifndef PTGS_BVH_CT
#define PTGS_BVH_CT 0.125f
#endif

namespace ptgs {

namespace {

constexpr int NB = 32;               // bins per axis (bvh.cpp NB)
constexpr uint32_t CH = 2048;        // references per phase-A chunk
#ifndef PTGS_SAH_T
#define PTGS_SAH_T 1024
#endif
constexpr uint32_t GS_SAH_T = PTGS_SAH_T;  // phase-A / phase-B boundary (task size)
constexpr int BT = 256;              // threads per workgroup
constexpr uint32_t EMPTY_LO = 0xFFFFFFFFu, EMPTY_HI = 0u;
constexpr int SB_STACK = 48;         // phase-B LDS task stack (depth <= max_depth + 1)

__device__ __forceinline__ uint32_t f2o(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }

struct Box {
  float lo[3], hi[3];
};
__device__ __forceinline__ void box_reset(Box& b) {
  for (int a = 0; a < 3; ++a) { b.lo[a] = __builtin_huge_valf(); b.hi[a] = -__builtin_huge_valf(); }
}
// std::min / std::max as bvh.cpp Box::grow uses them: (b < a) ? b : a
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ void box_grow(Box& b, const Box& o) {
  for (int a = 0; a < 3; ++a) { b.lo[a] = smin(b.lo[a], o.lo[a]); b.hi[a] = smax(b.hi[a], o.hi[a]); }
}
__device__ __forceinline__ float box_area(const Box& b) {  // bvh.cpp Box::area
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (dx < 0 || dy < 0 || dz < 0) return 0.0f;
  return 2.0f * (dx * dy + dy * dz + dz * dx);
}

// A reference: (box lo, triangle index bits) (box hi, 0); centroid = 0.5 (lo + hi) (bvh.cpp Ref::c)
struct RefBuf {
  float4* lo;
  float4* hi;
};
__device__ __forceinline__ float centroid(const float4& lo, const float4& hi, int a) {
  const float l = a == 0 ? lo.x : (a == 1 ? lo.y : lo.z), h = a == 0 ? hi.x : (a == 1 ? hi.y : hi.z);
  return 0.5f * (l + h);
}
__device__ __forceinline__ int bin_of(float c, float lo, float scale) {  // bvh.cpp: (int)((c - lo) * scale), clamped
  int k = (int)((c - lo) * scale);
  return min(NB - 1, max(0, k));
}

// Phase-A task. cb = centroid bounds as ordered uints (atomics of the parent's scatter).
struct Task {
  uint32_t begin, end, depth;
  int32_t parent;  // BVH2 node whose child slot `side` this task fills (-1: root)
  uint32_t side;
  uint32_t cb_lo[3], cb_hi[3];
  uint32_t chunk0, nchunks;  // this task's chunks
};
// The split decided for a phase-A task (read by its chunks' scatter)
struct Split {
  int32_t axis;        // -1: no partition (leaf / moved to phase B)
  int32_t bin;
  float lo, scale;     // the binning of `axis`
  uint32_t nleft;
  int32_t child_task[2];  // next-level phase-A task index of each side, -1 if the side is not one
};
struct Chunk {
  uint32_t task, begin, end;
};
struct PTask {  // phase-B task
  uint32_t begin, end, depth;
  int32_t parent;
  uint32_t side;
};
struct Global {
  uint32_t nodes;          // BVH2 nodes allocated (root = 0)
  uint32_t next_tasks;     // phase-A tasks of the next level
  uint32_t next_chunks;    // their chunks
  uint32_t ptasks;         // phase-B tasks
  uint32_t depth;          // max depth (bvh.cpp Builder::depth)
  uint32_t max_leaf;       // largest leaf
  uint32_t error;          // unsupported input (caller falls back to the host build)
  uint32_t maxabs;         // float bits of max |coordinate|
};

// host padding rule (bvh.cpp Builder::padded)
__device__ __forceinline__ void pad_box(const Box& b, float pad_abs, float* lo, float* hi) {
  const float ext = fmaxf(b.hi[0] - b.lo[0], fmaxf(b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]));
  const float p = ext * 1e-5f + pad_abs;
  for (int a = 0; a < 3; ++a) { lo[a] = b.lo[a] - p; hi[a] = b.hi[a] + p; }
}
// node layout (bvh.h): f4[0] = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y), f4[1] = same for c1,
// f4[2] = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z), f4[3] = (link0, link1, 0, 0)
__device__ __forceinline__ void write_node_boxes(float4* nodes, uint32_t idx, const Box& b0, const Box& b1, float pad_abs) {
  float l0[3], h0[3], l1[3], h1[3];
  pad_box(b0, pad_abs, l0, h0);
  pad_box(b1, pad_abs, l1, h1);
  float4* o = nodes + 4 * (size_t)idx;
  o[0] = make_float4(l0[0], h0[0], l0[1], h0[1]);
  o[1] = make_float4(l1[0], h1[0], l1[1], h1[1]);
  o[2] = make_float4(l0[2], h0[2], l1[2], h1[2]);
  o[3].z = 0.0f;
  o[3].w = 0.0f;
}
__device__ __forceinline__ void write_link(float4* nodes, int32_t parent, uint32_t side, int32_t link) {
  float* f = reinterpret_cast<float*>(nodes + 4 * (size_t)parent + 3);
  f[side] = __int_as_float(link);
}
__device__ __forceinline__ int32_t leaf_link(uint32_t begin, uint32_t count) {  // bvh.cpp make_leaf
  return ~(int32_t)(((count - 1u) << 27) | begin);
}

// The host's SAH sweeps (bvh.cpp :98-118) by 32 lanes of one wave, one axis per pass: prefix / suffix unions by
// shuffle scans (min / max are exact, so every union equals the sequential one), the costs of the
// host formula per split candidate, then the first minimum in (axis, bin) order (the host's strict
// "<" across bins, then across axes). Called by every lane of one wave; lanes >= 32 idle.
__device__ __noinline__ void sweep_wave(const uint32_t* bins /* [3][NB][7] */, const bool on[3], float& best_cost, int& best_axis,
                           int& best_bin) {
  const int lane = (int)(threadIdx.x & 63u), k = lane & 31;
  float bc = __builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int a = 0; a < 3; ++a) {
    if (!on[a]) continue;
    const uint32_t* b = bins + (a * NB + k) * 7;
    const uint32_t cnt = b[6];
    Box me;
    if (cnt) {
      for (int q = 0; q < 3; ++q) { me.lo[q] = o2f(b[q]); me.hi[q] = o2f(b[3 + q]); }
    } else {
      box_reset(me);
    }
    Box pre = me, suf = me;
    uint32_t pc = cnt, sc = cnt;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
      Box up, dn;
      for (int q = 0; q < 3; ++q) {
        up.lo[q] = __shfl_up(pre.lo[q], off, 32); up.hi[q] = __shfl_up(pre.hi[q], off, 32);
        dn.lo[q] = __shfl_down(suf.lo[q], off, 32); dn.hi[q] = __shfl_down(suf.hi[q], off, 32);
      }
      const uint32_t uc = __shfl_up(pc, off, 32), dc = __shfl_down(sc, off, 32);
      if (k >= off) { box_grow(pre, up); pc += uc; }
      if (k + off < 32) { box_grow(suf, dn); sc += dc; }
    }
    // candidate k: left = bins [0, k], right = bins [k + 1, NB)
    Box rs;
    for (int q = 0; q < 3; ++q) { rs.lo[q] = __shfl_down(suf.lo[q], 1, 32); rs.hi[q] = __shfl_down(suf.hi[q], 1, 32); }
    const uint32_t rc = __shfl_down(sc, 1, 32);
    if (k < NB - 1 && pc != 0 && rc != 0) {
      const float cost = box_area(pre) * (float)pc + box_area(rs) * (float)rc;
      if (cost < bc) { bc = cost; bi = a * NB + k; }
    }
  }
  // first minimum over (cost, axis * NB + bin)
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    const float oc = __shfl_xor(bc, off, 32);
    const int oi = __shfl_xor(bi, off, 32);
    if (oc < bc || (oc == bc && oi < bi)) { bc = oc; bi = oi; }
  }
  best_cost = bc;
  best_axis = bi == 0x7fffffff ? -1 : bi / NB;
  best_bin = bi == 0x7fffffff ? -1 : bi % NB;
}

__device__ __forceinline__ Box bins_union(const uint32_t* bins, int k0, int k1) {  // bins [k0, k1]
  Box acc;
  box_reset(acc);
  for (int k = k0; k <= k1; ++k) {
    const uint32_t* b = bins + 7 * k;
    if (!b[6]) continue;
    Box bb;
    for (int a = 0; a < 3; ++a) { bb.lo[a] = o2f(b[a]); bb.hi[a] = o2f(b[3 + a]); }
    box_grow(acc, bb);
  }
  return acc;
}

// block reductions of 256 work-items (4 waves); s: >= 4 * 12 floats of LDS
__device__ __forceinline__ void block_box_reduce(Box& b, Box& c, float* s) {
  float v[12];
  for (int a = 0; a < 3; ++a) { v[a] = b.lo[a]; v[3 + a] = b.hi[a]; v[6 + a] = c.lo[a]; v[9 + a] = c.hi[a]; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    for (int i = 0; i < 12; ++i) {
      const float o = __shfl_xor(v[i], off, 64);
      v[i] = (i % 6) < 3 ? fminf(v[i], o) : fmaxf(v[i], o);
    }
  __syncthreads();
  if ((threadIdx.x & 63u) == 0)
    for (int i = 0; i < 12; ++i) s[(threadIdx.x >> 6) * 12 + i] = v[i];
  __syncthreads();
  for (int i = 0; i < 12; ++i) {
    float r = s[i];
    for (int w = 1; w < BT / 64; ++w) r = (i % 6) < 3 ? fminf(r, s[w * 12 + i]) : fmaxf(r, s[w * 12 + i]);
    v[i] = r;
  }
  __syncthreads();
  for (int a = 0; a < 3; ++a) { b.lo[a] = v[a]; b.hi[a] = v[3 + a]; c.lo[a] = v[6 + a]; c.hi[a] = v[9 + a]; }
}
// exclusive scan of a 0/1 flag over the block; returns the prefix, total in *tot
__device__ __forceinline__ uint32_t block_scan1(bool f, uint32_t* s, uint32_t* tot) {
  const unsigned long long m = __ballot(f);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t in_wave = __popcll(m & ((1ull << lane) - 1ull));
  __syncthreads();
  if (lane == 0) s[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t base = 0, t = 0;
  for (uint32_t k = 0; k < BT / 64; ++k) {
    if (k < w) base += s[k];
    t += s[k];
  }
  *tot = t;
  return base + in_wave;
}

// ------------------------------------------------------------------------------------------------
__global__ void sah_refs_kernel(const BuildTri* __restrict__ tris, uint32_t n, RefBuf refs, Global* g, Task* root) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  float lo[3], hi[3], ma = 0.0f, cl[3], chh[3];
  for (int a = 0; a < 3; ++a) { lo[a] = hi[a] = 0.0f; cl[a] = __builtin_huge_valf(); chh[a] = -__builtin_huge_valf(); }
  if (i < n) {
    const BuildTri t = tris[i];
    for (int a = 0; a < 3; ++a) {  // bvh.cpp :184-189 (reset, grow v0, v1, v2)
      lo[a] = smin(__builtin_huge_valf(), t.v0[a]);
      hi[a] = smax(-__builtin_huge_valf(), t.v0[a]);
      lo[a] = smin(lo[a], t.v1[a]); hi[a] = smax(hi[a], t.v1[a]);
      lo[a] = smin(lo[a], t.v2[a]); hi[a] = smax(hi[a], t.v2[a]);
      const float c = 0.5f * (lo[a] + hi[a]);
      cl[a] = c; chh[a] = c;
      ma = fmaxf(ma, fmaxf(fabsf(lo[a]), fabsf(hi[a])));
    }
    refs.lo[i] = make_float4(lo[0], lo[1], lo[2], __uint_as_float(i));
    refs.hi[i] = make_float4(hi[0], hi[1], hi[2], 0.0f);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    for (int a = 0; a < 3; ++a) { cl[a] = fminf(cl[a], __shfl_xor(cl[a], off, 64)); chh[a] = fmaxf(chh[a], __shfl_xor(chh[a], off, 64)); }
    ma = fmaxf(ma, __shfl_xor(ma, off, 64));
  }
  __shared__ float s_r[4][7];
  if ((threadIdx.x & 63u) == 0) {
    for (int a = 0; a < 3; ++a) { s_r[threadIdx.x >> 6][a] = cl[a]; s_r[threadIdx.x >> 6][3 + a] = chh[a]; }
    s_r[threadIdx.x >> 6][6] = ma;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      for (int a = 0; a < 3; ++a) { cl[a] = fminf(cl[a], s_r[w][a]); chh[a] = fmaxf(chh[a], s_r[w][3 + a]); }
      ma = fmaxf(ma, s_r[w][6]);
    }
    for (int a = 0; a < 3; ++a) { atomicMin(&root->cb_lo[a], f2o(cl[a])); atomicMax(&root->cb_hi[a], f2o(chh[a])); }
    atomicMax(&g->maxabs, __float_as_uint(ma));
  }
}

// empty bins: lo fields EMPTY_LO, hi fields EMPTY_HI, counts 0 (7 words per bin)
__global__ void sah_bins_init_kernel(uint32_t* __restrict__ tbins, uint32_t words) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < words) tbins[i] = (i % 7) < 3 ? EMPTY_LO : EMPTY_HI;
}

// phase A: bins of one chunk (one task), merged into the task's bins; the chunk's counts kept
__global__ __launch_bounds__(BT) void sah_bin_kernel(RefBuf refs, const Chunk* __restrict__ chunks, uint32_t nchunks,
                                                     const Task* __restrict__ tasks, uint32_t* __restrict__ tbins,
                                                     uint32_t* __restrict__ ccount) {
  if (blockIdx.x >= nchunks) return;
  __shared__ uint32_t sb[3 * NB * 7];
  const Chunk ck = chunks[blockIdx.x];
  const Task& t = tasks[ck.task];
  for (uint32_t i = threadIdx.x; i < 3 * NB * 7; i += BT) {
    const uint32_t f = i % 7;
    sb[i] = f < 3 ? EMPTY_LO : (f < 6 ? EMPTY_HI : 0u);
  }
  float clo[3], scale[3];
  bool on[3];
  for (int a = 0; a < 3; ++a) {
    clo[a] = o2f(t.cb_lo[a]);
    const float ext = o2f(t.cb_hi[a]) - clo[a];
    on[a] = ext > 0.0f;
    scale[a] = on[a] ? (float)NB / ext : 0.0f;
  }
  __syncthreads();
  for (uint32_t i = ck.begin + threadIdx.x; i < ck.end; i += BT) {
    const float4 lo = refs.lo[i], hi = refs.hi[i];
    const uint32_t blo[3] = {f2o(lo.x), f2o(lo.y), f2o(lo.z)}, bhi[3] = {f2o(hi.x), f2o(hi.y), f2o(hi.z)};
    for (int a = 0; a < 3; ++a) {
      if (!on[a]) continue;
      uint32_t* b = sb + (a * NB + bin_of(centroid(lo, hi, a), clo[a], scale[a])) * 7;
      for (int q = 0; q < 3; ++q) { atomicMin(&b[q], blo[q]); atomicMax(&b[3 + q], bhi[q]); }
      atomicAdd(&b[6], 1u);
    }
  }
  __syncthreads();
  uint32_t* tb = tbins + (size_t)ck.task * 3 * NB * 7;
  for (uint32_t i = threadIdx.x; i < 3 * NB * 7; i += BT) {
    const uint32_t f = i % 7, v = sb[i];
    if (f == 6) {
      if (v) atomicAdd(&tb[i], v);
      ccount[(size_t)blockIdx.x * 3 * NB + i / 7] = v;
    } else if (f < 3) {
      if (v != EMPTY_LO) atomicMin(&tb[i], v);
    } else if (v != EMPTY_HI) {
      atomicMax(&tb[i], v);
    }
  }
}

// phase A: the split of each task (one workgroup of 64 per task)
__global__ __launch_bounds__(64) void sah_split_kernel(const Task* __restrict__ tasks, uint32_t ntasks, const uint32_t* __restrict__ tbins,
                                                       Split* __restrict__ splits, Task* __restrict__ next, Chunk* __restrict__ next_chunks,
                                                       PTask* __restrict__ ptasks, Global* __restrict__ g, float4* __restrict__ nodes,
                                                       uint32_t max_leaf, uint32_t max_depth) {
  const uint32_t ti = blockIdx.x;
  if (ti >= ntasks) return;
  const Task t = tasks[ti];
  const uint32_t* bins = tbins + (size_t)ti * 3 * NB * 7;
  const uint32_t n = t.end - t.begin;
  float ext[3];
  for (int a = 0; a < 3; ++a) ext[a] = o2f(t.cb_hi[a]) - o2f(t.cb_lo[a]);
  const bool on[3] = {ext[0] > 0.0f, ext[1] > 0.0f, ext[2] > 0.0f};
  float w_cost;
  int w_axis, w_bin;
  sweep_wave(bins, on, w_cost, w_axis, w_bin);
  if (threadIdx.x != 0) return;
  Split sp;
  sp.axis = -1; sp.bin = -1; sp.lo = 0.0f; sp.scale = 0.0f; sp.nleft = 0; sp.child_task[0] = sp.child_task[1] = -1;
  atomicMax(&g->depth, t.depth);
  int axis = 0;  // widest centroid extent (bvh.cpp :81-85)
  if (ext[1] > ext[axis]) axis = 1;
  if (ext[2] > ext[axis]) axis = 2;
  uint32_t need = 0;
  while (((uint64_t)max_leaf << need) < n) need++;
  int best_axis = -1, best_bin = -1;
  float best_cost = __builtin_huge_valf();
  const bool sah = ext[axis] > 0.0f && t.depth + need + 1 < max_depth;
  if (sah) { best_cost = w_cost; best_axis = w_axis; best_bin = w_bin; }
  // the node's box: union of all bins of an axis with non-zero extent (every reference is binned there)
  const int ba = ext[0] > 0.0f ? 0 : (ext[1] > 0.0f ? 1 : 2);
  if (!sah || best_axis < 0 || ext[ba] <= 0.0f) {
    // no SAH split here (depth budget / degenerate centroids): the whole subtree goes to phase B
    const uint32_t k = atomicAdd(&g->ptasks, 1u);
    ptasks[k] = PTask{t.begin, t.end, t.depth, t.parent, t.side};
    splits[ti] = sp;
    return;
  }
  const Box out_box = bins_union(bins + ba * NB * 7, 0, NB - 1);
  const float leaf_cost = box_area(out_box) * (float)n;
  const float split_cost = PTGS_BVH_CT * box_area(out_box) + best_cost;
  if (n <= max_leaf && leaf_cost <= split_cost && t.depth > 0) {  // (n > GS_SAH_T here: never)
    atomicMax(&g->max_leaf, n);
    if (t.parent >= 0) write_link(nodes, t.parent, t.side, leaf_link(t.begin, n));
    splits[ti] = sp;
    return;
  }
  const uint32_t* ab = bins + best_axis * NB * 7;
  uint32_t nl = 0;
  for (int k = 0; k <= best_bin; ++k) nl += ab[7 * k + 6];
  const Box b0 = bins_union(ab, 0, best_bin), b1 = bins_union(ab, best_bin + 1, NB - 1);
  const uint32_t idx = t.parent < 0 ? 0u : atomicAdd(&g->nodes, 1u);
  const float pad_abs = __uint_as_float(g->maxabs) * 4e-7f + 1e-30f;
  write_node_boxes(nodes, idx, b0, b1, pad_abs);
  if (t.parent >= 0) write_link(nodes, t.parent, t.side, (int32_t)idx);
  sp.axis = best_axis;
  sp.bin = best_bin;
  sp.lo = o2f(t.cb_lo[best_axis]);
  sp.scale = (float)NB / ext[best_axis];
  sp.nleft = nl;
  const uint32_t cb[2] = {t.begin, t.begin + nl}, ce[2] = {t.begin + nl, t.end};
  for (int s = 0; s < 2; ++s) {
    const uint32_t cn = ce[s] - cb[s];
    if (cn > GS_SAH_T) {
      const uint32_t k = atomicAdd(&g->next_tasks, 1u);
      const uint32_t nck = (cn + CH - 1) / CH;
      const uint32_t c0 = atomicAdd(&g->next_chunks, nck);
      Task c;
      c.begin = cb[s]; c.end = ce[s]; c.depth = t.depth + 1; c.parent = (int32_t)idx; c.side = (uint32_t)s;
      for (int a = 0; a < 3; ++a) { c.cb_lo[a] = EMPTY_LO; c.cb_hi[a] = EMPTY_HI; }
      c.chunk0 = c0; c.nchunks = nck;
      next[k] = c;
      for (uint32_t j = 0; j < nck; ++j) next_chunks[c0 + j] = Chunk{k, cb[s] + j * CH, min(ce[s], cb[s] + (j + 1) * CH)};
      sp.child_task[s] = (int32_t)k;
    } else {
      const uint32_t k = atomicAdd(&g->ptasks, 1u);
      ptasks[k] = PTask{cb[s], ce[s], t.depth + 1, (int32_t)idx, (uint32_t)s};
    }
  }
  splits[ti] = sp;
}

// phase A: partition of one chunk into the scratch buffer
__global__ __launch_bounds__(BT) void sah_scatter_kernel(RefBuf refs, RefBuf alt, const Chunk* __restrict__ chunks, uint32_t nchunks,
                                                         const Task* __restrict__ tasks, const Split* __restrict__ splits,
                                                         const uint32_t* __restrict__ ccount, Task* __restrict__ next) {
  if (blockIdx.x >= nchunks) return;
  __shared__ uint32_t s_scan[BT / 64];
  __shared__ float s_red[(BT / 64) * 12];
  __shared__ uint32_t s_off[2];
  const Chunk ck = chunks[blockIdx.x];
  const Split sp = splits[ck.task];
  if (sp.axis < 0) return;
  const Task& t = tasks[ck.task];
  if (threadIdx.x < 2) {  // left / right refs of the task's earlier chunks
    uint32_t l = 0, all = 0;
    for (uint32_t c = t.chunk0; c < blockIdx.x; ++c) {
      const uint32_t* cc = ccount + (size_t)c * 3 * NB + sp.axis * NB;
      for (int k = 0; k <= sp.bin; ++k) l += cc[k];
      all += chunks[c].end - chunks[c].begin;
    }
    s_off[threadIdx.x] = threadIdx.x == 0 ? t.begin + l : t.begin + sp.nleft + (all - l);
  }
  __syncthreads();
  uint32_t offl = s_off[0], offr = s_off[1];
  Box cbs[2];
  box_reset(cbs[0]);
  box_reset(cbs[1]);
  for (uint32_t base = ck.begin; base < ck.end; base += BT) {
    const uint32_t i = base + threadIdx.x;
    const bool v = i < ck.end;
    float4 lo = make_float4(0, 0, 0, 0), hi = lo;
    bool left = false;
    if (v) {
      lo = refs.lo[i];
      hi = refs.hi[i];
      left = bin_of(centroid(lo, hi, sp.axis), sp.lo, sp.scale) <= sp.bin;
    }
    uint32_t tl;
    const uint32_t pl = block_scan1(v && left, s_scan, &tl);
    const uint32_t nv = min((uint32_t)BT, ck.end - base);
    if (v) {
      const uint32_t dst = left ? offl + pl : offr + (threadIdx.x - pl);
      alt.lo[dst] = lo;
      alt.hi[dst] = hi;
      Box& cb = cbs[left ? 0 : 1];
      for (int a = 0; a < 3; ++a) {
        const float c = centroid(lo, hi, a);
        cb.lo[a] = fminf(cb.lo[a], c);
        cb.hi[a] = fmaxf(cb.hi[a], c);
      }
    }
    offl += tl;
    offr += nv - tl;
  }
  block_box_reduce(cbs[0], cbs[1], s_red);
  if (threadIdx.x == 0)
    for (int s = 0; s < 2; ++s) {
      if (sp.child_task[s] < 0 || cbs[s].lo[0] > cbs[s].hi[0]) continue;
      Task& c = next[sp.child_task[s]];
      for (int a = 0; a < 3; ++a) { atomicMin(&c.cb_lo[a], f2o(cbs[s].lo[a])); atomicMax(&c.cb_hi[a], f2o(cbs[s].hi[a])); }
    }
}

__global__ __launch_bounds__(BT) void sah_copy_kernel(RefBuf refs, RefBuf alt, const Chunk* __restrict__ chunks, uint32_t nchunks,
                                                      const Split* __restrict__ splits) {
  if (blockIdx.x >= nchunks) return;
  const Chunk ck = chunks[blockIdx.x];
  if (splits[ck.task].axis < 0) return;
  for (uint32_t i = ck.begin + threadIdx.x; i < ck.end; i += BT) {
    refs.lo[i] = alt.lo[i];
    refs.hi[i] = alt.hi[i];
  }
}

// phase B: one workgroup builds the subtree of one task, depth first
__global__ __launch_bounds__(BT) void sah_subtree_kernel(RefBuf refs, RefBuf alt, const PTask* __restrict__ ptasks, Global* __restrict__ g,
                                                         float4* __restrict__ nodes, uint32_t max_leaf, uint32_t max_depth) {
  __shared__ PTask s_stack[SB_STACK];
  __shared__ uint32_t sb[3 * NB * 7];
  __shared__ float s_red[(BT / 64) * 12];
  __shared__ uint32_t s_scan[BT / 64];
  __shared__ int s_sp;
  __shared__ int s_act;  // 0 leaf, 1 SAH split, 2 balanced split
  __shared__ int s_axis, s_bbin;
  __shared__ float s_lo, s_scale;
  __shared__ uint32_t s_nl;
  __shared__ int s_err;
  if (threadIdx.x == 0) {
    s_stack[0] = ptasks[blockIdx.x];
    s_sp = 1;
    s_err = 0;
  }
  __syncthreads();
  const float pad_abs = __uint_as_float(g->maxabs) * 4e-7f + 1e-30f;
  while (s_sp > 0) {
    const PTask t = s_stack[s_sp - 1];
    const uint32_t n = t.end - t.begin;
    __syncthreads();
    if (threadIdx.x == 0) --s_sp;
    if (threadIdx.x == 0) atomicMax(&g->depth, t.depth);
    if (n <= max_leaf && !(t.depth == 0 && n > 1)) {  // bvh.cpp :77
      if (threadIdx.x == 0) {
        atomicMax(&g->max_leaf, n);
        if (t.parent >= 0) write_link(nodes, t.parent, t.side, leaf_link(t.begin, n));
      }
      __syncthreads();
      continue;
    }
    // node box and centroid bounds (bvh.cpp :76, :79-80)
    Box ob, cb;
    box_reset(ob);
    box_reset(cb);
    for (uint32_t i = t.begin + threadIdx.x; i < t.end; i += BT) {
      const float4 lo = refs.lo[i], hi = refs.hi[i];
      const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
      for (int a = 0; a < 3; ++a) {
        ob.lo[a] = fminf(ob.lo[a], l3[a]);
        ob.hi[a] = fmaxf(ob.hi[a], h3[a]);
        const float c = 0.5f * (l3[a] + h3[a]);
        cb.lo[a] = fminf(cb.lo[a], c);
        cb.hi[a] = fmaxf(cb.hi[a], c);
      }
    }
    block_box_reduce(ob, cb, s_red);
    float ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = cb.hi[a] - cb.lo[a];
    int axis = 0;
    if (ext[1] > ext[axis]) axis = 1;
    if (ext[2] > ext[axis]) axis = 2;
    uint32_t need = 0;
    while (((uint64_t)max_leaf << need) < n) need++;
    const bool sah = ext[axis] > 0.0f && t.depth + need + 1 < max_depth;
    if (sah) {
      for (uint32_t i = threadIdx.x; i < 3 * NB * 7; i += BT) {
        const uint32_t f = i % 7;
        sb[i] = f < 3 ? EMPTY_LO : (f < 6 ? EMPTY_HI : 0u);
      }
      __syncthreads();
      float scale[3];
      for (int a = 0; a < 3; ++a) scale[a] = ext[a] > 0.0f ? (float)NB / ext[a] : 0.0f;
      for (uint32_t i = t.begin + threadIdx.x; i < t.end; i += BT) {
        const float4 lo = refs.lo[i], hi = refs.hi[i];
        const uint32_t blo[3] = {f2o(lo.x), f2o(lo.y), f2o(lo.z)}, bhi[3] = {f2o(hi.x), f2o(hi.y), f2o(hi.z)};
        for (int a = 0; a < 3; ++a) {
          if (!(ext[a] > 0.0f)) continue;
          uint32_t* b = sb + (a * NB + bin_of(centroid(lo, hi, a), cb.lo[a], scale[a])) * 7;
          for (int q = 0; q < 3; ++q) { atomicMin(&b[q], blo[q]); atomicMax(&b[3 + q], bhi[q]); }
          atomicAdd(&b[6], 1u);
        }
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const bool on[3] = {ext[0] > 0.0f, ext[1] > 0.0f, ext[2] > 0.0f};
        float best_cost;
        int best_axis, best_bin;
        sweep_wave(sb, on, best_cost, best_axis, best_bin);
        if (threadIdx.x == 0) {
        s_act = 2;
        if (best_axis >= 0) {
          const float leaf_cost = box_area(ob) * (float)n;
          const float split_cost = PTGS_BVH_CT * box_area(ob) + best_cost;
          if (n <= max_leaf && leaf_cost <= split_cost && t.depth > 0) {
            s_act = 0;
          } else {
            s_act = 1;
            s_axis = best_axis;
            s_bbin = best_bin;
            s_lo = cb.lo[best_axis];
            s_scale = scale[best_axis];
            uint32_t nl = 0;
            for (int k = 0; k <= best_bin; ++k) nl += sb[(best_axis * NB + k) * 7 + 6];
            s_nl = nl;
          }
        }
        }
      }
    } else if (threadIdx.x == 0) {
      s_act = 2;
    }
    __syncthreads();
    const int act = s_act;
    if (act == 0) {
      if (threadIdx.x == 0) {
        atomicMax(&g->max_leaf, n);
        write_link(nodes, t.parent, t.side, leaf_link(t.begin, n));
      }
      __syncthreads();
      continue;
    }
    uint32_t nl;
    if (act == 1) {
      nl = s_nl;
      const int ax = s_axis, bb = s_bbin;
      const float lo0 = s_lo, sc = s_scale;
      uint32_t offl = t.begin, offr = t.begin + nl;
      for (uint32_t base = t.begin; base < t.end; base += BT) {
        const uint32_t i = base + threadIdx.x;
        const bool v = i < t.end;
        float4 lo = make_float4(0, 0, 0, 0), hi = lo;
        bool left = false;
        if (v) {
          lo = refs.lo[i];
          hi = refs.hi[i];
          left = bin_of(centroid(lo, hi, ax), lo0, sc) <= bb;
        }
        uint32_t tl;
        const uint32_t pl = block_scan1(v && left, s_scan, &tl);
        const uint32_t nv = min((uint32_t)BT, t.end - base);
        if (v) {
          const uint32_t dst = left ? offl + pl : offr + (threadIdx.x - pl);
          alt.lo[dst] = lo;
          alt.hi[dst] = hi;
        }
        offl += tl;
        offr += nv - tl;
      }
    } else {
      // balanced split (bvh.cpp :134-147): the n/2 smallest centroids along `axis` go left; ties by
      // position (std::nth_element breaks them its own way: equal-centroid ties may differ)
      nl = n / 2;
      for (uint32_t base = t.begin; base < t.end; base += BT) {
        const uint32_t i = base + threadIdx.x;
        if (i >= t.end) continue;
        const float4 lo = refs.lo[i], hi = refs.hi[i];
        const float c = centroid(lo, hi, axis);
        uint32_t rank = 0;
        for (uint32_t j = t.begin; j < t.end; ++j) {
          const float cj = centroid(refs.lo[j], refs.hi[j], axis);
          rank += (cj < c || (cj == c && j < i)) ? 1u : 0u;
        }
        // rank is a permutation of [0, n): left keeps rank order, right too
        const uint32_t dst = t.begin + rank;
        alt.lo[dst] = lo;
        alt.hi[dst] = hi;
      }
    }
    __syncthreads();
    __threadfence_block();
    for (uint32_t i = t.begin + threadIdx.x; i < t.end; i += BT) {
      refs.lo[i] = alt.lo[i];
      refs.hi[i] = alt.hi[i];
    }
    __threadfence_block();
    __syncthreads();
    // child boxes (bvh.cpp: the children's range boxes)
    Box b0, b1;
    box_reset(b0);
    box_reset(b1);
    for (uint32_t i = t.begin + threadIdx.x; i < t.end; i += BT) {
      const float4 lo = refs.lo[i], hi = refs.hi[i];
      Box& b = i < t.begin + nl ? b0 : b1;
      b.lo[0] = fminf(b.lo[0], lo.x); b.lo[1] = fminf(b.lo[1], lo.y); b.lo[2] = fminf(b.lo[2], lo.z);
      b.hi[0] = fmaxf(b.hi[0], hi.x); b.hi[1] = fmaxf(b.hi[1], hi.y); b.hi[2] = fmaxf(b.hi[2], hi.z);
    }
    block_box_reduce(b0, b1, s_red);
    if (threadIdx.x == 0) {
      const uint32_t idx = t.parent < 0 ? 0u : atomicAdd(&g->nodes, 1u);
      write_node_boxes(nodes, idx, b0, b1, pad_abs);
      if (t.parent >= 0) write_link(nodes, t.parent, t.side, (int32_t)idx);
      if (s_sp + 2 > SB_STACK) {
        g->error = 1u;
        s_err = 1;
      } else {
        s_stack[s_sp++] = PTask{t.begin + nl, t.end, t.depth + 1, (int32_t)idx, 1u};
        s_stack[s_sp++] = PTask{t.begin, t.begin + nl, t.depth + 1, (int32_t)idx, 0u};
      }
    }
    __syncthreads();
    if (s_err) break;
  }
}

__global__ void sah_tris_kernel(const BuildTri* __restrict__ tris, const float4* __restrict__ rlo, uint32_t n,
                                float4* __restrict__ out, uint32_t* __restrict__ flags) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const BuildTri t = tris[__float_as_uint(rlo[k].w)];
  out[3 * k] = make_float4(t.v0[0], t.v0[1], t.v0[2], __uint_as_float(t.mesh));
  out[3 * k + 1] = make_float4(t.v1[0] - t.v0[0], t.v1[1] - t.v0[1], t.v1[2] - t.v0[2], __uint_as_float(t.prim));
  out[3 * k + 2] = make_float4(t.v2[0] - t.v0[0], t.v2[1] - t.v0[1], t.v2[2] - t.v0[2], __uint_as_float(t.gid));
  flags[k] = t.flags;
}

}  // namespace

hipError_t build_bvh_sah_gpu(const std::vector<BuildTri>& tris, uint32_t max_leaf, uint32_t max_depth, GpuBvh& out,
                             float* build_ms) {
  const uint32_t n = (uint32_t)tris.size();
  out = GpuBvh{};
  if (n < 2 || max_leaf < 1 || max_leaf > 16) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  BuildTri* d_tris = nullptr;
  RefBuf refs{nullptr, nullptr}, alt{nullptr, nullptr};
  Task *tasks[2] = {nullptr, nullptr};
  Chunk* chunks[2] = {nullptr, nullptr};
  Split* splits = nullptr;
  PTask* ptasks = nullptr;
  Global* g = nullptr;
  uint32_t *tbins = nullptr, *ccount = nullptr;
  float4 *nodes = nullptr, *trec = nullptr;
  uint32_t* tflags = nullptr;
  Global hg{};
  // bounds: phase-A tasks per level <= n / GS_SAH_T; chunks per level <= n / CH + tasks; phase-B tasks
  // <= n / 2 (every task holds >= 2 references... and >= 1: n); nodes <= n - 1
  const uint32_t max_tasks = n / GS_SAH_T + 2, max_chunks = n / CH + max_tasks + 1;
  const uint32_t max_nodes = n;  // interior nodes of a binary tree over n leaves: n - 1
#define CK(x) \
  if ((e = (x)) != hipSuccess) goto done
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMalloc(&d_tris, sizeof(BuildTri) * n));
  CK(hipMalloc(&refs.lo, 16ull * n));
  CK(hipMalloc(&refs.hi, 16ull * n));
  CK(hipMalloc(&alt.lo, 16ull * n));
  CK(hipMalloc(&alt.hi, 16ull * n));
  CK(hipMalloc(&tasks[0], sizeof(Task) * max_tasks));
  CK(hipMalloc(&tasks[1], sizeof(Task) * max_tasks));
  CK(hipMalloc(&chunks[0], sizeof(Chunk) * max_chunks));
  CK(hipMalloc(&chunks[1], sizeof(Chunk) * max_chunks));
  CK(hipMalloc(&splits, sizeof(Split) * max_tasks));
  CK(hipMalloc(&ptasks, sizeof(PTask) * n));
  CK(hipMalloc(&g, sizeof(Global)));
  CK(hipMalloc(&tbins, 4ull * 3 * NB * 7 * max_tasks));
  CK(hipMalloc(&ccount, 4ull * 3 * NB * max_chunks));
  CK(hipMalloc(&nodes, 64ull * max_nodes));
  CK(hipMemcpy(d_tris, tris.data(), sizeof(BuildTri) * n, hipMemcpyHostToDevice));
  {
    Global g0{};
    g0.nodes = 1;  // the root
    CK(hipMemcpy(g, &g0, sizeof(g0), hipMemcpyHostToDevice));
    Task root;
    root.begin = 0; root.end = n; root.depth = 0; root.parent = -1; root.side = 0;
    for (int a = 0; a < 3; ++a) { root.cb_lo[a] = EMPTY_LO; root.cb_hi[a] = EMPTY_HI; }
    root.chunk0 = 0; root.nchunks = (n + CH - 1) / CH;
    CK(hipMemcpy(tasks[0], &root, sizeof(root), hipMemcpyHostToDevice));
    std::vector<Chunk> rc(root.nchunks);
    for (uint32_t j = 0; j < root.nchunks; ++j) rc[j] = Chunk{0, j * CH, std::min(n, (j + 1) * CH)};
    CK(hipMemcpy(chunks[0], rc.data(), sizeof(Chunk) * rc.size(), hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(sah_refs_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d_tris, n, refs, g, tasks[0]);
  {
    uint32_t ntasks = 1, nchunks = (n + CH - 1) / CH;
    int cur = 0;
    if (n <= GS_SAH_T) {  // the root is a phase-B task
      const PTask p{0u, n, 0u, -1, 0u};
      CK(hipMemcpy(ptasks, &p, sizeof(p), hipMemcpyHostToDevice));
      const uint32_t one = 1;
      CK(hipMemcpy(&g->ptasks, &one, 4, hipMemcpyHostToDevice));
      ntasks = 0;
    }
    while (ntasks > 0) {
      CK(hipMemsetAsync(&g->next_tasks, 0, 8, 0));  // next_tasks, next_chunks
      hipLaunchKernelGGL(sah_bins_init_kernel, dim3((3 * NB * 7 * ntasks + 255) / 256), dim3(256), 0, 0, tbins,
                         3u * NB * 7u * ntasks);
      hipLaunchKernelGGL(sah_bin_kernel, dim3(nchunks), dim3(BT), 0, 0, refs, chunks[cur], nchunks, tasks[cur], tbins, ccount);
      hipLaunchKernelGGL(sah_split_kernel, dim3(ntasks), dim3(64), 0, 0, tasks[cur], ntasks, tbins, splits, tasks[cur ^ 1],
                         chunks[cur ^ 1], ptasks, g, nodes, max_leaf, max_depth);
      hipLaunchKernelGGL(sah_scatter_kernel, dim3(nchunks), dim3(BT), 0, 0, refs, alt, chunks[cur], nchunks, tasks[cur], splits,
                         ccount, tasks[cur ^ 1]);
      hipLaunchKernelGGL(sah_copy_kernel, dim3(nchunks), dim3(BT), 0, 0, refs, alt, chunks[cur], nchunks, splits);
      CK(hipGetLastError());
      CK(hipMemcpy(&hg, g, sizeof(hg), hipMemcpyDeviceToHost));
      ntasks = hg.next_tasks;
      nchunks = hg.next_chunks;
      if (ntasks > max_tasks || nchunks > max_chunks) { e = hipErrorUnknown; goto done; }
      cur ^= 1;
    }
    CK(hipMemcpy(&hg, g, sizeof(hg), hipMemcpyDeviceToHost));
    if (hg.ptasks) hipLaunchKernelGGL(sah_subtree_kernel, dim3(hg.ptasks), dim3(BT), 0, 0, refs, alt, ptasks, g, nodes, max_leaf, max_depth);
    CK(hipGetLastError());
  }
  CK(hipMalloc(&trec, 48ull * n));
  CK(hipMalloc(&tflags, 4ull * n));
  hipLaunchKernelGGL(sah_tris_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d_tris, refs.lo, n, trec, tflags);
  CK(hipGetLastError());
  CK(hipEventRecord(e1, 0));
  CK(hipMemcpy(&hg, g, sizeof(hg), hipMemcpyDeviceToHost));
  if (build_ms) (void)hipEventElapsedTime(build_ms, e0, e1);
  if (hg.error || hg.nodes > max_nodes) { e = hipErrorNotSupported; goto done; }
  out.nodes = nodes;
  out.tris = trec;
  out.tri_flags = tflags;
  out.num_nodes = hg.nodes;
  out.depth = hg.depth;
  out.max_leaf = hg.max_leaf;
  nodes = nullptr;
  trec = nullptr;
  tflags = nullptr;
  if (hg.depth >= max_depth + 1) e = hipErrorNotSupported;
done:
#undef CK
  (void)hipFree(d_tris);
  (void)hipFree(refs.lo);
  (void)hipFree(refs.hi);
  (void)hipFree(alt.lo);
  (void)hipFree(alt.hi);
  for (int k = 0; k < 2; ++k) {
    (void)hipFree(tasks[k]);
    (void)hipFree(chunks[k]);
  }
  (void)hipFree(splits);
  (void)hipFree(ptasks);
  (void)hipFree(g);
  (void)hipFree(tbins);
  (void)hipFree(ccount);
  (void)hipFree(nodes);
  (void)hipFree(trec);
  (void)hipFree(tflags);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (e != hipSuccess && e != hipErrorNotSupported) {
    (void)hipFree(out.nodes);
    (void)hipFree(out.tris);
    (void)hipFree(out.tri_flags);
    out = GpuBvh{};
  }
  return e;
}

}  // namespace ptgs
