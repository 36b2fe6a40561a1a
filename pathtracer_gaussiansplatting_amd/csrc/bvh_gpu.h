// bvh_gpu.h — GPU LBVH builder (bvh_gpu.hip) producing the device layout of bvh.h.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "bvh.h"

namespace ptgs {

struct GpuBvh {
  float4* nodes = nullptr;       // 4 float4 per interior node
  float4* tris = nullptr;        // 3 float4 per triangle, leaf order
  uint32_t* tri_flags = nullptr;
  uint32_t num_nodes = 0;
  uint32_t depth = 0;
  uint32_t max_leaf = 0;
};

// n >= 2 triangles. hipErrorNotSupported: the tree is deeper than max_depth (out holds it; free it
// and build on the host). build_ms: device time of the build kernels.
hipError_t build_bvh_gpu(const std::vector<BuildTri>& tris, uint32_t max_depth, GpuBvh& out, float* build_ms);

// GPU binned-SAH builder (bvh_sah_gpu.hip): the host builder's algorithm (build_bvh, bvh.cpp) with
// the same float operations, so the tree (node boxes, leaf ranges) is the host tree; BVH2 node
// numbering and the triangle order inside a leaf differ. hipErrorNotSupported: unsupported input
// (build on the host).
hipError_t build_bvh_sah_gpu(const std::vector<BuildTri>& tris, uint32_t max_leaf, uint32_t max_depth, GpuBvh& out,
                             float* build_ms);

// The 4-wide collapse of a device BVH2 (collapse_bvh4 of bvh.h, same output word for word) on the
// GPU: *nodes4 is a new device allocation of *num4 nodes (128 B each); max_stack / depth4 as there.
hipError_t collapse_bvh4_gpu(const float4* nodes2, uint32_t num2, int max_children, float4** nodes4, uint32_t* num4,
                             uint32_t* max_stack, uint32_t* depth4);

}  // namespace ptgs
