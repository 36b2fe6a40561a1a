// bvh.h — host BVH2 builder (binned SAH), replacing the driver-built BLAS/TLAS of the reference
// (buildBlas engine.cpp:534-655, ePreferFastTrace; initStaticTlas :1385-1520).
//
// Device layout (64 B per interior node, the two child boxes live in the parent so one node fetch
// tests both children):
//   f4[0] = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//   f4[1] = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//   f4[2] = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//   f4[3] = (child0, child1, 0, 0) as int bits: >= 0 interior node index; < 0 leaf = ~L with
//           L = (count-1) << 27 | first_triangle (count <= 16, first < 2^27)
// Triangle records (48 B, in leaf order): (v0, mesh) (v1-v0, prim) (v2-v0, gid) — the int fields
// are stored as float bit patterns.
#pragma once

#include <stdint.h>
#include <vector>

namespace ptgs {

struct BuildTri {
  float v0[3], v1[3], v2[3];
  uint32_t mesh, prim, gid;
  uint32_t flags;  // bit0 non-opaque
};

struct BvhOut {
  std::vector<float> nodes;     // 16 floats per node
  std::vector<float> tris;      // 12 floats per triangle
  std::vector<uint32_t> tri_flags;
  uint32_t num_nodes = 0;
  uint32_t depth = 0;
  uint32_t max_leaf = 0;
};

// max_leaf_size <= 16; the tree depth is bounded by max_depth (>= log2(n / max_leaf_size) + 2)
void build_bvh(const std::vector<BuildTri>& tris, int max_leaf_size, uint32_t max_depth, BvhOut& out);

// 4-wide collapse of a BVH2 (the layout above): each 4-wide node takes the children of a BVH2 node,
// repeatedly opening its largest-area interior child until it has 4 (leaves keep their encoding).
// Layout, 128 B per node (8 float4): lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4],
// child[4] (int bits, as in BVH2), unused. Empty slots are point boxes at 1e30 (every ray misses).
// max_stack: traversal stack entries the tree can need (sum over a path of children - 1).
// max_children (2..4) caps the fan-out (callers retry with fewer when max_stack would not fit).
void collapse_bvh4(const std::vector<float>& nodes2, std::vector<float>& nodes4, uint32_t& num_nodes4,
                   uint32_t& max_stack, uint32_t& depth4, int max_children = 4);

}  // namespace ptgs
