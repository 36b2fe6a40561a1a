// xcd.h — XCD-aware block -> tile mapping (gfx950: 8 XCDs, each with its own L2).
// Workgroups are dealt round-robin over the XCDs (MI355X_MICROARCH.md: blocks b and b + 8 share one),
// so consecutive block ids land on different L2s. xcd_tile maps the linear block id b of a grid of
// n blocks to a tile index such that the blocks of one XCD cover one contiguous run of tiles
// (row-major: a horizontal strip of the image), so neighbouring tiles — which fetch the same BVH
// nodes / Gaussian records — share an L2. A bijection on [0, n) for any n.
#pragma once

#include <hip/hip_runtime.h>

namespace ptgs {

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, j = b >> 3;
  return x * q + min(x, r) + j;
}

}  // namespace ptgs
