// splat.h — Gaussian-splatting / point-splat workspace owned by a ptgs_ctx (see splat.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ptgs/ptgs.h"

namespace ptgs {

struct SplatWorkspace;
SplatWorkspace* splat_workspace_create();
void splat_workspace_destroy(SplatWorkspace* w);

// Front end on a second stream (PTGS_FLAG_SPLAT_OVERLAP, fused frames): the front end (and, with
// own_order, the blend's tile order from this frame's own pair counts) runs on `fe` once `wait` has
// completed, or (wait null) once the word wait_flag holds at least wait_ordinal (a stream wait-value packet:
// the blend after the workspace's last one has started, SplatSeq); `done` is recorded behind it and the
// caller's stream waits for it before the blend. So the front end of frame k overlaps the blend of frame
// k - 1 (another workspace) on the caller's stream.
struct SplatOverlap {
  hipStream_t fe;
  hipEvent_t wait, done;
  unsigned long long* wait_flag;
  unsigned long long wait_ordinal;
  bool own_order;
};
// The blend ordinals of a context that overlaps frames: the first workgroup of the blend of this call stores
// `ordinal` in *flag (signal memory) when it starts. Blends run in the caller's stream's order, each kernel
// after the previous one has ended (its kernel-end cache write-back included), so ordinal n in the flag means
// every earlier blend has finished. `launched` is set when a blend was launched with it.
struct SplatSeq {
  unsigned long long* flag;
  unsigned long long ordinal;
  bool launched;
};

// view/mvp column-major float[16]; p00 = proj[0][0], p11 = proj[1][1] (negative: Vulkan y-down)
// depth / under (both null, or both device arrays of W*H): the hybrid "over" composite
// ov: null, or the front-end stream of an overlapped frame (see SplatOverlap; ignored by three-launch frames)
hipError_t splat_gaussians(SplatWorkspace* w, const ptgs_gaussians* g, const float* view, const float* mvp, float p00,
                           float p11, uint32_t W, uint32_t H, const float bg[3], const float* depth,
                           const float* under, uint32_t tile_row_begin, uint32_t tile_row_end, float* out,
                           ptgs_splat_stats* stats, bool time_stages, bool publish, bool publish_tight, hipStream_t s,
                           uint32_t* report,  // report: bit 0 an earlier frame was left incomplete, bit 1 ids >= N
                           const SplatOverlap* ov = nullptr, SplatSeq* seq = nullptr);
hipError_t splat_stage_ms(SplatWorkspace* w, float* out_ms);
// 3D Morton order of the means: a reordered copy + the original indices (synchronises s)
hipError_t splat_sort_spatial(const ptgs_gaussians* g, float* means, float* scales, float* rots, float* opac,
                              float* colors, uint32_t* ids, hipStream_t s);
// per 256-Gaussian chunk: box of the means + largest scale (8 floats; stream-ordered)
hipError_t splat_chunk_bounds(const ptgs_gaussians* g, float* bounds, hipStream_t s);
// grow the pair buffers and the spill pool to at least `pairs` (frees / reallocates: waits for the device)
hipError_t splat_reserve(SplatWorkspace* w, uint32_t pairs);
struct SplatStatusOut {
  uint32_t incomplete;        // frames with a tile the spill pool could not hold (since the last clear)
  uint32_t capacity;          // pair buffer
  uint32_t last_pairs;        // the latest pair count a frame published
  uint32_t spilled_tiles;     // tiles completed through the spill pool (since the last clear)
  uint32_t incomplete_tiles;  // tiles left at the background (pool exhausted; since the last clear)
  uint32_t spill_capacity;    // spill pool (pairs)
  uint32_t spill_demand;      // the largest spill demand of a frame so far (pairs)
};
// call after the workspace's stream has drained (reads device counters)
hipError_t splat_status(SplatWorkspace* w, bool clear, SplatStatusOut* out);
// the latest pair count any frame of this workspace published (a hint: no wait)
uint32_t splat_pair_hint(const SplatWorkspace* w);
// the latest frame's touched (workgroup, tile) runs and whether it ran the fused front end
void splat_front_end_info(const SplatWorkspace* w, uint32_t* touched_runs, uint32_t* fused);
void splat_get_buffers(const SplatWorkspace* w, ptgs_splat_buffers* out);
// the latest frame's fused per-tile slot rows (its front end's unsorted keys) and their capacity (0: not fused)
void splat_get_tile_rows(const SplatWorkspace* w, const unsigned long long** rows, uint32_t* cap);
hipError_t splat_point_keys(SplatWorkspace* w, size_t npix, unsigned long long** keys);

// GLSL mat4 * mat4, column-major, fixed evaluation order ((a0*b0 + a1*b1) + a2*b2) + a3*b3
inline void mat4_mul(const float* a, const float* b, float* out) {
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r)
      out[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) + a[2 * 4 + r] * b[c * 4 + 2]) +
                       a[3 * 4 + r] * b[c * 4 + 3];
}

}  // namespace ptgs
