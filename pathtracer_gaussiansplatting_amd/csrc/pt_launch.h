// pt_launch.h — host-visible launch interface of the path-tracer kernels (pt_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include "pt_device.h"

namespace ptgs {

// RayPushConstant fields read by rt_datacollect/raygen.rgen:13-19
struct TorusParams {
  float model[16];
  float major_radius, minor_radius, height;
};

struct ViewMat {  // ubo.view (column-major)
  float m[16];
};

hipError_t launch_pt_depth(const DevScene& sc, const CamParams& cp, const ViewMat& vm, float* depth, uint32_t W,
                           uint32_t H, uint32_t row0, uint32_t row1, uint32_t frame, hipStream_t stream);

// The megakernel's tile schedule: per-tile times of the last launch and the order built from them
// (tiles that took longest first); owned by the context, valid for the grid (gx, gy) it was recorded
// on and used only by launches on the stream that recorded it (another stream's order kernel could
// rewrite `order` while a launch reads it); the schedule moves to a new stream once the old one is idle
struct PtSched {
  uint32_t* cost = nullptr;
  uint32_t* order = nullptr;
  uint32_t cap = 0, gx = 0, gy = 0;
  hipStream_t stream = nullptr;
  bool owned = false;  // `stream` holds the schedule
};
void free_pt_sched(PtSched& ps);

hipError_t launch_pt_camera(const DevScene& sc, const CamParams& cp, float* accum, uint32_t W, uint32_t H,
                            uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0, uint32_t stride,
                            uint32_t mode, unsigned long long* counters, bool stats, PtSched* ps,
                            hipStream_t stream);

hipError_t launch_pt_torus(const DevScene& sc, const CamParams& cp, const TorusParams& tp,
                           const ptgs_ray_sample* samples, uint32_t n, uint32_t side, uint32_t frame,
                           ptgs_hitdata* hits, unsigned long long* counters, bool stats, hipStream_t stream);

}  // namespace ptgs
