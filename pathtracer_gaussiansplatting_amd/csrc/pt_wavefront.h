// pt_wavefront.h — host interface of the wavefront path tracer (pt_wavefront.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pt_device.h"

// rays per wave in the persistent extend / shadow kernels (each wave walks its own run of the queue,
// refilling finished lanes); shade-kernel workgroups (grid-stride over the queue)
#ifndef PTGS_WF_RAYS_PER_WAVE
#define PTGS_WF_RAYS_PER_WAVE 256u
#endif
#ifndef PTGS_WF_SHADE_BLOCKS
#define PTGS_WF_SHADE_BLOCKS 4096u
#endif

namespace ptgs {

struct WfArgs {
  uint32_t W, H, row0, row1;
  uint32_t tiles_x;  // 8x8 pixel tiles per row
  uint32_t slots;    // pixel slots of the row range (whole tiles)
  float4* st_thr;    // (throughput, last_pdf)
  float4* st_w;      // (payload weight, hit_flag)
  float4* st_acc;    // (acc, max_depth)
};

// device buffers, grown on demand and reused across calls
struct WfWorkspace {
  void* q[2] = {nullptr, nullptr};
  size_t q_bytes[2] = {0, 0};
  void* hits = nullptr;
  size_t hits_bytes = 0;
  void* sh = nullptr;
  size_t sh_bytes = 0;
  void* st = nullptr;
  size_t st_bytes = 0;
  void* cnt = nullptr;
  size_t cnt_bytes = 0;
};

void wf_workspace_free(WfWorkspace& w);

// ptgs_trace_camera through the wavefront stages: `spp` samples (frames frame0 + s * stride) over
// pixel rows [row0, row1), accumulated into accum (running mean or SUM) exactly as pt_camera_kernel
hipError_t launch_pt_wavefront(WfWorkspace& w, const DevScene& sc, const CamParams& cp, float* accum, uint32_t W,
                               uint32_t H, uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0,
                               uint32_t stride, uint32_t mode, unsigned long long* counters, bool stats,
                               hipStream_t s);

}  // namespace ptgs
