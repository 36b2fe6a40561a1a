// pt_wavefront.h — host interface of the wavefront path tracer (pt_wavefront.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pt_device.h"

// slots per wave: the run of pixel slots each wave of the extend / shadow kernels (persistent,
// refilling finished lanes) and of the shade kernel walks
#ifndef PTGS_WF_TRACE_RUN
#define PTGS_WF_TRACE_RUN 256u
#endif
#ifndef PTGS_WF_BATCH
#define PTGS_WF_BATCH 16u  // samples per batch (a tile's samples in adjacent waves)
#endif
#ifndef PTGS_WF_REFILL
#define PTGS_WF_REFILL 16u  // idle lanes of a traversal wave that trigger a refill from its run
#endif
#ifndef PTGS_WF_SHADE_RUN
#define PTGS_WF_SHADE_RUN 256u
#endif

namespace ptgs {

struct WfArgs {
  uint32_t W, H, row0, row1;
  uint32_t tiles_x;  // 8x8 pixel tiles per row
  uint32_t slots;    // slots of the batch: whole 8x8 tiles x batch samples
  uint32_t batch;    // samples per batch
  uint32_t frame0;   // frame count of the batch's first sample
  uint32_t stride;   // frame count step between samples
  float4 *ray_o, *ray_d;          // (origin, seed) (direction, -) of the pending extension ray
  float4* hits;                   // (t, u, v, gid)
  float4 *sh_o, *sh_d, *sh_acc;   // shadow ray: (origin, tmax) (direction, seed) (acc if unoccluded, -)
  float4* st_thr;                 // (throughput, last_pdf)
  float4* st_w;                   // (payload weight, hit_flag)
  float4* st_acc;                 // (acc, max_depth)
  uint8_t* flags;                 // bit 0 extension ray pending, bit 1 shadow ray pending
  uint32_t* part;                 // per-workgroup partial ray / sample counts [counter][block]
  uint32_t part_stride;
  uint32_t* live;                 // [2 d] extension rays pending at depth d, [2 d + 1] shadow rays
  int* ovf;                       // traversal-stack overflow (PTGS_WF_LDS_STACK < PTGS_STACK)
};

// device buffers, grown on demand and reused across calls
struct WfWorkspace {
  void* slots = nullptr;
  size_t slots_bytes = 0;
  void* part = nullptr;
  size_t part_bytes = 0;
  void* ovf = nullptr;
  size_t ovf_bytes = 0;
};

void wf_workspace_free(WfWorkspace& w);

// ptgs_trace_camera through the wavefront stages: `spp` samples (frames frame0 + s * stride) over
// pixel rows [row0, row1), accumulated into accum (running mean or SUM) exactly as pt_camera_kernel
hipError_t launch_pt_wavefront(WfWorkspace& w, const DevScene& sc, const CamParams& cp, float* accum, uint32_t W,
                               uint32_t H, uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0,
                               uint32_t stride, uint32_t mode, unsigned long long* counters, bool stats,
                               hipStream_t s);

}  // namespace ptgs
