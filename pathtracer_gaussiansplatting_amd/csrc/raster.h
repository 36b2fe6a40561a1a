// raster.h — launch interface of raster.hip (point splat, sRGB encode).
#pragma once

#include <hip/hip_runtime.h>
#include "../../include/ptgs/ptgs.h"

namespace ptgs {

hipError_t launch_encode_srgb8(const float* in, uint32_t* out, uint32_t n, hipStream_t s);
hipError_t launch_splat_points(const float* mvp, const float* model, float R, float r, float h, int mode,
                               const ptgs_hitdata* hits, const ptgs_ray_sample* samples, uint32_t n, uint32_t W,
                               uint32_t H, unsigned long long* keys, float* depth, uint32_t* rgba8, hipStream_t s);

}  // namespace ptgs
