// 3-nearest-neighbour mean squared distance and the 3DGS point-cloud initialisation (knn.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ptgs {

struct KnnTimes {
  float sort_ms = 0, query_ms = 0;
};

// dist2[i] (device, n floats) = mean of the 3 smallest squared distances from point i to the other
// points (xyz: device, 3n floats). Synchronises `s` (frees its temporaries).
hipError_t knn3_mean_dist2(const float* xyz, uint32_t n, float* dist2, hipStream_t s, KnnTimes* times);

// Kerbl et al. 2023 create_from_pcd in post-activation form (device arrays): means = xyz,
// scales = sqrt(max(dist2, 1e-7)) (x3), rotations = (1, 0, 0, 0), opacities = 0.1,
// colors = rgb / 255 (rgb may be null: black).
hipError_t gaussians_from_points(const float* xyz, const uint8_t* rgb, uint32_t n, float* means, float* scales,
                                 float* rots, float* opac, float* colors, hipStream_t s);

}  // namespace ptgs
