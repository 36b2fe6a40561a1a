// raster.hip — point-cloud raster (the reference's only splat raster) and the sRGB8 output
// encode, for gfx950.
//
//   ptgs_splat_points : shaders/pointcloud/pointcloud.vert:44-89 + pointcloud.frag:1-11 with the
//                       pipeline state of pipeline.cpp:29-82 (point list, 2-px sprites, depth test
//                       LESS + write, no blend, B8G8R8A8_SRGB target). Rasterization order is
//                       reproduced with one 64-bit atomicMin per fragment on (depth bits << 32 | i):
//                       smallest depth wins, ties go to the earlier point, as LESS in draw order.
//   ptgs_encode_srgb8 : the rgba32f -> sRGB8 blit of engine.cpp:2004-2020.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/ptgs/ptgs.h"
#include "detmath.h"
#include "raster.h"

namespace ptgs {

// linear -> sRGB8 (Vulkan UNORM_SRGB encode; exponent via detmath so the oracle matches bitwise)
__device__ __forceinline__ uint32_t srgb8(float c) {
  c = clampf(c, 0.0f, 1.0f);
  float s = (c <= 0.0031308f) ? c * 12.92f : 1.055f * powx(c, 0.41666666666666667f) - 0.055f;
  return (uint32_t)(s * 255.0f + 0.5f);
}

__global__ __launch_bounds__(256) void encode_srgb8_kernel(const float4* __restrict__ in, uint32_t* __restrict__ out,
                                                           uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 v = in[i];
  out[i] = srgb8(v.x) | (srgb8(v.y) << 8) | (srgb8(v.z) << 16) | (255u << 24);
}

struct PointParams {
  float mvp[16];  // proj * view (computed on the host, float, GLSL order)
  float model[16];
  float R, r, h;
  int mode;
  uint32_t W, H;
};

__device__ __forceinline__ v4 matvec4(const float* m, v4 v) {
  return mk4(((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * v.w,
             ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * v.w,
             ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * v.w,
             ((m[3] * v.x + m[7] * v.y) + m[11] * v.z) + m[15] * v.w);
}

__global__ __launch_bounds__(256) void point_fragments_kernel(PointParams pp, const ptgs_hitdata* __restrict__ hits,
                                                              const ptgs_ray_sample* __restrict__ samples, uint32_t n,
                                                              const float* __restrict__ depth_in,
                                                              unsigned long long* __restrict__ keys) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ptgs_hitdata hd = hits[i];
  if (!(hd.flag > 0.0f)) return;  // z = -2 (culled) / frag discard
  v3 fp;
  if (pp.mode == 1) {
    ptgs_ray_sample s = samples[i];
    const float PI = 3.14159265359f;
    float u = (s.uv[0] * 2.0f) * PI, v = (s.uv[1] * 2.0f) * PI;
    float su, cu, sv, cv;
    sincosx(u, &su, &cu);
    sincosx(v, &sv, &cv);
    v3 lp = mk3((pp.R + pp.r * cv) * cu, pp.r * sv + pp.h, (pp.R + pp.r * cv) * su);
    v3 ln = mk3(cv * cu, sv, cv * su);
    lp = lp + ln * 0.01f;
    v4 w = matvec4(pp.model, mk4(lp.x, lp.y, lp.z, 1.0f));
    fp = mk3(w.x, w.y, w.z);
  } else {
    fp = mk3(hd.pos[0], hd.pos[1], hd.pos[2]);
  }
  v4 clip = matvec4(pp.mvp, mk4(fp.x, fp.y, fp.z, 1.0f));
  // view-volume clip of the point vertex
  if (!(clip.w > 0.0f)) return;
  if (clip.x < -clip.w || clip.x > clip.w || clip.y < -clip.w || clip.y > clip.w) return;
  if (clip.z < 0.0f || clip.z > clip.w) return;
  float nx = clip.x / clip.w, ny = clip.y / clip.w, nz = clip.z / clip.w;
  float xw = nx * ((float)pp.W * 0.5f) + (float)pp.W * 0.5f;
  float yw = ny * ((float)pp.H * 0.5f) + (float)pp.H * 0.5f;
  // 2-px sprite: pixel centres c with xw-1 <= c < xw+1
  int x0 = (int)floorx(xw - 1.5f), y0 = (int)floorx(yw - 1.5f);
  unsigned long long key = ((unsigned long long)__float_as_uint(nz) << 32) | i;
  for (int py = y0; py <= y0 + 2; ++py) {
    float cy = (float)py + 0.5f;
    if (py < 0 || py >= (int)pp.H || !(cy >= yw - 1.0f && cy < yw + 1.0f)) continue;
    for (int px = x0; px <= x0 + 2; ++px) {
      float cx = (float)px + 0.5f;
      if (px < 0 || px >= (int)pp.W || !(cx >= xw - 1.0f && cx < xw + 1.0f)) continue;
      size_t pix = (size_t)py * pp.W + px;
      if (!(nz < depth_in[pix])) continue;  // LESS against the incoming depth buffer
      atomicMin(keys + pix, key);
    }
  }
}

__global__ __launch_bounds__(256) void point_resolve_kernel(const unsigned long long* __restrict__ keys,
                                                            const ptgs_hitdata* __restrict__ hits, uint32_t npix,
                                                            float* __restrict__ depth, uint32_t* __restrict__ rgba8) {
  uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  unsigned long long k = keys[p];
  if (k == ~0ull) return;
  uint32_t idx = (uint32_t)(k & 0xffffffffu);
  depth[p] = __uint_as_float((uint32_t)(k >> 32));
  const ptgs_hitdata& hd = hits[idx];
  rgba8[p] = srgb8(hd.color[0]) | (srgb8(hd.color[1]) << 8) | (srgb8(hd.color[2]) << 16) | (255u << 24);
}

hipError_t launch_encode_srgb8(const float* in, uint32_t* out, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(encode_srgb8_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const float4*)in, out, n);
  return hipGetLastError();
}

hipError_t launch_splat_points(const float* mvp, const float* model, float R, float r, float h, int mode,
                               const ptgs_hitdata* hits, const ptgs_ray_sample* samples, uint32_t n, uint32_t W,
                               uint32_t H, unsigned long long* keys, float* depth, uint32_t* rgba8, hipStream_t s) {
  PointParams pp;
  std::memcpy(pp.mvp, mvp, sizeof(pp.mvp));
  std::memcpy(pp.model, model, sizeof(pp.model));
  pp.R = R; pp.r = r; pp.h = h; pp.mode = mode; pp.W = W; pp.H = H;
  uint32_t npix = W * H;
  hipError_t e = hipMemsetAsync(keys, 0xff, (size_t)npix * 8, s);
  if (e != hipSuccess) return e;
  if (n) hipLaunchKernelGGL(point_fragments_kernel, dim3((n + 255) / 256), dim3(256), 0, s, pp, hits, samples, n, depth, keys);
  hipLaunchKernelGGL(point_resolve_kernel, dim3((npix + 255) / 256), dim3(256), 0, s, keys, hits, npix, depth, rgba8);
  return hipGetLastError();
}

}  // namespace ptgs
