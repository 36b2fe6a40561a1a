// splat.hip — 3D Gaussian splatting forward rasterizer for gfx950.
//
// The reference has no Gaussian rasterizer; this restates the published forward
// pass (Kerbl et al., SIGGRAPH 2023) in the reference's camera conventions (glm::lookAt RH view,
// Vulkan ZO projection with [1][1] negated, camera.cpp:186-187):
//   1. preprocess   one work-item per Gaussian: frustum cull (d <= 0.2), Sigma = R S^2 R^T,
//                   EWA Sigma' = J W Sigma W^T J^T (+0.3 low-pass), conic, 3-sigma radius, tile rect
//   2. scan         exclusive sum of tiles touched (hipcub)
//   3. duplicate    (tile << 32 | depth bits, gaussian) pairs, Gaussian order
//   4. sort         LSD radix over 32 + ceil(log2 tiles) bits (stable: ties keep Gaussian order)
//   5. ranges       per-tile [start, end) of the sorted list
//   6. blend        one 256-thread workgroup per 16x16 tile, Gaussians staged through LDS in
//                   batches of 256, front-to-back alpha blend with early termination at T < 1e-4
// Integer outputs (radii, tiles, keys, ranges) are the bit-exact contract with
// oracle/ptgs_oracle.c; the image is bit-identical as well (detmath exp, -ffp-contract=off).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "../../include/ptgs/ptgs.h"
#include "detmath.h"
#include "splat.h"

namespace ptgs {

#define GS_BLOCK_X 16
#define GS_BLOCK_Y 16
#define GS_BLOCK (GS_BLOCK_X * GS_BLOCK_Y)

struct SplatCam {
  float view[16];
  float mvp[16];  // proj * view
  float fx, fy;   // P00*W/2, P11*H/2 (fy negative: Vulkan y-down)
  float tan_fovx, tan_fovy;
  uint32_t W, H;
  uint32_t grid_x, grid_y;
  uint32_t row_begin, row_end;  // tile rows
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct SplatWorkspace {
  DevBuf means2d, depths, conic, rgb, radii, touched, offsets, keys_in, vals_in, keys_out, vals_out, ranges, temp,
      point_keys, total;
  uint32_t last_n = 0, last_k = 0, last_tiles = 0;
  hipEvent_t ev[7] = {};
  bool timed = false;
};

SplatWorkspace* splat_workspace_create() { return new SplatWorkspace(); }

void splat_workspace_destroy(SplatWorkspace* w) {
  if (!w) return;
  DevBuf* all[] = {&w->means2d, &w->depths, &w->conic, &w->rgb, &w->radii, &w->touched, &w->offsets, &w->keys_in,
                   &w->vals_in, &w->keys_out, &w->vals_out, &w->ranges, &w->temp, &w->point_keys, &w->total};
  for (DevBuf* b : all)
    if (b->p) (void)hipFree(b->p);
  for (hipEvent_t& e : w->ev)
    if (e) (void)hipEventDestroy(e);
  delete w;
}

static hipError_t ensure(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  size_t cap = bytes + bytes / 4;
  hipError_t e = hipMalloc(&b.p, cap);
  if (e == hipSuccess) b.bytes = cap;
  return e;
}

__device__ __forceinline__ v4 mv4(const float* m, float x, float y, float z, float w) {
  return mk4(((m[0] * x + m[4] * y) + m[8] * z) + m[12] * w, ((m[1] * x + m[5] * y) + m[9] * z) + m[13] * w,
             ((m[2] * x + m[6] * y) + m[10] * z) + m[14] * w, ((m[3] * x + m[7] * y) + m[11] * z) + m[15] * w);
}

__device__ __forceinline__ float ndc2pix(float v, int S) { return ((v + 1.0f) * (float)S - 1.0f) * 0.5f; }

__global__ __launch_bounds__(256) void gs_preprocess_kernel(SplatCam cam, const float* __restrict__ means,
                                                            const float* __restrict__ scales,
                                                            const float* __restrict__ rots,
                                                            const float* __restrict__ opac,
                                                            const float* __restrict__ colors, uint32_t n,
                                                            float2* __restrict__ means2d, float* __restrict__ depths,
                                                            float4* __restrict__ conic_o, float4* __restrict__ rgb,
                                                            int* __restrict__ radii, uint32_t* __restrict__ touched) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  radii[i] = 0;
  touched[i] = 0;
  float mx = means[3 * i], my = means[3 * i + 1], mz = means[3 * i + 2];
  // frustum: view-space depth d = -z (RH, camera looks down -Z)
  v4 pv = mv4(cam.view, mx, my, mz, 1.0f);
  float d = -pv.z;
  if (d <= 0.2f) return;
  v4 ph = mv4(cam.mvp, mx, my, mz, 1.0f);
  float pw = 1.0f / (ph.w + 0.0000001f);
  float px = ph.x * pw, py = ph.y * pw;

  // Sigma = R S^2 R^T
  float qr = rots[4 * i], qx = rots[4 * i + 1], qy = rots[4 * i + 2], qz = rots[4 * i + 3];
  float qn = sqrtx(((qr * qr + qx * qx) + qy * qy) + qz * qz);
  qr = qr / qn; qx = qx / qn; qy = qy / qn; qz = qz / qn;
  float sx = scales[3 * i], sy = scales[3 * i + 1], sz = scales[3 * i + 2];
  float R00 = 1.0f - 2.0f * (qy * qy + qz * qz), R01 = 2.0f * (qx * qy - qr * qz), R02 = 2.0f * (qx * qz + qr * qy);
  float R10 = 2.0f * (qx * qy + qr * qz), R11 = 1.0f - 2.0f * (qx * qx + qz * qz), R12 = 2.0f * (qy * qz - qr * qx);
  float R20 = 2.0f * (qx * qz - qr * qy), R21 = 2.0f * (qy * qz + qr * qx), R22 = 1.0f - 2.0f * (qx * qx + qy * qy);
  float M00 = R00 * sx, M01 = R01 * sy, M02 = R02 * sz;
  float M10 = R10 * sx, M11 = R11 * sy, M12 = R12 * sz;
  float M20 = R20 * sx, M21 = R21 * sy, M22 = R22 * sz;
  float S00 = (M00 * M00 + M01 * M01) + M02 * M02;
  float S01 = (M00 * M10 + M01 * M11) + M02 * M12;
  float S02 = (M00 * M20 + M01 * M21) + M02 * M22;
  float S11 = (M10 * M10 + M11 * M11) + M12 * M12;
  float S12 = (M10 * M20 + M11 * M21) + M12 * M22;
  float S22 = (M20 * M20 + M21 * M21) + M22 * M22;

  // EWA: J (2x3) at the clamped view-space point, W = view rotation rows
  float limx = 1.3f * cam.tan_fovx, limy = 1.3f * cam.tan_fovy;
  float txtz = pv.x / d, tytz = pv.y / d;
  float tx = fminx(limx, fmaxx(-limx, txtz)) * d;
  float ty = fminx(limy, fmaxx(-limy, tytz)) * d;
  float J00 = cam.fx / d, J02 = (cam.fx * tx) / (d * d);
  float J11 = cam.fy / d, J12 = (cam.fy * ty) / (d * d);
  const float* V = cam.view;  // column-major: row r, col c = V[c*4 + r]
  float T00 = J00 * V[0] + J02 * V[2], T01 = J00 * V[4] + J02 * V[6], T02 = J00 * V[8] + J02 * V[10];
  float T10 = J11 * V[1] + J12 * V[2], T11 = J11 * V[5] + J12 * V[6], T12 = J11 * V[9] + J12 * V[10];
  // cov = T Sigma T^T
  float U00 = (T00 * S00 + T01 * S01) + T02 * S02;
  float U01 = (T00 * S01 + T01 * S11) + T02 * S12;
  float U02 = (T00 * S02 + T01 * S12) + T02 * S22;
  float U10 = (T10 * S00 + T11 * S01) + T12 * S02;
  float U11 = (T10 * S01 + T11 * S11) + T12 * S12;
  float U12 = (T10 * S02 + T11 * S12) + T12 * S22;
  float ca = ((U00 * T00 + U01 * T01) + U02 * T02) + 0.3f;
  float cb = (U00 * T10 + U01 * T11) + U02 * T12;
  float cc = ((U10 * T10 + U11 * T11) + U12 * T12) + 0.3f;

  float det = ca * cc - cb * cb;
  if (det == 0.0f) return;
  float det_inv = 1.0f / det;
  float4 con = make_float4(cc * det_inv, -cb * det_inv, ca * det_inv, opac[i]);
  float mid = 0.5f * (ca + cc);
  float disc = sqrtx(fmaxx(0.1f, mid * mid - det));
  float l1 = mid + disc, l2 = mid - disc;
  float radius = __builtin_ceilf(3.0f * sqrtx(fmaxx(l1, l2)));
  float2 pimg = make_float2(ndc2pix(px, (int)cam.W), ndc2pix(py, (int)cam.H));
  int r = (int)radius;
  int rmin_x = min((int)cam.grid_x, max(0, (int)((pimg.x - (float)r) / (float)GS_BLOCK_X)));
  int rmin_y = min((int)cam.grid_y, max(0, (int)((pimg.y - (float)r) / (float)GS_BLOCK_Y)));
  int rmax_x = min((int)cam.grid_x, max(0, (int)((pimg.x + (float)r + (float)(GS_BLOCK_X - 1)) / (float)GS_BLOCK_X)));
  int rmax_y = min((int)cam.grid_y, max(0, (int)((pimg.y + (float)r + (float)(GS_BLOCK_Y - 1)) / (float)GS_BLOCK_Y)));
  rmin_y = max(rmin_y, (int)cam.row_begin);
  rmax_y = min(rmax_y, (int)cam.row_end);
  int area = (rmax_x - rmin_x) * (rmax_y - rmin_y);
  if (rmax_x <= rmin_x || rmax_y <= rmin_y || area == 0) return;
  depths[i] = d;
  radii[i] = r;
  means2d[i] = pimg;
  conic_o[i] = con;
  rgb[i] = make_float4(colors[3 * i], colors[3 * i + 1], colors[3 * i + 2], 0.0f);
  touched[i] = (uint32_t)area;
}

// recompute the (clamped) rect of a visible Gaussian — same integer math as preprocess
__device__ __forceinline__ void gs_rect(const SplatCam& cam, float2 p, int r, int& x0, int& y0, int& x1, int& y1) {
  x0 = min((int)cam.grid_x, max(0, (int)((p.x - (float)r) / (float)GS_BLOCK_X)));
  y0 = min((int)cam.grid_y, max(0, (int)((p.y - (float)r) / (float)GS_BLOCK_Y)));
  x1 = min((int)cam.grid_x, max(0, (int)((p.x + (float)r + (float)(GS_BLOCK_X - 1)) / (float)GS_BLOCK_X)));
  y1 = min((int)cam.grid_y, max(0, (int)((p.y + (float)r + (float)(GS_BLOCK_Y - 1)) / (float)GS_BLOCK_Y)));
  y0 = max(y0, (int)cam.row_begin);
  y1 = min(y1, (int)cam.row_end);
}

__global__ __launch_bounds__(256) void gs_duplicate_kernel(SplatCam cam, uint32_t n, const float2* __restrict__ means2d,
                                                           const float* __restrict__ depths,
                                                           const int* __restrict__ radii,
                                                           const uint32_t* __restrict__ offsets,
                                                           unsigned long long* __restrict__ keys,
                                                           uint32_t* __restrict__ vals) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int r = radii[i];
  if (r <= 0) return;
  uint32_t off = offsets[i];
  int x0, y0, x1, y1;
  gs_rect(cam, means2d[i], r, x0, y0, x1, y1);
  unsigned long long db = (unsigned long long)__float_as_uint(depths[i]);
  for (int y = y0; y < y1; ++y)
    for (int x = x0; x < x1; ++x) {
      unsigned long long tile = (unsigned long long)(y * (int)cam.grid_x + x);
      keys[off] = (tile << 32) | db;
      vals[off] = i;
      off++;
    }
}

__global__ __launch_bounds__(256) void gs_ranges_kernel(const unsigned long long* __restrict__ keys, uint32_t k,
                                                        uint2* __restrict__ ranges) {
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= k) return;
  uint32_t tile = (uint32_t)(keys[idx] >> 32);
  if (idx == 0) {
    ranges[tile].x = 0;
  } else {
    uint32_t prev = (uint32_t)(keys[idx - 1] >> 32);
    if (tile != prev) {
      ranges[prev].y = idx;
      ranges[tile].x = idx;
    }
  }
  if (idx == k - 1) ranges[tile].y = k;
}

__global__ __launch_bounds__(GS_BLOCK) void gs_blend_kernel(SplatCam cam, const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ vals,
                                                            const float2* __restrict__ means2d,
                                                            const float4* __restrict__ conic_o,
                                                            const float4* __restrict__ rgb, float bg_r, float bg_g,
                                                            float bg_b, float4* __restrict__ out) {
  __shared__ float2 s_xy[GS_BLOCK];
  __shared__ float4 s_co[GS_BLOCK];
  __shared__ float4 s_rgb[GS_BLOCK];
  const uint32_t tile_x = blockIdx.x, tile_y = cam.row_begin + blockIdx.y;
  const uint32_t tid = threadIdx.x;
  const uint32_t px = tile_x * GS_BLOCK_X + (tid % GS_BLOCK_X);
  const uint32_t py = tile_y * GS_BLOCK_Y + (tid / GS_BLOCK_X);
  const bool inside = px < cam.W && py < cam.H;
  bool done = !inside;
  const float pfx = (float)px, pfy = (float)py;
  uint2 range = ranges[tile_y * cam.grid_x + tile_x];
  int todo = (int)range.y - (int)range.x;
  float T = 1.0f;
  float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
  for (int base = (int)range.x; todo > 0; base += GS_BLOCK, todo -= GS_BLOCK) {
    if (__syncthreads_count(done) == GS_BLOCK) break;
    int idx = base + (int)tid;
    if (idx < (int)range.y) {
      uint32_t g = vals[idx];
      s_xy[tid] = means2d[g];
      s_co[tid] = conic_o[g];
      s_rgb[tid] = rgb[g];
    }
    __syncthreads();
    int cnt = todo < GS_BLOCK ? todo : GS_BLOCK;
    for (int j = 0; !done && j < cnt; ++j) {
      float2 xy = s_xy[j];
      float dx = xy.x - pfx, dy = xy.y - pfy;
      float4 co = s_co[j];
      float power = -0.5f * ((co.x * dx) * dx + (co.z * dy) * dy) - (co.y * dx) * dy;
      if (power > 0.0f) continue;
      float alpha = fminx(0.99f, co.w * expx(power));
      if (alpha < 1.0f / 255.0f) continue;
      float test_T = T * (1.0f - alpha);
      if (test_T < 0.0001f) { done = true; continue; }
      float4 c = s_rgb[j];
      C0 = C0 + (c.x * alpha) * T;
      C1 = C1 + (c.y * alpha) * T;
      C2 = C2 + (c.z * alpha) * T;
      T = test_T;
    }
  }
  if (inside) out[(size_t)py * cam.W + px] = make_float4(C0 + T * bg_r, C1 + T * bg_g, C2 + T * bg_b, 1.0f - T);
}

static uint32_t bits_for(uint32_t v) {
  uint32_t b = 0;
  while (b < 32 && (1ull << b) < (unsigned long long)v) b++;
  return b;
}

hipError_t splat_gaussians(SplatWorkspace* w, const ptgs_gaussians* g, const float* view, const float* mvp, float p00,
                           float p11, uint32_t W, uint32_t H, const float bg[3], uint32_t tile_row_begin,
                           uint32_t tile_row_end, float* out, ptgs_splat_stats* stats, bool time_stages,
                           hipStream_t s) {
  hipError_t e;
  if (time_stages && !w->ev[0])
    for (hipEvent_t& ev : w->ev)
      if ((e = hipEventCreate(&ev))) return e;
  w->timed = time_stages;
  auto mark = [&](int k) -> hipError_t { return time_stages ? hipEventRecord(w->ev[k], s) : hipSuccess; };
  const uint32_t n = g->count;
  SplatCam cam;
  std::memcpy(cam.view, view, sizeof(cam.view));
  std::memcpy(cam.mvp, mvp, sizeof(cam.mvp));
  cam.fx = p00 * (float)W * 0.5f;
  cam.fy = p11 * (float)H * 0.5f;
  cam.tan_fovx = 1.0f / p00;
  cam.tan_fovy = 1.0f / (p11 < 0.0f ? -p11 : p11);
  cam.W = W; cam.H = H;
  cam.grid_x = (W + GS_BLOCK_X - 1) / GS_BLOCK_X;
  cam.grid_y = (H + GS_BLOCK_Y - 1) / GS_BLOCK_Y;
  cam.row_begin = std::min(tile_row_begin, cam.grid_y);
  cam.row_end = std::min(tile_row_end, cam.grid_y);
  if (cam.row_end < cam.row_begin) cam.row_end = cam.row_begin;
  const uint32_t tiles = cam.grid_x * cam.grid_y;

  if ((e = ensure(w->means2d, (size_t)n * 8))) return e;
  if ((e = ensure(w->depths, (size_t)n * 4))) return e;
  if ((e = ensure(w->conic, (size_t)n * 16))) return e;
  if ((e = ensure(w->rgb, (size_t)n * 16))) return e;
  if ((e = ensure(w->radii, (size_t)n * 4))) return e;
  if ((e = ensure(w->touched, (size_t)n * 4 + 4))) return e;
  if ((e = ensure(w->offsets, (size_t)n * 4 + 4))) return e;
  if ((e = ensure(w->ranges, (size_t)tiles * 8))) return e;
  if ((e = ensure(w->total, 16))) return e;

  if ((e = mark(0))) return e;
  if (n) {
    hipLaunchKernelGGL(gs_preprocess_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cam, g->means, g->scales,
                       g->rotations, g->opacities, g->colors, n, (float2*)w->means2d.p, (float*)w->depths.p,
                       (float4*)w->conic.p, (float4*)w->rgb.p, (int*)w->radii.p, (uint32_t*)w->touched.p);
    if ((e = hipGetLastError())) return e;
  }
  if ((e = mark(1))) return e;
  // exclusive scan over n+1 entries (the last one = K)
  if ((e = hipMemsetAsync((uint32_t*)w->touched.p + n, 0, 4, s))) return e;
  size_t temp_bytes = 0;
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, (uint32_t*)w->touched.p, (uint32_t*)w->offsets.p,
                                            n + 1, s)))
    return e;
  if ((e = ensure(w->temp, temp_bytes))) return e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(w->temp.p, temp_bytes, (uint32_t*)w->touched.p, (uint32_t*)w->offsets.p,
                                            n + 1, s)))
    return e;
  if ((e = mark(2))) return e;
  uint32_t K = 0;
  if ((e = hipMemcpyAsync(&K, (uint32_t*)w->offsets.p + n, 4, hipMemcpyDeviceToHost, s))) return e;
  if ((e = hipStreamSynchronize(s))) return e;

  if ((e = ensure(w->keys_in, (size_t)K * 8))) return e;
  if ((e = ensure(w->vals_in, (size_t)K * 4))) return e;
  if ((e = ensure(w->keys_out, (size_t)K * 8))) return e;
  if ((e = ensure(w->vals_out, (size_t)K * 4))) return e;
  if ((e = hipMemsetAsync(w->ranges.p, 0, (size_t)tiles * 8, s))) return e;
  if (K > 0) {
    hipLaunchKernelGGL(gs_duplicate_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cam, n,
                       (const float2*)w->means2d.p, (const float*)w->depths.p, (const int*)w->radii.p,
                       (const uint32_t*)w->offsets.p, (unsigned long long*)w->keys_in.p, (uint32_t*)w->vals_in.p);
    if ((e = hipGetLastError())) return e;
    if ((e = mark(3))) return e;
    int end_bit = 32 + (int)bits_for(tiles);
    size_t sort_bytes = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (unsigned long long*)w->keys_in.p,
                                                (unsigned long long*)w->keys_out.p, (uint32_t*)w->vals_in.p,
                                                (uint32_t*)w->vals_out.p, (int)K, 0, end_bit, s)))
      return e;
    if ((e = ensure(w->temp, sort_bytes))) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(w->temp.p, sort_bytes, (unsigned long long*)w->keys_in.p,
                                                (unsigned long long*)w->keys_out.p, (uint32_t*)w->vals_in.p,
                                                (uint32_t*)w->vals_out.p, (int)K, 0, end_bit, s)))
      return e;
    if ((e = mark(4))) return e;
    hipLaunchKernelGGL(gs_ranges_kernel, dim3((K + 255) / 256), dim3(256), 0, s, (const unsigned long long*)w->keys_out.p,
                       K, (uint2*)w->ranges.p);
    if ((e = hipGetLastError())) return e;
  } else {
    if ((e = mark(3))) return e;
    if ((e = mark(4))) return e;
  }
  if ((e = mark(5))) return e;
  uint32_t rows = cam.row_end - cam.row_begin;
  if (rows > 0) {
    hipLaunchKernelGGL(gs_blend_kernel, dim3(cam.grid_x, rows), dim3(GS_BLOCK), 0, s, cam, (const uint2*)w->ranges.p,
                       (const uint32_t*)w->vals_out.p, (const float2*)w->means2d.p, (const float4*)w->conic.p,
                       (const float4*)w->rgb.p, bg[0], bg[1], bg[2], (float4*)out);
    if ((e = hipGetLastError())) return e;
  }
  if ((e = mark(6))) return e;
  w->last_n = n;
  w->last_k = K;
  w->last_tiles = tiles;
  if (stats) {
    stats->num_rendered = K;
    stats->tiles_x = cam.grid_x;
    stats->tiles_y = cam.grid_y;
    stats->num_visible = 0;
  }
  return hipSuccess;
}

hipError_t splat_stage_ms(SplatWorkspace* w, float* out_ms) {
  for (int k = 0; k < 6; ++k) out_ms[k] = 0.0f;
  if (!w->timed || !w->ev[0]) return hipSuccess;
  hipError_t e = hipEventSynchronize(w->ev[6]);
  if (e) return e;
  for (int k = 0; k < 6; ++k)
    if ((e = hipEventElapsedTime(&out_ms[k], w->ev[k], w->ev[k + 1]))) return e;
  return hipSuccess;
}

void splat_get_buffers(const SplatWorkspace* w, ptgs_splat_buffers* out) {
  out->radii = (const int32_t*)w->radii.p;
  out->tiles_touched = (const uint32_t*)w->touched.p;
  out->sorted_keys = (const uint64_t*)w->keys_out.p;
  out->sorted_values = (const uint32_t*)w->vals_out.p;
  out->tile_ranges = (const uint32_t*)w->ranges.p;
  out->means2d = (const float*)w->means2d.p;
  out->depths = (const float*)w->depths.p;
  out->conic_opacity = (const float*)w->conic.p;
  out->num_gaussians = w->last_n;
  out->num_rendered = w->last_k;
  out->num_tiles = w->last_tiles;
}

hipError_t splat_point_keys(SplatWorkspace* w, size_t npix, unsigned long long** keys) {
  hipError_t e = ensure(w->point_keys, npix * 8);
  *keys = (unsigned long long*)w->point_keys.p;
  return e;
}

}  // namespace ptgs
