// splat.hip — 3D Gaussian splatting forward rasterizer for gfx950.
//
// The reference has no Gaussian rasterizer; this restates the published forward
// pass (Kerbl et al., SIGGRAPH 2023) in the reference's camera conventions (glm::lookAt RH view,
// Vulkan ZO projection with [1][1] negated, camera.cpp:186-187):
//   1. preprocess   one work-item per Gaussian: frustum cull (d <= 0.2), Sigma = R S^2 R^T,
//                   EWA Sigma' = J W Sigma W^T J^T (+0.3 low-pass), conic, 3-sigma radius, tile rect
//                   + per-tile pair counts (atomics)
//   2. tile scan    one workgroup: per-tile [start, end) ranges, scatter cursors, K
//   3. scatter      (depth bits << 32 | gaussian) into each touched tile's segment (atomic cursor)
//   4. sort+blend   one 256-thread workgroup per 16x16 tile: bitonic sort of the tile's pairs by
//                   (depth, gaussian) in LDS -> the same order as a stable global sort of
//                   (tile << 32 | depth) keys; publish sorted keys/values; front-to-back alpha blend
//                   with Gaussians staged through LDS in batches of 256, early exit at T < 1e-4
// Integer outputs (radii, tiles, keys, ranges) are the bit-exact contract with
// oracle/ptgs_oracle.c; the image is bit-identical as well (detmath exp, -ffp-contract=off).
#include <hip/hip_runtime.h>

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
  DevBuf means2d, depths, conic, rgb, radii, touched, pairs, keys_out, vals_out, ranges, tile_local, cursor,
      point_keys, total, rect, geo, hist, block_sum, block_off, ticket;
  uint32_t* k_host = nullptr;  // pinned, coherent: the scan kernel stores K here
  uint32_t* k_dev = nullptr;   // its device-side address
  hipEvent_t k_event = nullptr;
  uint32_t last_n = 0, last_k = 0, last_tiles = 0;
  hipEvent_t ev[7] = {};
  bool timed = false;
};

SplatWorkspace* splat_workspace_create() { return new SplatWorkspace(); }

void splat_workspace_destroy(SplatWorkspace* w) {
  if (!w) return;
  DevBuf* all[] = {&w->means2d, &w->depths, &w->conic, &w->rgb, &w->radii, &w->touched, &w->pairs, &w->keys_out,
                   &w->vals_out, &w->ranges, &w->tile_local, &w->cursor, &w->point_keys, &w->total, &w->rect,
                   &w->geo, &w->hist, &w->block_sum, &w->block_off, &w->ticket};
  for (DevBuf* b : all)
    if (b->p) (void)hipFree(b->p);
  if (w->k_host) (void)hipHostFree(w->k_host);
  for (hipEvent_t& e : w->ev)
    if (e) (void)hipEventDestroy(e);
  if (w->k_event) (void)hipEventDestroy(w->k_event);
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
                                                            int* __restrict__ radii, uint32_t* __restrict__ touched,
                                                            ushort4* __restrict__ rects, float4* __restrict__ geo) {
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
  // alpha = min(0.99, o * exp(power)) < 1/255  <=>  power < -ln(255 o). Pairs below that threshold
  // minus a 1e-3 margin (>> the exp/log approximation error) are skipped without evaluating exp:
  // the skipped set is a subset of the pairs the exact test rejects, so the image is unchanged.
  float skip = -(log2x(255.0f * con.w) * 0.69314718055994531f) - 0.001f;
  rgb[i] = make_float4(colors[3 * i], colors[3 * i + 1], colors[3 * i + 2], skip);
  touched[i] = (uint32_t)area;
  rects[i] = make_ushort4((unsigned short)rmin_x, (unsigned short)rmin_y, (unsigned short)rmax_x,
                          (unsigned short)rmax_y);
  // half-extents of the ellipse power >= skip (q = d^T conic d <= -2 skip), +1% and +0.01 px margin;
  // used only to skip whole 8x8 pixel blocks whose pairs the per-pixel skip test would reject anyway
  float sq = -2.0f * skip;
  float ex = sq > 0.0f ? sqrtx(sq * ca) * 1.01f + 0.01f : -1.0f;
  float ey = sq > 0.0f ? sqrtx(sq * cc) * 1.01f + 0.01f : -1.0f;
  geo[i] = make_float4(pimg.x, pimg.y, ex, ey);
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

#define GS_BIN_THREADS 1024
#define GS_SCAN_TILES 256

// Binning without global atomics (scattered atomics run ~17x below the chip's atomic rate on
// gfx950, MI355X_MICROARCH.md "Global float atomics"): block b of B owns a contiguous chunk of
// Gaussians and counts its (gaussian, tile) pairs per tile in an LDS histogram (ds_add), written
// block-major to hist[b][t]. gs_bin_scan_kernel turns the columns into per-block offsets and the
// per-tile totals into tile starts; the scatter re-walks the same chunk and places each pair at
// start[t] + hist[b][t] + (LDS cursor). The order inside a tile's segment depends on LDS atomic
// order and is fixed by the blend kernel's per-tile sort.
__global__ __launch_bounds__(GS_BIN_THREADS) void gs_bin_count_kernel(const ushort4* __restrict__ rects,
                                                                      const int* __restrict__ radii, uint32_t n,
                                                                      uint32_t chunk, uint32_t tiles,
                                                                      uint32_t grid_x, uint32_t* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
  for (uint32_t t = threadIdx.x; t < tiles; t += GS_BIN_THREADS) s_hist[t] = 0;
  __syncthreads();
  const uint32_t b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  for (uint32_t i = b0 + threadIdx.x; i < b1; i += GS_BIN_THREADS) {
    if (radii[i] <= 0) continue;
    ushort4 rc = rects[i];
    for (uint32_t y = rc.y; y < rc.w; ++y)
      for (uint32_t x = rc.x; x < rc.z; ++x) atomicAdd(s_hist + y * grid_x + x, 1u);
  }
  __syncthreads();
  uint32_t* row = hist + (size_t)blockIdx.x * tiles;
  for (uint32_t t = threadIdx.x; t < tiles; t += GS_BIN_THREADS) row[t] = s_hist[t];
}

// One work-item per tile: column scan of hist[.][t] (in place -> per-block offsets), the tile total
// c, and a block-local exclusive scan of c over GS_SCAN_TILES tiles -> tile_local[t] = (prefix, c).
// The last block to finish (ticket) scans the block sums -> block_off[] and K = total[0]; the tile
// start is block_off[t / GS_SCAN_TILES] + tile_local[t].x (consumers add it themselves).
__global__ __launch_bounds__(GS_SCAN_TILES) void gs_bin_scan_kernel(uint32_t* __restrict__ hist, uint32_t rows,
                                                                    uint32_t tiles, uint2* __restrict__ tile_local,
                                                                    uint32_t* __restrict__ block_sum,
                                                                    uint32_t* __restrict__ block_off,
                                                                    uint32_t* __restrict__ total,
                                                                    uint32_t* __restrict__ ticket,
                                                                    uint32_t* k_host) {
  __shared__ uint32_t s_v[GS_SCAN_TILES];
  __shared__ bool s_last;
  const uint32_t tid = threadIdx.x, t = blockIdx.x * GS_SCAN_TILES + tid;
  uint32_t run = 0;
  if (t < tiles) {
    for (uint32_t b0 = 0; b0 < rows; b0 += 16) {  // 16 independent loads in flight per lane
      uint32_t c[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) c[k] = (b0 + k < rows) ? hist[(size_t)(b0 + k) * tiles + t] : 0u;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (b0 + k < rows) hist[(size_t)(b0 + k) * tiles + t] = run;
        run += c[k];
      }
    }
  }
  s_v[tid] = run;
  __syncthreads();
  for (uint32_t off = 1; off < GS_SCAN_TILES; off <<= 1) {  // Hillis-Steele inclusive scan
    uint32_t v = tid >= off ? s_v[tid - off] : 0u;
    __syncthreads();
    s_v[tid] += v;
    __syncthreads();
  }
  if (t < tiles) tile_local[t] = make_uint2(s_v[tid] - run, run);
  if (tid == GS_SCAN_TILES - 1) {
    block_sum[blockIdx.x] = s_v[tid];
    __threadfence();  // release the block sum before taking a ticket
    s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();  // acquire the other blocks' sums
  const uint32_t nb = gridDim.x;  // <= GS_LDS_TILES / GS_SCAN_TILES = 128 for the LDS path
  uint32_t acc = 0;
  for (uint32_t c0 = 0; c0 < nb; c0 += GS_SCAN_TILES) {
    const uint32_t k = c0 + tid;
    const uint32_t v0 = k < nb ? __atomic_load_n(block_sum + k, __ATOMIC_RELAXED) : 0u;
    __syncthreads();
    s_v[tid] = v0;
    __syncthreads();
    for (uint32_t off = 1; off < GS_SCAN_TILES; off <<= 1) {
      uint32_t v = tid >= off ? s_v[tid - off] : 0u;
      __syncthreads();
      s_v[tid] += v;
      __syncthreads();
    }
    if (k < nb) block_off[k] = acc + s_v[tid] - v0;
    acc += s_v[GS_SCAN_TILES - 1];
  }
  if (tid == 0) {
    *total = acc;
    __atomic_store_n(k_host, acc, __ATOMIC_RELAXED);  // pinned host word: the host's K read-back
    *ticket = 0;  // ready for the next frame (stream order)
  }
}

__device__ __forceinline__ uint32_t gs_tile_start(const uint2* tile_local, const uint32_t* block_off, uint32_t t) {
  return block_off[t / GS_SCAN_TILES] + tile_local[t].x;
}

// Pairs are written only when K fits the pair buffer (the host sizes it from the previous K and
// re-runs scatter + blend after growing it when it did not: see splat_gaussians).
__global__ __launch_bounds__(GS_BIN_THREADS) void gs_bin_scatter_kernel(
    const ushort4* __restrict__ rects, const int* __restrict__ radii, const float* __restrict__ depths, uint32_t n,
    uint32_t chunk, uint32_t tiles, uint32_t grid_x, const uint32_t* __restrict__ hist,
    const uint2* __restrict__ tile_local, const uint32_t* __restrict__ block_off, const uint32_t* __restrict__ total,
    uint32_t cap, uint2* __restrict__ ranges, unsigned long long* __restrict__ pairs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_cur[];
  if (*total > cap) return;
  const uint32_t* row = hist + (size_t)blockIdx.x * tiles;
  for (uint32_t t = threadIdx.x; t < tiles; t += GS_BIN_THREADS) {
    const uint2 tl = tile_local[t];
    const uint32_t st = block_off[t / GS_SCAN_TILES] + tl.x;
    s_cur[t] = st + row[t];
    if (blockIdx.x == 0) ranges[t] = tl.y ? make_uint2(st, st + tl.y) : make_uint2(0u, 0u);
  }
  __syncthreads();
  const uint32_t b0 = blockIdx.x * chunk, b1 = min(n, b0 + chunk);
  for (uint32_t i = b0 + threadIdx.x; i < b1; i += GS_BIN_THREADS) {
    if (radii[i] <= 0) continue;
    ushort4 rc = rects[i];
    unsigned long long key = ((unsigned long long)__float_as_uint(depths[i]) << 32) | i;
    for (uint32_t y = rc.y; y < rc.w; ++y)
      for (uint32_t x = rc.x; x < rc.z; ++x) {
        uint32_t pos = atomicAdd(s_cur + y * grid_x + x, 1u);
        pairs[pos] = key;
      }
  }
}

// Fallback for tile counts whose histogram does not fit LDS (> GS_LDS_TILES): global atomics into a
// single histogram row (hist, zeroed), the same scan kernel, then global cursors (zeroed).
__global__ __launch_bounds__(256) void gs_count_global_kernel(const ushort4* __restrict__ rects,
                                                              const int* __restrict__ radii, uint32_t n,
                                                              uint32_t grid_x, uint32_t* __restrict__ tile_count) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || radii[i] <= 0) return;
  ushort4 rc = rects[i];
  for (uint32_t y = rc.y; y < rc.w; ++y)
    for (uint32_t x = rc.x; x < rc.z; ++x) atomicAdd(tile_count + y * grid_x + x, 1u);
}

__global__ __launch_bounds__(256) void gs_ranges_kernel(const uint2* __restrict__ tile_local,
                                                        const uint32_t* __restrict__ block_off, uint32_t tiles,
                                                        const uint32_t* __restrict__ total, uint32_t cap,
                                                        uint2* __restrict__ ranges) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tiles || *total > cap) return;
  const uint2 tl = tile_local[t];
  const uint32_t st = block_off[t / GS_SCAN_TILES] + tl.x;
  ranges[t] = tl.y ? make_uint2(st, st + tl.y) : make_uint2(0u, 0u);
}

__global__ __launch_bounds__(256) void gs_scatter_global_kernel(
    const ushort4* __restrict__ rects, const int* __restrict__ radii, const float* __restrict__ depths, uint32_t n,
    uint32_t grid_x, const uint2* __restrict__ tile_local, const uint32_t* __restrict__ block_off,
    const uint32_t* __restrict__ total, uint32_t cap, uint32_t* __restrict__ cursor,
    unsigned long long* __restrict__ pairs) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || radii[i] <= 0 || *total > cap) return;
  ushort4 rc = rects[i];
  unsigned long long key = ((unsigned long long)__float_as_uint(depths[i]) << 32) | i;
  for (uint32_t y = rc.y; y < rc.w; ++y)
    for (uint32_t x = rc.x; x < rc.z; ++x) {
      const uint32_t t = y * grid_x + x;
      pairs[gs_tile_start(tile_local, block_off, t) + atomicAdd(cursor + t, 1u)] = key;
    }
}

#define GS_LDS_TILES 32768

// ascending bitonic sort ("flip" network: every comparator puts the min at the lower index) over
// n elements; indices >= n act as +inf and are never touched, so n need not be a power of two.
template <typename Swap>
__device__ __forceinline__ void bitonic_flip_sort(uint32_t n, Swap swap_if) {
  uint32_t npad = 1;
  while (npad < n) npad <<= 1;
  const uint32_t half = npad >> 1;
  for (uint32_t lk = 1; (1u << lk) <= npad; ++lk) {  // k = 2^lk; all strides are powers of two
    const uint32_t k = 1u << lk, lhk = lk - 1;
    for (uint32_t i = threadIdx.x; i < half; i += blockDim.x) {
      uint32_t blk = i >> lhk, off = i & ((1u << lhk) - 1u);
      uint32_t a = blk * k + off, b = blk * k + k - 1 - off;
      if (b < n) swap_if(a, b);
    }
    __syncthreads();
    for (int lj = (int)lk - 2; lj >= 0; --lj) {
      const uint32_t j = 1u << lj;
      for (uint32_t i = threadIdx.x; i < half; i += blockDim.x) {
        uint32_t a = ((i >> lj) << (lj + 1)) + (i & (j - 1u)), b = a + j;
        if (b < n) swap_if(a, b);
      }
      __syncthreads();
    }
  }
}

#define GS_SORT_CAP 1024

// One 256-thread workgroup per 16x16 tile: sort the tile's pairs by (depth, gaussian) in LDS
// (global memory for segments longer than GS_SORT_CAP), publish the sorted keys/values, then the
// front-to-back alpha blend with Gaussians staged through LDS in batches of 256.
__global__ __launch_bounds__(GS_BLOCK) void gs_sort_blend_kernel(SplatCam cam, const uint2* __restrict__ ranges,
                                                                 unsigned long long* __restrict__ pairs,
                                                                 unsigned long long* __restrict__ keys_out,
                                                                 uint32_t* __restrict__ vals_out,
                                                                 const float4* __restrict__ geo,
                                                                 const float4* __restrict__ conic_o,
                                                                 const float4* __restrict__ rgb, float bg_r,
                                                                 float bg_g, float bg_b,
                                                                 const uint32_t* __restrict__ total, uint32_t cap,
                                                                 float4* __restrict__ out) {
  __shared__ unsigned long long s_key[GS_SORT_CAP];
  if (*total > cap) return;  // pair buffer too small this frame: the host re-runs after growing it
  // staged Gaussians of the current batch; slot GS_BLOCK is a null Gaussian (alpha = 0) that pads
  // the per-quadrant lists to a multiple of 4
  __shared__ float4 s_ga[GS_BLOCK + 1];  // (x, y, -a/2, -b)
  __shared__ float4 s_gb[GS_BLOCK + 1];  // (-c/2, log2 o, r, g)
  __shared__ float s_gc[GS_BLOCK + 1];   // b
  __shared__ __attribute__((aligned(8))) uint16_t s_list[4][GS_BLOCK + 4];
  __shared__ uint32_t s_qcnt[4][4];  // [wave][quadrant]
  const uint32_t tile_x = blockIdx.x, tile_y = cam.row_begin + blockIdx.y;
  const uint32_t tile = tile_y * cam.grid_x + tile_x;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    s_ga[GS_BLOCK] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    s_gb[GS_BLOCK] = make_float4(0.0f, -__builtin_huge_valf(), 0.0f, 0.0f);
    s_gc[GS_BLOCK] = 0.0f;
  }
  const uint2 range = ranges[tile];
  const uint32_t n = range.y - range.x;
  const bool small = n <= GS_BLOCK;
  const bool in_lds = n <= GS_SORT_CAP;
  unsigned long long* seg = pairs + range.x;
  const unsigned long long tbits = (unsigned long long)tile << 32;
  unsigned long long my_key = ~0ull;  // small tiles: work-item tid holds sorted element tid
  if (small) {
    // one key per work-item: bitonic network in registers, lane exchanges by shuffle for strides
    // < 64 and through LDS (two barriers) for the 64/128 strides only
    if (tid < n) my_key = seg[tid];
    uint32_t npad = 1;
    while (npad < n) npad <<= 1;
    for (uint32_t k = 2; k <= npad; k <<= 1)
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        unsigned long long other;
        if (j >= 64) {
          __syncthreads();
          s_key[tid] = my_key;
          __syncthreads();
          other = s_key[tid ^ j];
        } else {
          other = __shfl_xor(my_key, (int)j);
        }
        const bool keep_min = ((tid & j) == 0) == ((tid & k) == 0);
        my_key = keep_min ? (other < my_key ? other : my_key) : (other < my_key ? my_key : other);
      }
    if (tid < n) {
      keys_out[range.x + tid] = tbits | (my_key >> 32);
      vals_out[range.x + tid] = (uint32_t)my_key;
    }
  } else {
    if (in_lds) {
      for (uint32_t k = tid; k < n; k += GS_BLOCK) s_key[k] = seg[k];
      __syncthreads();
      bitonic_flip_sort(n, [&](uint32_t a, uint32_t b) {
        unsigned long long x = s_key[a], y = s_key[b];
        if (y < x) { s_key[a] = y; s_key[b] = x; }
      });
    } else {
      bitonic_flip_sort(n, [&](uint32_t a, uint32_t b) {
        unsigned long long x = seg[a], y = seg[b];
        if (y < x) { seg[a] = y; seg[b] = x; }
      });
    }
    for (uint32_t k = tid; k < n; k += GS_BLOCK) {
      unsigned long long v = in_lds ? s_key[k] : seg[k];
      keys_out[range.x + k] = tbits | (v >> 32);
      vals_out[range.x + k] = (uint32_t)v;
    }
  }

#ifdef GS_PROBE_NO_BLEND
  return;
#endif
  // Blend. Wave w shades the 8x8 quadrant q = w of the tile (x half w & 1, y half w >> 1), one
  // pixel per lane. Per batch of 256 sorted Gaussians staged in LDS, each work-item tests its
  // Gaussian's skip-threshold ellipse box against the four quadrants; a ballot + LDS offsets compact
  // that into four ordered per-quadrant lists, so a wave iterates only the Gaussians that can touch
  // its 64 pixels. Per pair: alpha = min(0.99, 2^(power*log2e + log2 o)) with the hardware exp2
  // (within 1e-4 relative L2 of the oracle's exp, test_raster_gpu.py).
  const uint32_t wave = tid >> 6, lane = tid & 63u;
  const uint32_t px = tile_x * GS_BLOCK_X + (wave & 1u) * 8u + (lane & 7u);
  const uint32_t py = tile_y * GS_BLOCK_Y + (wave >> 1) * 8u + (lane >> 3);
  const float tx0 = (float)(tile_x * GS_BLOCK_X), ty0 = (float)(tile_y * GS_BLOCK_Y);
  const bool inside = px < cam.W && py < cam.H;
  bool done = !inside;
  const float pfx = (float)px, pfy = (float)py;
  float T = 1.0f;
  float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
  int todo = (int)n;
  for (uint32_t base = 0; todo > 0; base += GS_BLOCK, todo -= GS_BLOCK) {
    if (__syncthreads_count(done) == GS_BLOCK) break;
    const uint32_t idx = base + tid;
    uint32_t m = 0;
    if (idx < n) {
      const uint32_t g = small ? (uint32_t)my_key : (uint32_t)(in_lds ? s_key[idx] : seg[idx]);
      const float4 ge = geo[g], co = conic_o[g], c = rgb[g];
      s_ga[tid] = make_float4(ge.x, ge.y, -0.5f * co.x, -co.y);
      s_gb[tid] = make_float4(-0.5f * co.z, __log2f(co.w), c.x, c.y);
      s_gc[tid] = c.z;
      const float x0 = ge.x - ge.z, x1 = ge.x + ge.z, y0 = ge.y - ge.w, y1 = ge.y + ge.w;
      const bool xl = x0 <= tx0 + 7.0f && x1 >= tx0, xr = x0 <= tx0 + 15.0f && x1 >= tx0 + 8.0f;
      const bool yt = y0 <= ty0 + 7.0f && y1 >= ty0, yb = y0 <= ty0 + 15.0f && y1 >= ty0 + 8.0f;
      m = (uint32_t)(xl && yt) | ((uint32_t)(xr && yt) << 1) | ((uint32_t)(xl && yb) << 2) |
          ((uint32_t)(xr && yb) << 3);
    }
    uint32_t rank[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned long long bal = __ballot((m >> q) & 1u);
      rank[q] = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      if (lane == 0) s_qcnt[wave][q] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if ((m >> q) & 1u) {
        uint32_t off = rank[q];
        for (uint32_t w2 = 0; w2 < wave; ++w2) off += s_qcnt[w2][q];
        s_list[q][off] = (uint16_t)tid;
      }
#ifdef GS_PROBE_NO_EVAL
    const uint32_t cnt = 0;
#else
    const uint32_t cnt = s_qcnt[0][wave] + s_qcnt[1][wave] + s_qcnt[2][wave] + s_qcnt[3][wave];
#endif
    __syncthreads();
    // wave-uniform trip count; the list is padded with the null Gaussian up to a multiple of 4
    const uint32_t cntu = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt);
    if (lane < 4) s_list[wave][cntu + lane] = (uint16_t)GS_BLOCK;
    const uint16_t* list = s_list[wave];
    for (uint32_t j = 0; j < cntu; j += 4) {
      if (__ballot(!done) == 0) break;
      const uint2 k4 = *reinterpret_cast<const uint2*>(list + j);  // 4 list entries
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t k = ((u < 2 ? k4.x : k4.y) >> (16 * (u & 1))) & 0xFFFFu;
        const float4 ga = s_ga[k], gb = s_gb[k];
        const float gcz = s_gc[k];
        const float dx = ga.x - pfx, dy = ga.y - pfy;
        const float power = __builtin_fmaf(__builtin_fmaf(ga.z, dx, ga.w * dy), dx, (gb.x * dy) * dy);
        const float z = __builtin_fmaf(power, 1.4426950408889634f, gb.y);
        // alpha >= 1/255 <=> z >= log2(1/255) = -7.99435; power > 0 is skipped as in the reference
        const bool valid = !done && power <= 0.0f && z >= -7.9943534f;
        float alpha = valid ? fminf(0.99f, __builtin_amdgcn_exp2f(z)) : 0.0f;
        float test_T = T * (1.0f - alpha);
        const bool term = valid && test_T < 0.0001f;  // saturated: stop before this Gaussian
        done = done || term;
        alpha = term ? 0.0f : alpha;
        test_T = term ? T : test_T;
        const float wgt = alpha * T;
        C0 = __builtin_fmaf(gb.z, wgt, C0);
        C1 = __builtin_fmaf(gb.w, wgt, C1);
        C2 = __builtin_fmaf(gcz, wgt, C2);
        T = test_T;
      }
    }
  }
  if (inside) out[(size_t)py * cam.W + px] = make_float4(C0 + T * bg_r, C1 + T * bg_g, C2 + T * bg_b, 1.0f - T);
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
  if ((e = ensure(w->touched, (size_t)n * 4))) return e;
  if ((e = ensure(w->ranges, (size_t)tiles * 8))) return e;
  if ((e = ensure(w->tile_local, (size_t)tiles * 8))) return e;
  if ((e = ensure(w->rect, (size_t)n * 8))) return e;
  if ((e = ensure(w->geo, (size_t)n * 16))) return e;
  const uint32_t scan_blocks = (tiles + GS_SCAN_TILES - 1) / GS_SCAN_TILES;
  if ((e = ensure(w->block_sum, (size_t)scan_blocks * 4))) return e;
  if ((e = ensure(w->block_off, (size_t)scan_blocks * 4))) return e;
  if (!w->ticket.p) {
    if ((e = ensure(w->ticket, 16))) return e;
    if ((e = hipMemset(w->ticket.p, 0, 16))) return e;
  }
  const bool lds_bins = tiles <= GS_LDS_TILES;
  static bool lds_attr_set = false;
  if (lds_bins && !lds_attr_set) {  // the tile histogram may exceed the default 64 KiB dynamic LDS
    if ((e = hipFuncSetAttribute((const void*)gs_bin_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 GS_LDS_TILES * 4)))
      return e;
    if ((e = hipFuncSetAttribute((const void*)gs_bin_scatter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 GS_LDS_TILES * 4)))
      return e;
    lds_attr_set = true;
  }
  // histogram rows: enough blocks to spread the LDS atomics, few enough to keep the column scan short
  const uint32_t nblk = lds_bins ? std::max(1u, std::min(64u, (n + 2047u) / 2048u)) : 1u;
  const uint32_t chunk = (n + nblk - 1) / nblk;
  if ((e = ensure(w->hist, (size_t)nblk * tiles * 4))) return e;
  if (!lds_bins && (e = ensure(w->cursor, (size_t)tiles * 4))) return e;
  if ((e = ensure(w->total, 16))) return e;
  if (!w->k_host) {
    if ((e = hipHostMalloc((void**)&w->k_host, 16, hipHostMallocCoherent | hipHostMallocMapped))) return e;
    if ((e = hipHostGetDevicePointer((void**)&w->k_dev, w->k_host, 0))) return e;
  }
  if (!w->k_event && (e = hipEventCreateWithFlags(&w->k_event, hipEventDisableTiming))) return e;
  // The pair buffer is sized from the previous frame's K (x1.25, at least 8 pairs per Gaussian) so
  // that scatter and blend are enqueued before K is known: the host then waits only for the small
  // K read-back while the GPU runs on; if K did not fit, both kernels did nothing, the buffers grow
  // and they run again (first frame / growth only).
  if (w->pairs.bytes < (size_t)n * 64) {
    if ((e = ensure(w->pairs, (size_t)n * 64))) return e;
    if ((e = ensure(w->keys_out, (size_t)n * 64))) return e;
    if ((e = ensure(w->vals_out, (size_t)n * 32))) return e;
  }
  auto cap_now = [&]() -> uint32_t {
    size_t c = std::min(std::min(w->pairs.bytes / 8, w->keys_out.bytes / 8), w->vals_out.bytes / 4);
    return (uint32_t)std::min<size_t>(c, 0xFFFFFFFFu);
  };

  if ((e = mark(0))) return e;
  if (n) {
    hipLaunchKernelGGL(gs_preprocess_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cam, g->means, g->scales,
                       g->rotations, g->opacities, g->colors, n, (float2*)w->means2d.p, (float*)w->depths.p,
                       (float4*)w->conic.p, (float4*)w->rgb.p, (int*)w->radii.p, (uint32_t*)w->touched.p,
                       (ushort4*)w->rect.p, (float4*)w->geo.p);
    if ((e = hipGetLastError())) return e;
  }
  if ((e = mark(1))) return e;
  if (!n || !lds_bins) {
    if ((e = hipMemsetAsync(w->hist.p, 0, (size_t)nblk * tiles * 4, s))) return e;
    if (!lds_bins && (e = hipMemsetAsync(w->cursor.p, 0, (size_t)tiles * 4, s))) return e;
  }
  if (n && lds_bins) {
    hipLaunchKernelGGL(gs_bin_count_kernel, dim3(nblk), dim3(GS_BIN_THREADS), tiles * 4, s,
                       (const ushort4*)w->rect.p, (const int*)w->radii.p, n, chunk, tiles, cam.grid_x,
                       (uint32_t*)w->hist.p);
    if ((e = hipGetLastError())) return e;
  } else if (n) {
    hipLaunchKernelGGL(gs_count_global_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const ushort4*)w->rect.p,
                       (const int*)w->radii.p, n, cam.grid_x, (uint32_t*)w->hist.p);
    if ((e = hipGetLastError())) return e;
  }
  hipLaunchKernelGGL(gs_bin_scan_kernel, dim3(scan_blocks), dim3(GS_SCAN_TILES), 0, s, (uint32_t*)w->hist.p, nblk,
                     tiles, (uint2*)w->tile_local.p, (uint32_t*)w->block_sum.p, (uint32_t*)w->block_off.p,
                     (uint32_t*)w->total.p, (uint32_t*)w->ticket.p, w->k_dev);
  if ((e = hipGetLastError())) return e;
  if ((e = hipEventRecord(w->k_event, s))) return e;
  if ((e = mark(2))) return e;

  const uint32_t rows = cam.row_end - cam.row_begin;
  auto enqueue_tail = [&](uint32_t cap) -> hipError_t {
    if (lds_bins) {
      hipLaunchKernelGGL(gs_bin_scatter_kernel, dim3(nblk), dim3(GS_BIN_THREADS), tiles * 4, s,
                         (const ushort4*)w->rect.p, (const int*)w->radii.p, (const float*)w->depths.p, n, chunk,
                         tiles, cam.grid_x, (const uint32_t*)w->hist.p, (const uint2*)w->tile_local.p,
                         (const uint32_t*)w->block_off.p, (const uint32_t*)w->total.p, cap, (uint2*)w->ranges.p,
                         (unsigned long long*)w->pairs.p);
    } else {
      hipLaunchKernelGGL(gs_ranges_kernel, dim3((tiles + 255) / 256), dim3(256), 0, s,
                         (const uint2*)w->tile_local.p, (const uint32_t*)w->block_off.p, tiles,
                         (const uint32_t*)w->total.p, cap, (uint2*)w->ranges.p);
      if (n)
        hipLaunchKernelGGL(gs_scatter_global_kernel, dim3((n + 255) / 256), dim3(256), 0, s,
                           (const ushort4*)w->rect.p, (const int*)w->radii.p, (const float*)w->depths.p, n,
                           cam.grid_x, (const uint2*)w->tile_local.p, (const uint32_t*)w->block_off.p,
                           (const uint32_t*)w->total.p, cap, (uint32_t*)w->cursor.p, (unsigned long long*)w->pairs.p);
    }
    hipError_t e2 = hipGetLastError();
    if (e2) return e2;
    if ((e2 = mark(3))) return e2;
    if ((e2 = mark(4))) return e2;
    if ((e2 = mark(5))) return e2;
    if (rows > 0) {
      hipLaunchKernelGGL(gs_sort_blend_kernel, dim3(cam.grid_x, rows), dim3(GS_BLOCK), 0, s, cam,
                         (const uint2*)w->ranges.p, (unsigned long long*)w->pairs.p,
                         (unsigned long long*)w->keys_out.p, (uint32_t*)w->vals_out.p, (const float4*)w->geo.p,
                         (const float4*)w->conic.p, (const float4*)w->rgb.p, bg[0], bg[1], bg[2],
                         (const uint32_t*)w->total.p, cap, (float4*)out);
      if ((e2 = hipGetLastError())) return e2;
    }
    return mark(6);
  };
  if ((e = enqueue_tail(cap_now()))) return e;
  if ((e = hipEventSynchronize(w->k_event))) return e;
  const uint32_t K = *w->k_host;
  if (K > cap_now()) {  // did not fit: grow (hipFree/hipMalloc order after the no-op kernels) and re-run
    if ((e = ensure(w->pairs, (size_t)K * 8))) return e;
    if ((e = ensure(w->keys_out, (size_t)K * 8))) return e;
    if ((e = ensure(w->vals_out, (size_t)K * 4))) return e;
    if (!lds_bins && (e = hipMemsetAsync(w->cursor.p, 0, (size_t)tiles * 4, s))) return e;
    if ((e = mark(2))) return e;
    if ((e = enqueue_tail(cap_now()))) return e;
  }
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
