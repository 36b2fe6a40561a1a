// splat.hip — 3D Gaussian splatting forward rasterizer for gfx950.
//
// The reference has no Gaussian rasterizer; this restates the published forward
// pass (Kerbl et al., SIGGRAPH 2023) in the reference's camera conventions (glm::lookAt RH view,
// Vulkan ZO projection with [1][1] negated, camera.cpp:186-187). Four launches per frame:
//   1. count        (band of tile rows x chunk of Gaussians) workgroups: preprocess one Gaussian per
//                   work-item (frustum cull (d <= 0.2), Sigma = R S^2 R^T, EWA Sigma' = J W Sigma W^T J^T
//                   (+0.3 low-pass), conic, 3-sigma radius, tile rect, a 48-B blend record), then the
//                   chunk's pairs into an LDS tile histogram (load-balanced wave expansion)
//   2. colscan      per 64 tiles: prefix of the histograms over the chunks, tile totals, K (to pinned
//                   host memory)
//   3. scatter      same grid as 1: (depth << 32 | gaussian) into each touched tile's segment through
//                   LDS cursors; tile ranges
//   4. sort+blend   one workgroup per 16x16 tile: sort by (depth, gaussian) (= the order of a stable
//                   global sort of (tile << 32 | depth) keys), publish keys/values, per-quadrant
//                   culled front-to-back alpha blend
// 3 and 4 are enqueued before K is read back (pair buffer sized from the previous frame, re-run on
// growth), so the host never stalls the GPU. Integer outputs (radii, tiles, keys, values, ranges)
// are the bit-exact contract with oracle/ptgs_oracle.c; the image is within 1e-4 relative L2
// (hardware exp2 in the blend).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "../../include/ptgs/ptgs.h"
#include "detmath.h"
#include "splat.h"
#include "splat_probe.h"

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
  uint32_t cull;                // tile rows restricted and chunk bounds given: PreArgs.cskip is valid
  uint32_t tight;               // bin by the alpha box (frames without stats / published buffers)
  uint32_t rowcull;             // tile rows restricted: Gaussians whose radius bound misses them skip the rest
  float fmax2;                  // max(fx^2, fy^2)
  float w2;                     // an upper bound of the view rotation's squared spectral norm (1 for lookAt)
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct SplatWorkspace {
  DevBuf means2d, depths, conic, rec, radii, touched, pairs, keys_out, vals_out, ranges, hist, tile_info,
      group_total, tile_slots, point_keys, total, rect, large, large_ctr, sort_scratch;
  DevBuf cursor, fz, pub_offs, keys_pub, vals_pub;  // fused front end (see gs_bin_fused_kernel); fz: counters
  DevBuf dbg_depths, fzp, nzbuf, order;  // order: the blend's tile order (heavy first, fused frames)
  DevBuf crect, sp_keys, sp_vals;  // spilled tiles (gs_spill_tile): chunk rects, the spill pool
  DevBuf fsq;                 // the fused front end's slice queue
  DevBuf cskip;               // per 256-Gaussian chunk: skipped by a tile-row-restricted frame
  uint32_t sp_cap = 0;        // spill pool capacity (pairs)
  uint32_t incomplete = 0;    // frames reported incomplete (spill pool exhausted) since the last status clear
  uint32_t spilled_base = 0, incomplete_base = 0;  // device counters fz[9] / fz[10] at the last status clear
  bool ids_error = false;     // a frame met an out-of-range ptgs_gaussians.ids entry
  bool have_hint = false;     // a finished frame has published its largest tile: the fused path can size its rows
  bool hint_recorded = false;
  hipEvent_t hint_event = nullptr;
  bool last_fused = false;    // the last frame ran the fused front end
  uint32_t last_scap = 0;     // and its slot rows' capacity (ptgs_splat_get_tile_rows)
  uint32_t* k_host = nullptr;  // pinned, coherent [16]: K, largest tile, large tiles, -, touched runs,
                               // fused overflow, publishing path (1 fused / 2 three), -, spill demand,
                               // incomplete tile, bad ids, queued front-end slices, largest K (fused),
                               // largest K (three launches)
  uint32_t* k_dev = nullptr;   // its device-side address
  hipEvent_t k_event = nullptr;
  uint32_t last_n = 0, last_k = 0, last_tiles = 0;
  bool last_published = false;  // the last frame published its sorted keys / values and was synchronised
  uint32_t sort_r = 3;        // large-tile radix sort: items per work-item (from the previous frame's largest tile)
  uint32_t sort_grid = 256;   // its workgroups (from the previous frame's large-tile count)
  bool sort_attr = false;     // its dynamic-LDS limit raised
  hipEvent_t ev[7] = {};
  bool timed = false;
};

SplatWorkspace* splat_workspace_create() { return new SplatWorkspace(); }

void splat_workspace_destroy(SplatWorkspace* w) {
  if (!w) return;
  DevBuf* all[] = {&w->means2d, &w->depths, &w->conic, &w->rec, &w->radii, &w->touched, &w->pairs, &w->keys_out,
                   &w->vals_out, &w->ranges, &w->hist, &w->tile_info, &w->group_total, &w->tile_slots, &w->point_keys,
                   &w->total, &w->rect, &w->large, &w->large_ctr, &w->sort_scratch, &w->cursor, &w->fz,
                   &w->pub_offs, &w->keys_pub, &w->vals_pub, &w->dbg_depths, &w->fzp, &w->nzbuf, &w->order,
                   &w->crect, &w->sp_keys, &w->sp_vals, &w->fsq, &w->cskip};
  for (DevBuf* b : all)
    if (b->p) (void)hipFree(b->p);
  if (w->k_host) (void)hipHostFree(w->k_host);
  for (hipEvent_t& e : w->ev)
    if (e) (void)hipEventDestroy(e);
  if (w->k_event) (void)hipEventDestroy(w->k_event);
  if (w->hint_event) (void)hipEventDestroy(w->hint_event);
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

struct PreArgs {
  const float *means, *scales, *rots, *opac, *colors;
  uint32_t n;
  float2* means2d;
  float* depths;      // walk order (i): the three-launch scatter's depths
  float* dbg_depths;  // caller order (o): ptgs_splat_get_buffers
  float4* conic_o;
  int* radii;
  uint32_t* touched;
  ushort4* rects;
  float4* rec;
  const uint32_t* ids;  // caller's index of Gaussian i (NULL: i): keys, values, records and the
                        // per-Gaussian outputs use it, so a reordered set renders like the original
  uint32_t* bad_ids;    // pinned host word set to 1 when an id is >= n (the Gaussian is dropped)
  const uint8_t* cskip;  // per 256-Gaussian chunk: 1 = its bound misses the frame's rows (gs_chunk_cull_kernel)
  const float4* cbounds;  // the chunk bounds themselves (the fused front end tests its own chunk: no cull launch)
};

// Image stores stream past L2 (non-temporal): C2 0.0686 -> 0.0677 ms, fewer dirty lines at the kernel end.
// (Non-temporal blend records and key rows measured slower: the blend reads both right after.)
__device__ __forceinline__ void gs_st4_nt(float4* p, const float4& v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
}
// (Write-through (sc1) stores, which leave the XCD's L2 at once instead of at the kernel-end release,
// measured slower for every output: image 0.0633, key rows 0.0585, records 0.0603, all 0.0679 vs 0.0565 ms.)

// Upper bound (px) of the 3-sigma radius of a Gaussian of largest scale s at view-space point (x, y, d),
// d > 0.2: radius = ceil(3 sqrt(l1)) with l1 <= lambda_max(cov) + sqrt(0.1) (the max(0.1, .) clamp of
// gs_preprocess_one), cov = T Sigma T^T + 0.3 I, T = J W, so lambda_max(cov) <= |J|_2^2 |W|_2^2 s^2 + 0.3
// with |J|_2^2 = max(fx, fy)^2 (1 + a^2 + b^2) / d^2 (J = diag(fx, fy) / d [[1, 0, -a], [0, 1, -b]], a and b
// the clamped x / d and y / d of the EWA Jacobian). 1% and 2 px absorb the float rounding of both sides.
__device__ __forceinline__ float gs_radius_bound(const SplatCam& cam, float a, float b, float d, float s) {
  const float lam = cam.fmax2 * ((1.0f + a * a) + b * b) / (d * d) * cam.w2 * (s * s);
  return 3.0f * sqrtf(1.01f * (lam + 0.62f)) + 2.0f;
}

// Row pre-cull of a tile-row-restricted frame (cam.rowcull): from the mean and the scales only (one load
// round trip before the rotation / opacity / colour loads), true when the Gaussian cannot reach the
// frame's tile rows: its rect rows [(int)((y - r) / 16), (int)((y + r + 15) / 16)) miss [row_begin,
// row_end) for every r <= the radius bound (the exact rect is then empty: the skip is exact). False for
// d <= 0.2 and non-finite values (the exact path decides).
__device__ __forceinline__ bool gs_row_miss(const SplatCam& cam, float mx, float my, float mz, float sx, float sy,
                                            float sz) {
  const v4 pv = mv4(cam.view, mx, my, mz, 1.0f);
  const float d = -pv.z;
  if (!(d > 0.2f)) return false;
  const v4 ph = mv4(cam.mvp, mx, my, mz, 1.0f);
  const float y = ndc2pix(ph.y * (1.0f / (ph.w + 0.0000001f)), (int)cam.H);
  const float limx = 1.3f * cam.tan_fovx, limy = 1.3f * cam.tan_fovy;
  const float a = fminf(limx, fmaxf(-limx, pv.x / d)), b = fminf(limy, fmaxf(-limy, pv.y / d));
  const float R = gs_radius_bound(cam, a, b, d, fmaxf(fabsf(sx), fmaxf(fabsf(sy), fabsf(sz))));
  const float t = (float)GS_BLOCK_Y;
  return (y + R + t < t * (float)cam.row_begin) || (y - R - t > t * (float)cam.row_end);
}

// One Gaussian: frustum cull (d <= 0.2), Sigma = R S^2 R^T, EWA Sigma' = J W Sigma W^T J^T + 0.3,
// conic, 3-sigma radius, tile rect (returned; empty if culled) and, with STORE, every per-Gaussian
// output incl. the blend record. (Blocks of other bands recompute the rect without storing.)
// ROWCULL: a tile-row-restricted frame (cam.rowcull), its own instantiation of the front-end kernels (the
// full frame's preprocess keeps its single load round trip, unchanged code)
template <bool STORE, bool ROWCULL = false>
__device__ __forceinline__ ushort4 gs_preprocess_one(const SplatCam& cam, const PreArgs& A, uint32_t i,
                                                     float* dep_out = nullptr) {
  const float* __restrict__ means = A.means;
  const float* __restrict__ scales = A.scales;
  const float* __restrict__ rots = A.rots;
  const float* __restrict__ opac = A.opac;
  const float* __restrict__ colors = A.colors;
  float2* __restrict__ means2d = A.means2d;
  float* __restrict__ depths = A.depths;
  float4* __restrict__ conic_o = A.conic_o;
  int* __restrict__ radii = A.radii;
  uint32_t* __restrict__ touched = A.touched;
  ushort4* __restrict__ rects = A.rects;
  float4* __restrict__ rec = A.rec;
  const ushort4 none = make_ushort4(0, 0, 0, 0);
  // per-Gaussian outputs: rec (the blend's records) always; rects / depths (the three-launch scatter's
  // walk, at i) and radii / touched / means2d / conic (ptgs_splat_get_buffers) when their pointers are
  // set (the fused path without PTGS_FLAG_SPLAT_PUBLISH leaves them out)
  const uint32_t o = A.ids ? A.ids[i] : i;
  float mx = means[3 * i], my = means[3 * i + 1], mz = means[3 * i + 2];
  float sx = scales[3 * i], sy = scales[3 * i + 1], sz = scales[3 * i + 2];
  float qr = 0.0f, qx = 0.0f, qy = 0.0f, qz = 0.0f, op = 0.0f, cr = 0.0f, cg = 0.0f, cbl = 0.0f;
  bool miss = false;
  if (!ROWCULL) {
    // every input is loaded here, with the id and before the id check and the depth test: one memory round
    // trip per Gaussian (loads behind either branch were issued only once the id / the means had arrived)
    qr = rots[4 * i]; qx = rots[4 * i + 1]; qy = rots[4 * i + 2]; qz = rots[4 * i + 3];
    op = opac[i];
    if (STORE) {
      cr = colors[3 * i];
      cg = colors[3 * i + 1];
      cbl = colors[3 * i + 2];
      asm volatile("" : "+v"(cr), "+v"(cg), "+v"(cbl));
    }
    // (the empty asm needs the values here, so the compiler cannot sink the loads behind the branches)
    asm volatile("" : "+v"(mx), "+v"(my), "+v"(mz), "+v"(qr), "+v"(qx), "+v"(qy), "+v"(qz), "+v"(sx), "+v"(sy),
                 "+v"(sz), "+v"(op));
  } else {
    // a tile-row shard: most Gaussians miss its rows; the rest of the inputs are loaded only for those
    // whose radius bound reaches them (a second round trip for them, none for the others)
    miss = gs_row_miss(cam, mx, my, mz, sx, sy, sz);
    if (!miss) {
      qr = rots[4 * i]; qx = rots[4 * i + 1]; qy = rots[4 * i + 2]; qz = rots[4 * i + 3];
      op = opac[i];
      if (STORE) {
        cr = colors[3 * i];
        cg = colors[3 * i + 1];
        cbl = colors[3 * i + 2];
      }
    }
  }
  if (STORE && rects) rects[i] = none;  // empty rect: the scatter reads rects only
  if (o >= A.n) {  // ids must be a permutation of [0, n): an index outside it is dropped, not written
    if (STORE) __atomic_store_n(A.bad_ids, 1u, __ATOMIC_RELAXED);  // (reported by the next call)
    return none;
  }
  if (STORE && radii) {
    radii[o] = 0;
    touched[o] = 0;
  }
  if (miss) return none;
  // frustum: view-space depth d = -z (RH, camera looks down -Z)
  v4 pv = mv4(cam.view, mx, my, mz, 1.0f);
  float d = -pv.z;
  if (dep_out) *dep_out = d;
  if (d <= 0.2f) return none;
  v4 ph = mv4(cam.mvp, mx, my, mz, 1.0f);
  float pw = 1.0f / (ph.w + 0.0000001f);
  float px = ph.x * pw, py = ph.y * pw;

  // Sigma = R S^2 R^T
  float qn = sqrtx(((qr * qr + qx * qx) + qy * qy) + qz * qz);
  qr = qr / qn; qx = qx / qn; qy = qy / qn; qz = qz / qn;
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
  if (det == 0.0f) return none;
  float det_inv = 1.0f / det;
  float4 con = make_float4(cc * det_inv, -cb * det_inv, ca * det_inv, op);
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
  // (ex, ey): half-extents of the ellipse where alpha >= 1/255 can hold (power >= -ln(255 o), minus a
  // 1e-3 margin, +1% and +0.01 px): the blend skips whole 8x8 pixel blocks outside that box
  const float skip = -(log2x(255.0f * con.w) * 0.69314718055994531f) - 0.001f;
  const float sq = -2.0f * skip;
  const float ex = sq > 0.0f ? sqrtx(sq * ca) * 1.01f + 0.01f : -1.0f;
  const float ey = sq > 0.0f ? sqrtx(sq * cc) * 1.01f + 0.01f : -1.0f;
  if (cam.tight) {
    // Timed frames bin each Gaussian only to the tiles its alpha box overlaps (pixel x in [16 t, 16 t +
    // 15]); the reference's 3-sigma rectangle (kept for stats and published buffers) also holds tiles
    // where no pixel reaches alpha 1/255: 29% of C2's pairs. The blend skips such a pair (alpha 0:
    // T and colour unchanged, exactly), so the image is the same, bit for bit.
    if (!(sq > 0.0f)) return none;
    rmin_x = max(rmin_x, (int)__builtin_ceilf((pimg.x - ex - (float)(GS_BLOCK_X - 1)) * (1.0f / GS_BLOCK_X)));
    rmax_x = min(rmax_x, (int)__builtin_floorf((pimg.x + ex) * (1.0f / GS_BLOCK_X)) + 1);
    rmin_y = max(rmin_y, (int)__builtin_ceilf((pimg.y - ey - (float)(GS_BLOCK_Y - 1)) * (1.0f / GS_BLOCK_Y)));
    rmax_y = min(rmax_y, (int)__builtin_floorf((pimg.y + ey) * (1.0f / GS_BLOCK_Y)) + 1);
  }
  int area = (rmax_x - rmin_x) * (rmax_y - rmin_y);
  if (rmax_x <= rmin_x || rmax_y <= rmin_y || area == 0) return none;
  const ushort4 rect = make_ushort4((unsigned short)rmin_x, (unsigned short)rmin_y, (unsigned short)rmax_x,
                                    (unsigned short)rmax_y);
  if (!STORE) return rect;
  if (rects) {
    depths[i] = d;
    rects[i] = rect;
  }
  if (radii) {
    A.dbg_depths[o] = d;
    radii[o] = r;
    means2d[o] = pimg;
    conic_o[o] = con;
    touched[o] = (uint32_t)area;
  }
  // Blend record (3 x float4), the form the blend loop consumes:
  //   (x, y, A, B), (C, log2 o, r, g), (b, ex, ey, depth)  with  A = -a/2 log2e, B = -b log2e, C = -c/2 log2e
  // so that z = A dx^2 + B dx dy + C dy^2 + log2 o = power * log2e + log2 o and alpha = min(0.99, 2^z).
  // (ex, ey): the alpha box (above).
  const float L2E = 1.4426950408889634f;
  rec[3 * o] = make_float4(pimg.x, pimg.y, -0.5f * con.x * L2E, -con.y * L2E);
  rec[3 * o + 1] = make_float4(-0.5f * con.z * L2E, __log2f(con.w), cr, cg);
  rec[3 * o + 2] = make_float4(cbl, ex, ey, d);
  return rect;
}

// Can any Gaussian of a chunk touch a tile of the frame's rows (cam.row_begin, row_end) and columns?
// Conservative, from the chunk's bounds (box of the means, largest scale): view depths over the box's
// corners are exact (linear); every mean projects inside the hull of the corners' projections when all
// of them lie in front of the camera; and a Gaussian's 3-sigma radius is at most
// 3 sqrt(|J|_F^2 |W|_F^2 s_max^2 + 0.3 + sqrt(0.1)) + 1 px with |J|_F^2 <= (fx^2 (1 + (1.3 tan_x)^2)
// + fy^2 (1 + (1.3 tan_y)^2)) / d_min^2 (the EWA Jacobian at the clamped point, gs_preprocess_one).
// Margins of 1 % and a tile on every side absorb the rounding. Returns true when the chunk is sure to
// contribute nothing: every mean within the near plane (d <= 0.2), or its bound misses the rows /
// columns. Unbounded cases (a corner close to the camera, non-finite bounds) return false.
__device__ __forceinline__ bool gs_chunk_misses(const SplatCam& cam, const float4 lo, const float4 hi) {
  if (!(isfinite(lo.x) && isfinite(lo.y) && isfinite(lo.z) && isfinite(hi.x) && isfinite(hi.y) && isfinite(hi.z) &&
        isfinite(lo.w)))
    return false;
  float dmin = INFINITY, dmax = -INFINITY, xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
  bool front = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float x = (k & 1) ? hi.x : lo.x, y = (k & 2) ? hi.y : lo.y, z = (k & 4) ? hi.z : lo.z;
    const v4 pv = mv4(cam.view, x, y, z, 1.0f);
    const v4 ph = mv4(cam.mvp, x, y, z, 1.0f);
    const float d = -pv.z;
    dmin = fminf(dmin, d);
    dmax = fmaxf(dmax, d);
    front = front && ph.w > 0.1f;
    const float iw = 1.0f / ph.w;
    const float sx = ndc2pix(ph.x * iw, (int)cam.W), sy = ndc2pix(ph.y * iw, (int)cam.H);
    xmin = fminf(xmin, sx);
    xmax = fmaxf(xmax, sx);
    ymin = fminf(ymin, sy);
    ymax = fmaxf(ymax, sy);
  }
  if (dmax < 0.19f) return true;                // every Gaussian is culled by the near test
  if (dmin < 0.25f || !front) return false;     // too close to bound the projection
  // the largest |x / d|, |y / d| over the box: at its corners (x / d is linear-fractional, d > 0 on the box),
  // clamped like the EWA Jacobian's; the radius bound of gs_radius_bound at the nearest depth
  float amax = 0.0f, bmax = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float x = (k & 1) ? hi.x : lo.x, y = (k & 2) ? hi.y : lo.y, z = (k & 4) ? hi.z : lo.z;
    const v4 pv = mv4(cam.view, x, y, z, 1.0f);
    amax = fmaxf(amax, fabsf(pv.x / -pv.z));
    bmax = fmaxf(bmax, fabsf(pv.y / -pv.z));
  }
  amax = fminf(amax * 1.001f, 1.3f * cam.tan_fovx);
  bmax = fminf(bmax * 1.001f, 1.3f * cam.tan_fovy);
  const float R = gs_radius_bound(cam, amax, bmax, dmin * 0.999f, lo.w) + 1.0f;  // px
  if (!isfinite(R)) return false;
  const float t = (float)GS_BLOCK_Y;
  const float r0 = floorf((ymin - R) / t) - 1.0f, r1 = floorf((ymax + R + t) / t) + 1.0f;  // rows [r0, r1]
  const float c0 = floorf((xmin - R) / t) - 1.0f, c1 = floorf((xmax + R + t) / t) + 1.0f;
  return r1 < (float)cam.row_begin || r0 >= (float)cam.row_end || c1 < 0.0f || c0 >= (float)cam.grid_x;
}

// The stores a Gaussian of a skipped chunk owes: the empty rect (the scatter and gs_spill_tile read
// it) and, on a published frame, zero radius / tiles touched
__device__ __forceinline__ void gs_store_skipped(const PreArgs& A, uint32_t i) {
  if (A.rects) A.rects[i] = make_ushort4(0, 0, 0, 0);
  if (A.radii) {
    const uint32_t o = A.ids ? A.ids[i] : i;
    if (o < A.n) {
      A.radii[o] = 0;
      A.touched[o] = 0;
    }
  }
}

// One flag per 256-Gaussian chunk for a tile-row-restricted frame (its own small launch, so that the
// front-end kernels keep no bound arithmetic: they read the flag before loading a chunk)
__global__ __launch_bounds__(256) void gs_chunk_cull_kernel(SplatCam cam, const float4* __restrict__ cb, uint32_t nch,
                                                            uint8_t* __restrict__ skip) {
  const uint32_t c = blockIdx.x * 256u + threadIdx.x;
  if (c < nch) skip[c] = gs_chunk_misses(cam, cb[2 * c], cb[2 * c + 1]) ? 1 : 0;
}

// ---- binning --------------------------------------------------------------------------------------
// No global atomics per pair (contended scattered atomics measured 100 us for C2's 617k pairs). The
// grid is (bands, chunks): a band is a run of band_rows tile rows (as many as fit GS_BAND_TILES: the
// whole 1080p frame is one band, 4K takes 4), a chunk a contiguous range of Gaussians.
//  count    block (band, c) preprocesses chunk c (band-0 blocks store the per-Gaussian outputs, the
//           others only recompute the rects) and counts the chunk's pairs in its band into an LDS
//           histogram (ds_add), written to hist[c][t].
//  colscan  one block per 64 tiles: hist[c][t] -> exclusive prefix over the chunks (in place), the
//           tile totals, their exclusive scan inside the 64-tile group and the group totals; K and
//           the largest tile go to pinned host memory (last block).
//  scatter  block (band, c): tile starts = scan of the group totals + in-group offset; re-walks chunk
//           c and places each pair at start[t] + hist[c][t] + (LDS cursor). Chunk-0 blocks publish
//           the ranges.
// Order inside a tile's segment depends on LDS atomic order and is fixed by the blend's per-tile sort.
#define GS_BIN_THREADS 1024
#ifndef GS_COUNT_THREADS
#define GS_COUNT_THREADS 1024  // the count's workgroup (the scatter keeps GS_BIN_THREADS)
#endif
#define GS_MAX_CHUNKS 1024   // colscan: 16 waves x up to 64 chunks each
#ifndef GS_CHUNK_MIN
#define GS_CHUNK_MIN 512     // Gaussians per chunk (at least)
#endif
#define GS_BAND_TILES 8192   // max tiles per band (LDS: 32 KiB count, 64 KiB scatter); W <= 131072 px
#define GS_TILE_SLOTS 256    // fixed key slots per tile (= the register-sort limit)
#define GS_MID 512           // tiles of (256, GS_MID] pairs are sorted inside the blend (rank counting)
#define GS_MAX_GROUPS 4096   // 64-tile groups (262144 tiles)

// Inclusive wave64 prefix sum in DPP (row_shr 1/2/4/8 inside rows of 16, then row_bcast 15 / 31
// across rows): six VALU adds instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// The bands cover the frame's tile rows [row0, row1) only (a tile-row shard bins its own rows: one band of
// up to GS_MAX_CHUNKS chunks instead of the whole frame's bands); the 64-tile groups start at row0's first
// tile. hist, tile_info and ranges keep the frame's global tile ids (tiles = grid_x * grid_y).
// Wave64 min / max / sum in DPP (the scan pattern of wave_incl_scan: lane 63 ends with the reduction of
// all 64) and broadcast from lane 63: six VALU steps with no LDS round trip, where the __shfl_xor
// butterfly is six dependent ds_bpermute round trips.
template <int OP>  // 0 min, 1 max, 2 sum
__device__ __forceinline__ uint32_t wave_reduce(uint32_t x) {
  const int id = OP == 0 ? -1 : 0;  // (0xFFFFFFFF: the identity of an unsigned min)
  auto f = [](uint32_t a, uint32_t b) { return OP == 0 ? min(a, b) : OP == 1 ? max(a, b) : a + b; };
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
  x = f(x, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// x of lane ^ J without LDS: DPP inside rows of 16 (quad_perm for 1 / 2; half-row / row mirrors composed
// with them for 4 / 8) and the gfx950 permlane swaps across rows (16) and halves (32)
template <uint32_t J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, uint32_t lane) {
  if (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
  if (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
  if (J == 4) {  // (i ^ 7) ^ 3
    const int t = __builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    return (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x1B, 0xF, 0xF, false);     // quad_perm 3,2,1,0
  }
  if (J == 8) {  // (i ^ 15) ^ 7
    const int t = __builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    return (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x141, 0xF, 0xF, false);    // row_half_mirror
  }
  if (J == 16) {  // odd rows of the first result, even rows of the second (the rows as a constant lane mask)
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __builtin_amdgcn_inverse_ballot_w64(0xFFFF0000FFFF0000ull) ? r[0] : r[1];
  }
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // J == 32
  return __builtin_amdgcn_inverse_ballot_w64(0xFFFFFFFF00000000ull) ? r[0] : r[1];
}
template <uint32_t J>
__device__ __forceinline__ unsigned long long lane_xor64(unsigned long long x, uint32_t lane) {
  return ((unsigned long long)lane_xor<J>((uint32_t)(x >> 32), lane) << 32) | lane_xor<J>((uint32_t)x, lane);
}

struct BinGrid {
  uint32_t band_rows, bands, chunks, chunk, grid_x, grid_y, tiles, groups, row0, row1;
};

__device__ __forceinline__ void gs_band(const BinGrid& bg, uint32_t& ty0, uint32_t& ty1) {
  ty0 = bg.row0 + blockIdx.x * bg.band_rows;
  ty1 = min(bg.row1, ty0 + bg.band_rows);
}

// Pairs of one wave's 64 entries (gaussian g, x0 | w << 16, y0 | h << 16; h = 0: none), walked 64 per
// step: a shuffle scan of the rect areas; lane q's pair belongs to the first entry whose inclusive
// sum exceeds q (6-step binary search over shuffles), its tile is (x0 + r % w, y0 + r / w) for its
// rank r inside that rect. Every lane works on every step but the last (a per-Gaussian rect loop
// idles the lanes of the smaller rects: C2's rects hold 1 to ~100 tiles). f(g, x, y, depth).
template <bool WANT_DEPTH, typename F>
__device__ __forceinline__ void gs_expand(uint32_t lane, uint32_t eg, uint32_t exw, uint32_t eyh, float dep, F f) {
  const uint32_t a = (exw >> 16) * (eyh >> 16);
  const uint32_t incl = wave_incl_scan(a);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(incl, 63));
  const uint32_t excl = incl - a;
  for (uint32_t p = 0; p < total; p += 64) {
    const uint32_t qi = p + lane;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) lo = __shfl(incl, (int)(lo + step - 1)) <= qi ? lo + step : lo;
    const uint32_t og = __shfl(eg, (int)lo), oxw = __shfl(exw, (int)lo), oy = __shfl(eyh, (int)lo);
    const uint32_t oex = __shfl(excl, (int)lo);
    const float od = WANT_DEPTH ? __shfl(dep, (int)lo) : 0.0f;
    if (qi < total) {
      const uint32_t r = qi - oex, ow = oxw >> 16;
      uint32_t row = (uint32_t)((float)r * __builtin_amdgcn_rcpf((float)ow));  // r < 2^13: off by <= 1
      row = row * ow > r ? row - 1 : row;
      row = (row + 1) * ow <= r ? row + 1 : row;
      f(og, (oxw & 0xFFFFu) + (r - row * ow), (oy & 0xFFFFu) + row, od);
    }
  }
}

__device__ __forceinline__ void gs_clip(const ushort4& rc, uint32_t ty0, uint32_t ty1, uint32_t& xw, uint32_t& yh) {
  const uint32_t y0 = max((uint32_t)rc.y, ty0), y1 = min((uint32_t)rc.w, ty1);
  const bool hit = y0 < y1 && rc.x < rc.z;  // culled Gaussians hold the empty rect
  xw = (uint32_t)rc.x | ((uint32_t)(rc.z - rc.x) << 16);
  yh = hit ? (y0 | ((y1 - y0) << 16)) : 0u;
}

// Scatter's walk of chunk blockIdx.y inside the band: with several bands most rects miss the band, so
// each wave first filters (64 rects per step, GS_WALK_PF steps in flight; ballot + mbcnt append the
// hits to its GS_WQ-entry LDS ring) and expands 64 queued entries at a time (depths gathered then).
#define GS_WQ 128
#define GS_WALK_PF 4
template <typename F>
__device__ __forceinline__ void gs_walk_chunk(const BinGrid& bg, const ushort4* __restrict__ rects,
                                              const float* __restrict__ depths, const uint32_t* __restrict__ ids,
                                              uint32_t n, uint32_t ty0, uint32_t ty1, uint4* s_q, F f) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t b0 = blockIdx.y * bg.chunk, b1 = min(n, b0 + bg.chunk);
  const ushort4 zero = make_ushort4(0, 0, 0, 0);
  uint4* q = s_q + wave * GS_WQ;
  uint32_t base = b0 + wave * 64u;
  ushort4 pf[GS_WALK_PF];
#pragma unroll
  for (int k = 0; k < GS_WALK_PF; ++k) {  // (if/else: a ?: of two ushort4 lvalues selects addresses -> FLAT)
    const uint32_t i = base + k * GS_BIN_THREADS + lane;
    pf[k] = zero;
    if (i < b1) pf[k] = rects[i];
  }
  uint32_t head = 0, cnt = 0;  // wave-uniform ring state
  for (;;) {
    while (cnt < 64u && base < b1) {
      const ushort4 rc = pf[0];
#pragma unroll
      for (int k = 0; k < GS_WALK_PF - 1; ++k) pf[k] = pf[k + 1];
      {
        const uint32_t i = base + GS_WALK_PF * GS_BIN_THREADS + lane;
        pf[GS_WALK_PF - 1] = zero;
        if (i < b1) pf[GS_WALK_PF - 1] = rects[i];
      }
      uint32_t xw, yh;
      gs_clip(rc, ty0, ty1, xw, yh);
      const unsigned long long bal = __ballot(yh != 0u);
      if (bal) {
        if (yh) {
          const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          q[(head + cnt + pos) & (GS_WQ - 1u)] = make_uint4(base + lane, xw, yh, ids ? ids[base + lane] : base + lane);
        }
        cnt += (uint32_t)__popcll(bal);
      }
      base += GS_BIN_THREADS;
    }
    if (cnt == 0) break;
    const uint32_t take = min(64u, cnt);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 e = lane < take ? q[(head + lane) & (GS_WQ - 1u)] : make_uint4(0u, 0u, 0u, 0u);
    head += take;
    cnt -= take;
    const float dep = lane < take ? depths[e.x] : 0.0f;
    gs_expand<true>(lane, e.w, e.y, e.z, dep, f);  // (e.w: the caller's index for the key)
  }
}

// The blend's tile order, built by one extra workgroup of the front end's first launch (fused or
// count) while the others bin: the tiles [tb, te) by the previous frame's pair count, heaviest first (a counting
// sort on min(255, n / 2), descending; the order inside a bucket is the LDS atomics'). The blend's
// workgroups are dispatched in index order, so its long-running tiles start first and the kernel's
// ramp-down runs light tiles only. Any permutation renders the same image: the previous frame's
// counts (ranges[t].y - .x, whatever path wrote them) only steer the schedule.
#define GS_ORDER_BUCKETS 256u
#define GS_ORDER_B 4u  // previous tile counts in flight per work-item (16: 104 VGPRs in the front-end kernels)
// (order[b] = the tile. Carrying the previous frame's count of the tile in the word, so the blend loads
// only that much of the key row with the tile, measured slower: C2 0.0594 vs 0.0588 ms)
__device__ __forceinline__ uint32_t gs_order_bucket_n(uint32_t n) {
  return GS_ORDER_BUCKETS - 1u - min(GS_ORDER_BUCKETS - 1u, n >> 1);
}
__device__ __forceinline__ uint32_t gs_order_bucket(uint2 r) { return gs_order_bucket_n(r.y > r.x ? r.y - r.x : 0u); }
// (COUNTS: prev holds one u32 pair count per tile, the fused front end's cursors of the frame itself)
template <bool COUNTS = false>
__device__ __forceinline__ uint32_t gs_order_bucket_at(const void* prev, uint32_t t) {
  return COUNTS ? gs_order_bucket_n(static_cast<const uint32_t*>(prev)[t]) : gs_order_bucket(static_cast<const uint2*>(prev)[t]);
}
template <bool COUNTS = false>
__device__ void gs_tile_order(const void* __restrict__ prev, uint32_t* __restrict__ order, uint32_t tb, uint32_t te,
                              uint32_t* s_h /* >= GS_ORDER_BUCKETS */) {
  // (the previous counts are loaded GS_ORDER_B per work-item at a time, all in flight before the first
  // is used: a loop of one load and one LDS atomic per iteration waited for every load, 16 dependent
  // round trips per pass at 1080p on the front end's critical path)
  const uint32_t tid = threadIdx.x, lane = tid & 63u, nth = blockDim.x;  // (>= 64)
  for (uint32_t b = tid; b < GS_ORDER_BUCKETS; b += nth) s_h[b] = 0;
  __syncthreads();
  for (uint32_t t0 = tb + tid; t0 < te; t0 += GS_ORDER_B * nth) {
    uint32_t bk[GS_ORDER_B];
#pragma unroll
    for (uint32_t j = 0; j < GS_ORDER_B; ++j) {
      const uint32_t t = t0 + j * nth;
      bk[j] = t < te ? gs_order_bucket_at<COUNTS>(prev, t) : GS_ORDER_BUCKETS;
    }
#pragma unroll
    for (uint32_t j = 0; j < GS_ORDER_B; ++j)
      if (bk[j] < GS_ORDER_BUCKETS) atomicAdd(s_h + bk[j], 1u);
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the buckets: one wave, four per lane
    const uint32_t c0 = s_h[4 * lane], c1 = s_h[4 * lane + 1], c2 = s_h[4 * lane + 2], c3 = s_h[4 * lane + 3];
    const uint32_t sum = (c0 + c1) + (c2 + c3);
    const uint32_t ex = wave_incl_scan(sum) - sum;
    s_h[4 * lane] = ex;
    s_h[4 * lane + 1] = ex + c0;
    s_h[4 * lane + 2] = ex + c0 + c1;
    s_h[4 * lane + 3] = ex + c0 + c1 + c2;
  }
  __syncthreads();
  for (uint32_t t0 = tb + tid; t0 < te; t0 += GS_ORDER_B * nth) {
    uint32_t bk[GS_ORDER_B];
#pragma unroll
    for (uint32_t j = 0; j < GS_ORDER_B; ++j) {
      const uint32_t t = t0 + j * nth;
      bk[j] = t < te ? gs_order_bucket_at<COUNTS>(prev, t) : GS_ORDER_BUCKETS;
    }
#pragma unroll
    for (uint32_t j = 0; j < GS_ORDER_B; ++j)
      if (bk[j] < GS_ORDER_BUCKETS) order[atomicAdd(s_h + bk[j], 1u)] = t0 + j * nth;
  }
}

// The tile order of an overlapped fused frame (SplatOverlap::own_order), from the frame's OWN pair counts
// (the cursors its front end has just reserved): it runs on the front-end stream behind the front end,
// off the caller's stream, where the blend of the previous frame hides it; the in-kernel order
// workgroup of a serial frame can only use the previous frame's counts.
// Up to GS_ORDER_R * GS_ORDER_THREADS tiles (1080p: 8 160) each work-item keeps its tiles' buckets in
// registers (one load round) and the histogram has GS_ORDER_COLS columns per bucket, one per lane & 15:
// the LDS atomics of a wave's lanes on one bucket (most light tiles share a few buckets) meet 4-way
// instead of 64-way (a single-column histogram serialised ~8k same-address atomics per pass, ~3.5 us).
// Larger grids (4K) take the generic two-pass order.
#ifndef GS_ORDER_THREADS
#define GS_ORDER_THREADS 1024
#endif
#define GS_ORDER_COLS 16u
#define GS_ORDER_R ((8192u + GS_ORDER_THREADS - 1u) / GS_ORDER_THREADS)
#define GS_ORDER_E (GS_ORDER_BUCKETS * GS_ORDER_COLS / GS_ORDER_THREADS)  // scanned entries per work-item
static_assert(GS_ORDER_E * GS_ORDER_THREADS == GS_ORDER_BUCKETS * GS_ORDER_COLS, "the order scan's split");
__global__ __launch_bounds__(GS_ORDER_THREADS) void gs_tile_order_kernel(const uint32_t* __restrict__ counts,
                                                                         uint32_t* __restrict__ order, uint32_t tb,
                                                                         uint32_t te) {
  __shared__ uint32_t s_h[GS_ORDER_BUCKETS * GS_ORDER_COLS];
  __shared__ uint32_t s_part[GS_ORDER_THREADS / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, col = lane & (GS_ORDER_COLS - 1u);
  if (te - tb > GS_ORDER_R * GS_ORDER_THREADS) {
    gs_tile_order<true>(counts, order, tb, te, s_h);
    return;
  }
  uint32_t bk[GS_ORDER_R];
#pragma unroll
  for (uint32_t j = 0; j < GS_ORDER_R; ++j) {
    const uint32_t t = tb + tid + j * GS_ORDER_THREADS;
    bk[j] = t < te ? gs_order_bucket_n(counts[t]) : GS_ORDER_BUCKETS;
  }
  for (uint32_t k = tid; k < GS_ORDER_BUCKETS * GS_ORDER_COLS; k += GS_ORDER_THREADS) s_h[k] = 0;
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < GS_ORDER_R; ++j)
    if (bk[j] < GS_ORDER_BUCKETS) atomicAdd(s_h + bk[j] * GS_ORDER_COLS + col, 1u);
  __syncthreads();
  // exclusive scan of the (bucket, column) counts in bucket-major order
  uint32_t v[GS_ORDER_E], sum = 0;
#pragma unroll
  for (uint32_t e = 0; e < GS_ORDER_E; ++e) {
    v[e] = s_h[tid * GS_ORDER_E + e];
    sum += v[e];
  }
  const uint32_t incl = wave_incl_scan(sum);
  if (lane == 63u) s_part[wave] = incl;
  __syncthreads();
  uint32_t ex = incl - sum;
  for (uint32_t w = 0; w < wave; ++w) ex += s_part[w];
#pragma unroll
  for (uint32_t e = 0; e < GS_ORDER_E; ++e) {
    s_h[tid * GS_ORDER_E + e] = ex;
    ex += v[e];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < GS_ORDER_R; ++j)
    if (bk[j] < GS_ORDER_BUCKETS) order[atomicAdd(s_h + bk[j] * GS_ORDER_COLS + col, 1u)] = tb + tid + j * GS_ORDER_THREADS;
}

// Spill accounting (see gs_spill_tile), run by the first front-end launch's block (0, 0): the previous
// frame's spill demand (fz[8], the pool cursor its spilled tiles advanced; that frame's blend has
// finished: stream order) goes to the host (k_host[8], the pool's next size) and the running maximum
// (fz[11]); the cursor restarts at 0 for this frame's blend.
__device__ __forceinline__ void gs_spill_rearm(uint32_t* fz, uint32_t* k_host) {
  const uint32_t d = fz[8];
  __atomic_store_n(k_host + 8, d, __ATOMIC_RELAXED);
  if (d > fz[11]) fz[11] = d;
  fz[8] = 0;  // (k_host[8] reaches the host with the blend's system fence: no fence here)
}

// Bounding tile rect (x0, y0, x1, y1) of one front-end workgroup's clipped Gaussian rects, reduced over
// the workgroup (every work-item passes its running bounds; s_r: 4 x waves words of LDS); work-item 0
// stores it (empty: x0 > x1). A spilled tile's blend workgroup looks only at the chunks whose rect
// holds it.
template <uint32_t NT>
__device__ __forceinline__ void gs_store_chunk_rect(uint32_t bx0, uint32_t by0, uint32_t bx1, uint32_t by1,
                                                    uint32_t (*s_r)[NT / 64], ushort4* crect, uint32_t wg) {
  for (int off = 32; off > 0; off >>= 1) {
    bx0 = min(bx0, (uint32_t)__shfl_xor((int)bx0, off));
    by0 = min(by0, (uint32_t)__shfl_xor((int)by0, off));
    bx1 = max(bx1, (uint32_t)__shfl_xor((int)bx1, off));
    by1 = max(by1, (uint32_t)__shfl_xor((int)by1, off));
  }
  if ((threadIdx.x & 63u) == 0) {
    s_r[0][threadIdx.x >> 6] = bx0;
    s_r[1][threadIdx.x >> 6] = by0;
    s_r[2][threadIdx.x >> 6] = bx1;
    s_r[3][threadIdx.x >> 6] = by1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < NT / 64; ++w) {
      bx0 = min(bx0, s_r[0][w]);
      by0 = min(by0, s_r[1][w]);
      bx1 = max(bx1, s_r[2][w]);
      by1 = max(by1, s_r[3][w]);
    }
    crect[wg] = bx0 < bx1 ? make_ushort4((unsigned short)bx0, (unsigned short)by0, (unsigned short)bx1, (unsigned short)by1)
                          : make_ushort4(1, 1, 0, 0);
  }
}

// preprocess + count. Block (0, 0) also re-arms the frame's counters.
template <bool ROWCULL>
__global__ __launch_bounds__(GS_COUNT_THREADS, 4) void gs_bin_count_kernel(SplatCam cam, PreArgs A, BinGrid bg,
                                                                      uint32_t* __restrict__ hist,
                                                                      uint32_t* __restrict__ total,
                                                                      uint32_t* __restrict__ large_ctr,
                                                                      uint32_t* k_host, uint32_t* __restrict__ nzbuf,
                                                                      const uint2* __restrict__ prev_ranges,
                                                                      uint32_t* __restrict__ order, uint32_t order_tb,
                                                                      uint32_t order_te, uint32_t* __restrict__ fz,
                                                                      ushort4* __restrict__ crect) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];  // band_rows * grid_x (>= GS_ORDER_BUCKETS)
  if (order && blockIdx.y == gridDim.y - 1) {  // the extra row of blocks: the blend's tile order
    if (blockIdx.x == 0) gs_tile_order(prev_ranges, order, order_tb, order_te, s_hist);
    return;
  }
  uint32_t ty0, ty1;
  gs_band(bg, ty0, ty1);
  const uint32_t nt = (ty1 - ty0) * bg.grid_x;
  for (uint32_t k = threadIdx.x; k < nt; k += GS_COUNT_THREADS) s_hist[k] = 0;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    total[1] = 0;  // largest tile (colscan's atomicMax; the scatter hands it to the host)
    large_ctr[0] = 0;  // large-tile list length (colscan)
    gs_spill_rearm(fz, k_host);
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t b0 = blockIdx.y * bg.chunk, b1 = min(A.n, b0 + bg.chunk);
  uint32_t bx0 = 0xFFFFu, by0 = 0xFFFFu, bx1 = 0u, by1 = 0u;  // the chunk's rect in the band (gs_spill_tile)
  for (uint32_t base = b0 + wave * 64u; base < b1; base += GS_COUNT_THREADS) {
    const uint32_t i = base + lane;
    ushort4 rc = make_ushort4(0, 0, 0, 0);
    // (tile-row shard with chunk bounds: a 256-Gaussian chunk whose bound misses the rows is skipped
    // before its Gaussians are loaded; a wave's 64 lie in at most two chunks)
    const bool skip = cam.cull && i < b1 && A.cskip[i >> 8];
    if (i < b1 && !skip)
      rc = blockIdx.x == 0 ? gs_preprocess_one<true, ROWCULL>(cam, A, i) : gs_preprocess_one<false, ROWCULL>(cam, A, i);
    else if (i < b1 && blockIdx.x == 0) gs_store_skipped(A, i);
    uint32_t xw, yh;
    gs_clip(rc, ty0, ty1, xw, yh);
    if (yh) {
      bx0 = min(bx0, xw & 0xFFFFu);
      bx1 = max(bx1, (xw & 0xFFFFu) + (xw >> 16));
      by0 = min(by0, yh & 0xFFFFu);
      by1 = max(by1, (yh & 0xFFFFu) + (yh >> 16));
    }
    if (__ballot(yh != 0u))
      gs_expand<false>(lane, i, xw, yh, 0.0f, [&](uint32_t, uint32_t x, uint32_t y, float) {
        atomicAdd(s_hist + (y - ty0) * bg.grid_x + x, 1u);
      });
  }
  __syncthreads();
  uint32_t* row = hist + (size_t)blockIdx.y * bg.tiles + ty0 * bg.grid_x;
  uint32_t nz = 0;
  for (uint32_t k = threadIdx.x; k < nt; k += GS_COUNT_THREADS) {
    const uint32_t c = s_hist[k];
    row[k] = c;
    nz += c != 0u;
  }
  // touched (chunk, tile) entries, the front-end policy's measure of spatial coherence (the fused
  // path would reserve each with an atomic), per workgroup; the scatter's block (0, 0) sums them for
  // the host (k_host[4])
  for (int off = 32; off > 0; off >>= 1) nz += (uint32_t)__shfl_xor((int)nz, off);
  __shared__ uint32_t s_nz[GS_COUNT_THREADS / 64];
  if ((threadIdx.x & 63u) == 0) s_nz[threadIdx.x >> 6] = nz;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < GS_COUNT_THREADS / 64; ++w) t += s_nz[w];
    nzbuf[blockIdx.y * gridDim.x + blockIdx.x] = t;  // (summed by the scatter's block (0, 0): no fan-in atomics)
  }
  __shared__ uint32_t s_rr[4][GS_COUNT_THREADS / 64];
  gs_store_chunk_rect<GS_COUNT_THREADS>(bx0, by0, bx1, by1, s_rr, crect, blockIdx.y * gridDim.x + blockIdx.x);
}

// One 256-work-item block per 64-tile group g: wave w sums chunks [w*cpw, (w+1)*cpw) of the group's
// 64 tiles (lane = tile: coalesced rows), then rewrites hist[c][t] as the exclusive prefix over c.
// Outputs per tile (offset inside the group, total), per group its total, atomicMax of the largest
// tile into total[1], and the tiles of more than `thr` pairs appended to the large-tile list.
#ifndef GS_COLSCAN_WAVES
#define GS_COLSCAN_WAVES 16
#endif
#define GS_COLSCAN_THREADS (64 * GS_COLSCAN_WAVES)
#define GS_CS_REG 16u  // chunk rows per colscan wave kept in registers
static_assert(GS_MAX_CHUNKS <= GS_COLSCAN_WAVES * 64, "colscan: at most 64 chunk rows per wave");
__global__ __launch_bounds__(GS_COLSCAN_THREADS) void gs_bin_colscan_kernel(BinGrid bg, uint32_t* __restrict__ hist,
                                                             uint2* __restrict__ tile_info,
                                                             uint32_t* __restrict__ group_total,
                                                             uint32_t* __restrict__ total, uint32_t thr,
                                                             uint32_t* __restrict__ large,
                                                             uint32_t* __restrict__ large_ctr) {
  __shared__ uint32_t s_ws[GS_COLSCAN_WAVES][64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t t = bg.row0 * bg.grid_x + blockIdx.x * 64u + lane;
  const bool ok = t < bg.row1 * bg.grid_x;
  const uint32_t cpw = (bg.chunks + GS_COLSCAN_WAVES - 1u) / GS_COLSCAN_WAVES, c0 = wave * cpw,
                 c1 = min(bg.chunks, c0 + cpw);
  // the wave's first GS_CS_REG rows in flight at once and kept in registers (fully unrolled: every
  // frame of up to 256 chunks); rows beyond them (more chunks: 10M Gaussians at 4K, single-band tile-row
  // shards of large sets) in batches of GS_CS_REG, read again for the rewrite
  uint32_t h[GS_CS_REG];
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < GS_CS_REG; ++k) {
    h[k] = (ok && c0 + k < c1) ? hist[(size_t)(c0 + k) * bg.tiles + t] : 0u;
    sum += h[k];
  }
  for (uint32_t k0 = GS_CS_REG; k0 < cpw; k0 += GS_CS_REG) {
    uint32_t x[GS_CS_REG];
#pragma unroll
    for (uint32_t k = 0; k < GS_CS_REG; ++k) x[k] = (ok && c0 + k0 + k < c1) ? hist[(size_t)(c0 + k0 + k) * bg.tiles + t] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < GS_CS_REG; ++k) sum += x[k];
  }
  s_ws[wave][lane] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t w = 0; w < wave; ++w) run += s_ws[w][lane];
#pragma unroll
  for (uint32_t k = 0; k < GS_CS_REG; ++k)
    if (ok && c0 + k < c1) {
      hist[(size_t)(c0 + k) * bg.tiles + t] = run;
      run += h[k];
    }
  for (uint32_t k0 = GS_CS_REG; k0 < cpw; k0 += GS_CS_REG) {
    uint32_t x[GS_CS_REG];
#pragma unroll
    for (uint32_t k = 0; k < GS_CS_REG; ++k) x[k] = (ok && c0 + k0 + k < c1) ? hist[(size_t)(c0 + k0 + k) * bg.tiles + t] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < GS_CS_REG; ++k)
      if (ok && c0 + k0 + k < c1) {
        hist[(size_t)(c0 + k0 + k) * bg.tiles + t] = run;
        run += x[k];
      }
  }
  if (wave != 0) return;
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < GS_COLSCAN_WAVES; ++w) tot += s_ws[w][lane];
  const uint32_t incl = wave_incl_scan(tot);
  if (ok) tile_info[t] = make_uint2(incl - tot, tot);  // (offset inside the group, tile total)
  const bool big = ok && tot > thr;
  const unsigned long long bal = __ballot(big);
  if (bal) {
    uint32_t at = 0;
    if (lane == 0) at = atomicAdd(large_ctr, (uint32_t)__popcll(bal));
    at = (uint32_t)__shfl((int)at, 0);
    if (big) large[at + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = t;
  }
  uint32_t mx = tot;
  for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
  const uint32_t gsum = __shfl(incl, 63);
  if (lane == 0) {
    group_total[blockIdx.x] = gsum;
    if (mx) atomicMax(total + 1, mx);
  }
}

// K = the sum of the group totals (every block scans them all); block (0, 0) publishes it to total[0]
// (the blend's check) and, with the largest tile and the large-tile count, to pinned host memory. Pairs are written only when K fits the pair buffer
// (the host sizes it from the previous K and re-runs scatter + blend after growing it when it did
// not: see splat_gaussians).
__global__ __launch_bounds__(GS_BIN_THREADS) void gs_bin_scatter_kernel(
    BinGrid bg, const ushort4* __restrict__ rects, const float* __restrict__ depths, const uint32_t* __restrict__ ids,
    uint32_t n,
    const uint32_t* __restrict__ hist, const uint2* __restrict__ tile_info, const uint32_t* __restrict__ group_total,
    uint32_t* __restrict__ total, const uint32_t* __restrict__ large_ctr, uint32_t* k_host,
    const uint32_t* __restrict__ nzbuf, uint32_t nzn, uint32_t cap,
    uint2* __restrict__ ranges,
    unsigned long long* __restrict__ pairs, unsigned long long* __restrict__ tile_slots) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_cur[];  // 2 * band_rows * grid_x + groups
  __shared__ uint4 s_q[GS_BIN_THREADS / 64 * GS_WQ];
  __shared__ uint32_t s_part[GS_BIN_THREADS / 64];
  uint32_t ty0, ty1;
  gs_band(bg, ty0, ty1);
  const uint32_t nt = (ty1 - ty0) * bg.grid_x, t0 = ty0 * bg.grid_x;
  uint32_t* s_tot = s_cur + bg.band_rows * bg.grid_x;
  uint32_t* s_gpre = s_tot + bg.band_rows * bg.grid_x;
  const uint32_t c = blockIdx.y, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  // exclusive scan of the group totals
  const uint32_t gend = bg.groups;
  uint32_t carry = 0;
  for (uint32_t g0 = 0; g0 < gend; g0 += GS_BIN_THREADS) {
    const uint32_t g = g0 + tid;
    const uint32_t v = g < gend ? group_total[g] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) s_part[wv] = incl;
    __syncthreads();
    uint32_t woff = carry, all = carry;
    for (uint32_t w = 0; w < GS_BIN_THREADS / 64; ++w) {
      woff += w < wv ? s_part[w] : 0u;
      all += s_part[w];
    }
    if (g < gend) s_gpre[g] = woff + incl - v;
    carry = all;
    __syncthreads();
  }
  uint32_t nzsum = 0;
  if (blockIdx.x == 0 && blockIdx.y == 0) {  // the count's touched entries (per workgroup)
    for (uint32_t k = tid; k < nzn; k += GS_BIN_THREADS) nzsum += nzbuf[k];
    for (int off = 32; off > 0; off >>= 1) nzsum += (uint32_t)__shfl_xor((int)nzsum, off);
    if (lane == 0) s_part[wv] = nzsum;
    __syncthreads();
    nzsum = 0;
    for (uint32_t w = 0; w < GS_BIN_THREADS / 64; ++w) nzsum += s_part[w];
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
    total[0] = carry;
    __atomic_store_n(k_host + 1, total[1], __ATOMIC_RELAXED);      // largest tile (the next sort's LDS size)
    __atomic_store_n(k_host + 2, large_ctr[0], __ATOMIC_RELAXED);  // large tiles (the next sort grid)
    __atomic_store_n(k_host + 4, nzsum, __ATOMIC_RELAXED);         // touched (chunk, tile) entries
    __atomic_store_n(k_host + 5, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(k_host + 6, 2u, __ATOMIC_RELAXED);  // published by: three launches
    __atomic_store_n(k_host, carry, __ATOMIC_RELAXED);  // pinned host word: the host's K read-back
    if (carry > total[2]) total[2] = carry;  // the workspace's largest K (three launches; fused: fz[13])
    __atomic_store_n(k_host + 13, total[2], __ATOMIC_RELAXED);
    __threadfence_system();  // visible to the host before the kernel ends (the K event has no system fence)
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && (bg.row0 > 0 || bg.row1 < bg.grid_y)) {
    // a tile-row frame's bands cover its rows only: the other tiles' ranges are empty (as the oracle's)
    const uint32_t tb = bg.row0 * bg.grid_x, te = bg.row1 * bg.grid_x;
    for (uint32_t t = tid; t < bg.tiles; t += GS_BIN_THREADS)
      if (t < tb || t >= te) ranges[t] = make_uint2(0u, 0u);
  }
  // (K above the pair buffer: the tiles whose segment ends beyond it keep none of their pairs here and
  // are rendered by the blend through gs_spill_tile; the fixed rows of small tiles always fit)
  for (uint32_t k = tid; k < nt; k += GS_BIN_THREADS) {
    const uint32_t t = t0 + k;
    const uint2 ti = tile_info[t];
    const uint32_t start = s_gpre[(t - bg.row0 * bg.grid_x) >> 6] + ti.x;
    s_cur[k] = hist[(size_t)c * bg.tiles + t];
    // where the tile's pairs go: its fixed GS_TILE_SLOTS-slot row when they fit (the blend then
    // loads keys without waiting for the range), else its segment of the pair buffer (flag bit 31)
    s_tot[k] = ti.y <= GS_TILE_SLOTS ? t * GS_TILE_SLOTS : (start | 0x80000000u);
    if (c == 0) ranges[t] = ti.y ? make_uint2(start, start + ti.y) : make_uint2(0u, 0u);
  }
  __syncthreads();
  auto put = [&](uint32_t i, uint32_t x, uint32_t y, float d) {
    const unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | i;
    const uint32_t k = (y - ty0) * bg.grid_x + x;
    const uint32_t rel = atomicAdd(s_cur + k, 1u), dst = s_tot[k];
    if (dst & 0x80000000u) {
      const uint32_t at = (dst & 0x7FFFFFFFu) + rel;
      if (at < cap) pairs[at] = key;
    } else {
      tile_slots[dst + rel] = key;
    }
  };
  if (bg.bands == 1) {  // one band: every rect meets it, so no filtering ring (one Gaussian per lane, as the count;
                        // -0.4 us at C2, kernel trace)
    const uint32_t b0 = c * bg.chunk, b1 = min(n, b0 + bg.chunk);
    for (uint32_t base = b0 + wv * 64u; base < b1; base += GS_BIN_THREADS) {
      const uint32_t i = base + lane;
      ushort4 rc = make_ushort4(0, 0, 0, 0);
      float d = 0.0f;
      if (i < b1) {
        rc = rects[i];
        d = depths[i];
      }
      uint32_t xw, yh;
      gs_clip(rc, ty0, ty1, xw, yh);
      if (__ballot(yh != 0u)) gs_expand<true>(lane, ids && i < b1 ? ids[i] : i, xw, yh, d, put);
    }
    return;
  }
  gs_walk_chunk(bg, rects, depths, ids, n, ty0, ty1, s_q, put);
}

// ---- fused front end ------------------------------------------------------------------------------
// One launch instead of count + colscan + scatter: per-tile slot rows of a fixed capacity `scap`
// (a power of two >= the largest tile of recent frames) replace the exact tile segments, so a tile's
// pairs need no global prefix: block (band, c) preprocesses chunk c (one Gaussian per work-item,
// kept in registers), counts its pairs per tile in LDS, reserves each touched tile's run with one
// returning atomicAdd on the tile's cursor, then walks its pairs again and writes each key to
// tile_slots[t * scap + base + LDS rank]. The order inside a row depends on the atomics' order and is
// fixed by the per-tile sort (keys are unique), so keys / values / image equal the three-launch path.
// The blend reads the tile's count from its cursor and zeroes it (cursors are zero between frames).
// A tile whose count exceeds scap keeps its first scap keys only: the blend renders it through
// gs_spill_tile (its pairs gathered again from the per-Gaussian rects / depths band 0 stores here and
// the per-workgroup chunk rects), so the frame is complete; the next frame sizes its rows from it.
// fz: [1] largest tile above 256, [4] tiles above GS_MID pairs, [5] tiles above scap; per workgroup
// fzp: (pairs, reservations); published to the host by the blend's block (0, 0).
#ifndef GS_FUSED_OWN_CULL
// a tile-row frame of at most this many chunks: the fused workgroups test their own chunk's bound (no
// cull launch: C2 bands 1-2 us faster); above it the flags of a cull launch (each workgroup's bound
// test adds its latency to every round of workgroups: 10M at 4K, band 0 2.26 vs 2.09 ms)
#define GS_FUSED_OWN_CULL 1024u
#endif
#ifndef GS_FUSED_THREADS
#define GS_FUSED_THREADS 256  // Gaussians per fused workgroup (512 / 1 024 work-items: 1.5 us slower at C2)
#endif
struct GsFused {  // the sort's and the blend's view of a fused-front-end frame (scap == 0: three-launch path)
  uint32_t scap;
  uint32_t* cursor;   // per-tile pair counts (zeroed again by the blend)
  uint32_t* fz;       // counters (see above)
  uint32_t* k_host;   // pinned host words (published by blend block (0, 0))
  uint2* ranges;      // the tile ranges the blend writes (t * scap, t * scap + n)
  uint32_t* fzp;      // per front-end workgroup: (pairs, reservations)
  uint32_t nwg;
  const uint32_t* order;  // blend workgroup -> tile (heavy tiles first; null: row-major)
  uint2* fsq;             // the front end's slice queue (re-armed by block (0, 0): entries and fz[12..14])
  uint32_t fsq_cap;
  unsigned long long* seq_flag;  // frames in flight: the blend's first workgroup stores `seq` here (SplatSeq)
  unsigned long long seq;
};
// Work-items per fused workgroup (GS_FUSED_THREADS Gaussians; all walk the pairs): 512 for a frame on the
// caller's stream; 256 for an overlapped frame (SplatOverlap), whose front end runs beside the previous
// frame's blend: a 256-work-item workgroup of at most 64 VGPRs and ~14 KB of LDS takes the slot of one
// retiring blend workgroup (256 work-items, 64 VGPRs, 17 KB), where a 512-work-item one waited for the
// blend's tail (measured: the whole front end ran after the blend; C2 frames 63 vs 56 us serial).
#define GS_FUSED_WG 512
#ifndef GS_FUSED_WG_OV
#define GS_FUSED_WG_OV 256
#endif
template <uint32_t WG> struct GsFusedShape;
template <> struct GsFusedShape<512> {
  static constexpr uint32_t slice = 4096u;  // pairs per slice (C2's chunks hold 1.6k on average, 3.3k at most: one slice)
  static constexpr uint32_t lds_cap = 0u;   // histogram window in tiles (0: the band's)
};
template <> struct GsFusedShape<256> {
  static constexpr uint32_t slice = 2048u;
  static constexpr uint32_t lds_cap = 2048u;  // 8 KB (+ 5.6 KB static): within one blend workgroup's LDS
};

// The count walk of one slice [p0, p1) of a chunk's pairs (at most GS_FUSED_QREG per work-item): the
// chunk's rects (s_e: x0 | w << 16, y0 | h << 16, key index, depth bits) and the inclusive scan of
// their areas (s_incl) are in LDS; work-item t takes the contiguous pairs [p0 + t q, p0 + t q + q)
// (q = ceil((p1 - p0) / WG)): one binary search for its first pair, then it steps through the
// rects (a heavy Gaussian's pairs are spread over the whole workgroup instead of one wave). Returning
// LDS atomics give each pair its rank among the slice's pairs of its tile, kept in registers with the
// pair, packed as k | rank << 13 | j << 21 (k: tile in the chunk's rect, < 8192 = GS_BAND_TILES; rank
// < 256: one pair per Gaussian and tile; j: Gaussian in the chunk, < 256). The scatter then writes each
// kept pair at its run's base + rank without walking the rects again or touching an LDS atomic.
// Returns the work-item's pair count.
#ifndef GS_FUSED_QREG
#define GS_FUSED_QREG 8  // pairs per work-item of a slice (GsFusedShape<WG>::slice / WG; C2 needs <= 7)
#endif
#define GS_KEEP_RB (GS_FUSED_THREADS <= 256 ? 8u : 9u)  // bits of rank and of j (< GS_FUSED_THREADS)
static_assert(GS_FUSED_THREADS <= 512 && GS_BAND_TILES <= 8192, "gs_wg_count_keep's packing");
#define GS_PK_NONE 0xFFFFFFFFu  // a walked pair outside the histogram window (kept by another window's walk)
template <uint32_t WG>
__device__ __forceinline__ uint32_t gs_wg_count_keep(const uint32_t* s_incl, const uint4* s_e, uint32_t ng, uint32_t p0,
                                                     uint32_t p1, uint32_t* s_hist, uint32_t bx0, uint32_t by0,
                                                     uint32_t rw, uint32_t kw, uint32_t kcap,
                                                     uint32_t (&pk)[GS_FUSED_QREG]) {
  const uint32_t q = (p1 - p0 + WG - 1) / WG;
  uint32_t p = p0 + threadIdx.x * q;
  const uint32_t pe = min(p1, p + q);
  if (p >= pe) return 0;
  const uint32_t cnt = pe - p;
  uint32_t lo = 0, hi = ng - 1;  // first j with incl[j] > p
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s_incl[mid] > p) hi = mid;
    else lo = mid + 1;
  }
  uint32_t j = lo;
  uint4 e = s_e[j];
  uint32_t w = e.x >> 16, r = p - (s_incl[j] - w * (e.y >> 16));
  uint32_t ry = r / w, rx = r - ry * w;
#pragma unroll
  for (uint32_t c = 0; c < GS_FUSED_QREG; ++c) {
    if (c < cnt) {
      // (the tile's index in the rect, relative to the histogram window [kw, kw + kcap))
      const uint32_t k = ((e.y & 0xFFFFu) + ry - by0) * rw + ((e.x & 0xFFFFu) + rx - bx0) - kw;
      if (k < kcap) {
        const uint32_t rank = atomicAdd(s_hist + k, 1u);
        pk[c] = k | (rank << 13) | (j << (13u + GS_KEEP_RB));
      } else {
        pk[c] = GS_PK_NONE;
      }
      if (c + 1 < cnt && ++rx == w) {
        rx = 0;
        if (++ry == (e.y >> 16)) {  // next rect with pairs
          do {
            e = s_e[++j];
          } while ((e.y >> 16) == 0u || (e.x >> 16) == 0u);
          w = e.x >> 16;
          ry = 0;
        }
      }
    }
  }
  return cnt;
}

// Load balance. A chunk's pairs are walked in slices of at most GsFusedShape<WG>::slice pairs. The owner (the
// chunk's workgroup) walks slice 0 and publishes the others to a queue (fsq, entries (owner + 1, j));
// helper workgroups (the rows after the owners) claim queued slices, rebuild the chunk's rects (the
// same preprocess, no stores) and walk them: every (slice, tile) run reserves its own range, so a
// chunk that holds many times the mean pairs (Gaussians close to a moving camera) no longer sets the
// kernel's length alone. After its slice 0 an owner claims its own still-queued slices (it never
// waits), so no slice depends on a helper: a helper waits only for owners that have not published yet
// (owners precede helpers in dispatch order), and gives up after ~100 us (a slice it would have taken
// is then its owner's). Queue words: fz[GS_FSQ_W] claims (helpers), fz[GS_FSQ_W + 1] entries,
// fz[GS_FSQ_W + 2] owners done;
// entries are 0 (not written), owner + 1 (open), GS_FSQ_TAKEN; the blend's block (0, 0) re-arms them.
#ifndef GS_FUSED_HELPERS
#define GS_FUSED_HELPERS 128u  // helper workgroups per band (one queued slice each)
#endif
#define GS_FSQ_TAKEN 0xFFFFFFFFu
#define GS_FSQ_W 32  // the queue words' offset in fz: a cache line of their own (helpers poll them)
// waves per SIMD: 512 work-items 6 (3 workgroups per CU; 8 forced SGPR spills), 256 work-items 8 (64 VGPRs)
#define GS_FUSED_WAVES(WG) ((WG) == 512 ? 6 : 8)
static_assert(GsFusedShape<512>::slice <= 512u * GS_FUSED_QREG && GsFusedShape<256>::slice <= 256u * GS_FUSED_QREG,
              "a slice's pairs are kept in registers");
// chunk skip flags (cskip) and chunk bounds are per 256 Gaussians (ptgs_gaussians_chunk_bounds): the fused
// workgroups index them by their own chunk, so a fused chunk must be exactly that
static_assert(GS_FUSED_THREADS == 256, "the fused chunk is the chunk-bounds granule (256 Gaussians)");


template <bool ROWCULL, uint32_t WG>
__global__ __launch_bounds__(WG, GS_FUSED_WAVES(WG)) void gs_bin_fused_kernel(SplatCam cam, PreArgs A, BinGrid bg,
                                                                         uint32_t scap,
                                                                         uint32_t* __restrict__ cursor,
                                                                         uint32_t* __restrict__ fz,
                                                                         uint32_t* __restrict__ fzp,
                                                                         unsigned long long* __restrict__ tile_slots,
                                                                         const uint2* __restrict__ prev_ranges,
                                                                         uint32_t* __restrict__ order,
                                                                         uint32_t order_tb, uint32_t order_te,
                                                                         ushort4* __restrict__ crect,
                                                                         ushort4* __restrict__ rects_out,
                                                                         float* __restrict__ depths_out,
                                                                         uint32_t* k_host, uint2* __restrict__ fsq,
                                                                         uint32_t fsq_cap, uint32_t kcap) {
  // the histogram window: kcap entries (<= band_rows * grid_x); a chunk whose bounding tile rect holds
  // more tiles walks its slice once per window of kcap tiles (each walk counts, reserves and scatters
  // only its window's pairs), so the dynamic LDS need not cover a whole band
  extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
  __shared__ uint32_t s_red[4][WG / 64];
  __shared__ uint32_t s_tot[WG / 64];
  __shared__ uint32_t s_incl[GS_FUSED_THREADS];
  __shared__ uint4 s_e[GS_FUSED_THREADS];
  __shared__ uint32_t s_job[4];  // helpers: (owner, slice) claimed; owners: queue base of their slices
  static_assert(GS_FUSED_THREADS >= GS_ORDER_BUCKETS, "gs_tile_order's buckets live in s_incl");
  if (order && blockIdx.y == gridDim.y - 1) {  // the extra row of blocks: the blend's tile order
    if (blockIdx.x == 0) {
      STAMP(0, 0);
      gs_tile_order(prev_ranges, order, order_tb, order_te, s_incl);
      STAMP_SYNC();
      STAMP(0, 5);
    }
    return;
  }
  STAMP(0, 0);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nown = bg.chunks * gridDim.x;  // owner workgroups
  const bool owner = blockIdx.y < bg.chunks;
  if (owner && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) gs_spill_rearm(fz, k_host);
  uint32_t acc_pairs = 0, acc_res = 0;  // this workgroup's reservations over all its slices (per work-item)
  uint32_t wg = blockIdx.y * gridDim.x + blockIdx.x;  // the owner whose chunk is processed
  uint32_t slice = 0;
  {  // helpers claim one queued slice (one per helper: no loop keeps the camera's registers live)
    if (!owner) {
      if (threadIdx.x == 0) {
        // (owner, slice) in two words: an owner index is bands x chunks, beyond any packing's bits at 8K
        // with tens of millions of Gaussians
        uint32_t job = 0xFFFFFFFFu, jslice = 0, hidx = 0, spins = 0;
        for (;;) {
          if (!hidx) hidx = atomicAdd(fz + GS_FSQ_W, 1u) + 1u;  // (1-based: 0 = none claimed)
          const uint32_t idx = hidx - 1u;
          if (idx >= fsq_cap) break;
          // (the entry as one 64-bit word: owner + 1 and slice arrive together, no fence needed)
          const unsigned long long ev = __hip_atomic_load(reinterpret_cast<unsigned long long*>(fsq + idx),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t v = (uint32_t)ev;
          if (v == 0u) {  // not written yet: done when every owner has published and this index is past the end
            const uint32_t done = __hip_atomic_load(fz + GS_FSQ_W + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t tail = __hip_atomic_load(fz + GS_FSQ_W + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((done >= nown && idx >= tail) || ++spins > 200u) break;
            // (a few hundred helpers polling: every ~3 us, or their loads crowd out the owners' memory
            // traffic; measured 3x slower owner phases at ~0.05 us per poll)
            __builtin_amdgcn_s_sleep(127);
            continue;
          }
          hidx = 0;  // this index is settled: the next iteration claims another
          if (v != GS_FSQ_TAKEN && atomicCAS(&fsq[idx].x, v, GS_FSQ_TAKEN) == v) {
            job = v - 1u;
            jslice = (uint32_t)(ev >> 32);
            break;
          }
        }
        s_job[0] = job;
        s_job[3] = jslice;
      }
      __syncthreads();
      const uint32_t job = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_job[0]);
      if (job == 0xFFFFFFFFu) {
        if (threadIdx.x == 0) {
          const uint32_t fw = blockIdx.y * gridDim.x + blockIdx.x;
          fzp[2 * fw] = 0;
          fzp[2 * fw + 1] = 0;
        }
        return;
      }
      wg = job;
      slice = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_job[3]);
    }
    const uint32_t band = wg % gridDim.x, chunk = wg / gridDim.x;
    const uint32_t ty0 = bg.row0 + band * bg.band_rows, ty1 = min(bg.row1, ty0 + bg.band_rows);
    const uint32_t i = chunk * bg.chunk + threadIdx.x;  // chunk <= GS_FUSED_THREADS (host)
    const bool own = threadIdx.x < bg.chunk && i < A.n;
    const bool store = owner && band == 0;
    ushort4 rc = make_ushort4(0, 0, 0, 0);
    const uint32_t o = own && A.ids ? A.ids[i] : i;  // the key's index (the caller's)
    float d = 0.0f;  // view depth (every band's blocks need it for the keys; only band 0 stores it)
    // (tile-row shard with chunk bounds: a chunk whose bound misses the rows is skipped before its
    // Gaussians are loaded; it goes through the rest with no pairs)
    const bool skip = cam.cull && (A.cbounds ? gs_chunk_misses(cam, A.cbounds[2 * chunk], A.cbounds[2 * chunk + 1])
                                             : A.cskip[chunk] != 0);
    if (owner && skip) {
      // a culled chunk leaves at once (a tile-row shard of a large set culls most of its ~N / 256
      // workgroups): what it owes is the empty chunk rect (gs_spill_tile then never reads its Gaussians),
      // its published zeros, its arrival at the slice queue's owner count and zero partials
      if (own && store) gs_store_skipped(A, i);
      if (threadIdx.x == 0) {
        crect[wg] = make_ushort4(1, 1, 0, 0);
        atomicAdd(fz + GS_FSQ_W + 2, 1u);
        fzp[2 * wg] = 0;
        fzp[2 * wg + 1] = 0;
      }
      return;
    }
    if (own && !skip)
      rc = store ? gs_preprocess_one<true, ROWCULL>(cam, A, i, &d) : gs_preprocess_one<false, ROWCULL>(cam, A, i, &d);
    else if (own && store) gs_store_skipped(A, i);
    if (own && store) {  // for gs_spill_tile: the rect (empty: culled) and depth in walk order
      rects_out[i] = rc;
      depths_out[i] = d;
    }
    STAMP_WAITED(0, 6);  // (wave 0's preprocess, loads included)
    uint32_t xw, yh;
    gs_clip(rc, ty0, ty1, xw, yh);
    // the chunk's bounding tile rect (within the band): the LDS histogram covers only it, so zeroing
    // and the reservation scan touch ~100 entries for a spatially coherent chunk instead of the band's
    uint32_t bx0 = 0xFFFFu, by0 = 0xFFFFu, bx1 = 0u, by1 = 0u;
    if (yh) {
      bx0 = xw & 0xFFFFu;
      bx1 = bx0 + (xw >> 16);
      by0 = yh & 0xFFFFu;
      by1 = by0 + (yh >> 16);
    }
    bx0 = wave_reduce<0>(bx0);
    by0 = wave_reduce<0>(by0);
    bx1 = wave_reduce<1>(bx1);
    by1 = wave_reduce<1>(by1);
    // the rects and the inclusive scan of their areas for the workgroup walk: the per-wave partials of
    // both (rect bounds, area totals) meet behind one barrier
    const uint32_t area = yh ? (xw >> 16) * (yh >> 16) : 0u;
    const uint32_t incl = wave_incl_scan(area);
    if (lane == 0) {
      s_red[0][wave] = bx0;
      s_red[1][wave] = by0;
      s_red[2][wave] = bx1;
      s_red[3][wave] = by1;
    }
    if (lane == 63) s_tot[wave] = incl;
    if (threadIdx.x < GS_FUSED_THREADS) s_e[threadIdx.x] = make_uint4(xw, yh, o, __float_as_uint(d));
    __syncthreads();
    STAMP(0, 7);
    uint32_t run = incl, P = 0;
#pragma unroll
    for (uint32_t w = 0; w < WG / 64; ++w) {
      bx0 = min(bx0, s_red[0][w]);
      by0 = min(by0, s_red[1][w]);
      bx1 = max(bx1, s_red[2][w]);
      by1 = max(by1, s_red[3][w]);
      const uint32_t tw = s_tot[w];
      run += w < wave ? tw : 0u;
      P += tw;
    }
    if (threadIdx.x < GS_FUSED_THREADS) s_incl[threadIdx.x] = run;
    // (uniform: in SGPRs, the registers the slice loop keeps)
    bx0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bx0);
    by0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)by0);
    bx1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bx1);
    by1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)by1);
    P = (uint32_t)__builtin_amdgcn_readfirstlane((int)P);
    const uint32_t rw = bx1 > bx0 ? bx1 - bx0 : 0u, rh = by1 > by0 ? by1 - by0 : 0u, nt = rw * rh;
    const uint32_t nsl = (P + GsFusedShape<WG>::slice - 1u) / GsFusedShape<WG>::slice;  // slices of this chunk (uniform)
    if (owner) {
      if (threadIdx.x == 0) {  // the workgroup's bounding rect (gs_spill_tile; empty: x0 > x1)
        crect[wg] = nt ? make_ushort4((unsigned short)bx0, (unsigned short)by0, (unsigned short)bx1, (unsigned short)by1)
                       : make_ushort4(1, 1, 0, 0);
        // slices 1.. go to the queue (none fit: the owner walks them all itself)
        uint32_t qb = 0xFFFFFFFFu;
        if (nsl > 1u) {
          qb = atomicAdd(fz + GS_FSQ_W + 1, nsl - 1u);
          if (qb + (nsl - 1u) > fsq_cap) {  // (the part inside the queue is marked taken: helpers skip it)
            for (uint32_t k = qb; k < fsq_cap && k < qb + (nsl - 1u); ++k)
              __hip_atomic_store(reinterpret_cast<unsigned long long*>(fsq + k), (unsigned long long)GS_FSQ_TAKEN,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            qb = 0xFFFFFFFFu;
          } else {
            for (uint32_t j = 1; j < nsl; ++j)
              __hip_atomic_store(reinterpret_cast<unsigned long long*>(fsq + qb + j - 1u),
                                 ((unsigned long long)j << 32) | (wg + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        // published (helpers stop waiting once every owner has; no release fence: an agent-scope one
        // writes back the XCD's L2. A helper that sees every owner done before it sees its entry keeps
        // waiting while its index is below the tail; one that leaves early leaves the slice to its owner)
        atomicAdd(fz + GS_FSQ_W + 2, 1u);
        s_job[1] = qb;
      }
    }
    // the slices this pass walks: helpers one; owners slice 0, then each queued slice it can still
    // claim (or every slice when the queue was full)
    for (;;) {
      const uint32_t p0 = slice * GsFusedShape<WG>::slice, p1 = min(P, p0 + GsFusedShape<WG>::slice);
     for (uint32_t kw = 0; kw < nt; kw += kcap) {  // histogram windows of the rect (one for most chunks)
      const uint32_t nw = min(kcap, nt - kw);
      if (kw) __syncthreads();  // (the previous window's scatter has read s_hist)
      for (uint32_t k = threadIdx.x; k < nw; k += WG) s_hist[k] = 0;
      __syncthreads();  // (the scan and the zeroed histogram)
      STAMP(0, 1);
      STAMP_SYNC();
      STAMP(0, 2);
      uint32_t pk[GS_FUSED_QREG];
      const uint32_t kept =
          p1 > p0 ? gs_wg_count_keep<WG>(s_incl, s_e, GS_FUSED_THREADS, p0, p1, s_hist, bx0, by0, rw, kw, kcap, pk) : 0u;
      __syncthreads();
      STAMP(0, 3);
      // reserve: one returning atomic per touched tile (all of a work-item's issued before any is
      // used); the LDS entry becomes the run's base
      const float rcp_rw = 1.0f / (float)max(rw, 1u);
      for (uint32_t k0 = threadIdx.x; k0 < nw; k0 += 4 * WG) {
        uint32_t c[4], t[4], base[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t kl = k0 + j * WG, k = kw + kl;
          c[j] = kl < nw ? s_hist[kl] : 0u;
          uint32_t ry = (uint32_t)((float)k * rcp_rw);  // k < 2^13 * 2^13: exact after the fix-ups
          ry = ry * rw > k ? ry - 1 : ry;
          ry = (ry + 1) * rw <= k ? ry + 1 : ry;
          t[j] = (by0 + ry) * bg.grid_x + bx0 + (k - ry * rw);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) base[j] = c[j] ? atomicAdd(cursor + t[j], c[j]) : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!c[j]) continue;
          s_hist[k0 + j * WG] = base[j];
          acc_pairs += c[j];
          ++acc_res;
          if (base[j] <= scap && base[j] + c[j] > scap) atomicAdd(fz + 5, 1u);  // (one crossing per spilled tile)
          if (base[j] + c[j] > 256u) {
            atomicMax(fz + 1, base[j] + c[j]);
            if (base[j] <= GS_MID && base[j] + c[j] > GS_MID) atomicAdd(fz + 4, 1u);  // (one crossing per tile)
          }
        }
      }
      __syncthreads();  // every run's base is in s_hist
      STAMP(0, 4);
#pragma unroll
      for (uint32_t c = 0; c < GS_FUSED_QREG; ++c) {
        if (c < kept && pk[c] != GS_PK_NONE) {
          const uint32_t kl = pk[c] & 0x1FFFu, k = kw + kl;
          const uint32_t rel = s_hist[kl] + ((pk[c] >> 13) & ((1u << GS_KEEP_RB) - 1u));
          const uint4 e = s_e[pk[c] >> (13u + GS_KEEP_RB)];
          uint32_t ry = (uint32_t)((float)k * rcp_rw);  // k < 2^13: exact after the fix-ups
          ry = ry * rw > k ? ry - 1 : ry;
          ry = (ry + 1) * rw <= k ? ry + 1 : ry;
          const uint32_t t = (by0 + ry) * bg.grid_x + bx0 + (k - ry * rw);
          if (rel < scap) {
            const unsigned long long key = ((unsigned long long)e.w << 32) | e.z;
            tile_slots[(size_t)t * scap + rel] = key;
          }
        }
      }
     }  // (windows)
      if (!owner) break;
      // owner: the next of its slices that no helper has taken (uniform through LDS)
      __syncthreads();  // (every read of s_hist / s_job before they change)
      if (threadIdx.x == 0) {
        const uint32_t qb = s_job[1];
        uint32_t next = 0xFFFFFFFFu;
        for (uint32_t j = slice + 1; j < nsl; ++j) {
          if (qb == 0xFFFFFFFFu) {  // queue full: all of them here
            next = j;
            break;
          }
          if (atomicCAS(&fsq[qb + j - 1u].x, wg + 1u, GS_FSQ_TAKEN) == wg + 1u) {
            next = j;
            break;
          }
        }
        s_job[2] = next;
      }
      __syncthreads();
      const uint32_t next = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_job[2]);
      if (next == 0xFFFFFFFFu) break;
      slice = next;
    }
  }
  acc_pairs = wave_reduce<2>(acc_pairs);
  acc_res = wave_reduce<2>(acc_res);
  __syncthreads();
  if (lane == 0) {
    s_red[0][wave] = acc_pairs;
    s_red[1][wave] = acc_res;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // per-workgroup partials (the blend's block (0, 0) sums them: no fan-in atomics)
    uint32_t p = 0, r = 0;
    for (uint32_t w = 0; w < WG / 64; ++w) {
      p += s_red[0][w];
      r += s_red[1][w];
    }
    const uint32_t fw = blockIdx.y * gridDim.x + blockIdx.x;
    fzp[2 * fw] = p;
    fzp[2 * fw + 1] = r;
  }
  STAMP_SYNC();
  STAMP(0, 5);
}

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

// ---- large tiles: radix sort ----------------------------------------------------------------------
// Tiles of more than GS_MID pairs are listed by the colscan and sorted here, before the blend, by
// 256-work-item workgroups striding over the list:
//  load     the segment's depths (u32) and positions (u16) into LDS (tiles of up to 256 * rmax
//           pairs; rmax follows the previous frame's largest tile) or, above that, into a global
//           scratch at the tile's pair offset (10M Gaussians at 4K: ~28k-pair tiles, L2-resident)
//  passes   stable LSD radix sort on the depth minus the tile's minimum, 4-bit digits over the bits
//           of the depth range (C2's 4..12 depths: 24 bits, 6 passes); work-item t owns positions
//           [t R, t R + R) (R odd: bank-conflict free in LDS): per-digit counts in packed byte
//           registers, a (digit, work-item) scan of the 16 x 256 u16 counters in LDS, then each item
//           goes to (its digit's scanned base) + (earlier items of that digit in the work-item)
//  ties     equal depths are put in gaussian order (odd-even transposition inside equal-depth runs;
//           rare: the order of a stable global sort of (tile, depth) keys over gaussian indices)
//  publish  keys_out = tile << 32 | depth, vals_out = gaussian (the blend streams these)
// A 16-byte-per-comparator LDS bitonic network measured ~5 MB of LDS traffic per 2.6k-pair tile
// (LDS-bandwidth bound: ~130 us of the 1M-Gaussian frame); the radix moves ~0.2 MB.
#ifndef GS_SORT_THREADS
#define GS_SORT_THREADS 256
#endif
#ifndef GS_RADIX_MAXR
#define GS_RADIX_MAXR (8448 / GS_SORT_THREADS)  // items per work-item in LDS: up to 8448 keys
#endif
#define GS_RADIX_MAXN 65535u  // u16 positions: global bitonic above (never met by the configs)

__host__ __device__ constexpr size_t gs_radix_lds(uint32_t rmax) {
  return (size_t)GS_SORT_THREADS * rmax * 12u + 16u * GS_SORT_THREADS * 2u;
}

// Sort positions [0, n) of (dep[0], slot[0]) (dep[1] / slot[1]: the other half of the ping-pong) by
// depth; returns the half that holds the result. DEP / SLOT are LDS or global arrays (inlined per
// call site, so the address spaces are known); s_cnt and s_red are LDS.
__device__ __forceinline__ uint32_t gs_radix_tile(uint32_t* dep0, uint32_t* dep1, uint16_t* slot0, uint16_t* slot1,
                                                  uint16_t* s_cnt, uint32_t (*s_red)[GS_SORT_THREADS / 64],
                                                  const uint32_t* segw, uint32_t n, uint32_t R) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t vmin = ~0u, vmax = 0u;
  for (uint32_t k0 = tid; k0 < n; k0 += 8 * GS_SORT_THREADS) {  // 8 loads in flight per work-item
    uint32_t d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t k = k0 + j * GS_SORT_THREADS;
      d[j] = k < n ? segw[2 * k + 1] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t k = k0 + j * GS_SORT_THREADS;
      if (k < n) {
        vmin = min(vmin, d[j]);
        vmax = max(vmax, d[j]);
        dep0[k] = d[j];
        slot0[k] = (uint16_t)k;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    vmin = min(vmin, (uint32_t)__shfl_xor((int)vmin, off));
    vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, off));
  }
  if (lane == 0) {
    s_red[0][wave] = vmin;
    s_red[1][wave] = vmax;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < GS_SORT_THREADS / 64; ++w) {
    vmin = min(vmin, s_red[0][w]);
    vmax = max(vmax, s_red[1][w]);
  }
  // depth bits of positive floats order like the floats: sort (d - min) over the bits of max - min
  vmin = (uint32_t)__builtin_amdgcn_readfirstlane((int)vmin);
  vmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)vmax);
  const uint32_t nbits = vmax > vmin ? 32u - (uint32_t)__builtin_clz(vmax - vmin) : 0u;
  const uint32_t p0 = tid * R, p1 = min(n, p0 + R);  // this work-item's positions
  uint32_t cur = 0;
  for (uint32_t sh = 0; sh < nbits; sh += 4) {
    const uint32_t* sd = cur ? dep1 : dep0;
    const uint16_t* ss = cur ? slot1 : slot0;
    uint32_t* dd = cur ? dep0 : dep1;
    uint16_t* ds = cur ? slot0 : slot1;
    // counts: bytes of c0 (digits 0-7) and c1 (digits 8-15); R < 256
    unsigned long long c0 = 0, c1 = 0;
#pragma unroll 8
    for (uint32_t p = p0; p < p1; ++p) {
      const uint32_t d = ((sd[p] - vmin) >> sh) & 15u;
      const unsigned long long inc = 1ull << ((d & 7u) * 8u);
      c0 += d < 8u ? inc : 0ull;
      c1 += d < 8u ? 0ull : inc;
    }
#pragma unroll
    for (uint32_t d = 0; d < 8; ++d) {
      s_cnt[d * GS_SORT_THREADS + tid] = (uint16_t)((c0 >> (8u * d)) & 0xFFu);
      s_cnt[(d + 8) * GS_SORT_THREADS + tid] = (uint16_t)((c1 >> (8u * d)) & 0xFFu);
    }
    __syncthreads();
    // exclusive scan of the counters in (digit, work-item) order: work-item t holds entries [16t, 16t+16)
    uint4* cw = reinterpret_cast<uint4*>(s_cnt + 16u * tid);
    const uint4 a0 = cw[0], a1 = cw[1];
    uint32_t v[16] = {a0.x & 0xFFFFu, a0.x >> 16, a0.y & 0xFFFFu, a0.y >> 16, a0.z & 0xFFFFu, a0.z >> 16,
                      a0.w & 0xFFFFu, a0.w >> 16, a1.x & 0xFFFFu, a1.x >> 16, a1.y & 0xFFFFu, a1.y >> 16,
                      a1.z & 0xFFFFu, a1.z >> 16, a1.w & 0xFFFFu, a1.w >> 16};
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t x = v[k];
      v[k] = sum;
      sum += x;
    }
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_red[0][wave] = incl;
    __syncthreads();
    uint32_t base = incl - sum;
    for (uint32_t w = 0; w < wave; ++w) base += s_red[0][w];
    cw[0] = make_uint4((v[0] + base) | ((v[1] + base) << 16), (v[2] + base) | ((v[3] + base) << 16),
                       (v[4] + base) | ((v[5] + base) << 16), (v[6] + base) | ((v[7] + base) << 16));
    cw[1] = make_uint4((v[8] + base) | ((v[9] + base) << 16), (v[10] + base) | ((v[11] + base) << 16),
                       (v[12] + base) | ((v[13] + base) << 16), (v[14] + base) | ((v[15] + base) << 16));
    __syncthreads();
    // scatter, stable inside the work-item (running byte counters) and across work-items (the scan);
    // batches of 8: a batch's loads issue before its stores (which the compiler may not reorder
    // across: every array can alias)
    c0 = 0;
    c1 = 0;
    for (uint32_t q0 = p0; q0 < p1; q0 += 8) {
      uint32_t dv[8], sv[8], dst[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t p = min(q0 + j, p1 - 1);
        dv[j] = sd[p];
        sv[j] = ss[p];
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t d = ((dv[j] - vmin) >> sh) & 15u;
        const uint32_t bit = (d & 7u) * 8u;
        const unsigned long long cc = d < 8u ? c0 : c1;
        const uint32_t local = (uint32_t)(cc >> bit) & 0xFFu;
        const bool ok = q0 + j < p1;
        c0 += (ok && d < 8u) ? (1ull << bit) : 0ull;
        c1 += (ok && d >= 8u) ? (1ull << bit) : 0ull;
        dst[j] = (uint32_t)s_cnt[d * GS_SORT_THREADS + tid] + local;
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j)
        if (q0 + j < p1) {
          dd[dst[j]] = dv[j];
          ds[dst[j]] = (uint16_t)sv[j];
        }
    }
    __syncthreads();
    cur ^= 1u;
  }
  return cur;
}

// ties (equal depths in gaussian order) and publish of one sorted tile
__device__ __forceinline__ void gs_radix_publish(const uint32_t* sd, uint16_t* ss, const uint32_t* segw, uint32_t n,
                                                 unsigned long long tbits, unsigned long long* keys_out,
                                                 uint32_t* vals_out) {
  const uint32_t tid = threadIdx.x;
  int tie = 0;
  for (uint32_t k = tid; k + 1 < n; k += GS_SORT_THREADS) tie |= sd[k] == sd[k + 1];
  if (__syncthreads_or(tie)) {
    int changed;
    do {
      changed = 0;
      for (uint32_t ph = 0; ph < 2; ++ph) {
        for (uint32_t k = 2 * tid + ph; k + 1 < n; k += 2 * GS_SORT_THREADS)
          if (sd[k] == sd[k + 1]) {
            const uint16_t x = ss[k], y = ss[k + 1];
            if (segw[2 * (uint32_t)y] < segw[2 * (uint32_t)x]) {
              ss[k] = y;
              ss[k + 1] = x;
              changed = 1;
            }
          }
        __syncthreads();
      }
    } while (__syncthreads_or(changed));
  }
  for (uint32_t k0 = tid; k0 < n; k0 += 8 * GS_SORT_THREADS) {  // 8 gathers in flight per work-item
    uint32_t g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t k = k0 + j * GS_SORT_THREADS;
      g[j] = k < n ? segw[2 * (uint32_t)ss[k]] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t k = k0 + j * GS_SORT_THREADS;
      if (k < n) {
        if (keys_out) keys_out[k] = tbits | sd[k];  // (keys: only for a published frame)
        vals_out[k] = g[j];
      }
    }
  }
}

__global__ __launch_bounds__(GS_SORT_THREADS) void gs_sort_large_kernel(
    const uint2* __restrict__ ranges, unsigned long long* __restrict__ pairs,
    const unsigned long long* __restrict__ tile_slots, const uint32_t* __restrict__ large,
    const uint32_t* __restrict__ large_ctr, unsigned long long* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    const uint32_t* __restrict__ total, uint32_t cap, uint32_t rmax, uint32_t* __restrict__ g_dep,
    uint16_t* __restrict__ g_slot, uint32_t g_cap, GsFused fu, uint32_t ntiles) {
  // LDS: one array per field, halves at offsets (an array of LDS pointers indexed at run time would
  // turn every access into a FLAT one)
  extern __shared__ __attribute__((aligned(16))) char s_arena[];
  const uint32_t capn = GS_SORT_THREADS * rmax;
  uint32_t* s_dep = reinterpret_cast<uint32_t*>(s_arena);           // [2][capn]
  uint16_t* s_slot = reinterpret_cast<uint16_t*>(s_dep + 2 * capn);  // [2][capn]
  uint16_t* s_cnt = s_slot + 2 * capn;                                // [16 digits][256 work-items]
  __shared__ uint32_t s_red[2][GS_SORT_THREADS / 64];
  __shared__ uint32_t s_list[GS_SORT_THREADS + 1];  // fused: this block's large tiles
  const uint32_t tid = threadIdx.x;
  uint32_t count;
  if (fu.scap) {
    // fused front end: no tile list; block b checks tiles b, b + grid, ... (<= 256 of them: the host
    // sizes the grid) by their cursors and sorts those above GS_MID pairs that fit their rows (a
    // spilled tile, above scap, is gathered and sorted by its blend workgroup: gs_spill_tile)
    if (tid == 0) s_list[GS_SORT_THREADS] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x + tid * gridDim.x;
    if (t < ntiles) {
      const uint32_t c = fu.cursor[t];
      if (c > GS_MID && c <= fu.scap) s_list[atomicAdd(&s_list[GS_SORT_THREADS], 1u)] = t;
    }
    __syncthreads();
    count = s_list[GS_SORT_THREADS];
  } else {
    count = large_ctr[0];
  }
  // static striding over the list (a shared work counter serialises: ~30 ns per contended atomic,
  // 210 us for the 1M-Gaussian frame's 7k claims)
  for (uint32_t li = fu.scap ? 0 : blockIdx.x; li < count; li += fu.scap ? 1 : gridDim.x) {
    const uint32_t tile = fu.scap ? s_list[li] : large[li];
    const uint2 range = fu.scap ? make_uint2(tile * fu.scap, tile * fu.scap + fu.cursor[tile]) : ranges[tile];
    if (!fu.scap && range.y > cap) continue;  // segment beyond the pair buffer: spilled (gs_spill_tile)
    const uint32_t n = range.y - range.x;
    unsigned long long* seg = fu.scap ? const_cast<unsigned long long*>(tile_slots) + range.x
                            : n <= GS_TILE_SLOTS ? const_cast<unsigned long long*>(tile_slots) + (size_t)tile * GS_TILE_SLOTS
                                                 : pairs + range.x;
    const uint32_t* segw = reinterpret_cast<const uint32_t*>(seg);  // (gaussian, depth) word pairs
    const unsigned long long tbits = (unsigned long long)tile << 32;
    const uint32_t R = ((n + GS_SORT_THREADS - 1) / GS_SORT_THREADS) | 1u;
    if (R <= rmax) {
      const uint32_t h = gs_radix_tile(s_dep, s_dep + capn, s_slot, s_slot + capn, s_cnt, s_red, segw, n, R);
      gs_radix_publish(s_dep + h * capn, s_slot + h * capn, segw, n, tbits, keys_out ? keys_out + range.x : nullptr,
                       vals_out + range.x);
    } else if (g_dep && n <= GS_RADIX_MAXN && range.y <= g_cap) {
      // global scratch at the tile's pair offset: [2][g_cap] depths, [2][g_cap] positions
      uint32_t* d0 = g_dep + range.x;
      uint16_t* s0 = g_slot + range.x;
      const uint32_t h = gs_radix_tile(d0, d0 + g_cap, s0, s0 + g_cap, s_cnt, s_red, segw, n, R);
      gs_radix_publish(h ? d0 + g_cap : d0, h ? s0 + g_cap : s0, segw, n, tbits,
                       keys_out ? keys_out + range.x : nullptr, vals_out + range.x);
    } else {  // bitonic network in global memory (a frame whose tiles outgrew the scratch)
      bitonic_flip_sort(n, [&](uint32_t a, uint32_t b) {
        unsigned long long x = seg[a], y = seg[b];
        if (y < x) { seg[a] = y; seg[b] = x; }
      });
      for (uint32_t k = tid; k < n; k += GS_SORT_THREADS) {
        const unsigned long long v = seg[k];
        if (keys_out) keys_out[range.x + k] = tbits | (v >> 32);
        vals_out[range.x + k] = (uint32_t)v;
      }
    }
    __syncthreads();  // LDS reused by the next tile
  }
}

// ---- blend ----------------------------------------------------------------------------------------
// Merge ranking (tiles of more than GS_MERGE_MIN pairs): every wave sorts its 64 keys in registers
// (bitonic network over the lanes, ascending), the sorted runs go to LDS, and a key's rank is its lane
// plus, for every other run, the count of that run's keys below it (a binary search of 7 LDS reads):
// ~200 VALU per key for 2-4 runs and ~400 for 8 instead of n / 4 compares against every key (the
// counting below): keys are unique, so the ranks are the same.
// (the exchanges through DPP and the gfx950 permlane swaps: no LDS round trip per step)
// the lanes of a bitonic step (K, J) that keep the smaller key: ascending blocks' low halves and descending
// blocks' high halves (a compile-time lane mask)
template <uint32_t K, uint32_t J>
__host__ __device__ constexpr unsigned long long gs_keep_min_mask() {
  unsigned long long m = 0;
  for (uint32_t l = 0; l < 64u; ++l)
    if (((l & K) == 0u) == ((l & J) == 0u)) m |= 1ull << l;
  return m;
}
// one compare-exchange step: a lane takes its partner's key iff (partner < own) equals "keeps the
// minimum" — one 64-bit compare, the lane mask applied to its result in SGPRs, two selects (the min / max
// form compared twice and selected three times: 21 steps x ~6 VALU more per wave sort, ~0.7 M VALU per
// C2 frame)
template <uint32_t K, uint32_t J>
__device__ __forceinline__ unsigned long long gs_sort_step(unsigned long long x, uint32_t lane) {
  const unsigned long long y = lane_xor64<J>(x, lane);
  const unsigned long long take = ~(__builtin_amdgcn_ballot_w64(y < x) ^ gs_keep_min_mask<K, J>());
  return __builtin_amdgcn_inverse_ballot_w64(take) ? y : x;
}
__device__ __forceinline__ unsigned long long gs_wave_sort64(unsigned long long x, uint32_t lane) {
  x = gs_sort_step<2, 1>(x, lane);
  x = gs_sort_step<4, 2>(x, lane); x = gs_sort_step<4, 1>(x, lane);
  x = gs_sort_step<8, 4>(x, lane); x = gs_sort_step<8, 2>(x, lane); x = gs_sort_step<8, 1>(x, lane);
  x = gs_sort_step<16, 8>(x, lane); x = gs_sort_step<16, 4>(x, lane); x = gs_sort_step<16, 2>(x, lane);
  x = gs_sort_step<16, 1>(x, lane);
  x = gs_sort_step<32, 16>(x, lane); x = gs_sort_step<32, 8>(x, lane); x = gs_sort_step<32, 4>(x, lane);
  x = gs_sort_step<32, 2>(x, lane); x = gs_sort_step<32, 1>(x, lane);
  x = gs_sort_step<64, 32>(x, lane); x = gs_sort_step<64, 16>(x, lane); x = gs_sort_step<64, 8>(x, lane);
  x = gs_sort_step<64, 4>(x, lane); x = gs_sort_step<64, 2>(x, lane); x = gs_sort_step<64, 1>(x, lane);
  return x;
}
// keys below x in the sorted 64-key runs [0, m) of s_key except run `self` (m <= R): the binary searches
// of every run advance in lockstep, so each step's R LDS reads are in flight together (one round trip
// per step instead of one per step and run); runs >= m are read but not counted
template <uint32_t R>
__device__ __forceinline__ uint32_t gs_runs_below(const unsigned long long* s_key, uint32_t m, uint32_t self,
                                                  unsigned long long x) {
  uint32_t pos[R];
#pragma unroll
  for (uint32_t q = 0; q < R; ++q) pos[q] = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) {
    unsigned long long v[R];
#pragma unroll
    for (uint32_t q = 0; q < R; ++q) v[q] = s_key[64u * q + pos[q] + step - 1u];
#pragma unroll
    for (uint32_t q = 0; q < R; ++q) pos[q] += (q < m && q != self && v[q] < x) ? step : 0u;
  }
  uint32_t r = 0;
  unsigned long long v[R];
#pragma unroll
  for (uint32_t q = 0; q < R; ++q) v[q] = s_key[64u * q + pos[q]];
#pragma unroll
  for (uint32_t q = 0; q < R; ++q) r += (q < m && q != self) ? pos[q] + (v[q] < x ? 1u : 0u) : 0u;
  return r;
}
// keys of the sorted 64-key run b below x
__device__ __forceinline__ uint32_t gs_run_below(const unsigned long long* b, unsigned long long x) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1)
    if (b[pos + step - 1] < x) pos += step;
  return pos + (b[pos] < x ? 1u : 0u);
}
#ifndef GS_MERGE_MIN
#define GS_MERGE_MIN 96u  // (counting is cheaper for up to ~1.5 runs)
#endif
#define GS_ARENA (48 * (GS_BLOCK + 1) + 4 * (GS_BLOCK + 4) * 4)  // staged records + per-quadrant lists

struct GStage {  // one staged blend record (see gs_preprocess_one)
  float4 a, b, c;
};

// ---- spilled tiles --------------------------------------------------------------------------------
// A tile whose pairs the front end could not all store (fused: more than its row's scap pairs, e.g.
// the camera moved closer than the previous frame that sized the rows; three launches: a segment that
// ends beyond the pair buffer sized from earlier frames) is completed by its own blend workgroup, in
// the same launch: the front-end workgroups whose bounding rect (crect) holds the tile are listed,
// their Gaussians' stored rects tested against the tile, and the keys (depth << 32 | gaussian, the
// front ends' keys) collected; then sorted (bitonic: in the LDS arena up to GS_SPILL_LDS keys, else in
// the pool) and the sorted gaussians written to the spill pool, from which the blend streams them like
// a large tile's. Same keys, same order, same blend: the image equals a frame whose rows had fit (and
// the oracle's). The pool (cap pairs per workspace) is reserved per tile with one atomic (fz[8], re-armed
// by the next frame's front end, which also hands the demand to the host to size the pool); a tile that
// does not fit is left at the background and counted (fz[10]; k_host[9] = 1: the next call reports it).
struct GsSpill {
  uint32_t* fz;                   // device counters: [8] pool cursor, [9] spilled tiles, [10] incomplete tiles
  uint32_t* k_host;               // pinned host words: [9] <- 1 when a tile could not be completed
  unsigned long long* keys;       // pool: keys of tiles above GS_SPILL_LDS pairs
  uint32_t* vals;                 // pool: sorted gaussians of every spilled tile
  uint32_t cap;                   // pool capacity (pairs)
  const ushort4* crect;           // per front-end workgroup (chunk c of band b at c * bands + b): rect of its pairs
  uint32_t nwg, bands, chunk, n;  // front-end workgroups, bands, Gaussians per chunk, Gaussians
  const ushort4* rects;           // per Gaussian (walk order): tile rect (empty: culled)
  const float* depths;            // per Gaussian (walk order): view depth
  const uint32_t* ids;            // the caller's index (NULL: the walk index)
};
#define GS_SPILL_LDS 1984u  // keys sorted in the blend's LDS arena (15 872 B + the candidate list + counters)
#define GS_SPILL_CAND 128u  // front-end workgroups tested per round
static_assert(GS_ARENA >= 8u * GS_SPILL_LDS + 4u * (GS_SPILL_CAND + 3u), "gs_spill_tile's keys, candidates and counters fit the arena");

// Returns the sorted gaussians of tile (tx, ty) in the pool and their count in m (on entry: the
// tile's pair count), or nullptr when the pool is exhausted. Uses the arena (>= 16 400 B of LDS).
__device__ const uint32_t* gs_spill_tile(const GsSpill& sp, uint32_t tx, uint32_t ty, uint32_t& m, char* arena) {
  const uint32_t tid = threadIdx.x, n = m;
  unsigned long long* s_k = reinterpret_cast<unsigned long long*>(arena);
  uint32_t* s_c = reinterpret_cast<uint32_t*>(arena + 8 * GS_SPILL_LDS);
  uint32_t* s_w = s_c + GS_SPILL_CAND;  // [0] keys found, [1] pool offset, [2] candidates of the round
  const bool lds = n <= GS_SPILL_LDS;
  if (tid == 0) {
    s_w[0] = 0;
    s_w[2] = 0;
    uint32_t off = atomicAdd(sp.fz + 8, n);
    atomicAdd(sp.fz + 9, 1u);
    if (off > sp.cap || n > sp.cap - off) {
      off = 0xFFFFFFFFu;
      atomicAdd(sp.fz + 10, 1u);
      __atomic_store_n(sp.k_host + 9, 1u, __ATOMIC_RELAXED);
      __threadfence_system();
    }
    s_w[1] = off;
  }
  __syncthreads();
  const uint32_t off = s_w[1];
  if (off == 0xFFFFFFFFu) return nullptr;
  unsigned long long* gk = sp.keys + off;
  for (uint32_t w0 = 0; w0 < sp.nwg; w0 += GS_SPILL_CAND) {
    if (tid < GS_SPILL_CAND && w0 + tid < sp.nwg) {
      const ushort4 r = sp.crect[w0 + tid];
      if (r.x <= tx && tx < r.z && r.y <= ty && ty < r.w) s_c[atomicAdd(s_w + 2, 1u)] = w0 + tid;
    }
    __syncthreads();
    const uint32_t nc = s_w[2];
    for (uint32_t k = 0; k < nc; ++k) {
      const uint32_t c = s_c[k] / sp.bands;
      const uint32_t g0 = c * sp.chunk, g1 = min(sp.n, g0 + sp.chunk);
      for (uint32_t i = g0 + tid; i < g1; i += GS_BLOCK) {
        const ushort4 r = sp.rects[i];
        if (r.x <= tx && tx < r.z && r.y <= ty && ty < r.w) {
          const unsigned long long key =
              ((unsigned long long)__float_as_uint(sp.depths[i]) << 32) | (sp.ids ? sp.ids[i] : i);
          const uint32_t p = atomicAdd(s_w, 1u);
          if (p < n) {
            if (lds) s_k[p] = key;
            else gk[p] = key;
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) s_w[2] = 0;
    __syncthreads();
  }
  m = min(s_w[0], n);  // (= n: the rects are the ones the front end counted)
  const uint32_t mm = m;
  if (lds) {
    bitonic_flip_sort(mm, [&](uint32_t a, uint32_t b) {
      const unsigned long long x = s_k[a], y = s_k[b];
      if (y < x) { s_k[a] = y; s_k[b] = x; }
    });
    for (uint32_t k = tid; k < mm; k += GS_BLOCK) sp.vals[off + k] = (uint32_t)s_k[k];
  } else {
    bitonic_flip_sort(mm, [&](uint32_t a, uint32_t b) {
      const unsigned long long x = gk[a], y = gk[b];
      if (y < x) { gk[a] = y; gk[b] = x; }
    });
    for (uint32_t k = tid; k < mm; k += GS_BLOCK) sp.vals[off + k] = (uint32_t)gk[k];
  }
  __syncthreads();  // the values (and the arena's last reads) before the blend stages records over them
  return sp.vals + off;
}

// One 256-work-item workgroup per 16x16 tile (a persistent, software-pipelined variant that loads
// the next tile's keys during the current one measured slower: static tile assignment loses to the
// dispatcher's dynamic balancing, 103 vs 72 us at C2; a tile-pair workgroup shading two pixels per
// lane in packed f32 measured 133 vs 104 us per frame: the per-pixel done / valid bookkeeping of the
// pair and the strip lists cost more than the packing saved).
//  sort     tiles of <= 256 pairs: one key per work-item; up to GS_MERGE_MIN pairs ranked by counting
//           against all n keys in LDS, above that by merge ranking (gs_wave_sort64 + gs_run_below);
//           while it runs, the blend records of the unsorted keys are already in flight, and the
//           staging slot of sorted position r is recorded; then publish the sorted keys (tile << 32 |
//           depth) / values (gaussian). Tiles of (256, GS_MID] pairs are merge-ranked two keys per
//           work-item. Larger tiles were sorted and published by gs_sort_large_kernel: their values
//           are streamed in batches of 256, the records of batch b + 1 (and the values of b + 2) in
//           flight while batch b blends.
//  blend    wave w shades the 8x8 quadrant q = w of the tile (x half w & 1, y half w >> 1), one pixel
//           per lane. Each staged Gaussian's alpha box is tested against the four quadrants (a 4-bit
//           mask in LDS; small tiles add the exact per-quadrant test, stage_rec); every wave ballots
//           bit w over the batch's masks in sorted order into its own list (no cross-wave counts: one
//           barrier per batch), so a wave iterates only the Gaussians that can touch its 64 pixels.
//           alpha = min(0.99, 2^z) with the hardware exp2 (within 1e-4 relative L2 of the oracle's exp,
//           test_raster_gpu.py); front to back, stop before the Gaussian that would take T below 1e-4
//           (the reference's rule).
// OVER (hybrid composite): per-pixel depth limit and an "under" image instead of the background colour
// Measured and rejected here: per-4x4-sub-block lists, one per ds_read_b128 lane group of a wave (each
// group reads its own list's record in the cycle a broadcast takes, 16% fewer evaluation steps at C2):
// 0.0596 vs 0.0564 ms, the u16 lists' unpacking, four ballots per compaction round and the sub-block
// masks cost more than the steps saved (the machinery alone with quadrant lists: 0.0620 ms); and (git
// history: round 4) records read by one lane and broadcast with
// readfirstlane (C2 0.0784 vs 0.0565 ms), alphas of several entries computed ahead of the transmittance
// chain, the termination applied without its wave-uniform branch, an XCD-aware tile mapping, loading the
// key row only up to the previous frame's count, non-temporal records / key rows.
#define GS_DONE_EVERY 4u  // list entries between the wave's all-pixels-done tests (a power of two >= 4)
// (the termination as two selects per entry instead of the wave-uniform branch: 2 spilled VGPRs, C2 serial
// 0.0607 vs 0.0563 ms, round 6)
// (Measured and rejected, round 6: the quadratic as three packed v_pk_mul / v_pk_fma_f32 over the record's
// (A, C) (B, D) (E, F) pairs plus one add, and red / green as one packed FMA: 13 VALU per entry instead of
// 15, but C2 0.0574 vs 0.0558 ms: the packed ops' dependency stalls (s_nop) lengthen each wave's chain.)
#ifndef GS_BLEND_MIN_BLOCKS
#define GS_BLEND_MIN_BLOCKS 8  // 64 VGPRs: 8 waves per SIMD (vs 7 at 70 VGPRs): +3% at C2
#endif
template <bool OVER>
__global__ __launch_bounds__(GS_BLOCK, GS_BLEND_MIN_BLOCKS) void gs_sort_blend_kernel(SplatCam cam, const uint2* __restrict__ ranges,
                                                                 unsigned long long* __restrict__ pairs,
                                                                 uint32_t sorted_above,
                                                                 unsigned long long* __restrict__ keys_out,
                                                                 uint32_t* __restrict__ vals_out,
                                                                 const float4* __restrict__ rec, float bg_r,
                                                                 float bg_g, float bg_b,
                                                                 uint32_t cap, uint32_t slot_keys,
                                                                 const unsigned long long* __restrict__ tile_slots,
                                                                 const float* __restrict__ depth_lim,
                                                                 const float4* __restrict__ under,
                                                                 float4* __restrict__ out, GsFused fu, GsSpill sp) {
  // staged records of the current batch; slot GS_BLOCK is a null Gaussian (alpha = 0) that pads the
  // per-quadrant lists to a multiple of 4.
  __shared__ __attribute__((aligned(16))) char s_arena[GS_ARENA];
  GStage* s_stage = reinterpret_cast<GStage*>(s_arena);
  uint32_t(*s_list)[GS_BLOCK + 4] = reinterpret_cast<uint32_t(*)[GS_BLOCK + 4]>(s_arena + sizeof(GStage) * (GS_BLOCK + 1));
  // the merge ranks' sorted runs and a mid tile's ranked keys alias the arena: records are staged only
  // after the last read of either (behind a barrier)
  unsigned long long* s_key = reinterpret_cast<unsigned long long*>(s_arena);
  __shared__ uint8_t s_mask[GS_BLOCK];
  __shared__ uint8_t s_sslot[GS_BLOCK];  // small tiles: staging slot of sorted position p
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  STAMP(1, 0);
  if (fu.seq_flag && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0)  // (this blend has started: SplatSeq)
    __hip_atomic_store(fu.seq_flag, fu.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (fu.scap) {
    // fused front end: block (0, 0) hands the frame's counters to the host and re-arms them (the
    // fused kernel that produced them has finished; no other blend block reads them)
    uint32_t fp = 0, fr = 0;  // the front end's pairs and reservations (block (0, 0) sums the partials)
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      for (uint32_t k = tid; k < fu.nwg; k += GS_BLOCK) {
        fp += fu.fzp[2 * k];
        fr += fu.fzp[2 * k + 1];
      }
      for (int off = 32; off > 0; off >>= 1) {
        fp += (uint32_t)__shfl_xor((int)fp, off);
        fr += (uint32_t)__shfl_xor((int)fr, off);
      }
      uint32_t* s_r = reinterpret_cast<uint32_t*>(s_arena);  // (before any other use of the arena)
      if (lane == 0) {
        s_r[wave] = fp;
        s_r[4 + wave] = fr;
      }
      __syncthreads();
      fp = (s_r[0] + s_r[1]) + (s_r[2] + s_r[3]);
      fr = (s_r[4] + s_r[5]) + (s_r[6] + s_r[7]);
      __syncthreads();
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
      const uint32_t big = fu.fz[1];
      __atomic_store_n(fu.k_host + 1, big > 256u ? big : 256u, __ATOMIC_RELAXED);  // largest tile (bound)
      __atomic_store_n(fu.k_host + 2, fu.fz[4], __ATOMIC_RELAXED);                  // large tiles
      __atomic_store_n(fu.k_host + 4, fr, __ATOMIC_RELAXED);                        // reservations
      __atomic_store_n(fu.k_host + 5, fu.fz[5], __ATOMIC_RELAXED);                  // tiles above scap (spilled)
      __atomic_store_n(fu.k_host + 6, 1u, __ATOMIC_RELAXED);                       // published by: fused
      __atomic_store_n(fu.k_host, fp, __ATOMIC_RELAXED);
      if (fp > fu.fz[13]) fu.fz[13] = fp;  // the workspace's largest K (fused; three launches: total[2])
      __atomic_store_n(fu.k_host + 12, fu.fz[13], __ATOMIC_RELAXED);
      fu.fz[1] = 0;
      fu.fz[4] = 0;
      fu.fz[5] = 0;
      __threadfence_system();
    }
    if (blockIdx.x == 0 && blockIdx.y == 0) {  // the slice queue of the front end back to empty
      const uint32_t used = min(fu.fz[GS_FSQ_W + 1], fu.fsq_cap);
      for (uint32_t k = tid; k < used; k += GS_BLOCK) fu.fsq[k] = make_uint2(0u, 0u);
      if (tid == 0) {
        __atomic_store_n(fu.k_host + 11, fu.fz[GS_FSQ_W + 1], __ATOMIC_RELAXED);  // queued slices (helpers)
        fu.fz[GS_FSQ_W] = 0;
        fu.fz[GS_FSQ_W + 1] = 0;
        fu.fz[GS_FSQ_W + 2] = 0;
      }
    }
  }
  uint32_t tile_x = blockIdx.x, tile_y = cam.row_begin + blockIdx.y;
  uint32_t tile = tile_y * cam.grid_x + tile_x;
  if (fu.order) {  // heavy tiles first (gs_tile_order)
    tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)fu.order[blockIdx.y * gridDim.x + blockIdx.x]);
    tile_y = tile / cam.grid_x;
    tile_x = tile - tile_y * cam.grid_x;
  }
  STAMP(1, 4);
  const float tx0 = (float)(tile_x * GS_BLOCK_X), ty0 = (float)(tile_y * GS_BLOCK_Y);
  // Stage a record as the quadratic in tile-local pixel coordinates (ux, uy):
  // z = A ux^2 + B ux uy + C uy^2 + D ux + E uy + F (five FMAs per evaluation instead of seven), and
  // return the quadrant mask of its alpha box: bit q = (x half q & 1, y half q >> 1), the box tested
  // in tile-local coordinates against the quadrants' pixel ranges [0, 7] / [8, 15] (immediates: no
  // register holds a tile bound across the batch loop; the box's 1% + 0.01 px margin covers the
  // rounding of the local shift). exact: also the exact quadrant test (small tiles; the large-tile batch
  // loop keeps the box test: its copy of the test spilled 2 VGPRs).
  auto stage_rec = [&](uint32_t slot, const float4& ga, const float4& gb, const float4& gc, bool exact) -> uint32_t {
    const float gx = ga.x - tx0, gy = ga.y - ty0, A = ga.z, B = ga.w, C = gb.x;
    const float D = -2.0f * A * gx - B * gy, E = -B * gx - 2.0f * C * gy;
    const float F = ((A * gx * gx + B * gx * gy) + C * gy * gy) + gb.y;
    s_stage[slot].a = make_float4(A, B, C, D);
    s_stage[slot].b = make_float4(E, F, gb.z, gb.w);
    s_stage[slot].c = gc;
    const float x0 = gx - gc.y, x1 = gx + gc.y, y0 = gy - gc.z, y1 = gy + gc.z;
    const bool xl = x0 <= 7.0f && x1 >= 0.0f, xr = x0 <= 15.0f && x1 >= 8.0f;
    const bool yt = y0 <= 7.0f && y1 >= 0.0f, yb = y0 <= 15.0f && y1 >= 8.0f;
    uint32_t qm = (uint32_t)(xl && yt) | ((uint32_t)(xr && yt) << 1) | ((uint32_t)(xl && yb) << 2) |
                  ((uint32_t)(xr && yb) << 3);
    if (exact) {
      // exact quadrant test (C2 0.0585 -> 0.0577 ms, bit-exact): the largest z over a quadrant's pixel
      // square (z concave: A, C < 0) is at the centre when the centre lies inside, else on an edge, each
      // edge's a clamped 1D parabola. A quadrant whose largest z is below log2(1/255) (minus a 0.02
      // margin for the rounding of the staged form) has no pixel with alpha >= 1/255: the entry would be
      // evaluated to nothing by every lane of its wave.
      // the vertex u* = -q / (2p) = q * (-1 / (2p)) (an approximate reciprocal: the value at a point near
      // the vertex is within the margin of the maximum)
      const float i2a = -0.5f * __builtin_amdgcn_rcpf(A), i2c = -0.5f * __builtin_amdgcn_rcpf(C);
      auto vmax = [](float p, float q, float r, float inv, float u0, float u1) {
        const float u = fminf(fmaxf(q * inv, u0), u1);
        return __builtin_fmaf(__builtin_fmaf(p, u, q), u, r);
      };
      const float zk = -7.9943534f - 0.02f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo_x = (q & 1) ? 8.0f : 0.0f, lo_y = (q >> 1) ? 8.0f : 0.0f;
        const float hi_x = lo_x + 7.0f, hi_y = lo_y + 7.0f;
        const bool inside = gx >= lo_x && gx <= hi_x && gy >= lo_y && gy <= hi_y;
        // x = lo_x / hi_x over y in [lo_y, hi_y]; y = lo_y / hi_y over x in [lo_x, hi_x]
        const float m0 = vmax(C, __builtin_fmaf(B, lo_x, E), __builtin_fmaf(__builtin_fmaf(A, lo_x, D), lo_x, F), i2c, lo_y, hi_y);
        const float m1 = vmax(C, __builtin_fmaf(B, hi_x, E), __builtin_fmaf(__builtin_fmaf(A, hi_x, D), hi_x, F), i2c, lo_y, hi_y);
        const float m2 = vmax(A, __builtin_fmaf(B, lo_y, D), __builtin_fmaf(__builtin_fmaf(C, lo_y, E), lo_y, F), i2a, lo_x, hi_x);
        const float m3 = vmax(A, __builtin_fmaf(B, hi_y, D), __builtin_fmaf(__builtin_fmaf(C, hi_y, E), hi_y, F), i2a, lo_x, hi_x);
        const float m = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
        if (!inside && !(m >= zk)) qm &= ~(1u << q);
      }
    }
    return qm;
  };
  // the tile's slot row is loaded together with its count (no dependent round trip for small tiles;
  // every work-item loads its slot whatever the count)
  const uint32_t srow = fu.scap ? fu.scap : GS_TILE_SLOTS;
  const unsigned long long k_slot = tile_slots[(size_t)tile * srow + tid];
  uint2 range;
  if (fu.scap) {
    const uint32_t c = fu.cursor[tile];
    range = make_uint2(tile * fu.scap, tile * fu.scap + c);
  } else {
    range = ranges[tile];
  }
  uint32_t n = range.y - range.x;
  STAMP_WAITED(1, 5);  // (the slot row and the count have arrived)
  const uint32_t n_front = n;  // (the front end's count: n becomes the completed count of a spilled tile)
  const bool small = slot_keys && n <= GS_BLOCK;
  if (fu.scap && tid == 0) fu.ranges[tile] = range;
  // a tile whose pairs were not all stored (fused: above its row's capacity; three launches: its
  // segment ends beyond the pair buffer) is gathered and sorted here: its sorted gaussians come from
  // the spill pool (nullptr: pool exhausted, the tile stays at the background; counted)
  const bool spilled = fu.scap ? n > fu.scap : (n > GS_TILE_SLOTS && range.y > cap);
  const uint32_t* vsrc = vals_out + range.x;
  if (spilled) {
    vsrc = gs_spill_tile(sp, tile_x, tile_y, n, s_arena);
    if (!vsrc) n = 0;
  }
  const bool mid = !small && !spilled && n <= sorted_above;  // not sorted by gs_sort_large_kernel: sorted here
  // publish (PTGS_FLAG_SPLAT_PUBLISH) only where the tile's range fits the buffers: a three-launch frame
  // above the pair buffer is re-run by the host after growing them (the published layout is that run's)
  const bool pub = keys_out && (fu.scap || range.y <= cap);
  const bool mid_lds = mid && n <= GS_MID;
  const unsigned long long tbits = (unsigned long long)tile << 32;
  float4 ra, rb, rc;     // records in flight: the unsorted keys' (small) / batch b + 1's (large)
  uint32_t g_next = 0;   // large tiles: gaussian of batch b + 2
  unsigned long long key = ~0ull;
  if (small && tid < n) {
    const unsigned long long k_cur = k_slot;
    const uint32_t g = (uint32_t)k_cur;
    if (GS_PROBE(GS_PROBE_NO_REC)) {
      ra = rb = rc = make_float4((float)g, 0.f, 0.f, 0.f);
    } else {
      ra = rec[3 * g];
      rb = rec[3 * g + 1];
      rc = rec[3 * g + 2];
    }
    key = (k_cur & 0xFFFFFFFF00000000ull) | ((unsigned long long)g << 8) | tid;  // g < 2^24 (slot_keys)
  }
  if (small) STAMP_WAITED(1, 6);  // (wave 0's records have arrived)
  if (small && n > GS_MERGE_MIN) {
    // merge ranking: the wave's sorted run in LDS, ranks by binary searches of the other runs; the
    // work-item holding a sorted key (its slot in the low 8 bits) records slot and published key
    const uint32_t m = (n + 63u) >> 6;  // runs holding keys (uniform)
    unsigned long long sk = ~0ull;
    if (wave < m) {
      sk = GS_PROBE(GS_PROBE_NO_MERGE) ? key : gs_wave_sort64(key, lane);
      s_key[tid] = sk;
    }
    __syncthreads();
    uint32_t r = GS_PROBE(GS_PROBE_NO_MERGE) ? tid : lane;
    if (wave < m && !GS_PROBE(GS_PROBE_NO_MERGE)) r += gs_runs_below<GS_BLOCK / 64>(s_key, m, wave, sk);
    __syncthreads();  // every read of the keys is done before records overwrite them
    if (tid < n) s_mask[tid] = (uint8_t)stage_rec(tid, ra, rb, rc, !GS_PROBE(GS_PROBE_NO_EXACT));
    if (sk != ~0ull) {
      if (pub) {
        keys_out[range.x + r] = tbits | (sk >> 32);
        vals_out[range.x + r] = (uint32_t)(sk >> 8) & 0xFFFFFFu;
      }
      s_sslot[r] = (uint8_t)(sk & 0xFFu);
    }
  } else if (small) {
    // rank counting (keys are unique): every work-item of a wave holding keys counts the keys below
    // its own over all n in LDS (uniform reads, eight keys per step, no barrier in the loop) and
    // records its staging slot at that rank
    s_key[tid] = key;  // ~0 above n
    __syncthreads();
    uint32_t r = GS_PROBE(GS_PROBE_NO_RANK) ? tid : 0u;
    if (wave * 64u < n && !GS_PROBE(GS_PROBE_NO_RANK)) {
      // four uniform reads in flight (entries n .. 255 hold ~0: never below a key)
      const uint32_t nu = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);
      for (uint32_t j = 0; j < nu; j += 8) {
        const ulonglong2 x0 = *reinterpret_cast<const ulonglong2*>(s_key + j);
        const ulonglong2 x1 = *reinterpret_cast<const ulonglong2*>(s_key + j + 2);
        const ulonglong2 x2 = *reinterpret_cast<const ulonglong2*>(s_key + j + 4);
        const ulonglong2 x3 = *reinterpret_cast<const ulonglong2*>(s_key + j + 6);
        r += ((uint32_t)(x0.x < key) + (uint32_t)(x0.y < key)) + ((uint32_t)(x1.x < key) + (uint32_t)(x1.y < key)) +
             ((uint32_t)(x2.x < key) + (uint32_t)(x2.y < key)) + ((uint32_t)(x3.x < key) + (uint32_t)(x3.y < key));
      }
    }
    __syncthreads();  // every read of the keys is done before records overwrite them
    if (tid < n) {
      s_mask[tid] = (uint8_t)stage_rec(tid, ra, rb, rc, !GS_PROBE(GS_PROBE_NO_EXACT));
      if (pub) {
        keys_out[range.x + r] = tbits | (key >> 32);
        vals_out[range.x + r] = (uint32_t)(key >> 8) & 0xFFFFFFu;
      }
      s_sslot[r] = (uint8_t)tid;
    }
  } else {
    if (mid) {
      unsigned long long* seg = fu.scap ? const_cast<unsigned long long*>(tile_slots) + range.x
                              : n <= GS_TILE_SLOTS ? const_cast<unsigned long long*>(tile_slots) + (size_t)tile * GS_TILE_SLOTS
                                                   : pairs + range.x;
      if (mid_lds) {
        // merge ranking (above), two keys per work-item: wave w sorts runs w and w + 4 (slots tid and
        // tid + 256), then writes both keys to their ranks (keys are unique: the gaussian is in the
        // low word)
        unsigned long long k0 = tid < n ? seg[tid] : ~0ull;
        unsigned long long k1 = tid + GS_BLOCK < n ? seg[tid + GS_BLOCK] : ~0ull;
        const uint32_t m = (n + 63u) >> 6;  // runs holding keys: 5 .. 8 (uniform)
        k0 = gs_wave_sort64(k0, lane);
        if (wave + 4u < m) k1 = gs_wave_sort64(k1, lane);
        s_key[tid] = k0;
        s_key[tid + GS_BLOCK] = k1;
        __syncthreads();
        uint32_t r0 = lane, r1 = lane;
        for (uint32_t q = 0; q < m; ++q) {  // (8 runs in lockstep for two keys would spill at 64 VGPRs)
          const unsigned long long* run = s_key + 64u * q;
          if (q != wave) r0 += gs_run_below(run, k0);
          if (q != wave + 4u && wave + 4u < m) r1 += gs_run_below(run, k1);
        }
        __syncthreads();
        if (k0 != ~0ull) s_key[r0] = k0;  // (the slots below n hold exactly the keys other than ~0)
        if (k1 != ~0ull) s_key[r1] = k1;
        __syncthreads();
        if (pub)
          for (uint32_t k = tid; k < n; k += GS_BLOCK) {
            const unsigned long long v = s_key[k];
            keys_out[range.x + k] = tbits | (v >> 32);
            vals_out[range.x + k] = (uint32_t)v;
          }
      } else {  // beyond GS_MID without the sort kernel (a frame whose tiles outgrew the previous one's)
        bitonic_flip_sort(n, [&](uint32_t a, uint32_t b) {
          unsigned long long x = seg[a], y = seg[b];
          if (y < x) { seg[a] = y; seg[b] = x; }
        });
        for (uint32_t k = tid; k < n; k += GS_BLOCK) {
          const unsigned long long v = seg[k];
          if (pub) keys_out[range.x + k] = tbits | (v >> 32);
          vals_out[range.x + k] = (uint32_t)v;
        }
        __syncthreads();
      }
    }
    // sorted values (LDS for mid tiles, else vals_out): batch 0's records and batch 1's values in flight
    if (tid < n) {
      const uint32_t g = mid_lds ? (uint32_t)s_key[tid] : vsrc[tid];
      ra = rec[3 * g];
      rb = rec[3 * g + 1];
      rc = rec[3 * g + 2];
    }
    if (tid + GS_BLOCK < n) g_next = mid_lds ? (uint32_t)s_key[tid + GS_BLOCK] : vsrc[tid + GS_BLOCK];
  }
  if (tid == 0) {  // the null record (alpha 0) that pads the per-quadrant lists
    s_stage[GS_BLOCK].a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    s_stage[GS_BLOCK].b = make_float4(0.0f, -__builtin_huge_valf(), 0.0f, 0.0f);
    s_stage[GS_BLOCK].c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }

  const uint32_t px = tile_x * GS_BLOCK_X + (wave & 1u) * 8u + (lane & 7u);
  const uint32_t py = tile_y * GS_BLOCK_Y + (wave >> 1) * 8u + (lane >> 3);
  const bool inside = px < cam.W && py < cam.H;
  // the wave's finished pixels as a lane mask in SGPRs (set: outside the image, saturated, or behind the mesh):
  // the per-entry validity and the every-4-entries all-done test read it without moving it into a VGPR
  unsigned long long done = __builtin_amdgcn_ballot_w64(!inside);
  const float pfx = (float)px, pfy = (float)py;
  const float ux = pfx - tx0, uy = pfy - ty0, uxx = ux * ux, uxy = ux * uy, uyy = uy * uy;
  const float lim = (OVER && inside) ? depth_lim[(size_t)py * cam.W + px] : 0.0f;
  float T = 1.0f;
  float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
  const char* stage = reinterpret_cast<const char*>(s_stage);
  int todo = (int)n;
  STAMP(1, 1);
  for (uint32_t base = 0; todo > 0; base += GS_BLOCK, todo -= GS_BLOCK) {
    // (small tiles: the barrier also publishes the records, masks and sorted slots staged after the
    // sort; large tiles: every wave is done with the previous batch.) The first batch: done = !inside,
    // and every tile holds a pixel inside the image: a plain barrier instead of the counting one, which
    // reduces through LDS behind a second barrier.
    if (base == 0) __syncthreads();
    else if (__syncthreads_count(__builtin_amdgcn_inverse_ballot_w64(done)) == GS_BLOCK) break;
    const uint32_t idx = base + tid;
    if (!small) {
      if (idx < n) {
        s_mask[tid] = (uint8_t)stage_rec(tid, ra, rb, rc, false);  // (large tiles: the box test only)
      }
      // next batch: its records (values loaded a batch ago) and the values of the one after
      if (idx + GS_BLOCK < n) {
        const uint32_t g = g_next;
        ra = rec[3 * g];
        rb = rec[3 * g + 1];
        rc = rec[3 * g + 2];
      }
      if (idx + 2 * GS_BLOCK < n) g_next = vsrc[idx + 2 * GS_BLOCK];
      __syncthreads();  // the batch's records and masks are staged
    }
    // each wave compacts its own quadrant's list from every staged mask, in sorted order (no
    // cross-wave counts: one barrier per batch fewer, two fewer for a small tile)
    const uint32_t nb = min((uint32_t)GS_BLOCK, n - base);
    const uint32_t nbu = (uint32_t)__builtin_amdgcn_readfirstlane((int)nb);
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < GS_BLOCK / 64; ++k) {
      if (k * 64u >= nbu) break;  // (uniform: only the rounds that hold staged entries)
      const uint32_t p = k * 64u + lane;
      const uint32_t slot = small ? (uint32_t)s_sslot[p] : p;
      const bool bit = p < nb && ((s_mask[slot] >> wave) & 1u);
      const unsigned long long bal = __ballot(bit);
      if (bit)
        s_list[wave][cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] =
            slot * (uint32_t)sizeof(GStage);
      cnt += (uint32_t)__popcll(bal);
    }
    if (GS_PROBE(GS_PROBE_NO_EVAL)) cnt = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // wave-uniform trip count; the list is padded with the null Gaussian up to a multiple of 4
    const uint32_t cntu = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt);
    if (lane < 4) s_list[wave][cntu + lane] = GS_BLOCK * (uint32_t)sizeof(GStage);
    const uint32_t* list = s_list[wave];
    for (uint32_t j = 0; j < cntu; j += 4) {
      // (the all-done test every GS_DONE_EVERY entries: scalar, every lane of the wave is active here)
      if ((j & (GS_DONE_EVERY - 1u)) == 0u && done == __builtin_amdgcn_read_exec()) break;
      const uint4 o4 = *reinterpret_cast<const uint4*>(list + j);  // 4 list entries
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t o = u == 0 ? o4.x : u == 1 ? o4.y : u == 2 ? o4.z : o4.w;
        const float4 a = *reinterpret_cast<const float4*>(stage + o);
        const float4 b = *reinterpret_cast<const float4*>(stage + o + 16);
        const float cb = *reinterpret_cast<const float*>(stage + o + 32);
        if (OVER) {  // sorted by depth: the first Gaussian at or behind the mesh ends the pixel
          const float gd = *reinterpret_cast<const float*>(stage + o + 44);
          done |= __builtin_amdgcn_ballot_w64(!(gd < lim));
        }
        // z = A dx^2 + B dx dy + C dy^2 + log2 o as staged: a quadratic in the tile-local (ux, uy), five
        // FMAs (the centre-relative form costs seven; the expansion's rounding is ~1e-6 in z). (The
        // reference's power > 0 skip is not tested: the conic is positive definite (+0.3 low-pass),
        // so power <= 0 up to rounding at power ~ 0.)
        const float z = __builtin_fmaf(a.x, uxx, __builtin_fmaf(a.y, uxy, __builtin_fmaf(a.z, uyy,
                                       __builtin_fmaf(a.w, ux, __builtin_fmaf(b.x, uy, b.y)))));
        // alpha >= 1/255: z >= log2(1/255)
        const bool valid = __builtin_amdgcn_inverse_ballot_w64(__builtin_amdgcn_ballot_w64(z >= -7.9943534f) & ~done);
        const float alpha = valid ? fminf(0.99f, __builtin_amdgcn_exp2f(z)) : 0.0f;
        float wgt = alpha * T;
        float test_T = T - wgt;
        const unsigned long long term = __builtin_amdgcn_ballot_w64(test_T < 0.0001f);  // (only a valid pair)
        if (term) {  // rare: this Gaussian would saturate the pixel -> stop before it
          done |= term;
          const bool t = __builtin_amdgcn_inverse_ballot_w64(term);
          wgt = t ? 0.0f : wgt;
          test_T = t ? T : test_T;
        }
        C0 = __builtin_fmaf(b.z, wgt, C0);
        C1 = __builtin_fmaf(b.w, wgt, C1);
        C2 = __builtin_fmaf(cb, wgt, C2);
        T = test_T;
      }
    }
  }
  STAMP(1, 2);
  if (fu.scap && tid == 0 && n_front) fu.cursor[tile] = 0;  // (n > 0: every wave passed a barrier after reading it)
  if (inside) {
    // the pixel index is recomputed here from a laundered thread id, so that the one computed before
    // the batch loop is not kept (spilled) across it
    uint32_t t2 = tid;
    asm volatile("" : "+v"(t2));
    const uint32_t px2 = tile_x * GS_BLOCK_X + ((t2 >> 6) & 1u) * 8u + (t2 & 7u);
    const uint32_t py2 = tile_y * GS_BLOCK_Y + (t2 >> 7) * 8u + ((t2 & 63u) >> 3);
    const size_t pix = (size_t)py2 * cam.W + px2;
    if (OVER) {
      const float4 u4 = under[pix];
      gs_st4_nt(out + pix, make_float4(C0 + T * u4.x, C1 + T * u4.y, C2 + T * u4.z, (1.0f - T) + T * u4.w));
    } else {
      gs_st4_nt(out + pix, make_float4(C0 + T * bg_r, C1 + T * bg_g, C2 + T * bg_b, 1.0f - T));
    }
  }
  STAMP_SYNC();
  STAMP(1, 3);
}

// Published frame of the fused front end (PTGS_FLAG_SPLAT_PUBLISH, tests): the blend wrote each tile's
// sorted keys / values at t * scap; these two launches compact them into the three-launch layout
// (exclusive scan of the tile counts -> ranges, empty tiles (0, 0)) so both paths publish alike.
// Unpublished fused frames leave ranges[t] = (t * scap, t * scap + n): end - begin is the count.
#define GS_PUB_THREADS 1024
// (a spilled tile's count exceeds its row: only the row's scap keys are copied; a published frame with
// spilled tiles is re-run through the three-launch path by the host)
__global__ __launch_bounds__(GS_PUB_THREADS) void gs_publish_scan_kernel(const uint2* __restrict__ fr, uint32_t ntiles,
                                                                         uint32_t t_begin, uint32_t t_end, uint32_t scap,
                                                                         uint32_t* __restrict__ offs) {
  __shared__ uint32_t s_part[GS_PUB_THREADS / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t per = (ntiles + GS_PUB_THREADS - 1) / GS_PUB_THREADS, a = tid * per, b = min(ntiles, a + per);
  uint32_t sum = 0;
  for (uint32_t t = a; t < b; ++t) sum += (t >= t_begin && t < t_end) ? min(scap, fr[t].y - fr[t].x) : 0u;
  const uint32_t incl = wave_incl_scan(sum);
  if (lane == 63) s_part[wv] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for (uint32_t w = 0; w < wv; ++w) run += s_part[w];
  for (uint32_t t = a; t < b; ++t) {
    offs[t] = run;
    run += (t >= t_begin && t < t_end) ? min(scap, fr[t].y - fr[t].x) : 0u;
  }
}

__global__ __launch_bounds__(256) void gs_publish_copy_kernel(const uint2* __restrict__ fr, const uint32_t* __restrict__ offs,
                                                              uint32_t t_begin, uint32_t t_end, uint32_t scap,
                                                              const unsigned long long* __restrict__ keys_in,
                                                              const uint32_t* __restrict__ vals_in,
                                                              unsigned long long* __restrict__ keys_out,
                                                              uint32_t* __restrict__ vals_out, uint2* __restrict__ ranges) {
  const uint32_t t = blockIdx.x;
  const bool in = t >= t_begin && t < t_end;
  const uint2 r = in ? fr[t] : make_uint2(0u, 0u);
  const uint32_t n = min(scap, r.y - r.x), o = offs[t];
  __syncthreads();  // (ranges may be fr itself: every work-item has read fr[t])
  if (threadIdx.x == 0) ranges[t] = n ? make_uint2(o, o + n) : make_uint2(0u, 0u);
  for (uint32_t k = threadIdx.x; k < n; k += 256) {
    keys_out[o + k] = keys_in[r.x + k];
    vals_out[o + k] = vals_in[r.x + k];
  }
}

hipError_t splat_gaussians(SplatWorkspace* w, const ptgs_gaussians* g, const float* view, const float* mvp, float p00,
                           float p11, uint32_t W, uint32_t H, const float bg[3], const float* depth,
                           const float* under, uint32_t tile_row_begin, uint32_t tile_row_end, float* out,
                           ptgs_splat_stats* stats, bool time_stages, bool publish, bool publish_tight, hipStream_t s,
                           uint32_t* report, const SplatOverlap* ov, SplatSeq* seq) {
  hipError_t e;
  *report = 0;
  if (stats || publish || time_stages) ov = nullptr;  // (these frames are synchronous or instrumented: serial)
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
  cam.rowcull = (cam.row_begin > 0 || cam.row_end < cam.grid_y) ? 1u : 0u;
  cam.cull = (g->chunk_bounds && cam.rowcull) ? 1u : 0u;
  cam.fmax2 = std::max(cam.fx * cam.fx, cam.fy * cam.fy);
  {  // |W|_2^2 <= the largest Gershgorin row sum of W W^T (W: the view's rotation part; 1 for a lookAt view)
    double ww[3][3], w2 = 0.0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        ww[r][c] = (double)view[r] * view[c] + (double)view[4 + r] * view[4 + c] + (double)view[8 + r] * view[8 + c];
    for (int r = 0; r < 3; ++r) w2 = std::max(w2, std::fabs(ww[r][0]) + std::fabs(ww[r][1]) + std::fabs(ww[r][2]));
    cam.w2 = (float)(w2 * (1.0 + 1e-5));
  }
  // stream-ordered frames bin by the alpha box; stats / published frames by the 3-sigma rectangles, unless
  // PTGS_FLAG_SPLAT_PUBLISH_TIGHT asks for the timed frames' binning (parity tests of their integer outputs)
  cam.tight = ((!stats && !publish) || (publish && publish_tight)) ? 1u : 0u;
  const uint32_t tiles = cam.grid_x * cam.grid_y;

  if ((e = ensure(w->means2d, (size_t)n * 8))) return e;
  if ((e = ensure(w->depths, (size_t)n * 4))) return e;
  if ((e = ensure(w->conic, (size_t)n * 16))) return e;
  if ((e = ensure(w->rec, (size_t)n * 48))) return e;
  if ((e = ensure(w->radii, (size_t)n * 4))) return e;
  if ((e = ensure(w->dbg_depths, (size_t)n * 4))) return e;
  if ((e = ensure(w->touched, (size_t)n * 4))) return e;
  if ((e = ensure(w->rect, (size_t)n * 8))) return e;
  if ((e = ensure(w->ranges, (size_t)tiles * 8))) return e;
  // bands of as many tile rows as fit GS_BAND_TILES (1080p: one band, 4K: four) x chunks of >= GS_CHUNK_MIN
  // Gaussians, ~256 blocks in all (at most GS_MAX_CHUNKS chunks)
  if (cam.grid_x > GS_BAND_TILES) return hipErrorInvalidValue;  // W > 131072 px
  BinGrid bgrid;
  bgrid.grid_x = cam.grid_x;
  bgrid.grid_y = cam.grid_y;
  bgrid.tiles = tiles;
  if ((tiles + 63u) / 64u > GS_MAX_GROUPS) return hipErrorInvalidValue;
  bgrid.row0 = cam.row_begin;
  bgrid.row1 = cam.row_end;
  const uint32_t brows = cam.row_end - cam.row_begin;  // the frame's tile rows (the bands cover these)
  bgrid.groups = std::max(1u, (brows * cam.grid_x + 63u) / 64u);
  bgrid.band_rows = std::max(1u, std::min(std::max(brows, 1u), GS_BAND_TILES / cam.grid_x));
  bgrid.bands = std::max(1u, (brows + bgrid.band_rows - 1) / bgrid.band_rows);
  // Chunks: the count / scatter walks are latency-bound loops over a chunk's Gaussians, while every chunk
  // writes (count), scans (colscan) and reads (scatter) a histogram row of its band's tiles. So 256
  // workgroups in all as long as the rows cost about as much as the walks; beyond that (at least twice
  // as many Gaussians per chunk as band tiles: 10M at 4K, a single-band tile-row shard of it) up to
  // GS_MAX_CHUNKS (10M at 4K: front end 4.3 -> 2.9 ms; 1M at 1080p with 1 024 chunks: 0.289 -> 0.330 ms).
  const uint32_t band_tiles = bgrid.band_rows * cam.grid_x;
  const uint32_t want_chunks = std::max(256u / bgrid.bands, (uint32_t)std::min<uint64_t>(GS_MAX_CHUNKS, n / std::max(1u, band_tiles / 2u)));
  bgrid.chunks = std::max(1u, std::min({(uint32_t)GS_MAX_CHUNKS / bgrid.bands, (n + GS_CHUNK_MIN - 1) / GS_CHUNK_MIN,
                                        want_chunks}));
  bgrid.chunk = std::max(1u, (n + bgrid.chunks - 1) / bgrid.chunks);
  const size_t band_lds = (size_t)bgrid.band_rows * cam.grid_x * 4;
  if ((e = ensure(w->hist, (size_t)bgrid.chunks * tiles * 4))) return e;
  if ((e = ensure(w->nzbuf, (size_t)bgrid.chunks * bgrid.bands * 4))) return e;
  if ((e = ensure(w->tile_slots, (size_t)tiles * GS_TILE_SLOTS * 8))) return e;
  if ((e = ensure(w->tile_info, (size_t)tiles * 8))) return e;
  if ((e = ensure(w->group_total, (size_t)bgrid.groups * 4))) return e;
  if ((e = ensure(w->large, (size_t)tiles * 4))) return e;
  if (!w->large_ctr.p) {
    if ((e = ensure(w->large_ctr, 16))) return e;
    if ((e = hipMemset(w->large_ctr.p, 0, 16))) return e;
  }
  if (!w->total.p) {  // [0] = K (scatter), [1] = largest tile (colscan's atomicMax; count re-arms it)
    if ((e = ensure(w->total, 16))) return e;
    if ((e = hipMemset(w->total.p, 0, 16))) return e;
  }
  if (!w->k_host) {
    if ((e = hipHostMalloc((void**)&w->k_host, 64, hipHostMallocCoherent | hipHostMallocMapped))) return e;
    std::memset(w->k_host, 0, 64);
    if ((e = hipHostGetDevicePointer((void**)&w->k_dev, w->k_host, 0))) return e;
  }
  if (!w->fz.p) {  // device counters of both front ends, the blend and the spill pool (zero once)
    if ((e = ensure(w->fz, 256))) return e;
    if ((e = hipMemsetAsync(w->fz.p, 0, 256, s))) return e;
  }
  // An earlier frame of this workspace left a spilled tile incomplete (pool exhausted; k_host[9], a
  // device store seen once that frame has run) or met an id >= N (k_host[10]): reported by this call,
  // which renders its own frame after growing the pool (splat_common maps it to PTGS_EINCOMPLETE /
  // PTGS_EINVAL). A call with stats waits for the earlier frames first (it is synchronous anyway), so
  // their reports are its own and the flags its superseded runs may raise can be dropped below.
  if (stats && (e = hipStreamSynchronize(s))) return e;
  if (__atomic_exchange_n(w->k_host + 9, 0u, __ATOMIC_ACQ_REL)) {
    ++w->incomplete;
    *report |= 1u;
  }
  if (__atomic_exchange_n(w->k_host + 10, 0u, __ATOMIC_ACQ_REL)) *report |= 2u;
  // Spill pool: at least max(2^20, N) pairs, the reservation, and 1.25x the demand of the latest
  // frame whose front end has run (k_host[8]; a hint, no wait). Growth frees the old pool (waits).
  {
    const uint32_t demand = w->k_host[8];
    uint64_t want = std::max<uint64_t>(std::max<uint64_t>(1u << 20, n), w->sp_cap);
    if (demand > w->sp_cap) want = std::max<uint64_t>(want, (uint64_t)demand + demand / 4u);
    // a reported frame's own demand reaches k_host[8] only with the NEXT front end: its spilled
    // tiles hold at most its pair count, which is at most the largest K any frame of the workspace has
    // published (k_host[12] fused, [13] three launches: device-side running maxima, so a later lighter frame
    // cannot hide it), so the pool grows to that now and this frame cannot exhaust it the same way
    if (*report & 1u) {
      const uint32_t k = std::max({w->k_host[0], w->k_host[12], w->k_host[13]});
      want = std::max<uint64_t>(want, (uint64_t)k + k / 4u);
    }
    want = std::min<uint64_t>(want, 0xFFFFFFF0u);
    if (want > w->sp_cap || !w->sp_keys.p) {
      if ((e = ensure(w->sp_keys, want * 8)) || (e = ensure(w->sp_vals, want * 4))) return e;
      w->sp_cap = (uint32_t)std::min<size_t>(std::min(w->sp_keys.bytes / 8, w->sp_vals.bytes / 4), 0xFFFFFFF0u);
    }
  }
#ifndef GS_K_EVENT_FLAGS
#define GS_K_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
  // the K event only signals the host (stats requested): k_host is fine-grained (coherent) memory the
  // GPU writes past its caches, so the event needs no system-scope cache release
  if (!w->k_event && (e = hipEventCreateWithFlags(&w->k_event, GS_K_EVENT_FLAGS))) return e;
  // Pair capacity. The call is stream-ordered: scatter and blend are enqueued against the current
  // pair buffer and do nothing when the frame's K exceeds it (the device compares). The buffer starts
  // at 8 pairs per Gaussian and grows from the K that earlier frames' scatters wrote to pinned host
  // memory (k_host, read here without waiting: a hint); with stats requested the call waits for this
  // frame's K and re-runs scatter + blend after growing, so that frame is always complete.
  if (w->pairs.bytes < (size_t)n * 64) {
    if ((e = ensure(w->pairs, (size_t)n * 64))) return e;
    if ((e = ensure(w->vals_out, (size_t)n * 32))) return e;
  }
  if (publish && (e = ensure(w->keys_out, w->pairs.bytes))) return e;
  auto cap_now = [&]() -> uint32_t {
    size_t c = std::min(w->pairs.bytes / 8, w->vals_out.bytes / 4);
    if (publish) c = std::min(c, w->keys_out.bytes / 8);
    return (uint32_t)std::min<size_t>(c, 0xFFFFFFFFu);
  };
  auto grow = [&](uint32_t K) -> hipError_t {  // (hipFree waits for the frames that use the old buffers)
    hipError_t e2;
    if ((e2 = ensure(w->pairs, (size_t)K * 8))) return e2;
    if ((e2 = ensure(w->vals_out, (size_t)K * 4))) return e2;
    if (publish && (e2 = ensure(w->keys_out, (size_t)K * 8))) return e2;
    return hipSuccess;
  };
  if (w->k_host[0] > cap_now() && (e = grow(w->k_host[0]))) return e;

  const uint32_t slot_keys = n < (1u << 24) ? 1u : 0u;  // the register sort packs the gaussian in 24 bits
  PreArgs pa;
  pa.means = g->means;
  pa.scales = g->scales;
  pa.rots = g->rotations;
  pa.opac = g->opacities;
  pa.colors = g->colors;
  pa.n = n;
  pa.means2d = (float2*)w->means2d.p;
  pa.depths = (float*)w->depths.p;
  pa.conic_o = (float4*)w->conic.p;
  pa.radii = (int*)w->radii.p;
  pa.touched = (uint32_t*)w->touched.p;
  pa.rects = (ushort4*)w->rect.p;
  pa.rec = (float4*)w->rec.p;
  pa.ids = g->ids;
  pa.dbg_depths = (float*)w->dbg_depths.p;
  pa.bad_ids = w->k_dev + 10;
  // chunks whose bound misses the rows are skipped by the front end before their loads: the fused
  // kernel tests its own chunk's bound; the three-launch count reads flags of a small launch before it
  pa.cskip = nullptr;
  pa.cbounds = cam.cull ? (const float4*)g->chunk_bounds : nullptr;
  if (cam.cull) {
    const uint32_t nch = (n + 255u) / 256u;
    if ((e = ensure(w->cskip, nch))) return e;
    pa.cskip = (const uint8_t*)w->cskip.p;
  }
  auto cull_flags = [&](hipStream_t cs) -> hipError_t {
    if (!cam.cull) return hipSuccess;
    const uint32_t nch = (n + 255u) / 256u;
    hipLaunchKernelGGL(gs_chunk_cull_kernel, dim3((nch + 255u) / 256u), dim3(256), 0, cs, cam,
                       (const float4*)g->chunk_bounds, nch, (uint8_t*)w->cskip.p);
    return hipGetLastError();
  };
  if (!publish) {  // the per-Gaussian debug outputs only for a published frame (ptgs_splat_get_buffers)
    pa.radii = nullptr;
    pa.touched = nullptr;
    pa.means2d = nullptr;
    pa.conic_o = nullptr;
    pa.dbg_depths = nullptr;
  }
  // Front end: the fused single launch (gs_bin_fused_kernel) once an earlier frame of this workspace
  // has published its largest tile (the rows' capacity scap follows it with 1/4 headroom, a power of
  // two in [256, GS_FUSED_MAX_SCAP]); otherwise, or above that capacity, count + colscan + scatter.
#ifndef GS_FUSED_MAX_SCAP
#define GS_FUSED_MAX_SCAP 2048u  // larger tiles (1M Gaussians at 1080p): three launches measured faster
#endif
#ifndef GS_FUSED_RUNS_PER_TILE
#define GS_FUSED_RUNS_PER_TILE 32u  // (C2 Morton order: 6; random order: 51; orbit views up to ~20, where
                                    // fused measured 0.13 vs 0.24 ms for three launches)
#endif
  // policy (PTGS_GS_FRONTEND unset): the fused path while frames touch at most
  // GS_FUSED_RUNS_PER_TILE (workgroup, tile) runs per tile (Gaussians in a spatially coherent order:
  // each workgroup touches a compact set of tiles; in random order every workgroup touches most tiles
  // and the reservations cost more than the histograms), else three launches
  static const int frontend = [] {
    const char* v = getenv("PTGS_GS_FRONTEND");  // "fused" / "three" (A/B switch)
    if (v && !strcmp(v, "three")) return 0;
    if (v && !strcmp(v, "fused")) return 1;
    return 2;
  }();
  // both front ends publish the frame's touched (workgroup, tile) runs (k_host[4]: the fused kernel's
  // reservations, the count kernel's nonzero histogram entries); the latest one decides, so the
  // choice is made from the first finished frame on and follows the data's coherence both ways
  const bool want_fused = frontend == 1 || (frontend == 2 && w->k_host[4] <= GS_FUSED_RUNS_PER_TILE * tiles);
  uint32_t scap = 0;
  if (want_fused && w->have_hint && n) {
    const uint32_t big = std::max(256u, w->k_host[1] + w->k_host[1] / 4u);
    uint32_t c = 256;
    while (c < big && c < GS_FUSED_MAX_SCAP) c <<= 1;
    if (big <= GS_FUSED_MAX_SCAP && (size_t)tiles * c * 8 <= ((size_t)4 << 30)) scap = c;
  }
  const uint32_t rows = cam.row_end - cam.row_begin;
  // per front-end workgroup chunk rects (gs_spill_tile): fused (bands x 256-Gaussian chunks) or count
  const uint32_t nwg_fused = bgrid.bands * ((n + GS_FUSED_THREADS - 1) / GS_FUSED_THREADS);
  if ((e = ensure(w->crect, (size_t)std::max(nwg_fused, bgrid.bands * bgrid.chunks) * 8))) return e;
  auto spill_args = [&](bool fused_fe) -> GsSpill {
    GsSpill sp;
    sp.fz = (uint32_t*)w->fz.p;
    sp.k_host = w->k_dev;
    sp.keys = (unsigned long long*)w->sp_keys.p;
    sp.vals = (uint32_t*)w->sp_vals.p;
    sp.cap = w->sp_cap;
    sp.crect = (const ushort4*)w->crect.p;
    sp.bands = bgrid.bands;
    sp.chunk = fused_fe ? GS_FUSED_THREADS : bgrid.chunk;
    sp.nwg = fused_fe ? nwg_fused : bgrid.bands * bgrid.chunks;
    sp.n = n;
    sp.rects = (const ushort4*)w->rect.p;
    sp.depths = (const float*)w->depths.p;
    sp.ids = g->ids;
    return sp;
  };
  auto blend = [&](uint32_t cap, const GsFused& fu, unsigned long long* keys_out, bool sort_large) -> hipError_t {
    if (rows == 0) return hipSuccess;
    auto k = depth ? gs_sort_blend_kernel<true> : gs_sort_blend_kernel<false>;
    const dim3 grid(cam.grid_x, rows);
    hipLaunchKernelGGL(k, grid, dim3(GS_BLOCK), 0, s, cam, (const uint2*)w->ranges.p, (unsigned long long*)w->pairs.p,
                       sort_large ? (uint32_t)GS_MID : 0xFFFFFFFFu, keys_out, (uint32_t*)w->vals_out.p,
                       (const float4*)w->rec.p, bg[0], bg[1], bg[2], cap, slot_keys,
                       (const unsigned long long*)w->tile_slots.p, depth, (const float4*)under, (float4*)out, fu,
                       spill_args(fu.scap != 0));
    const hipError_t le = hipGetLastError();
    if (!le && seq && fu.seq_flag) seq->launched = true;
    return le;
  };
  auto sort_attr = [&]() -> hipError_t {
    if (w->sort_attr) return hipSuccess;
    hipError_t e2 = hipFuncSetAttribute((const void*)gs_sort_large_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)gs_radix_lds(GS_RADIX_MAXR));
    if (!e2) w->sort_attr = true;
    return e2;
  };
  // the blend's tile order (heaviest tiles of the previous frame first), built by the front end's
  // first launch
  uint32_t* order = nullptr;
  if (rows) {
    if ((e = ensure(w->order, (size_t)tiles * 4))) return e;
    order = (uint32_t*)w->order.p;
  }
  const GsFused no_fu = {0u, nullptr, nullptr, nullptr, nullptr, nullptr, 0u, order, nullptr, 0u,
                         seq ? seq->flag : nullptr, seq ? seq->ordinal : 0ull};

  auto enqueue_fused = [&]() -> hipError_t {
    hipError_t e2;
    if ((e2 = ensure(w->tile_slots, (size_t)tiles * scap * 8))) return e2;
    if ((e2 = ensure(w->vals_out, (size_t)tiles * scap * 4))) return e2;
    if (publish && (e2 = ensure(w->keys_out, (size_t)tiles * scap * 8))) return e2;
    // the front end's stream: the caller's, or (overlapped frame) the second stream once ov->wait is done
    const hipStream_t sf = ov ? ov->fe : s;
    if (ov && ov->wait && (e2 = hipStreamWaitEvent(sf, ov->wait, 0))) return e2;
    // (or the workspace's reuse from the blend ordinals, SplatSeq: a wait packet on the front end's queue,
    // which holds no workgroup slots while it waits and puts nothing on the caller's queue)
    if (ov && ov->wait_flag &&
        (e2 = hipStreamWaitValue64(sf, (void*)ov->wait_flag, ov->wait_ordinal, hipStreamWaitValueGte, ~0ull)))
      return e2;
    if (w->cursor.bytes < (size_t)tiles * 4) {  // zero between frames (the blend re-arms what it reads)
      if ((e2 = ensure(w->cursor, (size_t)tiles * 4))) return e2;
      if ((e2 = hipMemsetAsync(w->cursor.p, 0, w->cursor.bytes, sf))) return e2;
    }
    // helper workgroups only when the latest fused frame queued slices (k_host[11]: a static view whose
    // chunks all fit one slice launches none; the owners walk any slice no helper takes, so a frame
    // that queues more than the helpers take is complete anyway). Idle helpers polled the queue until
    // every owner had published, and their last poll (~3 us sleep) could end the kernel late.
    static const int helpers_env = [] {
      const char* v = getenv("PTGS_GS_HELPERS");  // "always" (A/B switch)
      return v && !strcmp(v, "always") ? 1 : 0;
    }();
    const uint32_t queued = w->k_host[11];
    const uint32_t helpers = helpers_env ? GS_FUSED_HELPERS
                             : queued ? std::min<uint32_t>(GS_FUSED_HELPERS, queued + queued / 2u + 8u) : 0u;
    // owners (bands x chunks) and helpers (bands x helpers) each publish their partials
    const uint32_t nwg = nwg_fused + bgrid.bands * helpers;
    if ((e2 = ensure(w->fzp, (size_t)nwg * 8))) return e2;
    // slice queue: room for twice the slices of the largest pair count seen (+ one per owner); zero
    // once here, re-armed by the blend after every frame
    const uint32_t qcap = std::max<uint32_t>(4096u, 2u * (w->k_host[0] / GsFusedShape<256>::slice) + nwg_fused);
    if (w->fsq.bytes < (size_t)qcap * 8) {
      if ((e2 = ensure(w->fsq, (size_t)qcap * 8))) return e2;
      if ((e2 = hipMemsetAsync(w->fsq.p, 0, w->fsq.bytes, sf))) return e2;
    }
    const uint32_t fsq_cap = (uint32_t)std::min<size_t>(w->fsq.bytes / 8, 0x7FFFFFFFu);
    GsFused fu = {scap, (uint32_t*)w->cursor.p, (uint32_t*)w->fz.p, w->k_dev, (uint2*)w->ranges.p,
                  (uint32_t*)w->fzp.p, nwg, order, (uint2*)w->fsq.p, fsq_cap, seq ? seq->flag : nullptr,
                  seq ? seq->ordinal : 0ull};
    PreArgs fpa = pa;  // the fused walk keeps rects / depths in registers (band 0 stores them for gs_spill_tile)
    if (cam.cull && (n + 255u) / 256u > GS_FUSED_OWN_CULL) {
      if ((e2 = cull_flags(sf))) return e2;
      fpa.cbounds = nullptr;
    }
    fpa.rects = nullptr;
    fpa.depths = nullptr;
    BinGrid fg = bgrid;
    fg.chunks = (n + GS_FUSED_THREADS - 1) / GS_FUSED_THREADS;
    fg.chunk = GS_FUSED_THREADS;
    // the tile order: the front end's extra workgroup from the previous frame's counts, or (overlapped,
    // own_order) a launch behind the front end from this frame's own counts
    const bool own_order = order && ov && ov->own_order;
    uint32_t* fe_order = own_order ? nullptr : order;
    // the workgroup shape (GsFusedShape: 256 work-items beside another frame's blend, else 512; PTGS_GS_FE_WG
    // overrides: A/B switch) and its histogram window (entries; 0: the whole band; at least the order's buckets)
    static const int wg_env = [] {
      const char* v = getenv("PTGS_GS_FE_WG");
      return v ? atoi(v) : 0;
    }();
    const uint32_t fwg = wg_env == 256 || wg_env == 512 ? (uint32_t)wg_env : ov ? (uint32_t)GS_FUSED_WG_OV : (uint32_t)GS_FUSED_WG;
    const uint32_t cap = fwg == 256 ? GsFusedShape<256>::lds_cap : GsFusedShape<512>::lds_cap;
    const size_t fe_lds = std::max<size_t>(cap ? std::min<size_t>(band_lds, (size_t)cap * 4u) : band_lds,
                                           (size_t)GS_ORDER_BUCKETS * 4u);
    auto fk = fwg == 256 ? (cam.rowcull ? gs_bin_fused_kernel<true, 256> : gs_bin_fused_kernel<false, 256>)
                         : (cam.rowcull ? gs_bin_fused_kernel<true, 512> : gs_bin_fused_kernel<false, 512>);
    hipLaunchKernelGGL(fk, dim3(fg.bands, fg.chunks + helpers + (fe_order ? 1u : 0u)), dim3(fwg), fe_lds, sf,
                       cam, fpa, fg, scap, (uint32_t*)w->cursor.p, (uint32_t*)w->fz.p, (uint32_t*)w->fzp.p,
                       (unsigned long long*)w->tile_slots.p, (const uint2*)w->ranges.p, fe_order,
                       cam.row_begin * cam.grid_x, cam.row_end * cam.grid_x, (ushort4*)w->crect.p, (ushort4*)w->rect.p,
                       (float*)w->depths.p, w->k_dev, (uint2*)w->fsq.p, fsq_cap, (uint32_t)(fe_lds / 4u));
    if ((e2 = hipGetLastError())) return e2;
    if (own_order) {
      hipLaunchKernelGGL(gs_tile_order_kernel, dim3(1), dim3(GS_ORDER_THREADS), 0, sf, (const uint32_t*)w->cursor.p,
                         order, cam.row_begin * cam.grid_x, cam.row_end * cam.grid_x);
      if ((e2 = hipGetLastError())) return e2;
    }
    if (ov && ((e2 = hipEventRecord(ov->done, sf)) || (e2 = hipStreamWaitEvent(s, ov->done, 0)))) return e2;
    if ((e2 = mark(1)) || (e2 = mark(2)) || (e2 = mark(3))) return e2;
    unsigned long long* keys_out = publish ? (unsigned long long*)w->keys_out.p : nullptr;
    const bool sort_large = w->k_host[1] > GS_MID;
    if (sort_large) {
      if ((e2 = sort_attr())) return e2;
      const uint32_t grid = std::max(w->sort_grid, (tiles + GS_SORT_THREADS - 1) / GS_SORT_THREADS);
      hipLaunchKernelGGL(gs_sort_large_kernel, dim3(grid), dim3(GS_SORT_THREADS), gs_radix_lds(w->sort_r), s,
                         (const uint2*)w->ranges.p, (unsigned long long*)w->pairs.p,
                         (const unsigned long long*)w->tile_slots.p, (const uint32_t*)w->large.p,
                         (const uint32_t*)w->large_ctr.p, keys_out, (uint32_t*)w->vals_out.p,
                         (const uint32_t*)w->total.p, 0u, w->sort_r, (uint32_t*)nullptr, (uint16_t*)nullptr, 0u, fu, tiles);
      if ((e2 = hipGetLastError())) return e2;
    }
    if ((e2 = mark(4)) || (e2 = mark(5))) return e2;
    if ((e2 = blend(0u, fu, keys_out, sort_large))) return e2;
    if (publish) {  // compact the published rows into the three-launch layout (tests only)
      if ((e2 = ensure(w->pub_offs, (size_t)tiles * 4))) return e2;
      if ((e2 = ensure(w->keys_pub, (size_t)tiles * scap * 8))) return e2;  // (K <= tiles * scap)
      if ((e2 = ensure(w->vals_pub, (size_t)tiles * scap * 4))) return e2;
      const uint32_t tb = cam.row_begin * cam.grid_x, te = cam.row_end * cam.grid_x;
      hipLaunchKernelGGL(gs_publish_scan_kernel, dim3(1), dim3(GS_PUB_THREADS), 0, s, (const uint2*)w->ranges.p, tiles,
                         tb, te, scap, (uint32_t*)w->pub_offs.p);
      hipLaunchKernelGGL(gs_publish_copy_kernel, dim3(tiles), dim3(256), 0, s, (const uint2*)w->ranges.p,
                         (const uint32_t*)w->pub_offs.p, tb, te, scap, (const unsigned long long*)w->keys_out.p,
                         (const uint32_t*)w->vals_out.p, (unsigned long long*)w->keys_pub.p, (uint32_t*)w->vals_pub.p,
                         (uint2*)w->ranges.p);
      if ((e2 = hipGetLastError())) return e2;
    }
    if (stats && (e2 = hipEventRecord(w->k_event, s))) return e2;  // K is on the host after the blend
    return mark(6);
  };

  auto enqueue_tail = [&](uint32_t cap) -> hipError_t {
    // (read here, not before: grow() may have moved the published-keys buffer since the last call)
    unsigned long long* keys_out = publish ? (unsigned long long*)w->keys_out.p : nullptr;
    hipLaunchKernelGGL(gs_bin_scatter_kernel, dim3(bgrid.bands, bgrid.chunks), dim3(GS_BIN_THREADS),
                       2 * band_lds + (size_t)bgrid.groups * 4, s, bgrid, (const ushort4*)w->rect.p,
                       (const float*)w->depths.p, g->ids, n, (const uint32_t*)w->hist.p, (const uint2*)w->tile_info.p,
                       (const uint32_t*)w->group_total.p, (uint32_t*)w->total.p, (const uint32_t*)w->large_ctr.p, w->k_dev,
                       (const uint32_t*)w->nzbuf.p, bgrid.bands * bgrid.chunks, cap,
                       (uint2*)w->ranges.p, (unsigned long long*)w->pairs.p, (unsigned long long*)w->tile_slots.p);
    hipError_t e2 = hipGetLastError();
    if (e2) return e2;
    if (stats && (e2 = hipEventRecord(w->k_event, s))) return e2;  // K is on the host after the scatter
    if ((e2 = mark(3))) return e2;
    // tiles above GS_MID pairs: sorted by gs_sort_large_kernel when the previous frame had any (else
    // the blend sorts the rare one itself)
    const bool sort_large = w->k_host[1] > GS_MID;
    if (sort_large) {
      if ((e2 = sort_attr())) return e2;
      // tiles beyond the LDS capacity sort in a global scratch ([2][g_cap] u32 + [2][g_cap] u16 at the
      // pair offsets), allocated once a frame has had such tiles
      uint32_t g_cap = 0;
      if (w->k_host[1] > GS_SORT_THREADS * GS_RADIX_MAXR) {
        if ((e2 = ensure(w->sort_scratch, (size_t)cap * 12u))) return e2;
        g_cap = (uint32_t)std::min<size_t>(w->sort_scratch.bytes / 12u, 0xFFFFFFFFu);
      }
      uint32_t* g_dep = g_cap ? (uint32_t*)w->sort_scratch.p : nullptr;
      uint16_t* g_slot = g_cap ? (uint16_t*)(g_dep + 2 * (size_t)g_cap) : nullptr;
      hipLaunchKernelGGL(gs_sort_large_kernel, dim3(w->sort_grid), dim3(GS_SORT_THREADS), gs_radix_lds(w->sort_r), s,
                         (const uint2*)w->ranges.p, (unsigned long long*)w->pairs.p,
                         (const unsigned long long*)w->tile_slots.p, (const uint32_t*)w->large.p,
                         (const uint32_t*)w->large_ctr.p, keys_out, (uint32_t*)w->vals_out.p,
                         (const uint32_t*)w->total.p, cap, w->sort_r, g_dep, g_slot, g_cap, no_fu, tiles);
      if ((e2 = hipGetLastError())) return e2;
    }
    if ((e2 = mark(4)) || (e2 = mark(5))) return e2;
    if ((e2 = blend(cap, no_fu, keys_out, sort_large))) return e2;
    return mark(6);
  };
  auto enqueue_three = [&]() -> hipError_t {
    hipError_t e2;
    if ((e2 = ensure(w->tile_slots, (size_t)tiles * GS_TILE_SLOTS * 8))) return e2;
    if ((e2 = cull_flags(s))) return e2;
    // (n == 0: one chunk of nothing; the count still zeroes the histograms and the colscan publishes K = 0)
    hipLaunchKernelGGL(cam.rowcull ? gs_bin_count_kernel<true> : gs_bin_count_kernel<false>,
                       dim3(bgrid.bands, bgrid.chunks + (order ? 1u : 0u)), dim3(GS_COUNT_THREADS),
                       std::max(band_lds, (size_t)GS_ORDER_BUCKETS * 4), s, cam, pa, bgrid, (uint32_t*)w->hist.p,
                       (uint32_t*)w->total.p, (uint32_t*)w->large_ctr.p, w->k_dev, (uint32_t*)w->nzbuf.p,
                       (const uint2*)w->ranges.p, order, cam.row_begin * cam.grid_x, cam.row_end * cam.grid_x,
                       (uint32_t*)w->fz.p, (ushort4*)w->crect.p);
    if ((e2 = hipGetLastError())) return e2;
    if ((e2 = mark(1))) return e2;
    hipLaunchKernelGGL(gs_bin_colscan_kernel, dim3(bgrid.groups), dim3(GS_COLSCAN_THREADS), 0, s, bgrid, (uint32_t*)w->hist.p,
                       (uint2*)w->tile_info.p, (uint32_t*)w->group_total.p, (uint32_t*)w->total.p, (uint32_t)GS_MID,
                       (uint32_t*)w->large.p, (uint32_t*)w->large_ctr.p);
    if ((e2 = hipGetLastError())) return e2;
    if ((e2 = mark(2))) return e2;
    return enqueue_tail(cap_now());
  };

  if ((e = mark(0))) return e;
  const bool fused = scap != 0;
  if ((e = fused ? enqueue_fused() : enqueue_three())) return e;
  uint32_t K = w->k_host[0];  // without stats: the latest K any frame published (a hint)
  bool redone = false;
  if (stats) {
    if ((e = hipEventSynchronize(w->k_event))) return e;
    K = w->k_host[0];
    // a fused frame with a tile above its row capacity, or a three-launch frame above the pair
    // buffer, was completed through the spill pool; a call with stats re-runs it so that its published
    // keys / values / ranges are the exact layout (three launches, grown buffers)
    if (fused && w->k_host[5]) {
      redone = true;
      if ((e = mark(0)) || (e = enqueue_three())) return e;
      if ((e = hipEventSynchronize(w->k_event))) return e;
      K = w->k_host[0];
    }
    bool regrown = false;
    if ((!fused || redone) && K > cap_now()) {
      if ((e = grow(K))) return e;
      if ((e = mark(2))) return e;
      if ((e = enqueue_tail(cap_now()))) return e;
      regrown = true;
    }
    if (redone || regrown) {  // the superseded run's spilled tiles may have exhausted the pool: the
                              // re-run completed the frame, so its report is dropped
      if ((e = hipStreamSynchronize(s))) return e;
      __atomic_store_n(w->k_host + 9, 0u, __ATOMIC_RELEASE);
    }
    stats->num_rendered = K;
    stats->tiles_x = cam.grid_x;
    stats->tiles_y = cam.grid_y;
    stats->num_visible = 0;
    stats->fused = fused && !redone ? 1u : 0u;
  }
  w->last_fused = fused && !redone;
  w->last_scap = w->last_fused ? scap : 0u;
  // the fused path sizes its rows from the largest tile of a finished frame: valid once the host has
  // seen one complete (a frame still in flight has not written its hint yet)
  if (!w->have_hint) {
    if (!w->hint_event && (e = hipEventCreateWithFlags(&w->hint_event, hipEventDisableTiming))) return e;
    if (w->hint_recorded && hipEventQuery(w->hint_event) == hipSuccess) w->have_hint = true;
    if (!w->hint_recorded || stats) {
      if ((e = hipEventRecord(w->hint_event, s))) return e;
      w->hint_recorded = true;
    }
    if (stats) w->have_hint = true;  // (waited for above)
  }
  {  // the next frame's large-tile sort: LDS capacity from the largest tile of a recent frame
     // (k_host[1]; +1/8 headroom), workgroups from its large-tile count (k_host[2]); hints only
    const uint32_t big = w->k_host[1] + w->k_host[1] / 8u;
    w->sort_r = std::min((uint32_t)GS_RADIX_MAXR, ((big + GS_SORT_THREADS - 1) / GS_SORT_THREADS) | 1u);
    w->sort_grid = std::max(64u, std::min(4096u, w->k_host[2] + w->k_host[2] / 4u));
  }
  w->last_n = n;
  w->last_k = K;
  w->last_tiles = tiles;
  w->last_published = publish && stats;
  return hipSuccess;
}

// ---- spatial order (ptgs_gaussians_sort_spatial) ---------------------------------------------------
__device__ __forceinline__ uint32_t gs_f2ord(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float gs_ord2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }
__device__ __forceinline__ uint32_t gs_spread3(uint32_t v) {  // 10 bits -> every 3rd bit
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ __launch_bounds__(256) void gs_means_bounds_kernel(const float* __restrict__ means, uint32_t n,
                                                              uint32_t* __restrict__ b) {  // b: lo[3], hi[3]
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (i < n)
    for (int a = 0; a < 3; ++a) lo[a] = hi[a] = means[3 * i + a];
  for (int off = 32; off > 0; off >>= 1)
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
    }
  if ((threadIdx.x & 63u) == 0)
    for (int a = 0; a < 3; ++a) {
      atomicMin(b + a, gs_f2ord(lo[a]));
      atomicMax(b + 3 + a, gs_f2ord(hi[a]));
    }
}

__global__ __launch_bounds__(256) void gs_means_morton_kernel(const float* __restrict__ means, uint32_t n,
                                                              const uint32_t* __restrict__ b,
                                                              unsigned long long* __restrict__ keys) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint32_t q[3];
  for (int a = 0; a < 3; ++a) {
    const float lo = gs_ord2f(b[a]), ext = gs_ord2f(b[3 + a]) - lo;
    const float u = ext > 0.0f ? (means[3 * i + a] - lo) / ext : 0.0f;
    q[a] = (uint32_t)fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
  }
  const uint32_t code = (gs_spread3(q[0]) << 2) | (gs_spread3(q[1]) << 1) | gs_spread3(q[2]);
  keys[i] = ((unsigned long long)code << 32) | i;
}

__global__ __launch_bounds__(256) void gs_gather_sorted_kernel(const unsigned long long* __restrict__ keys, uint32_t n,
                                                               ptgs_gaussians g, float* __restrict__ means,
                                                               float* __restrict__ scales, float* __restrict__ rots,
                                                               float* __restrict__ opac, float* __restrict__ colors,
                                                               uint32_t* __restrict__ ids) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = (uint32_t)keys[i];
  for (int a = 0; a < 3; ++a) {
    means[3 * i + a] = g.means[3 * j + a];
    scales[3 * i + a] = g.scales[3 * j + a];
    colors[3 * i + a] = g.colors[3 * j + a];
  }
  for (int a = 0; a < 4; ++a) rots[4 * i + a] = g.rotations[4 * j + a];
  opac[i] = g.opacities[j];
  ids[i] = g.ids ? g.ids[j] : j;
}

hipError_t splat_sort_spatial(const ptgs_gaussians* g, float* means, float* scales, float* rots, float* opac,
                              float* colors, uint32_t* ids, hipStream_t s) {
  const uint32_t n = g->count;
  if (n == 0) return hipSuccess;
  hipError_t e;
  uint32_t* b = nullptr;
  unsigned long long *k0 = nullptr, *k1 = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
  const dim3 grid((n + 255) / 256);
  auto done = [&](hipError_t r) {
    (void)hipStreamSynchronize(s);
    if (b) (void)hipFree(b);
    if (k0) (void)hipFree(k0);
    if (k1) (void)hipFree(k1);
    if (tmp) (void)hipFree(tmp);
    return r;
  };
  if ((e = hipMalloc(&b, 32)) || (e = hipMalloc(&k0, (size_t)n * 8)) || (e = hipMalloc(&k1, (size_t)n * 8))) return done(e);
  if ((e = hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, k0, k1, (int)n, 0, 62, s))) return done(e);
  if ((e = hipMalloc(&tmp, tmp_bytes))) return done(e);
  if ((e = hipMemcpyAsync(b, init, sizeof(init), hipMemcpyHostToDevice, s))) return done(e);
  hipLaunchKernelGGL(gs_means_bounds_kernel, grid, dim3(256), 0, s, g->means, n, b);
  hipLaunchKernelGGL(gs_means_morton_kernel, grid, dim3(256), 0, s, g->means, n, (const uint32_t*)b, k0);
  if ((e = hipGetLastError())) return done(e);
  if ((e = hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, k0, k1, (int)n, 0, 62, s))) return done(e);
  hipLaunchKernelGGL(gs_gather_sorted_kernel, grid, dim3(256), 0, s, (const unsigned long long*)k1, n, *g, means, scales,
                     rots, opac, colors, ids);
  return done(hipGetLastError());
}

// pairs: the pair buffer (three launches: a frame of K <= pairs stores every pair) and the spill pool
// (fused rows: a frame's spilled tiles hold at most K pairs) — a frame of at most `pairs` pairs is always
// rendered completely, whichever front end runs and whatever its row capacity (hipGraph replays too)
// ---- chunk bounds (ptgs_gaussians_chunk_bounds) -----------------------------------------------------
// chunk c = Gaussians [256 c, 256 c + 256): (min x, min y, min z, max |scale|), (max x, max y, max z, 0)
__global__ __launch_bounds__(256) void gs_chunk_bounds_kernel(const float* __restrict__ means,
                                                              const float* __restrict__ scales, uint32_t n,
                                                              float4* __restrict__ out) {
  __shared__ float s_b[7][4];
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  float b[7] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY, 0.0f};
  if (i < n) {
    for (int a = 0; a < 3; ++a) b[a] = b[3 + a] = means[3 * i + a];
    b[6] = fmaxf(fabsf(scales[3 * i]), fmaxf(fabsf(scales[3 * i + 1]), fabsf(scales[3 * i + 2])));
  }
  for (int off = 32; off > 0; off >>= 1)
    for (int a = 0; a < 3; ++a) {
      b[a] = fminf(b[a], __shfl_xor(b[a], off));
      b[3 + a] = fmaxf(b[3 + a], __shfl_xor(b[3 + a], off));
    }
  for (int off = 32; off > 0; off >>= 1) b[6] = fmaxf(b[6], __shfl_xor(b[6], off));
  if ((threadIdx.x & 63u) == 0)
    for (int a = 0; a < 7; ++a) s_b[a][threadIdx.x >> 6] = b[a];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      for (int a = 0; a < 3; ++a) {
        b[a] = fminf(b[a], s_b[a][w]);
        b[3 + a] = fmaxf(b[3 + a], s_b[3 + a][w]);
      }
      b[6] = fmaxf(b[6], s_b[6][w]);
    }
    out[2 * blockIdx.x] = make_float4(b[0], b[1], b[2], b[6]);
    out[2 * blockIdx.x + 1] = make_float4(b[3], b[4], b[5], 0.0f);
  }
}

hipError_t splat_chunk_bounds(const ptgs_gaussians* g, float* bounds, hipStream_t s) {
  if (g->count == 0) return hipSuccess;
  hipLaunchKernelGGL(gs_chunk_bounds_kernel, dim3((g->count + 255u) / 256u), dim3(256), 0, s, g->means, g->scales,
                     g->count, (float4*)bounds);
  return hipGetLastError();
}

hipError_t splat_reserve(SplatWorkspace* w, uint32_t pairs) {
  hipError_t e;
  if ((e = ensure(w->pairs, (size_t)pairs * 8))) return e;
  if ((e = ensure(w->vals_out, (size_t)pairs * 4))) return e;
  if (w->keys_out.p && (e = ensure(w->keys_out, (size_t)pairs * 8))) return e;
  if (pairs > w->sp_cap) {
    if ((e = ensure(w->sp_keys, (size_t)pairs * 8)) || (e = ensure(w->sp_vals, (size_t)pairs * 4))) return e;
    w->sp_cap = (uint32_t)std::min<size_t>(std::min(w->sp_keys.bytes / 8, w->sp_vals.bytes / 4), 0xFFFFFFF0u);
  }
  return hipSuccess;
}

hipError_t splat_status(SplatWorkspace* w, bool clear, SplatStatusOut* out) {
  *out = SplatStatusOut{};
  if (w->k_host && __atomic_exchange_n(w->k_host + 9, 0u, __ATOMIC_ACQ_REL)) ++w->incomplete;
  out->incomplete = w->incomplete;
  if (clear) w->incomplete = 0;
  const size_t c = std::min(w->pairs.bytes / 8, w->vals_out.bytes / 4);
  out->capacity = (uint32_t)std::min<size_t>(c, 0xFFFFFFFFu);
  out->last_pairs = w->k_host ? w->k_host[0] : 0u;
  out->spill_capacity = w->sp_cap;
  if (w->fz.p) {  // device counters (the caller has drained the workspace's stream)
    uint32_t fz[16];
    const hipError_t e = hipMemcpy(fz, w->fz.p, sizeof(fz), hipMemcpyDeviceToHost);
    if (e) return e;
    out->spilled_tiles = fz[9] - w->spilled_base;
    out->incomplete_tiles = fz[10] - w->incomplete_base;
    out->spill_demand = std::max(fz[8], fz[11]);
    if (clear) {
      w->spilled_base = fz[9];
      w->incomplete_base = fz[10];
    }
  }
  return hipSuccess;
}

uint32_t splat_pair_hint(const SplatWorkspace* w) { return w->k_host ? w->k_host[0] : 0u; }

void splat_front_end_info(const SplatWorkspace* w, uint32_t* touched_runs, uint32_t* fused) {
  *touched_runs = w->k_host ? w->k_host[4] : 0u;
  *fused = w->last_fused ? 1u : 0u;
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
  out->sorted_keys = !w->last_published ? nullptr : (const uint64_t*)(w->last_fused ? w->keys_pub.p : w->keys_out.p);
  out->sorted_values = !w->last_published ? nullptr : (const uint32_t*)(w->last_fused ? w->vals_pub.p : w->vals_out.p);
  out->tile_ranges = (const uint32_t*)w->ranges.p;
  out->means2d = (const float*)w->means2d.p;
  out->depths = (const float*)w->dbg_depths.p;
  out->conic_opacity = (const float*)w->conic.p;
  out->num_gaussians = w->last_n;
  out->num_rendered = w->last_k;
  out->num_tiles = w->last_tiles;
}

void splat_get_tile_rows(const SplatWorkspace* w, const unsigned long long** rows, uint32_t* cap) {
  *rows = w->last_scap ? (const unsigned long long*)w->tile_slots.p : nullptr;
  *cap = w->last_scap;
}

hipError_t splat_point_keys(SplatWorkspace* w, size_t npix, unsigned long long** keys) {
  hipError_t e = ensure(w->point_keys, npix * 8);
  *keys = (unsigned long long*)w->point_keys.p;
  return e;
}

}  // namespace ptgs

GS_STAMP_EXPORT
