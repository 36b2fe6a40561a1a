// pt_kernels.hip — path-tracer kernels for gfx950 (MI355X).
//
//   pt_camera_kernel : shaders/rt_render/raygen_camera.rgen:17-88 (one work-item per pixel,
//                      `spp` consecutive samples per launch; the running mean of :80-87 is kept in
//                      registers across samples, which is bit-identical to one RMW per frame).
//   pt_torus_kernel  : shaders/rt_datacollect/raygen.rgen:31-141 (one work-item per RaySample).
//   pt_depth_kernel  : primary-hit view depth per pixel (pixel-centre ray of raygen_camera.rgen:25-41)
//                      for the hybrid splat-over-path-trace composite.
//
// Launch geometry: 256-thread workgroups = 4 waves, each wave an 8x8 pixel tile (primary-ray
// coherence for the BVH walk), workgroup = 16x16 pixels; 1080p -> 8,160 workgroups (>> 256 CUs).
#include <hip/hip_runtime.h>

#include "pt_shade.h"
#include "pt_launch.h"
#include "xcd.h"

#ifndef PTGS_PT_XCD_REMAP
#define PTGS_PT_XCD_REMAP 0
#endif
#ifndef PTGS_PT_WG
#define PTGS_PT_WG 64  // pt_camera_kernel workgroup: one wave per 8x8 pixel tile (256: four tiles per workgroup)
#endif
#ifndef PTGS_PT_PAIR
#define PTGS_PT_PAIR 1  // one-wave workgroups: two lanes per pixel (even / odd samples) when spp >= 2
#endif
#ifndef PTGS_PT_LPP
#define PTGS_PT_LPP 2  // most lanes per pixel (1, 2, 4)
#endif
#ifndef PTGS_PT_SCHED
#define PTGS_PT_SCHED 1  // heavy-tiles-first schedule of pt_camera_kernel (PtSched)
#endif
#ifndef PTGS_PT_SCHED_MIN
#define PTGS_PT_SCHED_MIN (1u << 22)
#endif

namespace ptgs {

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v) {
  unsigned long long x = v;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ void flush_counters(unsigned long long* counters, uint32_t ext, uint32_t shadow,
                                               uint32_t samples, const TraversalCounters& tc, bool stats) {
  unsigned long long a = wave_sum(ext), b = wave_sum(shadow), c = wave_sum(samples);
  unsigned long long d = 0, e = 0, f = 0;
  if (stats) { d = wave_sum(tc.nodes); e = wave_sum(tc.tris); f = wave_sum(tc.hits); }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(counters + 0, a);
    atomicAdd(counters + 1, b);
    atomicAdd(counters + 2, c);
    if (stats) { atomicAdd(counters + 3, d); atomicAdd(counters + 4, e); atomicAdd(counters + 5, f); }
  }
}

// 4 waves per SIMD (<= 128 VGPRs; the 39-entry LDS stack allows no more workgroups anyway). With the
// NEE shadow ray traced after shading (resolve_shadow) the timed instantiation keeps 96 B per lane of
// scratch (spills in the shading code, once per bounce); round 1 held the shading state across the
// shadow traversal and spilled 164 B per lane. PTGS_PT_MIN_WAVES=3 compiles without scratch and
// measured 9% slower.
#ifndef PTGS_PT_MIN_WAVES
#define PTGS_PT_MIN_WAVES 4
#endif

// PT_STAMP builds (tools/pt_stamps.py): per-workgroup s_memrealtime (100 MHz) at start and end of
// pt_camera_kernel, read back with ptgs_debug_pt_stamps (the schedule's tail)
#ifdef PT_STAMP
#define PT_STAMP_WG 65536  // (>= 32400 8x8 tiles at 1080p)
__device__ unsigned long long g_pt_stamps[PT_STAMP_WG * 2];
#endif

// lanes per pixel of the one-wave tiles (log2): up to PTGS_PT_LPP (1, 2 or 4) when there are that many
// samples to share
__host__ __device__ __forceinline__ uint32_t pt_lanes_log2(uint32_t spp) {
  if (PTGS_PT_WG != 64 || !PTGS_PT_PAIR) return 0u;
  return (PTGS_PT_LPP >= 4 && spp >= 4u) ? 2u : (PTGS_PT_LPP >= 2 && spp >= 2u) ? 1u : 0u;
}

// DEEP: the traversal with the stack overflow (DevScene::deep_stack)
template <bool STATS, bool TEX, bool DEEP>
__global__ __launch_bounds__(PTGS_PT_WG, PTGS_PT_MIN_WAVES) void pt_camera_kernel(DevScene sc, CamParams cp, float4* __restrict__ accum,
                                                        uint32_t W, uint32_t H, uint32_t row0, uint32_t row1,
                                                        uint32_t spp, uint32_t frame0, uint32_t stride,
                                                        uint32_t mode, unsigned long long* counters,
                                                        const uint32_t* __restrict__ order, uint32_t* __restrict__ cost) {
  const uint32_t lid = threadIdx.x;
  const uint32_t wave = lid >> 6, lane = lid & 63u;
#ifdef PT_STAMP
  const uint32_t swg = blockIdx.y * gridDim.x + blockIdx.x;
  if (lid == 0 && swg < PT_STAMP_WG) g_pt_stamps[2 * swg] = __builtin_amdgcn_s_memrealtime();
#endif
#if PTGS_PT_XCD_REMAP
  static_assert(PTGS_PT_WG == 256, "the XCD remap maps 16x16 tiles");
  // XCD-aware: the workgroups of one XCD trace one horizontal strip of 16x16 tiles (shared L2 nodes)
  const uint32_t tl = xcd_tile(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const uint32_t bx = tl % gridDim.x, by = tl / gridDim.x;
#else
  // tile schedule (PtSched): workgroup b renders tile order[b], the tiles that took longest in the
  // previous launch first, so the launch ends on short tiles; each tile's time is recorded for the
  // next launch. Any order gives the same image.
  uint32_t bx = blockIdx.x, by = blockIdx.y;
  if (order) {
    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane((int)order[blockIdx.y * gridDim.x + blockIdx.x]);
    by = tl / gridDim.x;
    bx = tl - by * gridDim.x;
  }
  const unsigned long long t_start = cost ? __builtin_amdgcn_s_memrealtime() : 0ull;
#endif
#if PTGS_PT_WG == 64
  // One wave per workgroup. With spp >= 2 (pair) it shades an 8x4 tile with two lanes per pixel: lane
  // l < 32 traces the even samples, l + 32 the odd ones, and after each pair the even lane folds both
  // results into the pixel's running mean in sample order (the same operations, in the same order,
  // as one lane tracing every sample): half the samples per lane, so a tile takes half as long and the
  // launch's tail of last-started tiles is half as long. Otherwise an 8x8 tile, one sample stream.
  const uint32_t llpp = pt_lanes_log2(spp);               // log2 lanes per pixel: 0, 1, 2 (uniform)
  const bool pair = llpp != 0u;
  const uint32_t lpp = 1u << llpp, pw = 64u >> llpp;       // lanes per pixel, pixels per wave
  const uint32_t half = lane >> (6u - llpp);               // this lane's sample phase
  const uint32_t pl = lane & (pw - 1u);                    // its pixel in the 8 x (8 / lpp) tile
  const uint32_t x = bx * 8u + (pl & 7u);
  const uint32_t y = row0 + by * (8u >> llpp) + (pl >> 3);
#else
  const bool pair = false;
  const uint32_t lpp = 1u, pw = 64u;
  const uint32_t half = 0;
  const uint32_t x = bx * 16u + (wave & 1u) * 8u + (lane & 7u);
  const uint32_t y = row0 + by * 16u + (wave >> 1) * 8u + (lane >> 3);
#endif
  const bool active = (x < W) && (y < row1);

  __shared__ int s_stack[PTGS_STACK * PTGS_PT_WG];
  ShadeCtx c; c.sc = &sc; c.cp = &cp; c.stack = s_stack + threadIdx.x; c.shadow_rays = 0;
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  PT_LANES_INIT(tc);
  uint32_t ext_rays = 0, samples = 0;

  const size_t pix = (size_t)y * W + x;
  v3 state = mk3(0.0f);
  float state_a = 0.0f;
  if (active && half == 0u && (mode == PTGS_ACCUM_SUM || frame0 > 0)) {
    float4 prev = accum[pix];
    state = mk3(prev.x, prev.y, prev.z);
    state_a = prev.w;
  }
  auto fold = [&](const v3& acc, uint32_t s) {  // raygen_camera.rgen:80-87, sample s
    const uint32_t frame = frame0 + s * stride;
    if (mode == PTGS_ACCUM_SUM) {
      state = state + acc;
      state_a = state_a + 1.0f;
    } else if (frame > 0) {
      float blend = 1.0f / (float)(frame + 1u);
      state = mix3(state, acc, blend);
    } else {
      state = acc;
    }
  };
  const uint32_t iters = (spp + lpp - 1u) / lpp;
  for (uint32_t k = 0; k < iters; ++k) {
    const uint32_t s = k * lpp + half;
    v3 acc = mk3(0.0f);
    if (active && s < spp) {
      PT_LANE_TICK(tc, PT_L_SAMPLE);
      const uint32_t frame = frame0 + s * stride;
      v3 ro, rd;
      float4 blue;
      uint32_t seed;
      primary_ray(sc, cp, x, y, W, H, frame, ro, rd, blue, seed);

      v3 thr = mk3(1.0f);
      Payload p;
      p.seed = seed;
      p.blue = mk2(blue.z, blue.w);
      p.last_pdf = 0.0f;
      p.hit_flag = 0.0f;
      p.color = mk3(0.0f); p.weight = mk3(1.0f); p.next_o = ro; p.next_d = rd;
      int max_depth = 12;
      for (int depth = 0; depth < max_depth; ++depth) {
        PT_LANE_TICK(tc, PT_L_BOUNCE);
        p.depth = depth;
        Ray ray = make_ray(ro, rd, 0.001f, 10000.0f);
        ext_rays++;
        Hit h = trace_closest<STATS, TEX, PTGS_PT_WG, DEEP ? PTGS_STACK_OVF : 0>(sc, ray, p.seed, c.stack, tc);
        if (STATS && h.gid != 0xffffffffu) tc.hits++;
        ShadowQuery q;
        q.flags = 0;
        if (h.gid == 0xffffffffu) miss<false>(cp, p);
        else closest_hit<false, TEX>(c, p, ray, h, q);
        resolve_shadow<STATS, TEX, PTGS_PT_WG, DEEP ? PTGS_STACK_OVF : 0>(c, p.color, p.seed, q, tc);  // NEE visibility after shading
        acc = acc + p.color * thr;
        acc = vmin(acc, 5.0f);
        if (p.hit_flag < 0.0f) break;
        if (depth == 0 && p.hit_flag < 1.5f) max_depth = 4;
        thr = thr * p.weight;
        ro = p.next_o;
        rd = p.next_d;
        float mt = fmaxx(fmaxx(thr.x, thr.y), thr.z);
        if (mt < 0.001f) break;
        if (depth >= 4) {
          float pr = clampf(mt, 0.05f, 0.95f);
          if (rnd(p.seed) > pr) break;
          thr = thr / pr;
        }
      }
      samples++;
    }
    if (pair) {  // the other phases' results from lanes + pw, + 2 pw, + 3 pw (every lane exchanges)
      v3 got[4];
      got[0] = acc;
#pragma unroll
      for (uint32_t j = 1; j < 4; ++j) {
        const int src = (int)((lane + j * pw) & 63u);
        got[j] = mk3(__shfl(acc.x, src), __shfl(acc.y, src), __shfl(acc.z, src));
        if (j + 1u >= lpp) break;
      }
      if (active && half == 0u) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (j < lpp && s + j < spp) fold(got[j], s + j);
      }
    } else if (active) {
      fold(acc, s);
    }
  }
  if (active && half == 0u) {
    if (mode == PTGS_ACCUM_SUM) accum[pix] = make_float4(state.x, state.y, state.z, state_a);
    else accum[pix] = make_float4(state.x, state.y, state.z, 1.0f);
  }
  flush_counters(counters, ext_rays, c.shadow_rays, samples, tc, STATS);
  PT_LANES_FLUSH(tc);
#if !PTGS_PT_XCD_REMAP
  if (cost) {
    __syncthreads();  // (every wave of the tile is done)
    if (lid == 0) cost[by * gridDim.x + bx] = (uint32_t)min(__builtin_amdgcn_s_memrealtime() - t_start, 0xFFFFFFFFull);
  }
#endif
#ifdef PT_STAMP
  __syncthreads();
  if (lid == 0 && swg < PT_STAMP_WG) g_pt_stamps[2 * swg + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Untextured: 4 waves per SIMD (the LDS stack's limit) — the single trace / shade site fits 128 VGPRs
// without scratch (the former first-ray + bounce-loop pair of sites needed 143; same speed on the
// Cornell box's 1M-sample collection, tools/torus_ab.py: 0.62 ms per frame, 6.1 Grays/s). Textured:
// no bound (at 128 VGPRs the texture fetches would spill 96 B per lane).
#ifndef PTGS_TORUS_MIN_WAVES
#define PTGS_TORUS_MIN_WAVES 4
#endif
template <bool STATS, bool TEX, bool DEEP>
__global__ __launch_bounds__(256, TEX ? 1 : PTGS_TORUS_MIN_WAVES) void pt_torus_kernel(DevScene sc, CamParams cp, TorusParams tp,
                                                       const ptgs_ray_sample* __restrict__ samples,
                                                       uint32_t n, uint32_t side, uint32_t frame,
                                                       ptgs_hitdata* __restrict__ hits,
                                                       unsigned long long* counters) {
  const uint32_t index = blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ int s_stack[PTGS_STACK * PTGS_BLOCK];
  ShadeCtx c; c.sc = &sc; c.cp = &cp; c.stack = s_stack + threadIdx.x; c.shadow_rays = 0;
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  PT_LANES_INIT(tc);
  uint32_t ext_rays = 0, nsamp = 0;
  if (index < n) {
    const uint32_t lx = index % side, ly = index / side;
    uint32_t light_seed = index + frame * 719393u;
    ptgs_ray_sample smp = samples[index];
    float u = (smp.uv[0] * 2.0f) * PT_PI;
    float v = (smp.uv[1] * 2.0f) * PT_PI;
    float R = tp.major_radius, r = tp.minor_radius, hh = tp.height;
    float su, cu, sv, cv;
    sincosx(u, &su, &cu);
    sincosx(v, &sv, &cv);
    v3 lp = mk3((R + r * cv) * cu, r * sv + hh, (R + r * cv) * su);
    v3 ln = mk3(cv * cu, sv, cv * su);
    v4 wo = matvec(tp.model, mk4(lp.x, lp.y, lp.z, 1.0f));
    v4 wn4 = matvec(tp.model, mk4(ln.x, ln.y, ln.z, 0.0f));
    v3 wn = normalize3(mk3(wn4.x, wn4.y, wn4.z));
    v3 rd = wn;
    v3 so = mk3(wo.x, wo.y, wo.z) + rd * 0.05f;

    float4 blue = blue_noise_texel(sc, lx, ly, frame);
    v3 acc = mk3(0.0f);
    v3 thr = mk3(1.0f);
    Payload p;
    p.seed = light_seed;
    p.last_pdf = 0.0f;
    p.blue = mk2(blue.z, blue.w);
    p.depth = 0;
    p.hit_flag = 0.0f;
    p.color = mk3(0.0f); p.weight = mk3(1.0f); p.next_o = so; p.next_d = rd;
    p.hit_pos = mk3(0.0f); p.normal = mk3(0.0f, 1.0f, 0.0f);
    v3 fpos, fnorm;
    float fflag;
    // one trace / shade site for the first ray and the bounces (raygen.rgen:72-126 as one loop: the
    // first ray starts at tmin 0 and records the HitData position / flag / normal, its radiance is
    // added only on a hit and without the clamp; bounces update the throughput, roulette from depth 4)
    for (int depth = 0; depth < 12; ++depth) {
      if (depth > 0) {
        p.depth = depth;
        thr = thr * p.weight;
        float mt = fmaxx(fmaxx(thr.x, thr.y), thr.z);
        if (mt < 0.001f) break;
        if (depth >= 4) {
          float pr = clampf(mt, 0.05f, 0.95f);
          if (rnd(p.seed) > pr) break;
          thr = thr / pr;
        }
      }
      Ray ray = make_ray(p.next_o, p.next_d, depth == 0 ? 0.0f : 0.001f, 10000.0f);
      ext_rays++;
      Hit h = trace_closest<STATS, TEX, PTGS_BLOCK, DEEP ? PTGS_STACK_OVF : 0>(sc, ray, p.seed, c.stack, tc);
      if (STATS && h.gid != 0xffffffffu) tc.hits++;
      ShadowQuery q;
      q.flags = 0;
      if (h.gid == 0xffffffffu) miss<true>(cp, p);
      else closest_hit<true, TEX>(c, p, ray, h, q);
      resolve_shadow<STATS, TEX, PTGS_BLOCK, DEEP ? PTGS_STACK_OVF : 0>(c, p.color, p.seed, q, tc);
      if (depth == 0) {
        fpos = p.hit_pos;
        fflag = p.hit_flag;
        fnorm = p.normal;
        if (!(p.hit_flag > 0.5f)) break;
        acc = acc + p.color * thr;
      } else {
        acc = acc + p.color * thr;
        acc = vmin(acc, 5.0f);
        if (p.hit_flag < 1.5f) break;
      }
    }
    v3 cur = acc;
    ptgs_hitdata hd = hits[index];
    if (frame > 0) {
      v3 prev = mk3(hd.color[0], hd.color[1], hd.color[2]);
      float bf = 1.0f / (float)(frame + 1u);
      cur = mix3(prev, cur, bf);
    }
    hd.pos[0] = fpos.x; hd.pos[1] = fpos.y; hd.pos[2] = fpos.z;
    hd.flag = fflag;
    hd.normal[0] = fnorm.x; hd.normal[1] = fnorm.y; hd.normal[2] = fnorm.z;
    hd.color[0] = cur.x; hd.color[1] = cur.y; hd.color[2] = cur.z; hd.color[3] = 1.0f;
    hits[index] = hd;
    nsamp = 1;
  }
  flush_counters(counters, ext_rays, c.shadow_rays, nsamp, tc, STATS);
}

// Primary-hit depth: the camera ray of raygen_camera.rgen:25-41 through the pixel centre (no
// jitter), closest hit with the frame's any-hit seed (index + frame_count * 719393, :21); depth =
// view-space distance -(view * hit).z of the hit point, +inf on a miss. One work-item per pixel.
template <bool TEX, bool DEEP>
__global__ __launch_bounds__(256) void pt_depth_kernel(DevScene sc, CamParams cp, ViewMat vm, float* __restrict__ depth,
                                                       uint32_t W, uint32_t H, uint32_t row0, uint32_t row1,
                                                       uint32_t frame) {
  const uint32_t lid = threadIdx.x;
  const uint32_t wave = lid >> 6, lane = lid & 63u;
  const uint32_t x = blockIdx.x * 16u + (wave & 1u) * 8u + (lane & 7u);
  const uint32_t y = row0 + blockIdx.y * 16u + (wave >> 1) * 8u + (lane >> 3);
  __shared__ int s_stack[PTGS_STACK * PTGS_BLOCK];
  if (x >= W || y >= row1) return;
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  PT_LANES_INIT(tc);
  const uint32_t seed = y * W + x + frame * 719393u;
  const float ux = ((float)x + 0.5f) / (float)W, uy = ((float)y + 0.5f) / (float)H;
  const float dx = ux * 2.0f - 1.0f, dy = uy * 2.0f - 1.0f;
  const v4 origin = matvec(cp.inv_view, mk4(0.f, 0.f, 0.f, 1.f));
  const v4 target = matvec(cp.inv_proj, mk4(dx, dy, 1.f, 1.f));
  const v3 dirc = normalize3(mk3(target.x, target.y, target.z) / target.w);
  const v4 direction = matvec(cp.inv_view, mk4(dirc.x, dirc.y, dirc.z, 0.f));
  const v3 ro = mk3(origin.x, origin.y, origin.z);
  const v3 rd = normalize3(mk3(direction.x, direction.y, direction.z));
  const Ray ray = make_ray(ro, rd, 0.001f, 10000.0f);
  const Hit h = trace_closest<false, TEX, PTGS_BLOCK, DEEP ? PTGS_STACK_OVF : 0>(sc, ray, seed, s_stack + threadIdx.x, tc);
  float d = __builtin_huge_valf();
  if (h.gid != 0xffffffffu) {
    const v3 hp = ro + rd * h.t;
    const v4 pv = matvec(vm.m, mk4(hp.x, hp.y, hp.z, 1.0f));
    d = -pv.z;
  }
  depth[(size_t)y * W + x] = d;
}

// One workgroup: the tiles by the previous launch's time, longest first (counting sort over 256
// buckets of max / 256; the order inside a bucket is the LDS atomics')
#define PT_ORDER_THREADS 1024
__global__ __launch_bounds__(PT_ORDER_THREADS) void pt_order_kernel(const uint32_t* __restrict__ cost,
                                                                    uint32_t* __restrict__ order, uint32_t n) {
  __shared__ uint32_t s_h[256];
  __shared__ uint32_t s_max[PT_ORDER_THREADS / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  uint32_t mx = 0;
  for (uint32_t t = tid; t < n; t += PT_ORDER_THREADS) mx = max(mx, cost[t]);
  for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
  if (lane == 0) s_max[tid >> 6] = mx;
  if (tid < 256) s_h[tid] = 0;
  __syncthreads();
  mx = 0;
  for (uint32_t w = 0; w < PT_ORDER_THREADS / 64; ++w) mx = max(mx, s_max[w]);
  const float scale = 255.99f / (float)max(mx, 1u);
  auto bucket = [&](uint32_t c) { return 255u - min(255u, (uint32_t)((float)c * scale)); };
  for (uint32_t t = tid; t < n; t += PT_ORDER_THREADS) atomicAdd(s_h + bucket(cost[t]), 1u);
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the buckets, four per lane
    const uint32_t c0 = s_h[4 * lane], c1 = s_h[4 * lane + 1], c2 = s_h[4 * lane + 2], c3 = s_h[4 * lane + 3];
    const uint32_t sum = (c0 + c1) + (c2 + c3);
    uint32_t incl = sum;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= (uint32_t)off) incl += y;
    }
    const uint32_t ex = incl - sum;
    s_h[4 * lane] = ex;
    s_h[4 * lane + 1] = ex + c0;
    s_h[4 * lane + 2] = ex + c0 + c1;
    s_h[4 * lane + 3] = ex + c0 + c1 + c2;
  }
  __syncthreads();
  for (uint32_t t = tid; t < n; t += PT_ORDER_THREADS) order[atomicAdd(s_h + bucket(cost[t]), 1u)] = t;
}

void free_pt_sched(PtSched& ps) {
  if (ps.cost) (void)hipFree(ps.cost);
  if (ps.order) (void)hipFree(ps.order);
  ps = PtSched{};
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_pt_camera(const DevScene& sc, const CamParams& cp, float* accum, uint32_t W, uint32_t H,
                            uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0, uint32_t stride,
                            uint32_t mode, unsigned long long* counters, bool stats, PtSched* ps,
                            hipStream_t stream) {
  if (row1 <= row0 || spp == 0) return hipSuccess;
  // tiles: 16x16 (256-thread workgroups), 8x8 (one wave), 8x4 (one wave, two lanes per pixel: spp >= 2)
  const uint32_t tx = PTGS_PT_WG == 64 ? 8u : 16u;
  const uint32_t ty = PTGS_PT_WG == 64 ? 8u >> pt_lanes_log2(spp) : 16u;
  dim3 grid((W + tx - 1u) / tx, (row1 - row0 + ty - 1u) / ty);
  dim3 block(PTGS_PT_WG);
  const uint32_t *order = nullptr;
  uint32_t* cost = nullptr;
#if !PTGS_PT_XCD_REMAP
  // heavy tiles first once a launch of this grid has recorded its tile times; launches of fewer than
  // PTGS_PT_SCHED_MIN pixel-samples skip it (C1's 65k: the order kernel's launch would cost more than
  // the tail it saves)
  if (ps && PTGS_PT_SCHED && ps->owned && ps->stream != stream) {
    // another stream holds the schedule: take it over once that stream has drained (its launches may
    // still read `order`), else this launch runs unscheduled and records nothing
    if (hipStreamQuery(ps->stream) != hipErrorNotReady) {
      ps->owned = false;
      ps->gx = ps->gy = 0;  // (its recorded times belong to the old stream's grid: record afresh)
    } else {
      ps = nullptr;
    }
  }
  if (ps && PTGS_PT_SCHED && (uint64_t)W * (row1 - row0) * spp >= (uint64_t)PTGS_PT_SCHED_MIN) {
    const uint32_t n = grid.x * grid.y;
    hipError_t e;
    ps->stream = stream;
    ps->owned = true;
    if (n > ps->cap) {
      free_pt_sched(*ps);
      if ((e = hipMalloc(&ps->cost, (size_t)n * 4)) || (e = hipMalloc(&ps->order, (size_t)n * 4))) return e;
      ps->cap = n;
    }
    if (ps->gx == grid.x && ps->gy == grid.y) {
      hipLaunchKernelGGL(pt_order_kernel, dim3(1), dim3(PT_ORDER_THREADS), 0, stream, (const uint32_t*)ps->cost,
                         ps->order, n);
      if ((e = hipGetLastError())) return e;
      order = ps->order;
    }
    ps->gx = grid.x;
    ps->gy = grid.y;
    cost = ps->cost;
  }
#endif
  // (STATS, TEX, DEEP) instantiations: TEX only for scenes whose materials reference textures, DEEP only
  // for trees deeper than the LDS stack
  static void (*const ks[8])(DevScene, CamParams, float4*, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                             uint32_t, uint32_t, unsigned long long*, const uint32_t*, uint32_t*) = {
      pt_camera_kernel<false, false, false>, pt_camera_kernel<false, false, true>, pt_camera_kernel<false, true, false>,
      pt_camera_kernel<false, true, true>,   pt_camera_kernel<true, false, false>, pt_camera_kernel<true, false, true>,
      pt_camera_kernel<true, true, false>,   pt_camera_kernel<true, true, true>};
  auto k = ks[(stats ? 4 : 0) + (sc.uses_textures ? 2 : 0) + (sc.deep_stack ? 1 : 0)];
  hipLaunchKernelGGL(k, grid, block, 0, stream, sc, cp, (float4*)accum, W, H, row0, row1, spp, frame0, stride, mode,
                     counters, order, cost);
  return hipGetLastError();
}

hipError_t launch_pt_depth(const DevScene& sc, const CamParams& cp, const ViewMat& vm, float* depth, uint32_t W,
                           uint32_t H, uint32_t row0, uint32_t row1, uint32_t frame, hipStream_t stream) {
  row1 = row1 < H ? row1 : H;
  if (row1 <= row0) return hipSuccess;
  dim3 grid((W + 15u) / 16u, (row1 - row0 + 15u) / 16u);
  auto k = sc.uses_textures ? (sc.deep_stack ? pt_depth_kernel<true, true> : pt_depth_kernel<true, false>)
                           : (sc.deep_stack ? pt_depth_kernel<false, true> : pt_depth_kernel<false, false>);
  hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, sc, cp, vm, depth, W, H, row0, row1, frame);
  return hipGetLastError();
}

hipError_t launch_pt_torus(const DevScene& sc, const CamParams& cp, const TorusParams& tp,
                           const ptgs_ray_sample* samples, uint32_t n, uint32_t side, uint32_t frame,
                           ptgs_hitdata* hits, unsigned long long* counters, bool stats, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  dim3 grid((n + 255u) / 256u);
  dim3 block(256);
  static void (*const ks[8])(DevScene, CamParams, TorusParams, const ptgs_ray_sample*, uint32_t, uint32_t, uint32_t,
                             ptgs_hitdata*, unsigned long long*) = {
      pt_torus_kernel<false, false, false>, pt_torus_kernel<false, false, true>, pt_torus_kernel<false, true, false>,
      pt_torus_kernel<false, true, true>,   pt_torus_kernel<true, false, false>, pt_torus_kernel<true, false, true>,
      pt_torus_kernel<true, true, false>,   pt_torus_kernel<true, true, true>};
  auto k = ks[(stats ? 4 : 0) + (sc.uses_textures ? 2 : 0) + (sc.deep_stack ? 1 : 0)];
  hipLaunchKernelGGL(k, grid, block, 0, stream, sc, cp, tp, samples, n, side, frame, hits, counters);
  return hipGetLastError();
}

}  // namespace ptgs

#ifdef PT_LANES
// (diagnostic builds: the lane counts of pt_device.h PtLoop, read and cleared)
extern "C" int ptgs_debug_pt_lanes(unsigned long long* host, unsigned int n) {
  if (n > 2u * ptgs::PT_L_COUNT) n = 2u * ptgs::PT_L_COUNT;
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(ptgs::g_pt_lanes), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
  if (e) return (int)e;
  static const unsigned long long zero[2 * ptgs::PT_L_COUNT] = {};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(ptgs::g_pt_lanes), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif
#ifdef PT_STAMP
extern "C" int ptgs_debug_pt_stamps(unsigned long long* host, unsigned int n) {
  if (n > PT_STAMP_WG * 2u) n = PT_STAMP_WG * 2u;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ptgs::g_pt_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif
