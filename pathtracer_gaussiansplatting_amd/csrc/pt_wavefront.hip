// pt_wavefront.hip — wavefront path tracer for ptgs_trace_camera (gfx950).
//
// The per-pixel loop of raygen_camera.rgen:17-88 (one work-item carrying a path through every
// bounce, pt_kernels.hip's pt_camera_kernel) split into stages, one launch per stage and bounce:
//
//   raygen     one work-item per pixel slot: the jittered camera ray (:19-41), the path state
//              (:43-48), the slot's "extension ray pending" flag
//   extend     closest hit of every pending extension ray (:51)
//   shade      miss.rmiss / closesthit.rchit:324-621 on the hit: emission, NEE query, BSDF sample; the
//              bounce bookkeeping of :53-78 (accumulate + clamp, adaptive depth, throughput, RR); the
//              next ray and the NEE shadow ray of the slot, and its two flags
//   shadow     any-hit of every pending shadow ray (closesthit.rchit:115-126); an unoccluded ray
//              selects the accumulation that includes the light (precomputed by shade)
//   accumulate the running mean / sum of :80-87 per pixel, in sample order
//
// Everything is indexed by pixel slot (8x8 pixel tiles in row-major tile order: a wave's 64 slots
// are one tile), so no stage needs a global atomic or a queue counter (same-address atomics cost
// ~6-13 ns each on this part: one per wave of a 2M-path frame is ~0.4 ms). Compaction is wave-local
// instead: each wave owns a run of slots, reads their flags 64 at a time and appends the live ones
// to a 128-entry ring in LDS (ballot + mbcnt); extend / shadow lanes whose traversal finished take
// the next live slot from the ring at once (persistent per-lane refill: lanes do not idle behind
// the wave's longest traversal), shade takes 64 at a time, so every stage runs on full waves.
//
// Every path computes exactly what pt_camera_kernel computes for it (same device functions, same
// seed sequence: the BLEND any-hit hash reads the seed of the bounce, RR advances it after), so the
// images, ray counts and statistics are bit-identical to the megakernel and to the CPU oracle.
//
// Per slot (SoA, float4 for 16-B accesses): ray 32 B ((origin, seed) (direction, -)), hit 16 B
// (t, u, v, gid), shadow ray 48 B ((origin, tmax) (direction, seed) (acc if unoccluded, -)), path
// state 48 B ((throughput, last_pdf) (weight, hit_flag) (acc, max_depth)), 1 flag byte (bit 0
// extension ray pending, bit 1 shadow ray pending). Ray counts go to per-workgroup partial sums
// (no atomics) folded into the context's counters once per call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "pt_shade.h"
#include "pt_wavefront.h"

namespace ptgs {

namespace {

constexpr int WF_DONE = 0x7fffffff;
constexpr uint32_t WF_MAX_DEPTH = 12;  // raygen_camera.rgen:46 max_depth
constexpr uint8_t WF_EXT = 1u, WF_SHADOW = 2u;
constexpr uint32_t WF_RING = 128u;     // per-wave LDS ring of pending live slots
// per-workgroup partial counters: [counter][block] (counter 0 extension rays, 1 shadow rays,
// 2 samples, 3 node tests, 4 triangle tests, 5 closest hits)
constexpr uint32_t WF_NCNT = 6;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LDS written by some lanes of the wave and read by others: order the accesses within the wave
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }

// Path state streams through HBM once per bounce (GBs per batch): non-temporal loads / stores keep
// it from evicting the BVH and triangles (17 MB for C3) from L2 / Infinity Cache.
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt(const float4* p) {
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt(float4* p, float4 v) {
  f4v x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(p));
}

// slot -> (pixel, sample): slot = (tile * batch + s) * 64 + lane over 8x8 pixel tiles in row-major
// tile order; a wave holds one tile for one sample, and the batch's samples of a tile are adjacent
// (the megakernel's per-pixel sample loop reuses the same BVH nodes from cache; so do these waves)
__device__ __forceinline__ void slot_pixel(const WfArgs& a, uint32_t slot, uint32_t& x, uint32_t& y, uint32_t& frame) {
  const uint32_t w = slot >> 6, l = slot & 63u;
  const uint32_t t = w / a.batch, smp = w - t * a.batch;
  x = (t % a.tiles_x) * 8u + (l & 7u);
  y = a.row0 + (t / a.tiles_x) * 8u + (l >> 3);
  frame = a.frame0 + smp * a.stride;
}

// Wave-local stream of the live slots (flags & bit) of the run [cursor, end): windows of 64 flags
// are ballot-compacted into a 128-entry LDS ring; all fields are wave-uniform.
// Ring entries are 16-bit offsets from the run's first slot (runs are at most 65536 slots), so the
// traversal kernels' LDS (39-entry stack + 4 rings) is exactly 40 KiB: 4 workgroups per CU.
struct SlotStream {
  uint32_t cursor, end, head, tail, begin;
  uint16_t* ring;
  __device__ __forceinline__ uint32_t at(uint32_t k) const { return begin + ring[k & (WF_RING - 1u)]; }
};

__device__ __forceinline__ void ss_init(SlotStream& s, uint16_t* ring, uint32_t begin, uint32_t end) {
  s.cursor = begin; s.end = end; s.head = 0; s.tail = 0; s.begin = begin; s.ring = ring;
}

// append windows until `want` slots are pending or the run is exhausted (ring never overfilled)
__device__ __forceinline__ void ss_fill(SlotStream& s, const uint8_t* __restrict__ flags, uint8_t bit, uint32_t want) {
  while (s.tail - s.head < want && s.tail - s.head <= WF_RING - 64u && s.cursor < s.end) {
    const uint32_t slot = s.cursor + lane_id();
    const bool live = slot < s.end && (flags[slot] & bit) != 0;
    const unsigned long long m = __ballot(live);
    wave_sync();  // earlier reads of the ring are done before it is overwritten
    if (live) s.ring[(s.tail + mbcnt64(m)) & (WF_RING - 1u)] = (uint16_t)(slot - s.begin);
    s.tail += (uint32_t)__popcll(m);
    s.cursor += 64u;
  }
  wave_sync();
}

// Traversal stack of the extend / shadow kernels: the first WF_LDS_STACK entries in LDS (interleaved
// by work-item, as pt_device.h), deeper entries up to PTGS_STACK_TOTAL (rare: C3's tree needs up to
// 38, C5's 40) in a per-work-item global overflow area. A shorter LDS stack buys occupancy.
#ifndef PTGS_WF_AH_CALL
// textured any-hit inlined (true: out of line, pt_device.h anyhit_accept_call — round 2's workaround for
// the SLP miscompile that build.py now avoids with -slp-vectorize-hor=false)
#define PTGS_WF_AH_CALL false
#endif
#ifndef PTGS_WF_AH_CALL_EXT
#define PTGS_WF_AH_CALL_EXT PTGS_WF_AH_CALL
#endif
#ifndef PTGS_WF_AH_CALL_SHADOW
#define PTGS_WF_AH_CALL_SHADOW PTGS_WF_AH_CALL
#endif
#ifndef PTGS_WF_LDS_EXT
#define PTGS_WF_LDS_EXT PTGS_STACK  // extend kernel: LDS entries (39: 4 waves / SIMD, 86 VGPRs)
#endif
#ifndef PTGS_WF_LDS_SHADOW
#define PTGS_WF_LDS_SHADOW 25       // shadow kernel: 25 entries: 6 waves / SIMD (73 VGPRs)
#endif
__host__ __device__ constexpr int wf_min_waves(int n) { return n <= 25 ? 6 : (n <= 31 ? 5 : 4); }
template <int N>
struct TravStack {
  int* lds;       // this work-item's column
  int* ovf;       // this work-item's overflow column (stride ostride)
  uint32_t ostride;
  int sp;
  __device__ __forceinline__ void push(int v) {
    if (N >= PTGS_STACK_TOTAL || sp < N) lds[sp * PTGS_BLOCK] = v;
    else ovf[(size_t)(sp - N) * ostride] = v;
    ++sp;
  }
  __device__ __forceinline__ int pop_nz() {  // sp > 0
    --sp;
    if (N >= PTGS_STACK_TOTAL || sp < N) return lds[sp * PTGS_BLOCK];
    return ovf[(size_t)(sp - N) * ostride];
  }
};

// block-level sum of v into part[k * stride + blockIdx.x] (plain read-modify-write: each block owns
// its entry, successive launches are stream-ordered)
__device__ __forceinline__ void block_count(uint32_t* __restrict__ part, uint32_t stride, int k, uint32_t v,
                                            uint32_t* s_red) {
  unsigned long long x = v;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  __syncthreads();
  if (lane_id() == 0) s_red[threadIdx.x >> 6] = (uint32_t)x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < blockDim.x / 64u; ++w) t += s_red[w];
    part[k * stride + blockIdx.x] += t;
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// raygen_camera.rgen:19-48: primary rays of the batch's samples for every pixel of the row range
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pt_wf_raygen_kernel(DevScene sc, CamParams cp, WfArgs a) {
  __shared__ uint32_t s_red[4];
  const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
  uint32_t x, y, frame;
  slot_pixel(a, slot, x, y, frame);
  const bool valid = slot < a.slots && x < a.W && y < a.row1;
  if (valid) {
    v3 ro, rd;
    float4 blue;
    uint32_t seed;
    primary_ray(sc, cp, x, y, a.W, a.H, frame, ro, rd, blue, seed);
    stnt(a.ray_o + slot, make_float4(ro.x, ro.y, ro.z, u2f(seed)));
    stnt(a.ray_d + slot, make_float4(rd.x, rd.y, rd.z, 0.0f));
    // throughput 1, last_pdf 0 | weight 1, hit_flag 0 | acc 0, max_depth 12 (:43-48)
    stnt(a.st_thr + slot, make_float4(1.0f, 1.0f, 1.0f, 0.0f));
    stnt(a.st_w + slot, make_float4(1.0f, 1.0f, 1.0f, 0.0f));
    stnt(a.st_acc + slot, make_float4(0.0f, 0.0f, 0.0f, (float)WF_MAX_DEPTH));
  }
  if (slot < a.slots) a.flags[slot] = valid ? WF_EXT : 0u;
  if (blockIdx.x == 0 && threadIdx.x < 2u * (WF_MAX_DEPTH + 1u)) a.live[threadIdx.x] = threadIdx.x == 0 ? 1u : 0u;
  block_count(a.part, a.part_stride, 2, valid ? 1u : 0u, s_red);  // samples
}

// ------------------------------------------------------------------------------------------------
// extend: closest hit of the pending extension rays (raygen_camera.rgen:51, pt_device.h trace_closest)
// ------------------------------------------------------------------------------------------------
template <bool STATS, bool TEX>
__global__ __launch_bounds__(256, wf_min_waves(PTGS_WF_LDS_EXT)) void pt_wf_extend_kernel(DevScene sc, WfArgs a, uint32_t depth, uint32_t per_wave,
                                                              uint32_t refill) {
  if (a.live[2u * depth] == 0u) return;  // no path reached this bounce (adaptive depth / RR ended them)
  __shared__ int s_stack[PTGS_WF_LDS_EXT * PTGS_BLOCK];
  __shared__ uint16_t s_ring[4][WF_RING];
  uint32_t* s_red = reinterpret_cast<uint32_t*>(s_ring);  // after the loop: the count reduction
  TravStack<PTGS_WF_LDS_EXT> st;
  st.lds = s_stack + threadIdx.x;
  st.ovf = a.ovf + blockIdx.x * 256u + threadIdx.x;
  st.ostride = gridDim.x * 256u;
  st.sp = 0;
  const uint32_t begin = (blockIdx.x * 4u + (threadIdx.x >> 6)) * per_wave;  // this wave's run of slots
  SlotStream ss;
  ss_init(ss, s_ring[threadIdx.x >> 6], begin, min(a.slots, begin + per_wave));
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  PT_LANES_INIT(tc);
  uint32_t traced = 0;
  bool active = false;
  uint32_t slot = 0, seed = 0;
  Ray r = make_ray(mk3(0.0f), mk3(1.0f), 0.001f, 10000.0f);
  Hit h; h.t = 0.f; h.u = 0.f; h.v = 0.f; h.gid = 0xffffffffu; h.slot = 0;
  int node = WF_DONE, leaf = WF_DONE;
  auto push = [&](int v) { st.push(v); };
  auto pop = [&]() -> int { return st.sp ? st.pop_nz() : WF_DONE; };
  for (;;) {
    // lanes whose ray finished take the next pending rays of the run, once `refill` of them are
    // idle (or none is busy): one refill's loads stall the wave, so they are batched
    const unsigned long long idle = __ballot(!active);
    const uint32_t nidle = (uint32_t)__popcll(idle);
    if (nidle >= refill || nidle == 64u || idle == __ballot(true)) {
      ss_fill(ss, a.flags, WF_EXT, nidle);
      const uint32_t avail = ss.tail - ss.head, rk = mbcnt64(idle);
      if (!active && rk < avail) {
        slot = ss.at(ss.head + rk);
        const float4 ro = ldnt(a.ray_o + slot), rd = ldnt(a.ray_d + slot);
        r = make_ray(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), 0.001f, 10000.0f);
        seed = f2u(ro.w);
        h.t = r.tmax; h.u = 0.f; h.v = 0.f; h.gid = 0xffffffffu;
        node = 0; st.sp = 0; leaf = WF_DONE;
        active = true;
      }
      ss.head += min(avail, nidle);
      if (!active) break;  // the run is exhausted for this lane
    }
    if (!active) continue;  // idle below the refill threshold: wait for the busy lanes (they hold the loop)
    // one round of the while-while walk (postponed leaves, as trace_closest)
    while (node >= 0 && node != WF_DONE) {
      Box4 b;
      box4(r, sc, node, h.t, b);
      if (STATS) tc.nodes += 4;
      node = enter_box4(b, push, pop);
      if (node < 0 && leaf == WF_DONE) {
        leaf = node;
        node = pop();
      }
      if ((__builtin_amdgcn_ballot_w64(leaf != WF_DONE) | __builtin_amdgcn_ballot_w64(node == WF_DONE)) ==
          __builtin_amdgcn_read_exec())
        break;
    }
    if (leaf != WF_DONE) {
      leaf_closest<STATS, TEX, PTGS_WF_AH_CALL_EXT>(sc, r, leaf, h, seed, tc);
      leaf = WF_DONE;
    }
    if (node < 0) {
      leaf_closest<STATS, TEX, PTGS_WF_AH_CALL_EXT>(sc, r, node, h, seed, tc);
      node = pop();
    }
    if (node == WF_DONE) {
      stnt(a.hits + slot, make_float4(h.t, h.u, h.v, u2f(h.gid)));
      if (STATS && h.gid != 0xffffffffu) tc.hits++;
      traced++;
      active = false;
    }
  }
  block_count(a.part, a.part_stride, 0, traced, s_red);  // extension rays
  if (STATS) {
    block_count(a.part, a.part_stride, 3, tc.nodes, s_red);
    block_count(a.part, a.part_stride, 4, tc.tris, s_red);
    block_count(a.part, a.part_stride, 5, tc.hits, s_red);
  }
}

// ------------------------------------------------------------------------------------------------
// shade: miss / closest hit + the bounce bookkeeping of raygen_camera.rgen:53-78 for depth `depth`
// ------------------------------------------------------------------------------------------------
template <bool TEX>
__device__ __forceinline__ uint32_t wf_shade_slot(const DevScene& sc, const CamParams& cp, const WfArgs& a,
                                                  uint32_t depth, uint32_t slot) {
  ShadeCtx c; c.sc = &sc; c.cp = &cp; c.stack = nullptr; c.shadow_rays = 0;
  const float4 r_o = ldnt(a.ray_o + slot), r_d = ldnt(a.ray_d + slot), hv = ldnt(a.hits + slot);
  const float4 s_thr = ldnt(a.st_thr + slot), s_w = ldnt(a.st_w + slot), s_acc = ldnt(a.st_acc + slot);
  uint32_t x, y, frame;
  slot_pixel(a, slot, x, y, frame);
  const float4 blue = blue_noise_texel(sc, x, y, frame);
  Payload p;
  p.seed = f2u(r_o.w);
  p.blue = mk2(blue.z, blue.w);
  p.last_pdf = s_thr.w;
  p.hit_flag = s_w.w;
  p.weight = mk3(s_w.x, s_w.y, s_w.z);
  p.color = mk3(0.0f);
  p.next_o = mk3(r_o.x, r_o.y, r_o.z);
  p.next_d = mk3(r_d.x, r_d.y, r_d.z);
  p.depth = (int)depth;
  p.hit_pos = mk3(0.0f); p.normal = mk3(0.0f);
  const Ray ray = make_ray(p.next_o, p.next_d, 0.001f, 10000.0f);
  Hit h; h.t = hv.x; h.u = hv.y; h.v = hv.z; h.gid = f2u(hv.w); h.slot = 0;
  ShadowQuery sq;
  sq.flags = 0;
  if (h.gid == 0xffffffffu) miss<false>(cp, p);
  else closest_hit<false, TEX>(c, p, ray, h, sq);
  v3 thr = mk3(s_thr.x, s_thr.y, s_thr.z);
  v3 acc = mk3(s_acc.x, s_acc.y, s_acc.z);
  float max_depth = s_acc.w;
  // resolve_shadow's two outcomes (vis = 0 / 1 before max(vis, transmission)): the shadow kernel
  // keeps the occluded accumulation unless the ray reaches the light
  const bool traced = (sq.flags & SQ_TRACE) != 0;
  v3 col_occ = p.color;
  if (traced) {
    v3 col_vis = p.color;
    const float vo = fmaxx(0.0f, sq.trans), vv = fmaxx(1.0f, sq.trans);
    if (vo > 0.0f && (sq.flags & SQ_VALID)) {
      v3 contrib = (sq.pre * vo) * sq.post;
      if (sq.flags & SQ_MIXED) contrib = (mk3(0.0f) + contrib) * sq.scale;
      col_occ = col_occ + contrib;
    }
    if (vv > 0.0f && (sq.flags & SQ_VALID)) {
      v3 contrib = (sq.pre * vv) * sq.post;
      if (sq.flags & SQ_MIXED) contrib = (mk3(0.0f) + contrib) * sq.scale;
      col_vis = col_vis + contrib;
    }
    const v3 acc_vis = vmin(acc + col_vis * thr, 5.0f);
    // the any-hit seed is the bounce's seed: before this bounce's RR draw
    stnt(a.sh_o + slot, make_float4(sq.o.x, sq.o.y, sq.o.z, sq.tmax));
    stnt(a.sh_d + slot, make_float4(sq.d.x, sq.d.y, sq.d.z, u2f(p.seed)));
    stnt(a.sh_acc + slot, make_float4(acc_vis.x, acc_vis.y, acc_vis.z, 0.0f));
  }
  acc = vmin(acc + col_occ * thr, 5.0f);
  // :60-78
  bool alive = !(p.hit_flag < 0.0f);
  if (alive) {
    if (depth == 0 && p.hit_flag < 1.5f) max_depth = 4.0f;
    thr = thr * p.weight;
    const float mt = fmaxx(fmaxx(thr.x, thr.y), thr.z);
    if (mt < 0.001f) {
      alive = false;
    } else if (depth >= 4) {
      const float pr = clampf(mt, 0.05f, 0.95f);
      if (rnd(p.seed) > pr) alive = false;
      else thr = thr / pr;
    }
    if (alive && (float)(depth + 1u) >= max_depth) alive = false;
  }
  stnt(a.st_acc + slot, make_float4(acc.x, acc.y, acc.z, max_depth));
  if (alive) {
    stnt(a.st_thr + slot, make_float4(thr.x, thr.y, thr.z, p.last_pdf));
    stnt(a.st_w + slot, make_float4(p.weight.x, p.weight.y, p.weight.z, p.hit_flag));
    stnt(a.ray_o + slot, make_float4(p.next_o.x, p.next_o.y, p.next_o.z, u2f(p.seed)));
    stnt(a.ray_d + slot, make_float4(p.next_d.x, p.next_d.y, p.next_d.z, 0.0f));
  }
  const uint32_t fl = (alive ? WF_EXT : 0u) | (traced ? WF_SHADOW : 0u);
  a.flags[slot] = (uint8_t)fl;
  return fl;
}

template <bool TEX>
__global__ __launch_bounds__(256) void pt_wf_shade_kernel(DevScene sc, CamParams cp, WfArgs a, uint32_t depth,
                                                          uint32_t per_wave) {
  if (a.live[2u * depth] == 0u) return;
  __shared__ uint16_t s_ring[4][WF_RING];
  __shared__ uint32_t s_any;
  if (threadIdx.x == 0) s_any = 0u;
  __syncthreads();
  const uint32_t begin = (blockIdx.x * 4u + (threadIdx.x >> 6)) * per_wave;
  SlotStream ss;
  ss_init(ss, s_ring[threadIdx.x >> 6], begin, min(a.slots, begin + per_wave));
  uint32_t any = 0;
  for (;;) {  // full waves of live slots
    ss_fill(ss, a.flags, WF_EXT, 64u);
    const uint32_t take = min(64u, ss.tail - ss.head);
    if (take == 0) break;
    const bool ok = lane_id() < take;
    const uint32_t slot = ok ? ss.at(ss.head + lane_id()) : 0u;
    ss.head += take;
    if (ok) any |= wf_shade_slot<TEX>(sc, cp, a, depth, slot);
  }
  // which stages the next launches have work for (one word each, written once per workgroup)
  if (any) atomicOr(&s_any, any);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_any & WF_EXT) a.live[2u * (depth + 1u)] = 1u;
    if (s_any & WF_SHADOW) a.live[2u * depth + 1u] = 1u;
  }
}

// ------------------------------------------------------------------------------------------------
// shadow: any-hit of the pending NEE rays (pt_device.h trace_any); unoccluded -> the "visible" acc
// ------------------------------------------------------------------------------------------------
template <bool STATS, bool TEX>
__global__ __launch_bounds__(256, wf_min_waves(PTGS_WF_LDS_EXT)) void pt_wf_shadow_kernel(DevScene sc, WfArgs a, uint32_t depth, uint32_t per_wave,
                                                              uint32_t refill) {
  if (a.live[2u * depth + 1u] == 0u) return;  // no shadow ray at this bounce
  __shared__ int s_stack[PTGS_WF_LDS_SHADOW * PTGS_BLOCK];
  __shared__ uint16_t s_ring[4][WF_RING];
  uint32_t* s_red = reinterpret_cast<uint32_t*>(s_ring);  // after the loop: the count reduction
  TravStack<PTGS_WF_LDS_SHADOW> st;
  st.lds = s_stack + threadIdx.x;
  st.ovf = a.ovf + blockIdx.x * 256u + threadIdx.x;
  st.ostride = gridDim.x * 256u;
  st.sp = 0;
  const uint32_t begin = (blockIdx.x * 4u + (threadIdx.x >> 6)) * per_wave;
  SlotStream ss;
  ss_init(ss, s_ring[threadIdx.x >> 6], begin, min(a.slots, begin + per_wave));
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  PT_LANES_INIT(tc);
  uint32_t traced = 0;
  bool active = false;
  uint32_t slot = 0, seed = 0;
  Ray r = make_ray(mk3(0.0f), mk3(1.0f), 0.001f, 1.0f);
  int node = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!active);  // batched refill, as in the extend kernel
    const uint32_t nidle = (uint32_t)__popcll(idle);
    if (nidle >= refill || nidle == 64u || idle == __ballot(true)) {
      ss_fill(ss, a.flags, WF_SHADOW, nidle);
      const uint32_t avail = ss.tail - ss.head, rk = mbcnt64(idle);
      if (!active && rk < avail) {
        slot = ss.at(ss.head + rk);
        const float4 so = ldnt(a.sh_o + slot), sd = ldnt(a.sh_d + slot);
        r = make_ray(mk3(so.x, so.y, so.z), mk3(sd.x, sd.y, sd.z), 0.001f, so.w);
        seed = f2u(sd.w);
        node = 0; st.sp = 0;
        active = true;
      }
      ss.head += min(avail, nidle);
      if (!active) break;
    }
    if (!active) continue;
    // one round: walk interior nodes down to a leaf (or to the end of the tree: unoccluded)
    int state = 0;  // 0 running, 1 occluded, 2 unoccluded
    while (node >= 0) {
      Box4 b;
      box4(r, sc, node, r.tmax, b);
      if (STATS) tc.nodes += 4;
      int nxt = -0x7fffffff - 1;
      bool have = false;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (b.tn[j] != __builtin_huge_valf()) {
          if (!have) { nxt = b.c[j]; have = true; }
          else st.push(b.c[j]);
        }
      if (!have) {
        if (st.sp == 0) { state = 2; break; }
        node = st.pop_nz();
        continue;
      }
      node = nxt;
    }
    if (state == 0) {
      const uint32_t L = (uint32_t)(~node);
      const uint32_t start = L & 0x07ffffffu;
      const uint32_t count = (L >> 27) + 1u;
      for (uint32_t k = 0; k < count; ++k) {
        const float4* tp = sc.tris + 3u * (start + k);
        const float4 ta = tp[0], tb = tp[1], tcv = tp[2];
        if (STATS) tc.tris++;
        float t, u, v;
        if (!tri_isect(r, mk3(ta.x, ta.y, ta.z), mk3(tb.x, tb.y, tb.z), mk3(tcv.x, tcv.y, tcv.z), t, u, v)) continue;
        if (!(t >= r.tmin && t <= r.tmax)) continue;
        if (sc.has_transparent && (sc.tri_flags[start + k] & 1u)) {
          const bool acc = (TEX && PTGS_WF_AH_CALL_SHADOW) ? anyhit_accept_call(sc, f2u(ta.w), f2u(tb.w), u, v, seed, f2u(tcv.w))
                               : anyhit_accept<TEX>(sc, f2u(ta.w), f2u(tb.w), u, v, seed, f2u(tcv.w));
          if (!acc) continue;
        }
        state = 1;
        break;
      }
      if (state == 0) {
        if (st.sp == 0) state = 2;
        else node = st.pop_nz();
      }
    }
    if (state != 0) {
      if (state == 2) {  // reaches the light: the accumulation with the light's contribution
        const float4 v = ldnt(a.sh_acc + slot);
        float* dst = reinterpret_cast<float*>(a.st_acc + slot);
        dst[0] = v.x; dst[1] = v.y; dst[2] = v.z;
      }
      a.flags[slot] &= (uint8_t)~WF_SHADOW;
      traced++;
      active = false;
    }
  }
  block_count(a.part, a.part_stride, 1, traced, s_red);  // shadow rays
  if (STATS) {
    block_count(a.part, a.part_stride, 3, tc.nodes, s_red);
    block_count(a.part, a.part_stride, 4, tc.tris, s_red);
  }
}

// ------------------------------------------------------------------------------------------------
// raygen_camera.rgen:80-87: running mean (or SUM for the sample shard) of the batch's samples, in
// sample order, one work-item per pixel
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pt_wf_accumulate_kernel(WfArgs a, uint32_t mode, float4* __restrict__ accum) {
  const uint32_t p = blockIdx.x * 256u + threadIdx.x;  // tile * 64 + lane
  const uint32_t t = p >> 6, l = p & 63u;
  const uint32_t x = (t % a.tiles_x) * 8u + (l & 7u), y = a.row0 + (t / a.tiles_x) * 8u + (l >> 3);
  if (t >= a.slots / (64u * a.batch) || x >= a.W || y >= a.row1) return;
  const size_t pix = (size_t)y * a.W + x;
  float4 prev = accum[pix];
  v3 st = mk3(prev.x, prev.y, prev.z);
  float sa = prev.w;
  for (uint32_t smp = 0; smp < a.batch; ++smp) {
    const uint32_t frame = a.frame0 + smp * a.stride;
    const float4 s = ldnt(a.st_acc + ((size_t)t * a.batch + smp) * 64u + l);
    const v3 acc = mk3(s.x, s.y, s.z);
    if (mode == PTGS_ACCUM_SUM) {
      st = st + acc;
      sa = sa + 1.0f;
    } else if (frame > 0) {
      st = mix3(st, acc, 1.0f / (float)(frame + 1u));
    } else {
      st = acc;
    }
  }
  accum[pix] = make_float4(st.x, st.y, st.z, mode == PTGS_ACCUM_SUM ? sa : 1.0f);
}

// the per-workgroup partial counts of one call -> the context's counters, reset for the next call
__global__ __launch_bounds__(256) void pt_wf_fold_kernel(uint32_t* __restrict__ part, uint32_t stride,
                                                         unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long s_sum[4];
  for (uint32_t k = 0; k < WF_NCNT; ++k) {
    unsigned long long v = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < stride; i += gridDim.x * 256u) {
      v += part[k * stride + i];
      part[k * stride + i] = 0u;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane_id() == 0) s_sum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long t = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
      if (t) atomicAdd(counters + k, t);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static hipError_t wf_ensure(void*& p, size_t& have, size_t bytes, bool zero, hipStream_t s) {
  if (have >= bytes) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  have = 0;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) return e;
  have = bytes;
  return zero ? hipMemsetAsync(p, 0, bytes, s) : hipSuccess;
}

void wf_workspace_free(WfWorkspace& w) {
  for (void** p : {&w.slots, &w.part, &w.ovf})
    if (*p) (void)hipFree(*p);
  w = WfWorkspace{};
}

static uint32_t wf_env(const char* name, uint32_t dflt) {  // tuning / debugging overrides (multiple of 64)
  const char* e = getenv(name);
  const long v = e ? strtol(e, nullptr, 10) : 0;
  return v >= 64 ? (uint32_t)(std::min(v, 65536L) & ~63L) : dflt;  // (ring offsets are 16-bit)
}

hipError_t launch_pt_wavefront(WfWorkspace& w, const DevScene& sc, const CamParams& cp, float* accum, uint32_t W,
                               uint32_t H, uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0,
                               uint32_t stride, uint32_t mode, unsigned long long* counters, bool stats,
                               hipStream_t s) {
  if (row1 <= row0 || spp == 0) return hipSuccess;
  static const uint32_t trace_run = wf_env("PTGS_WF_TRACE_RUN", PTGS_WF_TRACE_RUN);
  static const uint32_t shade_run = wf_env("PTGS_WF_SHADE_RUN", PTGS_WF_SHADE_RUN);
  static const uint32_t refill = [] {  // idle lanes that trigger a refill (1..64)
    const char* e = getenv("PTGS_WF_REFILL");
    const long v = e ? strtol(e, nullptr, 10) : 0;
    return v >= 1 && v <= 64 ? (uint32_t)v : (uint32_t)PTGS_WF_REFILL;
  }();
  static const uint32_t batch_max = [] {  // samples per batch (tile-adjacent slots)
    const char* e = getenv("PTGS_WF_BATCH");
    const long v = e ? strtol(e, nullptr, 10) : 0;
    return v >= 1 && v <= 256 ? (uint32_t)v : (uint32_t)PTGS_WF_BATCH;
  }();
  WfArgs a;
  a.W = W; a.H = H; a.row0 = row0; a.row1 = row1;
  a.tiles_x = (W + 7u) / 8u;
  a.stride = stride;
  const uint32_t tiles = a.tiles_x * ((row1 - row0 + 7u) / 8u);
  // samples per batch: up to batch_max, within ~2^25 slots (145 B each: 4.9 GB at the cap)
  const uint32_t bcap = std::max(1u, (uint32_t)((1u << 25) / ((size_t)tiles * 64u)));
  const uint32_t bmax = std::min({batch_max, spp, bcap});
  const size_t Pmax = (size_t)tiles * 64u * bmax;
  if (Pmax >= (1ull << 32)) return hipErrorInvalidValue;
  const uint32_t grid_pmax = (uint32_t)((Pmax + 255u) / 256u);
  a.part_stride = grid_pmax;  // the largest grid of any stage (runs are >= 64 slots per wave)
  hipError_t e;
  // 9 float4 streams (ray o / d, hit, shadow o / d / acc, path throughput / weight / acc) + 1 flag byte per slot
  if ((e = wf_ensure(w.slots, w.slots_bytes, Pmax * (9 * 16 + 1), false, s))) return e;
  // the per-depth "work pending" words (2 per depth), then the partial counts [WF_NCNT][part_stride]
  if ((e = wf_ensure(w.part, w.part_bytes, ((size_t)WF_NCNT * a.part_stride + 64) * 4, true, s))) return e;
  {  // traversal-stack overflow: the entries beyond the LDS part, per work-item of the largest grid
    const int deep = PTGS_STACK_TOTAL - std::min(PTGS_WF_LDS_EXT, PTGS_WF_LDS_SHADOW);
    const size_t grid_tmax = (Pmax + 4u * trace_run - 1u) / (4u * trace_run);
    if (deep > 0 && (e = wf_ensure(w.ovf, w.ovf_bytes, grid_tmax * 256u * (size_t)deep * 4u, false, s))) return e;
    a.ovf = deep > 0 ? (int*)w.ovf : nullptr;
  }
  float4* f = (float4*)w.slots;
  const size_t P = Pmax;
  a.ray_o = f; a.ray_d = f + P; a.hits = f + 2 * P;
  a.sh_o = f + 3 * P; a.sh_d = f + 4 * P; a.sh_acc = f + 5 * P;
  a.st_thr = f + 6 * P; a.st_w = f + 7 * P; a.st_acc = f + 8 * P;
  a.flags = (uint8_t*)(f + 9 * P);
  // the "work pending" words first: at a fixed offset, so a later call with a larger grid (stride)
  // never counts a previous call's flags as partial ray counts
  a.live = (uint32_t*)w.part;
  a.part = a.live + 64;
  const bool tex = sc.uses_textures != 0;
  auto ext = stats ? (tex ? pt_wf_extend_kernel<true, true> : pt_wf_extend_kernel<true, false>)
                   : (tex ? pt_wf_extend_kernel<false, true> : pt_wf_extend_kernel<false, false>);
  auto shd = stats ? (tex ? pt_wf_shadow_kernel<true, true> : pt_wf_shadow_kernel<true, false>)
                   : (tex ? pt_wf_shadow_kernel<false, true> : pt_wf_shadow_kernel<false, false>);
  auto shade = tex ? pt_wf_shade_kernel<true> : pt_wf_shade_kernel<false>;
  for (uint32_t smp = 0; smp < spp; smp += a.batch) {
    a.batch = std::min(bmax, spp - smp);
    a.frame0 = frame0 + smp * stride;
    a.slots = tiles * 64u * a.batch;
    const uint32_t grid_p = (a.slots + 255u) / 256u;
    const uint32_t grid_t = (a.slots + 4u * trace_run - 1u) / (4u * trace_run);
    const uint32_t grid_s = (a.slots + 4u * shade_run - 1u) / (4u * shade_run);
    hipLaunchKernelGGL(pt_wf_raygen_kernel, dim3(grid_p), dim3(256), 0, s, sc, cp, a);
    for (uint32_t d = 0; d < WF_MAX_DEPTH; ++d) {
      hipLaunchKernelGGL(ext, dim3(grid_t), dim3(256), 0, s, sc, a, d, trace_run, refill);
      hipLaunchKernelGGL(shade, dim3(grid_s), dim3(256), 0, s, sc, cp, a, d, shade_run);
      hipLaunchKernelGGL(shd, dim3(grid_t), dim3(256), 0, s, sc, a, d, trace_run, refill);
    }
    hipLaunchKernelGGL(pt_wf_accumulate_kernel, dim3((tiles * 64u + 255u) / 256u), dim3(256), 0, s, a, mode,
                       (float4*)accum);
  }
  hipLaunchKernelGGL(pt_wf_fold_kernel, dim3(std::min(256u, (a.part_stride + 255u) / 256u)), dim3(256), 0, s, a.part,
                     a.part_stride, counters);
  return hipGetLastError();
}

}  // namespace ptgs
