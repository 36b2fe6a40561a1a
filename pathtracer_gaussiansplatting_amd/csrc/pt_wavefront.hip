// pt_wavefront.hip — wavefront path tracer for ptgs_trace_camera (gfx950).
//
// The per-pixel loop of raygen_camera.rgen:17-88 (one work-item carrying a path through every
// bounce, pt_kernels.hip's pt_camera_kernel) split into stages connected by compacted queues in HBM:
//
//   raygen     one work-item per pixel of the row range: the jittered camera ray (:19-41), the path
//              state (:43-48), the ray appended to the extension queue
//   extend     closest hit of every queued ray (:51). Persistent per-lane refill: each wave owns a
//              contiguous run of the queue and a lane whose traversal ended takes the next ray of the
//              run at once (ballot + mbcnt), so lanes do not idle behind the wave's longest traversal
//   shade      miss.rmiss / closesthit.rchit:324-621 on the hit: emission, NEE query, BSDF sample; the
//              bounce bookkeeping of :53-78 (accumulate + clamp, adaptive depth, throughput, RR); live
//              paths appended to the next extension queue, NEE shadow rays to the shadow queue (ballot +
//              prefix within the wave, one atomic per wave)
//   shadow     any-hit of every queued shadow ray (closesthit.rchit:115-126), same refill scheme; an
//              unoccluded ray selects the accumulation that includes the light (precomputed by shade)
//   accumulate the running mean / sum of :80-87 per pixel, in sample order
//
// Every path computes exactly what pt_camera_kernel computes for it (same device functions, same
// seed sequence: the BLEND any-hit hash reads the seed of the bounce, RR advances it after), so the
// images, ray counts and statistics are bit-identical to the megakernel and to the CPU oracle.
//
// Memory (per pixel slot, SoA float4 for 16-B coalesced accesses): two extension queues of 32 B
// ((origin, slot) (direction, seed)), hits 16 B (t, u, v, gid) by queue position, shadow records
// 48 B ((origin, tmax) (direction, seed) (acc if unoccluded, slot)), path state 48 B
// ((throughput, last_pdf) (weight, hit_flag) (acc, max_depth)).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "pt_shade.h"
#include "pt_wavefront.h"

namespace ptgs {

namespace {

constexpr int WF_DONE = 0x7fffffff;
constexpr uint32_t WF_MAX_DEPTH = 12;  // raygen_camera.rgen:46 max_depth

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// position of this lane's element in a queue (wave-aggregated: one atomic per wave); every lane of
// the wave that reaches the call must call it
__device__ __forceinline__ uint32_t wave_append(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m == 0) return 0;
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  uint32_t base = 0;
  if (lane_id() == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, (int)leader);
  return base + mbcnt64(m);
}

__device__ __forceinline__ unsigned long long wave_sum64(uint32_t v) {
  unsigned long long x = v;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

__device__ __forceinline__ void flush(unsigned long long* counters, int k, uint32_t v) {
  const unsigned long long s = wave_sum64(v);
  if (lane_id() == 0 && s) atomicAdd(counters + k, s);
}

// slot -> pixel: 8x8 pixel tiles in row-major tile order over the row range (a wave = one tile)
__device__ __forceinline__ void slot_pixel(uint32_t slot, uint32_t tiles_x, uint32_t row0, uint32_t& x, uint32_t& y) {
  const uint32_t t = slot >> 6, l = slot & 63u;
  x = (t % tiles_x) * 8u + (l & 7u);
  y = row0 + (t / tiles_x) * 8u + (l >> 3);
}

__device__ __forceinline__ float u2f(uint32_t u) { return __uint_as_float(u); }

}  // namespace

// ------------------------------------------------------------------------------------------------
// raygen_camera.rgen:19-48: primary rays of sample `frame` for every pixel of the row range
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pt_wf_raygen_kernel(DevScene sc, CamParams cp, WfArgs a, uint32_t frame,
                                                           float4* __restrict__ q, uint32_t* __restrict__ cnt,
                                                           unsigned long long* counters) {
  const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
  uint32_t x, y;
  slot_pixel(slot, a.tiles_x, a.row0, x, y);
  const bool valid = slot < a.slots && x < a.W && y < a.row1;
  v3 ro = mk3(0.0f), rd = mk3(0.0f);
  uint32_t seed = 0;
  if (valid) {
    float4 blue;
    primary_ray(sc, cp, x, y, a.W, a.H, frame, ro, rd, blue, seed);
    // throughput 1, last_pdf 0 | weight 1, hit_flag 0 | acc 0, max_depth 12 (:43-48)
    a.st_thr[slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    a.st_w[slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    a.st_acc[slot] = make_float4(0.0f, 0.0f, 0.0f, (float)WF_MAX_DEPTH);
  }
  const uint32_t at = wave_append(cnt, valid);
  if (valid) {
    q[2u * at] = make_float4(ro.x, ro.y, ro.z, u2f(slot));
    q[2u * at + 1u] = make_float4(rd.x, rd.y, rd.z, u2f(seed));
  }
  flush(counters, 2, valid ? 1u : 0u);  // samples
}

// ------------------------------------------------------------------------------------------------
// extend: closest hit of queue entries [0, *cnt) (raygen_camera.rgen:51, pt_device.h trace_closest)
// ------------------------------------------------------------------------------------------------
template <bool STATS, bool TEX>
__global__ __launch_bounds__(256, 4) void pt_wf_extend_kernel(DevScene sc, const float4* __restrict__ q,
                                                              const uint32_t* __restrict__ cnt, uint32_t per_wave,
                                                              float4* __restrict__ hits,
                                                              unsigned long long* counters) {
  __shared__ int s_stack[PTGS_STACK * PTGS_BLOCK];
  int* stack = s_stack + threadIdx.x;
  const uint32_t n = *cnt;
  uint32_t next = (blockIdx.x * 4u + (threadIdx.x >> 6)) * per_wave;  // this wave's run of the queue
  const uint32_t end = min(n, next + per_wave);
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  uint32_t traced = 0;
#ifdef PTGS_WF_DIRECT_CLOSEST
  for (uint32_t k = next + lane_id(); k < end; k += 64u) {
    const float4 qa = q[2u * k], qb = q[2u * k + 1u];
    const Ray rr = make_ray(mk3(qa.x, qa.y, qa.z), mk3(qb.x, qb.y, qb.z), 0.001f, 10000.0f);
    const Hit hh = trace_closest<STATS, TEX>(sc, rr, f2u(qb.w), stack, tc);
    hits[k] = make_float4(hh.t, hh.u, hh.v, u2f(hh.gid));
    if (STATS && hh.gid != 0xffffffffu) tc.hits++;
    traced++;
  }
  next = end;
#endif
  if (next < end) {
    bool active = false;
    uint32_t idx = 0, seed = 0;
    Ray r = make_ray(mk3(0.0f), mk3(1.0f), 0.001f, 10000.0f);
    Hit h; h.t = 0.f; h.u = 0.f; h.v = 0.f; h.gid = 0xffffffffu; h.slot = 0;
    int node = WF_DONE, sp = 0, leaf = WF_DONE;
    auto push = [&](int v) { stack[(sp++) * PTGS_BLOCK] = v; };
    auto pop = [&]() -> int { return sp ? stack[(--sp) * PTGS_BLOCK] : WF_DONE; };
    for (;;) {
      // refill the lanes whose ray finished with the next rays of the run
      const unsigned long long idle = __ballot(!active);
      if (idle != 0 && next < end) {
        const uint32_t k = next + mbcnt64(idle);
        if (!active && k < end) {
          idx = k;
          const float4 qa = q[2u * k], qb = q[2u * k + 1u];
          r = make_ray(mk3(qa.x, qa.y, qa.z), mk3(qb.x, qb.y, qb.z), 0.001f, 10000.0f);
          seed = f2u(qb.w);
          h.t = r.tmax; h.u = 0.f; h.v = 0.f; h.gid = 0xffffffffu;
          node = 0; sp = 0; leaf = WF_DONE;
          active = true;
        }
        next += (uint32_t)__popcll(idle);
      }
      if (!active) break;  // the run is exhausted for this lane
      // one round of the while-while walk (postponed leaves, as trace_closest)
      while (node >= 0 && node != WF_DONE) {
        Box4 b;
        box4(r, sc.nodes + 8 * node, h.t, b);
        if (STATS) tc.nodes += 4;
        if (b.hits == 0) {
          node = pop();
        } else {
          cswap4(b, 0, 1); cswap4(b, 2, 3); cswap4(b, 0, 2); cswap4(b, 1, 3); cswap4(b, 1, 2);
          if (b.hits > 3) push(b.c[3]);
          if (b.hits > 2) push(b.c[2]);
          if (b.hits > 1) push(b.c[1]);
          node = b.c[0];
        }
        if (node < 0 && leaf == WF_DONE) {
          leaf = node;
          node = pop();
        }
#if defined(PTGS_WF_DBG_NOALL)
        if (leaf != WF_DONE) break;
#elif defined(PTGS_WF_DBG_BALLOT)
        if (__ballot(leaf != WF_DONE || node == WF_DONE) == __ballot(1)) break;
#else
        if (__all(leaf != WF_DONE || node == WF_DONE)) break;
#endif
      }
      if (leaf != WF_DONE) {
        leaf_closest<STATS, TEX, true>(sc, r, leaf, h, seed, tc);
        leaf = WF_DONE;
      }
      if (node < 0) {
        leaf_closest<STATS, TEX, true>(sc, r, node, h, seed, tc);
        node = pop();
      }
      if (node == WF_DONE) {
        hits[idx] = make_float4(h.t, h.u, h.v, u2f(h.gid));
        if (STATS && h.gid != 0xffffffffu) tc.hits++;
        traced++;
        active = false;
      }
    }
  }
  flush(counters, 0, traced);  // extension rays
  if (STATS) { flush(counters, 3, tc.nodes); flush(counters, 4, tc.tris); flush(counters, 5, tc.hits); }
}

// ------------------------------------------------------------------------------------------------
// shade: miss / closest hit + the bounce bookkeeping of raygen_camera.rgen:53-78 for depth `depth`
// ------------------------------------------------------------------------------------------------
template <bool TEX>
__global__ __launch_bounds__(256) void pt_wf_shade_kernel(DevScene sc, CamParams cp, WfArgs a, uint32_t frame,
                                                          uint32_t depth, const float4* __restrict__ q,
                                                          const uint32_t* __restrict__ cnt,
                                                          const float4* __restrict__ hits, float4* __restrict__ qn,
                                                          uint32_t* __restrict__ cnt_next, float4* __restrict__ sh,
                                                          uint32_t* __restrict__ cnt_sh) {
  const uint32_t n = *cnt;
  ShadeCtx c; c.sc = &sc; c.cp = &cp; c.stack = nullptr; c.shadow_rays = 0;
  for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {  // wave-uniform bound
    const uint32_t i = base + threadIdx.x;
    const bool ok = i < n;
    bool alive = false, traced = false;
    uint32_t slot = 0, seed_sh = 0;
    v3 ro = mk3(0.0f), rd = mk3(0.0f), acc_vis = mk3(0.0f);  // next extension ray; shadow record
    ShadowQuery sq;
    sq.flags = 0;
    uint32_t seed = 0;
    if (ok) {
      const float4 qa = q[2u * i], qb = q[2u * i + 1u];
      const float4 hv = hits[i];
      slot = f2u(qa.w);
      const float4 s_thr = a.st_thr[slot], s_w = a.st_w[slot], s_acc = a.st_acc[slot];
      uint32_t x, y;
      slot_pixel(slot, a.tiles_x, a.row0, x, y);
      const float4 blue = blue_noise_texel(sc, x, y, frame);
      Payload p;
      p.seed = f2u(qb.w);
      p.blue = mk2(blue.z, blue.w);
      p.last_pdf = s_thr.w;
      p.hit_flag = s_w.w;
      p.weight = mk3(s_w.x, s_w.y, s_w.z);
      p.color = mk3(0.0f);
      p.next_o = mk3(qa.x, qa.y, qa.z);
      p.next_d = mk3(qb.x, qb.y, qb.z);
      p.depth = (int)depth;
      p.hit_pos = mk3(0.0f); p.normal = mk3(0.0f);
      const Ray ray = make_ray(p.next_o, p.next_d, 0.001f, 10000.0f);
      Hit h; h.t = hv.x; h.u = hv.y; h.v = hv.z; h.gid = f2u(hv.w); h.slot = 0;
      if (h.gid == 0xffffffffu) miss<false>(cp, p);
      else closest_hit<false, TEX>(c, p, ray, h, sq);
      v3 thr = mk3(s_thr.x, s_thr.y, s_thr.z);
      v3 acc = mk3(s_acc.x, s_acc.y, s_acc.z);
      float max_depth = s_acc.w;
      // resolve_shadow's two outcomes (vis = 0 / 1 before max(vis, transmission)): the shadow kernel
      // keeps the occluded accumulation unless the ray reaches the light
      traced = (sq.flags & SQ_TRACE) != 0;
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
        acc_vis = vmin(acc + col_vis * thr, 5.0f);
        seed_sh = p.seed;  // the any-hit seed: before this bounce's RR draw
      }
      acc = vmin(acc + col_occ * thr, 5.0f);
      // :60-78
      alive = !(p.hit_flag < 0.0f);
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
      a.st_acc[slot] = make_float4(acc.x, acc.y, acc.z, max_depth);
      if (alive) {
        a.st_thr[slot] = make_float4(thr.x, thr.y, thr.z, p.last_pdf);
        a.st_w[slot] = make_float4(p.weight.x, p.weight.y, p.weight.z, p.hit_flag);
      }
      seed = p.seed;
      ro = p.next_o;
      rd = p.next_d;
    }
    const uint32_t at = wave_append(cnt_next, alive);
    if (alive) {
      qn[2u * at] = make_float4(ro.x, ro.y, ro.z, u2f(slot));
      qn[2u * at + 1u] = make_float4(rd.x, rd.y, rd.z, u2f(seed));
    }
    const uint32_t as = wave_append(cnt_sh, traced);
    if (traced) {
      sh[3u * as] = make_float4(sq.o.x, sq.o.y, sq.o.z, sq.tmax);
      sh[3u * as + 1u] = make_float4(sq.d.x, sq.d.y, sq.d.z, u2f(seed_sh));
      sh[3u * as + 2u] = make_float4(acc_vis.x, acc_vis.y, acc_vis.z, u2f(slot));
    }
  }
}

// ------------------------------------------------------------------------------------------------
// shadow: any-hit of queued NEE rays (pt_device.h trace_any); unoccluded -> the "visible" accumulation
// ------------------------------------------------------------------------------------------------
template <bool STATS, bool TEX>
__global__ __launch_bounds__(256, 4) void pt_wf_shadow_kernel(DevScene sc, WfArgs a, const float4* __restrict__ sh,
                                                              const uint32_t* __restrict__ cnt, uint32_t per_wave,
                                                              unsigned long long* counters) {
  __shared__ int s_stack[PTGS_STACK * PTGS_BLOCK];
  int* stack = s_stack + threadIdx.x;
  const uint32_t n = *cnt;
  uint32_t next = (blockIdx.x * 4u + (threadIdx.x >> 6)) * per_wave;
  const uint32_t end = min(n, next + per_wave);
  TraversalCounters tc; tc.nodes = 0; tc.tris = 0; tc.hits = 0;
  uint32_t traced = 0;
#ifdef PTGS_WF_DIRECT_ANY
  for (uint32_t k = next + lane_id(); k < end; k += 64u) {
    const float4 sa = sh[3u * k], sb = sh[3u * k + 1u];
    const Ray rr = make_ray(mk3(sa.x, sa.y, sa.z), mk3(sb.x, sb.y, sb.z), 0.001f, sa.w);
    if (!trace_any<STATS, TEX>(sc, rr, f2u(sb.w), stack, tc)) {
      const float4 sc2 = sh[3u * k + 2u];
      float* dst = reinterpret_cast<float*>(a.st_acc + f2u(sc2.w));
      dst[0] = sc2.x; dst[1] = sc2.y; dst[2] = sc2.z;
    }
    traced++;
  }
  next = end;
#endif
  if (next < end) {
    bool active = false;
    uint32_t idx = 0, seed = 0;
    Ray r = make_ray(mk3(0.0f), mk3(1.0f), 0.001f, 1.0f);
    int node = 0, sp = 0;
    for (;;) {
      const unsigned long long idle = __ballot(!active);
      if (idle != 0 && next < end) {
        const uint32_t k = next + mbcnt64(idle);
        if (!active && k < end) {
          idx = k;
          const float4 sa = sh[3u * k], sb = sh[3u * k + 1u];
          r = make_ray(mk3(sa.x, sa.y, sa.z), mk3(sb.x, sb.y, sb.z), 0.001f, sa.w);
          seed = f2u(sb.w);
          node = 0; sp = 0;
          active = true;
        }
        next += (uint32_t)__popcll(idle);
      }
      if (!active) break;
      // one round: walk interior nodes down to a leaf (or to the end of the tree: unoccluded)
      int state = 0;  // 0 running, 1 occluded, 2 unoccluded
      while (node >= 0) {
        Box4 b;
        box4(r, sc.nodes + 8 * node, r.tmax, b);
        if (STATS) tc.nodes += 4;
        int nxt = -0x7fffffff - 1;
        bool have = false;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (b.tn[j] != __builtin_huge_valf()) {
            if (!have) { nxt = b.c[j]; have = true; }
            else stack[(sp++) * PTGS_BLOCK] = b.c[j];
          }
        if (!have) {
          if (sp == 0) { state = 2; break; }
          node = stack[(--sp) * PTGS_BLOCK];
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
            if (!anyhit_accept<TEX>(sc, f2u(ta.w), f2u(tb.w), u, v, seed, f2u(tcv.w))) continue;
          }
          state = 1;
          break;
        }
        if (state == 0) {
          if (sp == 0) state = 2;
          else node = stack[(--sp) * PTGS_BLOCK];
        }
      }
      if (state != 0) {
        if (state == 2) {  // reaches the light: the accumulation with the light's contribution
          const float4 sc2 = sh[3u * idx + 2u];
          const uint32_t slot = f2u(sc2.w);
          float* dst = reinterpret_cast<float*>(a.st_acc + slot);
          dst[0] = sc2.x; dst[1] = sc2.y; dst[2] = sc2.z;
        }
        traced++;
        active = false;
      }
    }
  }
  flush(counters, 1, traced);  // shadow rays
  if (STATS) { flush(counters, 3, tc.nodes); flush(counters, 4, tc.tris); }
}

// ------------------------------------------------------------------------------------------------
// raygen_camera.rgen:80-87: running mean (or SUM for the sample shard) of the finished sample
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pt_wf_accumulate_kernel(WfArgs a, uint32_t frame, uint32_t mode,
                                                               float4* __restrict__ accum) {
  const uint32_t slot = blockIdx.x * 256u + threadIdx.x;
  uint32_t x, y;
  slot_pixel(slot, a.tiles_x, a.row0, x, y);
  if (slot >= a.slots || x >= a.W || y >= a.row1) return;
  const size_t pix = (size_t)y * a.W + x;
  const float4 s = a.st_acc[slot];
  const v3 acc = mk3(s.x, s.y, s.z);
  if (mode == PTGS_ACCUM_SUM) {
    const float4 prev = accum[pix];
    const v3 st = mk3(prev.x, prev.y, prev.z) + acc;
    accum[pix] = make_float4(st.x, st.y, st.z, prev.w + 1.0f);
  } else if (frame > 0) {
    const float4 prev = accum[pix];
    const float blend = 1.0f / (float)(frame + 1u);
    const v3 st = mix3(mk3(prev.x, prev.y, prev.z), acc, blend);
    accum[pix] = make_float4(st.x, st.y, st.z, 1.0f);
  } else {
    accum[pix] = make_float4(acc.x, acc.y, acc.z, 1.0f);
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static hipError_t wf_ensure(void*& p, size_t& have, size_t bytes) {
  if (have >= bytes) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  have = 0;
  hipError_t e = hipMalloc(&p, bytes);
  if (e == hipSuccess) have = bytes;
  return e;
}

void wf_workspace_free(WfWorkspace& w) {
  for (void** p : {&w.q[0], &w.q[1], &w.hits, &w.sh, &w.st, &w.cnt})
    if (*p) (void)hipFree(*p);
  w = WfWorkspace{};
}

hipError_t launch_pt_wavefront(WfWorkspace& w, const DevScene& sc, const CamParams& cp, float* accum, uint32_t W,
                               uint32_t H, uint32_t row0, uint32_t row1, uint32_t spp, uint32_t frame0,
                               uint32_t stride, uint32_t mode, unsigned long long* counters, bool stats,
                               hipStream_t s) {
  if (row1 <= row0 || spp == 0) return hipSuccess;
  WfArgs a;
  a.W = W; a.H = H; a.row0 = row0; a.row1 = row1;
  a.tiles_x = (W + 7u) / 8u;
  const uint32_t tiles_y = (row1 - row0 + 7u) / 8u;
  a.slots = a.tiles_x * tiles_y * 64u;
  const size_t P = a.slots;
  hipError_t e;
  if ((e = wf_ensure(w.q[0], w.q_bytes[0], P * 32))) return e;
  if ((e = wf_ensure(w.q[1], w.q_bytes[1], P * 32))) return e;
  if ((e = wf_ensure(w.hits, w.hits_bytes, P * 16))) return e;
  if ((e = wf_ensure(w.sh, w.sh_bytes, P * 48))) return e;
  if ((e = wf_ensure(w.st, w.st_bytes, P * 48))) return e;
  if ((e = wf_ensure(w.cnt, w.cnt_bytes, 2 * (WF_MAX_DEPTH + 1) * sizeof(uint32_t) * 64))) return e;
  a.st_thr = (float4*)w.st;
  a.st_w = a.st_thr + P;
  a.st_acc = a.st_w + P;
  float4* q[2] = {(float4*)w.q[0], (float4*)w.q[1]};
  float4* hits = (float4*)w.hits;
  float4* sh = (float4*)w.sh;
  static const uint32_t per_wave = [] {  // (PTGS_WF_RAYS_PER_WAVE: tuning / debugging override, multiple of 64)
    const char* e = getenv("PTGS_WF_RAYS_PER_WAVE");
    const long v = e ? strtol(e, nullptr, 10) : 0;
    return v >= 64 ? (uint32_t)(v & ~63L) : (uint32_t)PTGS_WF_RAYS_PER_WAVE;
  }();
  const uint32_t grid_t = (uint32_t)((P + 4u * per_wave - 1u) / (4u * per_wave));
  const uint32_t grid_p = (uint32_t)((P + 255u) / 256u);
  const uint32_t grid_s = std::min<uint32_t>(grid_p, PTGS_WF_SHADE_BLOCKS);
  const bool tex = sc.uses_textures != 0;
  auto ext = stats ? (tex ? pt_wf_extend_kernel<true, true> : pt_wf_extend_kernel<true, false>)
                   : (tex ? pt_wf_extend_kernel<false, true> : pt_wf_extend_kernel<false, false>);
  auto shd = stats ? (tex ? pt_wf_shadow_kernel<true, true> : pt_wf_shadow_kernel<true, false>)
                   : (tex ? pt_wf_shadow_kernel<false, true> : pt_wf_shadow_kernel<false, false>);
  auto shade = tex ? pt_wf_shade_kernel<true> : pt_wf_shade_kernel<false>;
  for (uint32_t smp = 0; smp < spp; ++smp) {
    const uint32_t frame = frame0 + smp * stride;
    // per-depth counters, one 256-B line each (ext count at [64 d], shadow count at [64 d + 32])
    uint32_t* cnt = (uint32_t*)w.cnt;
    if ((e = hipMemsetAsync(cnt, 0, 2 * (WF_MAX_DEPTH + 1) * sizeof(uint32_t) * 64, s))) return e;
    hipLaunchKernelGGL(pt_wf_raygen_kernel, dim3(grid_p), dim3(256), 0, s, sc, cp, a, frame, q[0], cnt, counters);
    for (uint32_t d = 0; d < WF_MAX_DEPTH; ++d) {
      uint32_t* ce = cnt + 64u * d;
      uint32_t* cs = ce + 32u;
      uint32_t* cn = cnt + 64u * (d + 1u);
      hipLaunchKernelGGL(ext, dim3(grid_t), dim3(256), 0, s, sc, q[d & 1u], ce, per_wave, hits, counters);
      hipLaunchKernelGGL(shade, dim3(grid_s), dim3(256), 0, s, sc, cp, a, frame, d, q[d & 1u], ce, hits,
                         q[(d + 1u) & 1u], cn, sh, cs);
      hipLaunchKernelGGL(shd, dim3(grid_t), dim3(256), 0, s, sc, a, sh, cs, per_wave, counters);
    }
    hipLaunchKernelGGL(pt_wf_accumulate_kernel, dim3(grid_p), dim3(256), 0, s, a, frame, mode, (float4*)accum);
  }
  return hipGetLastError();
}

}  // namespace ptgs
