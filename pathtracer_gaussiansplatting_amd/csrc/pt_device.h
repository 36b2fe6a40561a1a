// pt_device.h — device-side path-tracing stages for gfx950.
//
// What the Vulkan RT pipeline of the reference does in shaders + fixed function, restated as
// plain HIP device code:
//   traversal  : software BVH2 walk (the reference uses the driver's HW traversal,
//                raygen_camera.rgen:51 / closesthit.rchit:115,124; gfx950 has no BVH instruction,
//                SURVEY.md §0.6) — closest hit with a deterministic tie-break (equal t -> lower
//                triangle id), any-hit for shadow rays.
//   closest_hit: shaders/rt_render/closesthit.rchit:324-621 (+ NEE helpers :113-320)
//   miss       : shaders/rt_render/miss.rmiss:9-14, shadow.rmiss:9-11
//   rnd        : shaders/rt_render/raytracing.glsl:141-146
// All float math goes through detmath.h so results are bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include "detmath.h"
#include "texture.h"
#include "../../include/ptgs/ptgs.h"

namespace ptgs {

// ---------------------------------------------------------------------------------------------
// Device scene (layouts chosen for gfx950: 16-B aligned float4 records, one node = 64 B = half a
// 128-B cache line, triangles pre-gathered as (v0, e1, e2) so traversal never touches the 80-B
// reference vertices).
// ---------------------------------------------------------------------------------------------
struct DevScene {
  const float4* nodes;            // 4 float4 per interior node (see bvh.h)
  const float4* tris;             // 3 float4 per triangle: (v0, mesh_bits) (e1, prim_bits) (e2, gid_bits)
  const uint32_t* tri_flags;      // bit0: non-opaque (any-hit shader runs)
  const ptgs_vertex* vertices;
  const uint32_t* indices;
  const ptgs_mesh_info* meshes;
  const ptgs_material* materials;
  const uint4* hitrec;            // per gid: the 3 global vertex indices + material index (precomputed
                                  // meshes -> indices -> vertices chain of closest_hit)
  const ptgs_light_triangle* light_tris;
  const ptgs_light_cdf* light_cdf;
  const ptgs_punctual_light* plights;
  const ptgs_punctual_cdf* pcdf;
  const float4* blue_noise;
  DevTextures tex;                // global_textures[] (texture.h)
  int32_t uses_textures;          // some material has a texture index > 0: launch the TEX kernels
  int32_t deep_stack;             // the tree's worst-case stack need exceeds PTGS_STACK: launch the
                                  // kernels with the stack overflow (OVF = PTGS_STACK_OVF)
  uint32_t num_light_cdf;
  uint32_t num_plights;
  int32_t bn_size;
  int32_t has_transparent;
};

// UBO fields the shaders read (raytracing.glsl:111-125), with the two matrix inverses the
// ray-gen computes per pixel (raygen_camera.rgen:32-34) precomputed once on the host.
struct CamParams {
  float inv_view[16];
  float inv_proj[16];
  float ambient[4];
  float emissive_flux, punctual_flux, p_emissive;
  float fov, win_height, use_lod, lod_factor;
};

struct Hit {
  float t, u, v;
  uint32_t gid;   // global triangle id (flattening order), 0xffffffff = miss
  uint32_t slot;  // triangle record index in BVH order (mesh/prim are re-fetched from it)
};

struct TraversalCounters {
  uint32_t nodes;  // child-box tests
  uint32_t tris;   // ray-triangle tests
  uint32_t hits;   // closest hits (shaded surface points)
#ifdef PT_LANES
  struct PtLaneCounts* lanes_p;
#endif
};

// PT_LANES builds (tools/pt_lanes.py, diagnostics only): per loop of the path tracer, how many times a wave
// ran it and how many lanes were active in those runs (lane utilisation by phase). g_pt_lanes[2 i] wave
// iterations, [2 i + 1] active lanes summed over them; i: PtLoop. Each work-item counts in registers and
// adds its totals once at the end of the kernel (pt_lanes_flush).
enum PtLoop { PT_L_NODE = 0, PT_L_LEAF, PT_L_TRI, PT_L_ANY_NODE, PT_L_ANY_TRI, PT_L_BOUNCE, PT_L_SAMPLE, PT_L_COUNT };
#ifdef PT_LANES
__device__ unsigned long long g_pt_lanes[2 * PT_L_COUNT];
struct PtLaneCounts {
  uint32_t w[PT_L_COUNT], l[PT_L_COUNT];
};
__device__ __forceinline__ void pt_lane_tick(PtLaneCounts& c, int i) {
  const unsigned long long ex = __builtin_amdgcn_read_exec();
  c.l[i] += 1u;
  if (__lane_id() == (uint32_t)__builtin_ctzll(ex)) c.w[i] += 1u;
}
__device__ __forceinline__ void pt_lanes_flush(const PtLaneCounts& c) {
  for (int i = 0; i < PT_L_COUNT; ++i) {
    atomicAdd(&g_pt_lanes[2 * i], (unsigned long long)c.w[i]);
    atomicAdd(&g_pt_lanes[2 * i + 1], (unsigned long long)c.l[i]);
  }
}
#define PT_LANE_TICK(cnt, i) pt_lane_tick(*(cnt).lanes_p, (i))
#define PT_LANES_INIT(tc) PtLaneCounts tc##_lanes = {}; (tc).lanes_p = &tc##_lanes
#define PT_LANES_FLUSH(tc) pt_lanes_flush(tc##_lanes)
#else
#define PT_LANE_TICK(cnt, i) ((void)0)
#define PT_LANES_INIT(tc) ((void)0)
#define PT_LANES_FLUSH(tc) ((void)0)
#endif

// Traversal stack: PTGS_STACK entries per work-item in LDS, interleaved across the 256 work-items
// of a workgroup (entry k of lane t at [k * 256 + t]: conflict-free ds_read/ds_write_b32).
// 39 x 256 x 4 B = 39 KiB per workgroup (+ 1 KiB of slot rings in the wavefront kernels: 4
// workgroups = 16 waves per CU fill the 160 KiB LDS). Deeper entries, up to PTGS_STACK_TOTAL, go
// to a per-work-item overflow: private (scratch) memory in the megakernel, a global column in the
// wavefront kernels. A 4-wide node pushes up to 3 entries: the scene upload (api.cpp kBvhTries)
// rebuilds with 4-triangle leaves, then caps the fan-out, only if the tree's worst-case stack need
// exceeds PTGS_STACK_TOTAL. C3's 250k-triangle atrium needs 38 with 3-triangle leaves, C5's
// 1M-triangle atrium 40 (tools/native/bvh_need.cpp): both keep 3-triangle leaves and 4-wide nodes.
// The overflow is compiled only into the DEEP kernel instantiations (DevScene::deep_stack: need >=
// PTGS_STACK), launched for C5's tree; C3's runs the LDS-only traversal (the overflow's test per push /
// pop cost 3.4% on C3 even unused, tools/ab_pt.py).
#ifndef PTGS_STACK
#define PTGS_STACK 39
#endif
#ifndef PTGS_STACK_OVF
#define PTGS_STACK_OVF 9  // overflow entries beyond the LDS part
#endif
#define PTGS_STACK_TOTAL (PTGS_STACK + PTGS_STACK_OVF)
#define PTGS_BLOCK 256

PTGS_HD float i2f(int x) { union { int i; float f; } c; c.i = x; return c.f; }
__device__ __forceinline__ int f2i(float x) { return __float_as_int(x); }
__device__ __forceinline__ uint32_t f2u(float x) { return __float_as_uint(x); }

// PCG hash, raytracing.glsl:141-146
__device__ __forceinline__ float rnd(uint32_t& state) {
  uint32_t prev = state;
  state = prev * 747796405u + 2891336453u;
  uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
  return (float)((word >> 22u) ^ word) / 4294967296.0f;
}

// Stateless hash used for stochastic (BLEND) any-hit decisions: the reference draws
// rnd(payload.seed) per candidate hit in driver traversal order (alpha.rahit:58), which no
// software traversal can reproduce; we hash (seed, triangle) instead (documented deviation).
__device__ __forceinline__ float alpha_hash(uint32_t seed, uint32_t gid) {
  uint32_t s = seed ^ (gid * 0x9E3779B9u);
  return rnd(s);
}

__device__ __forceinline__ v3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

// ---------------------------------------------------------------------------------------------
// Ray / box / triangle
// ---------------------------------------------------------------------------------------------
// PTGS_PT_NEARFAR: the box test reads each axis's near and far planes by the ray's direction signs
// (byte offsets in the node, below) instead of ordering both slab distances with a min and a max:
// the same slab values, 24 fewer VALU per 4-wide node
#ifndef PTGS_PT_NEARFAR
#define PTGS_PT_NEARFAR 1
#endif
// PTGS_PT_ASM_MIN: the far slab distance's min in inline asm: the compiler canonicalises the hit
// distance (tcap, a loop-carried value it cannot prove canonical) before every fminf, one VALU per node:
// C3 at 16 spp 5 380 -> 5 414 Mrays/s (tools/ab_pt.py, profiles/r05/pt_tweaks_ab.log). (Counting the hit
// children from the sorted distances instead of a running count measured equal: 5 374.)
#ifndef PTGS_PT_ASM_MIN
#define PTGS_PT_ASM_MIN 1
#endif

struct Ray {
  v3 o, d, inv;
  v3 oinv;  // o * inv: slab distances as one FMA per plane (box tests need conservativeness only)
  float tmin, tmax;
#if PTGS_PT_NEARFAR
  uint32_t nx, ny, nz;  // byte offset in a node of the near plane per axis: lo (0 / 32 / 64) or hi (+16)
#endif
};

__device__ __forceinline__ float safe_inv(float d) {
  const float eps = 1e-20f;
  float a = absx(d) < eps ? (d < 0.0f ? -eps : eps) : d;
  return 1.0f / a;
}

__device__ __forceinline__ Ray make_ray(v3 o, v3 d, float tmin, float tmax) {
  Ray r; r.o = o; r.d = d; r.tmin = tmin; r.tmax = tmax;
  r.inv = mk3(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
  r.oinv = mk3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
#if PTGS_PT_NEARFAR
  // inv > 0: fma(lo, inv, -oinv) <= fma(hi, inv, -oinv) (the rounded FMA is monotone in lo / hi), so
  // the near plane is lo; inv < 0: hi (inv is never 0: safe_inv)
  r.nx = r.inv.x < 0.0f ? 16u : 0u;
  r.ny = r.inv.y < 0.0f ? 48u : 32u;
  r.nz = r.inv.z < 0.0f ? 80u : 64u;
#endif
  return r;
}

// Moller-Trumbore, double-sided (TriangleFacingCullDisable, engine.cpp:1460). Operation order is
// part of the parity contract with the oracle (oracle/ptgs_oracle.c: tri_intersect).
__device__ __forceinline__ bool tri_isect(const Ray& r, v3 v0, v3 e1, v3 e2, float& t, float& u, float& v) {
  v3 pvec = cross3(r.d, e2);
  float det = dot3(e1, pvec);
  if (det == 0.0f) return false;
  float inv_det = 1.0f / det;
  v3 tvec = r.o - v0;
  u = dot3(tvec, pvec) * inv_det;
  if (u < 0.0f || u > 1.0f) return false;
  v3 qvec = cross3(tvec, e1);
  v = dot3(r.d, qvec) * inv_det;
  if (v < 0.0f || u + v > 1.0f) return false;
  t = dot3(e2, qvec) * inv_det;
  return true;
}

// ---------------------------------------------------------------------------------------------
// Materials / any-hit (alpha.rahit:14-61, untextured alpha = base_color_factor.a)
// ---------------------------------------------------------------------------------------------
// TEX = false: no material of the scene references a texture (scene flag), the texture branch is
// compiled out (it costs the path-tracer kernel registers even when never taken)
template <bool TEX>
__device__ __forceinline__ bool anyhit_accept(const DevScene& sc, uint32_t mesh, uint32_t prim, float u, float v,
                                              uint32_t seed, uint32_t gid) {
  const ptgs_mesh_info info = sc.meshes[mesh];
  const ptgs_material& m = sc.materials[info.material_index];
  float alpha_cutoff = m.alpha_cutoff;
  bool is_blend = m.pad > 0.5f;
  if (alpha_cutoff == 0.0f && !is_blend) return true;
  float alpha = m.base_color_factor[3];
  if (TEX && m.albedo_texture_index > 0) {  // alpha.rahit:28-45: interpolated UV, LOD 0
    const uint32_t i0 = sc.indices[info.index_offset + prim * 3u + 0u];
    const uint32_t i1 = sc.indices[info.index_offset + prim * 3u + 1u];
    const uint32_t i2 = sc.indices[info.index_offset + prim * 3u + 2u];
    const ptgs_vertex& v0 = sc.vertices[info.vertex_offset + i0];
    const ptgs_vertex& v1 = sc.vertices[info.vertex_offset + i1];
    const ptgs_vertex& v2 = sc.vertices[info.vertex_offset + i2];
    const float bx = (1.0f - u) - v;
    const float tu = (v0.tex_coord[0] * bx + v1.tex_coord[0] * u) + v2.tex_coord[0] * v;
    const float tv = (v0.tex_coord[1] * bx + v1.tex_coord[1] * u) + v2.tex_coord[1] * v;
    alpha = alpha * sample_texture(sc.tex, m.albedo_texture_index, tu, tv, 0.0f).w;
  }
  if (alpha_cutoff > 0.0f) return !(alpha < alpha_cutoff);
  return !(alpha_hash(seed, gid) > alpha);
}

// Out-of-line any-hit (PTGS_WF_AH_CALL=true builds of pt_wavefront.hip). Round 2 used it to sidestep
// a miscompile of the inlined textured any-hit in the wavefront extend kernel; root-caused in round 3
// (opt-bisect): the SLP vectorizer's horizontal-reduction seeding vectorizes the refill loop's
// ray-state phis and changes the traced rays; build.py compiles pt_wavefront.hip with
// -slp-vectorize-hor=false and inlines the any-hit.
__device__ __noinline__ bool anyhit_accept_call(const DevScene& sc, uint32_t mesh, uint32_t prim, float u, float v,
                                                uint32_t seed, uint32_t gid) {
  return anyhit_accept<true>(sc, mesh, prim, u, v, seed, gid);
}

// ---------------------------------------------------------------------------------------------
// Traversal
// ---------------------------------------------------------------------------------------------
template <bool STATS, bool TEX, bool AH_CALL = false>
__device__ __forceinline__ void leaf_closest(const DevScene& sc, const Ray& r, int leaf, Hit& h,
                                             uint32_t seed, TraversalCounters& cnt) {
  uint32_t L = (uint32_t)(~leaf);
  uint32_t start = L & 0x07ffffffu;
  uint32_t count = (L >> 27) + 1u;
  // the next triangle's 48 B are in flight while this one is tested (+3%)
  float4 na = sc.tris[3u * start], nb = sc.tris[3u * start + 1u], nc = sc.tris[3u * start + 2u];
  for (uint32_t k = 0; k < count; ++k) {
    PT_LANE_TICK(cnt, PT_L_TRI);
    float4 a = na, b = nb, c = nc;
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w),
                      "+v"(c.x), "+v"(c.y), "+v"(c.z), "+v"(c.w));
    if (k + 1 < count) {
      const float4* tn = sc.tris + 3u * (start + k + 1u);
      na = tn[0]; nb = tn[1]; nc = tn[2];
    }
    if (STATS) cnt.tris++;
    float t, u, v;
    if (!tri_isect(r, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), mk3(c.x, c.y, c.z), t, u, v)) continue;
    if (!(t >= r.tmin && t <= h.t)) continue;
    uint32_t gid = f2u(c.w);
    if (t == h.t && gid >= h.gid) continue;
    if (sc.has_transparent && (sc.tri_flags[start + k] & 1u)) {
      const bool acc = (AH_CALL && TEX) ? anyhit_accept_call(sc, f2u(a.w), f2u(b.w), u, v, seed, gid)
                                        : anyhit_accept<TEX>(sc, f2u(a.w), f2u(b.w), u, v, seed, gid);
      if (!acc) continue;
    }
    h.t = t; h.u = u; h.v = v; h.gid = gid; h.slot = start + k;
  }
}

// 4-wide nodes (bvh.h collapse_bvh4): one 112-B fetch tests four child boxes; hit children are put
// in near-to-far order by a 5-comparator network, the nearest is entered and the rest pushed
// farthest first. The slab test is lo * inv - o * inv as one FMA per plane: the host pads every box
// by >= 4e-7 x the scene's coordinate scale, which covers the extra rounding of o * inv, so the test
// is conservative w.r.t. the triangle test and the hits do not depend on the tree.
struct Box4 {
  float tn[4];
  int c[4];
  unsigned long long hm[4];  // per child, the wave's lanes whose ray hits it (SGPR masks: the hit-count logic of
                             // enter_box4 runs on the scalar unit instead of a per-lane count in VGPRs)
};
#if PTGS_PT_NEARFAR
__device__ __forceinline__ float4 node_ld(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ void box4(const Ray& r, const DevScene& sc, int node, float tcap, Box4& o) {
  // 32-bit byte offsets through a buffer descriptor (built from the kernel argument: wave-uniform):
  // one v_lshl_add per axis for the near plane, the far plane is 16 B beside it
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sc.nodes, 0, 0x7fffffff, 0x00020000);
  const uint32_t base = (uint32_t)node << 7;
  const uint32_t ox = base + r.nx, oy = base + r.ny, oz = base + r.nz;
  const float4 nx = node_ld(rs, ox), fx = node_ld(rs, ox ^ 16u);
  const float4 ny = node_ld(rs, oy), fy = node_ld(rs, oy ^ 16u);
  const float4 nz = node_ld(rs, oz), fz = node_ld(rs, oz ^ 16u);
  float4 ch = node_ld(rs, base + 96u);
  asm volatile("" : "+v"(ch.x), "+v"(ch.y), "+v"(ch.z), "+v"(ch.w));  // (pinned: box4 below)
  const float NX[4] = {nx.x, nx.y, nx.z, nx.w}, FX[4] = {fx.x, fx.y, fx.z, fx.w};
  const float NY[4] = {ny.x, ny.y, ny.z, ny.w}, FY[4] = {fy.x, fy.y, fy.z, fy.w};
  const float NZ[4] = {nz.x, nz.y, nz.z, nz.w}, FZ[4] = {fz.x, fz.y, fz.z, fz.w};
  const float CH[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = __builtin_fmaf(NX[j], r.inv.x, -r.oinv.x), x1 = __builtin_fmaf(FX[j], r.inv.x, -r.oinv.x);
    const float y0 = __builtin_fmaf(NY[j], r.inv.y, -r.oinv.y), y1 = __builtin_fmaf(FY[j], r.inv.y, -r.oinv.y);
    const float z0 = __builtin_fmaf(NZ[j], r.inv.z, -r.oinv.z), z1 = __builtin_fmaf(FZ[j], r.inv.z, -r.oinv.z);
    const float tn = fmaxf(fmaxf(x0, y0), fmaxf(z0, r.tmin));
#if PTGS_PT_ASM_MIN
    float tf;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(tf) : "v"(x1), "v"(y1), "v"(z1));
    asm("v_min_f32 %0, %1, %2" : "=v"(tf) : "v"(tf), "v"(tcap));
#else
    const float tf = fminf(fminf(x1, y1), fminf(z1, tcap));
#endif
    const bool h = tn <= tf * 1.0000004f;
    o.tn[j] = h ? tn : __builtin_huge_valf();
    o.c[j] = f2i(CH[j]);
    o.hm[j] = __builtin_amdgcn_ballot_w64(h);
  }
}
#else
__device__ __forceinline__ void box4(const Ray& r, const DevScene& sc, int node, float tcap, Box4& o) {
  const float4* np = sc.nodes + 8 * node;
  const float4 lx = np[0], hx = np[1], ly = np[2], hy = np[3], lz = np[4], hz = np[5];
  float4 ch = np[6];
  // the child links share the node's cache line: pin them here so the compiler cannot sink their
  // load into the hit branch (a second dependent L2 round trip per node): +4% Mrays/s
  asm volatile("" : "+v"(ch.x), "+v"(ch.y), "+v"(ch.z), "+v"(ch.w));
  const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, HX[4] = {hx.x, hx.y, hx.z, hx.w};
  const float LY[4] = {ly.x, ly.y, ly.z, ly.w}, HY[4] = {hy.x, hy.y, hy.z, hy.w};
  const float LZ[4] = {lz.x, lz.y, lz.z, lz.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
  const float CH[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = __builtin_fmaf(LX[j], r.inv.x, -r.oinv.x), x1 = __builtin_fmaf(HX[j], r.inv.x, -r.oinv.x);
    const float y0 = __builtin_fmaf(LY[j], r.inv.y, -r.oinv.y), y1 = __builtin_fmaf(HY[j], r.inv.y, -r.oinv.y);
    const float z0 = __builtin_fmaf(LZ[j], r.inv.z, -r.oinv.z), z1 = __builtin_fmaf(HZ[j], r.inv.z, -r.oinv.z);
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), r.tmin));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tcap));
    const bool h = tn <= tf * 1.0000004f;
    o.tn[j] = h ? tn : __builtin_huge_valf();
    o.c[j] = f2i(CH[j]);
    o.hm[j] = __builtin_amdgcn_ballot_w64(h);
  }
}
#endif
__device__ __forceinline__ void cswap4(Box4& b, int i, int j) {
  const bool sw = b.tn[j] < b.tn[i];
  const float ti = b.tn[i], tj = b.tn[j];
  const int ci = b.c[i], cj = b.c[j];
  b.tn[i] = sw ? tj : ti; b.tn[j] = sw ? ti : tj;
  b.c[i] = sw ? cj : ci; b.c[j] = sw ? ci : cj;
}
// The next node of a closest-hit walk after a 4-wide node test: the nearest hit child, the other hit
// children pushed farthest first; no hit child: pop().
template <typename Push, typename Pop>
__device__ __forceinline__ int enter_box4(Box4& b, Push push, Pop pop) {
  const unsigned long long h0 = b.hm[0], h1 = b.hm[1], h2 = b.hm[2], h3 = b.hm[3];
  if (!__builtin_amdgcn_inverse_ballot_w64(h0 | h1 | h2 | h3)) return pop();
  cswap4(b, 0, 1); cswap4(b, 2, 3); cswap4(b, 0, 2); cswap4(b, 1, 3); cswap4(b, 1, 2);
  // (the sorted hits come first: at least 4 / 3 / 2 of the four children hit, as lane masks)
  const unsigned long long a01 = h0 & h1, o01 = h0 | h1, a23 = h2 & h3, o23 = h2 | h3;
  if (__builtin_amdgcn_inverse_ballot_w64(a01 & a23)) push(b.c[3]);
  if (__builtin_amdgcn_inverse_ballot_w64((a01 & o23) | (o01 & a23))) push(b.c[2]);
  if (__builtin_amdgcn_inverse_ballot_w64(a01 | a23 | (o01 & o23))) push(b.c[1]);
  return b.c[0];
}

// SS: the LDS stack's stride (work-items sharing it); OVF: overflow entries beyond the LDS part (0 for
// a tree whose stack need fits PTGS_STACK: the overflow's branches and scratch cost 3.4% on C3)
template <bool STATS, bool TEX, int SS = PTGS_BLOCK, int OVF = PTGS_STACK_OVF>
__device__ __forceinline__ Hit trace_closest(const DevScene& sc, const Ray& r, uint32_t seed, int* stack,
                                             TraversalCounters& cnt) {
  Hit h; h.t = r.tmax; h.u = 0.f; h.v = 0.f; h.gid = 0xffffffffu; h.slot = 0;
  int sp = 0;
  int node = 0;
  // while-while with postponed leaves (Aila & Laine 2009): a lane that reaches a leaf parks it and
  // keeps walking interior nodes until every lane still in the loop holds a leaf, so the leaf phase
  // runs with more lanes busy (+2% Mrays/s on C3, tools/ab_pt.py; packing the slab FMAs of child
  // pairs into v_pk_fma_f32 measured -1.4%). The closest hit is the minimum over (t, gid) of every
  // candidate, so visiting order changes neither the hit nor the image.
  const int DONE = 0x7fffffff;
  int leaf = DONE;
  int ovf[OVF > 0 ? OVF : 1];  // entries beyond the LDS part (private: scratch)
  auto push = [&](int x) {
    if (OVF == 0 || sp < PTGS_STACK) stack[sp * SS] = x;
    else ovf[sp - PTGS_STACK] = x;
    ++sp;
  };
  auto pop = [&]() -> int {
    if (!sp) return DONE;
    --sp;
    return (OVF == 0 || sp < PTGS_STACK) ? stack[sp * SS] : ovf[sp - PTGS_STACK];
  };
  // (a register-cached stack top that hides the LDS read behind the node fetch measured -0.8%)
  for (;;) {
    while (node >= 0 && node != DONE) {
      PT_LANE_TICK(cnt, PT_L_NODE);
      Box4 b;
      box4(r, sc, node, h.t, b);
      if (STATS) cnt.nodes += 4;
      node = enter_box4(b, push, pop);
      if (node < 0 && leaf == DONE) {
        leaf = node;
        node = pop();
      }
      // (every active lane holds a leaf or is done: the compares' lane mask against exec, no VGPR round trip)
      if ((__builtin_amdgcn_ballot_w64(leaf != DONE) | __builtin_amdgcn_ballot_w64(node == DONE)) ==
          __builtin_amdgcn_read_exec())
        break;
    }
    if (leaf != DONE) {
      PT_LANE_TICK(cnt, PT_L_LEAF);
      leaf_closest<STATS, TEX>(sc, r, leaf, h, seed, cnt);
      leaf = DONE;
    }
    if (node < 0) {
      leaf_closest<STATS, TEX>(sc, r, node, h, seed, cnt);
      node = pop();
    }
    if (node == DONE) return h;
  }
}

template <bool STATS, bool TEX, int SS = PTGS_BLOCK, int OVF = PTGS_STACK_OVF>  // (as trace_closest)
__device__ __forceinline__ bool trace_any(const DevScene& sc, const Ray& r, uint32_t seed, int* stack,
                                          TraversalCounters& cnt) {
  int sp = 0;
  int node = 0;
  int ovf[OVF > 0 ? OVF : 1];  // entries beyond the LDS part (private: scratch)
  auto pop_nz = [&]() -> int {  // sp > 0
    --sp;
    return (OVF == 0 || sp < PTGS_STACK) ? stack[sp * SS] : ovf[sp - PTGS_STACK];
  };
  while (true) {
    while (node >= 0) {
      PT_LANE_TICK(cnt, PT_L_ANY_NODE);
      Box4 b;
      box4(r, sc, node, r.tmax, b);
      if (STATS) cnt.nodes += 4;
      // order is irrelevant for an any-hit query: enter the first hit child, push the others (the
      // closest-hit near-to-far order measured -9% for the shadow rays)
      int next = -0x7fffffff - 1;
      bool have = false;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (b.tn[j] != __builtin_huge_valf()) {
          if (!have) {
            next = b.c[j];
            have = true;
          } else {
            if (OVF == 0 || sp < PTGS_STACK) stack[sp * SS] = b.c[j];
            else ovf[sp - PTGS_STACK] = b.c[j];
            ++sp;
          }
        }
      if (!have) {
        if (sp == 0) return false;
        node = pop_nz();
        continue;
      }
      node = next;
    }
    uint32_t L = (uint32_t)(~node);
    uint32_t start = L & 0x07ffffffu;
    uint32_t count = (L >> 27) + 1u;
    for (uint32_t k = 0; k < count; ++k) {
      PT_LANE_TICK(cnt, PT_L_ANY_TRI);
      const float4* tp = sc.tris + 3u * (start + k);
      float4 a = tp[0], bb = tp[1], c = tp[2];
      if (STATS) cnt.tris++;
      float t, u, v;
      if (!tri_isect(r, mk3(a.x, a.y, a.z), mk3(bb.x, bb.y, bb.z), mk3(c.x, c.y, c.z), t, u, v)) continue;
      if (!(t >= r.tmin && t <= r.tmax)) continue;
      if (sc.has_transparent && (sc.tri_flags[start + k] & 1u)) {
        if (!anyhit_accept<TEX>(sc, f2u(a.w), f2u(bb.w), u, v, seed, f2u(c.w))) continue;
      }
      return true;
    }
    if (sp == 0) return false;
    node = pop_nz();
  }
}

__device__ __forceinline__ v4 matvec(const float* m, v4 v) {
  // GLSL mat4 * vec4 with columns m[0..3], m[4..7], ...: ((c0*x + c1*y) + c2*z) + c3*w
  return mk4(((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * v.w,
             ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * v.w,
             ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * v.w,
             ((m[3] * v.x + m[7] * v.y) + m[11] * v.z) + m[15] * v.w);
}

// r2 offset of the blue-noise lookup (raygen_camera.rgen:11-15, :19-23)
__device__ __forceinline__ float4 blue_noise_texel(const DevScene& sc, uint32_t lx, uint32_t ly, uint32_t frame) {
  const float a1 = 0.75487766624669276f;
  const float a2 = 0.56984029099805327f;
  float rx = fractx((float)frame * a1);
  float ry = fractx((float)frame * a2);
  int ox = (int)(rx * (float)sc.bn_size);
  int oy = (int)(ry * (float)sc.bn_size);
  int px = ((int)lx + ox) & (sc.bn_size - 1);
  int py = ((int)ly + oy) & (sc.bn_size - 1);
  return sc.blue_noise[py * sc.bn_size + px];
}

// raygen_camera.rgen:19-41: blue-noise jittered camera ray of pixel (x, y) for sample `frame`, and
// the payload seed (index + frame_count * 719393, :21)
__device__ __forceinline__ void primary_ray(const DevScene& sc, const CamParams& cp, uint32_t x, uint32_t y,
                                            uint32_t W, uint32_t H, uint32_t frame, v3& ro, v3& rd, float4& blue,
                                            uint32_t& seed) {
  blue = blue_noise_texel(sc, x, y, frame);
  seed = (y * W + x) + frame * 719393u;
  const float pcx = (float)x + blue.x, pcy = (float)y + blue.y;
  const float ux = pcx / (float)W, uy = pcy / (float)H;
  const float dx = ux * 2.0f - 1.0f, dy = uy * 2.0f - 1.0f;
  const v4 origin = matvec(cp.inv_view, mk4(0.f, 0.f, 0.f, 1.f));
  const v4 target = matvec(cp.inv_proj, mk4(dx, dy, 1.f, 1.f));
  const v3 dirc = normalize3(mk3(target.x, target.y, target.z) / target.w);
  const v4 direction = matvec(cp.inv_view, mk4(dirc.x, dirc.y, dirc.z, 0.f));
  ro = mk3(origin.x, origin.y, origin.z);
  rd = normalize3(mk3(direction.x, direction.y, direction.z));
}

// ---------------------------------------------------------------------------------------------
// Payload (raytracing.glsl:90-100; rt_datacollect adds hit_pos/normal)
// ---------------------------------------------------------------------------------------------
struct Payload {
  v3 color;
  v3 next_o;
  v3 next_d;
  float hit_flag;
  v3 weight;
  uint32_t seed;
  float last_pdf;
  v2 blue;
  int depth;
  v3 hit_pos;
  v3 normal;
};

struct ShadeCtx {
  const DevScene* sc;
  const CamParams* cp;
  int* stack;  // this work-item's LDS traversal stack (stride PTGS_BLOCK)
  uint32_t shadow_rays;
};

#define PT_PI 3.14159265359f
#define PT_PHI 1.61803398875f

// closesthit.rchit:16-19
__device__ __forceinline__ float blue_noise_dim(const Payload& p, int dim) {
  float base = (dim % 2 == 0) ? p.blue.x : p.blue.y;
  return fractx((base + ((float)p.depth * PT_PHI)) + ((float)dim * 0.754877f));
}

__device__ __forceinline__ v3 safe_normalize(v3 v) {
  float len = length3(v);
  return sel3(len < 1e-6f, mk3(0.0f, 1.0f, 0.0f), v / len);
}

// closesthit.rchit:49-51
__device__ __forceinline__ v3 f_schlick(float cos_theta, v3 f0) {
  float p = pow5(clampf(1.0f - cos_theta, 0.0f, 1.0f));
  return f0 + (1.0f - f0) * p;
}

// :54-58
__device__ __forceinline__ void ortho_basis(v3 n, v3& t, v3& b) {
  v3 up = sel3(absx(n.z) < 0.999f, mk3(0.f, 0.f, 1.f), mk3(1.f, 0.f, 0.f));
  t = safe_normalize(cross3(up, n));
  b = cross3(n, t);
}

// :60-69
__device__ __forceinline__ v3 sample_cosine(const Payload& p, v3 n) {
  float r1 = blue_noise_dim(p, 0);
  float r2 = blue_noise_dim(p, 1);
  float phi = (2.0f * PT_PI) * r1;
  float sq = sqrtx(r2);
  float s, c; sincosx(phi, &s, &c);
  v3 local = mk3(c * sq, s * sq, sqrtx(1.0f - r2));
  v3 t, b; ortho_basis(n, t, b);
  return safe_normalize((t * local.x + b * local.y) + n * local.z);
}

// :71-78
__device__ __forceinline__ float d_ggx(v3 n, v3 h, float roughness) {
  float a = roughness * roughness;
  float a2 = a * a;
  float ndh = fmaxx(dot3(n, h), 0.0f);
  float ndh2 = ndh * ndh;
  float denom = ndh2 * (a2 - 1.0f) + 1.0f;
  return a2 / (((PT_PI * denom) * denom) + 0.0001f);
}

// :80-85
__device__ __forceinline__ float v_smith(float ndv, float ndl, float roughness) {
  float a = roughness * roughness;
  float ggxv = ndl * (ndv * (1.0f - a) + a);
  float ggxl = ndv * (ndl * (1.0f - a) + a);
  return 0.5f / fmaxx(ggxv + ggxl, 0.0001f);
}

// :87-99 (dims 2,3)
__device__ __forceinline__ v3 sample_ggx(const Payload& p, v3 n, float roughness) {
  float r1 = blue_noise_dim(p, 2);
  float r2 = blue_noise_dim(p, 3);
  float a = roughness * roughness;
  float phi = (2.0f * PT_PI) * r1;
  float denom = 1.0f + (a * a - 1.0f) * r2;
  float cos_t = sqrtx((1.0f - r2) / fmaxx(denom, 0.0001f));
  float sin_t = sqrtx(1.0f - cos_t * cos_t);
  float s, c; sincosx(phi, &s, &c);
  v3 hl = mk3(sin_t * c, sin_t * s, cos_t);
  v3 t, b; ortho_basis(n, t, b);
  return safe_normalize((t * hl.x + b * hl.y) + n * hl.z);
}

// :101-107
__device__ __forceinline__ float pdf_ggx(v3 n, v3 v, v3 l, float roughness) {
  v3 h = safe_normalize(v + l);
  float ndh = fmaxx(dot3(n, h), 0.0f);
  float vdh = fmaxx(dot3(v, h), 0.0f);
  float dn = d_ggx(n, h, roughness) * ndh;
  return dn / (4.0f * vdh + 0.0001f);
}

// :109-111
__device__ __forceinline__ float pdf_lambert(v3 n, v3 l) { return fmaxx(dot3(n, l), 0.0f) / PT_PI; }

// NEE visibility, deferred. closest_hit (pt_shade.h) only records the shadow ray and the light's
// contribution with the visibility factor left out; the ray-gen loop traces the ray once shading is
// done (resolve_shadow), so no shading state is live across the any-hit traversal (round 1: 164 B
// per lane of scratch spills in pt_camera_kernel). The result is bit-identical to tracing inside
// sampleLights / samplePunctualLights (closesthit.rchit:115-126, :180-188, :290-318):
//   - the shadow ray (origin, direction, range) is built from the same expressions (:119-126);
//   - the contribution keeps the reference's operation order with vis in place:
//     lo + ((pre * vis) * post), and for mixed light sets lc = (0 + that) * (1 / p) (:476-488);
//   - vis = max(vis, transmission) and the `vis > 0` / `pdf_nee > 1e-10` guards are applied as
//     there, and the any-hit seed is the payload seed of the hit (unchanged until the loop's RR).
#define SQ_TRACE 1u  // a shadow ray was cast (counted in the shadow-ray statistics)
#define SQ_VALID 2u  // the light contributes when visible
#define SQ_MIXED 4u  // emissive + punctual lights: lc = lc * (1 / p_select) before lo += lc
struct ShadowQuery {
  v3 o, d;
  float tmax;
  v3 pre;       // contribution up to the visibility factor
  float post;   // factor applied after it (num_lights / ambientLight.w)
  float scale;  // 1 / p_emissive or 1 / (1 - p_emissive) for SQ_MIXED
  float trans;  // vis = max(vis, transmission)
  uint32_t flags;
};

// closesthit.rchit:119-126 traceShadow: ray from o towards light_pos, range dist - 0.005
__device__ __forceinline__ void shadow_towards(ShadowQuery& q, v3 o, v3 light_pos) {
  v3 l = light_pos - o;
  float dist = length3(l);
  q.o = o;
  q.d = safe_normalize(l);
  q.tmax = dist - 0.005f;
}

template <bool STATS, bool TEX, int SS = PTGS_BLOCK, int OVF = PTGS_STACK_OVF>  // (as trace_closest)
__device__ __forceinline__ void resolve_shadow(ShadeCtx& c, v3& color, uint32_t seed, const ShadowQuery& q,
                                               TraversalCounters& cnt) {
  if (!(q.flags & SQ_TRACE)) return;
  c.shadow_rays++;
  const Ray r = make_ray(q.o, q.d, 0.001f, q.tmax);
  float vis = trace_any<STATS, TEX, SS, OVF>(*c.sc, r, seed, c.stack, cnt) ? 0.0f : 1.0f;
  vis = fmaxx(vis, q.trans);
  if (vis > 0.0f && (q.flags & SQ_VALID)) {
    v3 contrib = (q.pre * vis) * q.post;
    if (q.flags & SQ_MIXED) contrib = (mk3(0.0f) + contrib) * q.scale;
    color = color + contrib;
  }
}

// binary search over a CDF (closesthit.rchit:131-137 / :197-203 / :262-268)
template <typename CDF>
__device__ __forceinline__ uint32_t cdf_search(const CDF* cdf, uint32_t n, float r) {
  uint32_t idx = 0, left = 0, right = n;
  while (left < right) {
    uint32_t mid = (left + right) >> 1;
    if (cdf[mid].cumulative_probability < r) left = mid + 1;
    else { idx = mid; right = mid; }
  }
  return idx;
}

// :128-192 (the shadow ray and the contribution go to q; see ShadowQuery)
__device__ void sample_punctual(const ShadeCtx& c, const Payload& p, v3 hit_pos, v3 n, v3 n_geo, v3 v, v3 albedo,
                                float roughness, v3 f0, float transmission, ShadowQuery& q) {
  const DevScene& sc = *c.sc;
  uint32_t num_lights = sc.num_plights;
  float r_select = blue_noise_dim(p, 4);
  uint32_t li = cdf_search(sc.pcdf, num_lights, r_select);
  const ptgs_punctual_light& light = sc.plights[li];
  v3 l;
  float attenuation = 1.0f;
  v3 lpos = ld3(light.position);
  v3 ldir = ld3(light.direction);
  if (light.type == 1) {
    l = normalize3(-ldir);
    attenuation = 1.0f;
  } else {
    v3 off = lpos - hit_pos;
    float dist_sq = dot3(off, off);
    dist_sq = fmaxx(dist_sq, 0.01f);
    float dist = sqrtx(dist_sq);
    l = off / dist;
    attenuation = 1.0f / dist_sq;
    if (light.range > 0.0f) {
      float ra = fmaxx(fminx(1.0f - pow4(dist / light.range), 1.0f), 0.0f) / dist_sq;
      attenuation = ra / dist_sq;
    }
    if (light.type == 2) {
      float cos_dir = dot3(-l, normalize3(ldir));
      float spot_scale = 1.0f / fmaxx(light.inner_cone_cos - light.outer_cone_cos, 0.001f);
      float spot_offset = -light.outer_cone_cos * spot_scale;
      float sa = clampf(cos_dir * spot_scale + spot_offset, 0.0f, 1.0f);
      attenuation = attenuation * (sa * sa);
    }
  }
  v3 le = (ld3(light.color) * light.intensity) * attenuation;
  float ndl = fmaxx(dot3(n, l), 0.0f);
  if (ndl < 0.001f) return;
  if (ndl > 0.0f && length3(le) > 0.0f) {
    v3 so = hit_pos + n_geo * 0.001f;
    if (light.type == 1) {  // traceShadowRay with a 1e4 range (:146, :175)
      q.o = so;
      q.d = l;
      q.tmax = 10000.0f;
    } else {
      shadow_towards(q, so, lpos);
    }
    q.trans = transmission;
    float weight = (float)num_lights;
    v3 h = safe_normalize(v + l);
    float ndf = d_ggx(n, h, roughness);
    float vis_t = v_smith(dot3(n, v), ndl, roughness);
    v3 f = f_schlick(dot3(h, v), f0);
    v3 kd = (mk3(1.0f) - f) * (1.0f - transmission);
    v3 spec = f * (ndf * vis_t);
    v3 diff = ((kd * albedo) / PT_PI) * (1.0f - transmission);
    q.pre = ((diff + spec) * le) * ndl;  // lo += ((((diff + spec) * le) * ndl) * vis) * weight
    q.post = weight;
    q.flags = SQ_TRACE | SQ_VALID;
  }
}

// :194-257 (sg == true) and :259-320 (sg == false); the shadow ray and the contribution go to q
__device__ void sample_emissive(const ShadeCtx& c, const Payload& p, bool sg, v3 hit_pos, v3 n, v3 n_geo, v3 v,
                                v3 albedo, float roughness, float metallic, v3 f0, float transmission, ShadowQuery& q) {
  const DevScene& sc = *c.sc;
  uint32_t num = sc.num_light_cdf;
  float r_select = blue_noise_dim(p, sg ? 4 : 7);
  uint32_t idx = cdf_search(sc.light_cdf, num, r_select);
  uint32_t tri_idx = sc.light_cdf[idx].triangle_index;
  ptgs_light_triangle tri = sc.light_tris[tri_idx];
  const uint32_t light_mat = tri.material_index;
  v3 p0 = ld3(sc.vertices[tri.v0].pos);
  v3 p1 = ld3(sc.vertices[tri.v1].pos);
  v3 p2 = ld3(sc.vertices[tri.v2].pos);
  float u = blue_noise_dim(p, sg ? 5 : 8);
  float w = blue_noise_dim(p, sg ? 6 : 9);
  if (u + w > 1.0f) { u = 1.0f - u; w = 1.0f - w; }
  v3 lp = (p0 * ((1.0f - u) - w) + p1 * u) + p2 * w;
  v3 cr = cross3(p1 - p0, p2 - p0);
  v3 ln = sg ? normalize3(cr) : safe_normalize(cr);
  v3 l = lp - hit_pos;
  float dist_sq = dot3(l, l);
  dist_sq = fmaxx(dist_sq, 0.0001f);
  float dist = sqrtx(dist_sq);
  l = l / dist;
  float ndl = fmaxx(dot3(n, l), 0.0f);
  if (ndl < 0.001f) return;
  float ldn = absx(dot3(-l, ln));
  if (ndl > 0.0f && ldn > 0.0f) {
    v3 so = hit_pos + n_geo * 0.001f;
    shadow_towards(q, so, lp);
    q.trans = transmission;
    q.flags = SQ_TRACE;
    const ptgs_material& lm = sc.materials[light_mat];
    v3 le = ld3(lm.emissive_factor_and_pad);
    float es = fmaxx(le.x, fmaxx(le.y, le.z));
    float pdf_nee = (es / c.cp->emissive_flux) * (dist_sq / ldn);
    float prob_spec;
    float pdf_spec, pdf_diff;
    if (sg) {
      pdf_spec = pdf_ggx(n, v, l, roughness);
      pdf_diff = pdf_lambert(n, l);
      prob_spec = clampf(length3(f0), 0.05f, 0.95f);
    } else {
      prob_spec = mixf(0.04f, 1.0f, metallic);
      pdf_spec = pdf_ggx(n, v, l, roughness);
      pdf_diff = pdf_lambert(n, l);
    }
    float prob_diff = 1.0f - prob_spec;
    float pdf_bsdf = pdf_spec * prob_spec + pdf_diff * prob_diff;
    float mis = (pdf_nee * pdf_nee) / (pdf_nee * pdf_nee + pdf_bsdf * pdf_bsdf);
    v3 h = safe_normalize(v + l);
    float ndf = d_ggx(n, h, roughness);
    float vis_t = v_smith(dot3(n, v), ndl, roughness);
    v3 f = f_schlick(dot3(h, v), f0);
    v3 kd = mk3(1.0f) - f;
    v3 spec = f * (ndf * vis_t);
    v3 diff = ((kd * albedo) / PT_PI) * (1.0f - transmission);
    v3 brdf = diff + spec;
    if (pdf_nee > 1e-10f) {
      // lo += (((((brdf * le) * ndl) * (1 / pdf_nee)) * mis) * vis) * ambientLight.w
      q.pre = (((brdf * le) * ndl) * (1.0f / pdf_nee)) * mis;
      q.post = c.cp->ambient[3];
      q.flags |= SQ_VALID;
    }
  }
}

}  // namespace ptgs
