// api.cpp — the C-ABI boundary (include/ptgs/ptgs.h): context, scene upload, trace dispatch.
//
// Replaces, on the reference side (Vulkan_Engine/engine.cpp):
//   createGlobalBindlessBuffers uploads :1658-1860 and buildBlas/initStaticTlas :534-655, :1385-1520
//       -> ptgs_scene_upload (host BVH build + hipMemcpy of the reference-layout arrays)
//   recordCommandBuffer's vkCmdTraceRaysKHR :1971-1976 + rt_output_image running mean
//       -> ptgs_trace_camera
//   torus trace :1893-1900 / :2787-2794 -> ptgs_trace_torus
// Largest BVH leaf (triangles). C3 at 64 spp (tools/ab_pt.py, interleaved): 1 -> 3 602, 2 -> 4 849,
// 3 -> 4 836, 4 -> 4 463, 8 -> -10% Mrays/s; 3 keeps the tree a level shallower than 2 for the
// traversal-stack budget of large meshes
#ifndef PTGS_BVH_LEAF
#define PTGS_BVH_LEAF 3
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs.h"
#include "bvh.h"
#include "bvh_gpu.h"
#include "knn.h"
#include "hostmath.h"
#include "pt_launch.h"
#include "pt_wavefront.h"
#include "comm.h"
#include "splat.h"
#include "textures.h"

using namespace ptgs;

// frames in flight of PTGS_FLAG_SPLAT_OVERLAP: workspaces in the ring (the front end of call k may run
// beside the blends of calls k - 1 .. k - depth + 1; PTGS_GS_OV_DEPTH=2 .. 4, default 3)
#define PTGS_OV_RING 4        // workspaces the ring may hold (PTGS_GS_OV_DEPTH)
#define PTGS_OV_DEPTH_DEFAULT 3

struct ptgs_ctx {
  int device = 0;
  std::string err;
  uint32_t flags = 0;
  bool has_scene = false;
  DevScene dsc{};
  std::vector<void*> scene_allocs;
  ptgs_scene_info info{};
  unsigned long long* counters = nullptr;  // 8 x u64
  SplatWorkspace* splat = nullptr;
  // ptgs_splat_gaussians_views: views 1.. run on their own workspaces and non-blocking streams,
  // forked from / joined back into the caller's stream with events (view 0 uses `splat` on it)
  SplatWorkspace* view_ws[PTGS_MAX_VIEWS] = {};
  hipStream_t view_stream[PTGS_MAX_VIEWS] = {};
  hipEvent_t view_fork = nullptr, view_join[PTGS_MAX_VIEWS] = {};
  // PTGS_FLAG_SPLAT_OVERLAP: a ring of workspaces (`splat` is always the latest call's; ov_ring[0] is the
  // context's own first workspace), the front-end stream, the caller's stream at the start of a run of
  // overlapped calls (ov_call[0]; see splat_overlap_begin), the front end's end
  SplatWorkspace* ov_ring[PTGS_OV_RING] = {};
  hipStream_t ov_stream = nullptr;
  hipEvent_t ov_call[1] = {}, ov_done = nullptr;
  uint32_t ov_pos = 0;      // ring slot of the latest overlapped call
  uint32_t ov_depth = 0;    // workspaces in use (2 .. PTGS_OV_RING)
  uint32_t pending_report = 0;  // earlier frames' reports a failing splat call collected (returned by the next)
  uint32_t ov_started = 0;  // consecutive overlapped calls so far (0: the next one starts a run from the caller's stream)
  // blend ordinals (SplatSeq): the device word the blends store theirs in, the next one, and per call of the
  // run (k % 4) the ordinal of its blend (0: none launched) and its stream
  unsigned long long* ov_flag = nullptr;
  unsigned long long ov_next = 1;
  unsigned long long ov_ord[4] = {};
  hipStream_t ov_strm[4] = {};
  ptgs::WfWorkspace wf;  // wavefront path tracer buffers (PTGS_FLAG_PT_WAVEFRONT)
  ptgs::PtSched pt_sched;  // megakernel tile schedule (heavy tiles first)
  void* comm = nullptr;  // RCCL communicator (ptgs_comm_create)
  int comm_ranks = 0, comm_rank = 0;
};

namespace {

// 4-wide collapse whose worst-case traversal stack fits PTGS_STACK_TOTAL (LDS + overflow) with fan-out
// `fan` (a 2-wide "collapse" needs the BVH2 depth, which the builders keep below PTGS_STACK)
static bool collapse_fit(const std::vector<float>& n2, std::vector<float>& n4, uint32_t& num4, uint32_t& dep4, int fan,
                         uint32_t& need) {
  need = 0;
  ptgs::collapse_bvh4(n2, n4, num4, need, dep4, fan);
  return need < PTGS_STACK_TOTAL;
}

// (leaf size, fan-out) tried in this order until the tree's worst-case stack need fits PTGS_STACK_TOTAL:
// a scene whose 3-triangle-leaf tree is too deep for a 4-wide collapse is rebuilt with 4-triangle
// leaves before the fan-out is narrowed (a 2-wide fallback traced C5 at 1.38 Grays/s, the
// 4-triangle-leaf 4-wide tree at ~2.1; with the stack overflow C5 keeps 3-triangle leaves: need 40)
// Each try also carries the SAH build's depth budget (bvh.cpp: past it, balanced splits).
struct BvhTry {
  int leaf, fan;
  uint32_t depth;
};
static const BvhTry kBvhTriesDefault[] = {{PTGS_BVH_LEAF, 4, PTGS_STACK - 1}, {PTGS_BVH_LEAF + 1, 4, PTGS_STACK - 1},
                                          {PTGS_BVH_LEAF, 3, PTGS_STACK - 1}, {PTGS_BVH_LEAF, 2, PTGS_STACK - 1}};
// PTGS_BVH_TRIES="leaf:fan:depth,..." replaces the list (A/B of tree shapes: tools/ab_pt.py AB_SCENE=c5)
static std::vector<BvhTry> bvh_tries() {
  std::vector<BvhTry> v;
  if (const char* e = getenv("PTGS_BVH_TRIES")) {
    for (const char* p = e; *p;) {
      int l = 0, f = 0;
      unsigned d = 0;
      if (sscanf(p, "%d:%d:%u", &l, &f, &d) == 3 && l >= 1 && l <= 16 && f >= 2 && f <= 4 && d >= 1 && d < PTGS_STACK)
        v.push_back({l, f, d});
      while (*p && *p != ',') ++p;
      if (*p == ',') ++p;
    }
  }
  if (v.empty()) v.assign(std::begin(kBvhTriesDefault), std::end(kBvhTriesDefault));
  return v;
}
// 4-wide nodes the traversal can address (PTGS_BVH_NODE_LIMIT lowers it: the guard's GPU test)
static uint32_t bvh_node_limit() {
  const uint32_t hw = 0x7fffffffu / 128u;
  const char* e = getenv("PTGS_BVH_NODE_LIMIT");
  const unsigned long v = e ? strtoul(e, nullptr, 10) : 0ul;
  return v && v < hw ? (uint32_t)v : hw;
}
static void bvh_log(const char* how, int leaf, int fan, uint32_t budget, uint32_t depth, uint32_t need) {
  if (getenv("PTGS_BVH_LOG"))
    fprintf(stderr, "[ptgs] %s tree: leaf %d fan %d depth budget %u -> depth %u, stack need %u%s\n", how, leaf, fan,
            budget, depth, need, need >= PTGS_STACK ? (need < PTGS_STACK_TOTAL ? " (DEEP)" : " (does not fit)") : "");
}

int fail(ptgs_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(ctx, expr)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(ctx, PTGS_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

void free_scene(ptgs_ctx* c) {
  for (void* p : c->scene_allocs) (void)hipFree(p);
  c->scene_allocs.clear();
  c->has_scene = false;
  c->dsc = DevScene{};
}

template <typename T>
int upload(ptgs_ctx* c, const T* src, size_t count, const T** dst) {
  if (count == 0) { *dst = nullptr; return PTGS_OK; }
  void* p = nullptr;
  HIPCHK(c, hipMalloc(&p, count * sizeof(T)));
  c->scene_allocs.push_back(p);
  HIPCHK(c, hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice));
  c->info.device_bytes += count * sizeof(T);
  *dst = (const T*)p;
  return PTGS_OK;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.devicePointer != nullptr;
}

int fill_cam(ptgs_ctx* c, const ptgs_ubo* ubo, CamParams& cp) {
  if (!inverse4(ubo->view, cp.inv_view)) return fail(c, PTGS_EINVAL, "ubo.view is singular");
  if (!inverse4(ubo->proj, cp.inv_proj)) return fail(c, PTGS_EINVAL, "ubo.proj is singular");
  for (int k = 0; k < 4; ++k) cp.ambient[k] = ubo->ambient_light[k];
  cp.emissive_flux = ubo->emissive_flux;
  cp.punctual_flux = ubo->punctual_flux;
  cp.p_emissive = ubo->p_emissive;
  cp.fov = ubo->fov;
  cp.win_height = ubo->height;
  cp.use_lod = ubo->use_lod;
  cp.lod_factor = ubo->lod_factor;
  return PTGS_OK;
}

}  // namespace

extern "C" {

int ptgs_abi_version(void) { return PTGS_ABI_VERSION; }
const char* ptgs_device_arch(void) { return "gfx950"; }

int ptgs_create(int hip_device, ptgs_ctx** out) {
  if (!out) return PTGS_EINVAL;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return PTGS_EHIP;
  if (hip_device < 0 || hip_device >= n) return PTGS_EINVAL;
  ptgs_ctx* c = new ptgs_ctx();
  c->device = hip_device;
  if (hipSetDevice(hip_device) != hipSuccess) { delete c; return PTGS_EHIP; }
  if (hipMalloc(&c->counters, 8 * sizeof(unsigned long long)) != hipSuccess) { delete c; return PTGS_EHIP; }
  if (hipMemset(c->counters, 0, 8 * sizeof(unsigned long long)) != hipSuccess) { delete c; return PTGS_EHIP; }
  c->splat = splat_workspace_create();
  *out = c;
  return PTGS_OK;
}

void ptgs_destroy(ptgs_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  free_scene(c);
  if (c->counters) (void)hipFree(c->counters);
  ptgs::wf_workspace_free(c->wf);
  ptgs::free_pt_sched(c->pt_sched);
  // (c->splat is one of the ring's workspaces once PTGS_FLAG_SPLAT_OVERLAP has been used: ring slot 0 is
  // the context's first one, freed here; the others below)
  splat_workspace_destroy(c->ov_ring[0] ? c->ov_ring[0] : c->splat);
  for (int v = 0; v < PTGS_MAX_VIEWS; ++v) {
    if (c->view_ws[v]) splat_workspace_destroy(c->view_ws[v]);
    if (c->view_stream[v]) (void)hipStreamDestroy(c->view_stream[v]);
    if (c->view_join[v]) (void)hipEventDestroy(c->view_join[v]);
  }
  if (c->view_fork) (void)hipEventDestroy(c->view_fork);
  for (SplatWorkspace* w : c->ov_ring)  // (ring slot 0 is the context's first workspace: freed above)
    if (w && w != c->ov_ring[0]) splat_workspace_destroy(w);
  if (c->ov_stream) (void)hipStreamDestroy(c->ov_stream);
  for (hipEvent_t ev : c->ov_call)
    if (ev) (void)hipEventDestroy(ev);
  if (c->ov_done) (void)hipEventDestroy(c->ov_done);
  if (c->ov_flag) (void)hipFree(c->ov_flag);
  if (c->comm) (void)comm_destroy(c->comm);
  delete c;
}

int ptgs_comm_unique_id(uint8_t id[PTGS_COMM_ID_BYTES]) {
  if (!id) return PTGS_EINVAL;
  if (!comm_available()) return PTGS_EHIP;
  return comm_unique_id(id) == 0 ? PTGS_OK : PTGS_EHIP;
}

int ptgs_comm_create(ptgs_ctx* c, const uint8_t id[PTGS_COMM_ID_BYTES], int nranks, int rank) {
  if (!c || !id) return PTGS_EINVAL;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(c, PTGS_EINVAL, "bad rank %d of %d", rank, nranks);
  if (!comm_available()) return fail(c, PTGS_EHIP, "RCCL (librccl.so.1) could not be loaded");
  HIPCHK(c, hipSetDevice(c->device));
  if (c->comm) {
    (void)comm_destroy(c->comm);
    c->comm = nullptr;
  }
  int e = comm_create(id, nranks, rank, &c->comm);
  if (e) return fail(c, PTGS_EHIP, "ncclCommInitRank: %s", comm_error(e));
  c->comm_ranks = nranks;
  c->comm_rank = rank;
  return PTGS_OK;
}

int ptgs_comm_destroy(ptgs_ctx* c) {
  if (!c) return PTGS_EINVAL;
  if (c->comm) {
    int e = comm_destroy(c->comm);
    c->comm = nullptr;
    if (e) return fail(c, PTGS_EHIP, "ncclCommDestroy: %s", comm_error(e));
  }
  return PTGS_OK;
}

static int reduce_common(ptgs_ctx* c, float* accum, size_t n, int root, bool all, void* stream) {
  if (!c || !accum) return PTGS_EINVAL;
  if (!c->comm) return fail(c, PTGS_EINVAL, "no communicator (ptgs_comm_create)");
  if (!is_device_ptr(accum)) return fail(c, PTGS_EINVAL, "accum is not a device pointer");
  HIPCHK(c, hipSetDevice(c->device));
  int e = all ? comm_allreduce_sum(c->comm, accum, n, (hipStream_t)stream)
              : comm_reduce_sum(c->comm, accum, n, root, (hipStream_t)stream);
  if (e) return fail(c, PTGS_EHIP, "%s: %s", all ? "ncclAllReduce" : "ncclReduce", comm_error(e));
  return PTGS_OK;
}

int ptgs_reduce_radiance(ptgs_ctx* c, float* accum, size_t n_floats, int root, void* stream) {
  return reduce_common(c, accum, n_floats, root, false, stream);
}

int ptgs_allreduce_radiance(ptgs_ctx* c, float* accum, size_t n_floats, void* stream) {
  return reduce_common(c, accum, n_floats, 0, true, stream);
}

int ptgs_gather_rows(ptgs_ctx* c, float* image, uint32_t width, uint32_t height, const uint32_t* row_ranges,
                     int root, void* stream) {
  if (!c || !image || !row_ranges) return PTGS_EINVAL;
  if (!c->comm) return fail(c, PTGS_EINVAL, "no communicator (ptgs_comm_create)");
  if (root < 0 || root >= c->comm_ranks) return fail(c, PTGS_EINVAL, "bad root %d", root);
  if (!is_device_ptr(image)) return fail(c, PTGS_EINVAL, "image is not a device pointer");
  for (int g = 0; g < c->comm_ranks; ++g)
    if (row_ranges[2 * g] > row_ranges[2 * g + 1] || row_ranges[2 * g + 1] > height)
      return fail(c, PTGS_EINVAL, "bad row range of rank %d", g);
  HIPCHK(c, hipSetDevice(c->device));
  int e = comm_gather_rows(c->comm, image, (size_t)width * 4u, row_ranges, c->comm_ranks, c->comm_rank, root,
                           (hipStream_t)stream);
  if (e) return fail(c, PTGS_EHIP, "ncclSend/ncclRecv: %s", comm_error(e));
  return PTGS_OK;
}

int ptgs_reduce_scatter_rows(ptgs_ctx* c, float* image, uint32_t width, uint32_t height, const uint32_t* row_ranges,
                             void* stream) {
  if (!c || !image || !row_ranges) return PTGS_EINVAL;
  if (!c->comm) return fail(c, PTGS_EINVAL, "no communicator (ptgs_comm_create)");
  if (!is_device_ptr(image)) return fail(c, PTGS_EINVAL, "image is not a device pointer");
  for (int g = 0; g < c->comm_ranks; ++g)
    if (row_ranges[2 * g] > row_ranges[2 * g + 1] || row_ranges[2 * g + 1] > height)
      return fail(c, PTGS_EINVAL, "bad row range of rank %d", g);
  HIPCHK(c, hipSetDevice(c->device));
  int e = comm_reduce_rows(c->comm, image, (size_t)width * 4u, row_ranges, c->comm_ranks, (hipStream_t)stream);
  if (e) return fail(c, PTGS_EHIP, "ncclReduce: %s", comm_error(e));
  return PTGS_OK;
}

const char* ptgs_last_error(const ptgs_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ptgs_scene_upload(ptgs_ctx* c, const ptgs_scene_desc* d) {
  if (!c || !d) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (!d->vertices && d->num_vertices) return fail(c, PTGS_EINVAL, "vertices is null");
  if (!d->indices && d->num_indices) return fail(c, PTGS_EINVAL, "indices is null");
  if (d->num_meshes && (!d->meshes || !d->mesh_index_count)) return fail(c, PTGS_EINVAL, "meshes is null");
  if (!d->materials || d->num_materials == 0) return fail(c, PTGS_EINVAL, "at least one material is required");
  if (!d->light_triangles || !d->light_cdf || d->num_light_cdf == 0 || d->num_light_triangles == 0)
    return fail(c, PTGS_EINVAL, "light triangle / CDF buffers must hold >= 1 entry (engine.cpp:1766-1769 dummy)");
  if (!d->punctual_lights || !d->punctual_cdf || d->num_punctual_lights == 0 || d->num_punctual_cdf == 0)
    return fail(c, PTGS_EINVAL, "punctual light / CDF buffers must hold >= 1 entry (engine.cpp:1795-1797 dummy)");
  uint32_t bn = d->blue_noise_size;
  if (!d->blue_noise_rgba32f || bn == 0 || (bn & (bn - 1)) != 0)
    return fail(c, PTGS_EINVAL, "blue noise must be a power-of-two square RGBA32F texture");
  if (d->num_textures && !d->textures) return fail(c, PTGS_EINVAL, "textures is null");
  TexturePool texpool;
  {
    std::string terr;
    if (!build_texture_pool(d->textures, d->num_textures, texpool, terr)) return fail(c, PTGS_EINVAL, "%s", terr.c_str());
    if (texpool.texels.size() >= (1ull << 32)) return fail(c, PTGS_ERANGE, "texture pool exceeds 2^32 texels");
  }

  // gather triangles in flattening order (gid), skipping meshes with < 3 indices (engine.cpp:545-547)
  std::vector<BuildTri> tris;
  std::vector<uint32_t> hitrec;  // per gid: global vertex indices + material (closest_hit's one fetch)
  bool has_transparent = false;
  for (uint32_t m = 0; m < d->num_meshes; ++m) {
    const ptgs_mesh_info& mi = d->meshes[m];
    uint32_t cnt = d->mesh_index_count[m];
    if (cnt < 3) continue;
    if (mi.material_index >= d->num_materials) return fail(c, PTGS_EINVAL, "mesh %u: material %u out of range", m, mi.material_index);
    if ((uint64_t)mi.index_offset + cnt > d->num_indices) return fail(c, PTGS_EINVAL, "mesh %u: index range out of bounds", m);
    const ptgs_material& mat = d->materials[mi.material_index];
    uint32_t flags = (mat.pad > 0.5f) ? 1u : 0u;  // non-opaque geometry (engine.cpp:562-567)
    has_transparent |= flags != 0;
    for (uint32_t p = 0; p < cnt / 3; ++p) {
      BuildTri t;
      for (int k = 0; k < 3; ++k) {
        uint32_t vi = d->indices[mi.index_offset + 3 * p + k] + mi.vertex_offset;
        if (vi >= d->num_vertices) return fail(c, PTGS_EINVAL, "mesh %u prim %u: vertex %u out of range", m, p, vi);
        float* dst = k == 0 ? t.v0 : (k == 1 ? t.v1 : t.v2);
        std::memcpy(dst, d->vertices[vi].pos, 12);
        hitrec.push_back(vi);
      }
      hitrec.push_back(mi.material_index);
      t.mesh = m; t.prim = p; t.gid = (uint32_t)tris.size(); t.flags = flags;
      tris.push_back(t);
    }
  }
  if (tris.size() >= (1u << 27)) return fail(c, PTGS_ERANGE, "too many triangles (%zu)", tris.size());
  if (d->num_punctual_cdf < d->num_punctual_lights)
    return fail(c, PTGS_EINVAL, "punctual CDF shorter than the light list (binary search runs over the light count)");
  for (uint32_t i = 0; i < d->num_light_cdf; ++i)
    if (d->light_cdf[i].triangle_index >= d->num_light_triangles)
      return fail(c, PTGS_EINVAL, "light CDF entry %u: triangle %u out of range", i, d->light_cdf[i].triangle_index);
  for (uint32_t i = 0; i < d->num_light_triangles; ++i) {
    const ptgs_light_triangle& lt = d->light_triangles[i];
    if (d->num_vertices == 0 || lt.v0 >= d->num_vertices || lt.v1 >= d->num_vertices || lt.v2 >= d->num_vertices) {
      if (d->num_light_triangles == 1 && lt.v0 == 0 && lt.v1 == 0 && lt.v2 == 0) continue;  // dummy
      return fail(c, PTGS_EINVAL, "light triangle %u references a vertex out of range", i);
    }
  }

  free_scene(c);
  c->info = ptgs_scene_info{};
  DevScene s{};
  int rc;
  // BVH: the host binned-SAH build (default), or with PTGS_FLAG_GPU_BVH the GPU LBVH (bvh_gpu.hip),
  // falling back to the host build when the LBVH is deeper than the traversal stack
  bool built = false;
  if ((c->flags & PTGS_FLAG_GPU_BVH) && tris.size() >= 16) {
    GpuBvh g;
    float ms = 0.0f;
    hipError_t e = hipSuccess;
    // (leaf, fan) as the host path (kBvhTries); the LBVH has fixed leaves: fan-out 4, 3, 2
    const bool lbvh = (c->flags & PTGS_FLAG_GPU_LBVH) != 0;
    const std::vector<BvhTry> tl = bvh_tries();
    const int tries = lbvh ? 3 : (int)tl.size();
    int built_leaf = -1;
    uint32_t built_depth = 0;
    float4* n4 = nullptr;
    uint32_t num4 = 0, need = PTGS_STACK_TOTAL, dep4 = 0;
    for (int k = 0; k < tries; ++k) {
      const int leaf = lbvh ? 0 : tl[k].leaf, fan = lbvh ? 4 - k : tl[k].fan;
      const uint32_t depth = lbvh ? PTGS_STACK - 1 : tl[k].depth;
      if (leaf != built_leaf || depth != built_depth) {  // (re)build the BVH2
        if (built_leaf >= 0) {
          (void)hipFree(g.nodes);
          (void)hipFree(g.tris);
          (void)hipFree(g.tri_flags);
          g = GpuBvh{};
        }
        float bms = 0.0f;
        e = lbvh ? build_bvh_gpu(tris, PTGS_STACK - 1, g, &bms) : build_bvh_sah_gpu(tris, leaf, depth, g, &bms);
        ms += bms;
        if (e != hipSuccess) break;
        built_leaf = leaf;
        built_depth = depth;
      }
      // 4-wide collapse on the GPU
      auto t0 = std::chrono::steady_clock::now();
      (void)hipFree(n4);
      n4 = nullptr;
      e = collapse_bvh4_gpu(g.nodes, g.num_nodes, fan, &n4, &num4, &need, &dep4);
      auto t1 = std::chrono::steady_clock::now();
      if (e == hipSuccess) bvh_log("GPU", leaf, fan, depth, dep4, need);
      ms += (float)std::chrono::duration<double, std::milli>(t1 - t0).count();  // build_ms includes it
      if (e != hipSuccess || need < PTGS_STACK_TOTAL) break;
    }
    if (e == hipSuccess && need >= PTGS_STACK_TOTAL) e = hipErrorNotSupported;
    if (e == hipSuccess || e == hipErrorNotSupported) {
      (void)hipFree(g.nodes);
      g.nodes = n4;
      g.num_nodes = num4;
      g.depth = dep4;
    } else {
      (void)hipFree(n4);
    }
    if (e == hipSuccess) {
      for (void* p : {(void*)g.nodes, (void*)g.tris, (void*)g.tri_flags}) c->scene_allocs.push_back(p);
      s.nodes = g.nodes;
      s.tris = g.tris;
      s.tri_flags = g.tri_flags;
      s.deep_stack = need >= PTGS_STACK ? 1 : 0;
      c->info.num_bvh_nodes = g.num_nodes;
      c->info.bvh_depth = g.depth;
      c->info.max_leaf_size = (c->flags & PTGS_FLAG_GPU_LBVH) ? 4u : g.max_leaf;
      c->info.build_ms = ms;
      c->info.device_bytes += (size_t)g.num_nodes * 128 + tris.size() * 52;
      built = true;
    } else if (e == hipErrorNotSupported) {
      (void)hipFree(g.nodes);
      (void)hipFree(g.tris);
      (void)hipFree(g.tri_flags);
    } else {
      (void)hipFree(g.nodes);
      (void)hipFree(g.tris);
      (void)hipFree(g.tri_flags);
      return fail(c, PTGS_EHIP, "GPU BVH build: %s", hipGetErrorString(e));
    }
  }
  if (!built) {
    auto t0 = std::chrono::steady_clock::now();
    BvhOut bvh;
    std::vector<float> n4;
    uint32_t num4 = 0, dep4 = 0, need = PTGS_STACK_TOTAL;
    int built_leaf = -1;
    bool fits = false;
    uint32_t built_depth = 0;
    for (const BvhTry& tr : bvh_tries()) {
      if (tr.leaf != built_leaf || tr.depth != built_depth) {
        build_bvh(tris, tr.leaf, tr.depth, bvh);
        built_leaf = tr.leaf;
        built_depth = tr.depth;
        if (bvh.depth >= PTGS_STACK) return fail(c, PTGS_ERANGE, "BVH depth %u exceeds the traversal stack", bvh.depth);
      }
      fits = collapse_fit(bvh.nodes, n4, num4, dep4, tr.fan, need);
      bvh_log("host", tr.leaf, tr.fan, tr.depth, dep4, need);
      if (fits) break;
    }
    auto t1 = std::chrono::steady_clock::now();
    if (!fits) return fail(c, PTGS_ERANGE, "BVH depth %u exceeds the traversal stack", bvh.depth);
    s.deep_stack = need >= PTGS_STACK ? 1 : 0;
    if ((rc = upload(c, (const float4*)n4.data(), n4.size() / 4, &s.nodes))) return rc;
    bvh.num_nodes = num4;
    bvh.depth = dep4;
    if ((rc = upload(c, (const float4*)bvh.tris.data(), bvh.tris.size() / 4, &s.tris))) return rc;
    if ((rc = upload(c, bvh.tri_flags.data(), bvh.tri_flags.size(), &s.tri_flags))) return rc;
    c->info.num_bvh_nodes = bvh.num_nodes;
    c->info.bvh_depth = bvh.depth;
    c->info.max_leaf_size = bvh.max_leaf;
    c->info.build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  }
  // The traversal reads 4-wide nodes through a buffer descriptor with 32-bit byte offsets (node << 7,
  // num_records 0x7fffffff: pt_device.h box4): nodes past 2 GiB would read as zeros (no boxes, child
  // link 0) without a fault. Such a tree (~16.7M nodes, some 50M triangles) is refused here.
  if (c->info.num_bvh_nodes > bvh_node_limit())
    return fail(c, PTGS_ERANGE, "BVH of %u 4-wide nodes exceeds the traversal's 2 GiB node window (%u nodes)",
                c->info.num_bvh_nodes, bvh_node_limit());
  // a zero vertex/index count still needs valid (never dereferenced) pointers
  ptgs_vertex dummy_v{};
  uint32_t dummy_i = 0;
  ptgs_mesh_info dummy_m{};
  if ((rc = upload(c, d->num_vertices ? d->vertices : &dummy_v, d->num_vertices ? d->num_vertices : 1, &s.vertices))) return rc;
  if ((rc = upload(c, d->num_indices ? d->indices : &dummy_i, d->num_indices ? d->num_indices : 1, &s.indices))) return rc;
  if ((rc = upload(c, d->num_meshes ? d->meshes : &dummy_m, d->num_meshes ? d->num_meshes : 1, &s.meshes))) return rc;
  if ((rc = upload(c, d->materials, d->num_materials, &s.materials))) return rc;
  {
    const uint32_t zero4[4] = {0, 0, 0, 0};
    if ((rc = upload(c, (const uint4*)(hitrec.empty() ? zero4 : hitrec.data()), hitrec.empty() ? 1 : hitrec.size() / 4,
                     &s.hitrec)))
      return rc;
  }
  if ((rc = upload(c, d->light_triangles, d->num_light_triangles, &s.light_tris))) return rc;
  if ((rc = upload(c, d->light_cdf, d->num_light_cdf, &s.light_cdf))) return rc;
  if ((rc = upload(c, d->punctual_lights, d->num_punctual_lights, &s.plights))) return rc;
  if ((rc = upload(c, d->punctual_cdf, d->num_punctual_cdf, &s.pcdf))) return rc;
  if ((rc = upload(c, (const float4*)d->blue_noise_rgba32f, (size_t)bn * bn, &s.blue_noise))) return rc;
  if ((rc = upload(c, texpool.texels.data(), texpool.texels.size(), &s.tex.texels))) return rc;
  if ((rc = upload(c, texpool.info.data(), texpool.info.size(), &s.tex.info))) return rc;
  if ((rc = upload(c, texpool.lut.data(), texpool.lut.size(), &s.tex.lut))) return rc;
  s.tex.count = d->num_textures;
  s.uses_textures = 0;
  for (uint32_t i = 0; i < d->num_materials; ++i) {
    const ptgs_material& m = d->materials[i];
    if (m.albedo_texture_index > 0 || m.normal_texture_index > 0 || m.metallic_roughness_texture_index > 0 ||
        m.emissive_texture_index > 0 || m.clearcoat_texture_index > 0 || m.clearcoat_roughness_texture_index > 0 ||
        m.sg_id > 0)
      s.uses_textures = 1;
  }
  s.num_light_cdf = d->num_light_cdf;
  s.num_plights = d->num_punctual_lights;
  s.bn_size = (int32_t)bn;
  s.has_transparent = has_transparent ? 1 : 0;
  c->dsc = s;
  c->has_scene = true;
  c->info.num_triangles = (uint32_t)tris.size();
  return PTGS_OK;
}

int ptgs_scene_get_info(const ptgs_ctx* c, ptgs_scene_info* out) {
  if (!c || !out) return PTGS_EINVAL;
  if (!c->has_scene) return PTGS_ENOSCENE;
  *out = c->info;
  return PTGS_OK;
}

int ptgs_scene_get_bvh(const ptgs_ctx* c, ptgs_bvh_buffers* out) {
  if (!c || !out) return PTGS_EINVAL;
  if (!c->has_scene) return PTGS_ENOSCENE;
  out->nodes = (const float*)c->dsc.nodes;
  out->num_nodes = c->info.num_bvh_nodes;
  out->triangles = (const float*)c->dsc.tris;
  out->num_triangles = c->info.num_triangles;
  return PTGS_OK;
}

int ptgs_trace_camera_rows(ptgs_ctx* c, const ptgs_ubo* ubo, uint32_t w, uint32_t h, uint32_t row_begin,
                           uint32_t row_end, float* accum, uint32_t spp, uint32_t frame_stride,
                           uint32_t accum_mode, void* stream) {
  if (!c || !ubo || !accum) return fail(c, PTGS_EINVAL, "null argument");
  if (!c->has_scene) return fail(c, PTGS_ENOSCENE, "no scene uploaded");
  if (w == 0 || h == 0 || w > 32768 || h > 32768) return fail(c, PTGS_EINVAL, "bad image size %ux%u", w, h);
  if (row_end > h) row_end = h;
  if (row_begin > row_end) return fail(c, PTGS_EINVAL, "bad row range");
  if (frame_stride == 0) return fail(c, PTGS_EINVAL, "frame_stride must be >= 1");
  if (accum_mode > PTGS_ACCUM_SUM) return fail(c, PTGS_EINVAL, "bad accum mode");
  if (!is_device_ptr(accum)) return fail(c, PTGS_EINVAL, "accum is not a device pointer");
  HIPCHK(c, hipSetDevice(c->device));
  CamParams cp;
  int rc = fill_cam(c, ubo, cp);
  if (rc) return rc;
  const bool stats = (c->flags & PTGS_FLAG_COUNT_TRAVERSAL) != 0;
  hipError_t e;
  if (c->flags & PTGS_FLAG_PT_WAVEFRONT) {
    e = ptgs::launch_pt_wavefront(c->wf, c->dsc, cp, accum, w, h, row_begin, row_end, spp, ubo->frame_count,
                                  frame_stride, accum_mode, c->counters, stats, (hipStream_t)stream);
    if (e != hipSuccess) return fail(c, PTGS_EHIP, "wavefront path tracer: %s", hipGetErrorString(e));
    return PTGS_OK;
  }
  e = launch_pt_camera(c->dsc, cp, accum, w, h, row_begin, row_end, spp, ubo->frame_count, frame_stride, accum_mode,
                       c->counters, stats, &c->pt_sched, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "pt_camera launch: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_trace_camera(ptgs_ctx* c, const ptgs_ubo* ubo, uint32_t w, uint32_t h, float* accum, uint32_t spp,
                      uint32_t frame_stride, uint32_t accum_mode, void* stream) {
  return ptgs_trace_camera_rows(c, ubo, w, h, 0, h, accum, spp, frame_stride, accum_mode, stream);
}

int ptgs_trace_depth(ptgs_ctx* c, const ptgs_ubo* ubo, uint32_t w, uint32_t h, float* depth, void* stream) {
  return ptgs_trace_depth_rows(c, ubo, w, h, 0, h, depth, stream);
}

int ptgs_trace_depth_rows(ptgs_ctx* c, const ptgs_ubo* ubo, uint32_t w, uint32_t h, uint32_t row_begin,
                          uint32_t row_end, float* depth, void* stream) {
  if (!c || !ubo || !depth) return fail(c, PTGS_EINVAL, "null argument");
  if (!c->has_scene) return fail(c, PTGS_ENOSCENE, "no scene uploaded");
  if (w == 0 || h == 0 || w > 32768 || h > 32768) return fail(c, PTGS_EINVAL, "bad image size %ux%u", w, h);
  if (!is_device_ptr(depth)) return fail(c, PTGS_EINVAL, "depth is not a device pointer");
  HIPCHK(c, hipSetDevice(c->device));
  CamParams cp;
  int rc = fill_cam(c, ubo, cp);
  if (rc) return rc;
  ViewMat vm;
  std::memcpy(vm.m, ubo->view, sizeof(vm.m));
  hipError_t e = launch_pt_depth(c->dsc, cp, vm, depth, w, h, row_begin, row_end, ubo->frame_count, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "pt_depth launch: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_trace_torus(ptgs_ctx* c, const ptgs_ubo* ubo, const ptgs_ray_push* push, const ptgs_ray_sample* samples,
                     uint32_t n, ptgs_hitdata* hits, void* stream) {
  if (!c || !ubo || !push) return fail(c, PTGS_EINVAL, "null argument");
  if (!c->has_scene) return fail(c, PTGS_ENOSCENE, "no scene uploaded");
  if (n == 0) return PTGS_OK;
  if (!is_device_ptr(samples) || !is_device_ptr(hits)) return fail(c, PTGS_EINVAL, "samples/hits must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  CamParams cp;
  int rc = fill_cam(c, ubo, cp);
  if (rc) return rc;
  TorusParams tp;
  std::memcpy(tp.model, push->model, sizeof(tp.model));
  tp.major_radius = push->major_radius;
  tp.minor_radius = push->minor_radius;
  tp.height = push->height;
  // side = ceil(sqrt(n)) (engine.cpp:2786)
  uint32_t side = (uint32_t)std::ceil(std::sqrt((double)n));
  while ((uint64_t)side * side < n) side++;
  hipError_t e = launch_pt_torus(c->dsc, cp, tp, samples, n, side, ubo->frame_count, hits, c->counters,
                                 (c->flags & PTGS_FLAG_COUNT_TRAVERSAL) != 0, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "pt_torus launch: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_set_flags(ptgs_ctx* c, uint32_t flags) {
  if (!c) return PTGS_EINVAL;
  c->flags = flags;
  return PTGS_OK;
}

int ptgs_stats_reset(ptgs_ctx* c, void* stream) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemsetAsync(c->counters, 0, 8 * sizeof(unsigned long long), (hipStream_t)stream));
  return PTGS_OK;
}

int ptgs_stats_read(ptgs_ctx* c, ptgs_trace_stats* out) {
  if (!c || !out) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipDeviceSynchronize());
  unsigned long long v[8];
  HIPCHK(c, hipMemcpy(v, c->counters, sizeof(v), hipMemcpyDeviceToHost));
  out->extension_rays = v[0];
  out->shadow_rays = v[1];
  out->samples = v[2];
  out->node_visits = v[3];
  out->tri_tests = v[4];
  out->closest_hits = v[5];
  return PTGS_OK;
}

int ptgs_device_alloc(ptgs_ctx* c, size_t bytes, void** out) {
  if (!c || !out) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMalloc(out, bytes ? bytes : 16));
  return PTGS_OK;
}
int ptgs_device_free(ptgs_ctx* c, void* p) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipFree(p));
  return PTGS_OK;
}
int ptgs_memcpy_h2d(ptgs_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return PTGS_OK;
}
int ptgs_memcpy_d2h(ptgs_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return PTGS_OK;
}
int ptgs_memset_d32(ptgs_ctx* c, void* dst, uint32_t value, size_t count, void* stream) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)dst, (int)value, count, (hipStream_t)stream));
  return PTGS_OK;
}
int ptgs_synchronize(ptgs_ctx* c) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipDeviceSynchronize());
  return PTGS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// rasterizers
// ---------------------------------------------------------------------------------------------
#include "raster.h"

extern "C" {

// Renders one frame; PTGS_OK means it was enqueued completely. *report (bit 0: an earlier frame was left
// incomplete, bit 1: an earlier frame met ids >= count) is about EARLIER frames of the workspace: the
// caller turns it into PTGS_EINCOMPLETE / PTGS_EINVAL (splat_report) once everything it renders is enqueued.
static int splat_render(ptgs_ctx* c, const ptgs_gaussians* g, const ptgs_ubo* ubo, uint32_t w, uint32_t h,
                        const float bg[3], const float* depth, const float* under, uint32_t tile_row_begin,
                        uint32_t tile_row_end, float* out, ptgs_splat_stats* stats, void* stream, uint32_t* report,
                        const SplatOverlap* ov = nullptr, SplatSeq* seq = nullptr) {
  *report = 0;
  if (w == 0 || h == 0 || w > 32768 || h > 32768) return fail(c, PTGS_EINVAL, "bad image size %ux%u", w, h);
  if (g->count && (!is_device_ptr(g->means) || !is_device_ptr(g->scales) || !is_device_ptr(g->rotations) ||
                   !is_device_ptr(g->opacities) || !is_device_ptr(g->colors) || (g->ids && !is_device_ptr(g->ids))))
    return fail(c, PTGS_EINVAL, "gaussian arrays must be device pointers");
  if (!is_device_ptr(out)) return fail(c, PTGS_EINVAL, "out is not a device pointer");
  if ((depth && !is_device_ptr(depth)) || (under && !is_device_ptr(under)))
    return fail(c, PTGS_EINVAL, "depth / under must be device pointers");
  if (ubo->proj[0] == 0.0f || ubo->proj[5] == 0.0f) return fail(c, PTGS_EINVAL, "degenerate projection");
  HIPCHK(c, hipSetDevice(c->device));
  float mvp[16];
  mat4_mul(ubo->proj, ubo->view, mvp);
  hipError_t e = splat_gaussians(c->splat, g, ubo->view, mvp, ubo->proj[0], ubo->proj[5], w, h, bg, depth, under,
                                 tile_row_begin, tile_row_end, out, stats, (c->flags & PTGS_FLAG_TIME_STAGES) != 0,
                                 (c->flags & PTGS_FLAG_SPLAT_PUBLISH) != 0, (c->flags & PTGS_FLAG_SPLAT_PUBLISH_TIGHT) != 0,
                                 (hipStream_t)stream, report, ov, seq);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "splat_gaussians: %s", hipGetErrorString(e));
  return PTGS_OK;
}

// (the frames of this call are rendered; the codes report earlier frames of the workspace(s))
static int splat_report(ptgs_ctx* c, uint32_t report);
// The reports a call collected (earlier frames' flags, consumed from the workspaces) and its own result:
// a failing call keeps them for the next call (they are returned once, never dropped); a
// successful one returns them together with any kept earlier.
static int splat_finish(ptgs_ctx* c, int rc, uint32_t report) {
  report |= c->pending_report;
  c->pending_report = 0;
  if (rc != PTGS_OK) {
    c->pending_report = report;
    return rc;
  }
  return splat_report(c, report);
}
static int splat_report(ptgs_ctx* c, uint32_t report) {
  if (report & 2u) return fail(c, PTGS_EBADIDS, "an earlier splat frame met ptgs_gaussians.ids entries >= count");
  if (report & 1u)
    return fail(c, PTGS_EINCOMPLETE, "an earlier splat frame left tiles incomplete (spill pool exhausted; grown)");
  return PTGS_OK;
}

// PTGS_FLAG_SPLAT_OVERLAP: the call takes the ring's next workspace (the one of the call depth calls back)
// and, for a stream-ordered frame, its front end runs on the context's second stream. The first call of a
// run of overlapped calls starts it after everything the caller's stream holds; later calls' front ends
// wait on the device for the earlier blends of their workspace only (gs_done_wait), so inputs the caller
// writes during a run are not seen by it. A call without the flag ends the run (ov_started is cleared).
// workspaces in the ring, fixed when a context first overlaps (PTGS_GS_OV_DEPTH=2 .. 4; A/B switch)
static uint32_t overlap_depth() {
  const char* v = getenv("PTGS_GS_OV_DEPTH");
  const int x = v ? atoi(v) : PTGS_OV_DEPTH_DEFAULT;
  return (uint32_t)std::max(2, std::min(x, PTGS_OV_RING));
}

static int splat_overlap_begin(ptgs_ctx* c, hipStream_t s, SplatOverlap* ov, SplatSeq* seq) {
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->ov_ring[0]) {  // the ring starts at the current workspace
    c->ov_ring[0] = c->splat;
    c->ov_pos = 0;
    c->ov_depth = overlap_depth();
  }
  const uint32_t depth = c->ov_depth;
  for (uint32_t i = 1; i < depth; ++i)
    if (!c->ov_ring[i]) c->ov_ring[i] = splat_workspace_create();
  if (!c->ov_stream) {
    // the front end's queue at the highest priority, so its workgroups take the CU slots of the blend's
    // retiring workgroups early instead of waiting for the blend's tail (PTGS_GS_OV_PRIO=normal: A/B switch)
    int least = 0, greatest = 0, prio = 0;
    const char* pv = getenv("PTGS_GS_OV_PRIO");
    if (!(pv && !strcmp(pv, "normal")) && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      prio = greatest;
    HIPCHK(c, hipStreamCreateWithPriority(&c->ov_stream, hipStreamNonBlocking, prio));
  }
  // (device-scope events: both streams are on this device, so no system-scope release (an L2 write-back)
  // is needed at the record; PTGS_GS_OV_FENCE=1 restores it: A/B switch)
  static const unsigned ev_flags = [] {
    const char* v = getenv("PTGS_GS_OV_FENCE");
    return (unsigned)(hipEventDisableTiming | (v && !strcmp(v, "1") ? 0u : (unsigned)hipEventDisableSystemFence));
  }();
  for (hipEvent_t* ev : {&c->ov_call[0], &c->ov_done})
    if (!*ev) HIPCHK(c, hipEventCreateWithFlags(ev, ev_flags));
  if (!c->ov_flag) {  // (signal memory for the front end's wait-value packet; zero before any blend stores)
    HIPCHK(c, hipExtMallocWithFlags((void**)&c->ov_flag, 8, hipMallocSignalMemory));
    HIPCHK(c, hipMemset(c->ov_flag, 0, 8));
  }
  // the next ring slot; the workspace there was last used depth calls ago (call k - depth). Its blend ran
  // before the blend of call k - depth + 1 on the caller's stream, so once THAT blend has started (its
  // ordinal in ov_flag, SplatSeq) the workspace is free: the front end's queue waits for that value and the
  // caller's queue carries no marker (a marker beside the cross-queue barrier had cost it ~3-5 us per frame:
  // tools/micro/queue_sync.hip, wait + marker 28.0 vs wait alone 25.1 us on a 22 us kernel; kernel trace
  // 10.5 vs 6.0 us between two blends). The first call of a run waits for a marker of the caller's stream
  // (everything enqueued before the run), as do calls whose ordering is not known (no blend launched, or a
  // call on another stream: then a new marker).
  const uint32_t cur = (c->ov_pos + 1) % depth;
  c->ov_pos = cur;
  c->splat = c->ov_ring[cur];
  const uint32_t k = c->ov_started, back = depth - 1;
  bool same = true;
  for (uint32_t j = 1; j <= std::min(k, back); ++j) same = same && c->ov_strm[(k - j) & 3u] == s;
  ov->fe = c->ov_stream;
  ov->done = c->ov_done;
  ov->wait = nullptr;
  ov->wait_flag = nullptr;
  ov->wait_ordinal = 0;
  if (k >= back && same && c->ov_ord[(k - back) & 3u]) {
    ov->wait_flag = c->ov_flag;
    ov->wait_ordinal = c->ov_ord[(k - back) & 3u];
  } else {
    // (k < back on the run's stream: the workspace was last used before the run, so the marker recorded at
    // the run's start (or a later one) covers it; otherwise a new marker)
    if (!(k > 0 && k < back && same)) HIPCHK(c, hipEventRecord(c->ov_call[0], s));
    ov->wait = c->ov_call[0];
  }
  seq->flag = c->ov_flag;
  seq->ordinal = c->ov_next;
  seq->launched = false;
  // the blend's tile order: the front end's order workgroup from the workspace's previous frame (default),
  // or PTGS_GS_OV_ORDER=own: a launch behind the front end from the frame's own counts (A/B switch;
  // measured slower at C2 static, 0.0531 vs 0.0521 ms, and not faster on the orbit: DESIGN §5 round 6)
  static const bool own_order = [] {
    const char* v = getenv("PTGS_GS_OV_ORDER");
    return v && !strcmp(v, "own");
  }();
  ov->own_order = own_order;
  return PTGS_OK;
}

// after the call's frame: its blend's ordinal and stream (see splat_overlap_begin)
static void splat_overlap_end(ptgs_ctx* c, hipStream_t s, const SplatSeq& seq) {
  const uint32_t k = c->ov_started;
  c->ov_ord[k & 3u] = seq.launched ? seq.ordinal : 0u;
  c->ov_strm[k & 3u] = s;
  if (seq.launched) c->ov_next = seq.ordinal + 1u;
  c->ov_started = k + 1u < 4u ? k + 1u : 4u + ((k + 1u) & 3u);  // (>= 4: every look-back valid; the index mod 4 kept)
}

static int splat_common(ptgs_ctx* c, const ptgs_gaussians* g, const ptgs_ubo* ubo, uint32_t w, uint32_t h,
                        const float bg[3], const float* depth, const float* under, uint32_t tile_row_begin,
                        uint32_t tile_row_end, float* out, ptgs_splat_stats* stats, void* stream) {
  uint32_t report = 0;
  SplatOverlap ov{};
  SplatSeq seq{};
  const SplatOverlap* ovp = nullptr;
  if (c->flags & PTGS_FLAG_SPLAT_OVERLAP) {
    const int rc = splat_overlap_begin(c, (hipStream_t)stream, &ov, &seq);
    if (rc != PTGS_OK) return rc;
    ovp = &ov;  // (splat_gaussians runs a frame with stats / publish / stage timing serially anyway)
  } else {
    c->ov_started = 0;
  }
  const int rc = splat_render(c, g, ubo, w, h, bg, depth, under, tile_row_begin, tile_row_end, out, stats, stream,
                              &report, ovp, ovp ? &seq : nullptr);
  if (ovp) splat_overlap_end(c, (hipStream_t)stream, seq);
  return splat_finish(c, rc, report);
}

int ptgs_splat_gaussians(ptgs_ctx* c, const ptgs_gaussians* g, const ptgs_ubo* ubo, uint32_t w, uint32_t h,
                         const float bg[3], uint32_t tile_row_begin, uint32_t tile_row_end, float* out,
                         ptgs_splat_stats* stats, void* stream) {
  if (!c || !g || !ubo || !out || !bg) return fail(c, PTGS_EINVAL, "null argument");
  return splat_common(c, g, ubo, w, h, bg, nullptr, nullptr, tile_row_begin, tile_row_end, out, stats, stream);
}

int ptgs_splat_gaussians_over(ptgs_ctx* c, const ptgs_gaussians* g, const ptgs_ubo* ubo, uint32_t w, uint32_t h,
                              const float* depth, const float* under_rgba32f, uint32_t tile_row_begin,
                              uint32_t tile_row_end, float* out, ptgs_splat_stats* stats, void* stream) {
  if (!c || !g || !ubo || !out || !depth || !under_rgba32f) return fail(c, PTGS_EINVAL, "null argument");
  const float zero[3] = {0.0f, 0.0f, 0.0f};
  return splat_common(c, g, ubo, w, h, zero, depth, under_rgba32f, tile_row_begin, tile_row_end, out, stats, stream);
}

int ptgs_splat_gaussians_views(ptgs_ctx* c, const ptgs_gaussians* g, uint32_t n_views, const ptgs_ubo* ubos,
                               uint32_t w, uint32_t h, const float bg[3], float* const* outs, void* stream) {
  if (!c || !g || !ubos || !outs || !bg) return fail(c, PTGS_EINVAL, "null argument");
  if (n_views == 0 || n_views > PTGS_MAX_VIEWS) return fail(c, PTGS_EINVAL, "n_views %u not in [1, %d]", n_views, PTGS_MAX_VIEWS);
  for (uint32_t v = 0; v < n_views; ++v)
    if (!outs[v]) return fail(c, PTGS_EINVAL, "null output of view %u", v);
  if (n_views == 1) return splat_common(c, g, &ubos[0], w, h, bg, nullptr, nullptr, 0, ~0u, outs[0], nullptr, stream);
  HIPCHK(c, hipSetDevice(c->device));
  c->ov_started = 0;  // (view 0 renders serially on the caller's stream with the latest workspace)
  const hipStream_t s = (hipStream_t)stream;
  if (!c->view_fork) HIPCHK(c, hipEventCreateWithFlags(&c->view_fork, hipEventDisableTiming));
  // every view's pair buffer starts from the largest pair count any slot has seen (views of one
  // Gaussian set have similar counts): a fresh view workspace would otherwise start at 8 pairs per
  // Gaussian and skip its first over-capacity frame (reported by ptgs_splat_status_read)
  uint32_t hint = splat_pair_hint(c->splat);
  for (uint32_t v = 1; v < n_views; ++v) {
    if (!c->view_ws[v]) c->view_ws[v] = splat_workspace_create();
    if (!c->view_stream[v]) HIPCHK(c, hipStreamCreateWithFlags(&c->view_stream[v], hipStreamNonBlocking));
    if (!c->view_join[v]) HIPCHK(c, hipEventCreateWithFlags(&c->view_join[v], hipEventDisableTiming));
    hint = std::max(hint, splat_pair_hint(c->view_ws[v]));
  }
  if (hint) {
    const uint32_t want = hint + hint / 8u;  // headroom for the views' differences
    for (uint32_t v = 1; v < n_views; ++v) HIPCHK(c, splat_reserve(c->view_ws[v], want));
  }
  HIPCHK(c, hipEventRecord(c->view_fork, s));  // the views start after the caller's earlier work
  // on any failure after a view was forked, the views already launched are joined back into the
  // caller's stream before returning (later work there must not race them)
  uint32_t launched = 1;
  uint32_t report = 0;  // the views' reports about their earlier frames (PTGS_EINCOMPLETE / PTGS_EINVAL)
  auto join = [&]() {
    for (uint32_t v = 1; v < launched; ++v) (void)hipStreamWaitEvent(s, c->view_join[v], 0);
  };
  for (uint32_t v = 1; v < n_views; ++v) {
    hipError_t e = hipStreamWaitEvent(c->view_stream[v], c->view_fork, 0);
    if (e != hipSuccess) {
      join();
      return splat_finish(c, fail(c, PTGS_EHIP, "hipStreamWaitEvent: %s", hipGetErrorString(e)), report);
    }
    SplatWorkspace* keep = c->splat;
    c->splat = c->view_ws[v];
    uint32_t rep = 0;
    const int rc = splat_render(c, g, &ubos[v], w, h, bg, nullptr, nullptr, 0, ~0u, outs[v], nullptr, c->view_stream[v],
                                &rep);
    c->splat = keep;
    report |= rep;  // (about earlier frames of view v's workspace: returned once every view is enqueued)
    // (record the join even after a failed view: kernels it did enqueue must be waited for)
    e = hipEventRecord(c->view_join[v], c->view_stream[v]);
    if (e == hipSuccess) launched = v + 1;
    if (rc != PTGS_OK) { join(); return splat_finish(c, rc, report); }
    if (e != hipSuccess) { join(); return splat_finish(c, fail(c, PTGS_EHIP, "hipEventRecord: %s", hipGetErrorString(e)), report); }
  }
  uint32_t rep = 0;
  const int rc = splat_render(c, g, &ubos[0], w, h, bg, nullptr, nullptr, 0, ~0u, outs[0], nullptr, stream, &rep);
  join();
  return splat_finish(c, rc, report | rep);
}

int ptgs_gaussians_sort_spatial(ptgs_ctx* c, const ptgs_gaussians* g, float* means, float* scales, float* rotations,
                                float* opacities, float* colors, uint32_t* ids, void* stream) {
  if (!c || !g) return fail(c, PTGS_EINVAL, "null argument");
  if (g->count) {
    const void* all[] = {g->means, g->scales, g->rotations, g->opacities, g->colors, means, scales, rotations,
                         opacities, colors, ids};
    for (const void* p : all)
      if (!is_device_ptr(p)) return fail(c, PTGS_EINVAL, "gaussian arrays must be device pointers");
    if (g->ids && !is_device_ptr(g->ids)) return fail(c, PTGS_EINVAL, "ids must be a device pointer");
  }
  HIPCHK(c, hipSetDevice(c->device));
  const hipError_t e = splat_sort_spatial(g, means, scales, rotations, opacities, colors, ids, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "ptgs_gaussians_sort_spatial: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_gaussians_chunk_bounds(ptgs_ctx* c, const ptgs_gaussians* g, float* bounds, void* stream) {
  if (!c || !g || !bounds) return fail(c, PTGS_EINVAL, "null argument");
  if (g->count && (!is_device_ptr(g->means) || !is_device_ptr(g->scales) || !is_device_ptr(bounds)))
    return fail(c, PTGS_EINVAL, "means / scales / bounds must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  const hipError_t e = splat_chunk_bounds(g, bounds, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "ptgs_gaussians_chunk_bounds: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_splat_status_read(ptgs_ctx* c, ptgs_splat_status* out, void* stream) {
  if (!c || !out) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  for (int v = 1; v < PTGS_MAX_VIEWS; ++v)
    if (c->view_stream[v]) HIPCHK(c, hipStreamSynchronize(c->view_stream[v]));
  if (c->ov_stream) HIPCHK(c, hipStreamSynchronize(c->ov_stream));
  *out = ptgs_splat_status{};
  out->pair_capacity = 0xFFFFFFFFu;
  // (slot 0 also holds the other ring workspaces of PTGS_FLAG_SPLAT_OVERLAP: indices >= PTGS_MAX_VIEWS here)
  for (int v = 0; v < PTGS_MAX_VIEWS + PTGS_OV_RING; ++v) {
    SplatWorkspace* ws = v == 0 ? c->splat : v < PTGS_MAX_VIEWS ? c->view_ws[v] : c->ov_ring[v - PTGS_MAX_VIEWS];
    if (!ws || (v >= PTGS_MAX_VIEWS && ws == c->splat)) continue;
    const int slot = v >= PTGS_MAX_VIEWS ? 0 : v;
    SplatStatusOut so;
    HIPCHK(c, splat_status(ws, true, &so));
    out->views[slot] += so.incomplete;
    out->frames += so.incomplete;
    out->spilled_tiles += so.spilled_tiles;
    out->incomplete_tiles += so.incomplete_tiles;
    if (v < PTGS_MAX_VIEWS || so.last_pairs) out->pair_capacity = std::min(out->pair_capacity, so.capacity);
    // the latest frame's pairs: the current workspace's (slot 0), else any view's
    if (v < PTGS_MAX_VIEWS) out->last_pairs = std::max(out->last_pairs, so.last_pairs);
    if (slot == 0) {
      out->spill_capacity = v == 0 ? so.spill_capacity : std::min(out->spill_capacity, so.spill_capacity);
      out->spill_demand = std::max(out->spill_demand, so.spill_demand);
    }
  }
  if (c->splat) splat_front_end_info(c->splat, &out->touched_runs, &out->fused);
  return PTGS_OK;
}

int ptgs_splat_reserve(ptgs_ctx* c, uint32_t pairs) {
  if (!c) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, splat_reserve(c->splat, pairs));
  for (int v = 1; v < PTGS_MAX_VIEWS; ++v)
    if (c->view_ws[v]) HIPCHK(c, splat_reserve(c->view_ws[v], pairs));
  for (SplatWorkspace* w : c->ov_ring)
    if (w && w != c->splat) HIPCHK(c, splat_reserve(w, pairs));
  return PTGS_OK;
}

int ptgs_splat_get_buffers(const ptgs_ctx* c, ptgs_splat_buffers* out) {
  if (!c || !out) return PTGS_EINVAL;
  splat_get_buffers(c->splat, out);
  return PTGS_OK;
}

int ptgs_splat_get_tile_rows(const ptgs_ctx* c, const uint64_t** rows, uint32_t* row_capacity) {
  if (!c || !rows || !row_capacity) return PTGS_EINVAL;
  const unsigned long long* r = nullptr;
  splat_get_tile_rows(c->splat, &r, row_capacity);
  *rows = (const uint64_t*)r;
  return PTGS_OK;
}

int ptgs_splat_stage_ms(ptgs_ctx* c, float out_ms[6]) {
  if (!c || !out_ms) return PTGS_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, splat_stage_ms(c->splat, out_ms));
  return PTGS_OK;
}

int ptgs_splat_points(ptgs_ctx* c, const ptgs_ubo* ubo, const ptgs_ray_push* push, const ptgs_hitdata* hits,
                      const ptgs_ray_sample* samples, uint32_t n, uint32_t w, uint32_t h, uint32_t* rgba8,
                      float* depth, void* stream) {
  if (!c || !ubo || !push || !rgba8 || !depth) return fail(c, PTGS_EINVAL, "null argument");
  if (w == 0 || h == 0 || w > 32768 || h > 32768) return fail(c, PTGS_EINVAL, "bad image size %ux%u", w, h);
  if (n && (!is_device_ptr(hits) || (push->mode == 1 && !is_device_ptr(samples))))
    return fail(c, PTGS_EINVAL, "hits/samples must be device pointers");
  if (!is_device_ptr(rgba8) || !is_device_ptr(depth)) return fail(c, PTGS_EINVAL, "rgba8/depth must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  float mvp[16];
  mat4_mul(ubo->proj, ubo->view, mvp);
  unsigned long long* keys = nullptr;
  HIPCHK(c, splat_point_keys(c->splat, (size_t)w * h, &keys));
  hipError_t e = launch_splat_points(mvp, push->model, push->major_radius, push->minor_radius, push->height,
                                     push->mode, hits, samples, n, w, h, keys, depth, rgba8, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "splat_points: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_encode_srgb8(ptgs_ctx* c, const float* rgba32f, uint32_t w, uint32_t h, uint32_t* rgba8, void* stream) {
  if (!c || !rgba32f || !rgba8) return fail(c, PTGS_EINVAL, "null argument");
  if (!is_device_ptr(rgba32f) || !is_device_ptr(rgba8)) return fail(c, PTGS_EINVAL, "buffers must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  hipError_t e = launch_encode_srgb8(rgba32f, rgba8, w * h, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "encode_srgb8: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_knn3_mean_dist2(ptgs_ctx* c, const float* xyz, uint32_t n, float* dist2, void* stream) {
  if (!c || (n && (!xyz || !dist2))) return fail(c, PTGS_EINVAL, "null argument");
  if (n == 0) return PTGS_OK;
  if (!is_device_ptr(xyz) || !is_device_ptr(dist2)) return fail(c, PTGS_EINVAL, "buffers must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  hipError_t e = ptgs::knn3_mean_dist2(xyz, n, dist2, (hipStream_t)stream, nullptr);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "knn3_mean_dist2: %s", hipGetErrorString(e));
  return PTGS_OK;
}

int ptgs_gaussians_from_points(ptgs_ctx* c, const float* xyz, const uint8_t* rgb, uint32_t n, float* means,
                               float* scales, float* rotations, float* opacities, float* colors, void* stream) {
  if (!c || (n && (!xyz || !means || !scales || !rotations || !opacities || !colors)))
    return fail(c, PTGS_EINVAL, "null argument");
  if (n == 0) return PTGS_OK;
  const void* ptrs[] = {xyz, means, scales, rotations, opacities, colors};
  for (const void* p : ptrs)
    if (!is_device_ptr(p)) return fail(c, PTGS_EINVAL, "buffers must be device pointers");
  if (rgb && !is_device_ptr(rgb)) return fail(c, PTGS_EINVAL, "buffers must be device pointers");
  HIPCHK(c, hipSetDevice(c->device));
  hipError_t e = ptgs::gaussians_from_points(xyz, rgb, n, means, scales, rotations, opacities, colors,
                                             (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, PTGS_EHIP, "gaussians_from_points: %s", hipGetErrorString(e));
  return PTGS_OK;
}

}  // extern "C"
