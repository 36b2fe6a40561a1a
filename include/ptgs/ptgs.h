/*
 * ptgs.h — C-ABI of the MI355X-native path tracer / Gaussian-splat renderer.
 *
 * This is the drop-in boundary for the two data-parallel hot paths of
 * FedericoCos/PathTracer_GaussianSplatting (reference tree: /root/reference, read-only).
 * The reference has no FFI; its hot path sits behind the Vulkan RT pipeline:
 *   - descriptor set bindings 0-14           Vulkan_Engine/engine.cpp:2169-2224, shaders/rt_render/raytracing.glsl:109-138
 *   - push constant RayPushConstant (80 B)   Helpers/GeneralHeaders.h:526-532
 *   - launch vkCmdTraceRaysKHR(W, H, 1)      Vulkan_Engine/engine.cpp:1971-1976 (camera), :2789 (torus)
 *   - per-frame protocol ubo.frame_count     Vulkan_Engine/engine.cpp:2134, :2070-2072
 * Every struct below is byte-compatible with Helpers/GeneralHeaders.h so the reference's
 * Engine can hand its host arrays straight to ptgs_scene_upload() and replace
 * vkCmdTraceRaysKHR + the running-mean image with ptgs_trace_camera().
 *
 * Conventions:
 *   - every entry point returns 0 (PTGS_OK) or a negative PTGS_E* code; no exceptions cross the ABI,
 *     nothing aborts; ptgs_last_error() returns a message for the last failure on a context.
 *   - compute entry points are stream-ordered (hipStream_t passed as void*); the caller synchronises.
 *   - "device pointer" arguments must be device-accessible memory of the context's HIP device.
 *   - a context is not thread-safe (thread-compatible): one host thread at a time per context.
 *   - a context owns device scratch its calls reuse (the splat workspace; the path tracer's tile
 *     schedule: per-tile times of the last ptgs_trace_camera launch and the order built from them):
 *     calls of one context on different streams must be ordered by the caller (events), or use one
 *     context per stream (ptgs_splat_gaussians_views has its own per-view workspaces).
 */
#ifndef PTGS_H_
#define PTGS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTGS_ABI_VERSION 4  /* 3: ptgs_gaussians.ids, ptgs_splat_stats.fused, ptgs_splat_status spill fields;
                             * 4: PTGS_EBADIDS, PTGS_FLAG_SPLAT_OVERLAP */

/* ---------------- error codes ---------------- */
#define PTGS_OK 0
#define PTGS_EINVAL (-1)   /* bad argument / null pointer / size mismatch */
#define PTGS_EHIP (-2)     /* HIP runtime error (allocation, launch, copy) */
#define PTGS_ENOSCENE (-3) /* trace before ptgs_scene_upload */
#define PTGS_ERANGE (-4)   /* size exceeds an implementation limit */
#define PTGS_EIO (-5)      /* file could not be read/parsed (host helpers) */
#define PTGS_EINCOMPLETE (-6) /* an EARLIER stream-ordered splat frame of this context could not be completed
                               * (its spill pool was exhausted: some tiles were left at the background).
                               * Returned once, by the first splat call that starts after that frame has
                               * finished on the device; that call has grown the pool to 1.25x the largest
                               * pair count any frame of the workspace has had (which bounds the reported
                               * frame's spilled pairs) and
                               * rendered its own frame completely unless its own spilled tiles need more.
                               * ptgs_splat_gaussians_views renders every view before it returns the code.
                               * ptgs_splat_reserve prevents it (see there). */
#define PTGS_EBADIDS (-7) /* an EARLIER stream-ordered splat frame of this context met ptgs_gaussians.ids
                           * entries >= count (those Gaussians were dropped). Returned once, like
                           * PTGS_EINCOMPLETE, by a call that has rendered its own frame; a code of its
                           * own so a caller can tell it from this call's PTGS_EINVAL. */

/* ---------------- reference struct layouts (Appendix B of SURVEY.md) ---------------- */

/* Vertex, GeneralHeaders.h:65-97 / InputVertex raytracing.glsl:7-17 — 80 B */
typedef struct ptgs_vertex {
    float pos[3];
    float pad1;
    float normal[3];
    float pad2;
    float color[3];
    float pad3;
    float tangent[4];
    float tex_coord[2];
    float tex_coord_1[2];
} ptgs_vertex;

/* MaterialPushConstant, GeneralHeaders.h:236-269 / MaterialData raytracing.glsl:20-45 — 308 B.
 * use_specular_glossiness_workflow is a float on the host but read as an int by the shaders
 * (SURVEY Appendix A.2); the kernels reproduce that bit-pun. */
typedef struct ptgs_material {
    float base_color_factor[4];
    float uv_normal[16];
    float uv_emissive[16];
    float uv_albedo[16];
    float emissive_factor_and_pad[4];
    float metallic_factor;
    float roughness_factor;
    float occlusion_strength;
    float specular_factor;
    float specular_color_factor[3];
    float alpha_cutoff;
    float transmission_factor;
    float clearcoat_factor;
    float clearcoat_roughness_factor;
    float pad; /* 1.0 = is_transparent (BLEND), engine.cpp:1706 */
    int32_t albedo_texture_index;
    int32_t normal_texture_index;
    int32_t metallic_roughness_texture_index;
    int32_t emissive_texture_index;
    int32_t occlusion_texture_index;
    int32_t clearcoat_texture_index;
    int32_t clearcoat_roughness_texture_index;
    int32_t sg_id;
    float use_specular_glossiness_workflow;
} ptgs_material;

/* UniformBufferObject, GeneralHeaders.h:300-318 (std140) — 192 B */
typedef struct ptgs_ubo {
    float view[16]; /* column-major (glm) */
    float proj[16]; /* column-major, Vulkan ZO, [1][1] negated (camera.cpp:186-187) */
    float camera_pos[3];
    uint32_t frame_count;
    float ambient_light[4]; /* xyz = sky radiance / 2, w = emissive-NEE scale */
    float emissive_flux;
    float punctual_flux;
    float total_flux;
    float p_emissive;
    float fov; /* radians */
    float height;
    float use_lod;
    float lod_factor;
} ptgs_ubo;

/* PunctualLight, GeneralHeaders.h:287-297 — 64 B; type 0 point, 1 directional, 2 spot */
typedef struct ptgs_punctual_light {
    float position[3];
    float intensity;
    float color[3];
    float range;
    float direction[3];
    float outer_cone_cos;
    float inner_cone_cos;
    int32_t type;
    float padding[2];
} ptgs_punctual_light;

/* MeshInfo GeneralHeaders.h:515-520, LightTriangle :594-597, LightCDF :599-603,
 * PunctualLightCDF :605-609 — 16 B each */
typedef struct ptgs_mesh_info {
    uint32_t material_index;
    uint32_t vertex_offset;
    uint32_t index_offset;
    uint32_t _pad1;
} ptgs_mesh_info;

typedef struct ptgs_light_triangle {
    uint32_t v0, v1, v2;
    uint32_t material_index;
} ptgs_light_triangle;

typedef struct ptgs_light_cdf {
    float cumulative_probability;
    uint32_t triangle_index;
    float padding[2];
} ptgs_light_cdf;

typedef struct ptgs_punctual_cdf {
    float cumulative_probability;
    uint32_t light_index;
    float padding[2];
} ptgs_punctual_cdf;

/* HitDataGPU GeneralHeaders.h:565-576 / HitData rt_datacollect/raytracing.glsl:102-108 — 48 B */
typedef struct ptgs_hitdata {
    float pos[3];
    float flag;
    float color[4];
    float normal[3];
    float padding;
} ptgs_hitdata;

/* RaySample GeneralHeaders.h:522-524 — 8 B */
typedef struct ptgs_ray_sample {
    float uv[2];
} ptgs_ray_sample;

/* RayPushConstant / PC GeneralHeaders.h:526-540 — 80 B */
typedef struct ptgs_ray_push {
    float model[16];
    int32_t mode;
    float major_radius;
    float minor_radius;
    float height;
} ptgs_ray_push;

/* Layout contract: every size / offset of the structs above against Helpers/GeneralHeaders.h (glm's
 * vec3 is 12 B, vec4 16 B with no over-alignment on the host: GeneralHeaders.h:65-97 Vertex, :236-269
 * MaterialPushConstant, :287-297 PunctualLight, :300-318 UniformBufferObject, :515-540 MeshInfo /
 * RaySample / RayPushConstant / PC, :565-576 HitDataGPU, :594-609 LightTriangle / LightCDF /
 * PunctualLightCDF). Any translation unit that includes this header (the library's C++ sources, a C
 * caller, tests/native/abi_layout.c) fails to compile on a drift. */
#if defined(__cplusplus)
#define PTGS_LAYOUT_ASSERT(cond, msg) static_assert(cond, msg)
#else
#define PTGS_LAYOUT_ASSERT(cond, msg) _Static_assert(cond, msg)
#endif
#define PTGS_AT(T, f, off) PTGS_LAYOUT_ASSERT(offsetof(T, f) == (off), #T "." #f " at " #off)
PTGS_LAYOUT_ASSERT(sizeof(ptgs_vertex) == 80, "Vertex is 80 B");
PTGS_AT(ptgs_vertex, pos, 0);
PTGS_AT(ptgs_vertex, pad1, 12);
PTGS_AT(ptgs_vertex, normal, 16);
PTGS_AT(ptgs_vertex, pad2, 28);
PTGS_AT(ptgs_vertex, color, 32);
PTGS_AT(ptgs_vertex, pad3, 44);
PTGS_AT(ptgs_vertex, tangent, 48);
PTGS_AT(ptgs_vertex, tex_coord, 64);
PTGS_AT(ptgs_vertex, tex_coord_1, 72);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_material) == 308, "MaterialPushConstant is 308 B");
PTGS_AT(ptgs_material, base_color_factor, 0);
PTGS_AT(ptgs_material, uv_normal, 16);
PTGS_AT(ptgs_material, uv_emissive, 80);
PTGS_AT(ptgs_material, uv_albedo, 144);
PTGS_AT(ptgs_material, emissive_factor_and_pad, 208);
PTGS_AT(ptgs_material, metallic_factor, 224);
PTGS_AT(ptgs_material, roughness_factor, 228);
PTGS_AT(ptgs_material, occlusion_strength, 232);
PTGS_AT(ptgs_material, specular_factor, 236);
PTGS_AT(ptgs_material, specular_color_factor, 240);
PTGS_AT(ptgs_material, alpha_cutoff, 252);
PTGS_AT(ptgs_material, transmission_factor, 256);
PTGS_AT(ptgs_material, clearcoat_factor, 260);
PTGS_AT(ptgs_material, clearcoat_roughness_factor, 264);
PTGS_AT(ptgs_material, pad, 268);
PTGS_AT(ptgs_material, albedo_texture_index, 272);
PTGS_AT(ptgs_material, normal_texture_index, 276);
PTGS_AT(ptgs_material, metallic_roughness_texture_index, 280);
PTGS_AT(ptgs_material, emissive_texture_index, 284);
PTGS_AT(ptgs_material, occlusion_texture_index, 288);
PTGS_AT(ptgs_material, clearcoat_texture_index, 292);
PTGS_AT(ptgs_material, clearcoat_roughness_texture_index, 296);
PTGS_AT(ptgs_material, sg_id, 300);
PTGS_AT(ptgs_material, use_specular_glossiness_workflow, 304);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_ubo) == 192, "UniformBufferObject is 192 B");
PTGS_AT(ptgs_ubo, view, 0);
PTGS_AT(ptgs_ubo, proj, 64);
PTGS_AT(ptgs_ubo, camera_pos, 128);
PTGS_AT(ptgs_ubo, frame_count, 140);
PTGS_AT(ptgs_ubo, ambient_light, 144);
PTGS_AT(ptgs_ubo, emissive_flux, 160);
PTGS_AT(ptgs_ubo, punctual_flux, 164);
PTGS_AT(ptgs_ubo, total_flux, 168);
PTGS_AT(ptgs_ubo, p_emissive, 172);
PTGS_AT(ptgs_ubo, fov, 176);
PTGS_AT(ptgs_ubo, height, 180);
PTGS_AT(ptgs_ubo, use_lod, 184);
PTGS_AT(ptgs_ubo, lod_factor, 188);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_punctual_light) == 64, "PunctualLight is 64 B");
PTGS_AT(ptgs_punctual_light, position, 0);
PTGS_AT(ptgs_punctual_light, intensity, 12);
PTGS_AT(ptgs_punctual_light, color, 16);
PTGS_AT(ptgs_punctual_light, range, 28);
PTGS_AT(ptgs_punctual_light, direction, 32);
PTGS_AT(ptgs_punctual_light, outer_cone_cos, 44);
PTGS_AT(ptgs_punctual_light, inner_cone_cos, 48);
PTGS_AT(ptgs_punctual_light, type, 52);
PTGS_AT(ptgs_punctual_light, padding, 56);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_mesh_info) == 16, "MeshInfo is 16 B");
PTGS_AT(ptgs_mesh_info, material_index, 0);
PTGS_AT(ptgs_mesh_info, vertex_offset, 4);
PTGS_AT(ptgs_mesh_info, index_offset, 8);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_light_triangle) == 16, "LightTriangle is 16 B");
PTGS_AT(ptgs_light_triangle, material_index, 12);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_light_cdf) == 16, "LightCDF is 16 B");
PTGS_AT(ptgs_light_cdf, triangle_index, 4);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_punctual_cdf) == 16, "PunctualLightCDF is 16 B");
PTGS_AT(ptgs_punctual_cdf, light_index, 4);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_hitdata) == 48, "HitDataGPU is 48 B");
PTGS_AT(ptgs_hitdata, pos, 0);
PTGS_AT(ptgs_hitdata, flag, 12);
PTGS_AT(ptgs_hitdata, color, 16);
PTGS_AT(ptgs_hitdata, normal, 32);
PTGS_AT(ptgs_hitdata, padding, 44);
PTGS_LAYOUT_ASSERT(sizeof(ptgs_ray_sample) == 8, "RaySample is 8 B");
PTGS_LAYOUT_ASSERT(sizeof(ptgs_ray_push) == 80, "RayPushConstant / PC is 80 B");
PTGS_AT(ptgs_ray_push, model, 0);
PTGS_AT(ptgs_ray_push, mode, 64);
PTGS_AT(ptgs_ray_push, major_radius, 68);
PTGS_AT(ptgs_ray_push, minor_radius, 72);
PTGS_AT(ptgs_ray_push, height, 76);
#undef PTGS_AT

/* ---------------- scene ---------------- */

/* Host arrays in the reference layouts, as produced by Engine::createGlobalBindlessBuffers
 * (engine.cpp:1658-1860). mesh_index_count[i] is the index count of the primitive behind
 * meshes[i] (Primitive::index_count, used by buildBlas engine.cpp:545-560); the reference keeps
 * it in the BLAS geometry, so it travels beside MeshInfo here. Meshes with fewer than 3
 * indices are skipped exactly like buildBlas does.
 * The context copies everything; the caller keeps ownership. */
/* One texture of global_textures[] (binding 14, raytracing.glsl:138): RGBA8 level 0. The library
 * builds the mip chain as Image::generateMipmaps does (image.cpp:203-290: linear blits, each level
 * max(1, w/2) x max(1, h/2), floor(log2(max(w, h))) + 1 levels, image.cpp:35) and samples it as the
 * reference's sampler does (image.cpp:124-138: linear min/mag/mip filtering, repeat addressing,
 * LOD clamped to the chain). Formats follow Gameobject::scanTextureFormats (gameobject.cpp:284-345):
 * base colour, emissive, spec-gloss and diffuse are sRGB; normal, metal-rough, occlusion, clearcoat
 * and transmission UNORM. Material texture indices index this array (0 = the default white). */
typedef struct ptgs_texture {
    const uint8_t* rgba8; /* width * height * 4 bytes, row-major; row 0 holds v in [0, 1/height) */
    uint32_t width;
    uint32_t height;
    uint32_t srgb;        /* 1 = VK_FORMAT_R8G8B8A8_SRGB, 0 = VK_FORMAT_R8G8B8A8_UNORM */
    uint32_t reserved;
} ptgs_texture;

typedef struct ptgs_scene_desc {
    const ptgs_vertex* vertices;
    uint32_t num_vertices;
    const uint32_t* indices;
    uint32_t num_indices;
    const ptgs_mesh_info* meshes;
    const uint32_t* mesh_index_count;
    uint32_t num_meshes;
    const ptgs_material* materials;
    uint32_t num_materials;
    const ptgs_light_triangle* light_triangles;
    uint32_t num_light_triangles;
    const ptgs_light_cdf* light_cdf;
    uint32_t num_light_cdf;
    const ptgs_punctual_light* punctual_lights;
    uint32_t num_punctual_lights;
    const ptgs_punctual_cdf* punctual_cdf;
    uint32_t num_punctual_cdf;
    /* blue-noise texture (binding 12): RGBA32F, size x size texels, size a power of two,
     * values already decoded with the stbi_loadf convention (RGB^2.2, A linear). */
    const float* blue_noise_rgba32f;
    uint32_t blue_noise_size;
    /* textures (binding 14); may be empty: every texture index then samples as white */
    const ptgs_texture* textures;
    uint32_t num_textures;
} ptgs_scene_desc;

typedef struct ptgs_scene_info {
    uint32_t num_triangles;   /* triangles in the acceleration structure */
    uint32_t num_bvh_nodes;   /* interior nodes (each holds two child boxes) */
    uint32_t bvh_depth;       /* max depth of the tree */
    uint32_t max_leaf_size;
    double build_ms;          /* host BVH build time */
    uint64_t device_bytes;    /* bytes resident on the device for the scene */
} ptgs_scene_info;

/* ---------------- context ---------------- */

typedef struct ptgs_ctx ptgs_ctx;

int ptgs_create(int hip_device, ptgs_ctx** out);
void ptgs_destroy(ptgs_ctx* ctx);
const char* ptgs_last_error(const ptgs_ctx* ctx);
int ptgs_abi_version(void);
/* device the library was compiled for, e.g. "gfx950" */
const char* ptgs_device_arch(void);

/* Replaces buildBlas/initStaticTlas (engine.cpp:534-655, :1385-1520) + the descriptor uploads. */
int ptgs_scene_upload(ptgs_ctx* ctx, const ptgs_scene_desc* desc);
int ptgs_scene_get_info(const ptgs_ctx* ctx, ptgs_scene_info* out);
/* Debug / parity access to the uploaded acceleration structure (device pointers owned by the
 * context, valid until the next upload): 4-wide nodes (bvh.h layout, 128 B each) and the triangle
 * records in leaf order (48 B each: (v0, mesh) (v1 - v0, prim) (v2 - v0, gid)). */
typedef struct ptgs_bvh_buffers {
    const float* nodes;
    uint32_t num_nodes;
    const float* triangles;
    uint32_t num_triangles;
} ptgs_bvh_buffers;
int ptgs_scene_get_bvh(const ptgs_ctx* ctx, ptgs_bvh_buffers* out);

/* ---------------- path tracer (raygen_camera.rgen + closesthit/miss/shadow) ---------------- */

#define PTGS_ACCUM_RUNNING_MEAN 0u /* reference semantics: mix(prev, cur, 1/(frame+1)), restart at frame 0 */
#define PTGS_ACCUM_SUM 1u          /* accum.rgb += radiance, accum.a += 1 (for sample-sharded multi-GPU) */

/* Renders `spp` consecutive samples per pixel, frame counts ubo->frame_count .. +spp-1, into
 * accum (device, W*H RGBA32F, row-major, caller-owned, read-modify-write). One call with spp=1
 * is exactly one vkCmdTraceRaysKHR(W,H,1) of the reference (engine.cpp:1971).
 * `frame_stride` (>=1) spaces the frame counts: sample s uses frame_count + s*frame_stride —
 * the sample-index shard of §8e (rank g of G: frame_count=g, frame_stride=G, mode SUM). */
int ptgs_trace_camera(ptgs_ctx* ctx, const ptgs_ubo* ubo, uint32_t width, uint32_t height,
                      float* accum_rgba32f, uint32_t spp, uint32_t frame_stride, uint32_t accum_mode,
                      void* hip_stream);

/* Same, restricted to pixel rows [row_begin, row_end) — screen-space sharding of a frame. */
int ptgs_trace_camera_rows(ptgs_ctx* ctx, const ptgs_ubo* ubo, uint32_t width, uint32_t height,
                           uint32_t row_begin, uint32_t row_end, float* accum_rgba32f, uint32_t spp,
                           uint32_t frame_stride, uint32_t accum_mode, void* hip_stream);

/* Primary-hit depth for compositing (hybrid C4): per pixel the camera ray of
 * raygen_camera.rgen:25-41 through the pixel centre (no jitter), closest hit (any-hit seed from
 * ubo->frame_count), view-space depth -(view * hit).z; +inf where the ray misses. depth: device
 * float[W*H]. */
int ptgs_trace_depth(ptgs_ctx* ctx, const ptgs_ubo* ubo, uint32_t width, uint32_t height, float* depth,
                     void* hip_stream);
/* The same for pixel rows [row_begin, row_end) only (the tile-row shard of the hybrid frame: each rank
 * traces the depth of its own rows); the other rows of depth are left untouched. */
int ptgs_trace_depth_rows(ptgs_ctx* ctx, const ptgs_ubo* ubo, uint32_t width, uint32_t height, uint32_t row_begin,
                          uint32_t row_end, float* depth, void* hip_stream);

/* Toroidal data-collection tracer (shaders/rt_datacollect/raygen.rgen:31-141): one ray per
 * RaySample (device array, n entries), launch grid side x side with side = ceil(sqrt(n))
 * (engine.cpp:2786), HitData running mean written in place (device array, n entries). */
int ptgs_trace_torus(ptgs_ctx* ctx, const ptgs_ubo* ubo, const ptgs_ray_push* push,
                     const ptgs_ray_sample* samples, uint32_t n, ptgs_hitdata* hits,
                     void* hip_stream);

/* Ray counters of the most recent trace call(s) since the last reset (device-side atomics,
 * read back synchronously). */
typedef struct ptgs_trace_stats {
    uint64_t extension_rays; /* closest-hit traversals (primary + bounces) */
    uint64_t shadow_rays;    /* any-hit traversals (NEE visibility) */
    uint64_t samples;        /* pixel samples completed */
    uint64_t node_visits;    /* child-box tests (only with PTGS_FLAG_COUNT_TRAVERSAL) */
    uint64_t tri_tests;      /* ray-triangle tests (only with PTGS_FLAG_COUNT_TRAVERSAL) */
    uint64_t closest_hits;   /* extension rays that hit a surface (only with PTGS_FLAG_COUNT_TRAVERSAL) */
} ptgs_trace_stats;

#define PTGS_FLAG_COUNT_TRAVERSAL 1u /* instrumented kernels: node / triangle / hit counters */
#define PTGS_FLAG_TIME_STAGES 2u     /* hipEvent timing of the splat pipeline stages */
#define PTGS_FLAG_GPU_BVH 4u         /* ptgs_scene_upload builds the BVH on the GPU: the host builder's
                                      * binned SAH run on the device (the same tree: same node boxes and
                                      * leaf ranges, so the same traversal cost); falls back to the host
                                      * build for inputs it does not handle */
#define PTGS_FLAG_SPLAT_PUBLISH 8u   /* ptgs_splat_gaussians also writes the sorted keys / values of every
                                      * tile (ptgs_splat_get_buffers; parity tests): off in production,
                                      * the blend needs neither */
#define PTGS_FLAG_SPLAT_PUBLISH_TIGHT 64u /* with PTGS_FLAG_SPLAT_PUBLISH (tests): published frames bin each
                                      * Gaussian like the stream-ordered frames do — only to the tiles its
                                      * alpha >= 1/255 box overlaps, not its whole 3-sigma rectangle — so the
                                      * timed path's keys / values / ranges can be compared with the oracle's
                                      * tight mode (oracle_splat_gaussians_tight). Same image either way. */
#define PTGS_FLAG_PT_WAVEFRONT 16u  /* ptgs_trace_camera runs the wavefront path tracer (raygen / extend /
                                      * shade / shadow / accumulate stages over compacted ray queues)
                                      * instead of the one-kernel-per-frame path loop; same image, same
                                      * ray counts */
#define PTGS_FLAG_GPU_LBVH 32u       /* with PTGS_FLAG_GPU_BVH: a linear BVH (Morton order, Karras 2012)
                                      * instead: fastest rebuilds, slower traversal; host fallback when it
                                      * exceeds the traversal stack depth */
#define PTGS_FLAG_SPLAT_OVERLAP 128u /* frames in flight for the splat (the viewer's loop: a new camera per
                                      * call, Gaussians unchanged): the front end of a stream-ordered
                                      * ptgs_splat_gaussians / _over call (no stats, not published, not timed)
                                      * runs on a second stream of the context, concurrently with the blend
                                      * of the previous call, which still runs on hip_stream; the two calls
                                      * use a ring of three workspaces. The blend, i.e. everything written to
                                      * out_rgba32f, stays ordered on hip_stream exactly as without the flag.
                                      * Contract: a run of overlapped calls (the first call with the flag, or
                                      * the first after a splat call without it) starts after the work enqueued
                                      * on hip_stream before it; the front ends of the later calls of the run
                                      * wait only for the earlier frames of their workspaces (on the device),
                                      * so inputs (Gaussians, ids, chunk bounds) written on the stream during a
                                      * run must be followed by one call without this flag — like a Vulkan frame
                                      * in flight, whose resources the application does not touch. Same image,
                                      * keys and counts as without the flag. */
int ptgs_set_flags(ptgs_ctx* ctx, uint32_t flags);
int ptgs_stats_reset(ptgs_ctx* ctx, void* hip_stream);
int ptgs_stats_read(ptgs_ctx* ctx, ptgs_trace_stats* out); /* synchronises the context's device */

/* ---------------- rasterizers ---------------- */

/* Point-cloud view (shaders/pointcloud/pointcloud.vert:44-89 + .frag:1-11; pipeline state
 * pipeline.cpp:29-82): point i with hits[i].flag > 0 is projected by proj*view (mode 0: hit pos,
 * mode 1: torus(u,v) + 0.01 n through push->model), drawn as a 2-px point sprite with depth test
 * LESS against `depth` (device W*H f32, caller clears to 1.0), no blending, colour = linear
 * hits[i].color.rgb encoded to sRGB8 into rgba8 (device W*H u32, R in the low byte). */
int ptgs_splat_points(ptgs_ctx* ctx, const ptgs_ubo* ubo, const ptgs_ray_push* push,
                      const ptgs_hitdata* hits, const ptgs_ray_sample* samples, uint32_t n,
                      uint32_t width, uint32_t height, uint32_t* rgba8_srgb, float* depth,
                      void* hip_stream);

/* 3D Gaussian splatting forward (Kerbl et al. 2023; absent from the reference).
 * SoA device arrays, N Gaussians: means xyz, scales xyz (linear, post-activation),
 * rotations (w,x,y,z) un-normalised, opacities [0,1], colors linear RGB. */
typedef struct ptgs_gaussians {
    const float* means;     /* 3N */
    const float* scales;    /* 3N */
    const float* rotations; /* 4N */
    const float* opacities; /* N  */
    const float* colors;    /* 3N */
    uint32_t count;
    /* NULL, or ids[i] = the caller's index of Gaussian i (u32 N, device): a reordered copy (e.g. from
     * ptgs_gaussians_sort_spatial) then renders exactly like the original order (sorted values, the
     * depth tie rule and the per-Gaussian buffers use the ids). ids must be a permutation of [0, N):
     * a Gaussian whose id is >= N is dropped (never written out of bounds) and the next splat call
     * returns PTGS_EINVAL; duplicate ids are not detected (their keys collide: undefined order) */
    const uint32_t* ids;
    /* NULL, or per chunk of 256 consecutive Gaussians (ptgs_gaussians_chunk_bounds, 8 floats each): a
     * frame restricted to tile rows skips whole chunks whose conservative screen bound misses them,
     * before loading any of their Gaussians (the tile-row shard of several GPUs: each rank preprocesses
     * the chunks that reach its rows instead of all N). Outputs are unchanged. */
    const float* chunk_bounds;
} ptgs_gaussians;

typedef struct ptgs_splat_stats {
    uint32_t num_rendered; /* K = (gaussian, tile) pairs */
    uint32_t tiles_x, tiles_y;
    uint32_t num_visible;  /* gaussians with radius > 0 */
    uint32_t fused;        /* 1: the frame ran the single-launch front end (gs_bin_fused_kernel), 0: count +
                            * column scan + scatter */
} ptgs_splat_stats;

/* out_rgba32f (device W*H): rgb = sum c_i a_i T_i + T_final * bg, a = 1 - T_final.
 * Camera = ubo->view / ubo->proj (reference conventions). Tiles 16x16. Rows of tiles
 * [tile_row_begin, tile_row_end) are rendered (full frame: 0, ~0u) — screen-tile sharding of §8e;
 * pixels outside are left untouched.
 * Stream-ordered when stats == NULL: no host synchronisation, so a frame can be captured into and
 * replayed from a hipGraph. PTGS_OK means the frame is rendered completely, whatever the camera did
 * since the previous frame: the (Gaussian, tile) pair buffer of the context's workspace (three-launch
 * front end: 8 pairs per Gaussian or ptgs_splat_reserve's size, grown from the pair counts of earlier
 * frames) and the per-tile rows of the fused front end (sized from an earlier frame's largest tile)
 * are hints: a tile whose pairs did not fit them is gathered again and sorted by its own blend
 * workgroup on the device, in the same launch, through a spill pool (max(2^20, N) pairs, grown from
 * the demand of earlier frames) — same keys, same order, same image (ptgs_splat_status_read counts
 * these spilled tiles). Only a frame whose spilled tiles exceed the spill pool is incomplete: those
 * tiles are left at the background and the next call returns PTGS_EINCOMPLETE (see there);
 * ptgs_splat_reserve(K) rules it out for frames of at most K pairs. Growth frees buffers, which
 * waits for the device and invalidates graphs captured before it (reserve first).
 * stats != NULL: the call waits for the earlier frames and for this frame's pair count; a frame with
 * spilled tiles or above the pair buffer is re-run after growing the buffer (the exact published
 * layout), and stats is filled. */
int ptgs_splat_gaussians(ptgs_ctx* ctx, const ptgs_gaussians* g, const ptgs_ubo* ubo,
                         uint32_t width, uint32_t height, const float bg[3],
                         uint32_t tile_row_begin, uint32_t tile_row_end, float* out_rgba32f,
                         ptgs_splat_stats* stats, void* hip_stream);

/* Several views of the same Gaussians in one call (the capture loop renders views of one scene):
 * view v = ptgs_splat_gaussians(ctx, g, &ubos[v], width, height, bg, 0, ~0u, outs[v], NULL, ...),
 * identical output. Stream-ordered: the views start after the work already on hip_stream, run
 * concurrently on context-owned streams and workspaces (view 0 on hip_stream), and later work on
 * hip_stream waits for all of them. n_views in [1, PTGS_MAX_VIEWS]. Not a replacement of
 * ptgs_splat_gaussians in ptgs_splat_get_buffers: the buffers are view 0's. */
#define PTGS_MAX_VIEWS 8
int ptgs_splat_gaussians_views(ptgs_ctx* ctx, const ptgs_gaussians* g, uint32_t n_views, const ptgs_ubo* ubos,
                               uint32_t width, uint32_t height, const float bg[3], float* const* outs,
                               void* hip_stream);

/* Front end. Once a finished frame of the context's workspace has reported its largest tile, frames
 * run a single-launch front end: per-tile key rows of a fixed capacity (a power of two >= 1.25x that
 * tile, <= 2048 pairs) filled through per-tile atomic reservations, instead of the exact tile
 * segments of count + column scan + scatter (first frame, larger tiles, PTGS_GS_FRONTEND=three).
 * Both give the same keys, values, ranges and image. A tile above its row capacity is completed
 * through the spill pool (above), and the next frame sizes its rows from it.
 *
 * Spatial order: the fused front end reserves one run per (workgroup, touched tile); Gaussians whose
 * neighbours in memory are neighbours in space touch few tiles per workgroup. This writes a copy of
 * g in 3D Morton order of the means (10 bits per axis over the means' bounding box, ties by index)
 * to the caller's device buffers (sizes as g's) and ids[i] = the original index of copy i (g->ids
 * composed when set): render the copy with .ids = ids for output identical to g's. Scene preparation
 * (like ptgs_scene_upload's BVH build): synchronises; device temporaries are freed. */
int ptgs_gaussians_sort_spatial(ptgs_ctx* ctx, const ptgs_gaussians* g, float* means, float* scales, float* rotations,
                                float* opacities, float* colors, uint32_t* ids, void* hip_stream);

/* Bounds of every chunk of 256 consecutive Gaussians of g (device float[8 * ceil(count / 256)]): the
 * box of its means (min x, y, z, then max x, y, z at [4..6]) and its largest scale ([3]); [7] = 0. For
 * ptgs_gaussians.chunk_bounds; useful when chunks are spatially compact (ptgs_gaussians_sort_spatial's
 * order). Recompute after the Gaussians change. Stream-ordered. */
int ptgs_gaussians_chunk_bounds(ptgs_ctx* ctx, const ptgs_gaussians* g, float* bounds, void* hip_stream);

/* Report of the stream-ordered splat (no stats): waits for hip_stream and the context's view streams,
 * then returns (and clears) the counts since the last query. frames / views[v]: frames left
 * incomplete (spill pool exhausted, see PTGS_EINCOMPLETE; each was also reported by a later call)
 * per view slot v (slot 0 counts ptgs_splat_gaussians / _over and view 0 of
 * ptgs_splat_gaussians_views); frames = their sum. spilled_tiles: tiles completed through the spill
 * pool (rendered; a measure of how far the camera outran the buffers sized from earlier frames);
 * incomplete_tiles: tiles left at the background. pair_capacity: the smallest pair capacity over the
 * slots in use; last_pairs: the largest pair count any slot's latest frame produced; spill_capacity /
 * spill_demand: slot 0's pool and the largest demand of one of its frames so far. */
typedef struct ptgs_splat_status {
    uint64_t frames;
    uint32_t views[PTGS_MAX_VIEWS];
    uint32_t pair_capacity;
    uint32_t last_pairs;
    uint32_t touched_runs;  /* slot 0's latest frame: (front-end workgroup, tile) runs, i.e. per-tile
                             * reservations of the fused front end / nonzero histogram entries of the
                             * count: the spatial coherence of the Gaussians' order */
    uint32_t fused;         /* slot 0's latest frame ran the fused front end */
    uint64_t spilled_tiles;
    uint64_t incomplete_tiles;
    uint32_t spill_capacity;
    uint32_t spill_demand;
} ptgs_splat_status;
int ptgs_splat_status_read(ptgs_ctx* ctx, ptgs_splat_status* out, void* hip_stream);

/* Grow the pair buffers and spill pools of every view slot to at least `pairs` (Gaussian, tile) pairs:
 * stream-ordered frames of up to that many pairs then store every pair (three-launch front end) or
 * complete every spilled tile (fused rows: a frame's spilled tiles hold at most its pair count), so
 * they are never incomplete — including hipGraph replays, whose row capacity is fixed at capture
 * (e.g. before capturing, or from a previous frame's stats.num_rendered plus headroom).
 * Synchronises the device when it grows. */
int ptgs_splat_reserve(ptgs_ctx* ctx, uint32_t pairs);

/* Hybrid composite (C4): the same splat, front to back over an image: a pixel stops at the first
 * Gaussian whose view depth is >= depth[pixel] (the mesh occludes it and everything behind), and
 * out = C + T * under (all four channels, C.a = 1 - T). depth: device float[W*H] (e.g. from
 * ptgs_trace_depth); under: device RGBA32F[W*H] (e.g. the ptgs_trace_camera accumulator); out may
 * alias under. Integer outputs (keys, values, ranges) are those of ptgs_splat_gaussians. */
int ptgs_splat_gaussians_over(ptgs_ctx* ctx, const ptgs_gaussians* g, const ptgs_ubo* ubo, uint32_t width,
                              uint32_t height, const float* depth, const float* under_rgba32f,
                              uint32_t tile_row_begin, uint32_t tile_row_end, float* out_rgba32f,
                              ptgs_splat_stats* stats, void* hip_stream);

/* 3DGS initialisation from a point cloud (Kerbl et al. 2023 create_from_pcd; the point cloud is the
 * reference's points3d.ply, Engine::savePly engine.cpp:2849-2895, read with ptgs_read_ply).
 * ptgs_knn3_mean_dist2: dist2[i] = mean of the 3 smallest squared distances from point i to the
 * other points, exact in f32 ((dx*dx + dy*dy) + dz*dz, no FMA; ((b0 + b1) + b2) / 3); fewer than 3
 * other points: mean of those, none: 0. ptgs_gaussians_from_points writes post-activation
 * parameters (ptgs_gaussians layout): means = xyz, scales = sqrt(max(dist2, 1e-7)) x3, rotations =
 * (1, 0, 0, 0), opacities = 0.1, colors = rgb / 255 (rgb: device uchar[3N] or NULL = black).
 * All buffers are device pointers; both calls synchronise the stream (temporaries are freed). */
int ptgs_knn3_mean_dist2(ptgs_ctx* ctx, const float* xyz, uint32_t n, float* dist2, void* hip_stream);
int ptgs_gaussians_from_points(ptgs_ctx* ctx, const float* xyz, const uint8_t* rgb, uint32_t n, float* means,
                               float* scales, float* rotations, float* opacities, float* colors, void* hip_stream);

/* Debug/parity access to the integer intermediates of the most recent ptgs_splat_gaussians call
 * (device buffers owned by the context, valid until the next splat call):
 * radii[N] (int32), tiles_touched[N] (u32), sorted keys[K] (u64: tile<<32 | depth bits),
 * sorted values[K] (u32 gaussian index), tile ranges[tiles] (uint2 start,end). sorted_keys /
 * sorted_values are NULL unless that call ran with PTGS_FLAG_SPLAT_PUBLISH and stats. */
/* radii / tiles_touched / means2d / depths / conic_opacity are written only by frames rendered with
 * PTGS_FLAG_SPLAT_PUBLISH (indexed by the caller's Gaussian index, see ptgs_gaussians.ids); tile_ranges
 * by every frame (unpublished fused frames: end - begin = the tile's pair count, begin = t * capacity). */
typedef struct ptgs_splat_buffers {
    const int32_t* radii;
    const uint32_t* tiles_touched;
    const uint64_t* sorted_keys;
    const uint32_t* sorted_values;
    const uint32_t* tile_ranges;
    const float* means2d;   /* 2N */
    const float* depths;    /* N */
    const float* conic_opacity; /* 4N */
    uint32_t num_gaussians;
    uint32_t num_rendered;
    uint32_t num_tiles;
} ptgs_splat_buffers;
int ptgs_splat_get_buffers(const ptgs_ctx* ctx, ptgs_splat_buffers* out);
/* Debug/parity access to the most recent splat call's own pair rows when its front end was the fused
 * one (every frame, published or not, timed or overlapped: the bench's frames): tile t's pairs are
 * rows[t * row_capacity .. t * row_capacity + n_t), n_t = end - begin of tile_ranges[t] (the blend
 * writes those ranges), each pair (depth bits << 32) | gaussian index, in no particular order (the blend
 * sorts them in LDS; a tile's row may be left permuted). A tile with n_t > row_capacity kept its first
 * row_capacity pairs only (completed through the spill pool). *rows = NULL, *row_capacity = 0 when that
 * frame ran the three-launch front end. Device memory owned by the context, valid until the next splat
 * call; synchronise the call's stream before reading. No reference counterpart (test access). */
int ptgs_splat_get_tile_rows(const ptgs_ctx* ctx, const uint64_t** rows, uint32_t* row_capacity);

/* With PTGS_FLAG_TIME_STAGES: milliseconds of the stages of the most recent ptgs_splat_gaussians
 * call, measured with hipEvents on its stream: [0] preprocess + count (tile histograms) [1] column
 * scan (tile totals) [2] scatter (pairs into tile segments, K) [3] radix sort of the tiles above 512 pairs
 * [4] 0 [5] sort (tiles up to 512 pairs) + blend. Synchronises. */
int ptgs_splat_stage_ms(ptgs_ctx* ctx, float out_ms[6]);

/* ---------------- dataset capture (Engine::captureSceneData, engine.cpp:2658-2814) -------- */
typedef struct ptgs_capture_desc {
    const char* out_dir;            /* writes out_dir/train/r_<i>.jpg, transforms_{train,test}.json, points3d.ply */
    uint32_t width, height;         /* render size (the reference's swapchain extent) */
    uint32_t total_positions;       /* camera views (settings "total_positions", default 336) */
    uint32_t accumulation_steps;    /* samples per view and torus frames (settings default 512) */
    float min_beta, max_beta;       /* torus elevation range, degrees (defaults -45, 45) */
    float fov_deg;                  /* camera fov (60) */
    float major_radius, torus_height; /* Camera::updateToroidalAngles radius / height */
    float image_divisor;            /* > 1: every 2nd pixel is kept (engine.cpp:2737-2754) */
    uint32_t seed;                  /* mt19937 seed (13) */
    uint32_t capture_images, capture_pointcloud;
    const ptgs_ubo* ubo;            /* template: ambient light, fluxes, lod settings (view/proj/frame set per view) */
    ptgs_ray_push torus;            /* torus push constants for the point cloud */
    const ptgs_ray_sample* samples; /* device array (Morton-sorted RaySamples), num_samples entries */
    uint32_t num_samples;
    void* hip_stream;
} ptgs_capture_desc;

/* Synchronous: traces every view (one batched ptgs_trace_camera call of accumulation_steps samples per
 * view), encodes/reads back/downsamples/writes JPEG quality 90, accumulates the torus point cloud,
 * writes the PLY and the two transforms files. Requires an uploaded scene. */
int ptgs_capture_dataset(ptgs_ctx* ctx, const ptgs_capture_desc* desc);

/* ---------------- multi-GPU frame reduce over RCCL / xGMI ---------------- */
/* The path tracer shards samples across GPUs (ptgs_trace_camera with PTGS_ACCUM_SUM and
 * frame_stride = number of GPUs) and sums the RGBA32F buffers; tile-row shards of the splat are
 * disjoint and combine with the same sum. One RCCL communicator per context: one rank calls
 * ptgs_comm_unique_id, the caller ships the 128 bytes to every rank (any channel), each rank calls
 * ptgs_comm_create with its rank. RCCL is loaded at run time; without it these return PTGS_EHIP. */
#define PTGS_COMM_ID_BYTES 128
int ptgs_comm_unique_id(uint8_t id[PTGS_COMM_ID_BYTES]);
int ptgs_comm_create(ptgs_ctx* ctx, const uint8_t id[PTGS_COMM_ID_BYTES], int nranks, int rank);
int ptgs_comm_destroy(ptgs_ctx* ctx);
/* In-place SUM of n_floats device floats: to `root` (ncclReduce) or to every rank (ncclAllReduce).
 * Stream-ordered on hip_stream. */
int ptgs_reduce_radiance(ptgs_ctx* ctx, float* accum, size_t n_floats, int root, void* hip_stream);
int ptgs_allreduce_radiance(ptgs_ctx* ctx, float* accum, size_t n_floats, void* hip_stream);
/* Tile-row shards of the splat: rank g's pixel rows [row_ranges[2 g], row_ranges[2 g + 1]) of its
 * RGBA32F width x height image are copied into the same rows of root's image (ncclSend / ncclRecv in
 * one group: each rank moves only its own rows, W*H*16/G bytes, instead of a full-frame reduce).
 * row_ranges holds every rank's range (2 x nranks, identical on all ranks). Stream-ordered. */
int ptgs_gather_rows(ptgs_ctx* ctx, float* image, uint32_t width, uint32_t height, const uint32_t* row_ranges,
                     int root, void* hip_stream);
/* Reduce-scatter by rows (the C5 hybrid's radiance): afterwards rank g's rows [row_ranges[2 g],
 * row_ranges[2 g + 1]) of its RGBA32F image hold the SUM over all ranks of those rows (other rows
 * unspecified); one ncclReduce per rank's rows (root = that rank) in one group: about one frame sent
 * per rank instead of an all-reduce's two. row_ranges as ptgs_gather_rows. Stream-ordered. */
int ptgs_reduce_scatter_rows(ptgs_ctx* ctx, float* image, uint32_t width, uint32_t height, const uint32_t* row_ranges,
                             void* hip_stream);

/* ---------------- output encode (blit rgba32f -> B8G8R8A8_SRGB, engine.cpp:2004-2020) --------- */
/* rgba8 (device W*H u32, R in the low byte): linear -> sRGB8 of clamp(rgb,0,1), alpha 255. */
int ptgs_encode_srgb8(ptgs_ctx* ctx, const float* rgba32f, uint32_t width, uint32_t height,
                      uint32_t* rgba8, void* hip_stream);

/* ---------------- device memory helpers (usable without any other GPU framework) ------------ */
int ptgs_device_alloc(ptgs_ctx* ctx, size_t bytes, void** out);
int ptgs_device_free(ptgs_ctx* ctx, void* ptr);
int ptgs_memcpy_h2d(ptgs_ctx* ctx, void* dst, const void* src, size_t bytes);
int ptgs_memcpy_d2h(ptgs_ctx* ctx, void* dst, const void* src, size_t bytes);
int ptgs_memset_d32(ptgs_ctx* ctx, void* dst, uint32_t value, size_t count, void* hip_stream);
int ptgs_synchronize(ptgs_ctx* ctx);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PTGS_H_ */
