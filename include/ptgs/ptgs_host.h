/*
 * ptgs_host.h — host-side mirror of the reference Engine's scene/camera API (C-ABI).
 *
 * These functions produce exactly the inputs the reference's hot path consumes, so a caller can
 * go from the reference's scene description to ptgs_scene_upload()/ptgs_trace_camera():
 *   camera  : Camera::updateToroidalAngles / freeCameraUpdate   Vulkan_Engine/camera.cpp:93-95, :195-228
 *   rt-box  : Engine::createRTBox                               Vulkan_Engine/engine.cpp:181-335
 *   objects : Gameobject emissive-triangle extraction           Vulkan_Engine/gameobject.cpp:567, :777-790
 *   flatten : Engine::createGlobalBindlessBuffers               Vulkan_Engine/engine.cpp:1658-1860
 *   export  : Engine::saveTransformsJson / savePly              Vulkan_Engine/engine.cpp:2816-2895
 *   ingest  : Gameobject::loadModel (glTF) / Engine::loadScene   gameobject.cpp:198-851, engine.cpp:1172-1352
 * Pure host code (no GPU needed).
 */
#ifndef PTGS_HOST_H_
#define PTGS_HOST_H_

#include "ptgs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* glm::radians + Camera::updateToroidalAngles (camera.cpp:195-228) followed by
 * glm::perspective(ZO) with [1][1] *= -1. position may be NULL. */
int ptgs_camera_toroidal(float alpha_deg, float beta_deg, float radius, float height, float fov_deg,
                         float aspect, float near_plane, float far_plane, float view[16], float proj[16],
                         float position[3]);
/* glm::lookAt (RH) */
int ptgs_camera_lookat(const float eye[3], const float center[3], const float up[3], float view[16]);
/* glm::perspective RH_ZO with [1][1] negated (camera.cpp:94-95) */
int ptgs_camera_perspective(float fovy_rad, float aspect, float near_plane, float far_plane, float proj[16]);
/* column-major 4x4 inverse (double internally, rounded once) */
int ptgs_mat4_inverse(const float m[16], float out[16]);
/* glm::inverse(mat4) in float, GLM 0.9.9 compute_inverse restated operation for operation (what the
 * reference writes into transforms.json, engine.cpp:2760) */
int ptgs_mat4_inverse_glm(const float m[16], float out[16]);

/* ----- capture writers (engine.cpp:2672-2681, :2816-2895; GeneralHeaders.cpp:178-190) ----- */
/* n (alpha, beta) pairs in degrees from std::mt19937(seed) + uniform_real_distribution<double>:
 * alpha U(0, 360) then beta U(min_beta, max_beta), each rounded to float */
int ptgs_capture_poses(uint32_t n, uint32_t seed, float min_beta, float max_beta, float* alpha_beta);
/* nlohmann::json dump(4) layout: camera_angle_x = 2 atan(tan(fov_y / 2) aspect), frames with file_path
 * and transform_matrix rows (transforms: n column-major 4x4) */
int ptgs_write_transforms_json(const char* path, float fov_y_deg, float aspect, uint32_t n,
                               const char* const* file_paths, const float* transforms);
/* ASCII PLY of the points with flag > 0 (Engine::savePly); num_written may be NULL */
int ptgs_write_ply(const char* path, const ptgs_hitdata* hits, uint32_t n, uint32_t* num_written);
/* baseline JFIF; comp 1/3/4 (alpha ignored); quality 1..100 (the reference uses 90) */
int ptgs_write_jpeg(const char* path, const uint8_t* pixels, uint32_t width, uint32_t height, uint32_t comp,
                    int quality);

/* ----- scene builder ----- */
typedef struct ptgs_scene_builder ptgs_scene_builder;

/* Primitive, GeneralHeaders.h:271-277 */
typedef struct ptgs_primitive {
    uint32_t first_index;
    uint32_t index_count;
    int32_t material_index;
} ptgs_primitive;

int ptgs_builder_create(ptgs_scene_builder** out);
void ptgs_builder_destroy(ptgs_scene_builder* b);
/* rt-box from the reference's JSON format (e.g. showcase/subjects/bunny_box.json) */
int ptgs_builder_add_rtbox_json(ptgs_scene_builder* b, const char* path);
/* One Gameobject with world-space (baked) vertices. Material texture indices are relative to the
 * object (0 = the object's default texture); punctual lights with intensity <= 0 are dropped
 * (engine.cpp:1744-1750). num_textures advances the global texture offset (engine.cpp:1752). */
int ptgs_builder_add_object(ptgs_scene_builder* b, const ptgs_vertex* vertices, uint32_t num_vertices,
                            const uint32_t* indices, uint32_t num_indices, const ptgs_primitive* prims,
                            uint32_t num_prims, const ptgs_material* materials, uint32_t num_materials,
                            const ptgs_punctual_light* lights, uint32_t num_lights, uint32_t num_textures);
/* createGlobalBindlessBuffers: objects in insertion order, then the rt-box. Fills `desc` with
 * pointers into builder-owned arrays (valid until the builder is destroyed or modified; the
 * blue-noise fields are left NULL/0) and the light fields of `ubo` (emissive_flux, punctual_flux,
 * total_flux, p_emissive). */
int ptgs_builder_finalize(ptgs_scene_builder* b, ptgs_scene_desc* desc, ptgs_ubo* ubo);
const char* ptgs_builder_last_error(const ptgs_scene_builder* b);

/* ----- scene ingest (§8f #3) ----- */
/* Decode a PNG / JPEG image held in memory to RGBA8 with the semantics of
 * stbi_load(..., STBI_rgb_alpha) (Image::createTextureImage, Vulkan_Engine/image.cpp:12).
 * rgba = NULL queries width / height / comp (channels in the file) only; PTGS_ERANGE when
 * capacity < width * height * 4; PTGS_EIO on malformed or unsupported data. */
int ptgs_image_decode_rgba8(const void* bytes, size_t size, uint8_t* rgba, size_t capacity, uint32_t* width,
                            uint32_t* height, uint32_t* comp);

/* substitute a 1x1 white texture for an image file that is missing or undecodable (the reference
 * throws "failed to load texture image", image.cpp:19-21) */
#define PTGS_INGEST_MISSING_IMAGES_WHITE 1u

/* One glTF 2.0 model (.gltf with external or data: buffers, or .glb) as one Gameobject
 * (Gameobject::loadModel, gameobject.cpp:198-851): frame-0 node transforms and CPU skinning,
 * KHR_lights_punctual, materials incl. KHR_materials_{pbrSpecularGlossiness, emissive_strength,
 * specular, transmission, clearcoat} and KHR_texture_transform, every image decoded (sRGB unless
 * only used as a linear map), vertex dedup and the duplicated index copy of the reference.
 * Then the scene-JSON placement is baked in (engine.cpp:1271-1331): translate(position) *
 * quat(radians(rotation_deg)) * scale(scale); NULL = 0 / 0 / 1. Returns PTGS_EIO with
 * ptgs_builder_last_error() set on any load failure. */
int ptgs_builder_add_gltf(ptgs_scene_builder* b, const char* path, const float position[3],
                          const float rotation_deg[3], const float scale[3], uint32_t flags);
/* A scene-level light placed before every object light and never filtered (the settings "sun",
 * engine.cpp:1225-1242). */
int ptgs_builder_add_punctual_light(ptgs_scene_builder* b, const ptgs_punctual_light* light);

/* Vertex element of a PLY point cloud: the ASCII file Engine::savePly writes (engine.cpp:2849-2895,
 * x y z nx ny nz red green blue) or binary little / big endian. x y z required; normals default 0;
 * colours from red green blue (uchar, or float in [0,1]) or, failing those, the SH DC term
 * f_dc_0..2 of a trained 3DGS file, else 0. Pass xyz = normals = rgb = NULL to get the count;
 * PTGS_ERANGE when capacity < count. Any output pointer may be NULL. */
int ptgs_read_ply(const char* path, float* xyz, float* normals, uint8_t* rgb, uint32_t capacity, uint32_t* count);

/* ----- torus RaySample generators (Vulkan_Engine/sampling.cpp:5-434, Sampling::updateSampling) ----- */
/* method = index into the reference's sampling_methods array (GeneralHeaders.h:552-560, the Engine's
 * current_sampling) */
#define PTGS_SAMPLING_RANDOM 0
#define PTGS_SAMPLING_UNIFORM 1
#define PTGS_SAMPLING_STRATIFIED 2
#define PTGS_SAMPLING_LHS 3
#define PTGS_SAMPLING_HALTON 4
#define PTGS_SAMPLING_IMP_COL 5 /* colour-gradient importance over the previous HitData */
#define PTGS_SAMPLING_IMP_HIT 6 /* hit-ratio importance over the previous HitData */
/* n RaySamples in the order the reference uploads them (Morton-sorted, sampling.cpp:356-361).
 * Random / Stratified / LHS / importance draw from std::mt19937(seed) (the reference: seed 13,
 * sampling.cpp:3). The importance methods bin the previous samples (prev_samples, n_prev) with their
 * read-back hits (prev_hits, n_prev_hits; binning stops at the shorter) on a grid_resolution² grid
 * (0 = the reference's 256); with n_prev == 0 they fall back to Halton (sampling.cpp:389-392).
 * out may alias prev_samples (the reference regenerates its sample vector in place). */
int ptgs_generate_samples(int method, uint32_t n, const ptgs_ray_sample* prev_samples, uint32_t n_prev,
                          const ptgs_hitdata* prev_hits, uint32_t n_prev_hits, uint32_t seed, int grid_resolution,
                          ptgs_ray_sample* out);
/* Sampling::sortSamples: std::sort by the 15-bit-per-axis Morton code (not stable; libstdc++ order) */
int ptgs_sort_samples(ptgs_ray_sample* samples, uint32_t n);
/* morton2D (sampling.cpp:346-354) */
uint32_t ptgs_morton2d(float u, float v);

/* Engine::loadScene settings (engine.cpp:1190-1255) with the Engine defaults for absent keys */
typedef struct ptgs_scene_settings {
    float ambient_light[4];      /* default (0, 0, 0, 1) */
    int32_t use_rt_box;
    int32_t render_torus;        /* default 1 */
    int32_t render_pointcloud;   /* default 1 */
    float torus_major_radius;    /* 16 */
    float torus_minor_radius;    /* 1 */
    float torus_height;          /* 8 */
    int32_t torus_major_segments;
    int32_t torus_minor_segments;
    uint32_t num_rays;           /* 1000000 */
    float use_lod;               /* 0 */
    float lod_factor;            /* 1 */
    uint32_t accumulation_steps; /* 512 */
    uint32_t total_positions;    /* 336 */
    float min_beta;              /* -45 */
    float max_beta;              /* 45 */
    float image_divisor;         /* 2 */
    int32_t capture_images;      /* 1 */
    int32_t capture_pointcloud;  /* 1 */
    uint32_t num_objects;        /* models loaded */
} ptgs_scene_settings;

/* Engine::loadScene (engine.cpp:1172-1352): `path` is either the scene JSON itself or a file whose
 * "scene" key names it (main_scene.json). Model / rt-box paths in the JSON are resolved against
 * root_dir (the reference resolves them against its working directory; NULL = as given). Objects are
 * appended in order, then the rt-box when settings.use_rt_box; the "sun" replaces the builder's
 * scene-level lights. settings may be NULL. */
int ptgs_builder_load_scene_json(ptgs_scene_builder* b, const char* path, const char* root_dir, uint32_t flags,
                                 ptgs_scene_settings* settings);

#ifdef __cplusplus
}
#endif

#endif /* PTGS_HOST_H_ */
