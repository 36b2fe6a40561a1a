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

#ifdef __cplusplus
}
#endif

#endif /* PTGS_HOST_H_ */
