// The scene builder's object store (internal): one entry per Gameobject, aggregated by
// ptgs_builder_finalize the way Engine::createGlobalBindlessBuffers does (engine.cpp:1658-1860).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs_host.h"

struct ptgs_scene_builder {
  struct Texture {  // one entry of Gameobject::textures (RGBA8, level 0)
    std::vector<uint8_t> rgba;
    uint32_t w = 1, h = 1;
    uint32_t srgb = 1;
  };
  struct Object {
    std::vector<ptgs_vertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<ptgs_primitive> prims;
    std::vector<ptgs_material> materials;  // texture ids object-relative, pad = is_transparent
    std::vector<ptgs_punctual_light> lights;
    struct ETri { uint32_t i0, i1, i2, mat; float area; };
    std::vector<ETri> etris;
    uint32_t num_textures = 1;
    std::vector<Texture> textures;  // empty = no pixel data supplied (add_object)
  };
  std::vector<Object> objects;
  std::vector<ptgs_punctual_light> global_lights;  // the scene "sun" (engine.cpp:1225-1242), unfiltered
  bool has_rtbox = false;
  Object rtbox;
  std::string err;
  // finalized arrays
  std::vector<ptgs_vertex> v;
  std::vector<uint32_t> idx;
  std::vector<ptgs_mesh_info> meshes;
  std::vector<uint32_t> mesh_count;
  std::vector<ptgs_material> mats;
  std::vector<ptgs_light_triangle> ltris;
  std::vector<ptgs_light_cdf> lcdf;
  std::vector<ptgs_punctual_light> plights;
  std::vector<ptgs_punctual_cdf> pcdf;
  std::vector<ptgs_texture> tex;
};

// Material{} defaults (GeneralHeaders.h:202-235) in the MaterialPushConstant layout
ptgs_material ptgs_default_material();
