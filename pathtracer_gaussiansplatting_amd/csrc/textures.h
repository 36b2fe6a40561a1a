// textures.h — host side of global_textures[]: mip chains and the device texel pool (texture.h).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ptgs/ptgs.h"

namespace ptgs {

#define PTGS_TEX_INFO 20        // words per texture in the info table
#define PTGS_TEX_MAX_LEVELS 16  // 32768 texels -> 16 levels

struct TexturePool {
  std::vector<uint32_t> texels;  // all levels of all textures, RGBA8 packed r | g<<8 | b<<16 | a<<24
  std::vector<uint32_t> info;    // PTGS_TEX_INFO words per texture: w0, h0, levels, srgb, level offsets
  std::vector<float> lut;        // 512: UNORM c/255, then sRGB -> linear
};

// Builds the pool; returns false (with a message) on a bad texture description.
bool build_texture_pool(const ptgs_texture* tex, uint32_t count, TexturePool& out, std::string& err);

}  // namespace ptgs
