// textures.cpp — mip chains for global_textures[], restating Image::createTextureImage /
// generateMipmaps (Vulkan_Engine/image.cpp:35, :203-290): floor(log2(max(w, h))) + 1 levels; level
// i is a vkCmdBlitImage of level i-1 with VK_FILTER_LINEAR onto max(1, w/2) x max(1, h/2). A linear
// blit samples the source at the destination texel centre mapped into the source extent, bilinear
// with clamp-to-edge, in linear space for sRGB formats (decode, filter, encode + round to 8 bits).
// oracle/ptgs_oracle.c (or_build_mips) restates the same arithmetic.
#include "textures.h"

#include <cmath>
#include <cstring>


namespace ptgs {

static float srgb_to_linear(float c) {
  return c <= 0.04045f ? c / 12.92f : std::pow((c + 0.055f) / 1.055f, 2.4f);
}

static float linear_to_srgb(float c) {
  return c <= 0.0031308f ? c * 12.92f : 1.055f * std::pow(c, 1.0f / 2.4f) - 0.055f;
}

static uint32_t to_u8(float c) {
  float v = std::floor(c * 255.0f + 0.5f);
  if (!(v > 0.0f)) return 0u;
  if (v > 255.0f) return 255u;
  return (uint32_t)v;
}

bool build_texture_pool(const ptgs_texture* tex, uint32_t count, TexturePool& out, std::string& err) {
  out.texels.clear();
  out.info.assign((size_t)count * PTGS_TEX_INFO, 0u);
  out.lut.resize(512);
  for (int i = 0; i < 256; ++i) {
    out.lut[i] = (float)i / 255.0f;
    out.lut[256 + i] = srgb_to_linear((float)i / 255.0f);
  }
  for (uint32_t t = 0; t < count; ++t) {
    const ptgs_texture& T = tex[t];
    if (!T.rgba8 || T.width == 0 || T.height == 0 || T.width > 32768 || T.height > 32768) {
      err = "texture " + std::to_string(t) + ": null data or size 0 / > 32768";
      return false;
    }
    uint32_t big = T.width > T.height ? T.width : T.height;
    uint32_t levels = 1;
    while ((big >> levels) > 0u) ++levels;  // floor(log2(max)) + 1
    if (levels > PTGS_TEX_MAX_LEVELS) levels = PTGS_TEX_MAX_LEVELS;
    uint32_t* info = &out.info[(size_t)t * PTGS_TEX_INFO];
    info[0] = T.width;
    info[1] = T.height;
    info[2] = levels;
    info[3] = T.srgb ? 1u : 0u;
    const float* dec = out.lut.data() + (T.srgb ? 256 : 0);
    // level 0
    size_t base = out.texels.size();
    info[4] = (uint32_t)base;
    out.texels.resize(base + (size_t)T.width * T.height);
    std::memcpy(out.texels.data() + base, T.rgba8, (size_t)T.width * T.height * 4);
    uint32_t sw = T.width, sh = T.height;
    for (uint32_t l = 1; l < levels; ++l) {
      const uint32_t dw = sw > 1 ? sw / 2 : 1, dh = sh > 1 ? sh / 2 : 1;
      const size_t src = info[4 + l - 1], dst = out.texels.size();
      info[4 + l] = (uint32_t)dst;
      out.texels.resize(dst + (size_t)dw * dh);
      const float sx = (float)sw / (float)dw, sy = (float)sh / (float)dh;
      for (uint32_t y = 0; y < dh; ++y) {
        const float fy = ((float)y + 0.5f) * sy - 0.5f;
        const float fy0 = std::floor(fy), b = fy - fy0;
        const int iy = (int)fy0;
        const uint32_t y0 = (uint32_t)(iy < 0 ? 0 : (iy >= (int)sh ? (int)sh - 1 : iy));
        const uint32_t y1 = (uint32_t)(iy + 1 < 0 ? 0 : (iy + 1 >= (int)sh ? (int)sh - 1 : iy + 1));
        for (uint32_t x = 0; x < dw; ++x) {
          const float fx = ((float)x + 0.5f) * sx - 0.5f;
          const float fx0 = std::floor(fx), a = fx - fx0;
          const int ix = (int)fx0;
          const uint32_t x0 = (uint32_t)(ix < 0 ? 0 : (ix >= (int)sw ? (int)sw - 1 : ix));
          const uint32_t x1 = (uint32_t)(ix + 1 < 0 ? 0 : (ix + 1 >= (int)sw ? (int)sw - 1 : ix + 1));
          const uint32_t p00 = out.texels[src + (size_t)y0 * sw + x0], p10 = out.texels[src + (size_t)y0 * sw + x1];
          const uint32_t p01 = out.texels[src + (size_t)y1 * sw + x0], p11 = out.texels[src + (size_t)y1 * sw + x1];
          uint32_t packed = 0;
          for (int ch = 0; ch < 4; ++ch) {
            const float* d = ch == 3 ? out.lut.data() : dec;  // alpha is linear in sRGB formats
            const int sh8 = 8 * ch;
            const float c00 = d[(p00 >> sh8) & 255u], c10 = d[(p10 >> sh8) & 255u];
            const float c01 = d[(p01 >> sh8) & 255u], c11 = d[(p11 >> sh8) & 255u];
            const float c = (c00 * (1.0f - a) + c10 * a) * (1.0f - b) + (c01 * (1.0f - a) + c11 * a) * b;
            const float e = (T.srgb && ch < 3) ? linear_to_srgb(c) : c;
            packed |= to_u8(e) << sh8;
          }
          out.texels[dst + (size_t)y * dw + x] = packed;
        }
      }
      sw = dw;
      sh = dh;
    }
  }
  if (out.texels.empty()) out.texels.push_back(0xFFFFFFFFu);
  if (out.info.empty()) out.info.assign(PTGS_TEX_INFO, 0u);
  return true;
}

}  // namespace ptgs
