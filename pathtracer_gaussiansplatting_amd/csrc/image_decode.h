// Texture image decode for scene ingest: PNG and JPEG files -> RGBA8, with the output semantics of
// stbi_load(path, &w, &h, &n, STBI_rgb_alpha) as Image::createTextureImage calls it
// (Vulkan_Engine/image.cpp:12; stb_image v2.30 vendored at Helpers/stb_image.h).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace ptgs {

struct DecodedImage {
  std::vector<uint8_t> rgba;  // w * h * 4, row 0 first (no vertical flip, as the reference)
  uint32_t w = 0, h = 0;
  uint32_t comp = 0;          // channels in the file as stbi reports them (1..4)
};

// header_only: fill w/h/comp and stop. Returns false with err set on malformed or unsupported input.
bool decode_image_rgba8(const uint8_t* data, size_t size, DecodedImage& out, std::string& err,
                        bool header_only = false);

bool read_file(const std::string& path, std::vector<uint8_t>& bytes);

}  // namespace ptgs
