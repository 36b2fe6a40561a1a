// jpeg.h — baseline JFIF encoder (jpeg.cpp) used by the capture pipeline.
#pragma once

#include <cstdint>
#include <vector>

namespace ptgs {

// pixels: w*h*comp bytes (comp 1 grey, 3 RGB, 4 RGBA with alpha ignored); quality 1..100
bool encode_jpeg(const uint8_t* pixels, uint32_t w, uint32_t h, uint32_t comp, int quality, std::vector<uint8_t>& out);

}  // namespace ptgs
