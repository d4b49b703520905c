// pt_jpeg.h — the JPEG decoder of pt_jpeg.cpp, for pt_image.cpp (host side only).
#pragma once

#include <cstddef>
#include <string>
#include <vector>

namespace pt {
// RGBA8, top row first, alpha 255; variant PT_JPEG_IJG9 (what pt_image_load uses) or PT_JPEG_IJG6.
bool decode_jpeg(const unsigned char* data, size_t size, int variant, int* width, int* height,
                 std::vector<unsigned char>& rgba, std::string& err);
}  // namespace pt
