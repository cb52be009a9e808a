// vr_exr.hpp -- minimal OpenEXR scanline reader (vr_exr.cpp).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace vr {

// Reads a single-part scanline OpenEXR file (NONE / RLE / ZIPS / ZIP) into
// half RGBA over its data window, as Imf::RgbaInputFile would deliver it.
// Returns 0, or -1 with the reason in `why`.
int read_exr_rgba_half(const char* path, std::vector<uint16_t>& rgba, uint32_t& width, uint32_t& height,
                       std::string& why);

} // namespace vr
