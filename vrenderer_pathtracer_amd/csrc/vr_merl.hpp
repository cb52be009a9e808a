// vr_merl.hpp -- MERL .binary BRDF reader (vr_merl.cpp), host only.
#pragma once
#include <stddef.h>
#include <string>

namespace vr {

// Floats in a MERL isotropic table: 3 x 90 x 90 x 180 (BRDF_SAMPLING_RES_*,
// include/vRenderer.h:23-25).
constexpr size_t kMerlFloats = 3u * 90u * 90u * 180u;

// vBRDFLoader::loadBinary (src/BRDFLoader.cpp:15-50): 3 int32 dims whose
// product must be 90*90*180, then 3*n doubles (planar R, G, B) -> `table`
// (kMerlFloats floats, same order).  Returns 0, or -1 with the reason in `why`
// (unreadable file, dimension mismatch, short file).
int read_merl(const char* path, float* table, std::string& why);

} // namespace vr
