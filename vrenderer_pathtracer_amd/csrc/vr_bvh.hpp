// vr_bvh.hpp -- host BVH builder + reference-layout flattener (vr_bvh.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <vector>

#include "vr_params.hpp"

namespace vr {

// Cap on tree depth (inner-node levels).  The traversal stack holds at most
// one entry per level plus the sentinel, so depth <= 30 fits the 32-entry
// LDS stack; deeper uploaded trees use the 64-entry variant.
constexpr uint32_t kMaxBuildDepth = 30;

struct FlatMesh {
    std::vector<vr4> bvh;       // 4 float4 per inner node
    std::vector<vr4> verts, normals, tangents;
    std::vector<vr2> uvs;
};

int build_flat(const float* positions, const float* normals, const float* tangents, const float* uvs,
               uint32_t n_verts, const uint32_t* tris, uint32_t n_tris, uint32_t max_leaf_tris,
               FlatMesh& out);

// depth = number of inner-node levels on the longest root-to-node path.
int validate_flat(const float* bvh, size_t n_bvh_f4, const float* verts, size_t n_slots,
                  uint32_t* depth, uint32_t* n_nodes);

} // namespace vr
