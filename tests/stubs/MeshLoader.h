#pragma once
#include <vector>
#include <ngl/Vec3.h>
#include "SBVH.h"
typedef struct vHVert { ngl::Vec3 m_vert, m_normal, m_tangent; float m_u, m_v; } vHVert;
typedef struct vHTriangle { unsigned int m_indices[3]; } vHTriangle;
typedef struct vMeshData { std::vector<vHTriangle> m_triangles; std::vector<vHVert> m_vertices; SBVH m_bvh; } vMeshData;
