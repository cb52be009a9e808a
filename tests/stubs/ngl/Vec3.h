#pragma once
namespace ngl { struct Vec3 { float m_x = 0.f, m_y = 0.f, m_z = 0.f; }; }
