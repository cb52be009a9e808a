#pragma once
// Stand-in for the reference's AABB (include/AABB.h): what the renderer reads.
#include <ngl/Vec3.h>
class AABB {
public:
  AABB() {}
  AABB(const ngl::Vec3 &_min, const ngl::Vec3 &_max) : m_min(_min), m_max(_max) {}
  ngl::Vec3 minBounds() const { return m_min; }
  ngl::Vec3 maxBounds() const { return m_max; }
private:
  ngl::Vec3 m_min, m_max;
};
