#pragma once
#include <ngl/Vec3.h>
class Camera {
public:
  void consume();
  bool isDirty() const;
  ngl::Vec3 getOrig() const;
  ngl::Vec3 getDir() const;
  ngl::Vec3 getUp() const;
  ngl::Vec3 getRight() const;
  float getFovScale() const;
};
