// Drives integration/vRendererHIP through the vRenderer interface the way
// NGLScene does (src/NGLScene.cpp:82-89,196-197,224,259,443-456), with
// stand-in Camera/GL implementations.  Writes the last RGBA8 image uploaded
// to the colour texture and the frame count to argv[1].
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "vRendererHIP.h"

static std::vector<unsigned char> g_colour;
static GLuint g_bound = 0;

void glBindTexture(GLenum, GLuint texture) { g_bound = texture; }
void glTexSubImage2D(GLenum, GLint, GLint, GLint, GLsizei w, GLsizei h, GLenum, GLenum, const void *pixels)
{
  if(g_bound == 1)
    g_colour.assign(static_cast<const unsigned char *>(pixels), static_cast<const unsigned char *>(pixels) + 4 * w * h);
}
int QImage::width() const { return 0; }
int QImage::height() const { return 0; }
QRgb QImage::pixel(int, int) const { return 0; }

// reference default camera (src/Camera.cpp:11-24,119-123)
void Camera::consume() {}
bool Camera::isDirty() const { return false; }
ngl::Vec3 Camera::getOrig() const { ngl::Vec3 v; v.m_z = 150.f; return v; }
ngl::Vec3 Camera::getDir() const { ngl::Vec3 v; v.m_z = -1.f; return v; }
ngl::Vec3 Camera::getUp() const { ngl::Vec3 v; v.m_y = 1.f; return v; }
ngl::Vec3 Camera::getRight() const { ngl::Vec3 v; v.m_x = 1.f; return v; }
float Camera::getFovScale() const
{
  const float kDegInRad = M_PI / 180.f;
  return std::tan(75.f * kDegInRad / 2.f);
}

int main(int argc, char **argv)
{
  if(argc < 2)
    return 2;
  vRendererHIP r;
  r.init(64, 64);
  GLuint tex = 1, depth = 2;
  r.registerTextureBuffer(tex);
  r.registerDepthBuffer(depth);
  Camera cam;
  r.setCamera(&cam);
  r.useCornellBox(true);
  r.useExampleSphere(true);
  r.setFresnelCoef(0.1f);
  r.setFresnelPower(3.f);
  for(int f = 0; f < 3; ++f)
    r.render();
  const unsigned int frames = r.getFrameCount();
  r.cleanUp();
  FILE *out = std::fopen(argv[1], "wb");
  std::fwrite(&frames, 4, 1, out);
  std::fwrite(g_colour.data(), 1, g_colour.size(), out);
  std::fclose(out);
  std::printf("frames=%u bytes=%zu\n", frames, g_colour.size());
  return 0;
}
