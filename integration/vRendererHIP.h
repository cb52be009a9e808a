///
/// \file vRendererHIP.h
/// \brief MI355X (HIP, gfx950) backend behind the reference's vRenderer
///        interface (include/vRenderer.h:30-168): the peer of vRendererCuda
///        (include/vRendererCuda.h) and vRendererCL.  All device work goes
///        through the C ABI of libvrhip.so (include/vrhip.h).
///
/// Drop into the reference tree as include/vRendererHIP.h + src/vRendererHIP.cpp
/// and select it with `#ifdef __VRENDERER_HIP__` in src/NGLScene.cpp (see
/// INTEGRATION.md).
///
#pragma once

#include <string>
#include <vector>

#include "vRenderer.h"
#include "vrhip.h"

class vRendererHIP : public vRenderer
{
public:
  vRendererHIP();
  ~vRendererHIP();

  void init(const unsigned int &_w, const unsigned int &_h) override;
  void registerTextureBuffer(GLuint &_texture) override;
  void registerDepthBuffer(GLuint &_depthTexture) override;
  void render() override;
  void cleanUp() override;
  void updateCamera() override;
  void initMesh(const vMeshData &_meshData) override;
  void loadHDR(const Imf::Rgba *_colours, const unsigned int &_w, const unsigned int &_h) override;
  void loadTexture(const QImage &_texture, const float &_gamma, const unsigned int &_type) override;
  void useBRDF(const bool &_newVal) override;
  void useExampleSphere(const bool &_newVal) override;
  void useCornellBox(const bool &_newVal) override;
  void clearBuffer() override;
  bool loadBRDF(const float *_brdf) override;
  unsigned int getFrameCount() const override;

  /// The reference's flattened mesh layout (src/vRendererCuda.cpp:204-279):
  /// float4 rows for bvh/verts/normals/tangents, float2 for uvs.
  struct FlatMesh
  {
    std::vector<float> bvh, verts, normals, tangents, uvs;
  };
  /// Flattens the application's SBVH (vMeshData::m_bvh) into that layout, as
  /// initMesh uploads it; false for an empty tree or a leaf root.  Host only.
  static bool flattenSBVH(const vMeshData &_meshData, FlatMesh &_out);
  /// VRHIP_DEVICES parsing ("0,1,2,3"): the GPUs init() spreads the image
  /// over (vrhip_create_multi) when it names more than one.  Host only.
  static std::vector<int> parseDevices(const char *_list);

private:
  /// Reference error behaviour (src/vRendererCuda.cpp:454-467): message,
  /// errorlog.txt, exit(0).  The C ABI itself only returns status codes.
  void validate(int _status, const std::string &_msg);

  vrhip_ctx *m_ctx;
  GLuint m_texture;
  GLuint m_depthTexture;
  bool m_interopTexture;
  bool m_interopDepth;
  bool m_hasTexture;
  bool m_hasDepth;
  std::vector<unsigned char> m_rgba;
  std::vector<unsigned char> m_depth;
  unsigned int m_width;
  unsigned int m_height;
  bool m_initialised;
};
