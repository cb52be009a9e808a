///
/// \file vRendererHIP.cpp
/// \brief vRenderer implementation over libvrhip.so (include/vrhip.h).
///
/// Mirrors vRendererCuda (src/vRendererCuda.cpp) method by method; the
/// device work (accumulation buffer, scene buffers, megakernel) lives in the
/// library.  Display: each frame's RGBA8 colour and depth images are read
/// back and uploaded to the two GL textures the scene registered (the CUDA
/// backend writes them through GL-interop surfaces, :57-67,117-162).
///
#include "vRendererHIP.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

vRendererHIP::vRendererHIP() :
  m_ctx(nullptr),
  m_texture(0),
  m_depthTexture(0),
  m_interopTexture(false),
  m_interopDepth(false),
  m_hasTexture(false),
  m_hasDepth(false),
  m_width(0),
  m_height(0),
  m_initialised(false)
{
  m_fresnelCoef = 0.1f;
  m_fresnelPow = 3.f;
}

vRendererHIP::~vRendererHIP()
{
  cleanUp();
}

std::vector<int> vRendererHIP::parseDevices(const char *_list)
{
  // "0,1,2,3" (commas or spaces); anything that is not a device index ends the list
  std::vector<int> out;
  if(!_list)
    return out;
  const char *p = _list;
  while(*p)
  {
    while(*p == ',' || *p == ' ')
      ++p;
    if(!*p)
      break;
    char *end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if(end == p || v < 0 || v > 1023)
      break;
    out.push_back(static_cast<int>(v));
    p = end;
  }
  return out;
}

void vRendererHIP::validate(int _status, const std::string &_msg)
{
  if(_status == VRHIP_OK)
    return;
  std::cerr << "Failed to perform a HIP operation: " << _msg << "\n";
  std::cerr << "Err: " << vrhip_last_error() << "\n";
  if(FILE *log = std::fopen("errorlog.txt", "w"))
  {
    std::fprintf(log, "%s: %s\n", _msg.c_str(), vrhip_last_error());
    std::fclose(log);
  }
  std::cerr << "Check errorlog.txt for more details\n";
  std::exit(0);
}

void vRendererHIP::init(const unsigned int &_w, const unsigned int &_h)
{
  m_width = _w;
  m_height = _h;
  // VRHIP_DEVICES="0,1,2,3": one renderer over those GPUs (the image's tiles
  // dealt over them, gathered to the first over RCCL every frame); else one
  // GPU, VRHIP_DEVICE (default 0)
  const std::vector<int> devices = parseDevices(std::getenv("VRHIP_DEVICES"));
  if(devices.size() > 1)
    validate(vrhip_create_multi(devices.data(), static_cast<uint32_t>(devices.size()), _w, _h, &m_ctx),
             "Create multi-GPU HIP context");
  else
  {
    const char *dev = std::getenv("VRHIP_DEVICE");
    validate(vrhip_create(devices.size() == 1 ? devices[0] : (dev ? std::atoi(dev) : 0), _w, _h, &m_ctx),
             "Create HIP context");
  }
  // no kernel-timing events on the launch path: nothing here reads them, and
  // at one synchronous frame per paint they cost ~8 us a frame
  validate(vrhip_set_kernel_timing(m_ctx, 0), "Kernel timing off");
  validate(vrhip_set_fresnel(m_ctx, m_fresnelCoef, m_fresnelPow), "Set Fresnel parameters");
  m_rgba.assign(static_cast<size_t>(_w) * _h * 4, 0);
  m_depth.assign(static_cast<size_t>(_w) * _h * 4, 0);
  m_initialised = true;
}

// GL interop first (HIP maps the texture; the frame is copied device to
// device), read-back + glTexSubImage2D when the driver refuses interop
// (e.g. a GL context on another device).
void vRendererHIP::registerTextureBuffer(GLuint &_texture)
{
  m_texture = _texture;
  m_hasTexture = true;
  m_interopTexture = vrhip_gl_register_image(m_ctx, 0, _texture, GL_TEXTURE_2D) == VRHIP_OK;
}

void vRendererHIP::registerDepthBuffer(GLuint &_depthTexture)
{
  m_depthTexture = _depthTexture;
  m_hasDepth = true;
  m_interopDepth = vrhip_gl_register_image(m_ctx, 1, _depthTexture, GL_TEXTURE_2D) == VRHIP_OK;
}

void vRendererHIP::updateCamera()
{
  m_virtualCamera->consume();
  const ngl::Vec3 o = m_virtualCamera->getOrig();
  const ngl::Vec3 d = m_virtualCamera->getDir();
  const ngl::Vec3 u = m_virtualCamera->getUp();
  const ngl::Vec3 r = m_virtualCamera->getRight();
  const float origin[3] = { o.m_x, o.m_y, o.m_z };
  const float dir[3] = { d.m_x, d.m_y, d.m_z };
  const float up[3] = { u.m_x, u.m_y, u.m_z };
  const float right[3] = { r.m_x, r.m_y, r.m_z };
  // resets the frame counter and clears the accumulation buffer
  validate(vrhip_set_camera(m_ctx, origin, dir, up, right, m_virtualCamera->getFovScale()), "Update camera");
}

void vRendererHIP::clearBuffer()
{
  // setFresnelCoef/Power (include/vRenderer.h:139-145) store the new value
  // and call clearBuffer; pass the current values with the clear
  validate(vrhip_set_fresnel(m_ctx, m_fresnelCoef, m_fresnelPow), "Set Fresnel parameters");
  validate(vrhip_clear(m_ctx), "Clear buffer");
}

void vRendererHIP::render()
{
  if(m_virtualCamera->isDirty())
    updateCamera();

  // wall-clock milliseconds seed the RNG, as src/vRendererCuda.cpp:114,153
  // (VRHIP_FIXED_TIME pins it for reproducible runs)
  const auto now = std::chrono::high_resolution_clock::now();
  unsigned int t = static_cast<unsigned int>(
      std::chrono::duration_cast<std::chrono::milliseconds>(now.time_since_epoch()).count());
  if(const char *fixed = std::getenv("VRHIP_FIXED_TIME"))
    t = static_cast<unsigned int>(std::strtoul(fixed, nullptr, 10));

  validate(vrhip_render(m_ctx, 1, nullptr, t), "Render");
  validate(vrhip_sync(m_ctx), "Synchronize");

  if((m_interopTexture || m_interopDepth) && vrhip_gl_present(m_ctx) != VRHIP_OK)
  {
    // the driver accepted the registration but cannot map it (no shared GL
    // context): use the read-back path from now on
    std::cerr << "GL interop unavailable (" << vrhip_last_error() << "), using read-back\n";
    m_interopTexture = m_interopDepth = false;
  }
  if(m_hasTexture && !m_interopTexture)
  {
    validate(vrhip_read_rgba8(m_ctx, m_rgba.data()), "Read colour buffer");
    glBindTexture(GL_TEXTURE_2D, m_texture);
    glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, m_width, m_height, GL_RGBA, GL_UNSIGNED_BYTE, m_rgba.data());
  }
  if(m_hasDepth && !m_interopDepth)
  {
    validate(vrhip_read_depth8(m_ctx, m_depth.data()), "Read depth buffer");
    glBindTexture(GL_TEXTURE_2D, m_depthTexture);
    glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, m_width, m_height, GL_RGBA, GL_UNSIGNED_BYTE, m_depth.data());
  }
}

void vRendererHIP::cleanUp()
{
  if(m_initialised)
  {
    vrhip_destroy(m_ctx);
    m_ctx = nullptr;
    m_initialised = false;
  }
}

// The device layout of src/vRendererCuda.cpp:204-279, built from the
// application's own SBVH: node = 4 float4 (child 0 x/y bounds, child 1 x/y
// bounds, both z bounds, child indices); a child index >= 0 is the float4
// offset of an inner node, < 0 the complement of the child leaf's first
// triangle slot; a leaf's triangles take 3 consecutive slots each (vertices,
// normals, tangents as float4, uvs as float2) in SBVH triangle-reference order
// and end with a 0x80000000 terminator slot.  Nodes are laid out in the order
// a LIFO walk from the root reaches them (children taken in order, so the
// second child's subtree is emitted first), as the CUDA backend does; the
// library keeps the tree's child order and leaf triangle order, hence the
// reference's visit order and equal-t tie resolution.
bool vRendererHIP::flattenSBVH(const vMeshData &_meshData, FlatMesh &_out)
{
  _out = FlatMesh();
  const BVHNode *root = _meshData.m_bvh.getRoot();
  if(!root || root->isLeaf())
    return false;
  auto bits = [](uint32_t _u) { float f; std::memcpy(&f, &_u, 4); return f; };
  auto pushRow = [](std::vector<float> &_v, float _a, float _b, float _c, float _d) {
    _v.push_back(_a); _v.push_back(_b); _v.push_back(_c); _v.push_back(_d);
  };
  struct Pending { const BVHNode *node; size_t row; };   // row = float4 offset of the node
  std::vector<Pending> todo{ { root, 0 } };
  _out.bvh.assign(16, 0.f);
  while(!todo.empty())
  {
    const Pending cur = todo.back();
    todo.pop_back();
    AABB box[2];
    int32_t link[2];
    for(unsigned int c = 0; c < 2; ++c)
    {
      const BVHNode *child = cur.node->childNode(c);
      box[c] = child->getBounds();
      if(!child->isLeaf())
      {
        link[c] = static_cast<int32_t>(_out.bvh.size() / 4);
        todo.push_back({ child, _out.bvh.size() / 4 });
        _out.bvh.resize(_out.bvh.size() + 16, 0.f);
        continue;
      }
      const LeafNode *leaf = static_cast<const LeafNode *>(child);
      link[c] = ~static_cast<int32_t>(_out.verts.size() / 4);
      for(unsigned int j = leaf->firstIndex(); j < leaf->lastIndex(); ++j)
      {
        const vHTriangle &tri = _meshData.m_triangles[_meshData.m_bvh.getTriIndex(j)];
        for(unsigned int k = 0; k < 3; ++k)
        {
          const vHVert &v = _meshData.m_vertices[tri.m_indices[k]];
          pushRow(_out.verts, v.m_vert.m_x, v.m_vert.m_y, v.m_vert.m_z, 0.f);
          pushRow(_out.normals, v.m_normal.m_x, v.m_normal.m_y, v.m_normal.m_z, 0.f);
          pushRow(_out.tangents, v.m_tangent.m_x, v.m_tangent.m_y, v.m_tangent.m_z, 0.f);
          _out.uvs.push_back(v.m_u);
          _out.uvs.push_back(v.m_v);
        }
      }
      pushRow(_out.verts, bits(0x80000000u), 0.f, 0.f, 0.f);
      pushRow(_out.normals, bits(0x80000000u), 0.f, 0.f, 0.f);
      pushRow(_out.tangents, bits(0x80000000u), 0.f, 0.f, 0.f);
      _out.uvs.push_back(bits(0x80000000u));
      _out.uvs.push_back(0.f);
    }
    float *n = &_out.bvh[4 * cur.row];
    const ngl::Vec3 lo0 = box[0].minBounds(), hi0 = box[0].maxBounds();
    const ngl::Vec3 lo1 = box[1].minBounds(), hi1 = box[1].maxBounds();
    const float rows[16] = { lo0.m_x, hi0.m_x, lo0.m_y, hi0.m_y,
                             lo1.m_x, hi1.m_x, lo1.m_y, hi1.m_y,
                             lo0.m_z, hi0.m_z, lo1.m_z, hi1.m_z,
                             bits(static_cast<uint32_t>(link[0])), bits(static_cast<uint32_t>(link[1])), 0.f, 0.f };
    std::memcpy(n, rows, sizeof(rows));
  }
  return true;
}

void vRendererHIP::initMesh(const vMeshData &_meshData)
{
  // Default: upload the application's SBVH in the reference's flattened
  // layout (the traversal then visits nodes and resolves equal-t ties exactly
  // as the CUDA backend does).  VRHIP_NATIVE_BVH=1 instead rebuilds a binned-
  // SAH tree from the indexed mesh in the library (same closest hits up to
  // the order of exactly tied triangles; the SBVH build is then unnecessary).
  const char *native = std::getenv("VRHIP_NATIVE_BVH");
  if(!(native && native[0] == '1'))
  {
    FlatMesh flat;
    if(!flattenSBVH(_meshData, flat))
      validate(VRHIP_ERR_BVH, "Flatten SBVH (empty tree or a leaf root)");
    validate(vrhip_upload_mesh_flat(m_ctx, flat.bvh.data(), flat.bvh.size() / 4, flat.verts.data(),
                                    flat.normals.data(), flat.tangents.data(), flat.uvs.data(), flat.verts.size() / 4),
             "Upload mesh");
    return;
  }
  const size_t nv = _meshData.m_vertices.size();
  std::vector<float> pos(3 * nv), nrm(3 * nv), tan(3 * nv), uv(2 * nv);
  for(size_t i = 0; i < nv; ++i)
  {
    const vHVert &v = _meshData.m_vertices[i];
    pos[3 * i + 0] = v.m_vert.m_x;    pos[3 * i + 1] = v.m_vert.m_y;    pos[3 * i + 2] = v.m_vert.m_z;
    nrm[3 * i + 0] = v.m_normal.m_x;  nrm[3 * i + 1] = v.m_normal.m_y;  nrm[3 * i + 2] = v.m_normal.m_z;
    tan[3 * i + 0] = v.m_tangent.m_x; tan[3 * i + 1] = v.m_tangent.m_y; tan[3 * i + 2] = v.m_tangent.m_z;
    uv[2 * i + 0] = v.m_u;            uv[2 * i + 1] = v.m_v;
  }
  const size_t nt = _meshData.m_triangles.size();
  std::vector<uint32_t> tris(3 * nt);
  for(size_t i = 0; i < nt; ++i)
    for(int k = 0; k < 3; ++k)
      tris[3 * i + k] = _meshData.m_triangles[i].m_indices[k];
  validate(vrhip_upload_mesh_indexed(m_ctx, pos.data(), nrm.data(), tan.data(), uv.data(),
                                     static_cast<uint32_t>(nv), tris.data(), static_cast<uint32_t>(nt), 2),
           "Upload mesh");
}

void vRendererHIP::loadHDR(const Imf::Rgba *_colours, const unsigned int &_w, const unsigned int &_h)
{
  // Imf::Rgba is four IEEE halves; the library converts them on the device
  // (src/vRendererCuda.cpp:322-327 converts on the host)
  static_assert(sizeof(Imf::Rgba) == 8, "Imf::Rgba must be 4 x half");
  validate(vrhip_upload_hdr_half(m_ctx, reinterpret_cast<const uint16_t *>(_colours), _w, _h), "Upload HDR map");
}

void vRendererHIP::loadTexture(const QImage &_texture, const float &_gamma, const unsigned int &_type)
{
  const unsigned int w = _texture.width();
  const unsigned int h = _texture.height();
  const float correction = (_gamma > 0.001f ? 1.f / _gamma : 1.f);
  std::vector<float> data(static_cast<size_t>(w) * h * 4);
  size_t k = 0;
  for(unsigned int j = 0; j < h; ++j)
    for(unsigned int i = 0; i < w; ++i)
    {
      const QColor pixel(_texture.pixel(i, j));
      const bool diffuse = (_type == VRHIP_TEX_DIFFUSE);
      // inverse gamma on diffuse maps only (src/vRendererCuda.cpp:344-368)
      data[k++] = diffuse ? std::pow(pixel.red() / 255.f, correction) : pixel.red() / 255.f;
      data[k++] = diffuse ? std::pow(pixel.green() / 255.f, correction) : pixel.green() / 255.f;
      data[k++] = diffuse ? std::pow(pixel.blue() / 255.f, correction) : pixel.blue() / 255.f;
      data[k++] = pixel.alpha() / 255.f;
    }
  validate(vrhip_upload_texture(m_ctx, static_cast<int>(_type), data.data(), w, h), "Upload texture");
}

bool vRendererHIP::loadBRDF(const float *_brdf)
{
  if(!_brdf)
    return false;
  const size_t n = 3u * BRDF_SAMPLING_RES_THETA_H * BRDF_SAMPLING_RES_THETA_D * BRDF_SAMPLING_RES_PHI_D / 2;
  validate(vrhip_upload_brdf(m_ctx, _brdf, n), "Upload BRDF");
  // the reference takes ownership of the table (src/vRendererCuda.cpp:430)
  delete [] _brdf;
  return true;
}

void vRendererHIP::useExampleSphere(const bool &_newVal)
{
  validate(vrhip_use_example_sphere(m_ctx, _newVal ? 1 : 0), "Use example sphere");
}

void vRendererHIP::useBRDF(const bool &_newVal)
{
  validate(vrhip_use_brdf(m_ctx, _newVal ? 1 : 0), "Use BRDF");
}

void vRendererHIP::useCornellBox(const bool &_newVal)
{
  validate(vrhip_use_cornell_box(m_ctx, _newVal ? 1 : 0), "Use Cornell box");
}

unsigned int vRendererHIP::getFrameCount() const
{
  uint32_t n = 0;
  vrhip_frame_count(m_ctx, &n);
  return n;
}
