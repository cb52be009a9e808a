// Drives integration/vRendererHIP through the vRenderer interface the way
// NGLScene does (src/NGLScene.cpp:82-89,196-197,205-231,259,345-457), with
// stand-in Camera/GL implementations.  Writes the last RGBA8 image uploaded
// to the colour texture and the frame count to argv[1].
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "vRendererHIP.h"

// loadBRDF takes ownership of the table and delete[]s it, as
// src/vRendererCuda.cpp:430 does: count the array deletions of that pointer
static const void *g_watch = nullptr;
static int g_watch_deleted = 0;
void operator delete[](void *p) noexcept
{
  if(p && p == g_watch)
    ++g_watch_deleted;
  std::free(p);
}
void operator delete[](void *p, std::size_t) noexcept { operator delete[](p); }
void *operator new[](std::size_t n)
{
  void *p = std::malloc(n ? n : 1);
  if(!p)
    throw std::bad_alloc();
  return p;
}

static std::vector<unsigned char> g_colour;
static GLuint g_bound = 0;

void glBindTexture(GLenum, GLuint texture) { g_bound = texture; }
void glTexSubImage2D(GLenum, GLint, GLint, GLint, GLsizei w, GLsizei h, GLenum, GLenum, const void *pixels)
{
  if(g_bound == 1)
    g_colour.assign(static_cast<const unsigned char *>(pixels), static_cast<const unsigned char *>(pixels) + 4 * w * h);
}

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

// ---- a host SBVH for the mesh mode -----------------------------------------
// The application hands initMesh a vMeshData whose m_bvh its SBVH builder
// made (src/SBVH.cpp); this driver stands in with a median-split tree over
// triangle centroids (leaves of <= 4 triangles) in the stand-in node classes.
static AABB triBounds(const vMeshData &_m, const std::vector<unsigned int> &_ref, size_t _a, size_t _b)
{
  ngl::Vec3 lo, hi;
  lo.m_x = lo.m_y = lo.m_z = 1e30f;
  hi.m_x = hi.m_y = hi.m_z = -1e30f;
  for(size_t i = _a; i < _b; ++i)
    for(int k = 0; k < 3; ++k)
    {
      const ngl::Vec3 &v = _m.m_vertices[_m.m_triangles[_ref[i]].m_indices[k]].m_vert;
      lo.m_x = std::fmin(lo.m_x, v.m_x); lo.m_y = std::fmin(lo.m_y, v.m_y); lo.m_z = std::fmin(lo.m_z, v.m_z);
      hi.m_x = std::fmax(hi.m_x, v.m_x); hi.m_y = std::fmax(hi.m_y, v.m_y); hi.m_z = std::fmax(hi.m_z, v.m_z);
    }
  return AABB(lo, hi);
}

static BVHNode *buildTree(const vMeshData &_m, std::vector<unsigned int> &_ref, size_t _a, size_t _b)
{
  const AABB box = triBounds(_m, _ref, _a, _b);
  if(_b - _a <= 4)
    return new LeafNode(box, static_cast<unsigned int>(_a), static_cast<unsigned int>(_b));
  const ngl::Vec3 lo = box.minBounds(), hi = box.maxBounds();
  const float ext[3] = { hi.m_x - lo.m_x, hi.m_y - lo.m_y, hi.m_z - lo.m_z };
  const int axis = ext[0] >= ext[1] && ext[0] >= ext[2] ? 0 : (ext[1] >= ext[2] ? 1 : 2);
  auto centroid = [&](unsigned int t) {
    float c = 0.f;
    for(int k = 0; k < 3; ++k)
    {
      const ngl::Vec3 &v = _m.m_vertices[_m.m_triangles[t].m_indices[k]].m_vert;
      c += axis == 0 ? v.m_x : (axis == 1 ? v.m_y : v.m_z);
    }
    return c;
  };
  const size_t mid = (_a + _b) / 2;
  std::nth_element(_ref.begin() + _a, _ref.begin() + mid, _ref.begin() + _b,
                   [&](unsigned int x, unsigned int y) { return centroid(x) < centroid(y) || (centroid(x) == centroid(y) && x < y); });
  BVHNode *l = buildTree(_m, _ref, _a, mid);
  BVHNode *r = buildTree(_m, _ref, mid, _b);
  return new InnerNode(box, l, r);
}

// mesh file (tests/test_adapter.py): u32 nv, nt; f32 pos[3nv], nrm[3nv], tan[3nv], uv[2nv]; u32 tris[3nt]
static bool loadMesh(const char *_path, vMeshData &_m)
{
  FILE *f = std::fopen(_path, "rb");
  if(!f)
    return false;
  uint32_t n[2];
  bool ok = std::fread(n, 4, 2, f) == 2;
  std::vector<float> pos(3 * n[0]), nrm(3 * n[0]), tan(3 * n[0]), uv(2 * n[0]);
  std::vector<uint32_t> tris(3 * n[1]);
  ok = ok && std::fread(pos.data(), 4, pos.size(), f) == pos.size() && std::fread(nrm.data(), 4, nrm.size(), f) == nrm.size() &&
       std::fread(tan.data(), 4, tan.size(), f) == tan.size() && std::fread(uv.data(), 4, uv.size(), f) == uv.size() &&
       std::fread(tris.data(), 4, tris.size(), f) == tris.size();
  std::fclose(f);
  if(!ok)
    return false;
  _m.m_vertices.resize(n[0]);
  for(uint32_t i = 0; i < n[0]; ++i)
  {
    vHVert &v = _m.m_vertices[i];
    v.m_vert.m_x = pos[3 * i]; v.m_vert.m_y = pos[3 * i + 1]; v.m_vert.m_z = pos[3 * i + 2];
    v.m_normal.m_x = nrm[3 * i]; v.m_normal.m_y = nrm[3 * i + 1]; v.m_normal.m_z = nrm[3 * i + 2];
    v.m_tangent.m_x = tan[3 * i]; v.m_tangent.m_y = tan[3 * i + 1]; v.m_tangent.m_z = tan[3 * i + 2];
    v.m_u = uv[2 * i]; v.m_v = uv[2 * i + 1];
  }
  _m.m_triangles.resize(n[1]);
  for(uint32_t t = 0; t < n[1]; ++t)
    for(int k = 0; k < 3; ++k)
      _m.m_triangles[t].m_indices[k] = tris[3 * t + k];
  _m.m_bvh.m_triIndices.resize(n[1]);
  for(uint32_t t = 0; t < n[1]; ++t)
    _m.m_bvh.m_triIndices[t] = t;
  _m.m_bvh.m_root.reset(buildTree(_m, _m.m_bvh.m_triIndices, 0, n[1]));
  return true;
}

static void writeFlat(FILE *_out, const vRendererHIP::FlatMesh &_flat)
{
  const uint32_t n[2] = { static_cast<uint32_t>(_flat.bvh.size() / 4), static_cast<uint32_t>(_flat.verts.size() / 4) };
  std::fwrite(n, 4, 2, _out);
  for(const std::vector<float> *v : { &_flat.bvh, &_flat.verts, &_flat.normals, &_flat.tangents, &_flat.uvs })
    std::fwrite(v->data(), 4, v->size(), _out);
}

// ---- scene files (tests/test_adapter.py) ---------------------------------------
// u32 W, H, frames, cornell, example_sphere, use_brdf, has_mesh
//   [mesh: as loadMesh]
// u32 has_hdr [u32 w, h; u16 halves[4wh] (Imf::Rgba)]
// u32 n_tex  [per texture: u32 type, w, h; f32 gamma; u32 argb[wh] (QRgb)]
// u32 has_brdf [f32 table[3 * 90 * 90 * 180] (MERL, planar R, G, B)]
struct Reader
{
  FILE *f;
  bool ok = true;
  template <typename T> T get() { T v{}; ok = ok && std::fread(&v, sizeof(T), 1, f) == 1; return v; }
  template <typename T> void get(T *dst, size_t n) { ok = ok && std::fread(dst, sizeof(T), n, f) == n; }
};

static bool readMeshFrom(Reader &_in, vMeshData &_m)
{
  const uint32_t nv = _in.get<uint32_t>(), nt = _in.get<uint32_t>();
  std::vector<float> pos(3 * nv), nrm(3 * nv), tan(3 * nv), uv(2 * nv);
  std::vector<uint32_t> tris(3 * nt);
  _in.get(pos.data(), pos.size()); _in.get(nrm.data(), nrm.size()); _in.get(tan.data(), tan.size());
  _in.get(uv.data(), uv.size()); _in.get(tris.data(), tris.size());
  if(!_in.ok)
    return false;
  _m.m_vertices.resize(nv);
  for(uint32_t i = 0; i < nv; ++i)
  {
    vHVert &v = _m.m_vertices[i];
    v.m_vert.m_x = pos[3 * i]; v.m_vert.m_y = pos[3 * i + 1]; v.m_vert.m_z = pos[3 * i + 2];
    v.m_normal.m_x = nrm[3 * i]; v.m_normal.m_y = nrm[3 * i + 1]; v.m_normal.m_z = nrm[3 * i + 2];
    v.m_tangent.m_x = tan[3 * i]; v.m_tangent.m_y = tan[3 * i + 1]; v.m_tangent.m_z = tan[3 * i + 2];
    v.m_u = uv[2 * i]; v.m_v = uv[2 * i + 1];
  }
  _m.m_triangles.resize(nt);
  for(uint32_t t = 0; t < nt; ++t)
    for(int k = 0; k < 3; ++k)
      _m.m_triangles[t].m_indices[k] = tris[3 * t + k];
  _m.m_bvh.m_triIndices.resize(nt);
  for(uint32_t t = 0; t < nt; ++t)
    _m.m_bvh.m_triIndices[t] = t;
  _m.m_bvh.m_root.reset(buildTree(_m, _m.m_bvh.m_triIndices, 0, nt));
  return true;
}

// Every ingestion entry point NGLScene calls, in its order: init, register*,
// setCamera, the toggles, setFresnel*, initMesh, loadHDR (Imf::Rgba halves),
// loadTexture (QImage, gamma; inverse gamma on diffuse only), loadBRDF (takes
// ownership), useBRDF; then `frames` render() calls.  Output: frames, the
// colour texture, whether loadBRDF delete[]d the table exactly once, and the
// flattened mesh the adapter uploaded (if any).
static int runSceneFile(const char *_out, const char *_scene)
{
  Reader in{ std::fopen(_scene, "rb") };
  if(!in.f)
    return 3;
  const uint32_t W = in.get<uint32_t>(), H = in.get<uint32_t>(), frames = in.get<uint32_t>();
  const bool cornell = in.get<uint32_t>() != 0, example = in.get<uint32_t>() != 0, useBrdf = in.get<uint32_t>() != 0;
  vMeshData mesh;
  const bool hasMesh = in.get<uint32_t>() != 0;
  if(hasMesh && !readMeshFrom(in, mesh))
    return 3;
  std::vector<Imf::Rgba> hdr;
  uint32_t hw = 0, hh = 0;
  if(in.get<uint32_t>() != 0)
  {
    hw = in.get<uint32_t>(); hh = in.get<uint32_t>();
    hdr.resize(static_cast<size_t>(hw) * hh);
    in.get(reinterpret_cast<uint16_t *>(hdr.data()), 4 * hdr.size());
  }
  struct Tex { uint32_t type; float gamma; QImage img; };
  std::vector<Tex> texs(in.get<uint32_t>());
  for(Tex &t : texs)
  {
    t.type = in.get<uint32_t>();
    const uint32_t w = in.get<uint32_t>(), h = in.get<uint32_t>();
    t.gamma = in.get<float>();
    t.img = QImage(static_cast<int>(w), static_cast<int>(h), QImage::Format_ARGB32);
    std::vector<uint32_t> px(static_cast<size_t>(w) * h);
    in.get(px.data(), px.size());
    for(uint32_t y = 0; y < h; ++y)
      for(uint32_t x = 0; x < w; ++x)
        t.img.setPixel(static_cast<int>(x), static_cast<int>(y), px[static_cast<size_t>(y) * w + x]);
  }
  float *brdf = nullptr;
  if(in.get<uint32_t>() != 0)
  {
    const size_t n = 3u * BRDF_SAMPLING_RES_THETA_H * BRDF_SAMPLING_RES_THETA_D * BRDF_SAMPLING_RES_PHI_D / 2;
    brdf = new float[n];                      // as vBRDFLoader::loadBinary hands it over
    in.get(brdf, n);
  }
  std::fclose(in.f);
  if(!in.ok)
    return 3;

  vRendererHIP r;
  r.init(W, H);
  GLuint tex = 1, depth = 2;
  r.registerTextureBuffer(tex);
  r.registerDepthBuffer(depth);
  Camera cam;
  r.setCamera(&cam);
  r.useCornellBox(cornell);
  r.useExampleSphere(example);
  r.setFresnelCoef(0.1f);
  r.setFresnelPower(3.f);
  if(hasMesh)
    r.initMesh(mesh);
  if(!hdr.empty())
    r.loadHDR(hdr.data(), hw, hh);
  for(const Tex &t : texs)
    r.loadTexture(t.img, t.gamma, t.type);
  uint32_t brdfDeleted = 0;
  if(brdf)
  {
    g_watch = brdf;
    const bool loaded = r.loadBRDF(brdf);
    brdfDeleted = (loaded && g_watch_deleted == 1) ? 1u : 0u;
    g_watch = nullptr;
  }
  r.useBRDF(useBrdf);
  r.clearBuffer();
  for(uint32_t f = 0; f < frames; ++f)
    r.render();
  const unsigned int n = r.getFrameCount();
  r.cleanUp();
  FILE *out = std::fopen(_out, "wb");
  std::fwrite(&n, 4, 1, out);
  std::fwrite(&brdfDeleted, 4, 1, out);
  std::fwrite(g_colour.data(), 1, g_colour.size(), out);
  if(hasMesh)
  {
    vRendererHIP::FlatMesh flat;
    vRendererHIP::flattenSBVH(mesh, flat);
    writeFlat(out, flat);
  }
  std::fclose(out);
  std::printf("frames=%u bytes=%zu brdf_deleted=%u\n", n, g_colour.size(), brdfDeleted);
  return 0;
}

// usage: adapter_driver <out>                      Cornell + example sphere, 64x64, 3 frames
//        adapter_driver <out> --scene <file>       a scene file (above) through every ingestion call
//        adapter_driver <out> <mesh> [--flatten]   Cornell + the mesh (its SBVH flattened by the
//                                                  adapter); --flatten: only write the flat arrays (no GPU)
//        adapter_driver <out> --devices <list>     write the device list init() parses from VRHIP_DEVICES (no GPU)
int main(int argc, char **argv)
{
  if(argc < 2)
    return 2;
  if(argc >= 4 && std::strcmp(argv[2], "--devices") == 0)
  {
    const std::vector<int> d = vRendererHIP::parseDevices(argv[3]);
    FILE *out = std::fopen(argv[1], "w");
    if(!out)
      return 4;
    for(size_t i = 0; i < d.size(); ++i)
      std::fprintf(out, i ? ",%d" : "%d", d[i]);
    std::fclose(out);
    return 0;
  }
  if(argc >= 4 && std::strcmp(argv[2], "--scene") == 0)
    return runSceneFile(argv[1], argv[3]);
  vMeshData mesh;
  const bool withMesh = argc >= 3;
  if(withMesh && !loadMesh(argv[2], mesh))
    return 3;
  if(argc >= 4 && std::strcmp(argv[3], "--flatten") == 0)
  {
    vRendererHIP::FlatMesh flat;
    if(!vRendererHIP::flattenSBVH(mesh, flat))
      return 4;
    FILE *out = std::fopen(argv[1], "wb");
    writeFlat(out, flat);
    std::fclose(out);
    std::printf("nodes=%zu slots=%zu\n", flat.bvh.size() / 16, flat.verts.size() / 4);
    return 0;
  }
  vRendererHIP r;
  r.init(64, 64);
  GLuint tex = 1, depth = 2;
  r.registerTextureBuffer(tex);
  r.registerDepthBuffer(depth);
  Camera cam;
  r.setCamera(&cam);
  r.useCornellBox(true);
  r.useExampleSphere(!withMesh);
  r.setFresnelCoef(0.1f);
  r.setFresnelPower(3.f);
  if(withMesh)
    r.initMesh(mesh);
  for(int f = 0; f < 3; ++f)
    r.render();
  const unsigned int frames = r.getFrameCount();
  r.cleanUp();
  FILE *out = std::fopen(argv[1], "wb");
  std::fwrite(&frames, 4, 1, out);
  std::fwrite(g_colour.data(), 1, g_colour.size(), out);
  if(withMesh)
  {
    vRendererHIP::FlatMesh flat;
    vRendererHIP::flattenSBVH(mesh, flat);
    writeFlat(out, flat);
  }
  std::fclose(out);
  std::printf("frames=%u bytes=%zu\n", frames, g_colour.size());
  return 0;
}
