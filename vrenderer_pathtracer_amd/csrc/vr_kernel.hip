// vr_kernel.hip -- gfx950 (CDNA4, wave64) path-tracing megakernel.
//
// Re-design of the reference per-pixel CUDA kernel `render`
// (cuda/src/PathTracer.cu:791-868) and everything it calls:
//   trace (:597-770), intersectScene (:136-468), SBVH while-while traversal
//   (:274-463), intersectTriangle (RayIntersection.cuh:54-111), lookupBRDF
//   (:473-566), hash + thrust minstd RNG (:574-580, :620-622).
// Results are defined by the reference algorithm in IEEE fp32 (no FMA
// contraction, correctly rounded div/sqrt, rsqrtf := 1/sqrtf) with the
// portable libm of vr_math.hpp; the CPU oracle (oracle/vro.c, portable
// mode) reproduces them bit for bit.
//
// MI355X mapping:
//   * one workgroup = one 16x16 pixel tile (the reference block, so grid
//     truncation is identical), four wave64s each owning an 8x8 sub-tile;
//   * the traversal stack lives in LDS, entry-major ([depth][256 lanes]) so
//     a wave's push/pop is one conflict-free ds_write/ds_read_b32;
//   * the while-while traversal switches to leaf processing on a wave64
//     __ballot (the reference's 32-lane vote.ballot, :353-363);
//   * leaf hits record only (t, slot, u, v); hit attributes are fetched once
//     per ray after traversal (result-identical: only the final accepted hit
//     is observable), cutting gathers on the hot loop;
//   * all K frames of a render step run in one launch with the pixel's
//     float4 accumulator kept in registers (one HBM read + one write per step).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include "vr_params.hpp"
#include "vr_math.hpp"

namespace vr {

#define VR_PI 3.14159265359f        // MathHelpers.cuh:16
#define VR_EPS 0.0000000003f        // MathHelpers.cuh:17

// Scene features are tested twice: against the kernel's compile-time feature
// set FEAT (code for absent features is compiled out, cutting VGPRs) and
// against the launch's runtime flags.
#define HAS(F) ((FEAT & (F)) != 0 && (p.flags & (F)) != 0)

// ---- float4 with the reference's operator semantics (MathHelpers.cuh:85-196)
__device__ __forceinline__ vr4 mk4(float x, float y, float z, float w) { vr4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
__device__ __forceinline__ vr4 add4(vr4 a, vr4 b) { return mk4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ vr4 sub4(vr4 a, vr4 b) { return mk4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ vr4 mul4(vr4 a, vr4 b) { return mk4(a.x * b.x, a.y * b.y, a.z * b.z, a.w); }
__device__ __forceinline__ vr4 mul4s(vr4 a, float b) { return mk4(a.x * b, a.y * b, a.z * b, a.w); }
__device__ __forceinline__ vr4 muls4(float a, vr4 b) { return mk4(a * b.x, a * b.y, a * b.z, b.w); }
__device__ __forceinline__ void muleq4(vr4& a, vr4 b) { a.x *= b.x; a.y *= b.y; a.z *= b.z; a.w *= b.w; }
__device__ __forceinline__ void muleq4s(vr4& a, float b) { a.x *= b; a.y *= b; a.z *= b; }
__device__ __forceinline__ float dot4(vr4 a, vr4 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ vr4 cross4(vr4 a, vr4 b) {
    return mk4(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x, 0.0f);
}
__device__ __forceinline__ vr4 normalize4(vr4 a) { const float inv = 1.0f / __builtin_sqrtf(dot4(a, a)); return mul4s(a, inv); }
__device__ __forceinline__ float clampi(int v, int lo, int hi) { const int m = hi < v ? hi : v; return (float)(lo > m ? lo : m); }
__device__ __forceinline__ float clampf(float v, float lo, float hi) { return __builtin_fmaxf(lo, __builtin_fminf(hi, v)); }
__device__ __forceinline__ vr4 tbn_mul(vr4 m0, vr4 m1, vr4 m2, vr4 b) {   // mat4 * float4, m3 = (0,0,0,1)
    return mk4(m0.x * b.x + m1.x * b.y + m2.x * b.z + 0.0f * b.w,
               m0.y * b.x + m1.y * b.y + m2.y * b.z + 0.0f * b.w,
               m0.z * b.x + m1.z * b.y + m2.z * b.z + 0.0f * b.w,
               m0.w * b.x + m1.w * b.y + m2.w * b.z + 1.0f * b.w);
}

// Kepler span helpers on integer bit patterns (MathHelpers.cuh:454-552):
// v_min/v_max_f32 per axis, then v_max3/v_min3_i32 on the bits.
__device__ __forceinline__ float span_begin(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    const int zc = max(min(__float_as_int(c0), __float_as_int(c1)), __float_as_int(d));
    return __int_as_float(max(max(__float_as_int(__builtin_fminf(a0, a1)), __float_as_int(__builtin_fminf(b0, b1))), zc));
}
__device__ __forceinline__ float span_end(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    const int zc = min(max(__float_as_int(c0), __float_as_int(c1)), __float_as_int(d));
    return __int_as_float(min(min(__float_as_int(__builtin_fmaxf(a0, a1)), __float_as_int(__builtin_fmaxf(b0, b1))), zc));
}

// ---- scene constants (PathTracer.cu:107-123)
struct Sph { float r, px, py, pz, ex, ey, ez, cr, cg, cb; int refl; };
__device__ __forceinline__ Sph cornell_sphere(int i) {
    switch (i) {
    case 0: return { 160.f, 0.f, 160.f + 49.f, 0.f, 4.f, 3.6f, 3.2f, 0.f, 0.f, 0.f, 1 };
    case 1: return { 1e5f, 1e5f + 50.f, 0.f, 0.f, 0.075f, 0.025f, 0.025f, 0.75f, 0.25f, 0.25f, 1 };
    case 2: return { 1e5f, -1e5f - 50.f, 0.f, 0.f, 0.025f, 0.075f, 0.025f, 0.25f, 0.75f, 0.25f, 1 };
    case 3: return { 1e5f, 0.f, 0.f, -1e5f - 100.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1 };
    case 4: return { 1e5f, 0.f, 1e5f + 50.f, 0.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1 };
    default: return { 1e5f, 0.f, -1e5f - 50.f, 0.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1 };
    }
}
__device__ __forceinline__ Sph small_sphere(int i) {
    if (i == 0) return { 3.5f, 15.f, 0.f, 15.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0 };   // mirror
    return { 3.5f, 25.f, 0.f, 15.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1 };             // grey, Fresnel
}
__device__ __forceinline__ Sph example_sphere() { return { 10.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1 }; }

struct Ray { vr4 o, d; };

// Sphere::intersect (PathTracer.cu:87-104)
__device__ __forceinline__ float sphere_intersect(const Sph& s, const Ray& r) {
    const vr4 op = sub4(mk4(s.px, s.py, s.pz, 0.f), r.o);
    const float eps = (float)1e-4;
    const float b = dot4(op, r.d);
    float det = b * b - dot4(op, op) + s.r * s.r;
    if (det < 0) return 0;
    det = __builtin_sqrtf(det);
    float t;
    return (t = b - det) > eps ? t : ((t = b + det) > eps ? t : 0.0f);
}

enum HitKind { HK_NONE = 0, HK_CORNELL = 1, HK_SMALL = 2, HK_EXAMPLE = 3, HK_MESH = 4 };
struct HitRec {
    float t;
    int kind, idx;          // sphere index or triangle slot
    float bu, bv;           // barycentrics for mesh hits
    float su, sv;           // example sphere texture coords (from the stale normal)
};
// Per-lane event counts for the counting variant (algorithmic bytes).
struct Cnt {
    uint32_t rays = 0, nodes = 0, slots = 0, tris = 0, attr = 0, tex = 0, hdr = 0, brdf = 0;
#ifdef VR_TIMING
    // diagnostic build only: per-lane s_memtime cycles in spheres, mesh
    // traversal, hit materialisation, shading, tonemap, whole kernel
    uint64_t tm[6] = { 0, 0, 0, 0, 0, 0 };
#endif
};
#ifdef VR_TIMING
#define VR_T0(name) const uint64_t name = __builtin_amdgcn_s_memtime()
#define VR_T1(name, slot) cnt.tm[slot] += __builtin_amdgcn_s_memtime() - name
#else
#define VR_T0(name) (void)0
#define VR_T1(name, slot) (void)0
#endif

struct Hit {                // vHitData, PathTracer.cuh:17-53
    vr4 hp, n, tan, em, col, spec;
    unsigned type;
};

__device__ __forceinline__ int tex_addr(uint32_t w, uint32_t h, float u, float v) {
    const int x = f2i((float)w * u);
    const int y = f2i((float)h * v);
    const int val = (int)((uint32_t)x + (uint32_t)y * w);
    return (int)clampi(val, 0, (int)(w * h - 1u));
}

// Normal of a sphere hit (the value the reference leaves in m_normal).
__device__ __forceinline__ vr4 sphere_normal(const HitRec& hr, const Ray& r) {
    const Sph s = hr.kind == HK_CORNELL ? cornell_sphere(hr.idx) : small_sphere(hr.idx);
    const vr4 hp = add4(r.o, mul4s(r.d, hr.t));
    return normalize4(sub4(hp, mk4(s.px, s.py, s.pz, 0.f)));
}

// Device mesh layout (built from the reference layout at upload, vrhip_api.cpp):
//   nodes: the reference's 4 x float4 per inner node, except that a leaf
//          child is ~((first_tri << 7) | tri_count) into the compact arrays;
//   tris:  3 float4 vertex positions per triangle, leaves contiguous, in the
//          reference's slot order (no terminator slots);
//   attributes (normals, tangents, uvs): same indexing, fetched only for the
//          final hit of a ray.
// The triangles tested and their order are those of the reference layout, so
// the closest hit (ties included) is unchanged.
constexpr int kLeafCountBits = 7;

// Per-block LDS: the traversal stacks (entry-major, one column per thread)
// and a copy of the first nodes of the area-ordered node array (rows 0-2 and
// the two child indices, 56 B per node).  The node cache takes what is left
// of a 40 KB budget, so four blocks (16 waves) still fit a CU's 160 KB.
#ifndef VR_LDS_BUDGET
#define VR_LDS_BUDGET (40960 - 256)
#endif
constexpr int kLdsBudget = VR_LDS_BUDGET;
constexpr int cache_nodes(int stack) { return (kLdsBudget - stack * kBlockThreads * 4) / 56 > 0 ?
                                              (kLdsBudget - stack * kBlockThreads * 4) / 56 : 1; }
// Raw buffer loads for the node and triangle arrays: a 32-bit lane offset
// against an SGPR descriptor (bounds-checked, no 64-bit address math), and an
// explicit width per fetch (16 B node rows, 8 B child indices, 12 B vertices).
typedef unsigned int vr_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int vr_u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int vr_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ vr4 buf_load4(__amdgpu_buffer_rsrc_t b, int off) {
    const vr_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(b, off, 0, 0);
    return mk4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ vr3 buf_load3(__amdgpu_buffer_rsrc_t b, int off) {
    const vr_u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(b, off, 0, 0);
    return vr3{ __uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z) };
}
__device__ __forceinline__ int2 buf_load2i(__amdgpu_buffer_rsrc_t b, int off) {
    const vr_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(b, off, 0, 0);
    return make_int2((int)v.x, (int)v.y);
}

struct Lds {
    int* stk;                 // this thread's column of the stack
    const vr4* nodes;         // 3 rows per cached node
    const int2* idx;          // child indices per cached node
    int n_cached;             // nodes [0, n_cached) are read from LDS
};

template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ void traverse_mesh(const RenderParams& p, const Ray& r, HitRec& hr, const Lds& L, Cnt& cnt)
{
    int* stk = L.stk;
    const __amdgpu_buffer_rsrc_t nbuf = buf_rsrc(p.bvh, p.n_nodes * 64u);
    const __amdgpu_buffer_rsrc_t tbuf = buf_rsrc(p.verts, p.n_tris * 36u);
    // CudaTracerLib-style while-while traversal (PathTracer.cu:276-463)
    const int Sentinel = 0x76543210;
    int sp = 0;
    stk[0] = Sentinel;
    int leafAddr = 0;
    int nodeAddr = 0;
    const float ivx = 1.f / (__builtin_fabsf(r.d.x) > VR_EPS ? r.d.x : VR_EPS);
    const float ivy = 1.f / (__builtin_fabsf(r.d.y) > VR_EPS ? r.d.y : VR_EPS);
    const float ivz = 1.f / (__builtin_fabsf(r.d.z) > VR_EPS ? r.d.z : VR_EPS);
    const float odx = r.o.x * ivx, ody = r.o.y * ivy, odz = r.o.z * ivz;
    float t = hr.t;
    // t-culling: a child whose slab entry lies beyond the closest hit so far
    // (times a 2^-10 safety margin) cannot hold a closer triangle.  The
    // reference visits every pierced box (span end clamped to 1e20,
    // :316,322); F_STRICT restores that exactly.
    const bool strict = HAS(F_STRICT);   // compile-time false in the specialised kernels
    const float kCull = 1.0009765625f;
    float tcull = strict ? __builtin_inff() : t * kCull;
    int best = -1;
    float bu = 0.f, bv = 0.f;

    while (nodeAddr != Sentinel) {
        while ((unsigned)nodeAddr < (unsigned)Sentinel) {
            if (COUNT) cnt.nodes++;
            vr4 n0, n1, nz;
            int2 ni;
            const int node = nodeAddr >> 2;
#if defined(VR_LDS_FIRST)
            // every lane reads LDS (uncached lanes read node 0), then the
            // uncached lanes alone overwrite from HBM/L2
            const bool cached = node < L.n_cached;
            const int ln = cached ? node : 0;
            n0 = L.nodes[3 * ln + 0];
            n1 = L.nodes[3 * ln + 1];
            nz = L.nodes[3 * ln + 2];
            ni = L.idx[ln];
            if (!cached) {
#else
            // wave-uniform choice: a diverged wave would pay both round trips
#ifdef VR_LANE_CACHE
            if (node < L.n_cached) {
#else
            if (__ballot(node >= L.n_cached) == 0ull) {
#endif
                n0 = L.nodes[3 * node + 0];
                n1 = L.nodes[3 * node + 1];
                nz = L.nodes[3 * node + 2];
                ni = L.idx[node];
            } else {
#endif
                const int off = nodeAddr * 16;                    // byte offset of the node
                n0 = buf_load4(nbuf, off);
                n1 = buf_load4(nbuf, off + 16);
                nz = buf_load4(nbuf, off + 32);
                ni = buf_load2i(nbuf, off + 48);                  // 8 of the row's 16 bytes are used
            }
            const int idx0 = ni.x, idx1 = ni.y;
            // slab distances n*inv - o*inv (:307-322); the culled mode lets
            // them contract to one v_fma each (more accurate)
            auto slab = [&](float n, float iv, float od) {
                return strict ? (n * iv - od) : __builtin_fmaf(n, iv, -od);
            };
            const float c0lox = slab(n0.x, ivx, odx);
            const float c0hix = slab(n0.y, ivx, odx);
            const float c0loy = slab(n0.z, ivy, ody);
            const float c0hiy = slab(n0.w, ivy, ody);
            const float c0loz = slab(nz.x, ivz, odz);
            const float c0hiz = slab(nz.y, ivz, odz);
            const float c1loz = slab(nz.z, ivz, odz);
            const float c1hiz = slab(nz.w, ivz, odz);
            const float c0min = span_begin(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 0.0f);
            const float c0max = span_end(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 1e20f);
            const float c1lox = slab(n1.x, ivx, odx);
            const float c1hix = slab(n1.y, ivx, odx);
            const float c1loy = slab(n1.z, ivy, ody);
            const float c1hiy = slab(n1.w, ivy, ody);
            const float c1min = span_begin(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, 0.0f);
            const float c1max = span_end(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, 1e20f);
            // keep the child-index load in the same round trip as the bounds
            asm volatile("" ::"v"(idx0), "v"(idx1));
            const bool swp = (c1min < c0min);
            const bool tc0 = (c0max >= c0min) && (c0min <= tcull);
            const bool tc1 = (c1max >= c1min) && (c1min <= tcull);
            // branch-free push/pop: near child next, far child pushed when both
            // are hit, pop when neither is (same order as :324-343)
            const bool both = tc0 && tc1;
            const bool none = !tc0 && !tc1;
            const int top = stk[sp * kBlockThreads];
            const int nearc = (both && swp) ? idx1 : (tc0 ? idx0 : idx1);
            const int farc = swp ? idx0 : idx1;
            if (both) stk[(sp + 1) * kBlockThreads] = farc;
            sp += both ? 1 : (none ? -1 : 0);
            nodeAddr = none ? top : nearc;
            if (nodeAddr < 0 && leafAddr >= 0) {                 // postpone max 1
                leafAddr = nodeAddr;
                nodeAddr = stk[sp * kBlockThreads];
                --sp;
            }
            if (__ballot(leafAddr >= 0) == 0ull) break;          // every lane holds a leaf
        }
        while (leafAddr < 0) {
            const int lv = ~leafAddr;
            const int kend = (lv >> kLeafCountBits) + (lv & ((1 << kLeafCountBits) - 1));
            for (int k = lv >> kLeafCountBits; k < kend; ++k) {
                const int triAddr = 3 * k;
                if (COUNT) cnt.tris++;
                const int toff = k * 36;
                const vr3 a0 = buf_load3(tbuf, toff), a1 = buf_load3(tbuf, toff + 12), a2 = buf_load3(tbuf, toff + 24);
                asm volatile("" ::"v"(a0.x), "v"(a1.x), "v"(a2.x));   // three dwordx3 loads, one trip
                const vr4 v0 = mk4(a0.x, a0.y, a0.z, 0.f);
                const vr4 v1 = mk4(a1.x, a1.y, a1.z, 0.f);
                const vr4 v2 = mk4(a2.x, a2.y, a2.z, 0.f);
                // intersectTriangle, RayIntersection.cuh:54-111, evaluated
                // branch-free: every early return of the reference becomes a
                // term of the final predicate (the values computed for a
                // surviving triangle are the same operations in the same order)
                const vr4 e1 = sub4(v1, v0), e2 = sub4(v2, v0);
                const vr4 pv = cross4(r.d, e2);
                const float det = dot4(e1, pv);
                const float inv_det = 1.f / det;
                const vr4 tv = sub4(r.o, v0);
                const float u = dot4(tv, pv) * inv_det;
                const vr4 q = cross4(tv, e1);
                const float v = dot4(r.d, q) * inv_det;
                const float dist = dot4(e2, q) * inv_det;
                const bool ok = !(det > -VR_EPS && det < VR_EPS) && !(u < 0.f || u > 1.f) &&
                                !(v < 0.f || u + v > 1.f);
                if (ok && dist > VR_EPS && dist < t) {
                    t = dist; best = triAddr; bu = u; bv = v;
                    tcull = strict ? tcull : t * kCull;
                }
            }
            leafAddr = nodeAddr;
            if (nodeAddr < 0) {
                nodeAddr = stk[sp * kBlockThreads];
                --sp;
            }
        }
    }
    if (best >= 0) { hr.t = t; hr.kind = HK_MESH; hr.idx = best; hr.bu = bu; hr.bv = bv; }
}

// intersectScene (PathTracer.cu:136-468): closest hit, attributes deferred.
template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool intersect_scene(const RenderParams& p, const Ray& r, HitRec& hr, const Lds& L, Cnt& cnt)
{
    if (COUNT) cnt.rays++;
    VR_T0(t_sph);
    hr.t = 1e20f; hr.kind = HK_NONE; hr.idx = 0; hr.bu = hr.bv = 0.f; hr.su = hr.sv = 0.f;
    if HAS(F_CORNELL) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const float dist = sphere_intersect(cornell_sphere(i), r);
            if (dist != 0.f && dist < hr.t) { hr.t = dist; hr.kind = HK_CORNELL; hr.idx = i; }
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float dist = sphere_intersect(small_sphere(i), r);
        if (dist != 0.f && dist < hr.t) { hr.t = dist; hr.kind = HK_SMALL; hr.idx = i; }
    }
    if HAS(F_EXAMPLE) {
        const float dist = sphere_intersect(example_sphere(), r);
        if (dist != 0.f && dist < hr.t) {
            if (HAS(F_TEX_DIFF) || HAS(F_TEX_NORM) || HAS(F_TEX_SPEC)) {
                // u,v from the normal left by the previous hit of this call (:202-204)
                const vr4 sn = hr.kind == HK_NONE ? mk4(0.f, 0.f, 0.f, 0.f) : sphere_normal(hr, r);
                hr.su = atan2_p(sn.x, sn.z) / (2.f * VR_PI) + 0.5f;
                hr.sv = sn.y * 0.5f + 0.5f;
            }
            hr.t = dist; hr.kind = HK_EXAMPLE; hr.idx = 0;
        }
    } else if HAS(F_MESH) {
        VR_T1(t_sph, 0);
        VR_T0(t_mesh);
        traverse_mesh<STACK, COUNT, FEAT>(p, r, hr, L, cnt);
        VR_T1(t_mesh, 1);
        return hr.t < 1e20f;
    }
    VR_T1(t_sph, 0);
    return hr.t < 1e20f;
}

// Materialise vHitData for the final hit (the values the reference's last
// accepted hit wrote; :160-168, :180-189, :198-266, :380-453).
template <uint32_t FEAT>
__device__ __forceinline__ void fill_hit(const RenderParams& p, const Ray& r, const HitRec& hr, Hit& h)
{
    h.tan = mk4(0.f, 0.f, 0.f, 0.f);
    const bool view_brdf = HAS(F_VIEW_BRDF);
    if (hr.kind == HK_CORNELL || hr.kind == HK_SMALL) {
        const Sph s = hr.kind == HK_CORNELL ? cornell_sphere(hr.idx) : small_sphere(hr.idx);
        h.hp = add4(r.o, mul4s(r.d, hr.t));
        h.n = normalize4(sub4(h.hp, mk4(s.px, s.py, s.pz, 0.f)));
        h.col = mk4(s.cr, s.cg, s.cb, 0.f);
        h.em = mk4(s.ex, s.ey, s.ez, 0.f);
        h.type = (unsigned)s.refl;
        h.spec = hr.kind == HK_CORNELL ? mk4(0.f, 0.f, 0.f, 0.f) : mk4(1.f, 1.f, 1.f, 0.f);
    } else if (hr.kind == HK_EXAMPLE) {
        const Sph s = example_sphere();
        h.hp = add4(r.o, mul4s(r.d, hr.t));
        if (HAS(F_TEX_DIFF) && !view_brdf)
            h.col = p.tex[0][tex_addr(p.tex_w[0], p.tex_h[0], hr.su, hr.sv)];
        else
            h.col = mk4(s.cr, s.cg, s.cb, 0.f);
        if HAS(F_TEX_NORM) {
            const int a = tex_addr(p.tex_w[1], p.tex_h[1], hr.su, hr.sv);
            vr4 normal = normalize4(sub4(h.hp, mk4(s.px, s.py, s.pz, 0.f)));
            normal.w = 0.f;
            const float rr = __builtin_sqrtf(dot4(h.hp, h.hp));
            const float theta = acos_p(h.hp.z / rr);
            const float phi = atan2_p(h.hp.y, h.hp.x);
            float st, ct, sph, cph;
            sincos_p(theta, &st, &ct);
            sincos_p(phi, &sph, &cph);
            h.tan = mk4(st * cph, st * sph, ct, 0.f);
            const vr4 bitangent = cross4(normal, h.tan);
            const vr4 nm = normalize4(sub4(muls4(2.f, p.tex[1][a]), mk4(1.f, 1.f, 1.f, 0.f)));
            h.n = normalize4(tbn_mul(h.tan, bitangent, normal, nm));
        } else {
            h.n = normalize4(sub4(h.hp, mk4(s.px, s.py, s.pz, 0.f)));
        }
        if (HAS(F_TEX_SPEC) && !view_brdf)
            h.spec = p.tex[2][tex_addr(p.tex_w[2], p.tex_h[2], hr.su, hr.sv)];
        else
            h.spec = mk4(0.f, 0.f, 0.f, 0.f);
        h.em = mk4(0.f, 0.f, 0.f, 0.f);
        h.type = view_brdf ? 2u : 1u;
    } else {   // HK_MESH
        const int a = hr.idx;
        h.hp = add4(r.o, mul4s(r.d, hr.t));
        const float b0 = 1.f - hr.bu - hr.bv;
        const vr2 uv0 = p.uvs[a], uv1 = p.uvs[a + 1], uv2 = p.uvs[a + 2];
        const float uvx = (b0 * uv0.x + hr.bu * uv1.x) + hr.bv * uv2.x;
        const float uvy = (b0 * uv0.y + hr.bu * uv1.y) + hr.bv * uv2.y;
        vr4 tangent = normalize4(add4(add4(muls4(b0, p.tangents[a]), muls4(hr.bu, p.tangents[a + 1])),
                                      muls4(hr.bv, p.tangents[a + 2])));
        tangent.w = 0.f;
        if (HAS(F_TEX_DIFF) && !view_brdf)
            h.col = p.tex[0][tex_addr(p.tex_w[0], p.tex_h[0], uvx, uvy)];
        else
            h.col = mk4(1.f, 1.f, 1.f, 0.f);
        if (HAS(F_TEX_NORM) && dot4(tangent, tangent) > VR_EPS) {
            const int ta = tex_addr(p.tex_w[1], p.tex_h[1], uvx, uvy);
            vr4 normal = normalize4(add4(add4(muls4(b0, p.normals[a]), muls4(hr.bu, p.normals[a + 1])),
                                         muls4(hr.bv, p.normals[a + 2])));
            normal.w = 0.f;
            const vr4 bitangent = cross4(normal, tangent);
            const vr4 nm = normalize4(sub4(muls4(2.f, p.tex[1][ta]), mk4(1.f, 1.f, 1.f, 0.f)));
            h.n = normalize4(tbn_mul(tangent, bitangent, normal, nm));
        } else {
            const vr3 a0 = p.verts[a], a1 = p.verts[a + 1], a2 = p.verts[a + 2];
            const vr4 v0 = mk4(a0.x, a0.y, a0.z, 0.f), v1 = mk4(a1.x, a1.y, a1.z, 0.f), v2 = mk4(a2.x, a2.y, a2.z, 0.f);
            h.n = normalize4(cross4(sub4(v0, v1), sub4(v0, v2)));
        }
        if (HAS(F_TEX_SPEC) && !view_brdf)
            h.spec = p.tex[2][tex_addr(p.tex_w[2], p.tex_h[2], uvx, uvy)];
        else
            h.spec = mk4(0.f, 0.f, 0.f, 0.f);
        h.tan = tangent;
        h.em = mk4(0.f, 0.f, 0.f, 0.f);
        h.type = view_brdf ? 2u : 1u;
    }
}

// Emission of a hit (the only vHitData field the last bounce observes).
__device__ __forceinline__ vr4 emission_of(const HitRec& hr) {
    if (hr.kind == HK_CORNELL || hr.kind == HK_SMALL) {
        const Sph s = hr.kind == HK_CORNELL ? cornell_sphere(hr.idx) : small_sphere(hr.idx);
        return mk4(s.ex, s.ey, s.ez, 0.f);
    }
    return mk4(0.f, 0.f, 0.f, 0.f);
}

// MERL index maps (PathTracer.cu:473-506)
__device__ __forceinline__ int phi_diff_index(float phi_diff) {
    if (phi_diff < 0.0) phi_diff = (float)((double)phi_diff + 3.14159265358979323846);
    return (int)clampi(d2i((double)phi_diff * (1.0 / (double)VR_PI * (360 / 2))), 0, 360 / 2 - 1);
}
__device__ __forceinline__ int theta_half_index(float theta_half) {
    if (theta_half <= 0.0) return 0;
    const float s = __builtin_sqrtf((float)((double)theta_half * (2.0 / (double)VR_PI)));
    return (int)clampi(f2i(s * 90), 0, 90 - 1);
}
__device__ __forceinline__ int theta_diff_index(float theta_diff) {
    return (int)clampi(d2i((double)theta_diff * (2.0 / (double)VR_PI * 90)), 0, 90 - 1);
}

// lookupBRDF (PathTracer.cu:519-566)
__device__ __forceinline__ vr4 lookup_brdf(const float* __restrict__ T, vr4 refl, vr4 cur, vr4 normal, vr4 tangent) {
    const vr4 bitangent = cross4(normal, tangent);
    const vr4 H = normalize4(sub4(refl, cur));
    float theta_H = acos_p(clampf(dot4(normal, H), 0.f, 1.f));
    const float theta_diff = acos_p(clampf(dot4(H, refl), 0.f, 1.f));
    float phi_diff = 0.f;
    if ((double)theta_diff < 1e-3) {
        phi_diff = atan2_p(clampf(-dot4(refl, bitangent), -1.f, 1.f), clampf(dot4(refl, tangent), -1.f, 1.f));
    } else if ((double)theta_H > 1e-3) {
        const vr4 u = muls4(-1.f, normalize4(sub4(normal, muls4(dot4(normal, H), H))));
        const vr4 v = cross4(H, u);
        phi_diff = atan2_p(clampf(dot4(refl, v), -1.f, 1.f), clampf(dot4(refl, u), -1.f, 1.f));
    } else {
        theta_H = 0.f;
    }
    const int ind = phi_diff_index(phi_diff) + theta_diff_index(theta_diff) * 360 / 2
                    + theta_half_index(theta_H) * 360 / 2 * 90;
    return mk4((float)((double)T[ind] * (1.0 / 1500.0)),
               (float)((double)T[ind + 1458000] * (1.15 / 1500.0)),
               (float)((double)T[ind + 2916000] * (1.66 / 1500.0)), 0.f);
}

// thrust::minstd_rand + uniform_real_distribution<float>(0,1) (rocThrust
// random/detail/{linear_congruential_engine.inl,mod.h,uniform_real_distribution.inl})
struct Rng {
    uint32_t x;
    __device__ __forceinline__ void seed(uint32_t s) {
        uint32_t v = s >= 2147483647u ? s - 2147483647u : s;    // s % (2^31-1) for s < 2^32
        v = v >= 2147483647u ? v - 2147483647u : v;
        x = v ? v : 1u;
    }
    __device__ __forceinline__ float uniform() {
        const uint64_t prod = (uint64_t)x * 48271u;             // Mersenne-prime reduction
        uint32_t r = (uint32_t)(prod & 0x7fffffffu) + (uint32_t)(prod >> 31);
        r = r >= 2147483647u ? r - 2147483647u : r;
        x = r;
        return (float)(r - 1u) * 4.656612873077392578125e-10f;  // / 2^31 (exact)
    }
};

__device__ __forceinline__ uint32_t hash_seeds(uint32_t& s0, uint32_t& s1) {   // PathTracer.cu:574-580
    s0 = 36969u * (s0 & 65535u) + (s0 >> 16);
    s1 = 18000u * (s1 & 65535u) + (s1 >> 16);
    return s0 * s1;
}

// trace (PathTracer.cu:597-770)
template <int STACK, bool COUNT, uint32_t FEAT>
__device__ vr4 trace(const RenderParams& p, Ray ray, const HitRec& hr0, bool hit0, uint32_t& s0, uint32_t& s1,
                     const Lds& L, Cnt& cnt)
{
    vr4 accum = mk4(0.f, 0.f, 0.f, 0.f);
    vr4 mask = mk4(1.f, 1.f, 1.f, 0.f);
    float depth = 1.f;
    Rng rng;
    rng.seed(hash_seeds(s0, s1));

    for (unsigned bounces = 0; bounces < 4; bounces++) {
        HitRec hr;
        bool hit;
        if (!COUNT && bounces == 0) {
            // the camera ray is the same for both samples of every frame (no
            // jitter, PathTracer.cu:842-844): its hit is computed once per pixel
            hr = hr0;
            hit = hit0;
        } else {
            hit = intersect_scene<STACK, COUNT, FEAT>(p, ray, hr, L, cnt);
        }
        if (!hit) {
            if (!HAS(F_CORNELL)) {                                    // :631-648
                float lx = atan2_p(ray.d.x, ray.d.z);
                float ly = acos_p(ray.d.y);
                lx = lx < 0 ? (float)((double)lx + 2.0 * (double)VR_PI) : lx;
                lx = (float)((double)lx / (2.0 * (double)VR_PI));
                ly = ly / VR_PI;
                const int x = f2i(lx * (float)p.hdr_w);
                const int y = f2i(ly * (float)p.hdr_h);
                const int val = (int)((uint32_t)x + (uint32_t)y * p.hdr_w);
                const int addr = (int)clampi(val, 0, (int)(p.hdr_w * p.hdr_h - 1u));
                if (COUNT) cnt.hdr++;
                accum = add4(accum, mul4(mul4s(mask, 2.f), p.hdr[addr]));
                accum.w = depth;
                return accum;
            }
            return mk4(0.f, 0.f, 0.f, 0.f);
        }
        if (!COUNT && bounces == 3) {
            // last bounce: only the emission term is observable; the material
            // branch below would only prepare a ray that is never traced
            accum = add4(accum, mul4(mask, emission_of(hr)));
            break;
        }
        Hit h;
        VR_T0(t_fill);
        fill_hit<FEAT>(p, ray, hr, h);
        VR_T1(t_fill, 2);
        if (COUNT) {
            if (hr.kind == HK_MESH) {
                cnt.attr += 24 + 48;
                const bool vb = HAS(F_VIEW_BRDF);
                cnt.tex += (HAS(F_TEX_DIFF) && !vb) + (HAS(F_TEX_SPEC) && !vb);
                if (HAS(F_TEX_NORM) && dot4(h.tan, h.tan) > VR_EPS) { cnt.attr += 48; cnt.tex++; }
            } else if (hr.kind == HK_EXAMPLE) {
                const bool vb = HAS(F_VIEW_BRDF);
                cnt.tex += (HAS(F_TEX_DIFF) && !vb) + (HAS(F_TEX_SPEC) && !vb) + (HAS(F_TEX_NORM) != 0);
            }
        }
        if (bounces == 0) {
            const vr4 l = sub4(ray.o, h.hp);
            depth = __builtin_sqrtf(dot4(l, l)) / 150.f;
        }
        accum = add4(accum, mul4(mask, h.em));
        ray.o = h.hp;
        const vr4 normal = h.n;
        VR_T0(t_shade);
        if (h.type == 0) {                                                   // :671-676
            ray.d = sub4(ray.d, mul4s(mul4s(normal, 2.f), dot4(normal, ray.d)));
            ray.o = add4(ray.o, mul4s(normal, 0.05f));
        } else if (h.type == 1) {                                            // :678-722
            const float aoi = dot4(h.n, muls4(-1.f, ray.d));
            // powf only matters when spec.x != 0: X * 0 == 0 for finite X and
            // NaN * 0 compares false, so u < fe is false either way.
            float fe = 0.f;
            if (h.spec.x != 0.f)
                fe = ((1.f - p.fresnel_coef) * pow_p(1.f - aoi, p.fresnel_pow) + p.fresnel_coef * 1.f) * h.spec.x;
            const bool reflect = (rng.uniform() < fe);
            vr4 newdir;
            const vr4 w = normal;
            const vr4 axis = __builtin_fabsf(w.x) > 0.1f ? mk4(0.f, 1.f, 0.f, 0.f) : mk4(1.f, 0.f, 0.f, 0.f);
            if (reflect) {
                muleq4(mask, h.spec);
                newdir = normalize4(sub4(ray.d, mul4s(mul4s(normal, 2.f), dot4(normal, ray.d))));
            } else {
                const float rand1 = 2.f * VR_PI * rng.uniform();
                const float rand2 = rng.uniform();
                const float rand2s = __builtin_sqrtf(rand2);
                const vr4 u = normalize4(cross4(axis, w));
                const vr4 v = cross4(w, u);
                float sn, cs;
                sincos_p(rand1, &sn, &cs);
                newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                         mul4s(w, __builtin_sqrtf(1 - rand2))));
                muleq4(mask, h.col);
                muleq4s(mask, dot4(newdir, normal));
                muleq4s(mask, 2.f);
            }
            ray.o = add4(ray.o, mul4s(normal, 0.05f));
            ray.d = newdir;
        } else if (h.type == 2) {                                            // :724-764
            const vr4 w = normal;
            const vr4 axis = __builtin_fabsf(w.x) > 0.1f ? mk4(0.f, 1.f, 0.f, 0.f) : mk4(1.f, 0.f, 0.f, 0.f);
            const float rand1 = 2.f * VR_PI * rng.uniform();
            const float rand2 = rng.uniform();
            const float rand2s = __builtin_sqrtf(rand2);
            const vr4 u = normalize4(cross4(axis, w));
            const vr4 v = cross4(w, u);
            float sn, cs;
            sincos_p(rand1, &sn, &cs);
            const vr4 newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                               mul4s(w, __builtin_sqrtf(1 - rand2))));
            if HAS(F_BRDF) {
                const float dw = 24 * pow_p(newdir.x * newdir.x + newdir.y * newdir.y + newdir.z * newdir.z, -1.5f);
                if (COUNT) cnt.brdf++;
                const vr4 b = lookup_brdf(p.brdf, newdir, ray.d, h.n, h.tan);
                const vr4 bm = mk4(__builtin_fmaxf(b.x, 0.f), __builtin_fmaxf(b.y, 0.f), __builtin_fmaxf(b.z, 0.f),
                                   __builtin_fmaxf(b.w, 0.f));
                muleq4(mask, muls4(dw, bm));
            } else {
                muleq4(mask, h.col);
                muleq4s(mask, dot4(newdir, normal));
                muleq4s(mask, 2.f);
            }
            ray.o = add4(ray.o, mul4s(normal, 0.05f));
            ray.d = newdir;
        }
        VR_T1(t_shade, 3);
    }
    accum.w = depth;
    return accum;
}

// colour of the accumulated radiance after `frame` frames (PathTracer.cu:850-866)
__device__ __forceinline__ u8x4 tonemap(vr4 io, uint32_t frame) {
    const float coef = 1.f / (float)frame;
    const vr4 sc = mul4s(io, coef);
    const float inv_gamma = 1.f / 2.2f;
    u8x4 c;
    c.x = f2u8(pow_p(clampf(sc.x, 0.f, 1.f), inv_gamma) * 255);
    c.y = f2u8(pow_p(clampf(sc.y, 0.f, 1.f), inv_gamma) * 255);
    c.z = f2u8(pow_p(clampf(sc.z, 0.f, 1.f), inv_gamma) * 255);
    c.w = 0xff;
    return c;
}

// Split launches: sums each pixel's path results in path order (the same
// float4 operations, in the same order, as the unsplit kernel), then writes
// the accumulation, colour and depth.
__global__ void __launch_bounds__(kBlockThreads) finish_kernel(const RenderParams p)
{
    const uint32_t tile = blockIdx.x, tid = threadIdx.x;
    const int wave = (int)tid >> 6, lane = (int)tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;      // tiles dealt round-robin to ranks
    const uint32_t tile_y = gtile / p.tiles_x;
    const uint32_t tile_x = gtile - tile_y * p.tiles_x;
    const uint32_t x = tile_x * 16u + (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t y = tile_y * 16u + (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    if (x >= p.wr || y >= p.hr) return;
    const uint32_t ind = x + y * p.W;
    vr4 io = p.first_frame != 1u ? p.accum[ind] : mk4(0.f, 0.f, 0.f, 0.f);
    const uint32_t n_paths = 2u * p.n_frames;
    const vr4* src = p.paths + (size_t)tile * kBlockThreads + tid;
    vr4 result = mk4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t q = 0; q < n_paths; ++q) {
        result = src[(size_t)q * p.path_stride];
        io = add4(io, mul4s(result, 1.f / 2.f));
    }
    const unsigned char db = f2u8((1.f - result.w) * 255);
    u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
    p.depth[ind] = dv;
    p.rgba[ind] = tonemap(io, p.first_frame + p.n_frames - 1u);
    p.accum[ind] = io;
}

// render (PathTracer.cu:791-868), K frames per launch.
#ifndef VR_MIN_WAVES_PER_SIMD
#define VR_MIN_WAVES_PER_SIMD 4
#endif
template <int STACK, bool COUNT, uint32_t FEAT>
__global__ void __launch_bounds__(kBlockThreads, VR_MIN_WAVES_PER_SIMD) render_kernel(const RenderParams p)
{
    constexpr int CN = cache_nodes(STACK);
    __shared__ int lds_stack[STACK * kBlockThreads];
    __shared__ vr4 lds_nodes[3 * CN];
    __shared__ int2 lds_idx[CN];
    const int tid = threadIdx.x;
    Lds L;
    L.stk = lds_stack + tid;
    L.nodes = lds_nodes;
    L.idx = lds_idx;
    L.n_cached = 0;
#ifndef VR_NO_NODE_CACHE
    if (HAS(F_MESH)) {
        L.n_cached = (int)(p.n_nodes < (uint32_t)CN ? p.n_nodes : (uint32_t)CN);
        for (int i = tid; i < 3 * L.n_cached; i += kBlockThreads) lds_nodes[i] = p.bvh[(i / 3) * 4 + i % 3];
        for (int i = tid; i < L.n_cached; i += kBlockThreads)
            lds_idx[i] = *reinterpret_cast<const int2*>(p.bvh + 4 * i + 3);
        __syncthreads();
    }
#endif
    // block -> (tile, path group): the 2*n_frames paths of a pixel are split
    // into p.split contiguous groups run by different blocks (strong-scaling
    // and tail balance); group g of tile t is block t*split + g
    const uint32_t T = p.split;
    const uint32_t tile = blockIdx.x / T;
    const uint32_t g = blockIdx.x - tile * T;
    const int wave = tid >> 6, lane = tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;      // tiles dealt round-robin to ranks
    const uint32_t tile_y = gtile / p.tiles_x;
    const uint32_t tile_x = gtile - tile_y * p.tiles_x;
    const uint32_t x = tile_x * 16u + (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t y = tile_y * 16u + (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    if (x >= p.wr || y >= p.hr) return;   // never true for a valid launch
    Cnt cnt;
    VR_T0(t_kernel);

    const uint32_t ind = x + y * p.W;
    const float sx = (float)((0.25 + (double)x) / (double)p.W - 0.5);   // :842
    const float sy = (float)((0.25 + (double)y) / (double)p.H - 0.5);
    Ray cam;
    cam.o = p.cam_o;
    cam.d = normalize4(add4(add4(p.cam_d, mul4s(p.cx, sx)), mul4s(p.cy, sy)));
    HitRec hr0;
    bool hit0 = false;
    if (!COUNT) hit0 = intersect_scene<STACK, COUNT, FEAT>(p, cam, hr0, L, cnt);

    // path q = 2*f + s (frame f of the launch, sample s); the seeds of a
    // frame's second sample are its first sample's after one hash (:620-622)
    const uint32_t n_paths = 2u * p.n_frames;
    const uint32_t chunk = (n_paths + T - 1u) / T;
    const uint32_t q0 = g * chunk;
    const uint32_t q1 = q0 + chunk < n_paths ? q0 + chunk : n_paths;
    vr4 io = (T == 1u && p.first_frame != 1u) ? p.accum[ind] : mk4(0.f, 0.f, 0.f, 0.f);
    uint32_t s1 = 0, s2 = 0;
    float last_w = 0.f;
#pragma unroll 1
    for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t f = q >> 1;
        if ((q & 1u) == 0u || q == q0) {
            s1 = x * (p.first_frame + f);
            s2 = y * p.times[f];
            if (q & 1u) (void)hash_seeds(s1, s2);
        }
        const vr4 result = trace<STACK, COUNT, FEAT>(p, cam, hr0, hit0, s1, s2, L, cnt);
        if (T == 1u)
            io = add4(io, mul4s(result, 1.f / 2.f));
        else
            p.paths[(size_t)q * p.path_stride + (size_t)tile * kBlockThreads + tid] = result;
        last_w = result.w;
    }
    if (T != 1u) return;   // finish_kernel accumulates the groups' results in path order
    VR_T0(t_tone);
    // only the launch's last frame is observable in the colour and depth
    // surfaces (each frame of the reference overwrites them, :846-866)
    const unsigned char db = f2u8((1.f - last_w) * 255);
    u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
    p.depth[ind] = dv;
    p.rgba[ind] = tonemap(io, p.first_frame + p.n_frames - 1u);
    p.accum[ind] = io;
    VR_T1(t_tone, 4);
#ifdef VR_TIMING
    VR_T1(t_kernel, 5);
    if (p.counters) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            unsigned long long x = cnt.tm[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (lane == 0) atomicAdd(p.counters + 8 + k, x);
        }
    }
#endif
    if (COUNT) {
        // one wave-level reduction and one 64-bit atomic per counter per wave
        uint32_t v[8] = { cnt.rays, cnt.nodes, cnt.slots, cnt.tris, cnt.attr, cnt.tex, cnt.hdr, cnt.brdf };
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            unsigned long long x = v[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
            if (lane == 0 && x) atomicAdd(p.counters + k, x);
        }
    }
}

// ---- small helper kernels ------------------------------------------------
__global__ void half_to_float_kernel(const uint16_t* __restrict__ src, vr4* __restrict__ dst, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint16_t* s = src + 4 * i;
    dst[i] = mk4(__half2float(__ushort_as_half(s[0])), __half2float(__ushort_as_half(s[1])),
                 __half2float(__ushort_as_half(s[2])), __half2float(__ushort_as_half(s[3])));
}

// Copies this rank's tiles between the full image and a packed buffer: owned
// tile j (global tile rank + j*nranks) occupies packed pixels [256j, 256j+256)
// in row-major order within the tile.
__global__ void pack_tiles_kernel(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t wpp,
                                  uint32_t W, uint32_t tiles_x, uint32_t rank, uint32_t nranks, int unpack)
{
    const uint32_t j = blockIdx.x;
    const uint32_t gt = rank + j * nranks;
    const uint32_t ty = gt / tiles_x, tx = gt - ty * tiles_x;
    for (uint32_t w = threadIdx.x; w < 256u * wpp; w += blockDim.x) {
        const uint32_t px = w / wpp, word = w - px * wpp;
        const size_t full = ((size_t)(ty * 16u + px / 16u) * W + tx * 16u + px % 16u) * wpp + word;
        const size_t packed = ((size_t)j * 256u + px) * wpp + word;
        if (unpack) dst[full] = src[packed];
        else dst[packed] = src[full];
    }
}

__global__ void selftest_math_kernel(int fn, const float* a, const float* b, float* out, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s, c, r = 0.f;
    switch (fn) {
    case 0: sincos_p(a[i], &s, &c); r = s; break;
    case 1: sincos_p(a[i], &s, &c); r = c; break;
    case 2: r = acos_p(a[i]); break;
    case 3: r = atan2_p(a[i], b[i]); break;
    case 4: r = pow_p(a[i], b[i]); break;
    case 5: r = __builtin_fminf(a[i], b[i]); break;
    case 6: r = __builtin_fmaxf(a[i], b[i]); break;
    case 7: r = __int_as_float(f2i(a[i])); break;
    default: r = 0.f;
    }
    out[i] = r;
}

// ---- host launchers --------------------------------------------------------
// Feature specialisations, smallest first (BASELINE configs C1..C5); the
// generic kernel covers everything else, deep trees and the counting variant.
constexpr uint32_t kFeatAll =
    F_CORNELL | F_EXAMPLE | F_VIEW_BRDF | F_MESH | F_BRDF | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC | F_STRICT;
constexpr uint32_t kFeatCornellMesh = F_CORNELL | F_MESH;                                   // C2, Cornell-only
constexpr uint32_t kFeatCornellSphere = F_CORNELL | F_EXAMPLE;                              // C1
constexpr uint32_t kFeatHdriMesh = F_MESH;                                                  // C5
constexpr uint32_t kFeatHdriMeshTex = F_MESH | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC;        // C3
constexpr uint32_t kFeatHdriBrdfSphere = F_EXAMPLE | F_VIEW_BRDF | F_BRDF;                  // C4

template <uint32_t FEAT>
static void launch_spec(const RenderParams& p, uint32_t blocks, int stack_depth, hipStream_t s)
{
#ifndef VR_MIN_SPEC_STACK
#define VR_MIN_SPEC_STACK 16
#endif
    if (stack_depth <= 16 && VR_MIN_SPEC_STACK <= 16)
        hipLaunchKernelGGL((render_kernel<16, false, FEAT>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
    else
        hipLaunchKernelGGL((render_kernel<32, false, FEAT>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
}

int launch_render(const RenderParams& p, uint32_t n_tiles, int stack_depth, bool count, void* stream)
{
    if (n_tiles == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t need = p.flags & kFeatAll;
    auto covers = [need](uint32_t feat) { return (need & ~feat) == 0u; };
    const uint32_t blocks = n_tiles * p.split;   // split == 1 for the counting variant
    if (count || stack_depth > 32) {
        if (count) {
            if (stack_depth <= 32) hipLaunchKernelGGL((render_kernel<32, true, kFeatAll>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
            else hipLaunchKernelGGL((render_kernel<64, true, kFeatAll>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
        } else {
            hipLaunchKernelGGL((render_kernel<64, false, kFeatAll>), dim3(blocks), dim3(kBlockThreads), 0, s, p);
        }
    } else if (covers(kFeatCornellMesh)) {
        launch_spec<kFeatCornellMesh>(p, blocks, stack_depth, s);
    } else if (covers(kFeatCornellSphere)) {
        launch_spec<kFeatCornellSphere>(p, blocks, stack_depth, s);
    } else if (covers(kFeatHdriMesh)) {
        launch_spec<kFeatHdriMesh>(p, blocks, stack_depth, s);
    } else if (covers(kFeatHdriMeshTex)) {
        launch_spec<kFeatHdriMeshTex>(p, blocks, stack_depth, s);
    } else if (covers(kFeatHdriBrdfSphere)) {
        launch_spec<kFeatHdriBrdfSphere>(p, blocks, stack_depth, s);
    } else {
        launch_spec<kFeatAll>(p, blocks, stack_depth, s);
    }
    return (int)hipGetLastError();
}

int launch_finish(const RenderParams& p, uint32_t n_tiles, void* stream)
{
    if (n_tiles == 0 || p.split <= 1u) return 0;
    hipLaunchKernelGGL(finish_kernel, dim3(n_tiles), dim3(kBlockThreads), 0, (hipStream_t)stream, p);
    return (int)hipGetLastError();
}

int launch_half_to_float(const uint16_t* src, vr4* dst, size_t n, void* stream)
{
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(half_to_float_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, dst, n);
    return (int)hipGetLastError();
}

int launch_pack_tiles(const void* src, void* dst, uint32_t elem_bytes, uint32_t W, uint32_t tiles_x,
                      uint32_t n_owned, uint32_t rank, uint32_t nranks, int unpack, void* stream)
{
    if (n_owned == 0) return 0;
    hipLaunchKernelGGL(pack_tiles_kernel, dim3(n_owned), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t*)src, (uint32_t*)dst, elem_bytes / 4u, W, tiles_x, rank, nranks, unpack);
    return (int)hipGetLastError();
}

int launch_selftest_math(int fn, const float* a, const float* b, float* out, size_t n, void* stream)
{
    if (n == 0) return 0;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(selftest_math_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, fn, a, b, out, n);
    return (int)hipGetLastError();
}

} // namespace vr
