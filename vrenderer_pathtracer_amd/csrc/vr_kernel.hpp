// vr_kernel.hpp -- gfx950 (CDNA4, wave64) path-tracing megakernel: device code
// and kernel templates, shared by vr_kernel.hip (dispatch, finish / order /
// helper kernels) and the vr_spec_*.hip translation units (one per scene
// specialisation, compiled in parallel).
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
//   * mesh scenes: a persistent path-pool kernel (render_wave_kernel) drains
//     work queues of 64-path chunks; each lane runs one path at a time
//     through a resumable state machine and takes the next path when its
//     own ends (ballot + mbcnt refill), so divergent path lengths do not idle
//     the SIMD;
//   * sphere-only scenes: render_kernel, one workgroup per 16x16 pixel tile
//     (the reference block, so grid truncation is identical), four wave64s
//     each owning an 8x8 sub-tile;
//   * the traversal stack lives in LDS, entry-major ([depth][lanes]) so a
//     wave's push/pop is one conflict-free ds_write/ds_read_b32, next to an
//     LDS copy of the top of the (area-ordered) tree;
//   * the while-while traversal switches to leaf processing on a wave64
//     __ballot (the reference's 32-lane vote.ballot, :353-363);
//   * leaf hits record only (t, slot, u, v); hit attributes are fetched once
//     per ray after traversal (result-identical: only the final accepted hit
//     is observable), cutting gathers on the hot loop;
//   * all K frames of a render step run in one launch.  Paths store their
//     radiance to a scratch buffer and finish_kernel adds each pixel's paths
//     in path order (bit-identical to the reference's in-order sums); one-path-
//     group sphere launches accumulate in registers instead (render_kernel,
//     RenderParams::use_scratch = 0).
#pragma once
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
// Feature test inside a kernel specialised on FEAT.  Specialisations marked
// F_EXACT are launched only when the scene's flags equal their feature set,
// so their tests fold at compile time; the generic kernel tests the flags.
constexpr uint32_t F_EXACT = 1u << 31;
// Feature-class specialisations (F_CLASS) are launched when the scene's
// geometry flags (kClassGeom) equal theirs and its other flags are a subset
// of FEAT: geometry tests fold at compile time, material features (texture
// maps, BRDF view) are tested against the flags.  Every flag combination the
// Qt UI produces on a mesh or sphere scene lands on one of them instead of the
// generic kernel (vr_kernel.hip launch_scene).
constexpr uint32_t F_CLASS = 1u << 30;
constexpr uint32_t kClassGeom = 1u << 0 | 1u << 3;     // F_CORNELL | F_MESH
#define HAS(F) ((FEAT & (F)) != 0 && ((FEAT & F_EXACT) != 0 || ((FEAT & F_CLASS) != 0 && ((F) & ~kClassGeom) == 0u) || \
                                      (p.flags & (F)) != 0))

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
__device__ __forceinline__ vr4 normalize4(vr4 a) { const float inv = inv_sqrt_exact(dot4(a, a)); return mul4s(a, inv); }
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
    det = sqrt_exact(det);
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
    // instrumented production kernels (F_COUNT_EXEC) only
    // and its lane loads by width (16 / 12 / 8 / 4 B) at every global-load site
    uint32_t nodes_lds = 0, tri_loads = 0, mesh_hits = 0, nmap_hits = 0, ld128 = 0, ld96 = 0, ld64 = 0, ld32 = 0;
    uint32_t shared_miss = 0;      // paths served by their pixel's shared escape radiance (render_kernel)
    // the path kernel's cost of the lane's current path (node visits), summed
    // per sub-tile for the next launch's longest-first order (RenderParams::sub_cost)
    uint32_t work = 0;
};

// Counting launches (COUNT) come in two kinds: the reference algorithm's
// event counts (no primary-hit reuse, no last-bounce shortcut)
// and the instrumented production kernels (F_COUNT_EXEC in FEAT), which run
// exactly what vrhip_render runs and count the memory operations issued.
template <bool COUNT, uint32_t FEAT>
__device__ constexpr bool ref_alg() { return COUNT && (FEAT & F_COUNT_EXEC) == 0u; }

// One wave-level reduction and one 64-bit atomic per counter per wave.
__device__ __forceinline__ void flush_counts(const RenderParams& p, const Cnt& cnt, int lane, bool exec)
{
    const uint32_t v[kCounters + kExecCounters] = { cnt.rays, cnt.nodes, cnt.slots, cnt.tris, cnt.attr, cnt.tex,
                                                    cnt.hdr, cnt.brdf, cnt.nodes_lds, cnt.tri_loads,
                                                    cnt.mesh_hits, cnt.nmap_hits, cnt.ld128, cnt.ld96, cnt.ld64,
                                                    cnt.ld32, cnt.shared_miss };
#pragma unroll
    for (int k = 0; k < kCounters + kExecCounters; ++k) {
        if (k >= kCounters && !exec) break;
        unsigned long long x = v[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        const int slot = k < kCounters ? k : kExecCounterBase + (k - kCounters);
        if (lane == 0 && x) atomicAdd(p.counters + slot, x);
    }
}

struct Hit {                // vHitData, PathTracer.cuh:17-53
    vr4 hp, n, tan, em, col, spec;
    unsigned type;
};

// A uniform image dimension as a float, converted where it is used: the
// asm hides the value's loop invariance, so the conversion is not hoisted
// out of the path loop into a VGPR held across it (the C3 kernels spilled
// exactly those: float texture heights and the HDRI size)
__device__ __forceinline__ float dim_f(uint32_t n) {
    asm volatile("" : "+s"(n));
    return (float)n;
}
__device__ __forceinline__ int tex_addr(uint32_t w, uint32_t h, float u, float v) {
    const int x = f2i(dim_f(w) * u);
    const int y = f2i(dim_f(h) * v);
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
constexpr int cache_nodes(int stack, int extra = 0, int bt = kBlockThreads) {
    return ((bt / kBlockThreads) * kLdsBudget - stack * bt * 4 - extra) / 56 > 0 ?
           ((bt / kBlockThreads) * kLdsBudget - stack * bt * 4 - extra) / 56 : 1;
}
// Raw buffer loads for the node and triangle arrays: a 32-bit lane offset
// against an SGPR descriptor (bounds-checked, no 64-bit address math), and an
// explicit width per fetch (16 B node rows and triangle-pair rows, 8 B child
// indices and pair tails).
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
__device__ __forceinline__ int2 buf_load2i(__amdgpu_buffer_rsrc_t b, int off) {
    const vr_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(b, off, 0, 0);
    return make_int2((int)v.x, (int)v.y);
}

// The t-culled traversal (default) reads conservative fp16 node boxes: two
// 16-B loads per node visit instead of four, the vector-memory instructions
// this kernel is bound by (C2 +9 %, C3 +5 %, C5 +5 % on the 6-wave kernel).
// Rounded outward, a box only grows, so no hit is lost; the looser boxes
// change the visit order, which the exact equal-t tie-break (ref_first) makes
// irrelevant to the result: images equal the fp32 and the strict traversal
// bit for bit (C5 differed in one pixel in 8.3 M without it).  The strict
// traversal (F_STRICT) reads the reference's fp32 rows.

struct Lds {
    int* stk;                 // this thread's column of the stack
    const vr4* nodes;         // fp32 nodes: 3 rows per cached node; fp16 nodes: 2 rows per node
    const int2* idx;          // fp32 nodes: child indices per cached node
    int n_cached;             // nodes [0, n_cached) are read from LDS
    int stride;               // stack entry stride (threads per block; entry-major [depth][threads])
};

// CudaTracerLib-style while-while traversal (PathTracer.cu:276-463), split
// into init / one outer iteration / finish so a wave can pause it between
// outer iterations (render_wave_kernel) without changing any lane's sequence
// of node visits and triangle tests.
constexpr int kSentinel = 0x76543210;
struct Trav {
    float ivx, ivy, ivz, odx, ody, odz;
    float t, tcull, bu, bv;   // tcull: read only by kernels with helper lanes (tcull_kept)
    int best, sp, nodeAddr;
};
// The culling distance is t x (1 + 2^-10) (infinite for the strict walk),
// recomputed per node visit -- one v_mul against a register held through the
// whole walk (C2 +0.5 %, C5 +0.5 %) -- except in the small-launch kernels,
// whose helper lanes cull with the smaller of their own and their owner's
// (help_step).
#ifndef VR_TCULL_KEPT
#define VR_TCULL_KEPT 0           // 1: every kernel keeps tcull in a register (A/B builds)
#endif
template <uint32_t FEAT>
constexpr bool tcull_kept() { return VR_TCULL_KEPT != 0 || (FEAT & F_SMALL) != 0u; }

template <uint32_t FEAT>
__device__ __forceinline__ void trav_init(const RenderParams& p, const Ray& r, float t0, Trav& tr, const Lds& L)
{
    tr.sp = 0;
    L.stk[0] = kSentinel;
    tr.nodeAddr = 0;
    // invDir (PathTracer.cu:289-294): components with |d| <= eps become +eps,
    // so |d| >= eps > 2^-32 and rcp_rn is the IEEE quotient unless a
    // component exceeds 2^125 (then the wave divides)
    const float dx = __builtin_fabsf(r.d.x) > VR_EPS ? r.d.x : VR_EPS;
    const float dy = __builtin_fabsf(r.d.y) > VR_EPS ? r.d.y : VR_EPS;
    const float dz = __builtin_fabsf(r.d.z) > VR_EPS ? r.d.z : VR_EPS;
    if (__builtin_expect(__ballot(!(__builtin_fabsf(dx) <= kRcpRnHi && __builtin_fabsf(dy) <= kRcpRnHi &&
                                    __builtin_fabsf(dz) <= kRcpRnHi)) != 0ull, 0)) {
        tr.ivx = 1.f / dx; tr.ivy = 1.f / dy; tr.ivz = 1.f / dz;
    } else {
        tr.ivx = rcp_rn(dx); tr.ivy = rcp_rn(dy); tr.ivz = rcp_rn(dz);
    }
    tr.odx = r.o.x * tr.ivx; tr.ody = r.o.y * tr.ivy; tr.odz = r.o.z * tr.ivz;
    tr.t = t0;
    // t-culling: a child whose slab entry lies beyond the closest hit so far
    // (times a 2^-10 safety margin) cannot hold a closer triangle.  The
    // reference visits every pierced box (span end clamped to 1e20,
    // :316,322); F_STRICT restores that exactly.
    tr.tcull = HAS(F_STRICT) ? __builtin_inff() : t0 * 1.0009765625f;
    tr.best = -1;
    tr.bu = tr.bv = 0.f;
}

// Pop (:339-342 and the leaf-loop pops).  sp reaches -1 only by popping the
// sentinel, after which nothing is popped.
__device__ __forceinline__ int trav_pop(Trav& tr, const Lds& L)
{
    return L.stk[(tr.sp--) * L.stride];
}

// Whether node visits may read the block's LDS copy of the tree top.  Off
// (VR_SVC_LDS_NODES=0, A/B builds) in the Cornell-box service kernels: the
// wave-uniform choice almost never finds a diverged wave entirely in the
// cached top there (0.2 % of node bytes, r05), so the test per visit is spent
// for nothing.
#ifndef VR_SVC_LDS_NODES
#define VR_SVC_LDS_NODES 1
#endif
#ifndef VR_LDS_PER_LANE
#define VR_LDS_PER_LANE 0
#endif
template <uint32_t FEAT>
constexpr bool lds_nodes_on() {
    return VR_SVC_LDS_NODES != 0 || (FEAT & F_SERVICE) == 0u || (FEAT & F_CORNELL) == 0u;
}

// One inner-node visit (:295-343): fetch (LDS copy or L2/HBM), two slab
// tests, near child next, far child pushed when both are entered, pop when
// neither is.  Leaves in tr.nodeAddr are left to the caller.
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ void node_step(const RenderParams& p, const Ray& r, Trav& tr, const Lds& L, Cnt& cnt)
{
    int* stk = L.stk;
    const bool strict = HAS(F_STRICT);   // compile-time false in the specialised kernels
    const float tcull = tcull_kept<FEAT>() ? tr.tcull : strict ? __builtin_inff() : tr.t * 1.0009765625f;
    if (COUNT) cnt.nodes += 1u;
    if ((FEAT & F_SMALL) != 0u) cnt.work++;
    vr4 n0, n1, nz;
    int idx0, idx1;
    const int node = tr.nodeAddr >> 2;
    // wave-uniform choice between the LDS copy and L2/HBM: a diverged wave
    // would pay both round trips (VR_LDS_PER_LANE=1: each lane on its own)
    const bool in_lds = lds_nodes_on<FEAT>() &&
                        (VR_LDS_PER_LANE ? node < L.n_cached : __ballot(node >= L.n_cached) == 0ull);
    if (COUNT) {
        cnt.nodes_lds += in_lds ? 1u : 0u;
        if (!in_lds) { cnt.ld128 += strict ? 3u : 2u; cnt.ld64 += strict ? 1u : 0u; }
    }
    if (!strict) {
        // conservative fp16 boxes (lows rounded down, highs up): two 16-B
        // fetches per node instead of four; a box can only grow, so no hit
        // the exact box admits is lost
        vr4 a, b;
        if (in_lds) {
            a = L.nodes[2 * node];
            b = L.nodes[2 * node + 1];
        } else {
            const __amdgpu_buffer_rsrc_t hbuf = buf_rsrc(p.bvh16, p.n_nodes * 32u);
            const int off = node * 32;
            a = buf_load4(hbuf, off);
            b = buf_load4(hbuf, off + 16);
        }
        auto lo = [](float w) { return __half2float(__ushort_as_half((unsigned short)(__float_as_uint(w) & 0xffffu))); };
        auto hi = [](float w) { return __half2float(__ushort_as_half((unsigned short)(__float_as_uint(w) >> 16))); };
        n0 = mk4(lo(a.x), hi(a.x), lo(a.y), hi(a.y));          // c0 x, y
        nz = mk4(lo(a.z), hi(a.z), lo(b.y), hi(b.y));          // c0 z, c1 z
        n1 = mk4(lo(a.w), hi(a.w), lo(b.x), hi(b.x));          // c1 x, y
        idx0 = __float_as_int(b.z);
        idx1 = __float_as_int(b.w);
    } else {
        int2 ni;
        if (in_lds) {
            const int row = __mul24(3, node);                 // v_mul_u32_u24 (full rate)
            n0 = L.nodes[row + 0];
            n1 = L.nodes[row + 1];
            nz = L.nodes[row + 2];
            ni = L.idx[node];
        } else {
            const __amdgpu_buffer_rsrc_t nbuf = buf_rsrc(p.bvh, p.n_nodes * 64u);
            const int off = tr.nodeAddr * 16;                 // byte offset of the node
            n0 = buf_load4(nbuf, off);
            n1 = buf_load4(nbuf, off + 16);
            nz = buf_load4(nbuf, off + 32);
            ni = buf_load2i(nbuf, off + 48);                  // 8 of the row's 16 bytes are used
        }
        idx0 = ni.x;
        idx1 = ni.y;
    }
    // slab distances n*inv - o*inv (:307-322); the culled mode lets
    // them contract to one v_fma each (more accurate)
    auto slab = [&](float n, float iv, float od) {
        return strict ? (n * iv - od) : __builtin_fmaf(n, iv, -od);
    };
    const float c0lox = slab(n0.x, tr.ivx, tr.odx);
    const float c0hix = slab(n0.y, tr.ivx, tr.odx);
    const float c0loy = slab(n0.z, tr.ivy, tr.ody);
    const float c0hiy = slab(n0.w, tr.ivy, tr.ody);
    const float c0loz = slab(nz.x, tr.ivz, tr.odz);
    const float c0hiz = slab(nz.y, tr.ivz, tr.odz);
    const float c1loz = slab(nz.z, tr.ivz, tr.odz);
    const float c1hiz = slab(nz.w, tr.ivz, tr.odz);
    const float c0min = span_begin(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 0.0f);
    const float c0max = span_end(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 1e20f);
    const float c1lox = slab(n1.x, tr.ivx, tr.odx);
    const float c1hix = slab(n1.y, tr.ivx, tr.odx);
    const float c1loy = slab(n1.z, tr.ivy, tr.ody);
    const float c1hiy = slab(n1.w, tr.ivy, tr.ody);
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
    const int nearc = (both && swp) ? idx1 : (tc0 ? idx0 : idx1);
    const int farc = swp ? idx0 : idx1;
    const int top = stk[tr.sp * L.stride];
    if (both) stk[(tr.sp + 1) * L.stride] = farc;
    tr.sp += both ? 1 : (none ? -1 : 0);
    tr.nodeAddr = none ? top : nearc;
}

// The root visit at ray setup (path kernels).  Every lane that starts a walk
// is at the root, so node_step's wave-uniform choice takes the block's LDS
// copy of the tree top: the walk's first visit -- the same fetch of the same
// node, the same slab tests, the same push and pop -- without the two global
// loads and the round trip it cost inside trav_iter, and a ray that enters
// neither child of the root (most Cornell-box bounce rays run wall to wall
// past the mesh) leaves for shading at once instead of passing through the
// traversal state machine.  The walk then resumes from the root's near child
// exactly as it would have, so every lane's sequence of visits and tests is
// unchanged.  false: the walk is over (no mesh hit).
#ifndef VR_ROOT_AT_SETUP
#define VR_ROOT_AT_SETUP 0
#endif
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool root_visit(const RenderParams& p, const Ray& r, Trav& tr, const Lds& L, Cnt& cnt)
{
    if (VR_ROOT_AT_SETUP == 0 || L.n_cached < 1) return true;
    node_step<COUNT, FEAT>(p, r, tr, L, cnt);
    return tr.nodeAddr != kSentinel;
}

// Equal-t tie-break of the culled traversal.  The reference keeps the first
// of two triangles hit at exactly the same distance (strict `<`,
// PathTracer.cu:379), i.e. the one its depth-first walk tests first: slot
// order inside a leaf; otherwise the child of the two leaves' lowest common
// ancestor that the walk enters first for this ray -- the nearer by slab entry,
// child 0 on equal entries (:324-343), computed here with the reference's own
// (uncontracted) slab arithmetic.  The t-culled walk skips boxes and its
// contracted slabs can order near-equal children differently, so it asks
// this whenever a triangle ties the closest hit: any visit order then yields
// the reference's hit.  Rare (exact fp32 ties: rays through shared edges).
__device__ __forceinline__ bool ref_first(const RenderParams& p, const Trav& tr, int ka, int kb)
{
    const unsigned long long a = p.tpath[ka], b = p.tpath[kb];
    if (a == b) return ka < kb;                                    // one leaf: slot order
    const int L = __builtin_ctzll(a ^ b);                          // depth where the paths part
    const int da = 63 - __builtin_clzll(a), db = 63 - __builtin_clzll(b);
    if (L >= da || L >= db) return ka < kb;                        // not a tree path (cannot happen)
    const __amdgpu_buffer_rsrc_t nbuf = buf_rsrc(p.bvh, p.n_nodes * 64u);
    int off = 0;                                                   // byte offset of the root
    for (int i = 0; i < L; ++i) {
        const int2 ni = buf_load2i(nbuf, off + 48);
        off = (((a >> i) & 1ull) ? ni.y : ni.x) * 16;              // child float4 offset -> bytes
    }
    const vr4 n0 = buf_load4(nbuf, off), n1 = buf_load4(nbuf, off + 16), nz = buf_load4(nbuf, off + 32);
    auto sl = [](float n, float iv, float od) { return n * iv - od; };   // -ffp-contract=off: no FMA
    const float c0min = span_begin(sl(n0.x, tr.ivx, tr.odx), sl(n0.y, tr.ivx, tr.odx), sl(n0.z, tr.ivy, tr.ody),
                                   sl(n0.w, tr.ivy, tr.ody), sl(nz.x, tr.ivz, tr.odz), sl(nz.y, tr.ivz, tr.odz), 0.0f);
    const float c1min = span_begin(sl(n1.x, tr.ivx, tr.odx), sl(n1.y, tr.ivx, tr.odx), sl(n1.z, tr.ivy, tr.ody),
                                   sl(n1.w, tr.ivy, tr.ody), sl(nz.z, tr.ivz, tr.odz), sl(nz.w, tr.ivz, tr.odz), 0.0f);
    const unsigned first = (c1min < c0min) ? 1u : 0u;
    return (unsigned)((a >> L) & 1ull) == first;
}

// intersectTriangle (RayIntersection.cuh:54-111) for compact triangle k and
// the closest-hit update (:379-386).  Evaluated branch-free: every early
// return of the reference becomes a term of the final predicate (the values
// computed for a surviving triangle are the same operations in the same order).
struct TriV { vr3 a0, a1, a2; };        // v0, e1 = v1 - v0, e2 = v2 - v0 (p.tri_e)
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ void tri_test_v(const RenderParams& p, const Ray& r, Trav& tr, int k, const TriV& t, Cnt& cnt)
{
    const bool strict = HAS(F_STRICT);
    if (COUNT) cnt.tris++;
    const vr4 v0 = mk4(t.a0.x, t.a0.y, t.a0.z, 0.f);
    const vr4 e1 = mk4(t.a1.x, t.a1.y, t.a1.z, 0.f);         // v1 - v0, v2 - v0 (RayIntersection.cuh:62-63), from the upload
    const vr4 e2 = mk4(t.a2.x, t.a2.y, t.a2.z, 0.f);
    const vr4 pv = cross4(r.d, e2);
    const float det = dot4(e1, pv);
    // 1/det (RayIntersection.cuh:75): only lanes with |det| >= VR_EPS (> 2^-32) can accept the
    // hit, and there rcp_rn is the IEEE quotient up to |det| = 2^125; a wave
    // holding a larger (or non-finite) det takes the division
    float inv_det;
    if (__builtin_expect(__ballot(!(__builtin_fabsf(det) <= kRcpRnHi)) != 0ull, 0)) inv_det = 1.f / det;
    else inv_det = rcp_rn(det);
    const vr4 tv = sub4(r.o, v0);
    const float u = dot4(tv, pv) * inv_det;
    const vr4 q = cross4(tv, e1);
    const float v = dot4(r.d, q) * inv_det;
    const float dist = dot4(e2, q) * inv_det;
    const bool ok = !(det > -VR_EPS && det < VR_EPS) && !(u < 0.f || u > 1.f) &&
                    !(v < 0.f || u + v > 1.f);
    if (ok && dist > VR_EPS && dist < tr.t) {
        tr.t = dist; tr.best = 3 * k; tr.bu = u; tr.bv = v;
        tr.tcull = strict ? tr.tcull : tr.t * 1.0009765625f;
    }
    // a tie with the mesh's closest hit so far: keep the reference's first
    // (the strict walk tests in the reference order already)
    const bool tie = !strict && ok && dist > VR_EPS && dist == tr.t && tr.best >= 0 && 3 * k != tr.best;
    if (__builtin_expect(__ballot(tie) != 0ull, 0)) {
        if (tie && ref_first(p, tr, k, tr.best / 3)) { tr.best = 3 * k; tr.bu = u; tr.bv = v; }
    }
}

// One outer iteration of the while-while loop: the inner node loop until
// this lane holds a leaf and the wave agrees (ballot, :353-363), with one
// leaf postponed (:345-351), then the leaf loop.  tr.nodeAddr is an inner
// node, a leaf (a helper's first entry) or kSentinel (no-op).
#ifndef VR_NODE_BREAK
// measured (path kernel with paired triangle loads): 0 (the reference's
// all-lanes vote) C2 2,294, 2: 2,503, 4: 2,563, 6: 2,577, 8: 2,583 (C3 -2 %).
// Since the Cornell-box and listed-pixel kernels have their own thresholds
// (below) this one serves the one-frame kernels and the HDRI primary-pass
// kernels: r05, 8 against 6, one frame per call C2 0.695 -> 0.686 ms, C3
// 0.398 -> 0.393, C5 1.717 -> 1.707 (4: +1.5-2 % slower), 16-frame rates
// unchanged (profiles/r05x_node_break_one_frame_*.txt); 12 against 8: C2
// 0.687 -> 0.677, C3 0.394 -> 0.389 (profiles/r05y_node_break12_one_frame_*);
// 16 ties, 20 loses (profiles/r05z_node_break16_20_one_frame_*)
#define VR_NODE_BREAK 12
#endif
#ifndef VR_NODE_BREAK_CORNELL
// Cornell-box kernels (every bounce ray stays inside the box and most lanes
// keep traversing the mesh): r02 6-wave kernel, C2 6: 3,910, 10: 3,986;
// the HDRI scenes lose at 10 (C3 -1.3 %, C5 -1.2 %) and keep VR_NODE_BREAK.
// Re-measured on the r05 7-wave service kernel (profiles/r05x_node_break_*):
// C2 8: -1.2 %, 12: +1.0 %, 14: +1.9 %, 16: +2.0-2.4 %, 20: +1.7-2.0 %
// against 10 (C2D 16: +1.2-2.2 %)
#define VR_NODE_BREAK_CORNELL 16
#endif
// Kernels over the listed pixels of HDRI scenes (F_SPARSE: every lane's path
// hit the mesh at its camera ray): 8 (r04, against 6: C3 +0.7 %, C5 +0.7 %,
// C3D +1.3 %; 10: -1.5 / +0.4 / +0.7 %)
#ifndef VR_NODE_BREAK_SPARSE
#define VR_NODE_BREAK_SPARSE 8
#endif
template <uint32_t FEAT>
constexpr int node_break() {
    if ((FEAT & F_SPARSE) != 0u) return VR_NODE_BREAK_SPARSE;
    // one-frame kernels (F_INLINE_PRIM) keep VR_NODE_BREAK: the interactive
    // C2 rate fell 2,147 -> 2,103 Mpaths/s with 10 (r02h)
    return ((FEAT & (F_EXACT | F_CLASS)) && (FEAT & F_CORNELL) && !(FEAT & F_INLINE_PRIM)) ? VR_NODE_BREAK_CORNELL : VR_NODE_BREAK;
}
// The node-loop exit is proportional to the lanes in the call: a full wave
// leaves once at most node_break of its 64 lanes still search (throughput:
// the rest of the wave need not wait for its slowest searches), a wave with
// few traversing lanes -- the sparse waves of a launch's drain, or a wave
// whose other lanes are shading -- waits for all of them, as the reference's
// vote does (:353-363).  A fixed threshold made a sparse wave's lanes leave
// after ONE node visit per outer iteration: the most expensive paths (C2:
// ~200 node visits, ~100 triangle tests) then needed 50-150 outer iterations
// and ran 300-770 us, the critical path of a one-frame launch (r03 drain
// diagnostics, removed in r04; git history).
#ifndef VR_NODE_BREAK_PROP
#define VR_NODE_BREAK_PROP 1
#endif
template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ void trav_iter(const RenderParams& p, const Ray& r, Trav& tr, const Lds& L, Cnt& cnt)
{
#if VR_NODE_BREAK_PROP
    const int brk = node_break<FEAT>() * __popcll(__ballot(1));  // exit when searching * 64 <= brk
#else
    const int brk = node_break<FEAT>() * 64;
#endif
    int leafAddr = 0;
    if (tr.nodeAddr < 0) {                                      // a leaf to start with (a helper's subtree)
        leafAddr = tr.nodeAddr;
        tr.nodeAddr = trav_pop(tr, L);
    }
    while ((unsigned)tr.nodeAddr < (unsigned)kSentinel) {
        node_step<COUNT, FEAT>(p, r, tr, L, cnt);
        if (tr.nodeAddr < 0 && leafAddr >= 0) {                 // postpone max 1
            leafAddr = tr.nodeAddr;
            tr.nodeAddr = trav_pop(tr, L);
        }
        // the wave moves on to the leaves once (nearly) every lane holds one;
        // lanes still searching resume in the next outer iteration
        if (__popcll(__ballot(leafAddr >= 0)) * 64 <= brk) break;
    }
    while (leafAddr < 0) {
        const int lv = ~leafAddr;
        const int kend = (lv >> kLeafCountBits) + (lv & ((1 << kLeafCountBits) - 1));
        // the loads of two triangles in one trip (the tests stay in slot order):
        // a leaf's triangles need half the dependent round trips (C2 +1 %, C3 +4 %),
        // the pair's 72 contiguous bytes as 4 x 16 B + 8 B (5 loads instead of 6:
        // C2 +1 %, C3 +1 %, C5 +3 %); past the array end the buffer descriptor
        // returns zeros (never tested)
        for (int k = lv >> kLeafCountBits; k < kend; k += 2) {
            const bool two = k + 1 < kend;
            TriV ta, tb;
            {
                const __amdgpu_buffer_rsrc_t tbuf = buf_rsrc(p.tri_e, p.n_tris * 36u);
                const int o = k * 36;
                const vr4 q0 = buf_load4(tbuf, o), q1 = buf_load4(tbuf, o + 16), q2 = buf_load4(tbuf, o + 32),
                          q3 = buf_load4(tbuf, o + 48);
                const int2 q4 = buf_load2i(tbuf, o + 64);
                ta.a0 = vr3{ q0.x, q0.y, q0.z }; ta.a1 = vr3{ q0.w, q1.x, q1.y }; ta.a2 = vr3{ q1.z, q1.w, q2.x };
                tb.a0 = vr3{ q2.y, q2.z, q2.w }; tb.a1 = vr3{ q3.x, q3.y, q3.z };
                tb.a2 = vr3{ q3.w, __int_as_float(q4.x), __int_as_float(q4.y) };
            }
            if (COUNT) {                                        // an odd leaf's last pair loads its triangle twice
                cnt.tri_loads += 2;
                cnt.ld128 += 4; cnt.ld64 += 1;
            }
            asm volatile("" ::"v"(ta.a0.x), "v"(ta.a1.x), "v"(ta.a2.x), "v"(tb.a0.x), "v"(tb.a1.x), "v"(tb.a2.x));
            tri_test_v<COUNT, FEAT>(p, r, tr, k, ta, cnt);
            if (two) tri_test_v<COUNT, FEAT>(p, r, tr, k + 1, tb, cnt);
        }
        leafAddr = tr.nodeAddr;
        if (tr.nodeAddr < 0) tr.nodeAddr = trav_pop(tr, L);
    }
}

__device__ __forceinline__ void trav_finish(const Trav& tr, HitRec& hr)
{
    if (tr.best >= 0) { hr.t = tr.t; hr.kind = HK_MESH; hr.idx = tr.best; hr.bu = tr.bu; hr.bv = tr.bv; }
}

template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ void traverse_mesh(const RenderParams& p, const Ray& r, HitRec& hr, const Lds& L, Cnt& cnt,
                                              bool any_hit = false)
{
    Trav tr;
    trav_init<FEAT>(p, r, hr.t, tr, L);
    while (tr.nodeAddr != kSentinel) {
        trav_iter<STACK, COUNT, FEAT>(p, r, tr, L, cnt);
        if (any_hit && tr.best >= 0) tr.nodeAddr = kSentinel;     // (any_hit_enough)
    }
    trav_finish(tr, hr);
}
// intersectScene (PathTracer.cu:136-468): closest hit, attributes deferred.
// intersectScene (PathTracer.cu:136-468), sphere part: Cornell walls and
// light, the two small spheres, the example sphere.  Returns true when the
// mesh must still be traversed (kMeshInitialised and no example sphere).
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool intersect_spheres(const RenderParams& p, const Ray& r, HitRec& hr, Cnt& cnt)
{
    if (COUNT) cnt.rays++;
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
        return false;
    }
    return HAS(F_MESH);
}

// intersectScene: closest hit, attributes deferred (fill_hit).
template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool intersect_scene(const RenderParams& p, const Ray& r, HitRec& hr, const Lds& L, Cnt& cnt)
{
    const bool mesh = intersect_spheres<COUNT, FEAT>(p, r, hr, cnt);
    if (mesh) {
        traverse_mesh<STACK, COUNT, FEAT>(p, r, hr, L, cnt);
    }
    return hr.t < 1e20f;
}

// Materialise vHitData for the final hit (the values the reference's last
// accepted hit wrote; :160-168, :180-189, :198-266, :380-453).
// Face normals from the traversal's triangle edges (fill_hit): on in every
// kernel but the Cornell-box one-frame kernels, which spill 2 VGPRs with it
// (C2 16-frame steps +0.7 %, C5 one frame per call -1 %, r05s)
#ifndef VR_FACE_FROM_EDGES
#define VR_FACE_FROM_EDGES 1
#endif
template <uint32_t FEAT>
constexpr bool face_from_edges() {
    return VR_FACE_FROM_EDGES != 0 && !((FEAT & F_INLINE_PRIM) != 0u && (FEAT & F_CORNELL) != 0u);
}
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
        } else if constexpr (face_from_edges<FEAT>()) {
            // the face normal from the traversal's copy of the triangle, whose
            // lines the leaf loop just fetched (L1 / L2-hot, 24 B instead of
            // the 36 B of p.verts): its edges e1 = v1 - v0, e2 = v2 - v0 were
            // rounded at upload as the reference's v0 - v1, v0 - v2 negated
            // (IEEE subtraction is sign-symmetric), and the cross product of
            // two negated vectors is the same bits -- the same normal
            const __amdgpu_buffer_rsrc_t tbuf = buf_rsrc(p.tri_e, p.n_tris * 36u);
            const int o = (a / 3) * 36;
            const vr_u32x3 q1 = __builtin_amdgcn_raw_buffer_load_b96(tbuf, o + 12, 0, 0);
            const vr_u32x3 q2 = __builtin_amdgcn_raw_buffer_load_b96(tbuf, o + 24, 0, 0);
            const vr4 e1 = mk4(__uint_as_float(q1.x), __uint_as_float(q1.y), __uint_as_float(q1.z), 0.f);
            const vr4 e2 = mk4(__uint_as_float(q2.x), __uint_as_float(q2.y), __uint_as_float(q2.z), 0.f);
            h.n = normalize4(cross4(e1, e2));
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

// Whether the mesh must be traversed for a ray whose closest SPHERE hit is
// `hr`, on bounce `bounce`.  On the last bounce (3) only the closest hit's
// emission is observable (bounce_step adds mask * emission and ends the path;
// the reference's material sampling after it, PathTracer.cu:663-764,
// prepares a ray it never traces) -- or, for a ray that hits nothing, the
// miss branch (the Cornell escape's 0, or the HDRI's radiance, :631-652).
// The mesh's emission is exactly (+0, +0, +0, 0) (:454-462; fill_hit,
// emission_of), and so is that of every sphere but the Cornell box's light
// and its two coloured walls.  So when the closest sphere hit has that
// emission, whether a triangle lies in front of it changes no bit of the
// result (the same product with the same zero vector is added) and the
// traversal is skipped.  A ray that hits no sphere, or an emitting one, is
// traversed (the mesh decides between a miss and a hit, or occludes the
// emitter).  Not in the reference-algorithm counting variant or the strict
// walk, which keep the reference's work.  C2: the last bounce is a third of
// the rays a path traces (+6 %, r06b).
#ifndef VR_LAST_BOUNCE_SKIP
#define VR_LAST_BOUNCE_SKIP 1         // 0: off, 1: skip + any-hit (below), 2: skip only (A/B builds)
#endif
#ifndef VR_LAST_BOUNCE_HDRI
#define VR_LAST_BOUNCE_HDRI 1         // 0: the Cornell box only (A/B builds)
#endif
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool last_bounce_opt(const RenderParams& p, int bounce)
{
    // (HDRI scenes: C3 +1 %, C5 +0.6 %, r06c; not the textured one-frame
    // kernel, where it cost 5 spilled VGPRs)
    constexpr bool TEX1 = (FEAT & F_INLINE_PRIM) != 0u && (FEAT & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
    return VR_LAST_BOUNCE_SKIP != 0 && !ref_alg<COUNT, FEAT>() && !HAS(F_STRICT) && bounce == 3 &&
           (HAS(F_CORNELL) || (VR_LAST_BOUNCE_HDRI != 0 && !TEX1));
}
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool mesh_needed(const RenderParams& p, const HitRec& hr, int bounce)
{
    if (!last_bounce_opt<COUNT, FEAT>(p, bounce) || (hr.kind != HK_CORNELL && hr.kind != HK_SMALL)) return true;
    const vr4 e = emission_of(hr);
    return (__float_as_uint(e.x) | __float_as_uint(e.y) | __float_as_uint(e.z)) != 0u;
}
// The traversals that remain on that bounce (the closest sphere emits, or
// none is hit) need only WHETHER a triangle lies closer than the sphere hit:
// any triangle the walk accepts makes the hit a mesh hit, whose emission is
// 0 whichever triangle it is.  So the walk may stop at the end of the outer
// iteration in which it first accepts one (any-hit instead of closest-hit;
// C2 a further +1.3 %, r06b).
template <bool COUNT, uint32_t FEAT>
__device__ __forceinline__ bool any_hit_enough(const RenderParams& p, int bounce)
{
    return VR_LAST_BOUNCE_SKIP == 1 && last_bounce_opt<COUNT, FEAT>(p, bounce);
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
    const float* e = T + 3 * ind;    // interleaved on the device (vrhip_upload_brdf)
    return mk4((float)((double)e[0] * (1.0 / 1500.0)),
               (float)((double)e[1] * (1.15 / 1500.0)),
               (float)((double)e[2] * (1.66 / 1500.0)), 0.f);
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
// State of one path between bounces (trace, PathTracer.cu:597-770).
struct PathState {
    vr4 accum, mask;
    float depth;
    int bounce;
    Rng rng;
};

// trace's prologue (:603-622); s0, s1 are updated as the reference's seeds
__device__ __forceinline__ void path_begin(PathState& ps, uint32_t& s0, uint32_t& s1) {
    ps.accum = mk4(0.f, 0.f, 0.f, 0.f);
    ps.mask = mk4(1.f, 1.f, 1.f, 0.f);
    ps.depth = 1.f;
    ps.bounce = 0;
    ps.rng.seed(hash_seeds(s0, s1));
}

// The depth term of a path (PathTracer.cu:656-661): |hit - origin| / 150 of
// its bounce-0 hit, i.e. of the camera ray's closest hit (no jitter: the same
// for every path of the pixel).  Path-pool launches with a primary pass take
// it from primary_kernel, which stores it once per pixel, and their path
// kernels carry no depth register (bounce_step<..., false>).
__device__ __forceinline__ float depth_term(const vr4& o, const vr4& hp)
{
    const vr4 l = sub4(o, hp);
    return sqrt_exact(dot4(l, l)) / 150.f;
}

// Coherence probe (-DVR_PROBE_COHERENT=G; INVALID images, measurement only):
// the lanes sampling a diffuse / BRDF bounce in the same step are split into
// G groups of 64/G lanes, and every lane takes its group leader's (first
// active lane's) direction sample -- G = 1: one sample per wave-step (the
// ideal bound), G = 64: no change.  Bounds what binning bounce rays by
// direction could return at a given number of distinct directions per wave
// (C2, r04: G = 1 +15.3 %, G = 4 +3.7 %, G = 16 +0.5 %).
__device__ __forceinline__ void probe_coherent(float& rand1, float& rand2)
{
#ifdef VR_PROBE_COHERENT
    constexpr int G = VR_PROBE_COHERENT, span = 64 / G;
    const int lane = (int)__lane_id();
    const unsigned long long act = __ballot(1);
    const int g0 = (lane / span) * span;
    const unsigned long long grp = (span == 64 ? ~0ull : ((1ull << span) - 1ull)) << g0;
    const int leader = __builtin_ctzll(act & grp);
    rand1 = __shfl(rand1, leader, 64);
    rand2 = __shfl(rand2, leader, 64);
#else
    (void)rand1; (void)rand2;
#endif
}

// One bounce of trace's loop body (:627-769) for the closest hit `hr` of
// `ray` (hr.t == 1e20: miss).  Returns true when the path ends, with its
// radiance (w = depth) in `out`; otherwise `ray` is the next bounce's ray.
// bounce_step's exits call `sink` with the path's result (the render
// service's store at each exit; the default stores nothing)
struct NoSink { __device__ __forceinline__ void operator()(const vr4&) const {} };
template <bool COUNT, uint32_t FEAT, bool DEPTH = true, typename Sink = NoSink>
__device__ __forceinline__ bool bounce_step(const RenderParams& p, Ray& ray, const HitRec& hr, PathState& ps,
                                            vr4& out, Cnt& cnt, const Sink& sink = Sink())
{
    const bool hit = hr.t < 1e20f;
    if (!hit) {
        if (!HAS(F_CORNELL)) {                                    // :631-648
            float lx = atan2_p(ray.d.x, ray.d.z);
            float ly = acos_p(ray.d.y);
            lx = lx < 0 ? (float)((double)lx + 2.0 * (double)VR_PI) : lx;
            lx = (float)((double)lx / (2.0 * (double)VR_PI));
            ly = ly / VR_PI;
            // (textured kernels: C5's plain HDRI kernels hold the floats
            // without spilling, and hoisted they cost it nothing)
            constexpr bool TEX = (FEAT & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
            const int x = f2i(lx * (TEX ? dim_f(p.hdr_w) : (float)p.hdr_w));
            const int y = f2i(ly * (TEX ? dim_f(p.hdr_h) : (float)p.hdr_h));
            const int val = (int)((uint32_t)x + (uint32_t)y * p.hdr_w);
            const int addr = (int)clampi(val, 0, (int)(p.hdr_w * p.hdr_h - 1u));
            if (COUNT) { cnt.hdr++; cnt.ld128++; }
            ps.accum = add4(ps.accum, mul4(mul4s(ps.mask, 2.f), p.hdr[addr]));
            ps.accum.w = ps.depth;
            out = ps.accum;
            sink(out);
            return true;
        }
        // Cornell escape (:649-650): radiance and .w are 0.  The x channel
        // is -0.0 -- equal to +0 in every sum it enters (a running sum that
        // starts at +0 under round-to-nearest is never -0, so adding -0 or +0
        // leaves its bits unchanged) -- and marks the escape in the
        // path-result scratch, which does not store .w (store_path).
        out = mk4(-0.f, 0.f, 0.f, 0.f);
        sink(out);
        return true;
    }
    if (!ref_alg<COUNT, FEAT>() && ps.bounce == 3) {
        // last bounce: only the emission term is observable; the material
        // branch below would only prepare a ray that is never traced
        ps.accum = add4(ps.accum, mul4(ps.mask, emission_of(hr)));
        ps.accum.w = ps.depth;
        out = ps.accum;
        sink(out);
        return true;
    }
    // The diffuse branch's direction sample (the two draws after the Fresnel
    // draw, sincos of the azimuth, the two square roots) computed before the
    // material is known, from a copy of the generator: it depends on the
    // generator alone, so it interleaves with the hit's normal / Fresnel
    // chain instead of trailing it; committed only when the bounce takes that
    // branch.  VR_SPEC_SAMPLE 2: before fill_hit, 1: after it, 0: off.  On in
    // the Cornell-box service and one-frame kernels, whose bounces are almost
    // all diffuse (C2 16-frame steps +0.5 %, one frame per call 0.718 ->
    // 0.714 ms, r05s); the HDRI kernels spilled with it (C3 one frame +1 %)
    // and the 7-wave whole-frame kernel spilled 4 VGPRs.
#ifndef VR_SPEC_SAMPLE
#define VR_SPEC_SAMPLE 2
#endif
#ifndef VR_SPEC_HDRI_SVC
#define VR_SPEC_HDRI_SVC 0
#endif
// (also measured, off: the HDRI service kernels -- C3 -0.4 %, C5 +0.3 %,
// noise -- and the Cornell whole-frame kernel: ±0, r05v)
#ifndef VR_SPEC_WHOLE
#define VR_SPEC_WHOLE 0
#endif
    constexpr bool SPEC = VR_SPEC_SAMPLE != 0 && !ref_alg<COUNT, FEAT>() && (FEAT & (F_BRDF | F_VIEW_BRDF)) == 0u &&
                          (((FEAT & F_CORNELL) != 0u &&
                            ((FEAT & (F_SERVICE | F_INLINE_PRIM)) != 0u || (VR_SPEC_WHOLE != 0 && (FEAT & F_SMALL) == 0u))) ||
                           (VR_SPEC_HDRI_SVC != 0 && (FEAT & F_SERVICE) != 0u));
    Rng srng = ps.rng;
    float su0 = 0.f, srand2s = 0.f, srand1m = 0.f, ssn = 0.f, scs = 0.f;
    auto spec_sample = [&]() {
        su0 = srng.uniform();
        const float rand1 = 2.f * VR_PI * srng.uniform();
        const float rand2 = srng.uniform();
        srand2s = sqrt_exact(rand2);
        srand1m = sqrt_exact(1 - rand2);
        sincos_p(rand1, &ssn, &scs);
    };
    if constexpr (SPEC && VR_SPEC_SAMPLE == 2) spec_sample();
    Hit h;
    fill_hit<FEAT>(p, ray, hr, h);
    if constexpr (SPEC && VR_SPEC_SAMPLE == 1) spec_sample();
    if (COUNT) {
        if (hr.kind == HK_MESH) {
            cnt.attr += 24 + 48;
            cnt.mesh_hits++;
            const bool vb = HAS(F_VIEW_BRDF);
            const uint32_t nt = (HAS(F_TEX_DIFF) && !vb) + (HAS(F_TEX_SPEC) && !vb);
            cnt.tex += nt;
            cnt.ld128 += nt;
            // the kernel specialised on the scene's features loads the uvs
            // only when a texture is bound and the tangents only for a normal
            // map or a BRDF (the generic kernel counting here loads both)
            if ((p.flags & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u) cnt.ld64 += 3;
            if ((p.flags & (F_TEX_NORM | F_BRDF)) != 0u) cnt.ld128 += 3;
            if (HAS(F_TEX_NORM) && dot4(h.tan, h.tan) > VR_EPS) {
                cnt.attr += 48; cnt.tex++; cnt.nmap_hits++;
                cnt.ld128 += 3 + 1;                            // normals + the normal-map texel
            } else if (!ref_alg<COUNT, FEAT>()) {
                // the face normal's edges (face_from_edges) or vertices (the
                // reference has them from its triangle test)
                cnt.attr += face_from_edges<FEAT>() ? 24 : 36;
                cnt.ld96 += face_from_edges<FEAT>() ? 2 : 3;
            }
        } else if (hr.kind == HK_EXAMPLE) {
            const bool vb = HAS(F_VIEW_BRDF);
            const uint32_t nt = (HAS(F_TEX_DIFF) && !vb) + (HAS(F_TEX_SPEC) && !vb) + (HAS(F_TEX_NORM) != 0);
            cnt.tex += nt;
            cnt.ld128 += nt;
        }
    }
    if (DEPTH && ps.bounce == 0) ps.depth = depth_term(ray.o, h.hp);
    ps.accum = add4(ps.accum, mul4(ps.mask, h.em));
    ray.o = h.hp;
    const vr4 normal = h.n;
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
        const bool reflect = ((SPEC ? su0 : ps.rng.uniform()) < fe);
        vr4 newdir;
        const vr4 w = normal;
        const vr4 axis = __builtin_fabsf(w.x) > 0.1f ? mk4(0.f, 1.f, 0.f, 0.f) : mk4(1.f, 0.f, 0.f, 0.f);
        if (reflect) {
            if constexpr (SPEC) (void)ps.rng.uniform();        // the Fresnel draw only
            muleq4(ps.mask, h.spec);
            newdir = normalize4(sub4(ray.d, mul4s(mul4s(normal, 2.f), dot4(normal, ray.d))));
        } else if constexpr (SPEC) {
            ps.rng = srng;                                      // the three draws
            const vr4 u = normalize4(cross4(axis, w));
            const vr4 v = cross4(w, u);
            newdir = normalize4(add4(add4(mul4s(mul4s(u, scs), srand2s), mul4s(mul4s(v, ssn), srand2s)),
                                     mul4s(w, srand1m)));
            muleq4(ps.mask, h.col);
            muleq4s(ps.mask, dot4(newdir, normal));
            muleq4s(ps.mask, 2.f);
        } else {
            float rand1 = 2.f * VR_PI * ps.rng.uniform();
            float rand2 = ps.rng.uniform();
            probe_coherent(rand1, rand2);
            const float rand2s = sqrt_exact(rand2);
            const vr4 u = normalize4(cross4(axis, w));
            const vr4 v = cross4(w, u);
            float sn, cs;
            sincos_p(rand1, &sn, &cs);
            newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                     mul4s(w, sqrt_exact(1 - rand2))));
            muleq4(ps.mask, h.col);
            muleq4s(ps.mask, dot4(newdir, normal));
            muleq4s(ps.mask, 2.f);
        }
        ray.o = add4(ray.o, mul4s(normal, 0.05f));
        ray.d = newdir;
    } else if (h.type == 2) {                                            // :724-764
        const vr4 w = normal;
        const vr4 axis = __builtin_fabsf(w.x) > 0.1f ? mk4(0.f, 1.f, 0.f, 0.f) : mk4(1.f, 0.f, 0.f, 0.f);
        float rand1 = 2.f * VR_PI * ps.rng.uniform();
        float rand2 = ps.rng.uniform();
        probe_coherent(rand1, rand2);
        const float rand2s = sqrt_exact(rand2);
        const vr4 u = normalize4(cross4(axis, w));
        const vr4 v = cross4(w, u);
        float sn, cs;
        sincos_p(rand1, &sn, &cs);
        const vr4 newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                           mul4s(w, sqrt_exact(1 - rand2))));
        if HAS(F_BRDF) {
            const float dw = 24 * pow_p(newdir.x * newdir.x + newdir.y * newdir.y + newdir.z * newdir.z, -1.5f);
            if (COUNT) { cnt.brdf++; cnt.ld96 += 1; }
            const vr4 b = lookup_brdf(p.brdf, newdir, ray.d, h.n, h.tan);
            const vr4 bm = mk4(__builtin_fmaxf(b.x, 0.f), __builtin_fmaxf(b.y, 0.f), __builtin_fmaxf(b.z, 0.f),
                               __builtin_fmaxf(b.w, 0.f));
            muleq4(ps.mask, muls4(dw, bm));
        } else {
            muleq4(ps.mask, h.col);
            muleq4s(ps.mask, dot4(newdir, normal));
            muleq4s(ps.mask, 2.f);
        }
        ray.o = add4(ray.o, mul4s(normal, 0.05f));
        ray.d = newdir;
    }
    ++ps.bounce;
    // the production kernels ended the path at bounce 3 above, so only the
    // reference algorithm reaches a fourth here; the compiler keeps the test
    // otherwise, and the textured (C3) one-frame kernel spilled the radiance
    // around it on every bounce.  The untextured kernels keep it: they have
    // no spill there, and without it C2 lost 0.5 % (code placement) and C5's
    // one-frame kernel gained a spill.
    constexpr bool LIVE4 = ref_alg<COUNT, FEAT>() || (FEAT & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) == 0u;
    if (LIVE4 && ps.bounce == 4) {
        ps.accum.w = ps.depth;
        out = ps.accum;
        sink(out);
        return true;
    }
    return false;
}

template <int STACK, bool COUNT, uint32_t FEAT>
__device__ __forceinline__ vr4 trace(const RenderParams& p, Ray ray, const HitRec& hr0, bool hit0, uint32_t& s0, uint32_t& s1,
                     const Lds& L, Cnt& cnt, float& depth)
{
    PathState ps;
    path_begin(ps, s0, s1);
    for (;;) {
        HitRec hr;
        if (!ref_alg<COUNT, FEAT>() && ps.bounce == 0) {
            // the camera ray is the same for both samples of every frame (no
            // jitter, PathTracer.cu:842-844): its hit is computed once per pixel
            hr = hr0;
            (void)hit0;
        } else if (intersect_spheres<COUNT, FEAT>(p, ray, hr, cnt) && mesh_needed<COUNT, FEAT>(p, hr, ps.bounce)) {
            traverse_mesh<STACK, COUNT, FEAT>(p, ray, hr, L, cnt, any_hit_enough<COUNT, FEAT>(p, ps.bounce));
        }
        vr4 out;
        if (bounce_step<COUNT, FEAT>(p, ray, hr, ps, out, cnt)) { depth = ps.depth; return out; }
    }
}

// One colour byte of the tonemap (PathTracer.cu:850-866): f2u8 of
// pow(c, 1/2.2) * 255 for the clamped channel c in [0, 1] (clampf maps NaN
// to 1 and leaves -0.0, whose byte is 0).
__device__ __forceinline__ unsigned char tone_byte_ref(float c) { return f2u8(pow_p(c, 1.f / 2.2f) * 255); }
// The same byte from the context's threshold table (RenderParams::tone_t,
// tone_table_kernel): T[k] = the smallest c with tone_byte_ref(c) >= k, so
// the byte is the number of thresholds in (0, c] -- found from the hardware
// log2 / exp2 estimate (off by at most one) and checked against T[k] and
// T[k + 1].  Equal to tone_byte_ref for every float in [-0, 1]: an
// exhaustive comparison (vrhip_selftest_tonemap) shows the byte is
// monotonic there.  Two table loads instead of the f64 log2 / exp2 of
// pow_p: the one-frame finish pass 23.4 -> 16.9 us on C2 (r05w).
__device__ __forceinline__ unsigned char tone_byte(float c, const float* __restrict__ T)
{
    int k = (int)(__builtin_amdgcn_exp2f(__builtin_amdgcn_logf(c) * (1.f / 2.2f)) * 255.f);
    k = k < 0 ? 0 : (k > 255 ? 255 : k);
    while (k < 255 && c >= T[k + 1]) ++k;
    while (k > 0 && c < T[k]) --k;
    return (unsigned char)k;
}
// colour of the accumulated radiance after `frame` frames (PathTracer.cu:850-866)
__device__ __forceinline__ u8x4 tonemap(vr4 io, uint32_t frame, const float* __restrict__ T) {
    const float coef = 1.f / (float)frame;
    const vr4 sc = mul4s(io, coef);
    u8x4 c;
    if (T) {
        c.x = tone_byte(clampf(sc.x, 0.f, 1.f), T);
        c.y = tone_byte(clampf(sc.y, 0.f, 1.f), T);
        c.z = tone_byte(clampf(sc.z, 0.f, 1.f), T);
    } else {
        c.x = tone_byte_ref(clampf(sc.x, 0.f, 1.f));
        c.y = tone_byte_ref(clampf(sc.y, 0.f, 1.f));
        c.z = tone_byte_ref(clampf(sc.z, 0.f, 1.f));
    }
    c.w = 0xff;
    return c;
}

// A path's result in the scratch (RenderParams::paths): its radiance, 12 B.
// The .w bounce_step returns is the primary hit's depth term (ps.depth, set
// at bounce 0, the same for every path of a pixel: no camera jitter) on
// every exit but a Cornell escape, which returns 0 and marks itself with
// x = -0.0.  So .w is not stored per path: path 0 of the pixel stores the
// depth term once (path_w) and finish_kernel rebuilds each path's .w from
// it and the escape mark -- a quarter less scratch written by the path
// kernel and read by the (HBM-bound) finish pass.
__device__ __forceinline__ bool escaped(float x) { return __float_as_uint(x) == 0x80000000u; }
// Split sphere launches (render_kernel with RenderParams::split > 1): a pixel
// whose camera ray escapes (shared_miss) has the same result for every path,
// so group 0 stores it once -- paths[0][slot] -- and marks the pixel with a
// depth term of -1 (a real one is >= 0); the other groups store nothing and
// finish_kernel adds that one result for every path, in path order.
constexpr float kSharedMissW = -1.0f;
// The listed pixel count of an F_SPARSE launch, after the drained-queue
// mask (a render-service session: in its device control block).
__device__ __forceinline__ uint32_t* sparse_count_of(uint32_t* chunk_ctr) { return chunk_ctr + VR_MAX_QUEUES * kQueueStride + 2u; }
__device__ __forceinline__ uint32_t* sparse_count(const RenderParams& p)
{
    return p.svc_dev ? &p.svc_dev->sparse_n : sparse_count_of(p.chunk_ctr);
}
__device__ __forceinline__ void store_path(const RenderParams& p, uint32_t q, uint32_t slot, const vr4& out, float depth)
{
    p.paths[(size_t)q * p.path_stride + slot] = vr3{ out.x, out.y, out.z };
    if (q == 0u) p.path_w[slot] = depth;
}
// the radiance only: primary_kernel stored the pixel's depth term
__device__ __forceinline__ void store_path_rgb(const RenderParams& p, uint32_t q, uint32_t slot, const vr4& out)
{
    p.paths[(size_t)q * p.path_stride + slot] = vr3{ out.x, out.y, out.z };
}

// Binds this thread's stack column and fills the block's node cache with
// the first nodes of the area-ordered node array.
template <uint32_t FEAT, int BT = kBlockThreads>
__device__ __forceinline__ Lds lds_setup(const RenderParams& p, int* lds_stack, vr4* lds_nodes, int2* lds_idx,
                                         int cn, int tid)
{
    Lds L;
    L.stk = lds_stack + tid;
    L.stride = BT;
    L.nodes = lds_nodes;
    L.idx = lds_idx;
    L.n_cached = 0;
    if (HAS(F_MESH)) {
        if (!HAS(F_STRICT)) {            // fp16 nodes, 32 B: 1.5x as many fit
            const uint32_t cap = (uint32_t)(3 * cn / 2);
            L.n_cached = (int)(p.n_nodes < cap ? p.n_nodes : cap);
            for (int i = tid; i < 2 * L.n_cached; i += BT) lds_nodes[i] = p.bvh16[i];
        } else {
            L.n_cached = (int)(p.n_nodes < (uint32_t)cn ? p.n_nodes : (uint32_t)cn);
            for (int i = tid; i < 3 * L.n_cached; i += BT) lds_nodes[i] = p.bvh[(i / 3) * 4 + i % 3];
            for (int i = tid; i < L.n_cached; i += BT)
                lds_idx[i] = *reinterpret_cast<const int2*>(p.bvh + 4 * i + 3);
        }
        __syncthreads();
    }
    return L;
}

// Camera ray through pixel (x, y) (PathTracer.cu:842-844: no jitter).
__device__ __forceinline__ Ray camera_ray(const RenderParams& p, uint32_t x, uint32_t y)
{
    // (float)((0.25 + x) / W - 0.5) and the same for y, evaluated in double
    // on the host once per column / row (vrhip_create)
    const float sx = p.cam_sxy[x];
    const float sy = p.cam_sxy[p.W + y];
    Ray cam;
    cam.o = p.cam_o;
    cam.d = normalize4(add4(add4(p.cam_d, mul4s(p.cx, sx)), mul4s(p.cy, sy)));
    return cam;
}

// render (PathTracer.cu:791-868), K frames per launch.
#ifndef VR_MIN_WAVES_PER_SIMD
#define VR_MIN_WAVES_PER_SIMD 4
#endif
// 64-entry stacks take 64 KiB of LDS per 256 threads: at most 2 waves/SIMD
constexpr int min_waves(int stack) { return stack > 32 ? 2 : VR_MIN_WAVES_PER_SIMD; }
// Sphere-only kernels (no F_MESH in FEAT: C1, C4 and the sphere classes) have
// no traversal stack or node cache in LDS, and ask for this many waves per
// SIMD: their paths are chains of dependent gathers (BRDF table, HDRI) and
// portable-libm transcendentals.  r04 (`scripts/ab.py`, against the kernels
// with the mesh kernels' 40-KB LDS footprint, 4 waves): 4 / 6 / 8 waves C4
// +2.0 / +1.6 / -14.5 %, C1 +2.1 / +4.4 / +2.7 % (8: 17 and 6 VGPRs spilled).
#ifndef VR_SPHERE_MIN_WAVES
#define VR_SPHERE_MIN_WAVES 6
#endif
template <uint32_t FEAT>
constexpr int render_waves(int stack) { return (FEAT & F_MESH) != 0u ? min_waves(stack) : VR_SPHERE_MIN_WAVES; }
template <int STACK, bool COUNT, uint32_t FEAT>
__global__ void __launch_bounds__(kBlockThreads, render_waves<FEAT>(STACK)) render_kernel(const RenderParams p)
{
    constexpr bool MK = (FEAT & F_MESH) != 0u;           // a kernel that may traverse the mesh
    constexpr int CN = MK ? cache_nodes(STACK) : 1;
    __shared__ int lds_stack[MK ? STACK * kBlockThreads : 1];
    __shared__ vr4 lds_nodes[3 * CN];
    __shared__ int2 lds_idx[CN];
    const int tid = threadIdx.x;
    const Lds L = lds_setup<FEAT>(p, lds_stack, lds_nodes, lds_idx, CN, tid);
    // block -> (tile, path group): the 2*n_frames paths of a pixel are split
    // into p.split contiguous groups run by different blocks (strong-scaling
    // and tail balance); group g of tile t is block t*split + g
    const uint32_t T = p.split;
    const uint32_t tile = blockIdx.x / T;
    const uint32_t g = blockIdx.x - tile * T;
    const int wave = tid >> 6, lane = tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;      // tiles dealt round-robin to ranks
    const uint32_t tile_y = tile_row(gtile, p.tiles_x);
    const uint32_t tile_x = tile_col(gtile, p.tiles_x, p.nranks);
    const uint32_t x = tile_x * 16u + (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t y = tile_y * 16u + (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    if (x >= p.wr || y >= p.hr) return;   // never true for a valid launch
    Cnt cnt;

    const uint32_t ind = x + y * p.W;
    const Ray cam = camera_ray(p, x, y);
    HitRec hr0;
    bool hit0 = false;
    if (!ref_alg<COUNT, FEAT>()) hit0 = intersect_scene<STACK, COUNT, FEAT>(p, cam, hr0, L, cnt);
    // Shared escape: in an HDRI scene a camera ray that escapes gives every
    // path of the pixel the same result -- the first bounce's miss branch
    // (:631-648) with mask 1, no jitter (:842-844) and no random number drawn
    // -- so it is evaluated once per pixel (one HDRI fetch instead of one per
    // path) and the paths' sums below stay in path order, bit for bit the
    // same.  ~98 % of C4's paths (the sphere covers ~2 % of the image).
    const bool shared_miss = !ref_alg<COUNT, FEAT>() && !HAS(F_CORNELL) && !hit0;
    // path q = 2*f + s (frame f of the launch, sample s); the seeds of a
    // frame's second sample are its first sample's after one hash (:620-622)
    const uint32_t n_paths = 2u * p.n_frames;
    const uint32_t chunk = (n_paths + T - 1u) / T;
    const uint32_t q0 = g * chunk < n_paths ? g * chunk : n_paths;
    const uint32_t q1 = q0 + chunk < n_paths ? q0 + chunk : n_paths;
    const bool direct = !p.use_scratch;                  // accumulate here (counting launches)
    // split launches: an escaped pixel's group 0 stores its one record
    // (kSharedMissW) and no group runs its paths
    const bool one_record = shared_miss && !direct;
    vr4 miss_r = mk4(0.f, 0.f, 0.f, 0.f);
    if (shared_miss && (direct || g == 0u)) {
        PathState ps;
        uint32_t d0 = 0, d1 = 0;                           // the miss branch draws no random number
        path_begin(ps, d0, d1);
        Ray r0 = cam;
        (void)bounce_step<COUNT, FEAT>(p, r0, hr0, ps, miss_r, cnt);
        if (one_record) {
            const uint32_t slot = tile * kBlockThreads + (uint32_t)tid;
            p.paths[slot] = vr3{ miss_r.x, miss_r.y, miss_r.z };
            p.path_w[slot] = kSharedMissW;
        }
    }
    if (COUNT && one_record) cnt.shared_miss += q1 - q0;
    const uint32_t q_end = one_record ? q0 : q1;
    vr4 io = (direct && p.first_frame != 1u) ? p.accum[ind] : mk4(0.f, 0.f, 0.f, 0.f);
    uint32_t s1 = 0, s2 = 0;
    float last_w = 0.f;
#pragma unroll 1
    for (uint32_t q = q0; q < q_end; ++q) {
        const uint32_t f = q >> 1;
        if ((q & 1u) == 0u || q == q0) {
            s1 = x * (p.first_frame + f);
            s2 = y * p.times[f];
            if (q & 1u) (void)hash_seeds(s1, s2);
        }
        float depth = 1.f;
        vr4 result = miss_r;
        if (shared_miss) {
            if (COUNT) cnt.shared_miss++;
        } else {
            result = trace<STACK, COUNT, FEAT>(p, cam, hr0, hit0, s1, s2, L, cnt, depth);
        }
        if (direct)
            io = add4(io, mul4s(result, 1.f / 2.f));
        else
            store_path(p, q, tile * kBlockThreads + (uint32_t)tid, result, depth);
        last_w = result.w;
    }
    if (direct) {   // else finish_kernel accumulates the paths' results in path order
        // only the launch's last frame is observable in the colour and depth
        // surfaces (each frame of the reference overwrites them, :846-866)
        const unsigned char db = f2u8((1.f - last_w) * 255);
        u8x4 dv; dv.x = db; dv.y = db; dv.z = db; dv.w = 0xff;
        p.depth[ind] = dv;
        p.rgba[ind] = tonemap(io, p.first_frame + p.n_frames - 1u, p.tone_t);
        p.accum[ind] = io;
    }
    if (COUNT) flush_counts(p, cnt, lane, (FEAT & F_COUNT_EXEC) != 0u);
}

// Specialisations that may run F_SPARSE launches: HDRI mesh scenes (an
// escaped camera ray ends the path at once), exact or feature-class kernels,
// multi-frame launches with a primary pass.
template <uint32_t FEAT>
constexpr bool sparse_ok() {
    return (FEAT & F_MESH) != 0u && (FEAT & F_CORNELL) == 0u && (FEAT & (F_EXACT | F_CLASS)) != 0u &&
           (FEAT & (F_INLINE_PRIM | F_SMALL | F_SERVICE)) == 0u;
}

// Kernels without the example sphere (whose hits need the u,v slots) store
// the camera ray's direction in the primary record instead, so a path starts
// without recomputing it (two f64 divisions and a normalisation).
template <uint32_t FEAT>
constexpr bool prim_has_dir() { return (FEAT & F_EXAMPLE) == 0; }

// The camera origin for a path that starts from its primary record.  The
// 7-wave C2 kernel's only VGPR spills are vector copies of it (two scratch
// stores per wave in the prologue, two reloads per refill: ~4 MB of the
// launch's 996 MiB WRITE_SIZE, so not the write amplification -- DESIGN.md 5).
// With VR_CAM_RELOAD it is reloaded from the kernel argument segment at the
// point of use instead: 0 spills, but slower -- C2 -1.0 %, C3 -1.6 %, C5
// -3.0 % (r04, scripts/ab.py): the allocator's other choices cost more than
// the reloads did.  Off.
#ifndef VR_CAM_RELOAD
#define VR_CAM_RELOAD 0
#endif
static_assert(offsetof(RenderParams, cam_o) == 0, "cam_o leads the kernel argument");
__device__ __forceinline__ vr4 cam_origin(const RenderParams& p)
{
#if VR_CAM_RELOAD
    const vr4* k = (const vr4*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));                 // opaque: reloaded at every use
    (void)p;
    return *k;
#else
    return p.cam_o;
#endif
}

// Primary hits, one thread per owned pixel: the camera ray's closest hit
// (the HitRec intersect_scene returns: t, kind, idx, barycentrics,
// example-sphere u,v), two float4s per pixel in the scratch order of
// p.paths, read by every path of the pixel in render_wave_kernel.  One ray
// per thread, so no LDS node cache.
template <int STACK, uint32_t FEAT>
__global__ void __launch_bounds__(kBlockThreads) primary_kernel(const RenderParams p)
{
    __shared__ int lds_stack[STACK * kBlockThreads];
    const int tid = threadIdx.x;
    Lds L;
    L.stk = lds_stack + tid;
    L.stride = kBlockThreads;
    L.nodes = nullptr;
    L.idx = nullptr;
    L.n_cached = 0;
    const uint32_t tile = blockIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const uint32_t gtile = p.rank + tile * p.nranks;      // tiles dealt round-robin to ranks
    const uint32_t tile_y = tile_row(gtile, p.tiles_x);
    const uint32_t tile_x = tile_col(gtile, p.tiles_x, p.nranks);
    const uint32_t x = tile_x * 16u + (uint32_t)((wave & 1) * 8 + (lane & 7));
    const uint32_t y = tile_y * 16u + (uint32_t)((wave >> 1) * 8 + (lane >> 3));
    constexpr bool CNT = (FEAT & F_COUNT_EXEC) != 0u;
    Cnt cnt;
    HitRec hr;
    const Ray cam = camera_ray(p, x, y);
    const bool hit = intersect_scene<STACK, CNT, FEAT>(p, cam, hr, L, cnt);
    const uint32_t slot = tile * kBlockThreads + (uint32_t)tid;
    vr4* dst = p.prim + 2u * (size_t)slot;
    dst[0] = mk4(hr.t, __int_as_float(hr.kind), __int_as_float(hr.idx), hr.bu);
    // the pixel's depth term for the path kernel's finish pass (bounce 0 is
    // this hit for every path; 1 when the camera ray escapes, path_begin)
    {
        const float dt = hit ? depth_term(cam.o, add4(cam.o, mul4s(cam.d, hr.t))) : 1.f;
        if (p.svc_dev) reinterpret_cast<float*>(p.paths + (size_t)2u * p.svc_kmax * p.path_stride)[slot] = dt;
        else p.path_w[slot] = dt;
    }
    if constexpr (prim_has_dir<FEAT>())
        dst[1] = mk4(hr.bv, cam.d.x, cam.d.y, cam.d.z);   // the paths reuse the camera ray too
    else
        dst[1] = mk4(hr.bv, hr.su, hr.sv, 0.f);
    if constexpr (sparse_ok<FEAT>()) {
        if (p.sparse_px) {
            // F_SPARSE launch: an escaped camera ray gives every path of the
            // pixel the same result (render_kernel's shared escape), stored
            // once; the pixels that hit the scene join the path kernel's list
            // (one atomic per wave, the wave's hits contiguous: an 8x8
            // sub-tile's pixels stay together in the path kernel's chunks)
            if (!hit) {
                PathState ps;
                uint32_t d0 = 0, d1 = 0;                   // the miss branch draws no random number
                path_begin(ps, d0, d1);
                Ray r0 = cam;
                vr4 miss_r;
                (void)bounce_step<CNT, FEAT>(p, r0, hr, ps, miss_r, cnt);
                if (p.svc_dev) {
                    // a render-service session: the result serves every launch
                    // of the session, kept in the pixel's primary record
                    // (svc_finish_kernel reads it there)
                    dst[1] = mk4(0.f, miss_r.x, miss_r.y, miss_r.z);
                } else {
                    p.paths[slot] = vr3{ miss_r.x, miss_r.y, miss_r.z };
                    p.path_w[slot] = kSharedMissW;
                }
                if (CNT) cnt.shared_miss += 2u * p.n_frames;
            }
            const unsigned long long hm = __ballot(hit);
            if (hm != 0ull) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(sparse_count(p), (uint32_t)__popcll(hm));
                base = (uint32_t)__shfl((int)base, 0, 64);
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
                if (hit) p.sparse_px[base + r] = slot;
            }
        }
    }
    if (CNT) flush_counts(p, cnt, lane, true);
}

// Path-pool render (the default for mesh scenes), a persistent kernel over
// work queues.  The launch's paths are cut into chunks of 64 items: chunk =
// (sub-tile s, path q), s an 8x8 quadrant of one of the rank's tiles, item i
// = pixel i of s.  The grid is one resident wave set; each wave takes chunks
// from the queues and its lanes run one path each through a small state
// machine (setup = sphere tests, traverse the mesh, shade).  A lane whose path
// ends stores the radiance to p.paths[q][pixel] and takes the next item
// (ballot + mbcnt give each idle lane its item in one wave-uniform step), so
// lanes whose rays finish early do not idle while the wave's other lanes
// traverse, and no wave waits at the end of the launch for blocks of uneven
// cost.  Traversal pauses between outer iterations (trav_iter) once
// VR_SHADE_BATCH lanes wait for shading.
//
// Primary hits: the camera ray is the same for every path of a pixel (no
// jitter, PathTracer.cu:842-844), so primary_kernel traces it once per pixel
// per launch and every path of the pixel starts at its shading.  Launches of
// one frame (2 paths per pixel, the reference's render() cadence) skip that
// serial pass (RenderParams::inline_prim): each path traces its camera ray in
// the pool, where the primary pass's latency tail overlaps other lanes' work.
//
// Every path runs exactly the operations of trace(); only the interleaving
// of paths on the SIMD changes, so results are bit-identical.
// finish_kernel then sums each pixel's paths in path order.
#ifndef VR_SHADE_BATCH
#define VR_SHADE_BATCH 16
#endif
#ifndef VR_SHADE_RATIO
#define VR_SHADE_RATIO 1
#endif
// Once the queues are drained, the paths waiting to be shaded are shaded
// together once n_shade * VR_DRAIN_SHADE_NUM >= n_trav * VR_DRAIN_SHADE_DEN
// (or no lane traverses): each shading round costs the wave a whole pass
// through the shading code, and in the drain the traversing lanes' paths --
// the launch's longest -- wait through every such round.  Measured (r03o,
// one frame per call; 8-rank shard steps): shading at the first waiting
// path C3 0.504 / C2 0.765 ms, 0.631 / 1.333 ms; at n_shade >= n_trav 0.470 /
// 0.731, 0.612 / 1.343; at 2 n_shade >= n_trav 0.476 / 0.740.
#ifndef VR_DRAIN_SHADE_NUM
#define VR_DRAIN_SHADE_NUM 1
#endif
#ifndef VR_DRAIN_SHADE_DEN
#define VR_DRAIN_SHADE_DEN 1
#endif
enum LaneState : int { LS_SETUP = 0, LS_TRAV = 1, LS_SHADE = 2, LS_DONE = 3, LS_CAMERA = 4, LS_HELP = 5, LS_HELPDONE = 6 };

// Helpers (the launch's drain).  Once the work queues are empty, a wave's
// lanes idle as their paths end while a few lanes still walk long
// traversals -- the paths that end the launch.  Then an idle lane takes the
// top entry of a traversing lane's stack (a subtree or a leaf the owner
// would visit next), walks it with the owner's ray, its closest hit so far
// and its culling distance, and hands its closest hit back; the owner shades
// once its own walk and all its helpers' are done.  The closest hit does not
// depend on the order in which subtrees are visited: a triangle at exactly
// the closest distance is resolved by the reference's own order (ref_first),
// so the merged hit is the reference's.  Not used by the strict walk, whose
// exact result relies on the reference's visit order.
#ifndef VR_HELPERS
#define VR_HELPERS 1
#endif
template <uint32_t FEAT>
constexpr bool helpers() { return VR_HELPERS != 0 && (FEAT & F_STRICT) == 0u && (FEAT & F_SMALL) != 0u; }

// One wave-synchronous help round: (1) finished helpers hand their closest
// hit to their owners, one at a time; (2) idle lanes take a subtree each from
// traversing lanes (one per owner per round, pairing the k-th idle lane with
// the k-th owner).  For helpers `slot` holds the owner's lane.
__device__ __forceinline__ uint32_t help_step(const RenderParams& p, int lane, int& state, int& pend, uint32_t& slot,
                                              Ray& ray, Trav& tr, const Lds& L)
{
    unsigned long long hd = __ballot(state == LS_HELPDONE);
    while (hd != 0ull) {
        const int h = __ffsll((long long)hd) - 1;
        hd &= hd - 1ull;
        const int o = __builtin_amdgcn_readlane((int)slot, h);
        const float ht = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tr.t), h));
        const int hb = __builtin_amdgcn_readlane(tr.best, h);
        const float hu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tr.bu), h));
        const float hv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tr.bv), h));
        if (lane == o) {
            // the helper started from this lane's closest hit at the hand-out:
            // it returns that one, a closer one, or a tie it resolved
            const bool closer = hb >= 0 && (ht < tr.t || (ht == tr.t && hb != tr.best &&
                                                          (tr.best < 0 || ref_first(p, tr, hb / 3, tr.best / 3))));
            if (closer) {
                tr.t = ht; tr.best = hb; tr.bu = hu; tr.bv = hv;
                tr.tcull = tr.t * 1.0009765625f;
            }
            --pend;
        }
        if (lane == h) state = LS_DONE;
    }
    // helpers cull with the owner's closest hit as it improves
    const int own = state == LS_HELP ? (int)slot : lane;
    const float ot = __shfl(tr.t, own, 64);
    if (state == LS_HELP) tr.tcull = __builtin_fminf(tr.tcull, ot * 1.0009765625f);
    const bool idle = state == LS_DONE;
    const bool can = state == LS_TRAV && tr.nodeAddr != kSentinel && tr.sp >= 1;
    const unsigned long long im = __ballot(idle), cm = __ballot(can);
    if (im == 0ull || cm == 0ull) return 0u;
    const uint32_t ni = (uint32_t)__popcll(im), nc = (uint32_t)__popcll(cm), n = ni < nc ? ni : nc;
    const uint32_t rc = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
    const uint32_t ri = __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
    int give = 0;
    if (can && rc < n) {                                   // the owner hands out its next stack entry
        give = L.stk[tr.sp * L.stride];
        tr.sp--;
        ++pend;
    }
    int src = lane;                                        // idle lane ri takes the ri-th owner
    unsigned long long m = cm;
    for (uint32_t k = 0; k < n; ++k) {
        const int ol = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        if (idle && ri == k) src = ol;
    }
    const bool take = idle && ri < n;
    const int e = __shfl(give, src, 64);
    auto pull = [&](float& v) { v = __shfl(v, src, 64); };
    pull(ray.o.x); pull(ray.o.y); pull(ray.o.z); pull(ray.o.w);
    pull(ray.d.x); pull(ray.d.y); pull(ray.d.z); pull(ray.d.w);
    pull(tr.ivx); pull(tr.ivy); pull(tr.ivz); pull(tr.odx); pull(tr.ody); pull(tr.odz);
    pull(tr.t); pull(tr.tcull); pull(tr.bu); pull(tr.bv);
    tr.best = __shfl(tr.best, src, 64);
    if (take) {
        state = LS_HELP;
        slot = (uint32_t)src;
        tr.sp = 0;
        L.stk[0] = kSentinel;
        tr.nodeAddr = e;
    }
    return n;                                              // subtrees handed out this round
}
// Age-based wave priority (s_setprio) in the path kernel, thresholds in us:
// VR_AGE_PRIO 1 in every path kernel, 2 in the one-frame kernels only
// (F_INLINE_PRIM: the reference's render() cadence, where a launch ends on
// its oldest paths), 0 off.  Measured (r03e, 1xMI355X): one frame per call
// C2 0.840 -> 0.799 ms, C3 0.564 -> 0.570 (noise); 16-frame launches C2
// -0.4 %, C3 -0.1 %.
#ifndef VR_AGE_PRIO
#define VR_AGE_PRIO 2
#endif
template <uint32_t FEAT>
constexpr bool age_prio() { return VR_AGE_PRIO == 1 || (VR_AGE_PRIO == 2 && (FEAT & F_INLINE_PRIM) != 0u); }
#ifndef VR_AGE_T1
#define VR_AGE_T1 100
#endif
#ifndef VR_AGE_T2
#define VR_AGE_T2 200
#endif
#ifndef VR_AGE_T3
#define VR_AGE_T3 300
#endif


// Block size of the path kernel: its blocks hold no tiles, so one block of
// 1,024 threads per CU shares one LDS node cache four times the size of a
// 256-thread block's (at the same 4 waves/SIMD).
// Path-kernel residency by stack size: with 16- and 24-entry stacks (C2, C3;
// C5) VR_PATH_WAVES waves per SIMD in VR_PATH_BLOCK-thread blocks; 32-entry
// stacks 4 waves in one 1,024-thread block per CU (the stacks alone take
// 128 KB); 64-entry stacks 2 waves in 256-thread blocks.  Measured (C2 / C3,
// no packed f32): 4 waves in 1,024 threads 3,029 / 10,724; 5 in 256: 2,956 /
// 10,503; 6 in 256: 3,228 / 11,352; 6 in 512: 2,952 / 10,483; 6 in 768:
// 3,406 / 12,193; 7 in 256 (spills): 3,317 / 11,290.
#ifndef VR_PATH_WAVES
#define VR_PATH_WAVES 6
#endif
#ifndef VR_PATH_BLOCK
#define VR_PATH_BLOCK 768
#endif
static_assert(VR_PATH_BLOCK % kBlockThreads == 0, "VR_PATH_BLOCK must be a multiple of 256");
static_assert((4 * VR_PATH_WAVES * 64) % VR_PATH_BLOCK == 0, "whole blocks per CU");
// Cornell-box mesh kernels with 16-entry stacks (C2) run 7 waves per SIMD in
// 256-thread blocks (72 VGPRs, SGPR spills only): C2 3,991 -> 4,109 Mpaths/s,
// while the HDRI scenes lose with it (C3 -2 %, C5 -17 %: their longer shading
// code spills) and keep VR_PATH_WAVES in VR_PATH_BLOCK-thread blocks.
#ifndef VR_PATH_WAVES_CORNELL
#define VR_PATH_WAVES_CORNELL 7
#endif
#ifndef VR_PATH_BLOCK_CORNELL
#define VR_PATH_BLOCK_CORNELL 256
#endif
static_assert(VR_PATH_BLOCK_CORNELL % kBlockThreads == 0, "VR_PATH_BLOCK_CORNELL must be a multiple of 256");
static_assert((4 * VR_PATH_WAVES_CORNELL * 64) % VR_PATH_BLOCK_CORNELL == 0, "whole blocks per CU");
// c: the kernel is a Cornell-box specialisation (cornell_kernel<FEAT>())
constexpr bool cornell_res(int stack, bool c) { return c && stack <= 16; }
constexpr int wave_block(int stack, bool c) {
    return cornell_res(stack, c) ? VR_PATH_BLOCK_CORNELL : stack <= 24 ? VR_PATH_BLOCK : stack <= 32 ? 1024 : kBlockThreads;
}
// Launches of fewer than 2^24 paths (sharded frames, RenderParams::small_blocks)
// take 256-thread blocks at the same residency: a block frees its CU slot once
// its 4 waves are done rather than 12, so the launch's drain overlaps the next
// launch sooner.  Projected 8-rank C2 step 1.283 -> 1.193 ms (C3 0.468 ->
// 0.420 ms), while whole frames keep the 768-thread blocks (C2 3,437 vs 3,244).
constexpr int wave_block_small(int stack, bool c) { return stack <= 24 ? kBlockThreads : wave_block(stack, c); }
constexpr int path_waves(int stack, bool c) {
    return cornell_res(stack, c) ? VR_PATH_WAVES_CORNELL : stack <= 24 ? VR_PATH_WAVES : stack <= 32 ? 4 : 2;
}
constexpr int path_blocks_per_cu(int stack, int bt, bool c) { return 4 * path_waves(stack, c) * 64 / bt; }
// LDS per block: an equal share of the CU's 160 KB less 256 B per 256 threads;
// the node cache takes what the stacks leave (56 B per node)
constexpr int path_cache_nodes(int stack, int bt, bool c) {
    return (163840 / path_blocks_per_cu(stack, bt, c) - bt - stack * bt * 4) / 56 > 0
               ? (163840 / path_blocks_per_cu(stack, bt, c) - bt - stack * bt * 4) / 56 : 1;
}
// The Cornell-box render-service kernels take the 7-wave residency of the
// Cornell path kernels (r05: with the single refill site and the polynomial
// constants produced at each use, 4 VGPR spills; C2 whole frames on the
// service 4,185 -> 4,313 Mpaths/s; at 6 waves they lost 2 % to the launch path)
#ifndef VR_SVC_CORNELL_RES
#define VR_SVC_CORNELL_RES 1
#endif
#ifndef VR_ONEFRAME_CORNELL_RES
#define VR_ONEFRAME_CORNELL_RES 0    // 1: one-frame Cornell kernels at the 7-wave residency (A/B builds)
#endif
template <uint32_t FEAT>
constexpr bool cornell_kernel() {
    // the one-frame kernels (F_INLINE_PRIM) keep 6 waves: at 7 the interactive
    // C2 rate fell 2,147 -> 2,100 Mpaths/s (r02g); so do the small-launch
    // kernels (F_SMALL), which spilled 19 VGPRs at 7 with helper lanes and
    // cost counting (8-rank C2 shard step 1.317 -> 1.257 ms at 6, r03p)
    if (VR_ONEFRAME_CORNELL_RES && (FEAT & F_EXACT) != 0u && (FEAT & F_CORNELL) != 0u && (FEAT & F_INLINE_PRIM) != 0u)
        return true;
    return (FEAT & F_EXACT) != 0u && (FEAT & F_CORNELL) != 0u && (FEAT & F_INLINE_PRIM) == 0u &&
           (FEAT & (F_SMALL | (VR_SVC_CORNELL_RES ? 0u : (uint32_t)F_SERVICE))) == 0u;
}

#ifndef VR_XCD_BANDS
#define VR_XCD_BANDS 128
#endif

template <int STACK, uint32_t FEAT, int BT>
__device__ __forceinline__ void wave_body(const RenderParams& p, const Lds& L);

// Pixel of item `px` of this rank's 8x8 sub-tile `sub` (wave-uniform in the
// path kernel, so the tile arithmetic, a division included, stays scalar).
__device__ __forceinline__ void sub_pixel(const RenderParams& p, uint32_t sub, uint32_t px, uint32_t& x, uint32_t& y)
{
    const uint32_t tile = sub >> 2, quad = sub & 3u;
    const uint32_t gtile = p.rank + tile * p.nranks;       // tiles dealt round-robin to ranks
    const uint32_t tile_y = tile_row(gtile, p.tiles_x);
    const uint32_t tile_x = tile_col(gtile, p.tiles_x, p.nranks);
    x = tile_x * 16u + (quad & 1u) * 8u + (px & 7u);
    y = tile_y * 16u + (quad >> 1) * 8u + (px >> 3);
}

// The launch's drained-queue mask (bit q: head q has handed out its last
// chunk), after the VR_MAX_QUEUES heads; reset with them by finish_kernel.
__device__ __forceinline__ unsigned long long* queue_drained_mask(uint32_t* chunk_ctr)
{
    return reinterpret_cast<unsigned long long*>(chunk_ctr + VR_MAX_QUEUES * kQueueStride);
}
__device__ __forceinline__ unsigned long long all_q_of(uint32_t Q) { return Q >= 64u ? ~0ull : ((1ull << Q) - 1ull); }

// The sub-tile that value v of work-queue head q hands out (>= n_sub: the
// queue is drained; non-decreasing in v), and the path in `path`.
// Chunk = (sub-tile, path): the paths of one sub-tile are handed out
// together.  With VR_XCD_BANDS queue q serves XCD q % 8 (blocks b % 16 == q
// under round-robin dispatch): bands of VR_XCD_BANDS sub-tiles are dealt
// round-robin to the XCDs, each XCD's chunks sub-major, alternated between
// its Q / 8 queues.
__device__ __forceinline__ uint32_t queue_item(uint32_t q, uint32_t v, uint32_t Q, uint32_t n_paths, uint32_t& path)
{
#if VR_XCD_BANDS
    const uint32_t x = q % 8u, h = q / 8u;
    const uint32_t e = v * (Q / 8u) + h;
    const uint32_t per_band = (uint32_t)VR_XCD_BANDS * n_paths;
    const uint32_t g = e / per_band, o = e - g * per_band;
    const uint32_t r = o / n_paths;
    path = o - r * n_paths;
    return (g * 8u + x) * (uint32_t)VR_XCD_BANDS + r;
#else
    const uint32_t c = v * Q + q;
    const uint32_t sb = c / n_paths;
    path = c - sb * n_paths;
    return sb;
#endif
}

// The textured small-launch kernels (C3 shards) keep a path's index in LDS,
// 4 B per lane taken from the node cache (wave_body lane_q)
template <uint32_t FEAT>
constexpr bool lds_q() {
    return (FEAT & F_SMALL) != 0u && (FEAT & (F_INLINE_PRIM | F_SERVICE)) == 0u &&
           (FEAT & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
}
template <int STACK, uint32_t FEAT, int BT>
__global__ void __launch_bounds__(BT, path_waves(STACK, cornell_kernel<FEAT>())) render_wave_kernel(const RenderParams p)
{
    constexpr int CN = path_cache_nodes(STACK, BT, cornell_kernel<FEAT>()) - (lds_q<FEAT>() ? (4 * BT + 55) / 56 : 0);
    __shared__ int lds_stack[STACK * BT];
    __shared__ vr4 lds_nodes[3 * CN];
    __shared__ int2 lds_idx[CN];
    const Lds L = lds_setup<FEAT, BT>(p, lds_stack, lds_nodes, lds_idx, CN, (int)threadIdx.x);
    wave_body<STACK, FEAT, BT>(p, L);
}

template <int STACK, uint32_t FEAT, int BT>
__device__ __forceinline__ void wave_body(const RenderParams& p, const Lds& L)
{
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const uint32_t n_paths = 2u * p.n_frames;
    constexpr bool SPARSE = (FEAT & F_SPARSE) != 0u;       // the listed pixels only
    // chunk rows: the 8x8 sub-tiles of the rank's tiles, or (F_SPARSE) runs
    // of 64 listed pixels -- the last run padded with the last pixel, whose
    // paths then run twice and store the same bits to the same slots
    const uint32_t n_px = SPARSE ? __builtin_amdgcn_readfirstlane(*sparse_count(p)) : 0u;
    const uint32_t n_sub = SPARSE ? (n_px + 63u) >> 6 : p.path_stride >> 6;
    constexpr bool CNT = (FEAT & F_COUNT_EXEC) != 0u;      // instrumented copy (vrhip_render_profiled)
    Cnt cnt;

    // Work queues: chunk c = (sub-tile c / n_paths, path c % n_paths), so the
    // paths of one sub-tile are handed out together (coherent rays, the
    // sub-tile's primary records in cache).  p.n_queues heads, queue j hands
    // out chunks j, j + Q, j + 2Q, ... (one device-scope atomic per chunk; a
    // single head saturates: MI355X_MICROARCH "dequeue").  A wave draws from
    // its block's queue and, once that is drained, from the following ones.
    // With VR_XCD_BANDS (default 128 sub-tiles = 32 tiles) the sub-tiles are
    // dealt to the 8 XCDs in bands, so each XCD's L2 serves a coherent part of
    // the image (C2 +0.7 %, C3 +1.7 %, C5 +0.7 % over chunk-interleaved queues).
    const uint32_t Q = p.n_queues;                         // power of two, multiple of the 8 XCDs
    uint32_t qj = blockIdx.x & (Q - 1u);
    // queues this wave knows to be drained (its own failed dequeues and the
    // launch's drained-queue mask, queue_drained_mask), kept in LDS: the
    // kernel is at its register limits and this is consulted only at the end
    __shared__ unsigned long long lds_dead[BT / 64];
    unsigned long long* const my_dead = lds_dead + (tid >> 6);
    if (lane == 0) *my_dead = 0ull;
    uint32_t drained = 0;                                  // whole-frame launches: queues found drained
    auto grab = [&](uint32_t& sub, uint32_t& path) {       // wave-uniform; sub = ~0u when no work is left
        for (;;) {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(p.chunk_ctr + qj * kQueueStride, 1u);
            const uint32_t sb = queue_item(qj, __builtin_amdgcn_readfirstlane(v), Q, n_paths, path);
            if (sb < n_sub) {
                if constexpr (SPARSE) { sub = sb; return; }   // a run of listed pixels
#if VR_XCD_BANDS
                // longest-first: the XCD's sub-tiles in the order of the
                // previous launch's cost (order_kernel); else band order
                if (p.sub_order) {
                    const uint32_t x = qj % 8u, r = sb % (uint32_t)VR_XCD_BANDS, g = sb / (8u * (uint32_t)VR_XCD_BANDS);
                    sub = p.sub_order[x * p.order_cap + g * (uint32_t)VR_XCD_BANDS + r];
                    return;
                }
#endif
                sub = sb;
                return;
            }
            // queue qj is drained.
            if constexpr ((FEAT & F_SMALL) == 0u) {
                // whole-frame launches (a drain of ~1 % of the launch; the
                // 7-wave kernel has no register to spare): the next queues
                // in turn, one failed dequeue each
                if (++drained == Q) { sub = ~0u; path = 0; return; }
                qj = qj + 1u == Q ? 0u : qj + 1u;
                continue;
            }
            // Small launches (one frame per call, shards: the drain is a large
            // share of them) publish a drained queue once (the first wave to
            // see it) and skip every queue the mask holds: a wave learns that
            // the launch is out of work from one failed dequeue and one load,
            // instead of one failed atomic on each of the Q heads -- at the end
            // of a launch all of its waves did that together, n_waves x Q
            // atomics on Q words (~88 per us per word), tens of us before the
            // grid could retire.  Every bit stands for a failed dequeue, so the
            // wave leaves only when all queues are drained.
            uint32_t m0 = 0, m1 = 0;
            if (lane == 0) {
                unsigned long long* const dmask = queue_drained_mask(p.chunk_ctr);
                // the first failed dequeue of a queue (exactly one per queue:
                // no storm of ORs on the mask word when many waves run dry at
                // once) publishes it; the others read the mask with an
                // L1-bypassing load (a stale copy only hides drained queues,
                // which then cost a failed dequeue each, as without the mask)
                uint32_t pth;
                const uint32_t v0 = __builtin_amdgcn_readfirstlane(v);
                const bool first = v0 == 0u || queue_item(qj, v0 - 1u, Q, n_paths, pth) < n_sub;
                const unsigned long long m = first ? atomicOr(dmask, 1ull << qj)
                                                   : __hip_atomic_load(dmask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long d = *my_dead | m | (1ull << qj);
                *my_dead = d;
                m0 = (uint32_t)d; m1 = (uint32_t)(d >> 32);
            }
            const unsigned long long live = all_q_of(Q) & ~(((unsigned long long)__builtin_amdgcn_readfirstlane(m1) << 32) |
                                                             (unsigned long long)__builtin_amdgcn_readfirstlane(m0));
            if (live == 0ull) { sub = ~0u; path = 0; return; }
            const unsigned long long after = qj + 1u < 64u ? (live >> (qj + 1u)) << (qj + 1u) : 0ull;
            qj = (uint32_t)__builtin_ctzll(after != 0ull ? after : live);
        }
    };
    uint32_t cur_sub, cur_q;
    grab(cur_sub, cur_q);                                  // wave-uniform: chunk being handed out
    uint32_t next = 64u;                                   // items of the current chunk handed out
    int state = LS_DONE;
    uint32_t q = 0, slot = 0;                              // this lane's path and pixel slot
    // textured one-frame kernels (C3): the path index -- 0 or 1, one frame --
    // rides in bit 0 of `slot` (slot << 1 | q): one VGPR less, and the
    // kernel no longer spills the path's throughput mask in its texture
    // shading (4 -> 0; the small-shard kernels, packed as slot | q << 24,
    // only moved theirs).  While a lane helps (help_step), `slot` holds its
    // owner's lane as everywhere.
    constexpr bool PACKQ = (FEAT & F_INLINE_PRIM) != 0u && (FEAT & (F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
    // the textured small-launch kernels keep it in LDS (lds_q: 3 spills -> 0)
    constexpr bool LDSQ = lds_q<FEAT>();
    __shared__ uint32_t lds_path[LDSQ ? BT : 1];
    auto lane_q = [&]() -> uint32_t { return PACKQ ? (slot & 1u) : LDSQ ? lds_path[tid] : q; };
    auto lane_slot = [&]() -> uint32_t { return PACKQ ? (slot >> 1) : slot; };
    uint32_t cam_xy = 0;                                   // F_INLINE_PRIM: its pixel (x << 16 | y) until LS_CAMERA
    Ray ray;
    PathState ps;
    HitRec hr;
    Trav tr;
    int pend = 0;                                          // helpers: subtrees this lane's walk handed out, not yet merged
    uint32_t born = 0;                                     // age_prio: this lane's path start (s_memrealtime, 100 MHz)
    uint32_t now_tick = age_prio<FEAT>() ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    auto start = [&](uint32_t sub, uint32_t path, uint32_t px) {   // render's per-sample prologue (:817-844)
        if (sub == ~0u) { state = LS_DONE; return; }
        q = path;
        if constexpr (LDSQ) lds_path[tid] = path;
        slot = sub * 64u + px;
        if constexpr (SPARSE) {                            // the listed pixel
            const uint32_t k = slot < n_px ? slot : n_px - 1u;
            slot = p.sparse_px[k];
        }
        const uint32_t f = q >> 1;
        uint32_t x, y;
        sub_pixel(p, slot >> 6, slot & 63u, x, y);
        uint32_t s1 = x * (p.first_frame + f);
        uint32_t s2 = y * p.times[f];
        if (q & 1u) (void)hash_seeds(s1, s2);              // the frame's second sample
        path_begin(ps, s1, s2);
        born = now_tick;
        if constexpr ((FEAT & F_SMALL) != 0u) cnt.work = 0;
        if constexpr ((FEAT & F_INLINE_PRIM) != 0u) {      // few paths per pixel: trace the camera ray here
            cam_xy = (x << 16) | y;                        // (set up at the top of the loop, out of the refill)
            if constexpr (PACKQ) slot = (slot << 1) | q;
            state = LS_CAMERA;
            return;
        }
        if (CNT) cnt.ld128 += 2;
        const vr4 a = p.prim[2u * slot], b = p.prim[2u * slot + 1u];
        hr.t = a.x; hr.kind = __float_as_int(a.y); hr.idx = __float_as_int(a.z); hr.bu = a.w;
        hr.bv = b.x;
        if constexpr (prim_has_dir<FEAT>()) {
            hr.su = hr.sv = 0.f;
            ray.o = cam_origin(p);
            ray.d = mk4(b.y, b.z, b.w, (p.cam_d.w + p.cx.w) + p.cy.w);   // camera_ray's .w
        } else {
            hr.su = b.y; hr.sv = b.z;
            ray = camera_ray(p, x, y);
        }
        state = LS_SHADE;
    };
    start(cur_sub, cur_q, (uint32_t)lane);

    for (;;) {
        if constexpr (age_prio<FEAT>()) {
            // age-based issue priority: a wave holding an old path issues
            // ahead of the SIMD's other waves, so the longest paths -- the
            // end of the launch -- are not also the slowest
            now_tick = (uint32_t)__builtin_amdgcn_s_memrealtime();
            const uint32_t age = state != LS_DONE ? now_tick - born : 0u;
            if (__ballot(age > (uint32_t)(VR_AGE_T3 * 100)) != 0ull) __builtin_amdgcn_s_setprio(3);
            else if (__ballot(age > (uint32_t)(VR_AGE_T2 * 100)) != 0ull) __builtin_amdgcn_s_setprio(2);
            else if (__ballot(age > (uint32_t)(VR_AGE_T1 * 100)) != 0ull) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if constexpr ((FEAT & F_INLINE_PRIM) != 0u) {
            if (state == LS_CAMERA) {
                ray = camera_ray(p, cam_xy >> 16, cam_xy & 0xffffu);
                state = LS_SETUP;
            }
        }
        if (state == LS_SETUP) {
            if (intersect_spheres<CNT, FEAT>(p, ray, hr, cnt) && mesh_needed<CNT, FEAT>(p, hr, ps.bounce)) {
                trav_init<FEAT>(p, ray, hr.t, tr, L);
                state = root_visit<CNT, FEAT>(p, ray, tr, L, cnt) ? LS_TRAV : LS_SHADE;
            } else {
                state = LS_SHADE;
            }
        }
        if (HAS(F_MESH)) {
            for (;;) {
                const int n_trav = __popcll(__ballot(state == LS_TRAV || state == LS_HELP));
                if (n_trav == 0) break;
                const int n_shade = __popcll(__ballot(state == LS_SHADE));
                if (n_shade >= VR_SHADE_BATCH && n_shade * VR_SHADE_RATIO >= n_trav) break;
                // queue drained: no lane will be refilled; shade in batches
                if (cur_sub == ~0u && n_shade > 0 && n_shade * VR_DRAIN_SHADE_NUM >= n_trav * VR_DRAIN_SHADE_DEN)
                    break;
                if constexpr (helpers<FEAT>()) {
                    if (cur_sub == ~0u || __ballot(state == LS_HELP || state == LS_HELPDONE) != 0ull)
                        (void)help_step(p, lane, state, pend, slot, ray, tr, L);
                }
                if (state == LS_TRAV || state == LS_HELP) {
                    trav_iter<STACK, CNT, FEAT>(p, ray, tr, L, cnt);
                    if (state == LS_TRAV && any_hit_enough<CNT, FEAT>(p, ps.bounce) && tr.best >= 0) tr.nodeAddr = kSentinel;
                    if (tr.nodeAddr == kSentinel) {
                        if (state == LS_HELP) {
                            state = LS_HELPDONE;           // its best hit waits for the owner (help_step)
                        } else if (pend == 0) {
                            trav_finish(tr, hr);
                            state = LS_SHADE;
                        }                                  // else: the owner waits for its helpers
                    }
                }
            }
        }
        bool ended = false;
        if (state == LS_SHADE) {
            vr4 out;
            // one-frame kernels (the path traced its own camera ray) of the
            // Cornell box and of textured scenes: path 0 of the pixel stores
            // the depth term at bounce 0 (primary_kernel's formula), so no
            // register carries it to the path's end -- C3's one-frame kernel
            // 11 -> 6 spilled VGPRs, C2 one frame per call 0.731 -> 0.722 ms;
            // the plain HDRI mesh kernel (C5, no spills) keeps it to the end
            // (1.770 -> 1.790 ms with the early store, r05g)
            constexpr bool INL = (FEAT & F_INLINE_PRIM) != 0u;
            constexpr bool EARLY_DEPTH = INL && (FEAT & F_EXACT) != 0u &&
                                         (FEAT & (F_CORNELL | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
            if constexpr (EARLY_DEPTH) {
                if (ps.bounce == 0 && lane_q() == 0u)
                    p.path_w[lane_slot()] = hr.t < 1e20f ? depth_term(ray.o, add4(ray.o, mul4s(ray.d, hr.t))) : 1.f;
            }
            // Stores at each exit of the bounce step (bit 1: the plain HDRI
            // small-launch kernels, C5 shards: 2 spills -> 0; bit 2: the
            // Cornell whole-frame kernels, C2 without the service +0.3 %;
            // bit 4: the Cornell one-frame kernels, measured +0.5 % per
            // synchronous frame, off); elsewhere the join form compiles
            // spill-free or better (r05v)
#ifndef VR_WAVE_AT_EXIT
#define VR_WAVE_AT_EXIT 3
#endif
            constexpr bool CORN = (FEAT & F_CORNELL) != 0u;
            constexpr bool AT_EXIT =
                ((VR_WAVE_AT_EXIT & 1) && (FEAT & F_SMALL) != 0u && !INL &&
                 (FEAT & (F_CORNELL | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) == 0u) ||
                ((VR_WAVE_AT_EXIT & 2) && CORN && !INL && (FEAT & F_SMALL) == 0u) ||
                ((VR_WAVE_AT_EXIT & 4) && CORN && INL);
            if constexpr (AT_EXIT) {
                if (bounce_step<CNT, FEAT, INL && !EARLY_DEPTH>(p, ray, hr, ps, out, cnt, [&](const vr4& o) {
                        if constexpr (INL && !EARLY_DEPTH) store_path(p, lane_q(), lane_slot(), o, ps.depth);
                        else store_path_rgb(p, lane_q(), lane_slot(), o);
                        if constexpr ((FEAT & F_SMALL) != 0u) {
                            if (p.path_cost)
                                p.path_cost[(size_t)lane_q() * p.path_stride + lane_slot()] =
                                    (uint8_t)(cnt.work < 510u ? cnt.work >> 1 : 255u);
                        }
                    })) {
                    ended = true;
                } else {
                    state = LS_SETUP;
                }
            } else if (bounce_step<CNT, FEAT, INL && !EARLY_DEPTH>(p, ray, hr, ps, out, cnt)) {
                if constexpr (INL && !EARLY_DEPTH) store_path(p, lane_q(), lane_slot(), out, ps.depth);
                else store_path_rgb(p, lane_q(), lane_slot(), out);
                if constexpr ((FEAT & F_SMALL) != 0u) {
                    if (p.path_cost)
                        p.path_cost[(size_t)lane_q() * p.path_stride + lane_slot()] =
                            (uint8_t)(cnt.work < 510u ? cnt.work >> 1 : 255u);
                }
                ended = true;
            } else {
                state = LS_SETUP;
            }
        }
        const unsigned long long em = __ballot(ended);
        if (em != 0ull) {
            const uint32_t need = (uint32_t)__popcll(em);
            uint32_t nsub = cur_sub, nq = cur_q;
            if (next + need > 64u && cur_sub != ~0u) grab(nsub, nq);
            if (ended) {
                const uint32_t r = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
                if (r < 64u) start(cur_sub, cur_q, r);
                else start(nsub, nq, r - 64u);
            }
            if (next + need > 64u) { cur_sub = nsub; cur_q = nq; next = next + need - 64u; }
            else next += need;
        }
        if (__ballot(state != LS_DONE) == 0ull) break;
    }
    if (CNT) flush_counts(p, cnt, lane, true);
}

// ---- render service ---------------------------------------------------------
// A session (vrhip_api.cpp) runs consecutive render launches on ONE
// persistent kernel: the drain of launch L -- its last, longest paths, a
// large share of a short launch (a 16-frame C3 shard of 3.7 M paths is
// ~280 us of work next to a ~300-400 us longest path) --
// overlaps launch L+1's paths instead of ending a kernel.  The host appends
// launch descriptors (first frame, frame count, per-frame seeds) to a ring in
// host-pinned memory; the ring wave mirrors them into device memory; every
// other wave takes chunks of (sub-tile, path) of launch L, then of L+1, ...,
// exactly as render_wave_kernel does for one launch.  A session's camera,
// scene and tiling are fixed (the host closes it on any change), so the
// camera rays' closest hits are the same for all its launches: primary_kernel
// traces them once when the session opens, and every path of every launch
// starts from them.  Results go to the launch's scratch slot; the session
// finish pass (svc_finish_kernel) sums every pixel's paths launch by launch in
// path order, so the image is the reference's bit for bit whatever the
// interleaving.
__device__ __forceinline__ uint32_t svc_ld(const uint32_t* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// a path's radiance into its launch's slot (the store_path layout per slot)
// (the pixel's depth term: primary_kernel, once per session, in slot 0)
__device__ __forceinline__ void svc_store_path(const RenderParams& p, uint32_t L, uint32_t q, uint32_t slot, const vr4& out)
{
    vr3* const base = reinterpret_cast<vr3*>(reinterpret_cast<uint8_t*>(p.paths) + (size_t)L * p.svc_slot_bytes);
    base[(size_t)q * p.path_stride + slot] = vr3{ out.x, out.y, out.z };
}

// The ring wave (the last wave of block 0; it takes no paths): mirrors the
// host ring into device memory every ~1 us -- newly posted descriptors (sc1
// stores, drained, then the control word), the host's close, or, after
// svc_idle_ticks without a new launch, the session's retirement -- until
// the session is closed.  The host writes `closed` only after its last post
// and this reads `closed` before `posted`, so a close carries the final count.
// Retiring on its own, the wave first announces it in the host ring's
// `retired` word, then reads `posted` once more (a store-fence-load pair
// against svc_post's): a launch posted meanwhile is either seen here and
// served, or the host sees `retired` and renders it elsewhere (it then
// excludes the launch's slot from the session's finish pass).  On every exit
// `retired` holds the launches consumed, which the host checks.
__device__ __forceinline__ void svc_publish(const RenderParams& p, uint32_t v, int lane)
{
    if (lane == 0) __hip_atomic_store(&p.svc_host->retired, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void svc_ring_wave(const RenderParams& p, int lane)
{
    SvcDevCtl* const d = p.svc_dev;
    uint32_t dp = 0, last = (uint32_t)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint32_t hc = 0, hp = 0;
        if (lane == 0) {
            hc = __hip_atomic_load(&p.svc_host->closed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            hp = __hip_atomic_load(&p.svc_host->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        hc = __builtin_amdgcn_readfirstlane(hc);
        hp = __builtin_amdgcn_readfirstlane(hp);
        if (hp > kSvcMaxLaunches) hp = kSvcMaxLaunches;
        const uint32_t now = (uint32_t)__builtin_amdgcn_s_memrealtime();
        if (hp > dp) {
            for (uint32_t k = dp; k < hp; ++k) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(&p.svc_host->desc[k]);
                uint32_t* dst = reinterpret_cast<uint32_t*>(&d->desc[k]);
                for (uint32_t w = (uint32_t)lane; w < kSvcLaunchWords; w += 64u) {
                    const uint32_t v = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(dst + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) atomicMax(&d->ctl, hp | (hc ? kSvcClosed : 0u));
            dp = hp;
            last = now;
            if (hc) { svc_publish(p, dp | kSvcClosed, lane); return; }
        } else if (hc != 0u) {                             // closed by the host
            if (lane == 0) atomicMax(&d->ctl, dp | kSvcClosed);
            svc_publish(p, dp | kSvcClosed, lane);
            return;
        } else if (now - last > p.svc_idle_ticks) {        // idle: retire, unless a launch races it
            svc_publish(p, dp | kSvcClosed, lane);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
            uint32_t hp2 = 0;
            if (lane == 0) hp2 = __hip_atomic_load(&p.svc_host->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            hp2 = __builtin_amdgcn_readfirstlane(hp2);
            if (hp2 <= dp) {
                if (lane == 0) atomicMax(&d->ctl, dp | kSvcClosed);
                return;
            }
            // serve it (mirrored next round); the host may already have seen
            // the announcement, then it renders the launch elsewhere as well
            svc_publish(p, 0u, lane);
            last = now;
            continue;
        }
        __builtin_amdgcn_s_sleep(32);
    }
}

template <int STACK, uint32_t FEAT, int BT>
__device__ __forceinline__ void service_body(const RenderParams& p, const Lds& L)
{
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    if (blockIdx.x == 0u && (tid >> 6) == BT / 64 - 1) { svc_ring_wave(p, lane); return; }
    constexpr bool SPARSE = (FEAT & F_SPARSE) != 0u;       // the session's listed pixels only
    // chunk rows: 8x8 sub-tiles, or (F_SPARSE) runs of 64 pixels the
    // session's primary pass listed (the last run padded, render_wave_kernel)
    const uint32_t n_px = SPARSE ? __builtin_amdgcn_readfirstlane(*sparse_count(p)) : 0u;
    const uint32_t n_sub = SPARSE ? (n_px + 63u) >> 6 : p.path_stride >> 6;
    Cnt cnt;
    const uint32_t Q = p.n_queues;
    const uint32_t q0 = blockIdx.x & (Q - 1u);
    uint32_t qj = q0;
    __shared__ unsigned long long lds_dead[BT / 64];
    unsigned long long* const my_dead = lds_dead + (tid >> 6);
    if (lane == 0) *my_dead = 0ull;
    // per wave, in LDS (read at grabs only; the kernel is at its register
    // limits): the launch sL this wave takes chunks from, the launches it
    // knows to be posted, launch sL's frame count
    struct Ring { uint32_t sL, posted, l_nf; };
    __shared__ Ring lds_ring[BT / 64];
    Ring* const rg = lds_ring + (tid >> 6);
    if (lane == 0) *rg = Ring{ 0u, 0u, 0u };
    enum { GOT = 0, WAIT = 1, DONE = 2 };
    // the seeds' frame base (first frame + frame) and time of the chunks the
    // wave hands out -- the current one and the next one -- in LDS (cslot:
    // which of the two records is the current chunk's)
    __shared__ uint32_t lds_seed[BT / 64][2][2];
    uint32_t (*const seed)[2] = lds_seed[tid >> 6];
    uint32_t cslot = 0;
    // next chunk (wave-uniform) into seed record `rec`: sub-tile, path and
    // launch; GOT, WAIT (the ring holds nothing more yet) or DONE (the session
    // is closed and drained)
    auto grab = [&](uint32_t& sub, uint32_t& path, uint32_t& lc, uint32_t rec) -> int {
        uint32_t sL = __builtin_amdgcn_readfirstlane(rg->sL), posted = __builtin_amdgcn_readfirstlane(rg->posted);
        uint32_t l_nf = __builtin_amdgcn_readfirstlane(rg->l_nf);
        for (;;) {
            if (sL >= posted) {
                uint32_t c = 0;
                if (lane == 0) c = svc_ld(&p.svc_dev->ctl);
                c = __builtin_amdgcn_readfirstlane(c);
                posted = c & ~kSvcClosed;
                if (sL >= posted) {
                    if (lane == 0) { rg->sL = sL; rg->posted = posted; rg->l_nf = l_nf; }
                    sub = ~0u;
                    return (c & kSvcClosed) ? DONE : WAIT;
                }
            }
            if (l_nf == 0u) {
                uint32_t nf = 0;
                if (lane == 0) nf = svc_ld(&p.svc_dev->desc[sL].n_frames);
                l_nf = __builtin_amdgcn_readfirstlane(nf);
                if (l_nf == 0u || l_nf > p.svc_kmax) l_nf = 1u;   // (never: the host posts 1..svc_kmax frames)
            }
            const uint32_t np = 2u * l_nf;
            uint32_t* const heads = p.svc_qctl + (size_t)sL * kSvcQctlWords;
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(heads + qj * kQueueStride, 1u);
            v = __builtin_amdgcn_readfirstlane(v);
            uint32_t pth;
            const uint32_t sb = queue_item(qj, v, Q, np, pth);
            if (sb < n_sub) {
                if (lane == 0) {
                    rg->sL = sL; rg->posted = posted; rg->l_nf = l_nf;
                    seed[rec][0] = svc_ld(&p.svc_dev->desc[sL].first_frame) + (pth >> 1);
                    seed[rec][1] = svc_ld(&p.svc_dev->desc[sL].times[pth >> 1]);
                }
                sub = sb; path = pth; lc = sL;
                return GOT;
            }
            // queue qj of launch sL is drained: the drained-queue mask of the
            // small launches (render_wave_kernel grab)
            uint32_t m0 = 0, m1 = 0;
            if (lane == 0) {
                unsigned long long* const dmask = queue_drained_mask(heads);
                uint32_t pq;
                const bool first = v == 0u || queue_item(qj, v - 1u, Q, np, pq) < n_sub;
                const unsigned long long m = first ? atomicOr(dmask, 1ull << qj)
                                                   : __hip_atomic_load(dmask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long dd = *my_dead | m | (1ull << qj);
                *my_dead = dd;
                m0 = (uint32_t)dd; m1 = (uint32_t)(dd >> 32);
            }
            const unsigned long long live = all_q_of(Q) & ~(((unsigned long long)__builtin_amdgcn_readfirstlane(m1) << 32) |
                                                             (unsigned long long)__builtin_amdgcn_readfirstlane(m0));
            if (live == 0ull) {                            // launch sL is out of work: the next one
                ++sL;
                l_nf = 0u;
                if (lane == 0) *my_dead = 0ull;
                qj = q0;
                continue;
            }
            const unsigned long long after = qj + 1u < 64u ? (live >> (qj + 1u)) << (qj + 1u) : 0ull;
            qj = (uint32_t)__builtin_ctzll(after != 0ull ? after : live);
        }
    };
    int ring = WAIT;                                       // the status of the last grab
    uint32_t cur_sub = ~0u, cur_q = 0, cur_L = 0;
    uint32_t next = 64u;                                   // items of the current chunk handed out
    int state = LS_DONE;
    uint32_t q = 0, slot = 0;                              // this lane's path | launch << 8, and pixel slot
    Ray ray;
    PathState ps;
    HitRec hr;
    Trav tr;
    auto start = [&](uint32_t sub, uint32_t path, uint32_t lc, uint32_t px, uint32_t rec) {
        if (sub == ~0u) { state = LS_DONE; return; }       // render's per-sample prologue (:817-844)
        q = path | (lc << 8);
        slot = sub * 64u + px;
        if constexpr (SPARSE) {                            // the listed pixel
            const uint32_t k = slot < n_px ? slot : n_px - 1u;
            slot = p.sparse_px[k];
        }
        uint32_t x, y;
        sub_pixel(p, slot >> 6, slot & 63u, x, y);
        uint32_t s1 = x * seed[rec][0];                    // x * (first frame + frame)
        uint32_t s2 = y * seed[rec][1];
        if (path & 1u) (void)hash_seeds(s1, s2);           // the frame's second sample
        path_begin(ps, s1, s2);
        const vr4 a = p.prim[2u * slot], b = p.prim[2u * slot + 1u];
        hr.t = a.x; hr.kind = __float_as_int(a.y); hr.idx = __float_as_int(a.z); hr.bu = a.w;
        hr.bv = b.x;
        if constexpr (prim_has_dir<FEAT>()) {
            hr.su = hr.sv = 0.f;
            ray.o = cam_origin(p);
            ray.d = mk4(b.y, b.z, b.w, (p.cam_d.w + p.cx.w) + p.cy.w);   // camera_ray's .w
        } else {
            hr.su = b.y; hr.sv = b.z;
            ray = camera_ray(p, x, y);
        }
        state = LS_SHADE;
    };
    // every lane idle (the wave's first chunk too): the next chunk, waiting
    // for the ring if need be; false: the session is over for this wave
    auto wait_chunk = [&]() -> bool {
        const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
        for (;;) {
            ring = grab(cur_sub, cur_q, cur_L, cslot);
            if (ring != WAIT) return ring == GOT;
            // failsafe: a wave that waited twice the session's idle limit
            // leaves (the ring wave retires the session after one)
            if ((uint32_t)__builtin_amdgcn_s_memrealtime() - t0 > 2u * p.svc_idle_ticks + 200000u) return false;
            __builtin_amdgcn_s_sleep(32);
        }
    };
    // every lane idle (LS_DONE): the loop's refill waits for the first chunk
    for (;;) {
        if (state == LS_SETUP) {
            if (intersect_spheres<false, FEAT>(p, ray, hr, cnt) && mesh_needed<false, FEAT>(p, hr, ps.bounce)) {
                trav_init<FEAT>(p, ray, hr.t, tr, L);
                state = root_visit<false, FEAT>(p, ray, tr, L, cnt) ? LS_TRAV : LS_SHADE;
            } else {
                state = LS_SHADE;
            }
        }
        if (HAS(F_MESH)) {
            for (;;) {
                const int n_trav = __popcll(__ballot(state == LS_TRAV));
                if (n_trav == 0) break;
                const int n_shade = __popcll(__ballot(state == LS_SHADE));
                if (n_shade >= VR_SHADE_BATCH && n_shade * VR_SHADE_RATIO >= n_trav) break;
                if (cur_sub == ~0u && n_shade > 0 && n_shade * VR_DRAIN_SHADE_NUM >= n_trav * VR_DRAIN_SHADE_DEN) break;
                if (state == LS_TRAV) {
                    trav_iter<STACK, false, FEAT>(p, ray, tr, L, cnt);
                    if (any_hit_enough<false, FEAT>(p, ps.bounce) && tr.best >= 0) tr.nodeAddr = kSentinel;
                    if (tr.nodeAddr == kSentinel) {
                        trav_finish(tr, hr);
                        state = LS_SHADE;
                    }
                }
            }
        }
        bool ended = false;
        if (state == LS_SHADE) {
            vr4 out;
            // Cornell-box and textured kernels store the result at each of
            // bounce_step's exits: stored after the join, the merged radiance
            // was spilled around it -- three scratch loads on every bounce of
            // C2's service kernel (6 spills -> 0, C2 +0.5 %, C3 +1 %); the
            // plain HDRI kernels (C5, no spills) keep the join (-0.4 % without)
            constexpr bool AT_EXIT = (FEAT & (F_CORNELL | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC)) != 0u;
            bool done;
            if constexpr (AT_EXIT) {
                done = bounce_step<false, FEAT, false>(p, ray, hr, ps, out, cnt, [&](const vr4& o) {
                    svc_store_path(p, q >> 8, q & 0xffu, slot, o);
                });
            } else {
                done = bounce_step<false, FEAT, false>(p, ray, hr, ps, out, cnt);
                if (done) svc_store_path(p, q >> 8, q & 0xffu, slot, out);
            }
            if (done) ended = true;
            else state = LS_SETUP;
        }
        // refill: lanes whose path ended take the next items; when every
        // lane is idle the wave waits for the ring's next chunk and all 64
        // lanes take it (one start() site, so one inlined copy of it)
        bool take = ended;
        bool over = false;
        for (;;) {
            const unsigned long long em = __ballot(take);
            if (em != 0ull) {
                const uint32_t need = (uint32_t)__popcll(em);
                uint32_t nsub = ~0u, nq = 0, nL = 0;
                if (next + need > 64u && cur_sub != ~0u) {
                    ring = grab(nsub, nq, nL, cslot ^ 1u);
                    if (ring != GOT) nsub = ~0u;
                }
                if (take) {
                    const uint32_t r = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
                    const bool here = r < 64u;
                    start(here ? cur_sub : nsub, here ? cur_q : nq, here ? cur_L : nL, here ? r : r - 64u,
                          here ? cslot : cslot ^ 1u);
                }
                if (next + need > 64u) { cur_sub = nsub; cur_q = nq; cur_L = nL; cslot ^= 1u; next = next + need - 64u; }
                else next += need;
            }
            if (__ballot(state != LS_DONE) != 0ull) break;
            if (ring == DONE || !wait_chunk()) { over = true; break; }
            next = 0u;
            take = true;
        }
        if (over) break;
    }
}

// residency of the service kernel (waves per SIMD; 0: the scene kernel's)
#ifndef VR_SVC_WAVES
#define VR_SVC_WAVES 0
#endif
constexpr int svc_waves(int stack, bool c) { return VR_SVC_WAVES > 0 && stack <= 24 ? VR_SVC_WAVES : path_waves(stack, c); }
constexpr int svc_cache_nodes(int stack, int bt, bool c) {
    return (163840 / (4 * svc_waves(stack, c) * 64 / bt) - bt - stack * bt * 4) / 56 > 0
               ? (163840 / (4 * svc_waves(stack, c) * 64 / bt) - bt - stack * bt * 4) / 56 : 1;
}
template <int STACK, uint32_t FEAT, int BT>
__global__ void __launch_bounds__(BT, svc_waves(STACK, cornell_kernel<FEAT>())) render_service_kernel(const RenderParams p)
{
    constexpr int CN = svc_cache_nodes(STACK, BT, cornell_kernel<FEAT>());
    __shared__ int lds_stack[STACK * BT];
    __shared__ vr4 lds_nodes[3 * CN];
    __shared__ int2 lds_idx[CN];
    const Lds L = lds_setup<FEAT, BT>(p, lds_stack, lds_nodes, lds_idx, CN, (int)threadIdx.x);
    service_body<STACK, FEAT, BT>(p, L);
}

// ---- host launchers --------------------------------------------------------
// Feature specialisations, smallest first (BASELINE configs C1..C5); the
// generic kernel covers everything else, deep trees and the counting variant.
constexpr uint32_t kFeatAll =
    F_CORNELL | F_EXAMPLE | F_VIEW_BRDF | F_MESH | F_BRDF | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC | F_STRICT;
static_assert((kFeatAll & F_COUNT_EXEC) == 0u, "F_COUNT_EXEC is a compile-time kernel variant, not a scene flag");
constexpr uint32_t kFeatCornellMesh = F_CORNELL | F_MESH;                                  // C2
constexpr uint32_t kFeatCornellSphere = F_CORNELL | F_EXAMPLE;                              // C1
constexpr uint32_t kFeatHdriMesh = F_MESH;                                                 // C5
constexpr uint32_t kFeatHdriMeshTex = F_MESH | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC;        // C3
constexpr uint32_t kFeatHdriBrdfSphere = F_EXAMPLE | F_VIEW_BRDF | F_BRDF;                  // C4
// Feature classes (F_CLASS): Cornell box or HDRI x mesh or spheres, any
// material features (texture maps, BRDF view; the example sphere in the
// sphere classes), no strict traversal.  The host never sets F_MESH with
// F_EXAMPLE (the reference ignores the mesh then, PathTracer.cu:192,268).
constexpr uint32_t kMaterialFeats = F_VIEW_BRDF | F_BRDF | F_TEX_DIFF | F_TEX_NORM | F_TEX_SPEC;
constexpr uint32_t kClassCornellMesh = F_CLASS | F_CORNELL | F_MESH | kMaterialFeats;
constexpr uint32_t kClassHdriMesh = F_CLASS | F_MESH | kMaterialFeats;
constexpr uint32_t kClassCornellSphere = F_CLASS | F_CORNELL | F_EXAMPLE | kMaterialFeats;
constexpr uint32_t kClassHdriSphere = F_CLASS | F_EXAMPLE | kMaterialFeats;
static_assert((kClassGeom & kMaterialFeats) == 0u && (kClassGeom & F_EXAMPLE) == 0u, "class geometry bits");
// the feature class of a launch's flags (kFeatAll bits), 0: the generic kernel
constexpr uint32_t feature_class(uint32_t need) {
    return (need & F_STRICT) != 0u ? 0u
         : (need & kClassGeom) == (F_CORNELL | F_MESH) ? ((need & F_EXAMPLE) ? 0u : kClassCornellMesh)
         : (need & kClassGeom) == F_MESH ? ((need & F_EXAMPLE) ? 0u : kClassHdriMesh)
         : (need & kClassGeom) == F_CORNELL ? kClassCornellSphere
         : kClassHdriSphere;
}

// Multi-frame launches of fewer than 2^24 paths (shards) on the small-launch
// kernels (F_SMALL: helper lanes, per-path costs, longest-first order) or,
// with 0, on the whole-frame kernels in 256-thread blocks
#ifndef VR_SHARD_SMALL
#define VR_SHARD_SMALL 0
#endif
template <int STACK, uint32_t FEAT>
inline void launch_wave(const RenderParams& p, uint32_t n_tiles, hipStream_t s)
{
    // one-frame launches trace the camera ray in the path kernel (a separate
    // instantiation); the instrumented copy always takes the primary pass
    if constexpr ((FEAT & (F_INLINE_PRIM | F_COUNT_EXEC)) == 0u) {
        if (p.inline_prim) { launch_wave<STACK, FEAT | F_INLINE_PRIM>(p, n_tiles, s); return; }
    }
    if constexpr ((FEAT & (F_SMALL | F_COUNT_EXEC)) == 0u) {
        if (p.small_blocks && (VR_SHARD_SMALL != 0 || (FEAT & F_INLINE_PRIM) != 0u)) {
            launch_wave<STACK, FEAT | F_SMALL>(p, n_tiles, s);
            return;
        }
    }
    if constexpr ((FEAT & F_INLINE_PRIM) == 0u)
        hipLaunchKernelGGL((primary_kernel<STACK, FEAT & ~F_SMALL>), dim3(n_tiles), dim3(kBlockThreads), 0, s, p);
    // one resident set: path_waves(STACK, C) waves per SIMD, 4 SIMDs per CU;
    // small launches (and the instrumented copy of one) in the smaller blocks
    constexpr bool C = cornell_kernel<FEAT>();
    constexpr int BT = ((FEAT & F_SMALL) != 0u) ? wave_block_small(STACK, C) : wave_block(STACK, C);
    constexpr int BTS = wave_block_small(STACK, C);
    // counted, or multi-frame shards on the whole-frame kernel: block size picked at run time below
    constexpr bool runtime_bt = (FEAT & F_COUNT_EXEC) != 0u || ((FEAT & F_SMALL) == 0u && VR_SHARD_SMALL == 0);
    constexpr int B = (runtime_bt && BTS != BT) ? 0 : BT;
    // blocks per CU: the kernel's full residency, or fewer under a waves-per-SIMD cap
    auto per_cu = [&](int bt) {
        const uint32_t full = (uint32_t)path_blocks_per_cu(STACK, bt, C);
        if (p.waves_cap == 0u) return full;
        const uint32_t capped = p.waves_cap * 4u * 64u / (uint32_t)bt;
        return capped < 1u ? 1u : (capped < full ? capped : full);
    };
    if constexpr (sparse_ok<FEAT>()) {
        if (p.sparse_px) {                        // the listed pixels only (same shape and residency)
            const int bt = (B == 0 && p.small_blocks) ? BTS : BT;
            if (bt == BTS)
                hipLaunchKernelGGL((render_wave_kernel<STACK, FEAT | F_SPARSE, BTS>), dim3(p.wave_blocks * per_cu(BTS)),
                                   dim3(BTS), 0, s, p);
            else
                hipLaunchKernelGGL((render_wave_kernel<STACK, FEAT | F_SPARSE, BT>), dim3(p.wave_blocks * per_cu(BT)),
                                   dim3(BT), 0, s, p);
            return;
        }
    }
    if constexpr (B == 0) {
        if (p.small_blocks) {
            hipLaunchKernelGGL((render_wave_kernel<STACK, FEAT, BTS>), dim3(p.wave_blocks * per_cu(BTS)), dim3(BTS), 0, s, p);
            return;
        }
    }
    hipLaunchKernelGGL((render_wave_kernel<STACK, FEAT, BT>), dim3(p.wave_blocks * per_cu(BT)), dim3(BT), 0, s, p);
}

// One scene specialisation, production (FEAT) or instrumented
// (FEAT | F_COUNT_EXEC: same launch shape, residency, node-loop threshold and
// queues as the production kernel of the same scene, plus load counters).
// The render service's persistent kernel (one per session): 256-thread
// blocks at the scene kernel's residency, one resident set.
template <int STACK, uint32_t FEAT>
inline void launch_service_wave(const RenderParams& p, hipStream_t s)
{
    constexpr uint32_t F = FEAT | F_SERVICE;
    constexpr bool C = cornell_kernel<F>();
    constexpr int BT = kBlockThreads;
    // the session's camera-ray hits (camera, scene and tiling are fixed for it)
    hipLaunchKernelGGL((primary_kernel<STACK, FEAT>), dim3(p.path_stride / kBlockThreads), dim3(kBlockThreads), 0, s, p);
    const uint32_t per_cu = (uint32_t)(4 * svc_waves(STACK, C) * 64 / BT);
    if constexpr (sparse_ok<FEAT>()) {
        if (p.sparse_px) {                        // the listed pixels only
            hipLaunchKernelGGL((render_service_kernel<STACK, F | F_SPARSE, BT>), dim3(p.wave_blocks * per_cu), dim3(BT), 0, s, p);
            return;
        }
    }
    hipLaunchKernelGGL((render_service_kernel<STACK, F, BT>), dim3(p.wave_blocks * per_cu), dim3(BT), 0, s, p);
}

template <uint32_t FEAT>
inline void launch_spec(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, bool svc = false)
{
    constexpr bool CNT = (FEAT & F_COUNT_EXEC) != 0u;
    if constexpr ((FEAT & F_MESH) == 0u) {
        // sphere-only scenes: one pixel per thread, primary hit shared by its paths
        hipLaunchKernelGGL((render_kernel<16, CNT, FEAT>), dim3(n_tiles * p.split), dim3(kBlockThreads), 0, s, p);
    } else if constexpr (!CNT) {
        if (svc) {                                  // a render-service session (mesh scenes only)
            if (stack_depth <= 16) launch_service_wave<16, FEAT>(p, s);
            else if (stack_depth <= 24) launch_service_wave<24, FEAT>(p, s);
            else launch_service_wave<32, FEAT>(p, s);
            return;
        }
    }
    if constexpr ((FEAT & F_MESH) != 0u) {
        // mesh scenes: the path-pool kernel (traversal divergence)
        if ((p.flags & F_MESH) == 0u)
            hipLaunchKernelGGL((render_kernel<16, CNT, FEAT>), dim3(n_tiles * p.split), dim3(kBlockThreads), 0, s, p);
        else if (stack_depth <= 16)
            launch_wave<16, FEAT>(p, n_tiles, s);
        else if (stack_depth <= 24)
            launch_wave<24, FEAT>(p, n_tiles, s);
        else
            launch_wave<32, FEAT>(p, n_tiles, s);
    }
}

// Per-specialisation launchers, one translation unit each (vr_spec_*.hip);
// mode 0 production, 1 the instrumented copy (F_COUNT_EXEC), 2 the render
// service's persistent kernel (mesh scenes).
void launch_spec_c1(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_spec_c2(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_spec_c3(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_spec_c4(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_spec_c5(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_spec_generic(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
// feature classes (kClass*): Cornell box + mesh, HDRI + mesh, and both sphere classes
void launch_cls_cornell_mesh(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_cls_hdri_mesh(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
void launch_cls_sphere(const RenderParams& p, uint32_t n_tiles, int stack_depth, hipStream_t s, int mode);
// trees deeper than 30 levels (64-entry stacks), production or instrumented
void launch_spec_deep(const RenderParams& p, uint32_t n_tiles, hipStream_t s, bool exec);
// the reference algorithm's counting variant (strict traversal, in place)
void launch_counting(const RenderParams& p, uint32_t blocks, int stack_depth, hipStream_t s);

} // namespace vr
