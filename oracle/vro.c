/*
 * vro.c -- CPU ORACLE (test infrastructure only; see vro.h).
 *
 * A plain-C restatement of the reference CUDA path tracer.  Every function
 * cites the reference lines it follows (paths relative to the reference
 * repository root).  Reference operator semantics are kept exactly:
 *   float4 ops with the nonstandard .w rules of MathHelpers.cuh:85-196,
 *   dot() over xyz only (:328-331), normalize keeps .w (:349-353),
 *   clamp(int) returning float (:362-365), slab spans on integer bit
 *   patterns (:454-552), double-precision sub-expressions where the
 *   reference mixes double literals with floats.
 * Build: -O2 -ffp-contract=off (no FMA contraction), no -ffast-math.
 */
#include "vro.h"
#include "vro_math.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y, z, w; } vf4;
typedef struct { float x, y; } vf2;

/* MathHelpers.cuh:16-17 (__constant__ float PI, epsilon) */
#define VR_PI      3.14159265359f
#define VR_EPSILON 0.0000000003f

static inline vf4 f4(float x, float y, float z, float w) { vf4 r = { x, y, z, w }; return r; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline int32_t fibits(float f) { int32_t u; memcpy(&u, &f, 4); return u; }
static inline float ibitsf(int32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* fminf/fmaxf as on the GPU: NaN operands ignored, -0 < +0. */
static inline float vmin(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b;
}
static inline float vmax(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a;
}

/* float -> int as CUDA's cvt.rzi.s32.f32: truncate, saturate, NaN -> 0 */
static inline int f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int)0x80000000u;
    return (int)f;
}
static inline int d2i(double f) {
    if (f != f) return 0;
    if (f >= 2147483648.0) return 2147483647;
    if (f <= -2147483648.0) return (int)0x80000000u;
    return (int)f;
}
/* float -> unsigned char with saturation (cvt.rzi.u8.f32) */
static inline uint8_t f2u8(float f) {
    if (f != f) return 0;
    if (f <= 0.0f) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)(int)f;
}

/* ---- float4 operators, MathHelpers.cuh:85-196 ---- */
static inline vf4 add4(vf4 a, vf4 b) { return f4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline vf4 sub4(vf4 a, vf4 b) { return f4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline void addeq4(vf4 *a, vf4 b) { a->x += b.x; a->y += b.y; a->z += b.z; a->w += b.w; }
static inline void muleq4(vf4 *a, vf4 b) { a->x *= b.x; a->y *= b.y; a->z *= b.z; a->w *= b.w; }
static inline void muleq4s(vf4 *a, float b) { a->x *= b; a->y *= b; a->z *= b; }
static inline vf4 mul4(vf4 a, vf4 b) { return f4(a.x * b.x, a.y * b.y, a.z * b.z, a.w); }
static inline vf4 mul4s(vf4 a, float b) { return f4(a.x * b, a.y * b, a.z * b, a.w); }
static inline vf4 muls4(float a, vf4 b) { return f4(a * b.x, a * b.y, a * b.z, b.w); }
static inline float dot4(vf4 a, vf4 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline vf4 cross4(vf4 a, vf4 b) {
    return f4(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x, 0.0f);
}
/* :349-353, rsqrtf(x) restated as 1/sqrtf(x) */
static inline vf4 normalize4(vf4 a) { float inv = 1.0f / sqrtf(dot4(a, a)); return mul4s(a, inv); }
/* :362-365 clamp(int) -> float */
static inline float clampi(int v, int lo, int hi) {
    int m = (hi < v) ? hi : v;
    return (float)((lo > m) ? lo : m);
}
/* :374-377 */
static inline float clampf(float v, float lo, float hi) { return vmax(lo, vmin(hi, v)); }
/* :386-392 */
static inline vf4 clamp4(vf4 v, float lo, float hi) {
    return f4(clampf(v.x, lo, hi), clampf(v.y, lo, hi), clampf(v.z, lo, hi), v.w);
}
/* :400-403 */
static inline vf4 max4(vf4 a, vf4 b) { return f4(vmax(a.x, b.x), vmax(a.y, b.y), vmax(a.z, b.z), vmax(a.w, b.w)); }
/* :446-449 */
static inline float lerpf_(float a, float b, float w) { return (1.0f - w) * a + w * b; }

/* mat4 * float4, MathHelpers.cuh:22-76; rows m0..m3, m3 defaults to (0,0,0,1) */
static inline vf4 tbn_mul(vf4 m0, vf4 m1, vf4 m2, vf4 b) {
    vf4 m3 = f4(0.0f, 0.0f, 0.0f, 1.0f);
    return f4(m0.x * b.x + m1.x * b.y + m2.x * b.z + m3.x * b.w,
              m0.y * b.x + m1.y * b.y + m2.y * b.z + m3.y * b.w,
              m0.z * b.x + m1.z * b.y + m2.z * b.z + m3.z * b.w,
              m0.w * b.x + m1.w * b.y + m2.w * b.z + m3.w * b.w);
}

/* Kepler span helpers on integer bit patterns, MathHelpers.cuh:454-552 */
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline float span_begin(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    int zc = imax(imin(fibits(c0), fibits(c1)), fibits(d));             /* fmin_fmax */
    return ibitsf(imax(imax(fibits(vmin(a0, a1)), fibits(vmin(b0, b1))), zc)); /* fmax_fmax */
}
static inline float span_end(float a0, float a1, float b0, float b1, float c0, float c1, float d) {
    int zc = imin(imax(fibits(c0), fibits(c1)), fibits(d));             /* fmax_fmin */
    return ibitsf(imin(imin(fibits(vmax(a0, a1)), fibits(vmax(b0, b1))), zc)); /* fmin_fmin */
}

/* ---- libm selection ---- */
typedef struct { int libm; } mctx;
static inline void m_sincos(const mctx *m, float x, float *s, float *c) {
    if (m->libm == VRO_LIBM_PORTABLE) vro_p_sincosf(x, s, c);
    else { *s = sinf(x); *c = cosf(x); }
}
static inline float m_acosf(const mctx *m, float x) { return m->libm == VRO_LIBM_PORTABLE ? vro_p_acosf(x) : acosf(x); }
static inline float m_atan2f(const mctx *m, float y, float x) { return m->libm == VRO_LIBM_PORTABLE ? vro_p_atan2f(y, x) : atan2f(y, x); }
static inline float m_powf(const mctx *m, float x, float y) { return m->libm == VRO_LIBM_PORTABLE ? vro_p_powf(x, y) : powf(x, y); }

/* ---- scene constants, PathTracer.cu:50-123 ---- */
enum { R_SPEC = 0, R_DIFF = 1, R_BRDF = 2 };
typedef struct { float r; vf4 pos, emission, col; int refl; } sphere_t;

static const sphere_t k_spheres[2] = {   /* :107-111 */
    { 3.5f, { 15.f, 0.f, 15.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, R_SPEC },
    { 3.5f, { 25.f, 0.f, 15.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 1.f, 1.f, 1.f, 0.f }, R_DIFF },
};
static const sphere_t k_cornell[6] = {   /* :113-121 */
    { 160.f, { 0.f, 160.f + 49.f, 0.f, 0.f }, { 4.f, 3.6f, 3.2f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, R_DIFF },
    { 1e5f, { 1e5f + 50.f, 0.f, 0.f, 0.f }, { 0.075f, 0.025f, 0.025f, 0.f }, { 0.75f, 0.25f, 0.25f, 0.f }, R_DIFF },
    { 1e5f, { -1e5f - 50.f, 0.f, 0.f, 0.f }, { 0.025f, 0.075f, 0.025f, 0.f }, { 0.25f, 0.75f, 0.25f, 0.f }, R_DIFF },
    { 1e5f, { 0.f, 0.f, -1e5f - 100.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 1.f, 1.f, 1.f, 0.f }, R_DIFF },
    { 1e5f, { 0.f, 1e5f + 50.f, 0.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 1.f, 1.f, 1.f, 0.f }, R_DIFF },
    { 1e5f, { 0.f, -1e5f - 50.f, 0.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 1.f, 1.f, 1.f, 0.f }, R_DIFF },
};
static const sphere_t k_example = { 10.f, { 0.f, 0.f, 0.f, 0.f }, { 0.f, 0.f, 0.f, 0.f }, { 1.f, 1.f, 1.f, 0.f }, R_DIFF }; /* :123 */

typedef struct { vf4 o, d; } ray_t;                 /* RayIntersection.cuh:23-41 */
typedef struct {                                    /* PathTracer.cuh:17-53 */
    vf4 hitPoint, normal, tangent, emission, color, spec;
    unsigned hitType;
} hit_t;

/* Sphere::intersect, PathTracer.cu:87-104 */
static float sphere_intersect(const sphere_t *s, const ray_t *r)
{
    vf4 op = sub4(s->pos, r->o);
    float t;
    float eps = (float)1e-4;
    float b = dot4(op, r->d);
    float det = b * b - dot4(op, op) + s->r * s->r;
    if (det < 0) return 0;
    det = sqrtf(det);
    return (t = b - det) > eps ? t : ((t = b + det) > eps ? t : 0.0f);
}

/* intersectTriangle, RayIntersection.cuh:54-111 (Moller-Trumbore, no culling) */
static vf4 intersect_triangle(vf4 v1, vf4 v2, vf4 v3, const ray_t *r)
{
    vf4 e1 = sub4(v2, v1), e2 = sub4(v3, v1);
    vf4 p = cross4(r->d, e2);
    float det = dot4(e1, p);
    if (det > -VR_EPSILON && det < VR_EPSILON) return f4(0, 0, 0, 0);
    float inv_det = 1.0f / det;
    vf4 t = sub4(r->o, v1);
    float u = dot4(t, p) * inv_det;
    if (u < 0.0f || u > 1.0f) return f4(0, 0, 0, 0);
    vf4 q = cross4(t, e1);
    float v = dot4(r->d, q) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return f4(0, 0, 0, 0);
    float dist = dot4(e2, q) * inv_det;
    if (dist > VR_EPSILON) return f4(dist, u, v, 0.0f);
    return f4(0, 0, 0, 0);
}

static inline vf4 ld4(const float *a, size_t i) { return f4(a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]); }
static inline vf2 ld2(const float *a, size_t i) { vf2 r = { a[2 * i], a[2 * i + 1] }; return r; }

/* texture address: PathTracer.cu:209-212 / 398-401 (clamp(int) returns float) */
static inline int tex_addr(uint32_t w, uint32_t h, float u, float v)
{
    int x = f2i((float)w * u);
    int y = f2i((float)h * v);
    int val = (int)((uint32_t)x + (uint32_t)y * w);
    int hi = (int)(w * h - 1u);
    return (int)clampi(val, 0, hi);
}

typedef struct {
    const vro_scene *sc;
    mctx m;
    vro_counters *cnt;      /* thread-local, may be NULL */
    int err;
} tctx;

#define CNT(field, v) do { if (tc->cnt) tc->cnt->field += (v); } while (0)

static inline void set_sphere_hit(hit_t *h, const ray_t *r, float t, const sphere_t *s, vf4 spec)
{
    h->hitPoint = add4(r->o, mul4s(r->d, t));
    h->normal = normalize4(sub4(h->hitPoint, s->pos));
    h->color = s->col;
    h->emission = s->emission;
    h->hitType = (unsigned)s->refl;
    h->spec = spec;
}

/* leaf triangle loop body for one slot run, PathTracer.cu:367-455 */
static void leaf_hit(tctx *tc, const ray_t *r, int triAddr, vf4 vert0, vf4 vert1, vf4 vert2,
                     vf4 I, float *t, hit_t *h)
{
    const vro_scene *sc = tc->sc;
    *t = I.x;
    h->hitPoint = add4(r->o, mul4s(r->d, *t));
    float b0 = 1.0f - I.y - I.z;
    vf2 uv0 = ld2(sc->uvs, triAddr), uv1 = ld2(sc->uvs, triAddr + 1), uv2 = ld2(sc->uvs, triAddr + 2);
    vf2 uv;
    uv.x = (b0 * uv0.x + I.y * uv1.x) + I.z * uv2.x;
    uv.y = (b0 * uv0.y + I.y * uv1.y) + I.z * uv2.y;
    vf4 tangent = normalize4(add4(add4(muls4(b0, ld4(sc->tangents, triAddr)),
                                       muls4(I.y, ld4(sc->tangents, triAddr + 1))),
                                  muls4(I.z, ld4(sc->tangents, triAddr + 2))));
    tangent.w = 0.0f;
    CNT(hits, 1);
    CNT(attr_bytes, 24 + 48);
    if (sc->tex[0] && !sc->view_brdf) {
        int a = tex_addr(sc->tex_w[0], sc->tex_h[0], uv.x, uv.y);
        h->color = ld4(sc->tex[0], a);
        CNT(tex_fetches, 1);
    } else {
        h->color = f4(1.f, 1.f, 1.f, 0.f);
    }
    if (sc->tex[1] && dot4(tangent, tangent) > VR_EPSILON) {
        int a = tex_addr(sc->tex_w[1], sc->tex_h[1], uv.x, uv.y);
        vf4 normal = normalize4(add4(add4(muls4(b0, ld4(sc->normals, triAddr)),
                                          muls4(I.y, ld4(sc->normals, triAddr + 1))),
                                     muls4(I.z, ld4(sc->normals, triAddr + 2))));
        normal.w = 0.0f;
        vf4 bitangent = cross4(normal, tangent);
        vf4 nm = normalize4(sub4(muls4(2.0f, ld4(sc->tex[1], a)), f4(1.f, 1.f, 1.f, 0.f)));
        h->normal = normalize4(tbn_mul(tangent, bitangent, normal, nm));
        CNT(attr_bytes, 48);
        CNT(tex_fetches, 1);
    } else {
        h->normal = normalize4(cross4(sub4(vert0, vert1), sub4(vert0, vert2)));
    }
    if (sc->tex[2] && !sc->view_brdf) {
        int a = tex_addr(sc->tex_w[2], sc->tex_h[2], uv.x, uv.y);
        h->spec = ld4(sc->tex[2], a);
        CNT(tex_fetches, 1);
    } else {
        h->spec = f4(0.f, 0.f, 0.f, 0.f);
    }
    h->tangent = tangent;
    h->emission = f4(0.f, 0.f, 0.f, 0.f);
    h->hitType = sc->view_brdf ? R_BRDF : R_DIFF;
}

static void leaf_loop(tctx *tc, const ray_t *r, int leafAddr, float *t, hit_t *h)
{
    const vro_scene *sc = tc->sc;
    for (int triAddr = ~leafAddr;; triAddr += 3) {
        vf4 vert0 = ld4(sc->verts, triAddr);
        CNT(slot_reads, 1);
        if (fbits(vert0.x) == 0x80000000u) break;
        vf4 vert1 = ld4(sc->verts, triAddr + 1);
        vf4 vert2 = ld4(sc->verts, triAddr + 2);
        CNT(tri_tests, 1);
        vf4 I = intersect_triangle(vert0, vert1, vert2, r);
        if (I.x > VR_EPSILON && I.x < *t) leaf_hit(tc, r, triAddr, vert0, vert1, vert2, I, t, h);
    }
}

/* intersectScene, PathTracer.cu:136-468 */
static int intersect_scene(tctx *tc, const ray_t *r, hit_t *h)
{
    const vro_scene *sc = tc->sc;
    const mctx *m = &tc->m;
    float inf = 1e20f;
    float t = inf;
    CNT(rays, 1);

    if (sc->use_cornell) {                                          /* :149-171 */
        for (unsigned i = 0; i < 6; ++i) {
            float dist = sphere_intersect(&k_cornell[i], r);
            if (dist != 0.f && dist < t) { t = dist; set_sphere_hit(h, r, t, &k_cornell[i], f4(0, 0, 0, 0)); }
        }
    }
    for (int i = 0; i < 2; ++i) {                                   /* :174-190 */
        float dist = sphere_intersect(&k_spheres[i], r);
        if (dist != 0.f && dist < t) { t = dist; set_sphere_hit(h, r, t, &k_spheres[i], f4(1, 1, 1, 0)); }
    }

    if (sc->use_example_sphere) {                                   /* :192-268 */
        float dist = sphere_intersect(&k_example, r);
        if (dist != 0.f && dist < t) {
            t = dist;
            h->hitPoint = add4(r->o, mul4s(r->d, t));
            /* u,v from the (stale) normal of this call's previous hit, :202-204 */
            float u = m_atan2f(m, h->normal.x, h->normal.z) / (2.f * VR_PI) + 0.5f;
            float v = h->normal.y * 0.5f + 0.5f;
            if (sc->tex[0] && !sc->view_brdf) {
                h->color = ld4(sc->tex[0], tex_addr(sc->tex_w[0], sc->tex_h[0], u, v));
                CNT(tex_fetches, 1);
            } else {
                h->color = k_example.col;
            }
            if (sc->tex[1]) {
                int a = tex_addr(sc->tex_w[1], sc->tex_h[1], u, v);
                vf4 normal = normalize4(sub4(h->hitPoint, k_example.pos));
                normal.w = 0.0f;
                float rr = sqrtf(dot4(h->hitPoint, h->hitPoint));
                float theta = m_acosf(m, h->hitPoint.z / rr);
                float phi = m_atan2f(m, h->hitPoint.y, h->hitPoint.x);
                float st, ct, sph, cph;
                m_sincos(m, theta, &st, &ct);
                m_sincos(m, phi, &sph, &cph);
                h->tangent = f4(st * cph, st * sph, ct, 0.0f);
                vf4 bitangent = cross4(normal, h->tangent);
                vf4 nm = normalize4(sub4(muls4(2.0f, ld4(sc->tex[1], a)), f4(1.f, 1.f, 1.f, 0.f)));
                h->normal = normalize4(tbn_mul(h->tangent, bitangent, normal, nm));
                CNT(tex_fetches, 1);
            } else {
                h->normal = normalize4(sub4(h->hitPoint, k_example.pos));
            }
            if (sc->tex[2] && !sc->view_brdf) {
                h->spec = ld4(sc->tex[2], tex_addr(sc->tex_w[2], sc->tex_h[2], u, v));
                CNT(tex_fetches, 1);
            } else {
                h->spec = f4(0.f, 0.f, 0.f, 0.f);
            }
            h->emission = k_example.emission;
            h->hitType = sc->view_brdf ? R_BRDF : R_DIFF;
        }
    } else if (sc->mesh_initialised && sc->brute_force) {
        /* validation mode: every slot, array order (result equals the BVH
         * traversal except for exact-t ties between different triangles) */
        size_t i = 0;
        while (i < sc->n_slots) {
            vf4 vert0 = ld4(sc->verts, i);
            if (fbits(vert0.x) == 0x80000000u) { i += 1; continue; }
            vf4 vert1 = ld4(sc->verts, i + 1), vert2 = ld4(sc->verts, i + 2);
            vf4 I = intersect_triangle(vert0, vert1, vert2, r);
            if (I.x > VR_EPSILON && I.x < t) leaf_hit(tc, r, (int)i, vert0, vert1, vert2, I, &t, h);
            i += 3;
        }
    } else if (sc->mesh_initialised) {                              /* :269-464 */
        const int Sentinel = 0x76543210;
        int stack[64];
        int sp = 0;
        stack[0] = Sentinel;
        int leafAddr = 0;
        int nodeAddr = 0;
        float ivx = 1.f / (fabsf(r->d.x) > VR_EPSILON ? r->d.x : VR_EPSILON);
        float ivy = 1.f / (fabsf(r->d.y) > VR_EPSILON ? r->d.y : VR_EPSILON);
        float ivz = 1.f / (fabsf(r->d.z) > VR_EPSILON ? r->d.z : VR_EPSILON);
        float odx = r->o.x * ivx, ody = r->o.y * ivy, odz = r->o.z * ivz;
        const float *B = sc->bvh;

        while (nodeAddr != Sentinel) {
            while ((unsigned)nodeAddr < (unsigned)Sentinel) {
                const float *n = B + 4 * (size_t)nodeAddr;
                CNT(node_visits, 1);
                int idx0 = fibits(n[12]), idx1 = fibits(n[13]);
                const float c0lox = n[0] * ivx - odx;
                const float c0hix = n[1] * ivx - odx;
                const float c0loy = n[2] * ivy - ody;
                const float c0hiy = n[3] * ivy - ody;
                const float c0loz = n[8] * ivz - odz;
                const float c0hiz = n[9] * ivz - odz;
                const float c1loz = n[10] * ivz - odz;
                const float c1hiz = n[11] * ivz - odz;
                const float c0min = span_begin(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 0.0f);
                const float c0max = span_end(c0lox, c0hix, c0loy, c0hiy, c0loz, c0hiz, 1e20f);
                const float c1lox = n[4] * ivx - odx;
                const float c1hix = n[5] * ivx - odx;
                const float c1loy = n[6] * ivy - ody;
                const float c1hiy = n[7] * ivy - ody;
                const float c1min = span_begin(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, 0.0f);
                const float c1max = span_end(c1lox, c1hix, c1loy, c1hiy, c1loz, c1hiz, 1e20f);
                int swp = (c1min < c0min);
                int tc0 = (c0max >= c0min);
                int tc1 = (c1max >= c1min);
                if (!tc0 && !tc1) {
                    nodeAddr = stack[sp--];
                } else {
                    nodeAddr = tc0 ? idx0 : idx1;
                    if (tc0 && tc1) {
                        if (swp) { int tmp = nodeAddr; nodeAddr = idx1; idx1 = tmp; }
                        if (sp + 1 >= 64) { tc->err = -3; return 0; }
                        stack[++sp] = idx1;
                        if (tc->cnt && (uint64_t)sp > tc->cnt->max_stack) tc->cnt->max_stack = (uint64_t)sp;
                    }
                }
                if (nodeAddr < 0 && leafAddr >= 0) {                /* postpone max 1 */
                    leafAddr = nodeAddr;
                    nodeAddr = stack[sp--];
                }
                /* single-lane vote.ballot(leafAddr >= 0), :353-363 */
                if (!(leafAddr >= 0)) break;
            }
            while (leafAddr < 0) {                                  /* :365-462 */
                leaf_loop(tc, r, leafAddr, &t, h);
                leafAddr = nodeAddr;
                if (nodeAddr < 0) nodeAddr = stack[sp--];
            }
        }
    }
    return t < inf;
}

/* MERL index maps, PathTracer.cu:473-506 */
static int phi_diff_index(float phi_diff)
{
    if (phi_diff < 0.0) phi_diff = (float)((double)phi_diff + M_PI);
    return (int)clampi(d2i((double)phi_diff * (1.0 / (double)VR_PI * (360 / 2))), 0, 360 / 2 - 1);
}
static int theta_half_index(float theta_half)
{
    if (theta_half <= 0.0) return 0;
    float s = sqrtf((float)((double)theta_half * (2.0 / (double)VR_PI)));
    return (int)clampi(f2i(s * 90), 0, 90 - 1);
}
static int theta_diff_index(float theta_diff)
{
    return (int)clampi(d2i((double)theta_diff * (2.0 / (double)VR_PI * 90)), 0, 90 - 1);
}

/* lookupBRDF index part, PathTracer.cu:519-554 */
static int brdf_index(const mctx *m, vf4 refl, vf4 cur, vf4 normal, vf4 tangent)
{
    vf4 bitangent = cross4(normal, tangent);
    vf4 H = normalize4(sub4(refl, cur));
    float theta_H = m_acosf(m, clampf(dot4(normal, H), 0.f, 1.f));
    float theta_diff = m_acosf(m, clampf(dot4(H, refl), 0.f, 1.f));
    float phi_diff = 0.f;
    if ((double)theta_diff < 1e-3) {
        phi_diff = m_atan2f(m, clampf(-dot4(refl, bitangent), -1.f, 1.f), clampf(dot4(refl, tangent), -1.f, 1.f));
    } else if ((double)theta_H > 1e-3) {
        vf4 u = muls4(-1.f, normalize4(sub4(normal, muls4(dot4(normal, H), H))));
        vf4 v = cross4(H, u);
        phi_diff = m_atan2f(m, clampf(dot4(refl, v), -1.f, 1.f), clampf(dot4(refl, u), -1.f, 1.f));
    } else {
        theta_H = 0.f;
    }
    return phi_diff_index(phi_diff) + theta_diff_index(theta_diff) * 360 / 2
           + theta_half_index(theta_H) * 360 / 2 * 90;
}

/* PathTracer.cu:556-565 */
static vf4 lookup_brdf(tctx *tc, vf4 refl, vf4 cur, vf4 normal, vf4 tangent)
{
    int ind = brdf_index(&tc->m, refl, cur, normal, tangent);
    const float *T = tc->sc->brdf;
    CNT(brdf_fetches, 1);
    return f4((float)((double)T[ind] * (1.0 / 1500.0)),
              (float)((double)T[ind + 1458000] * (1.15 / 1500.0)),
              (float)((double)T[ind + 2916000] * (1.66 / 1500.0)),
              0.f);
}

/* hash, PathTracer.cu:574-580 */
uint32_t vro_hash(uint32_t *seed0, uint32_t *seed1)
{
    *seed0 = 36969u * ((*seed0) & 65535u) + ((*seed0) >> 16);
    *seed1 = 18000u * ((*seed1) & 65535u) + ((*seed1) >> 16);
    return *seed0 * *seed1;
}

/* thrust::minstd_rand (linear_congruential_engine<uint32, 48271, 0, 2^31-1>)
 * seeded with s -> s % m, or 1 if that is 0; uniform_real_distribution<float>
 * (0,1): float(x - 1) / (1.0f + float(2^31 - 3)) = float(x-1) * 2^-31.
 * rocThrust 7.2 random/detail/{linear_congruential_engine.inl,mod.h,
 * uniform_real_distribution.inl}; PathTracer.cu:620-622. */
typedef struct { uint32_t x; } rng_t;
static inline void rng_seed(rng_t *g, uint32_t s) { uint32_t v = s % 2147483647u; g->x = v ? v : 1u; }
static inline float rng_uniform(rng_t *g)
{
    g->x = (uint32_t)(((uint64_t)g->x * 48271u) % 2147483647u);
    float r = (float)(g->x - 1u);
    r /= (1.0f + (float)(2147483646u - 1u));
    return r * (1.0f - 0.0f) + 0.0f;
}

void vro_rng_uniforms(uint32_t seed, int n, float *out)
{
    rng_t g; rng_seed(&g, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_uniform(&g);
}

/* trace, PathTracer.cu:597-770 */
static vf4 trace(tctx *tc, const ray_t *camray, uint32_t *s0, uint32_t *s1)
{
    const vro_scene *sc = tc->sc;
    const mctx *m = &tc->m;
    ray_t ray = *camray;
    vf4 accum = f4(0.f, 0.f, 0.f, 0.f);
    vf4 mask = f4(1.f, 1.f, 1.f, 0.f);
    float depth = 1.f;
    uint32_t seed = vro_hash(s0, s1);
    rng_t rng; rng_seed(&rng, seed);
    CNT(paths, 1);

    for (unsigned bounces = 0; bounces < 4; bounces++) {
        hit_t h;
        memset(&h, 0, sizeof(h));   /* the reference leaves vHitData uninitialised; defined as zero */
        if (!intersect_scene(tc, &ray, &h)) {
            if (!sc->use_cornell) {                                 /* :631-648 */
                float lx = m_atan2f(m, ray.d.x, ray.d.z);
                float ly = m_acosf(m, ray.d.y);
                lx = lx < 0 ? (float)((double)lx + 2.0 * (double)VR_PI) : lx;
                lx = (float)((double)lx / (2.0 * (double)VR_PI));
                ly = ly / VR_PI;
                int x = f2i(lx * (float)sc->hdr_w);
                int y = f2i(ly * (float)sc->hdr_h);
                int val = (int)((uint32_t)x + (uint32_t)y * sc->hdr_w);
                int addr = (int)clampi(val, 0, (int)(sc->hdr_w * sc->hdr_h - 1u));
                addeq4(&accum, mul4(mul4s(mask, 2.f), ld4(sc->hdr, addr)));
                CNT(hdr_fetches, 1);
                accum.w = depth;
                return accum;
            }
            return f4(0.f, 0.f, 0.f, 0.f);                          /* :649-652 */
        }
        if (bounces == 0) {                                         /* :656-661 */
            vf4 l = sub4(ray.o, h.hitPoint);
            depth = sqrtf(dot4(l, l)) / 150.f;
        }
        addeq4(&accum, mul4(mask, h.emission));                     /* :664 */
        ray.o = h.hitPoint;
        vf4 normal = h.normal;

        if (h.hitType == 0) {                                       /* :671-676 */
            ray.d = sub4(ray.d, mul4s(mul4s(normal, 2.f), dot4(normal, ray.d)));
            addeq4(&ray.o, mul4s(normal, 0.05f));
        } else if (h.hitType == 1) {                                /* :678-722 */
            float aoi = dot4(h.normal, muls4(-1.f, ray.d));
            float fe = lerpf_(m_powf(m, 1.f - aoi, sc->fresnel_pow), 1.f, sc->fresnel_coef) * h.spec.x;
            int reflect = (rng_uniform(&rng) < fe);
            vf4 newdir;
            vf4 w = normal;
            vf4 axis = fabsf(w.x) > 0.1f ? f4(0.f, 1.f, 0.f, 0.f) : f4(1.f, 0.f, 0.f, 0.f);
            if (reflect) {
                muleq4(&mask, h.spec);
                newdir = normalize4(sub4(ray.d, mul4s(mul4s(normal, 2.f), dot4(normal, ray.d))));
            } else {
                float rand1 = 2.f * VR_PI * rng_uniform(&rng);
                float rand2 = rng_uniform(&rng);
                float rand2s = sqrtf(rand2);
                vf4 u = normalize4(cross4(axis, w));
                vf4 v = cross4(w, u);
                float sn, cs;
                m_sincos(m, rand1, &sn, &cs);
                newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                         mul4s(w, sqrtf(1 - rand2))));
                muleq4(&mask, h.color);
                muleq4s(&mask, dot4(newdir, normal));
                muleq4s(&mask, 2.f);
            }
            addeq4(&ray.o, mul4s(normal, 0.05f));
            ray.d = newdir;
        } else if (h.hitType == 2) {                                /* :724-764 */
            vf4 w = normal;
            vf4 axis = fabsf(w.x) > 0.1f ? f4(0.f, 1.f, 0.f, 0.f) : f4(1.f, 0.f, 0.f, 0.f);
            float rand1 = 2.f * VR_PI * rng_uniform(&rng);
            float rand2 = rng_uniform(&rng);
            float rand2s = sqrtf(rand2);
            vf4 u = normalize4(cross4(axis, w));
            vf4 v = cross4(w, u);
            float sn, cs;
            m_sincos(m, rand1, &sn, &cs);
            vf4 newdir = normalize4(add4(add4(mul4s(mul4s(u, cs), rand2s), mul4s(mul4s(v, sn), rand2s)),
                                         mul4s(w, sqrtf(1 - rand2))));
            if (sc->brdf) {
                float dw = 24 * m_powf(m, newdir.x * newdir.x + newdir.y * newdir.y + newdir.z * newdir.z, -1.5f);
                muleq4(&mask, muls4(dw, max4(lookup_brdf(tc, newdir, ray.d, h.normal, h.tangent), f4(0, 0, 0, 0))));
            } else {
                muleq4(&mask, h.color);
                muleq4s(&mask, dot4(newdir, normal));
                muleq4s(&mask, 2.f);
            }
            addeq4(&ray.o, mul4s(normal, 0.05f));
            ray.d = newdir;
        }
    }
    accum.w = depth;
    return accum;
}

static void camera_basis(const vro_scene *sc, vf4 *cx, vf4 *cy)
{
    vf4 right = f4(sc->cam_right[0], sc->cam_right[1], sc->cam_right[2], sc->cam_right[3]);
    vf4 up = f4(sc->cam_up[0], sc->cam_up[1], sc->cam_up[2], sc->cam_up[3]);
    *cx = muls4(sc->fov_scale * (float)sc->width / (float)sc->height, right);   /* :833 */
    *cy = muls4(sc->fov_scale, up);                                             /* :836 */
}

static ray_t primary_ray(const vro_scene *sc, vf4 cx, vf4 cy, uint32_t x, uint32_t y)
{
    vf4 dir = f4(sc->cam_dir[0], sc->cam_dir[1], sc->cam_dir[2], sc->cam_dir[3]);
    float sx = (float)((0.25 + (double)x) / (double)sc->width - 0.5);          /* :842 */
    float sy = (float)((0.25 + (double)y) / (double)sc->height - 0.5);
    vf4 d = add4(add4(dir, mul4s(cx, sx)), mul4s(cy, sy));
    ray_t r;
    r.o = f4(sc->cam_origin[0], sc->cam_origin[1], sc->cam_origin[2], sc->cam_origin[3]);
    r.d = normalize4(d);
    return r;
}

void vro_primary_ray(const vro_scene *sc, uint32_t x, uint32_t y, float *o4, float *d4)
{
    vf4 cx, cy; camera_basis(sc, &cx, &cy);
    ray_t r = primary_ray(sc, cx, cy, x, y);
    memcpy(o4, &r.o, 16); memcpy(d4, &r.d, 16);
}

void vro_trace_sample(const vro_scene *sc, uint32_t x, uint32_t y, uint32_t frame,
                      uint32_t time, int sample, float *out4)
{
    tctx tc = { sc, { sc->libm }, NULL, 0 };
    vf4 cx, cy; camera_basis(sc, &cx, &cy);
    uint32_t s1 = x * frame, s2 = y * time;
    vf4 res = f4(0, 0, 0, 0);
    for (int s = 0; s <= sample; ++s) {
        ray_t r = primary_ray(sc, cx, cy, x, y);
        res = trace(&tc, &r, &s1, &s2);
    }
    memcpy(out4, &res, 16);
}

/* render, PathTracer.cu:791-868, for one frame over a row range */
static void render_row(tctx *tc, float *accum, uint8_t *rgba, uint8_t *depthbuf,
                       uint32_t y, uint32_t frame, uint32_t time, uint32_t wr, vf4 cx, vf4 cy)
{
    const vro_scene *sc = tc->sc;
    const uint32_t W = sc->width;
    for (uint32_t x = 0; x < wr; ++x) {
        uint32_t ind = x + y * W;
        uint32_t s1 = x * frame;
        uint32_t s2 = y * time;
        vf4 *io = (vf4 *)(accum + 4 * (size_t)ind);
        if (frame == 1) *io = f4(0.f, 0.f, 0.f, 0.f);
        for (unsigned s = 0; s < 2; ++s) {
            ray_t r = primary_ray(sc, cx, cy, x, y);
            vf4 result = trace(tc, &r, &s1, &s2);
            uint8_t db = f2u8((1.f - result.w) * 255);
            if (depthbuf) {
                uint8_t *dp = depthbuf + 4 * (size_t)ind;
                dp[0] = db; dp[1] = db; dp[2] = db; dp[3] = 0xff;
            }
            addeq4(io, mul4s(result, 1.f / 2.f));
        }
        float coef = 1.f / (float)frame;
        vf4 color = clamp4(mul4s(*io, coef), 0.f, 1.f);
        const mctx *m = &tc->m;
        const float inv_gamma = 1.f / 2.2f;
        if (rgba) {
            uint8_t *p = rgba + 4 * (size_t)ind;
            p[0] = f2u8(m_powf(m, color.x, inv_gamma) * 255);
            p[1] = f2u8(m_powf(m, color.y, inv_gamma) * 255);
            p[2] = f2u8(m_powf(m, color.z, inv_gamma) * 255);
            p[3] = 0xff;
        }
        if (tc->cnt) tc->cnt->pixel_io_bytes += 92 + (frame == 1 ? 16 : 0);
    }
}

int vro_render(const vro_scene *sc, float *accum, uint8_t *rgba, uint8_t *depth,
               uint32_t first_frame, uint32_t n_frames, const uint32_t *times,
               uint32_t row_begin, uint32_t row_end, int n_threads, vro_counters *cnt)
{
    if (!sc || !accum || !times) return -1;
    if (!sc->use_cornell && !sc->hdr) return -2;            /* reference would read a null _hdr */
    const uint32_t wr = (sc->width / 16) * 16;               /* grid truncation, :888-889 */
    const uint32_t hr = (sc->height / 16) * 16;
    if (row_end > hr) row_end = hr;
    if (row_begin >= row_end) return 0;
    vf4 cx, cy; camera_basis(sc, &cx, &cy);
    int err = 0;
    if (cnt) memset(cnt, 0, sizeof(*cnt));
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    for (uint32_t f = 0; f < n_frames; ++f) {
        uint32_t frame = first_frame + f, time = times[f];
#pragma omp parallel
        {
            vro_counters local;
            memset(&local, 0, sizeof(local));
            tctx tc = { sc, { sc->libm }, cnt ? &local : NULL, 0 };
#pragma omp for schedule(dynamic, 1)
            for (int64_t y = row_begin; y < (int64_t)row_end; ++y)
                render_row(&tc, accum, rgba, depth, (uint32_t)y, frame, time, wr, cx, cy);
#pragma omp critical
            {
                if (tc.err) err = tc.err;
                if (cnt) {
                    uint64_t *dst = (uint64_t *)cnt, *src = (uint64_t *)&local;
                    size_t nf = sizeof(vro_counters) / sizeof(uint64_t);
                    for (size_t i = 0; i + 1 < nf; ++i) dst[i] += src[i];
                    if (local.max_stack > cnt->max_stack) cnt->max_stack = local.max_stack;
                }
            }
        }
        if (err) return err;
    }
    return 0;
}

/* ---- known-answer helpers ---- */
void vro_intersect_triangle(const float *v0, const float *v1, const float *v2,
                            const float *o, const float *d, float *out4)
{
    ray_t r; memcpy(&r.o, o, 16); memcpy(&r.d, d, 16);
    vf4 a, b, c; memcpy(&a, v0, 16); memcpy(&b, v1, 16); memcpy(&c, v2, 16);
    vf4 res = intersect_triangle(a, b, c, &r);
    memcpy(out4, &res, 16);
}

float vro_sphere_intersect(int which, const float *o, const float *d)
{
    ray_t r; memcpy(&r.o, o, 16); memcpy(&r.d, d, 16);
    const sphere_t *s = which < 6 ? &k_cornell[which] : (which < 8 ? &k_spheres[which - 6] : &k_example);
    return sphere_intersect(s, &r);
}

int vro_brdf_index(const float *refl, const float *cur, const float *n, const float *t, int libm)
{
    mctx m = { libm };
    vf4 a, b, c, e; memcpy(&a, refl, 16); memcpy(&b, cur, 16); memcpy(&c, n, 16); memcpy(&e, t, 16);
    return brdf_index(&m, a, b, c, e);
}

void vro_span(const float *s, float *be)
{
    be[0] = span_begin(s[0], s[1], s[2], s[3], s[4], s[5], 0.0f);
    be[1] = span_end(s[0], s[1], s[2], s[3], s[4], s[5], 1e20f);
}
