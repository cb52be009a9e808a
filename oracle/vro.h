/*
 * vro.h -- CPU ORACLE for the vRenderer path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libvrhip.so, the
 * vRendererHIP adapter, the Python host mirror) may link, load or call this
 * code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, as the checker / CPU baseline.
 *
 * It is a plain-C restatement of the reference CUDA megakernel
 * (/root/reference/cuda/src/PathTracer.cu:87-868 and the helpers in
 * cuda/include/{MathHelpers,RayIntersection}.cuh), operating on the
 * reference's flattened scene layout (src/vRendererCuda.cpp:204-279).
 * Semantics = the reference algorithm evaluated in IEEE fp32 with no FMA
 * contraction, correctly rounded division/sqrt, rsqrtf(x) := 1/sqrtf(x), and
 * one of two libms (glibc, or the portable vro_math.c).
 */
#ifndef VRO_H
#define VRO_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { VRO_LIBM_GLIBC = 0, VRO_LIBM_PORTABLE = 1 };

typedef struct vro_scene {
    /* vCamera (cuda/include/PathTracer.cuh:58-84) */
    float cam_origin[4], cam_dir[4], cam_up[4], cam_right[4];
    float fov_scale;
    uint32_t width, height;
    float fresnel_coef, fresnel_pow;
    /* __constant__ flags (cuda/src/PathTracer.cu:25-32) */
    int use_cornell, use_example_sphere, view_brdf, mesh_initialised;
    /* flattened mesh (src/vRendererCuda.cpp:204-279); float4 / float2 arrays */
    const float *bvh;       size_t n_bvh_f4;
    const float *verts;     /* float4[n_slots] */
    const float *normals;   /* float4[n_slots] */
    const float *tangents;  /* float4[n_slots] */
    const float *uvs;       /* float2[n_slots] */
    size_t n_slots;
    /* environment (float4[hdr_w*hdr_h]) */
    const float *hdr; uint32_t hdr_w, hdr_h;
    /* textures: 0 diffuse, 1 normal, 2 specular (float4[w*h]); NULL if unset */
    const float *tex[3]; uint32_t tex_w[3], tex_h[3];
    /* MERL table, float[3*1458000] planar R,G,B; NULL if unset */
    const float *brdf;
    int libm;               /* VRO_LIBM_* */
    int brute_force;        /* 1: test every triangle slot instead of the BVH */
} vro_scene;

typedef struct vro_counters {
    uint64_t paths, rays, node_visits, slot_reads, tri_tests, hits;
    uint64_t attr_bytes, tex_fetches, hdr_fetches, brdf_fetches;
    uint64_t pixel_io_bytes, max_stack;
} vro_counters;

/* Render n_frames frames (frame numbers first_frame .. first_frame+n-1, with
 * per-frame _time seeds times[i]) over rows [row_begin, row_end) of the
 * reference's rendered region (grid truncation, PathTracer.cu:888-889).
 * accum: float4[W*H] in/out (io_colors); rgba, depth: uchar4[W*H] out (may
 * be NULL).  n_threads <= 0: OpenMP default.  cnt may be NULL.
 * Returns 0, or a negative error code (e.g. traversal stack overflow). */
int vro_render(const vro_scene *sc, float *accum, uint8_t *rgba, uint8_t *depth,
               uint32_t first_frame, uint32_t n_frames, const uint32_t *times,
               uint32_t row_begin, uint32_t row_end, int n_threads,
               vro_counters *cnt);

/* ---- known-answer helpers (unit tests) ---- */
uint32_t vro_hash(uint32_t *s0, uint32_t *s1);                 /* PathTracer.cu:574-580 */
void vro_rng_uniforms(uint32_t seed, int n, float *out);       /* thrust minstd + uniform_real */
void vro_intersect_triangle(const float *v0, const float *v1, const float *v2,
                            const float *o, const float *d, float *out4);
float vro_sphere_intersect(int which, const float *o, const float *d);
int vro_brdf_index(const float *refl, const float *cur, const float *n, const float *t, int libm);
void vro_span(const float *six, float *begin_end);             /* MathHelpers.cuh:544-552 */
void vro_primary_ray(const vro_scene *sc, uint32_t x, uint32_t y, float *o4, float *d4);
/* trace one path from (x,y) at (frame,time) sample s; returns float4 */
void vro_trace_sample(const vro_scene *sc, uint32_t x, uint32_t y, uint32_t frame,
                      uint32_t time, int sample, float *out4);

#ifdef __cplusplus
}
#endif
#endif
