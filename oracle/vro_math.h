/*
 * vro_math.h -- ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Portable, bit-reproducible single-precision libm used by the CPU oracle in
 * "portable" mode.  The HIP kernel carries its own independent copy
 * (vrenderer_pathtracer_amd/csrc/vr_math.hpp) written to the same spec; the
 * GPU self-test compares the two bit for bit.  Every function uses only IEEE
 * basic operations (+ - * / sqrt, fmaf/fma) in a fixed order, so a compiler
 * with -ffp-contract=off produces identical bits on x86-64 and gfx950.
 *
 * Why: the reference kernel (cuda/src/PathTracer.cu) calls sinf/cosf/acosf/
 * atan2f/powf; its build uses nvcc --use_fast_math (vRenderer.pri:48), so no
 * single libm is "the" reference.  Glibc mode (the default oracle) uses the
 * host libm; portable mode uses these, which are within ~1 ulp of glibc and
 * give the GPU an exactly reproducible target.
 */
#ifndef VRO_MATH_H
#define VRO_MATH_H

#ifdef __cplusplus
extern "C" {
#endif

void  vro_p_sincosf(float x, float *s, float *c);
float vro_p_sinf(float x);
float vro_p_cosf(float x);
float vro_p_atanf(float x);
float vro_p_atan2f(float y, float x);
float vro_p_acosf(float x);
float vro_p_powf(float x, float y);

#ifdef __cplusplus
}
#endif
#endif
