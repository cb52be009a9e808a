// vr_math.hpp -- device libm for the gfx950 path tracer.
//
// The reference kernel calls sinf/cosf/acosf/atan2f/powf
// (cuda/src/PathTracer.cu:202,233-235,528-542,636,684,711,740,747,860) under
// nvcc --use_fast_math (vRenderer.pri:48).  Here every transcendental is a
// fixed sequence of IEEE operations (basic ops, sqrt, fma) so the result is
// bit-reproducible on the host: sincos and pow are evaluated in double and
// rounded once (nearly always the correctly rounded float), atan2/acos follow
// the fdlibm float algorithms.  Compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vr {

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint64_t dbits(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double bitsd(uint64_t u) { return __longlong_as_double((long long)u); }

// Polynomial constants are materialised into an SGPR pair at each use: gfx9
// VOP3 has no 64-bit literal, and letting the compiler hoist ~40 of them out
// of the bounce loop into VGPR pairs costs registers (and occupancy).
//
// Two forms.  The path-pool kernels (mesh scenes, bound by the texture
// path) produce each constant by two s_mov_b32 inside volatile asm at the
// point of use, so it can neither be hoisted nor kept live in SGPRs across
// the loop (r05: C2 path kernel SGPR spills 82 -> 41, VGPR spills 2 -> 0,
// C2 +1.0 %, C3 +0.8 %, C5 +1.4 %).  The sphere-only kernels (C1, C4 and the
// sphere classes: VALU-bound, no traversal state) keep the round-4 form, an
// asm that pins an SGPR pair the compiler may materialise once per loop: the
// per-use s_mov pairs cost them 1-3 % (translation units that define
// VR_DK_HOISTED before including this header).
#ifndef VR_DK_HOISTED
template <uint64_t B>
__device__ __forceinline__ double dk_bits()
{
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((int32_t)(uint32_t)B));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((int32_t)(uint32_t)(B >> 32)));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
#define dk(c) dk_bits<__builtin_bit_cast(uint64_t, (double)(c))>()
#else
__device__ __forceinline__ double dk(double c) { asm volatile("" : "+s"(c)); return c; }
#endif

// ------------------------------------------------------------------ sincos
__device__ __forceinline__ void sincos_p(float x, float* s, float* c)
{
    if (!(__builtin_fabsf(x) <= 1.0e6f)) { *s = bitsf(0x7fc00000u); *c = bitsf(0x7fc00000u); return; }
    const double xd = (double)x;
    const double k = __builtin_rint(xd * dk(0.6366197723675814));
    double r = __builtin_fma(-k, dk(1.5707963267948966), xd);
    r = __builtin_fma(-k, dk(6.123233995736766e-17), r);
    const double z = r * r;
    double ps = dk(-1.0 / 1307674368000.0);
    ps = __builtin_fma(ps, z, dk(1.0 / 6227020800.0));
    ps = __builtin_fma(ps, z, dk(-1.0 / 39916800.0));
    ps = __builtin_fma(ps, z, dk(1.0 / 362880.0));
    ps = __builtin_fma(ps, z, dk(-1.0 / 5040.0));
    ps = __builtin_fma(ps, z, dk(1.0 / 120.0));
    ps = __builtin_fma(ps, z, dk(-1.0 / 6.0));
    const double sd = __builtin_fma(r * z, ps, r);
    double pc = dk(1.0 / 20922789888000.0);
    pc = __builtin_fma(pc, z, dk(-1.0 / 87178291200.0));
    pc = __builtin_fma(pc, z, dk(1.0 / 479001600.0));
    pc = __builtin_fma(pc, z, dk(-1.0 / 3628800.0));
    pc = __builtin_fma(pc, z, dk(1.0 / 40320.0));
    pc = __builtin_fma(pc, z, dk(-1.0 / 720.0));
    pc = __builtin_fma(pc, z, dk(1.0 / 24.0));
    pc = __builtin_fma(pc, z, dk(-0.5));
    const double cd = __builtin_fma(z, pc, dk(1.0));
    const float sp = (float)sd, cp = (float)cd;
    const int q = ((int)k) & 3;
    float so, co;
    if (q == 0)      { so = sp;  co = cp;  }
    else if (q == 1) { so = cp;  co = -sp; }
    else if (q == 2) { so = -sp; co = -cp; }
    else             { so = -cp; co = sp;  }
    *s = so; *c = co;
}

// -------------------------------------------------------------------- atan
__device__ __forceinline__ float atan_p(float x)
{
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
                atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
                atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
    const uint32_t hx = fbits(x);
    const uint32_t ix = hx & 0x7fffffffu;
    const bool neg = (hx >> 31) != 0;
    int id;
    if (ix >= 0x4c800000u) {
        if (ix > 0x7f800000u) return x + x;
        return neg ? -atanhi3 - atanlo3 : atanhi3 + atanlo3;
    }
    if (ix < 0x3ee00000u) {
        if (ix < 0x39800000u) return x;
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000u) {
            if (ix < 0x3f300000u) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else                  { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000u) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else                  { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (3.3333328366e-01f + w * (1.4253635705e-01f + w * 6.1687607318e-02f));
    const float s2 = w * (-1.9999158382e-01f + w * -1.0648017377e-01f);
    if (id < 0) return x - x * (s1 + s2);
    const float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
    const float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
    const float r = hi - ((x * (s1 + s2) - lo) - x);
    return neg ? -r : r;
}

__device__ __forceinline__ float atan2_p(float y, float x)
{
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const float pio2 = 1.5707963705e+00f, pio4 = 7.8539818525e-01f;
    const uint32_t hx = fbits(x), hy = fbits(y);
    const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
    if (hx == 0x3f800000u) return atan_p(y);
    int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));
    if (iy == 0) {
        if (m == 0 || m == 1) return y;
        return (m == 2) ? pi : -pi;
    }
    if (ix == 0) return (hy >> 31) ? -pio2 : pio2;
    if (ix == 0x7f800000u) {
        if (iy == 0x7f800000u) {
            if (m == 0) return pio4;
            if (m == 1) return -pio4;
            if (m == 2) return 3.0f * pio4;
            return -3.0f * pio4;
        }
        if (m == 0) return 0.0f;
        if (m == 1) return -0.0f;
        if (m == 2) return pi;
        return -pi;
    }
    if (iy == 0x7f800000u) return (hy >> 31) ? -pio2 : pio2;
    const int k = ((int)iy - (int)ix) >> 23;
    float z;
    if (k > 26) { z = pio2 + 0.5f * pi_lo; m &= 1; }
    else if (k < -26 && (hx >> 31)) z = 0.0f;
    else z = atan_p(__builtin_fabsf(y / x));
    if (m == 0) return z;
    if (m == 1) return -z;
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

// -------------------------------------------------------------------- acos
__device__ __forceinline__ float acos_p(float x)
{
    const float pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    const float pS0 = 1.6666586697e-01f, pS1 = -4.2743422091e-02f, pS2 = -8.6563630030e-03f,
                qS1 = -7.0662963390e-01f;
    const uint32_t hx = fbits(x);
    const uint32_t ix = hx & 0x7fffffffu;
    if (ix >= 0x3f800000u) {
        if (ix == 0x3f800000u) return (hx >> 31) ? pi + 2.0f * pio2_lo : 0.0f;
        return bitsf(0x7fc00000u);
    }
    if (ix < 0x3f000000u) {
        if (ix <= 0x32800000u) return pio2_hi + pio2_lo;
        const float z = x * x;
        const float p = z * (pS0 + z * (pS1 + z * pS2));
        const float q = 1.0f + z * qS1;
        const float r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx >> 31) {
        const float z = (1.0f + x) * 0.5f;
        const float p = z * (pS0 + z * (pS1 + z * pS2));
        const float q = 1.0f + z * qS1;
        const float s = __builtin_sqrtf(z);
        const float r = p / q;
        const float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    } else {
        const float z = (1.0f - x) * 0.5f;
        const float s = __builtin_sqrtf(z);
        const float df = bitsf(fbits(s) & 0xfffff000u);
        const float c = (z - df * df) / (s + df);
        const float p = z * (pS0 + z * (pS1 + z * pS2));
        const float q = 1.0f + z * qS1;
        const float r = p / q;
        const float w = r * s + c;
        return 2.0f * (df + w);
    }
}

// --------------------------------------------------------------------- pow
__device__ __forceinline__ double log2d_p(double x)
{
    const uint64_t b = dbits(x);
    int e = (int)((b >> 52) & 0x7ffu) - 1023;
    double m = bitsd((b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    const double t = (m - 1.0) / (m + 1.0);
    const double t2 = t * t;
    double p = dk(1.0 / 23.0);
    p = __builtin_fma(p, t2, dk(1.0 / 21.0));
    p = __builtin_fma(p, t2, dk(1.0 / 19.0));
    p = __builtin_fma(p, t2, dk(1.0 / 17.0));
    p = __builtin_fma(p, t2, dk(1.0 / 15.0));
    p = __builtin_fma(p, t2, dk(1.0 / 13.0));
    p = __builtin_fma(p, t2, dk(1.0 / 11.0));
    p = __builtin_fma(p, t2, dk(1.0 / 9.0));
    p = __builtin_fma(p, t2, dk(1.0 / 7.0));
    p = __builtin_fma(p, t2, dk(1.0 / 5.0));
    p = __builtin_fma(p, t2, dk(1.0 / 3.0));
    const double lnm = 2.0 * __builtin_fma(t * t2, p, t);
    return __builtin_fma(lnm, dk(1.4426950408889634), (double)e);
}

__device__ __forceinline__ double exp2d_p(double z)
{
    const double k = __builtin_rint(z);
    const double f = z - k;
    const double g = f * dk(0.6931471805599453);
    double p = dk(1.0 / 6227020800.0);
    p = __builtin_fma(p, g, dk(1.0 / 479001600.0));
    p = __builtin_fma(p, g, dk(1.0 / 39916800.0));
    p = __builtin_fma(p, g, dk(1.0 / 3628800.0));
    p = __builtin_fma(p, g, dk(1.0 / 362880.0));
    p = __builtin_fma(p, g, dk(1.0 / 40320.0));
    p = __builtin_fma(p, g, dk(1.0 / 5040.0));
    p = __builtin_fma(p, g, dk(1.0 / 720.0));
    p = __builtin_fma(p, g, dk(1.0 / 120.0));
    p = __builtin_fma(p, g, dk(1.0 / 24.0));
    p = __builtin_fma(p, g, dk(1.0 / 6.0));
    p = __builtin_fma(p, g, dk(0.5));
    p = __builtin_fma(p, g, dk(1.0));
    p = __builtin_fma(p, g, dk(1.0));
    const int ki = (int)k;
    const double scale = bitsd((uint64_t)(ki + 1023) << 52);
    return p * scale;
}

__device__ __forceinline__ float pow_p(float x, float y)
{
    const uint32_t ux = fbits(x), uy = fbits(y);
    const uint32_t axb = ux & 0x7fffffffu, ayb = uy & 0x7fffffffu;
    if (ayb == 0) return 1.0f;
    if (ux == 0x3f800000u) return 1.0f;
    if (axb > 0x7f800000u || ayb > 0x7f800000u) return x + y;
    const float ax = bitsf(axb);
    bool yint = false, yodd = false;
    if (ayb >= 0x4b800000u) { yint = true; }
    else {
        const float t = __builtin_truncf(y);
        if (t == y) { yint = true; yodd = (((long long)t) & 1) != 0; }
    }
    const bool xneg = (ux >> 31) != 0;
    if (xneg && axb != 0 && !yint) return bitsf(0x7fc00000u);
    const float sign = (xneg && yodd) ? -1.0f : 1.0f;
    if (axb == 0) return (uy >> 31) ? sign * bitsf(0x7f800000u) : sign * 0.0f;
    if (axb == 0x7f800000u) return (uy >> 31) ? sign * 0.0f : sign * bitsf(0x7f800000u);
    if (ayb == 0x7f800000u) {
        if (ax == 1.0f) return 1.0f;
        const bool big = ax > 1.0f;
        const bool ypos = (uy >> 31) == 0;
        return (big == ypos) ? bitsf(0x7f800000u) : 0.0f;
    }
    double l = log2d_p((double)ax) * (double)y;
    if (l > 200.0) l = 200.0;
    if (l < -200.0) l = -200.0;
    const double r = exp2d_p(l);
    return sign * (float)r;
}

// 1/x rounded to nearest from the hardware reciprocal (v_rcp_f32, 1 ulp) and
// one Newton step on the fma residual: 3 VALU ops instead of the 11 of the
// IEEE division sequence.  Equal to 1.f / x (IEEE) for every |x| in
// [2^-32, 2^125], shown on gfx950 by exhaustive comparison
// (vrhip_selftest_rcp, tests/test_gpu_parity.py::test_rcp_exhaustive).
__device__ __forceinline__ float rcp_rn(float x)
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
constexpr float kRcpRnHi = 0x1p125f;

// sqrt rounded to nearest for x in [2^-96, FLT_MAX]: v_sqrt_f32 and the two
// neighbour tests on the fma residual of LLVM's correctly rounded expansion,
// without its input scaling (x < 2^-96) and special-value fix-ups (0, inf,
// NaN), which are identities on that range; 9 VALU ops instead of 17.
// Exhaustive GPU check: vrhip_selftest_sqrt.
__device__ __forceinline__ float sqrt_rn(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float t = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : t;
}
constexpr float kSqrtRnLo = 0x1p-96f;

// sqrtf(x) and 1.0f / sqrtf(x), bit for bit: the short sequences when every
// active lane of the wave is in their exact range, else the IEEE expansions
__device__ __forceinline__ float sqrt_exact(float x)
{
    if (__builtin_expect(__ballot(!(x >= kSqrtRnLo && x <= 0x1.fffffep127f)) != 0ull, 0)) return __builtin_sqrtf(x);
    return sqrt_rn(x);
}
__device__ __forceinline__ float inv_sqrt_exact(float x)
{
    // x >= 2^-64: sqrt(x) >= 2^-32, inside rcp_rn's range [2^-32, 2^125]
    if (__builtin_expect(__ballot(!(x >= 0x1p-64f && x <= 0x1.fffffep127f)) != 0ull, 0))
        return 1.0f / __builtin_sqrtf(x);
    return rcp_rn(sqrt_rn(x));
}

// float -> int with CUDA cvt.rzi.s32.f32 semantics (truncate, saturate, NaN -> 0)
__device__ __forceinline__ int f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int)0x80000000u;
    return (int)f;
}
__device__ __forceinline__ int d2i(double f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0) return 2147483647;
    if (f <= -2147483648.0) return (int)0x80000000u;
    return (int)f;
}
__device__ __forceinline__ unsigned char f2u8(float f)
{
    if (f != f) return 0;
    if (f <= 0.0f) return 0;
    if (f >= 255.0f) return 255;
    return (unsigned char)(int)f;
}

} // namespace vr
