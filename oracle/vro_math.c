/*
 * vro_math.c -- ORACLE / TEST INFRASTRUCTURE ONLY (see vro_math.h).
 *
 * Portable single-precision transcendentals.  Algorithms:
 *   sincos : evaluated in IEEE double (Cody-Waite reduction by pi/2,
 *            Taylor polynomials) and rounded once to float.
 *   atan, atan2, acos : the fdlibm (Sun, 1993) float algorithms.
 *   pow    : evaluated in IEEE double (log2 by atanh series, exp2 by Taylor
 *            series, both Horner with fma) and rounded once to float.
 * Compile with -ffp-contract=off.  No host libm call is made here.
 */
#include "vro_math.h"
#include <stdint.h>
#include <string.h>
#include <math.h>

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* ---------------------------------------------------------------- sincos -- */
/* pi/2 as a sum of two doubles, and 2/pi */
#define VR_PIO2_D1 1.5707963267948966
#define VR_PIO2_D2 6.123233995736766e-17
#define VR_2_OVER_PI_D 0.6366197723675814

/* Evaluated in double (Cody-Waite reduction, Taylor polynomials to degree
 * 15/16 on [-pi/4, pi/4]) and rounded once: nearly always the correctly
 * rounded float.  Domain |x| <= 1e6 (the path only uses |x| <= 2*pi). */
void vro_p_sincosf(float x, float *s, float *c)
{
    if (!(fabsf(x) <= 1.0e6f)) {           /* NaN, inf, out of domain */
        *s = u2f(0x7fc00000u); *c = u2f(0x7fc00000u); return;
    }
    double xd = (double)x;
    double k = rint(xd * VR_2_OVER_PI_D);
    double r = fma(-k, VR_PIO2_D1, xd);
    r = fma(-k, VR_PIO2_D2, r);
    double z = r * r;
    double ps = -1.0 / 1307674368000.0;    /* -1/15! */
    ps = fma(ps, z, 1.0 / 6227020800.0);
    ps = fma(ps, z, -1.0 / 39916800.0);
    ps = fma(ps, z, 1.0 / 362880.0);
    ps = fma(ps, z, -1.0 / 5040.0);
    ps = fma(ps, z, 1.0 / 120.0);
    ps = fma(ps, z, -1.0 / 6.0);
    double sd = fma(r * z, ps, r);
    double pc = 1.0 / 20922789888000.0;    /* 1/16! */
    pc = fma(pc, z, -1.0 / 87178291200.0);
    pc = fma(pc, z, 1.0 / 479001600.0);
    pc = fma(pc, z, -1.0 / 3628800.0);
    pc = fma(pc, z, 1.0 / 40320.0);
    pc = fma(pc, z, -1.0 / 720.0);
    pc = fma(pc, z, 1.0 / 24.0);
    pc = fma(pc, z, -0.5);
    double cd = fma(z, pc, 1.0);
    float sp = (float)sd, cp = (float)cd;
    int q = ((int)k) & 3;
    if (q == 0)      { *s = sp;  *c = cp;  }
    else if (q == 1) { *s = cp;  *c = -sp; }
    else if (q == 2) { *s = -sp; *c = -cp; }
    else             { *s = -cp; *c = sp;  }
}

float vro_p_sinf(float x) { float s, c; vro_p_sincosf(x, &s, &c); return s; }
float vro_p_cosf(float x) { float s, c; vro_p_sincosf(x, &s, &c); return c; }

/* ------------------------------------------------------------------ atan -- */
static const float vr_atanhi[4] = {
    4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f };
static const float vr_atanlo[4] = {
    5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f };
#define VR_AT0  3.3333328366e-01f
#define VR_AT1 -1.9999158382e-01f
#define VR_AT2  1.4253635705e-01f
#define VR_AT3 -1.0648017377e-01f
#define VR_AT4  6.1687607318e-02f

float vro_p_atanf(float x)
{
    uint32_t hx = f2u(x);
    uint32_t ix = hx & 0x7fffffffu;
    int neg = (hx >> 31) != 0;
    int id;
    if (ix >= 0x4c800000u) {                 /* |x| >= 2^26 */
        if (ix > 0x7f800000u) return x + x;  /* NaN */
        return neg ? -vr_atanhi[3] - vr_atanlo[3] : vr_atanhi[3] + vr_atanlo[3];
    }
    if (ix < 0x3ee00000u) {                  /* |x| < 0.4375 */
        if (ix < 0x39800000u) return x;      /* |x| < 2^-12 */
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000u) {              /* |x| < 1.1875 */
            if (ix < 0x3f300000u) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else                  { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000u) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else                  { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (VR_AT0 + w * (VR_AT2 + w * VR_AT4));
    float s2 = w * (VR_AT1 + w * VR_AT3);
    if (id < 0) return x - x * (s1 + s2);
    z = vr_atanhi[id] - ((x * (s1 + s2) - vr_atanlo[id]) - x);
    return neg ? -z : z;
}

#define VR_PI_F   3.1415927410e+00f
#define VR_PI_LO -8.7422776573e-08f
#define VR_PIO2_F 1.5707963705e+00f
#define VR_PIO4_F 7.8539818525e-01f

float vro_p_atan2f(float y, float x)
{
    uint32_t hx = f2u(x), hy = f2u(y);
    uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;   /* NaN */
    if (hx == 0x3f800000u) return vro_p_atanf(y);              /* x == 1 */
    int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));      /* 2*sign(x)+sign(y) */
    if (iy == 0) {
        if (m == 0 || m == 1) return y;
        return (m == 2) ? VR_PI_F : -VR_PI_F;
    }
    if (ix == 0) return (hy >> 31) ? -VR_PIO2_F : VR_PIO2_F;
    if (ix == 0x7f800000u) {
        if (iy == 0x7f800000u) {
            switch (m) {
            case 0: return VR_PIO4_F;
            case 1: return -VR_PIO4_F;
            case 2: return 3.0f * VR_PIO4_F;
            default: return -3.0f * VR_PIO4_F;
            }
        } else {
            switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return VR_PI_F;
            default: return -VR_PI_F;
            }
        }
    }
    if (iy == 0x7f800000u) return (hy >> 31) ? -VR_PIO2_F : VR_PIO2_F;
    int k = ((int)iy - (int)ix) >> 23;
    float z;
    if (k > 26) { z = VR_PIO2_F + 0.5f * VR_PI_LO; m &= 1; }
    else if (k < -26 && (hx >> 31)) z = 0.0f;
    else z = vro_p_atanf(fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return VR_PI_F - (z - VR_PI_LO);
    default: return (z - VR_PI_LO) - VR_PI_F;
    }
}

/* ------------------------------------------------------------------ acos -- */
#define VR_ACOS_PI     3.1415925026e+00f   /* 0x40490fda */
#define VR_ACOS_PIO2HI 1.5707962513e+00f   /* 0x3fc90fda */
#define VR_ACOS_PIO2LO 7.5497894159e-08f   /* 0x33a22168 */
#define VR_PS0  1.6666586697e-01f
#define VR_PS1 -4.2743422091e-02f
#define VR_PS2 -8.6563630030e-03f
#define VR_QS1 -7.0662963390e-01f

float vro_p_acosf(float x)
{
    uint32_t hx = f2u(x);
    uint32_t ix = hx & 0x7fffffffu;
    float z, p, q, r, s, w;
    if (ix >= 0x3f800000u) {
        if (ix == 0x3f800000u)
            return (hx >> 31) ? VR_ACOS_PI + 2.0f * VR_ACOS_PIO2LO : 0.0f;
        return u2f(0x7fc00000u);
    }
    if (ix < 0x3f000000u) {                 /* |x| < 0.5 */
        if (ix <= 0x32800000u) return VR_ACOS_PIO2HI + VR_ACOS_PIO2LO;
        z = x * x;
        p = z * (VR_PS0 + z * (VR_PS1 + z * VR_PS2));
        q = 1.0f + z * VR_QS1;
        r = p / q;
        return VR_ACOS_PIO2HI - (x - (VR_ACOS_PIO2LO - x * r));
    } else if (hx >> 31) {                  /* x < -0.5 */
        z = (1.0f + x) * 0.5f;
        p = z * (VR_PS0 + z * (VR_PS1 + z * VR_PS2));
        q = 1.0f + z * VR_QS1;
        s = sqrtf(z);
        r = p / q;
        w = r * s - VR_ACOS_PIO2LO;
        return VR_ACOS_PI - 2.0f * (s + w);
    } else {                                /* x > 0.5 */
        z = (1.0f - x) * 0.5f;
        s = sqrtf(z);
        float df = u2f(f2u(s) & 0xfffff000u);
        float c = (z - df * df) / (s + df);
        p = z * (VR_PS0 + z * (VR_PS1 + z * VR_PS2));
        q = 1.0f + z * VR_QS1;
        r = p / q;
        w = r * s + c;
        return 2.0f * (df + w);
    }
}

/* ------------------------------------------------------------------- pow -- */
#define VR_INV_LN2 1.4426950408889634
#define VR_LN2     0.6931471805599453

/* log2 of a positive, finite double (any float converts to a normal double). */
static double vr_log2d(double x)
{
    uint64_t b = d2u(x);
    int e = (int)((b >> 52) & 0x7ffu) - 1023;
    double m = u2d((b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double t = (m - 1.0) / (m + 1.0);
    double t2 = t * t;
    double p = 1.0 / 23.0;
    p = fma(p, t2, 1.0 / 21.0);
    p = fma(p, t2, 1.0 / 19.0);
    p = fma(p, t2, 1.0 / 17.0);
    p = fma(p, t2, 1.0 / 15.0);
    p = fma(p, t2, 1.0 / 13.0);
    p = fma(p, t2, 1.0 / 11.0);
    p = fma(p, t2, 1.0 / 9.0);
    p = fma(p, t2, 1.0 / 7.0);
    p = fma(p, t2, 1.0 / 5.0);
    p = fma(p, t2, 1.0 / 3.0);
    double lnm = 2.0 * fma(t * t2, p, t);
    return fma(lnm, VR_INV_LN2, (double)e);
}

/* 2^z for |z| <= 200 */
static double vr_exp2d(double z)
{
    double k = rint(z);
    double f = z - k;                      /* exact, |f| <= 0.5 */
    double g = f * VR_LN2;
    double p = 1.0 / 6227020800.0;         /* 1/13! */
    p = fma(p, g, 1.0 / 479001600.0);
    p = fma(p, g, 1.0 / 39916800.0);
    p = fma(p, g, 1.0 / 3628800.0);
    p = fma(p, g, 1.0 / 362880.0);
    p = fma(p, g, 1.0 / 40320.0);
    p = fma(p, g, 1.0 / 5040.0);
    p = fma(p, g, 1.0 / 720.0);
    p = fma(p, g, 1.0 / 120.0);
    p = fma(p, g, 1.0 / 24.0);
    p = fma(p, g, 1.0 / 6.0);
    p = fma(p, g, 0.5);
    p = fma(p, g, 1.0);
    p = fma(p, g, 1.0);
    int ki = (int)k;
    double scale = u2d((uint64_t)(ki + 1023) << 52);
    return p * scale;
}

float vro_p_powf(float x, float y)
{
    uint32_t ux = f2u(x), uy = f2u(y);
    uint32_t ax_b = ux & 0x7fffffffu, ay_b = uy & 0x7fffffffu;
    if (ay_b == 0) return 1.0f;
    if (ux == 0x3f800000u) return 1.0f;
    if (ax_b > 0x7f800000u || ay_b > 0x7f800000u) return x + y;
    float ax = u2f(ax_b);
    int yint = 0, yodd = 0;
    if (ay_b >= 0x4b800000u) { yint = 1; }              /* |y| >= 2^24: even integer */
    else {
        float t = truncf(y);
        if (t == y) { yint = 1; yodd = (((int64_t)t) & 1) != 0; }
    }
    int xneg = (ux >> 31) != 0;
    if (xneg && ax_b != 0 && !yint) return u2f(0x7fc00000u);
    float sign = (xneg && yodd) ? -1.0f : 1.0f;
    if (ax_b == 0) return (uy >> 31) ? sign * u2f(0x7f800000u) : sign * 0.0f;
    if (ax_b == 0x7f800000u) return (uy >> 31) ? sign * 0.0f : sign * u2f(0x7f800000u);
    if (ay_b == 0x7f800000u) {
        if (ax == 1.0f) return 1.0f;
        int big = ax > 1.0f;
        int ypos = (uy >> 31) == 0;
        return (big == ypos) ? u2f(0x7f800000u) : 0.0f;
    }
    double l = vr_log2d((double)ax) * (double)y;
    if (l > 200.0) l = 200.0;
    if (l < -200.0) l = -200.0;
    double r = vr_exp2d(l);
    return sign * (float)r;
}
