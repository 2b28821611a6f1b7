/*
 * oracle/detmath.h — TEST INFRASTRUCTURE (CPU oracle only; never linked into librmr).
 *
 * Deterministic float32 math shared *by definition* (not by code) with the HIP kernels in
 * raymarchrenderer_amd/csrc/rmr_math.h. The reference GLSL leaves sin/acos/pow/normalize precision
 * to the driver (RayMarch.glsl:43-57 rand() is a chained fract(sin(x)*43758.5453) hash, so its
 * stream is implementation-defined). rmr pins one implementation:
 *   - only IEEE-754 single ops that are correctly rounded on both x86-64 and gfx950:
 *     + - * / sqrt, fmaf, floorf, rintf, fminf, fmaxf, fabsf;
 *   - every multiply-add that is fused is written as an explicit fmaf; everything else is
 *     compiled with -ffp-contract=off on both sides;
 *   - sin/cos: 3-part Cody-Waite reduction by pi/2 + minimax polynomials on [-pi/4, pi/4];
 *   - acos: the published FreeBSD/musl acosf rational approximation;
 *   - integer pow: fixed multiplication trees.
 * With these, the oracle and the GPU path agree bit for bit (tests/test_gpu_parity.py).
 */
#ifndef RMR_ORACLE_DETMATH_H
#define RMR_ORACLE_DETMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float x, y; } o_v2;
typedef struct { float x, y, z; } o_v3;

static inline o_v2 o2(float x, float y) { o_v2 r = {x, y}; return r; }
static inline o_v3 o3(float x, float y, float z) { o_v3 r = {x, y, z}; return r; }
static inline o_v3 o3s(float s) { o_v3 r = {s, s, s}; return r; }

static inline o_v3 v_add(o_v3 a, o_v3 b) { return o3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline o_v3 v_sub(o_v3 a, o_v3 b) { return o3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline o_v3 v_mul(o_v3 a, o_v3 b) { return o3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline o_v3 v_div(o_v3 a, o_v3 b) { return o3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline o_v3 v_scale(o_v3 a, float s) { return o3(a.x * s, a.y * s, a.z * s); }
static inline o_v3 v_neg(o_v3 a) { return o3(-a.x, -a.y, -a.z); }
static inline o_v3 v_abs(o_v3 a) { return o3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline o_v3 v_max0(o_v3 a) { return o3(fmaxf(a.x, 0.0f), fmaxf(a.y, 0.0f), fmaxf(a.z, 0.0f)); }
static inline o_v3 v_min(o_v3 a, o_v3 b) { return o3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
static inline o_v3 v_max(o_v3 a, o_v3 b) { return o3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
static inline int v_is_zero(o_v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static inline int v_eq(o_v3 a, o_v3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

/* dot(a,b) = fma(a.x,b.x, fma(a.y,b.y, a.z*b.z)) */
static inline float v_dot(o_v3 a, o_v3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
static inline float v_dot2(o_v2 a, o_v2 b) { return fmaf(a.x, b.x, a.y * b.y); }
static inline float v_length(o_v3 a) { return sqrtf(v_dot(a, a)); }
/* normalize(a) = a * (1/length(a)) */
static inline o_v3 v_normalize(o_v3 a) { float inv = 1.0f / v_length(a); return v_scale(a, inv); }
/* a*s + b, fused per component */
static inline o_v3 v_fma(o_v3 a, float s, o_v3 b) { return o3(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z)); }
static inline o_v3 v_cross(o_v3 a, o_v3 b) {
    return o3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* mix(x,y,a) = fma(a, y-x, x) */
static inline float f_mix(float x, float y, float a) { return fmaf(a, y - x, x); }
static inline o_v3 v_mix(o_v3 x, o_v3 y, float a) { return o3(f_mix(x.x, y.x, a), f_mix(x.y, y.y, a), f_mix(x.z, y.z, a)); }
/* mat3(c0,c1,c2) * v = fma(c0, v.x, fma(c1, v.y, c2*v.z)) */
static inline o_v3 m_mul(o_v3 c0, o_v3 c1, o_v3 c2, o_v3 v) {
    return o3(fmaf(c0.x, v.x, fmaf(c1.x, v.y, c2.x * v.z)),
              fmaf(c0.y, v.x, fmaf(c1.y, v.y, c2.y * v.z)),
              fmaf(c0.z, v.x, fmaf(c1.z, v.y, c2.z * v.z)));
}
static inline float f_clamp(float x, float a, float b) { return fminf(fmaxf(x, a), b); }
static inline float f_fract(float x) { return x - floorf(x); }
/* mod(x,y) = x - y*floor(x/y), fused */
static inline float f_mod(float x, float y) { return fmaf(-y, floorf(x / y), x); }
/* reflect(I,N) = I - 2 dot(N,I) N */
static inline o_v3 v_reflect(o_v3 I, o_v3 N) { float k = 2.0f * v_dot(N, I); return v_fma(N, -k, I); }
/* refract(I,N,eta) (GLSL definition), plain ops */
static inline o_v3 v_refract(o_v3 I, o_v3 N, float eta) {
    float d = v_dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return o3s(0.0f);
    float m = eta * d + sqrtf(k);
    return o3(eta * I.x - m * N.x, eta * I.y - m * N.y, eta * I.z - m * N.z);
}
static inline float f_pow2(float x) { return x * x; }
static inline float f_pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

/* ---- sin / cos ------------------------------------------------------------------------- */
#define DM_TWO_OVER_PI 0.636619772367581343f
#define DM_PIO2_1 1.57079637050628662109375f
#define DM_PIO2_2 (-4.37113882867379e-08f)
#define DM_PIO2_3 (-1.71512451e-15f)

static inline float dm_sin_poly(float r, float s) {
    float p = fmaf(s, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(s, p, -1.6666654611e-1f);
    return fmaf(r * s, p, r);
}
static inline float dm_cos_poly(float s) {
    float p = fmaf(s, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(s, p, 4.166664568298827e-2f);
    float t = fmaf(s, -0.5f, 1.0f);
    return fmaf(s * s, p, t);
}
/* k = rint(x*2/pi) clamped to +-2^23 (keeps the quadrant defined for NaN/inf), r = x - k*pi/2 */
static inline float dm_reduce(float x, int* q) {
    float k = rintf(x * DM_TWO_OVER_PI);
    k = fminf(fmaxf(k, -8388608.0f), 8388608.0f);
    float r = fmaf(-k, DM_PIO2_1, x);
    r = fmaf(-k, DM_PIO2_2, r);
    r = fmaf(-k, DM_PIO2_3, r);
    *q = ((int)k) & 3;
    return r;
}
static inline float det_sin(float x) {
    int q; float r = dm_reduce(x, &q); float s = r * r;
    float sv = dm_sin_poly(r, s), cv = dm_cos_poly(s);
    float v = (q & 1) ? cv : sv;
    return (q & 2) ? -v : v;
}
static inline float det_cos(float x) {
    int q; float r = dm_reduce(x, &q); float s = r * r;
    float sv = dm_sin_poly(r, s), cv = dm_cos_poly(s);
    float v = (q & 1) ? sv : cv;
    return ((q + 1) & 2) ? -v : v;
}

/* ---- acos (FreeBSD / musl acosf algorithm) --------------------------------------------- */
static inline uint32_t dm_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float dm_from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline float dm_acos_R(float z) {
    float p = z * (1.6666586697e-01f + z * (-4.2743422091e-02f + z * -8.6563630030e-03f));
    float q = 1.0f + z * -7.0662963390e-01f;
    return p / q;
}
static inline float det_acos(float x) {
    const float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    uint32_t hx = dm_bits(x), ix = hx & 0x7fffffffu;
    if (ix >= 0x3f800000u) {
        if (ix == 0x3f800000u) return (hx >> 31) ? 3.14159274101257324219f : 0.0f;
        return NAN;
    }
    if (ix < 0x3f000000u) {
        if (ix <= 0x32800000u) return 1.57079637050628662109375f;
        return pio2_hi - (x - (pio2_lo - x * dm_acos_R(x * x)));
    }
    if (hx >> 31) {
        float z = (1.0f + x) * 0.5f;
        float s = sqrtf(z);
        float w = dm_acos_R(z) * s - pio2_lo;
        return 2.0f * (pio2_hi - (s + w));
    }
    float z = (1.0f - x) * 0.5f;
    float s = sqrtf(z);
    float df = dm_from_bits(dm_bits(s) & 0xfffff000u);
    float c = (z - df * df) / (s + df);
    float w = dm_acos_R(z) * s + c;
    return 2.0f * (df + w);
}

/* ---- log / exp / atan2 / pow (Mandelbulb node only) ------------------------------------ */
/* log(x): x = 2^e * m, m in [sqrt(2)/2, sqrt(2)); log(m) via f = m-1, s = f/(2+f) series. */
static inline float det_log(float x) {
    if (!(x > 0.0f)) return (x == 0.0f) ? -INFINITY : NAN;
    if (x == INFINITY) return x;
    uint32_t u = dm_bits(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 16777216.0f; u = dm_bits(x); e = -24; }
    u += 0x3f800000u - 0x3f3504f3u;
    e += (int)(u >> 23) - 0x7f;
    u = (u & 0x007fffffu) + 0x3f3504f3u;
    float m = dm_from_bits(u);
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float z = s * s;
    float w = z * z;
    float t1 = w * fmaf(w, 0.24279078841f, 0.40000972152f);
    float t2 = z * fmaf(w, 0.28498786688f, 0.66666662693f);
    float R = t2 + t1;
    float hfsq = 0.5f * f * f;
    float dk = (float)e;
    return fmaf(dk, 6.9313812256e-01f, -((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f));
}
/* exp(x) = 2^k * e^r, r = x - k ln2 (Cody-Waite), degree-5 polynomial */
static inline float det_exp(float x) {
    if (x > 88.7f) return INFINITY;
    if (x < -103.0f) return 0.0f;
    if (x != x) return x;
    float k = rintf(x * 1.44269504089f);
    float r = fmaf(-k, 6.93145752e-1f, x);
    r = fmaf(-k, 1.42860677e-6f, r);
    float p = fmaf(r, 1.9875691500e-4f, 1.3981999507e-3f);
    p = fmaf(r, p, 8.3334519073e-3f);
    p = fmaf(r, p, 4.1665795894e-2f);
    p = fmaf(r, p, 1.6666665459e-1f);
    p = fmaf(r, p, 5.0000001201e-1f);
    float e = fmaf(r * r, p, r) + 1.0f;
    int ki = (int)k;
    /* scale by 2^k in two steps so that k in [-150,128] stays exact */
    int k1 = ki / 2, k2 = ki - k1;
    return (e * dm_from_bits((uint32_t)(k1 + 127) << 23)) * dm_from_bits((uint32_t)(k2 + 127) << 23);
}
static inline float det_pow(float x, float y) {
    if (y == 0.0f) return 1.0f;
    if (x == 0.0f) return 0.0f;
    return det_exp(y * det_log(x));
}
/* atan(x) on all reals: reduce to [0, 1] via 1/x, then odd minimax polynomial (|err| ~ 2 ulp) */
static inline float det_atan(float x) {
    float a = fabsf(x);
    int inv = a > 1.0f;
    float t = inv ? 1.0f / a : a;
    float s = t * t;
    float p = fmaf(s, -0.0117212f, 0.05265332f);
    p = fmaf(s, p, -0.11643287f);
    p = fmaf(s, p, 0.19354346f);
    p = fmaf(s, p, -0.33262347f);
    p = fmaf(s, p, 0.99997726f);
    float r = t * p;
    if (inv) r = 1.57079637050628662109375f - r;
    return (x < 0.0f) ? -r : r;
}
static inline float det_atan2(float y, float x) {
    if (x == 0.0f && y == 0.0f) return 0.0f;
    float r;
    if (fabsf(x) >= fabsf(y)) {
        r = det_atan(y / x);
        if (x < 0.0f) r = (y < 0.0f) ? r - 3.14159274101257324219f : r + 3.14159274101257324219f;
    } else {
        r = det_atan(x / y);
        r = ((y < 0.0f) ? -1.57079637050628662109375f : 1.57079637050628662109375f) - r;
    }
    return r;
}

#endif
