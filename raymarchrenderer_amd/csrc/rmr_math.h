// rmr_math.h — gfx950 device math for the rmr kernels.
//
// Float semantics (shared *by definition* with the CPU oracle, oracle/detmath.h; compiled with
// -ffp-contract=off so that only the fmaf calls below fuse):
//   dot(a,b) = fma(a.x,b.x, fma(a.y,b.y, a.z*b.z));  normalize(a) = a * (1/length(a));
//   mix(x,y,a) = fma(a, y-x, x);  mod(x,y) = fma(-y, floor(x/y), x);  mat3*v fused column sum;
//   sin/cos: Cody-Waite pi/2 reduction + minimax polynomials; acos: FreeBSD acosf rational form.
// sqrt and '/' are the correctly rounded IEEE operations (hipcc's default lowering), which is what
// makes a bit-exact CPU restatement possible.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#else  // hipRTC (per-scene specialisation, rmr_jit.cpp): no <stdint.h>
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::int64_t int64_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
#endif

namespace rmr {

struct V2 { float x, y; };
struct V3 { float x, y, z; };

#define RMR_D __device__ __forceinline__

RMR_D V2 v2(float x, float y) { return V2{x, y}; }
RMR_D V3 v3(float x, float y, float z) { return V3{x, y, z}; }
RMR_D V3 v3s(float s) { return V3{s, s, s}; }
RMR_D V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RMR_D V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RMR_D V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RMR_D V3 operator/(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
RMR_D V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
RMR_D V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
RMR_D V3 vabs(V3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
RMR_D V3 vmax0(V3 a) { return v3(fmaxf(a.x, 0.0f), fmaxf(a.y, 0.0f), fmaxf(a.z, 0.0f)); }
RMR_D V3 vmin(V3 a, V3 b) { return v3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
RMR_D V3 vmax(V3 a, V3 b) { return v3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
RMR_D bool is_zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
RMR_D bool veq(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
RMR_D float dot(V3 a, V3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
RMR_D float dot2(V2 a, V2 b) { return fmaf(a.x, b.x, a.y * b.y); }
// Correctly rounded sqrt, bit-identical to sqrtf() for every input: v_sqrt_f32 (<= 1 ulp) plus the
// one-ulp fixup (as hipcc's own lowering), without its denormal scaling and class check, which only
// matter for 0 < x < 2^-96 — that rare range (and x < 0) takes a divergent branch to sqrtf(); +-0, inf
// and NaN come out of the fast path unchanged. Verified exhaustively (tools/probes/sqrt_exhaustive.hip).
RMR_D float sqrt_cr(float x) {
#ifdef RMR_PLAIN_SQRT
    return sqrtf(x);
#else
    const float s0 = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s0) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s0) + 1u);
    const float rm = fmaf(-sm, s0, x), rp = fmaf(-sp, s0, x);
    float s = (rm <= 0.0f) ? sm : s0;
    s = (rp > 0.0f) ? sp : s;
    if (__builtin_expect(x < 0x1p-96f && x != 0.0f, 0)) s = sqrtf(x);  // tiny or negative (not +-0, NaN)
    return s;
#endif
}
// sqrt_cr without its tiny-input branch: equal to sqrtf() for x == +-0, x >= 2^-96, +inf and NaN
// (the caller routes 0 < x < 2^-96 and x < 0 elsewhere)
RMR_D float sqrt_cr_big(float x) {
    const float s0 = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s0) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s0) + 1u);
    const float rm = fmaf(-sm, s0, x), rp = fmaf(-sp, s0, x);
    float s = (rm <= 0.0f) ? sm : s0;
    return (rp > 0.0f) ? sp : s;
}
// Correctly rounded reciprocal and quotient without the IEEE division sequence (div_scale / fmas /
// fixup), for operands the caller keeps in range: v_rcp_f32 (<= 1 ulp) plus one Newton step gives
// RN(1/b) for |b| in [2^-125, 2^125]; Markstein's correction q' = RN(q + RN(a - b q) y) of
// q = RN(a y), y = RN(1/b), is RN(a / b) when nothing over- or underflows. Verified on the box
// (tools/probes/div_markstein.hip): every b of that range, every a of the Mandelbulb iteration's
// sqrt(a) / a^4, and 2^34 random pairs.
RMR_D float rcp_cr(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return fmaf(fmaf(-b, r, 1.0f), r, r);
}
RMR_D float div_mk(float a, float b) {
    const float y = rcp_cr(b);
    const float q = a * y;
    return fmaf(fmaf(-b, q, a), y, q);
}
// RN(1/b) for every b: rcp_cr where 2^-125 <= |b| <= 2^125 (one unsigned compare on the bits; NaN
// and inf fail it), the IEEE division only in a wave with a lane outside that range (0, denormal,
// huge, inf, NaN) — 3 VALU instead of the 10 of div_scale / fmas / fixup
#ifndef RMR_RCP_FAST
#define RMR_RCP_FAST 1
#endif
RMR_D float rcp_rn(float b) {
#if RMR_RCP_FAST
    const bool in = (__float_as_uint(b) & 0x7fffffffu) - 0x01000000u <= 0x7e000000u - 0x01000000u;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(!in) == 0, 1)) return rcp_cr(b);
    return in ? rcp_cr(b) : 1.0f / b;
#else
    return 1.0f / b;
#endif
}
RMR_D float length(V3 a) { return sqrt_cr(dot(a, a)); }
RMR_D V3 normalize(V3 a) { float inv = rcp_rn(length(a)); return a * inv; }
RMR_D V3 vfma(V3 a, float s, V3 b) { return v3(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z)); }
RMR_D V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
RMR_D float fmix(float x, float y, float a) { return fmaf(a, y - x, x); }
RMR_D V3 vmix(V3 x, V3 y, float a) { return v3(fmix(x.x, y.x, a), fmix(x.y, y.y, a), fmix(x.z, y.z, a)); }
RMR_D V3 mat_mul(V3 c0, V3 c1, V3 c2, V3 v) {
    return v3(fmaf(c0.x, v.x, fmaf(c1.x, v.y, c2.x * v.z)),
              fmaf(c0.y, v.x, fmaf(c1.y, v.y, c2.y * v.z)),
              fmaf(c0.z, v.x, fmaf(c1.z, v.y, c2.z * v.z)));
}
RMR_D float clampf(float x, float a, float b) { return fminf(fmaxf(x, a), b); }
RMR_D float fractf(float x) { return x - floorf(x); }
RMR_D float modf_glsl(float x, float y) { return fmaf(-y, floorf(x / y), x); }
// x / 3.14f (rand()'s mod(dt, 3.14), RM1:52) by two FMAs: q0 = x RN(1/3.14), one residual correction.
// Bit-identical to the IEEE quotient for every finite |x| >= 2^-100 (all 2^32 inputs checked:
// tools/probes/divconst_exhaustive.c); smaller, infinite and NaN inputs take the IEEE division.
RMR_D float div_314(float x) {
    const float y = 3.14f, rc = 0x1.461d58p-2f;
    if (__builtin_expect(!(fabsf(x) >= 0x1p-100f) || fabsf(x) == __builtin_inff(), 0)) return x / y;
    const float q0 = x * rc;
    const float r = fmaf(-q0, y, x);
    return fmaf(r, rc, q0);
}
// x / c for a literal c by the same two FMAs (RN(1/c) folded at compile time), where the caller's
// x range is checked against the IEEE quotient (tools/probes/wl_divconst_check.c; RMR_DIV_K=0: IEEE)
#ifndef RMR_DIV_K
#define RMR_DIV_K 1
#endif
RMR_D float div_k(float x, float c) {
#if RMR_DIV_K
    const float rc = 1.0f / c;
    const float q0 = x * rc;
    return fmaf(fmaf(-q0, c, x), rc, q0);
#else
    return x / c;
#endif
}
RMR_D float mod_314(float x) { return fmaf(-3.14f, floorf(div_314(x)), x); }
RMR_D V3 reflect(V3 I, V3 N) { float k = 2.0f * dot(N, I); return vfma(N, -k, I); }
RMR_D V3 refract(V3 I, V3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return v3s(0.0f);
    float m = eta * d + sqrt_cr(k);
    return v3(eta * I.x - m * N.x, eta * I.y - m * N.y, eta * I.z - m * N.z);
}
RMR_D float pow2(float x) { return x * x; }
RMR_D float pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

// ---- sin / cos -----------------------------------------------------------------------------
RMR_D float sin_poly(float r, float s) {
    float p = fmaf(s, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(s, p, -1.6666654611e-1f);
    return fmaf(r * s, p, r);
}
RMR_D float cos_poly(float s) {
    float p = fmaf(s, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(s, p, 4.166664568298827e-2f);
    float t = fmaf(s, -0.5f, 1.0f);
    return fmaf(s * s, p, t);
}
RMR_D float reduce_pio2(float x, int& q) {
    float k = rintf(x * 0.636619772367581343f);
    k = fminf(fmaxf(k, -8388608.0f), 8388608.0f);
    float r = fmaf(-k, 1.57079637050628662109375f, x);
    r = fmaf(-k, -4.37113882867379e-08f, r);
    r = fmaf(-k, -1.71512451e-15f, r);
    q = ((int)k) & 3;
    return r;
}
RMR_D float det_sin(float x) {
    int q; float r = reduce_pio2(x, q); float s = r * r;
    float v = (q & 1) ? cos_poly(s) : sin_poly(r, s);
    return (q & 2) ? -v : v;
}
RMR_D float det_cos(float x) {
    int q; float r = reduce_pio2(x, q); float s = r * r;
    float v = (q & 1) ? sin_poly(r, s) : cos_poly(s);
    return ((q + 1) & 2) ? -v : v;
}
// sin and cos of one argument (one reduction)
RMR_D void det_sincos(float x, float& sv, float& cv) {
    int q; float r = reduce_pio2(x, q); float s = r * r;
    float sp = sin_poly(r, s), cp = cos_poly(s);
    float a = (q & 1) ? cp : sp;
    float b = (q & 1) ? sp : cp;
    sv = (q & 2) ? -a : a;
    cv = ((q + 1) & 2) ? -b : b;
}

// ---- acos (FreeBSD acosf) -------------------------------------------------------------------
RMR_D float acos_R(float z) {
    float p = z * (1.6666586697e-01f + z * (-4.2743422091e-02f + z * -8.6563630030e-03f));
    float q = 1.0f + z * -7.0662963390e-01f;
    return p / q;
}
// The three argument ranges share one acos_R and one sqrt_cr on the range's own z (the same
// operations per lane as the branchy form, so the same bits; a wave with lanes in all three ranges
// runs the rational once instead of three times).
RMR_D float det_acos(float x) {
    const float pio2_hi = 1.5707962513e+00f, pio2_lo = 7.5497894159e-08f;
    uint32_t hx = __float_as_uint(x), ix = hx & 0x7fffffffu;
    if (ix >= 0x3f800000u) {
        if (ix == 0x3f800000u) return (hx >> 31) ? 3.14159274101257324219f : 0.0f;
        return __uint_as_float(0x7fc00000u);
    }
    const bool small = ix < 0x3f000000u, neg = (hx >> 31) != 0;
    if (small && ix <= 0x32800000u) return 1.57079637050628662109375f;
    const float z = small ? x * x : (neg ? (1.0f + x) * 0.5f : (1.0f - x) * 0.5f);
    const float R = acos_R(z);
    if (small) return pio2_hi - (x - (pio2_lo - x * R));
    const float s = sqrt_cr(z);
    if (neg) {
        float w = R * s - pio2_lo;
        return 2.0f * (pio2_hi - (s + w));
    }
    float df = __uint_as_float(__float_as_uint(s) & 0xfffff000u);
    float c = (z - df * df) / (s + df);
    float w = R * s + c;
    return 2.0f * (df + w);
}

// ---- log / exp / pow / atan2 (Mandelbulb) ---------------------------------------------------
#ifndef RMR_LOG_DIVMK
#define RMR_LOG_DIVMK 1   // det_log's f / (2 + f) by div_mk (tools/probes/logdiv_exhaustive.c: every input)
#endif
RMR_D float det_log(float x) {
    if (!(x > 0.0f)) return (x == 0.0f) ? -__builtin_huge_valf() : __uint_as_float(0x7fc00000u);
    if (x == __builtin_huge_valf()) return x;
    uint32_t u = __float_as_uint(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 16777216.0f; u = __float_as_uint(x); e = -24; }
    u += 0x3f800000u - 0x3f3504f3u;
    e += (int)(u >> 23) - 0x7f;
    u = (u & 0x007fffffu) + 0x3f3504f3u;
    float m = __uint_as_float(u);
    float f = m - 1.0f;
#if RMR_LOG_DIVMK
    // f = m - 1 in [-0.293, 0.415] is 0 or a multiple of 2^-24 of magnitude >= 2^-24: the quotient
    // (|s| <= 0.172) and Markstein's residual (~2^-24 |s|) stay normal, the divisor is in
    // rcp_cr's range — div_mk is the IEEE quotient here for every input
    float s = div_mk(f, 2.0f + f);
#else
    float s = f / (2.0f + f);
#endif
    float z = s * s;
    float w = z * z;
    float t1 = w * fmaf(w, 0.24279078841f, 0.40000972152f);
    float t2 = z * fmaf(w, 0.28498786688f, 0.66666662693f);
    float R = t2 + t1;
    float hfsq = 0.5f * f * f;
    float dk = (float)e;
    return fmaf(dk, 6.9313812256e-01f, -((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f));
}
RMR_D float det_exp(float x) {
    if (x > 88.7f) return __builtin_huge_valf();
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
    int k1 = ki / 2, k2 = ki - k1;
    return (e * __uint_as_float((uint32_t)(k1 + 127) << 23)) * __uint_as_float((uint32_t)(k2 + 127) << 23);
}
RMR_D float det_pow(float x, float y) {
    if (y == 0.0f) return 1.0f;
    if (x == 0.0f) return 0.0f;
    return det_exp(y * det_log(x));
}
RMR_D float det_atan(float x) {
    float a = fabsf(x);
    bool inv = a > 1.0f;
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
// (one division and one det_atan for both octant cases: the same operations per lane as
// r = |x| >= |y| ? atan(y / x) (+-pi) : +-pi/2 - atan(x / y))
// det_atan for |x| <= 1 or NaN (its a > 1 branch is never taken there: the same bits, no division)
RMR_D float det_atan_unit(float x) {
    float t = fabsf(x);
    float s = t * t;
    float p = fmaf(s, -0.0117212f, 0.05265332f);
    p = fmaf(s, p, -0.11643287f);
    p = fmaf(s, p, 0.19354346f);
    p = fmaf(s, p, -0.33262347f);
    p = fmaf(s, p, 0.99997726f);
    float r = t * p;
    return (x < 0.0f) ? -r : r;
}
RMR_D float det_atan2(float y, float x) {
    if (x == 0.0f && y == 0.0f) return 0.0f;
    const bool xa = fabsf(x) >= fabsf(y);
    // |num| <= |den|, so the rounded quotient is in [-1, 1] (or NaN for inf / inf)
    float r = det_atan_unit((xa ? y : x) / (xa ? x : y));
    if (xa) {
        if (x < 0.0f) r = (y < 0.0f) ? r - 3.14159274101257324219f : r + 3.14159274101257324219f;
    } else {
        r = ((y < 0.0f) ? -1.57079637050628662109375f : 1.57079637050628662109375f) - r;
    }
    return r;
}

}  // namespace rmr


