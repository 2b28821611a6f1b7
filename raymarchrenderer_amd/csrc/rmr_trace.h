// rmr_trace.h — device code of the rmr SDF ray-march path tracer (gfx950). Included by the
// ahead-of-time build (rmr_kernels.hip) and, as an embedded string, by the per-scene hipRTC
// specialisation (rmr_jit.cpp), which supplies its own map() with the scene baked in.
//
// Hot path of RayMarch.glsl / RayMarch2.glsl / RayMarch3.glsl ("RM1/RM2/RM3", under
// /root/reference/RayMarch Renderer/): main -> trace -> march -> map, re-designed for CDNA4:
//
//  * k_trace<VARIANT, PERSIST>: one wave64 = 64 independent path states ("lanes"). Every loop
//    iteration evaluates the scene SDF map() ONCE for every lane that needs one — a march step
//    (RM1:233-257), a getNormal probe (RM1:259-268, its 6 map() calls become 6 iterations) or an
//    RM2 shadow-march step (RM2:481) — so the expensive, wave-uniform prim loop always runs with
//    as many lanes as possible. Lanes that reach a hit/miss park in a SHADE phase; shading (node
//    materials, RNG, bounce logic) runs for the parked lanes in batches once enough of them wait
//    (wave ballot). Finished lanes are refilled from a global atomic unit counter by ballot +
//    mbcnt prefix ranks (PERSIST), so a wave never idles on its longest path.
//  * Scene tables are read through the constant address space: the prim loop index is
//    wave-uniform, so each prim is an s_load into SGPRs (no VGPR/LDS traffic in the hot loop).
//  * A unit = (sample k, 8x8 tile, lane). Each path's radiance is written once, coalesced, to a
//    per-sample plane samp[k][tile][64]; k_fold then applies the reference's FP32 running mean
//    (RM1:600-612) in sample order, so the result equals nspp Graphics::Render calls bit for bit.
//
// Float semantics: rmr_math.h (compiled with -ffp-contract=off). All per-lane RNG call orders
// follow the GLSL exactly; the CPU oracle (oracle/rmr_oracle.c) is the bitwise checker.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include "rmr_math.h"
#include "rmr_internal.h"

namespace rmr {

typedef const __attribute__((address_space(4))) rmr_prim CPrim;
typedef const __attribute__((address_space(4))) rmr_op COp;
typedef const __attribute__((address_space(4))) float CFloat;
typedef const __attribute__((address_space(4))) rmr_material CMat;
typedef const __attribute__((address_space(4))) DPrim CDPrim;

#define PI_F 3.14159274101257324219f

enum Phase : int {
    // marching phases first and shading phases last: is_active and is_shade are one compare each
    PH_MARCH = 0,   // march() step of the primary / bounce ray
    PH_NORMAL = 1,  // getNormal() probe 0..5
    PH_SHADOW = 2,  // RM2 light-march step
    PH_IDLE = 3,
    PH_RESTART = 4, // separateChannels: next channel's trace starts at the next refill point
    PH_HIT = 5,     // march hit, normal ready: run the material
    PH_MISS = 6,    // march miss: sky
    PH_NEE = 7,     // RM2: shadow march finished
};

// Per-lane path state. Kept small on purpose (the fast kernels run 8 waves/SIMD = 64 VGPRs):
//  * the march sign (distMult, RM1:498-505) is `inside`; the march step counter and the
//    getNormal probe index share `ctr`; getNormal accumulates +probe then subtracts -probe in nrm;
//  * the primary direction is recomputed from `unit` when separateChannels restarts a trace;
//  * the sample result goes straight to the sample plane (partial channel sums included);
//  * HO kernels (hit-in-origin: RM1 without node programs, RM3) keep the hit point in `o`: the
//    ray origin is dead between a hit and the next bounce there. RM2 (shadow ray from the hit) and
//    node-program materials (ray.origin is an input of shader_mix / volumeScatter) keep `hit`.
//    In HO kernels the march does not write `o`: a finished march leaves (o, d, t), and the hit /
//    miss point fma(d, t, o) is written to `o` when the lane enters its shading batch (one fma per
//    component per shading event instead of an fma and a select per component in every map()
//    iteration); the getNormal probes add their offset `e` to the same fma(d, t, o).
struct Lane {
    uint32_t unit;
    float gxt, gyt, rc;
    V3 o, d;
    float t;
    int ctr;
    V3 hit;
    float mid;
    V3 nrm;
    V3 color;
    int chan, bounces;
    bool inside;
    float time;    // RM2 samplePDF seed
    V3 fin;        // RM2 finalColor
    uint32_t wl;   // RM3 hero wavelength
    float power;   // RM3
    int phase;
    // nearest-primitive cache (MAP::kCache, see npc_* below): leaf-order index of the last exact
    // minimiser, lower bound of every other primitive's distance minus the error terms (relative to
    // the anchor point), and the anchor's ray parameter t
    int cw, cw2;   // (cw2: the second cached primitive when RMR_NPC_K == 2, else == cw)
    float cs, cta;
    float texit;   // escape bound of the current ray (ray_exit)
    V3 e;          // HO kernels: the getNormal probe offset of probe ctr (normal_update cycles it)
};
// HO kernels: the march point is fma(d, t, o) + e, with e = (-0, -0, -0) while a ray marches (x + -0 = x
// for every x, -0 and NaN included) and the probe offset from the hit on: the first probe's
// (+h, +0, +0), set at the hit; the six-probe cycle of normal_update returns to it, and the shading
// batch resets it to -0
RMR_D void init_probe(Lane& L) { L.e = v3s(-0.0f); }
template <bool HO> RMR_D V3& hitref(Lane& L) {
    if constexpr (HO) return L.o;
    else return L.hit;
}
template <bool HO> RMR_D const V3& hitref(const Lane& L) {
    if constexpr (HO) return L.o;
    else return L.hit;
}
template <int VAR, bool PROG> constexpr bool hit_in_origin() { return VAR != RMR_VARIANT_RM2 && !PROG; }

// ------------------------------------------------------------------------------------------
// Executed-work counting (roofline, bench.py's count pass). Only kernels built with
// -DRMR_COUNT_FLOPS count (the hipRTC kernel with RMR_JIT_OPTS=-DRMR_COUNT_FLOPS, a separate code
// object): P.counters[11] += algorithmic flops of the SDF evaluations the kernel actually performed
// (SURVEY §8d prices: box 22, sphere 10, opU fold 2; Mandelbulb per call 6 + per iteration 27),
// [12] += their transcendentals (sqrt, acos, atan2, log, exp, sin, cos: 1 per sphere/box, Mandelbulb
// 1 per call + 10 per iteration), [13] += the Mandelbulb iteration flops alone. Lane-level sums, one
// atomic per wave and event, so the counting kernel is slower; it computes the same bits.
// ------------------------------------------------------------------------------------------
#ifdef RMR_COUNT_FLOPS
RMR_D void count_work(unsigned long long* cnt, uint64_t lanes, uint64_t flops_per_lane, uint64_t transc_per_lane,
                      uint64_t mb_flops_per_lane = 0) {
    const uint64_t m = __ballot(1);
    if (cnt && lanes && __lane_id() == __ffsll((unsigned long long)m) - 1) {
        atomicAdd(cnt + 11, (unsigned long long)(lanes * flops_per_lane));
        if (transc_per_lane) atomicAdd(cnt + 12, (unsigned long long)(lanes * transc_per_lane));
        if (mb_flops_per_lane) atomicAdd(cnt + 13, (unsigned long long)(lanes * mb_flops_per_lane));
    }
}
#define RMR_COUNT(cnt, lanes, f, t) count_work((cnt), (lanes), (f), (t))
// Mandelbulb iteration (|z| included): 27 flops + 10 transcendentals (trigonometric form); power 8:
// 51 flops + 2 square roots (mb_iter8_poly; divisions count as one flop), 59 + 2 (mb_iter8)
#define RMR_COUNT_MB(cnt, lanes, power)                                                            \
    ((power) == 8.0f ? (RMR_MB_POLY ? count_work((cnt), (lanes), 51, 2, 51) : count_work((cnt), (lanes), 59, 2, 59)) \
                     : count_work((cnt), (lanes), 27, 10, 27))
#else
#define RMR_COUNT(cnt, lanes, f, t) ((void)0)
#define RMR_COUNT_MB(cnt, lanes, power) ((void)0)
#endif
RMR_D uint64_t active_lanes() { return (uint64_t)__popcll(__ballot(1)); }

// ------------------------------------------------------------------------------------------
// RNG: rand(co), RM1:44-57 (chained fract(sin) hash, state randChange per invocation)
// ------------------------------------------------------------------------------------------
RMR_D float rand_step(float gxt, float gyt, float& rc, V2 co) {
    co.x = fmaf(gxt, rc, co.x);
    co.y = fmaf(gyt, rc, co.y);
    float dt = dot2(co, v2(12.9898f, 78.233f));
    float sn = mod_314(dt);   // == modf_glsl(dt, 3.14f) bit for bit
    rc = fractf(det_sin(sn) * 43758.5453f);
    return rc;
}
RMR_D float lrand(Lane& L, V2 co) { return rand_step(L.gxt, L.gyt, L.rc, co); }

// randHemisphere, RM1:270-304. RMR_HEMI_ALGEBRAIC (default; oracle/rmr_oracle.c o_hemisphere the
// same): cos(acos(u)) = u and sin(acos(u)) = sqrt(1 - u^2) >= 0 algebraically instead of det_acos and
// one det_sincos — the same direction, rounded differently (distribution and PSNR tests pin it)
#ifndef RMR_HEMI_ALGEBRAIC
#define RMR_HEMI_ALGEBRAIC 1
#endif
RMR_D V3 hemisphere(Lane& L, V2 s1, V2 s2, V3 n) {
    float theta = 6.28318548202514648438f * lrand(L, s1);
    float sp, cp, st, ct;
    if (RMR_HEMI_ALGEBRAIC) {
        const float u = 2.0f * lrand(L, s2) - 1.0f;
        cp = u;
        sp = sqrt_cr(fmaxf(fmaf(-u, u, 1.0f), 0.0f));
    } else {
        const float phi = det_acos(2.0f * lrand(L, s2) - 1.0f);
        det_sincos(phi, sp, cp);
    }
    det_sincos(theta, st, ct);
    V3 b = normalize(v3(sp * ct, cp, sp * st));
    if (!is_zero(n)) {
        if (b.z < 0.0f) b = -b;
        // one cross + normalize with the axis selected per lane (same operations as the two-sided form)
        const bool up = veq(n, v3(0.0f, 1.0f, 0.0f));
        V3 lx = normalize(cross(n, v3(0.0f, up ? 0.0f : 1.0f, up ? 1.0f : 0.0f)));
        V3 ly = normalize(cross(n, lx));
        b = mat_mul(lx, ly, n, b);
    }
    return b;
}

// ------------------------------------------------------------------------------------------
// scene SDF
// ------------------------------------------------------------------------------------------
RMR_D float sd_sphere(V3 p, V3 c, float r) { return length(p - c) - r; }            // RM1:170-174
RMR_D float sd_box(V3 p, V3 c, V3 r) {                                               // RM1:176-180
    V3 q = vabs(p - c) - r;
    return fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f) + length(vmax0(q));
}
// inlined into the scene-specialised kernels (hipRTC, rmr_jit.cpp: C3 +4%); a call in the
// table-driven general kernel (inlining it into the node interpreter measured 4% slower)
#ifndef RMR_MANDELBULB_INLINE
#define RMR_MANDELBULB_INLINE 0
#endif
#if RMR_MANDELBULB_INLINE
#define RMR_MB_ATTR __device__ __forceinline__
#else
#define RMR_MB_ATTR __device__ __noinline__
#endif
// Power 8 without transcendentals: z^8 in the same spherical form, with cos/sin of
// theta = acos(z.z / r) and of phi = atan2(z.y, z.x) taken from the components (sin theta >= 0 as
// acos's range gives; phi = 0 on the z axis, as atan2(0, 0)) and 8 theta, 8 phi by three angle
// doublings (sin 2a = 2 sin a cos a, cos 2a = cos^2 a - sin^2 a), r^8 and r^7 by products. The same
// function as the trigonometric iteration below, rounded differently (oracle/rmr_oracle.c states
// the identical operations; the llvmpipe golden of the trigonometric GLSL statement pins it by PSNR).
RMR_D void mb_iter8(V3& z, float& dr, V3 p0, float r) {
    float ct = z.z / r;
    float st = sqrt_cr(fmaxf(fmaf(-ct, ct, 1.0f), 0.0f));
    const float rho2 = fmaf(z.x, z.x, z.y * z.y);
    float cp = 1.0f, sp = 0.0f;
    if (rho2 > 0.0f) {
        const float inv = 1.0f / sqrt_cr(rho2);
        cp = z.x * inv;
        sp = z.y * inv;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float st2 = (2.0f * st) * ct, ct2 = fmaf(ct, ct, -(st * st));
        const float sp2 = (2.0f * sp) * cp, cp2 = fmaf(cp, cp, -(sp * sp));
        st = st2; ct = ct2; sp = sp2; cp = cp2;
    }
    const float r2 = r * r, r4 = r2 * r2, r8 = r4 * r4, r7 = (r4 * r2) * r;
    dr = fmaf(8.0f * r7, dr, 1.0f);
    z = vfma(v3(st * cp, sp * st, ct), r8, p0);
}
// Power 8 as complex powers (the default): with b = z.z^2, c = z.x^2, d = z.y^2, a = c + d,
// (z.z + i sqrt(a))^8 = r^8 (cos 8 theta + i sin 8 theta) and (z.x + i z.y)^8 = a^4 (cos 8 phi +
// i sin 8 phi), each by two squarings of (re, im) written in a, b (c, d): z^8 = (t Re', t Im', Re)
// with t = 8 z.z (b - a) Re4 sqrt(a) / a^4 — one correctly rounded square root and one division
// per iteration instead of two of each. The same function as mb_iter8, rounded differently; near
// the z axis (a < 2^-30, where a^4 would leave the normal range) the iteration is mb_iter8's.
// (oracle/rmr_oracle.c states the identical operations.)
#ifndef RMR_MB_POLY
#define RMR_MB_POLY 1
#endif
#ifndef RMR_MB_DIVMK
#define RMR_MB_DIVMK 1   // sqrt(a) / a^4 by div_mk (rmr_math.h) instead of the IEEE division sequence
#endif
RMR_D void mb_iter8_poly(V3& z, float& dr, V3 p0, float r) {
    const float c = z.x * z.x, d = z.y * z.y, b = z.z * z.z;
    const float a = c + d;
    if (!(a >= 0x1p-30f)) {   // (NaN too)
        mb_iter8(z, dr, p0, r);
        return;
    }
    const float bma = b - a;
    const float ab4 = (4.0f * a) * b;
    const float re4 = fmaf(bma, bma, -ab4);                         // r^4 cos 4 theta
    const float re8 = fmaf(re4, re4, -((4.0f * ab4) * (bma * bma)));  // r^8 cos 8 theta
    const float cmd = c - d;
    const float re4p = fmaf(cmd, cmd, -((4.0f * c) * d));            // a^2 cos 4 phi
    const float im4p = ((4.0f * z.x) * z.y) * cmd;                     // a^2 sin 4 phi
    const float re8p = fmaf(re4p, re4p, -(im4p * im4p));              // a^4 cos 8 phi
    const float im8p = (2.0f * re4p) * im4p;                          // a^4 sin 8 phi
    const float a2 = a * a;
#if RMR_MB_DIVMK
    // a >= 2^-30 here (and a <= bail^2); for a <= 2^31 the quotient and its residual stay normal
    // (div_mk's range): the IEEE division only in a wave with a lane beyond that (bail > 2^15.5)
    const float sa = sqrt_cr_big(a), a4 = a2 * a2;
    float w;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(a <= 0x1p31f)) == 0, 1)) w = div_mk(sa, a4);
    else w = (a <= 0x1p31f) ? div_mk(sa, a4) : sa / a4;
#else
    const float w = sqrt_cr(a) / (a2 * a2);
#endif
    const float t = (((8.0f * z.z) * bma) * re4) * w;                 // r^8 sin 8 theta / a^4
    const float r2 = r * r, r4 = r2 * r2, r7 = (r4 * r2) * r;
    dr = fmaf(8.0f * r7, dr, 1.0f);
    z = v3(t * re8p, t * im8p, re8) + p0;
}

// One iteration of the distance estimator's loop body after the bailout test (r = |z| <= bail):
// z <- z^power + p0 in spherical form, dr <- power r^(power-1) dr + 1.
RMR_D void mb_iter(V3& z, float& dr, V3 p0, float power, float r) {
    if (power == 8.0f) {
        if (RMR_MB_POLY) mb_iter8_poly(z, dr, p0, r);
        else mb_iter8(z, dr, p0, r);
        return;
    }
    float theta = det_acos(z.z / r);
    float phi = det_atan2(z.y, z.x);
    // det_pow(r, power - 1) and det_pow(r, power) with their shared det_log(r) computed once,
    // and sin/cos of one angle from one reduction (det_sincos): the same operations as the
    // separate calls, so the same bits
    const float lr = (r == 0.0f) ? 0.0f : det_log(r);
    const float pm1 = power - 1.0f;
    const float pw1 = (pm1 == 0.0f) ? 1.0f : ((r == 0.0f) ? 0.0f : det_exp(pm1 * lr));
    dr = fmaf(pw1 * power, dr, 1.0f);
    const float zr = (power == 0.0f) ? 1.0f : ((r == 0.0f) ? 0.0f : det_exp(power * lr));
    theta = theta * power;
    phi = phi * power;
    float st, ct, sph, cph;
    det_sincos(theta, st, ct);
    det_sincos(phi, sph, cph);
    z = vfma(v3(st * cph, sph * st, ct), zr, p0);
}
RMR_D float mb_de(float r, float dr) { return 0.5f * det_log(r) * r / dr; }
// cnt: the count build's counters (P.counters), nullptr where the caller has none
RMR_MB_ATTR float sd_mandelbulb(V3 p, V3 c, V3 prm, unsigned long long* cnt = nullptr) {
    V3 p0 = p - c, z = p0;
    float power = prm.x, bail = prm.z;
    int iters = (int)prm.y;
    float dr = 1.0f, r = 0.0f;
    (void)cnt;
    for (int i = 0; i < iters; i++) {
        r = length(z);
        if (r > bail) break;
        RMR_COUNT_MB(cnt, active_lanes(), power);   // one iteration of the lanes still iterating
        mb_iter(z, dr, p0, power, r);
    }
    return mb_de(r, dr);
}
// The same estimator one loop iteration at a time (the stepped map of the scene-specialised kernels,
// trace_main): a lane's map() spreads over as many wave passes as its own point needs, and the rest
// of the map() (the other primitives, the estimate, the fold, the march update) runs in batches once
// enough lanes have finished theirs, instead of every lane waiting for the wave's slowest bailout.
// Per lane the same operations as sd_mandelbulb's loop: mb_step runs loop iteration s.i; true when
// the loop is over, with s.r = the final |z|.
struct MBStep {
    V3 z, p0;
    float dr, r;
    int i;
    bool fin;   // estimator finished: waits for the next finishing batch
};
// The loop's bailout test runs at the end of each iteration (and in mb_begin for the first), not at
// the start of the next step: a lane whose point is outside the bailout radius (most march points:
// 0.92 iterations per map) is finished from mb_begin on and joins the next finishing
// batch without a pass, and a bailing lane finishes in the pass of its last iteration. The same
// operations in the same order per lane (RMR_MB_EARLY=0: the test at the start of mb_step, A/B).
#ifndef RMR_MB_EARLY
#define RMR_MB_EARLY 1
#endif
RMR_D void mb_begin(MBStep& s, V3 p0, int iters, float bail) {
    s.z = p0;
    s.p0 = p0;
    s.dr = 1.0f;
    s.r = 0.0f;   // (iters <= 0: the loop does not run, r stays 0)
    s.i = 0;
    s.fin = iters <= 0;
#if RMR_MB_EARLY
    if (!s.fin) {
        s.r = length(s.z);
        s.fin = s.r > bail;
    }
#else
    (void)bail;
#endif
}
RMR_D bool mb_step(MBStep& s, float power, int iters, float bail, unsigned long long* cnt) {
    (void)cnt;
    const V3 p0 = s.p0;
#if !RMR_MB_EARLY
    s.r = length(s.z);
    if (s.r > bail) return true;
#endif
    RMR_COUNT_MB(cnt, active_lanes(), power);
    mb_iter(s.z, s.dr, p0, power, s.r);
    s.i++;
#if RMR_MB_EARLY
    if (s.i >= iters) return true;   // r: the last |z| tested, as the loop leaves it
    s.r = length(s.z);
    return s.r > bail;
#else
    return s.i >= iters;
#endif
}
// lanes finishing their estimator accumulate until RMR_MB_FIN of them (or every running lane) have
// finished; then the rest of their map() runs once for all of them
#ifndef RMR_MB_FIN
#define RMR_MB_FIN 44
#endif
#ifndef RMR_MB_STEPPED
#define RMR_MB_STEPPED 1   // (0: the generated stepped map's kernel runs the whole map per pass, A/B)
#endif

// Register file of a generated function (vec3 vars[total_vars]); indices are wave-uniform.
struct VarFile {
    float x[RMR_MAX_VARS], y[RMR_MAX_VARS], z[RMR_MAX_VARS];
    RMR_D void clear() {
#pragma unroll
        for (int i = 0; i < RMR_MAX_VARS; i++) { x[i] = 0.0f; y[i] = 0.0f; z[i] = 0.0f; }
    }
    RMR_D V3 get(int i) const { return v3(x[i], y[i], z[i]); }
    RMR_D void set(int i, V3 v) { x[i] = v.x; y[i] = v.y; z[i] = v.z; }
};

RMR_D V3 cvec(const KParams& P, int ref) {
    CFloat* c = (CFloat*)P.consts + 3 * RMR_OPND_CONST_INDEX(ref);
    return v3(c[0], c[1], c[2]);
}

// One object node (RM1:121-215 node functions; all values vec3). Shared by the table interpreter
// below and the per-scene generated code (rmr_jit.cpp), which calls it with a literal code.
RMR_D V3 obj_node(int code, V3 a, V3 b, V3 c) {
    V3 r = v3s(0.0f);
    switch (code) {
    case RMR_OP_GET_X: r = v3s(a.x); break;
    case RMR_OP_GET_Y: r = v3s(a.y); break;
    case RMR_OP_GET_Z: r = v3s(a.z); break;
    case RMR_OP_ADD: r = a + b; break;
    case RMR_OP_SUB: r = a - b; break;
    case RMR_OP_MUL: r = a * b; break;
    case RMR_OP_DIV: r = a / b; break;
    case RMR_OP_SIN: r = v3(det_sin(a.x), det_sin(a.y), det_sin(a.z)); break;
    case RMR_OP_COS: r = v3(det_cos(a.x), det_cos(a.y), det_cos(a.z)); break;
    case RMR_OP_MAP_SPHERE: r = v3s(sd_sphere(a, b, c.x)); break;
    case RMR_OP_MAP_BOX: r = v3s(sd_box(a, b, c)); break;
    case RMR_OP_UNION: r = vmin(a, b); break;
    case RMR_OP_SUBTRACT: r = vmax(a, -b); break;
    case RMR_OP_INTERSECT: r = vmax(a, b); break;
    case RMR_OP_DOMAIN_REPEAT:
        r = a;
        if (b.x != 0.0f) r.x = modf_glsl(a.x, b.x) - b.x * 0.5f;
        if (b.y != 0.0f) r.y = modf_glsl(a.y, b.y) - b.y * 0.5f;
        if (b.z != 0.0f) r.z = modf_glsl(a.z, b.z) - b.z * 0.5f;
        break;
    case RMR_OP_MAP_MANDELBULB: r = v3s(sd_mandelbulb(a, b, c)); break;
    default: break;
    }
    return r;
}

// obj_func_j of Graphics.cpp:648-702 — a generic object node program (uniform across the wave)
__device__ __noinline__ float obj_program(const KParams& P, int begin, int end, int dist_var, V3 p) {
    VarFile vf;
    vf.clear();
    COp* ops = (COp*)P.ops;
    for (int k = begin; k < end; k++) {
        V3 a = v3s(0.0f), b = v3s(0.0f), c = v3s(0.0f);
        int i0 = ops[k].in[0], i1 = ops[k].in[1], i2 = ops[k].in[2];
        if (i0 != RMR_OPND_NONE) a = (i0 == RMR_OPND_P) ? p : (RMR_OPND_IS_CONST(i0) ? cvec(P, i0) : vf.get(i0));
        if (i1 != RMR_OPND_NONE) b = (i1 == RMR_OPND_P) ? p : (RMR_OPND_IS_CONST(i1) ? cvec(P, i1) : vf.get(i1));
        if (i2 != RMR_OPND_NONE) c = (i2 == RMR_OPND_P) ? p : (RMR_OPND_IS_CONST(i2) ? cvec(P, i2) : vf.get(i2));
        vf.set(ops[k].out[0], obj_node(ops[k].code, a, b, c));
    }
    return vf.get(dist_var).x;
}

// map(p), RM1:224-231 + the //#OBJINSERT fold (Graphics.cpp:107-112): opU keeps the later object
// on ties (RM1:219-222). The prim index is wave-uniform: every table read is a scalar load.
//
// NP > 0 : sphere/box scene padded to NP prims, loop fully unrolled -> all s_loads issue at the
//          top of map() and one wait covers them;
// NP == 0: sphere/box scene of any size, software-pipelined scalar loads (prim j+1 in flight
//          while prim j is evaluated);
// NP < 0 : general scene (node programs, Mandelbulb) through the 48-byte rmr_prim rows.
// opU(a, b) = a.x < b.x ? a : b with the reference's NaN behaviour as compiled by Mesa llvmpipe
// (per component: distance = min ignoring NaN, id = ordered select; oracle/rmr_oracle.c o_map).
// Same bits as the plain select for every non-NaN input; d.x never becomes NaN.
RMR_D void opu(V2& d, float dj, float mid) {
    const bool take_id = !(d.x < dj);
    const bool take_d = d.x >= dj;
    d.y = take_id ? mid : d.y;
    d.x = take_d ? dj : d.x;
}

// Exact culling for the per-scene specialised map() (rmr_jit.cpp). opU's result (distance, id) is
// unchanged by a primitive whose distance is strictly greater than the running minimum d.x (never
// NaN), so a wave may skip a primitive when, for every active lane, a lower bound of its distance
// exceeds d.x + |d.x| 2^-20 + 2^-100. The bounds, in float: box: max(q) (sd_box = min(max q, 0) +
// sqrt_cr(len2) >= max q up to the last ulp of the sqrt); sphere: sqrt_cr(len2) - r with len2
// compared against (d.x + r)^2 widened by the same margin. Lanes that evaluate compute exactly the
// table expressions (sd_box / sd_sphere), so the results stay bit-identical.
RMR_D float cull_threshold(float dx) { return fmaf(fabsf(dx), 0x1p-20f, dx) + 0x1p-100f; }
RMR_D void opu_box_culled(V2& d, V3 p, V3 c, V3 r, float mid) {
    const V3 q = vabs(p - c) - r;
    const float mq = fmaxf(q.x, fmaxf(q.y, q.z));
    const bool need = !(mq > cull_threshold(d.x));
    if (__ballot(need)) opu(d, fminf(mq, 0.0f) + length(vmax0(q)), mid);
}
RMR_D void opu_sphere_culled(V2& d, V3 p, V3 c, float r, float mid) {
    const V3 v = p - c;
    const float len2 = dot(v, v);
    const float t = cull_threshold(d.x + r);
    const bool far = (d.x + r < 0.0f) || (t > 0.0f && len2 > t * t * (1.0f + 0x1p-20f));
    if (__ballot(!far)) opu(d, sqrt_cr(len2) - r, mid);
}


// Approximate-then-exact map() for sphere/box scenes (bit-identical to the opU fold above).
// Every primitive's distance is first formed with the bare v_sqrt_f32 (within 1 ulp of the
// correctly rounded sqrt for x >= 2^-96 — the premise sqrt_cr's fix-up is proven on, exhaustively —
// and within 2^-47 absolutely below) instead of sqrt_cr's 10-instruction fix-up and tiny-input
// branch. The fold tracks the approximate minimum a (first index on equal values), the
// second-smallest value s2 (one v_med3), and the minimiser's (len2, k) with d = RN(sqrt(len2) + k):
// box k = min(max q, 0) (sd_box = k + length(max(q, 0))), sphere k = -r. Error of an approximate
// distance: |a_j - d_j| <= 2^-21 (|a_j| + R) + 2^-40, R = the largest |sphere radius| (a sphere's
// sqrt is d + r). If s2 - a exceeds both minimisers' bounds (am_margin, with 2x slack), every other
// primitive's exact distance is strictly above the minimiser's, so the fold's closed form
// (map_bvh) is opU((maxDist, -1), exact d_w, id_w): one sqrt_cr per map() instead of one
// per primitive. Lanes where it is not (near ties, NaN p) run the exact fold (wave-uniform branch).
struct AMin {
    float a, s2, l2, k, id;
};
RMR_D void am_take(AMin& m, float a, float l2, float k, float id) {
    m.s2 = __builtin_amdgcn_fmed3f(m.a, a, m.s2);
    const bool t = a < m.a;
    m.a = t ? a : m.a;
    m.l2 = t ? l2 : m.l2;
    m.k = t ? k : m.k;
    m.id = t ? id : m.id;
}
// the fold's first primitive initialises the state (a NaN there keeps a NaN, which am_unique rejects)
RMR_D void am_first(AMin& m, float a, float l2, float k, float id) {
    m.a = a;
    m.s2 = __builtin_inff();
    m.l2 = l2;
    m.k = k;
    m.id = id;
}
RMR_D void am_box0(AMin& m, V3 p, V3 c, V3 r, float id) {
    const V3 q = vabs(p - c) - r;
    const float k = fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f);
    const V3 o = vmax0(q);
    const float l2 = dot(o, o);
    am_first(m, k + __builtin_amdgcn_sqrtf(l2), l2, k, id);
}
RMR_D void am_sphere0(AMin& m, V3 p, V3 c, float r, float id) {
    const V3 v = p - c;
    const float l2 = dot(v, v);
    am_first(m, __builtin_amdgcn_sqrtf(l2) - r, l2, -r, id);
}
RMR_D void am_box(AMin& m, V3 p, V3 c, V3 r, float id) {
    const V3 q = vabs(p - c) - r;
    const float k = fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f);
    const V3 o = vmax0(q);
    const float l2 = dot(o, o);
    am_take(m, k + __builtin_amdgcn_sqrtf(l2), l2, k, id);
}
RMR_D void am_sphere(AMin& m, V3 p, V3 c, float r, float id) {
    const V3 v = p - c;
    const float l2 = dot(v, v);
    am_take(m, __builtin_amdgcn_sqrtf(l2) - r, l2, -r, id);
}
// Boxes fold without a sqrt each: sd_box = k + length(max(q, 0)) has k = 0 when the point is outside
// (len2 > 0) and len2 = 0 inside, so the key (len2 outside, k <= 0 inside, NaN for a NaN point)
// orders boxes as their distances do (sqrt_cr is monotonic). The two smallest keys become the
// approximate minimum and runner-up (one bare v_sqrt_f32 each), which the spheres then fold into:
// every other box's exact distance is >= the runner-up key's, so am_unique's bound is unchanged.
struct BMin {
    float k1, k2, id;
};
RMR_D float bm_key(V3 p, V3 c, V3 r) {
    const V3 q = vabs(p - c) - r;
    const float k = fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f);
    const V3 o = vmax0(q);
    const float l2 = dot(o, o);
    // one of the two is zero (outside: max q > 0, so k = 0; inside: every q <= 0, so len2 = 0; a
    // positive q whose square underflows gives 0 + 0), so l2 + k is exactly the selected key
    // (len2 outside, k inside), NaN for a NaN point; only -0 becomes +0, which orders, folds and
    // square-roots the same
    return l2 + k;
}
RMR_D void bm_box0(BMin& b, V3 p, V3 c, V3 r, float id) {
    b.k1 = bm_key(p, c, r);
    b.k2 = __builtin_inff();
    b.id = id;
}
RMR_D void bm_box(BMin& b, V3 p, V3 c, V3 r, float id) {
    const float key = bm_key(p, c, r);
    b.k2 = __builtin_amdgcn_fmed3f(b.k1, key, b.k2);
    const bool t = key < b.k1;
    b.k1 = t ? key : b.k1;
    b.id = t ? id : b.id;
}
RMR_D float bm_dist(float key) { return key > 0.0f ? __builtin_amdgcn_sqrtf(key) : key; }
RMR_D void am_boxes(AMin& m, const BMin& b) {
    const bool out = b.k1 > 0.0f;
    am_first(m, bm_dist(b.k1), out ? b.k1 : 0.0f, out ? 0.0f : b.k1, b.id);
    m.s2 = bm_dist(b.k2);
}
// true when the minimiser is certain (see above); false for near ties, NaN and infinite values, and
// for a minimiser whose len2 is in sqrt_cr's tiny range (0 < len2 < 2^-96: the exact fold handles it)
RMR_D bool am_unique(const AMin& m, float R2) {   // R2 = 2 R
    const float margin = fmaf(fabsf(m.a) + fabsf(m.s2) + R2, 0x1p-20f, 0x1p-39f);
    // len2 (never negative; a NaN one fails the gap test) is +0 or >= 2^-96: one unsigned compare,
    // and both tests without a short-circuit branch
    const bool big = (__float_as_uint(m.l2) - 1u) >= (__float_as_uint(0x1p-96f) - 1u);
    return (m.s2 - m.a > margin) & big;
}
// exact result of a unique fold: opU((maxDist, -1), d_w, id_w); d_w = sqrt_cr(len2) + k is the same
// expression as sd_box (k + length) and sd_sphere (length - r == length + (-r)). sqrt_cr_big: the
// tiny range is excluded by am_unique (those lanes take the exact fold).
RMR_D V2 am_result(const KParams& P, const AMin& m) {
    V2 d = v2(P.max_dist, -1.0f);
    opu(d, sqrt_cr_big(m.l2) + m.k, m.id);
    return d;
}

// ---- getNormal from one primitive (HO sphere/box kernels with the approximate map) ----------------
// The generated approximate map (rmr_jit.cpp) can carry each primitive's scene index j (< 256) in the
// low 8 mantissa bits of its material-id literal: ids are integer-valued floats of magnitude < 2^15,
// whose low 9 mantissa bits are zero, so the fold's selects move (id | j) and am_id_of recovers the id
// bit for bit (0 | j is a denormal pattern, & ~0xff gives +0 back; -1 keeps its bits). The minimiser's
// index w = am_w_of then names the primitive the hit is on.
RMR_D float am_pack(float id, int j) { return __int_as_float(__float_as_int(id) | j); }
RMR_D float am_id_of(float packed) { return __int_as_float(__float_as_int(packed) & ~0xff); }
RMR_D int am_w_of(float packed) { return __float_as_int(packed) & 0xff; }
RMR_D V2 am_result_packed(const KParams& P, const AMin& m) {
    V2 d = v2(P.max_dist, -1.0f);
    opu(d, sqrt_cr_big(m.l2) + m.k, am_id_of(m.id));
    return d;
}
#define NPC_PROBE_DELTA 0.0010001f
// Certificate, at a hit, that getNormal's six probes p +- h e_c (RM1:259-268) all have w as the unique
// minimiser of the opU fold, so each probe's map() is opU((maxDist, -1), F_w(probe), id_w) (the fold's
// closed form, map_bvh) and its distance is primitive w's alone. With eps the float evaluation error of
// any box/sphere distance at the probes (npc_eps, 4x slack) and delta = NPC_PROBE_DELTA >= |probe - p|,
// SDFs being 1-Lipschitz:
//   F_w(probe) <= a + err(a) + 2 eps + delta,   F_j(probe) >= s2 - err(s2) - 2 eps - delta  (j != w),
// a / s2 the approximate minimum / runner-up (am_*: |a_j - F_j| <= err(a_j) = 2^-21 (|a_j| + R) +
// 2^-40, monotonic in a_j). So s2 - a > err(a) + err(s2) + 4 eps + 2 delta suffices. At a hit the
// point is within ~0.002 of primitive w, so |p|_inf <= E + 0.003 (E = max |c|_inf + |r|_inf) and eps
// is a per-scene constant; with |a| < 0.002 the test becomes s2 (1 - 2^-20) - a > K (host, rmr_api.cpp
// cert_k: (0.002 + 2R) 2^-20 + 2^-39 + 4 eps(E + 0.005) + 2 delta, widened for this fma's rounding,
// with am_unique's doubled error terms). NaN: false. Meaningful at hits only (march_update uses it so).
RMR_D bool am_normal_cert(const KParams& P, const AMin& m) {
    return (fabsf(m.a) < 0.002f) & (fmaf(m.s2, 1.0f - 0x1p-20f, -m.a) > P.cert_k);
}

// One scalar load per prim (the 32-byte DPrim as a single s_load_dwordx8), with prim j+1's load
// in flight while prim j is evaluated (A/B: +2% over loading at use). The IEEE sqrt sequence hipcc
// is replaced by rmr::sqrt_cr (same bits, 6 fewer VALU per sqrt; rmr_math.h).
typedef int int8v __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) int8v CInt8v;

template <int NP>
RMR_D V2 map_fixed(const KParams& P, V3 p) {
    CInt8v* pr = (CInt8v*)P.dprims;
    V2 d = v2(P.max_dist, -1.0f);
    int8v cur = pr[0];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        int8v nxt;
        if (j + 1 < NP) nxt = pr[j + 1];
        const int type = cur[6];
        const V3 c = v3(__int_as_float(cur[0]), __int_as_float(cur[1]), __int_as_float(cur[2]));
        const V3 r = v3(__int_as_float(cur[3]), __int_as_float(cur[4]), __int_as_float(cur[5]));
        const float mid = __int_as_float(cur[7]);
        if (type == RMR_PRIM_BOX) opu(d, sd_box(p, c, r), mid);
        else if (type == RMR_PRIM_SPHERE) opu(d, sd_sphere(p, c, r.x), mid);
        if (j + 1 < NP) cur = nxt;
    }
    return d;
}

RMR_D V2 map_loop(const KParams& P, V3 p) {
    CDPrim* pr = (CDPrim*)P.dprims;
    V2 d = v2(P.max_dist, -1.0f);
    const int n = P.n_prims;
    int type = pr[0].type;
    V3 c = v3(pr[0].c[0], pr[0].c[1], pr[0].c[2]);
    V3 r = v3(pr[0].r[0], pr[0].r[1], pr[0].r[2]);
    float mid = pr[0].mat_id;
    for (int j = 0; j < n; ++j) {
        const int jn = (j + 1 < n) ? j + 1 : j;
        const int ntype = pr[jn].type;
        const V3 nc = v3(pr[jn].c[0], pr[jn].c[1], pr[jn].c[2]);
        const V3 nr = v3(pr[jn].r[0], pr[jn].r[1], pr[jn].r[2]);
        const float nmid = pr[jn].mat_id;
        if (type == RMR_PRIM_BOX) opu(d, sd_box(p, c, r), mid);
        else if (type == RMR_PRIM_SPHERE) opu(d, sd_sphere(p, c, r.x), mid);
        type = ntype; c = nc; r = nr; mid = nmid;
    }
    return d;
}

RMR_D V2 map_general(const KParams& P, V3 p) {
    CPrim* pr = (CPrim*)P.prims;
    V2 d = v2(P.max_dist, -1.0f);
    const int n = P.n_prims;
    for (int j = 0; j < n; ++j) {
        const int type = pr[j].type;
        const V3 c = v3(pr[j].c[0], pr[j].c[1], pr[j].c[2]);
        const V3 r = v3(pr[j].r[0], pr[j].r[1], pr[j].r[2]);
        float dj;
        if (type == RMR_PRIM_BOX) dj = sd_box(p, c, r);
        else if (type == RMR_PRIM_SPHERE) dj = sd_sphere(p, c, r.x);
        else if (type == RMR_PRIM_MANDELBULB) dj = sd_mandelbulb(p, c, r, P.counters);
        else dj = obj_program(P, pr[j].prog_begin, pr[j].prog_end, pr[j].dist_var, p);
        opu(d, dj, pr[j].mat_id);
    }
    return d;
}

// map() policies of the trace kernel: table-driven (ahead of time, NP as above) or generated per
// scene (rmr_jit.cpp: struct JitMap with the same eval signature).
// NP == -2: exact culling through a bounding-volume hierarchy (scenes of > 32 spheres/boxes).
// opU's sequential fold (RM1:219-231 with the NaN rule of opu()) has an order-free closed form:
// distance = min(maxDist, all non-NaN dj); id = the id of the highest scene index j whose dj equals
// that minimum or is NaN (-1 if none). So primitives may be visited in any order and skipped when
// they cannot attain the minimum: a node is skipped when, for every active lane, the distance from
// p to the node's box exceeds the running minimum by a margin (|d| 2^-18 + bvh_margin, the latter
// 1e-4 + 2^-16 x the scene extent — sd_box/sd_sphere are >= that Euclidean distance up to a few
// ulps of the coordinates). Traversal is wave-uniform (stackless pre-order
// with skip links), so node and primitive reads stay scalar loads.
RMR_D V2 map_bvh(const KParams& P, V3 p) {
    typedef const __attribute__((address_space(4))) BvhNode CNode;
    CNode* nodes = (CNode*)P.bvh;
    CDPrim* pr = (CDPrim*)P.dprims;
    float dbest = P.max_dist, mbest = -1.0f, mnan = -1.0f;
    int jbest = -1, jnan = -1;
    int i = 0;
    while (i < P.n_nodes) {
        const V3 lo = v3(nodes[i].lo[0], nodes[i].lo[1], nodes[i].lo[2]);
        const V3 hi = v3(nodes[i].hi[0], nodes[i].hi[1], nodes[i].hi[2]);
        const int count = nodes[i].count, skip = nodes[i].skip;
        const V3 q = vmax0(vmax(lo - p, p - hi));
        const float lb2 = dot(q, q);
        const float t = fmaxf(dbest + fmaf(fabsf(dbest), 0x1p-18f, P.bvh_margin), P.bvh_margin);
        const bool need = !(lb2 > t * t);   // NaN p: lb2 NaN -> needed
        if (!__ballot(need)) { i = skip; continue; }
        if (count == 0) { i++; continue; }
        const int first = nodes[i].first;
        for (int k = first; k < first + count; k++) {
            const int tw = pr[k].type;
            const int type = tw & 0xff, j = tw >> 8;
            const V3 c = v3(pr[k].c[0], pr[k].c[1], pr[k].c[2]);
            const V3 r = v3(pr[k].r[0], pr[k].r[1], pr[k].r[2]);
            const float mid = pr[k].mat_id;
            const float dj = (type == RMR_PRIM_BOX) ? sd_box(p, c, r) : sd_sphere(p, c, r.x);
            RMR_COUNT(P.counters, active_lanes(), (type == RMR_PRIM_BOX ? 22 : 10) + 2, 1);
            if (dj < dbest || (dj == dbest && j > jbest)) { dbest = dj; mbest = mid; jbest = j; }
            if (dj != dj && j > jnan) { jnan = j; mnan = mid; }
        }
        i = skip;
    }
    return v2(dbest, jnan > jbest ? mnan : mbest);
}

// ---- nearest-primitive cache (exact culling over time; NP == -3) --------------------------------
// A full map() at the anchor point p0 (map_bvh_npc) also returns its minimiser w (leaf-order index)
// and s2, a lower bound of every other primitive's float distance at p0 (the second-smallest
// evaluated distance, or a skipped node's box distance minus the culling margin). Box and sphere
// SDFs are 1-Lipschitz, and the float evaluation F of either differs from the exact f by at most
// eps(p) = 2^-17 (|p|_inf + E) (E = max |c|_inf + |r|_inf over the scene, 4x slack over the
// rounding analysis; it also covers the rounding of p itself), so at any later point p at distance
// <= delta from p0:  F_j(p) >= s2 - eps(p0) - delta - eps(p)  for every j != w.  When that exceeds
// F_w(p) — evaluated exactly, one primitive — w is the unique minimiser and map(p) is
// opU((maxDist, -1), F_w(p), id_w) by the fold's closed form (map_bvh): one primitive instead of a
// BVH traversal. delta: along a ray (t - t0)(1 + 2^-21) (|d| <= 1 + 2^-22 for the normalized
// directions of the HO kernels); getNormal probes h (1 + 2^-21) from the hit point; a bounce origin
// hit +- N 0.003 (0.0031). NaN points always take the full map(). The cached bound also drops
// |s2| 2^-20 for the rounding of the check's subtractions (bounded by s2, delta and eps, each
// covered by that term or eps's slack).
RMR_D float npc_eps(const KParams& P, V3 p) {
    const float ax = fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z)));
    return fmaf(ax, 0x1p-17f, P.npc_eps0);
}
#define NPC_BOUNCE_DELTA 0.0031f
// exact distance of leaf-order primitive k at p, bit-identical to sd_box / sd_sphere at points
// without NaN: a sphere is the box of half-extent 0 (|v| - 0 = |v|, max(|v|, 0) = |v|, dot(|v|,|v|) =
// dot(v,v) for non-NaN v, 0 + S = S) minus its radius; a box subtracts 0 (x - 0 = x). (At a NaN
// point fmaxf / fminf drop the NaN: a sphere then gives -r where sd_sphere gives NaN.) Per-lane
// index: vector loads.
// Where the cached primitives are read from: the leaf-ordered DPrim table itself (global, per-lane
// vector loads through the L1) or a copy of it staged in the workgroup's LDS at kernel start (scenes
// of <= RMR_NPC_LDS_MAX primitives).
// (csg256 8 spp at 6 waves / SIMD: 24.0 -> 22.2 ms with the table in LDS; at 8 waves the block's LDS
// had to stay at 20 KiB for 8 blocks per CU)
#ifndef RMR_NPC_LDS_MAX
#define RMR_NPC_LDS_MAX 256
#endif
// 1: the scene has <= RMR_NPC_LDS_MAX primitives, the table is always in LDS (the hipRTC kernels know
// it: rmr_jit.cpp); 0: always global; -1: decided per launch (the ahead-of-time kernels). A per-launch
// choice leaves a select between an LDS and a global pointer, which the compiler can only serve with
// generic flat_load instructions: on C4 that was 2e10 flat loads per frame, each counted against both
// vmcnt and lgkmcnt (profiles/r05_attr_c4.json), instead of ds_read_b128
#ifndef RMR_NPC_DP_LDS
#define RMR_NPC_DP_LDS -1
#endif
// the generator states the scene's primitive count with an LDS choice (rmr_jit.cpp): the LDS table of
// trace_main (s_dp, 2 x RMR_NPC_LDS_MAX float4) must hold every one of them
#if defined(RMR_NPC_NPRIMS) && RMR_NPC_DP_LDS == 1
static_assert(RMR_NPC_NPRIMS <= RMR_NPC_LDS_MAX, "RMR_NPC_DP_LDS=1 with more primitives than the LDS table holds");
#endif
// Layout of the table the cache kernel gathers from per lane (dtab / s_dp): entry k is two float4 (a, b).
// AoS (a at [2k], b at [2k + 1]): the global P.dprims and the ahead-of-time kernels' LDS copy. SoA for the
// hipRTC cache kernels' LDS copy (RMR_NPC_TAB_SOA, rmr_jit.cpp): a at [k], b at [k + RMR_NPC_LDS_MAX].
// A ds_read_b128 serves 16 lanes per LDS cycle from one 256-B bank row of 16 16-B slots; with 32-B
// entries every a (and every b) sits in an even (odd) slot, so 16 lanes gathering random entries
// share 8 slots, against 16 with 16-B entries (C4's profile: 1.7 bank-conflict cycles per LDS
// instruction, r05_attr_c4_ds.json)
#ifndef RMR_NPC_TAB_SOA
#define RMR_NPC_TAB_SOA 0
#endif
static_assert(!RMR_NPC_TAB_SOA || RMR_NPC_DP_LDS == 1, "the SoA table is the compile-time LDS copy");
constexpr int kTabStep = RMR_NPC_TAB_SOA ? 1 : 2;               // float4s from entry k to entry k + 1
constexpr int kTabHi = RMR_NPC_TAB_SOA ? RMR_NPC_LDS_MAX : 1;   // float4s from an entry's a to its b
RMR_D float prim_dist_at(const float4* q, V3 p, float& mid, int& j, int hi = 1) {
    const float4 a = q[0], b = q[hi];  // c.xyz r.x | r.yz type|index<<8 mat_id (hi: kTabHi for a table)
    const bool box = (__float_as_int(b.z) & 0xff) == RMR_PRIM_BOX;
    const V3 c = v3(a.x, a.y, a.z);
    const V3 h = box ? v3(a.w, b.x, b.y) : v3s(0.0f);
    const float rad = box ? 0.0f : a.w;
    mid = b.w;
    j = __float_as_int(b.z) >> 8;
    const V3 qq = vabs(p - c) - h;
    const float k0 = fminf(fmaxf(qq.x, fmaxf(qq.y, qq.z)), 0.0f);
    return (k0 + length(vmax0(qq))) - rad;
}
RMR_D float prim_dist(const KParams& P, int k, V3 p, float& mid, int& j) {
    return prim_dist_at((const float4*)(P.dprims + k), p, mid, j);
}
// The LDS copy of the table without per-lane selects (hipRTC cache kernels whose table is in LDS and
// whose material ids all carry a scene index in their low mantissa bits, am_pack; rmr_jit.cpp emits
// RMR_NPC_PACKED): a = (c.xyz, sphere ? r : 0), b = (box ? r.xyz : 0, am_pack(mat_id, j)). The same
// operations as prim_dist_at on the values it selects (a sphere is the box of half-extent 0 minus its
// radius, a box subtracts 0), so the same bits; a.xyzw of a sphere stays (c, r) for am_sphere_at.
#ifndef RMR_NPC_PACKED
#define RMR_NPC_PACKED 0
#endif
constexpr bool kNpcPacked = RMR_NPC_PACKED && RMR_NPC_DP_LDS == 1;
RMR_D void npc_pack_entry(float4& a, float4& b) {
    const int tw = __float_as_int(b.z);
    const bool box = (tw & 0xff) == RMR_PRIM_BOX;
    const float4 na = make_float4(a.x, a.y, a.z, box ? 0.0f : a.w);
    const float4 nb = make_float4(box ? a.w : 0.0f, box ? b.x : 0.0f, box ? b.y : 0.0f, am_pack(b.w, tw >> 8));
    a = na;
    b = nb;
}
RMR_D float prim_dist_packed(const float4* q, V3 p, float& mid, int& j) {
    const float4 a = q[0], b = q[kTabHi];
    mid = am_id_of(b.w);
    j = am_w_of(b.w);
    const V3 qq = vabs(p - v3(a.x, a.y, a.z)) - v3(b.x, b.y, b.z);
    const float k0 = fminf(fmaxf(qq.x, fmaxf(qq.y, qq.z)), 0.0f);
    return (k0 + length(vmax0(qq))) - a.w;
}
// prim_dist_at on the table the cache kernel reads (dtab / the LDS copy)
RMR_D float prim_dist_tab(const float4* q, V3 p, float& mid, int& j) {
    if constexpr (kNpcPacked) return prim_dist_packed(q, p, mid, j);
    else return prim_dist_at(q, p, mid, j, kTabHi);
}
// Primitives per lane in the nearest-primitive cache (1 or 2): with 2 the cache holds the two
// nearest primitives and bounds every other one (a ray passing between two neighbours keeps them).
#ifndef RMR_NPC_K
#define RMR_NPC_K 2
#endif
// map_bvh plus the cache's primitives kw, kw2 (leaf indices; kw -1: none at or below maxDist, or a
// NaN) and sb, a lower bound of every other primitive's distance: the smallest exact distance among
// the evaluated non-cached primitives, or a skipped node's box distance minus the culling margin.
// Seeded with the lane's cached primitive (leaf index ks, scene index js, exact distance ds, id ms;
// ks < 0: none): visiting it first is the fold's closed form in another order, and its exact
// distance tightens the culling bound from the first node on.
RMR_D V2 map_bvh_npc_exact(const KParams& P, V3 p, int& kw, int& kw2, float& sb, int ks, int js, float ds, float ms,
                           bool count = true) {
    (void)count;
    typedef const __attribute__((address_space(4))) BvhNode CNode;
    CNode* nodes = (CNode*)P.bvh;
    CDPrim* pr = (CDPrim*)P.dprims;
    float dbest = P.max_dist, mbest = -1.0f, mnan = -1.0f;
    int jbest = -1, jnan = -1, kbest = -1;
    // the three smallest evaluated distances (u1 <= u2 <= u3), the leaf indices of the first two,
    // and the smallest skipped-node bound
    float u1 = __builtin_inff(), u2 = __builtin_inff(), u3 = __builtin_inff(), lbs = __builtin_inff();
    int k1 = -1, k2 = -1;
    if (ks >= 0) {   // (a NaN ds is never seeded: the caller passes ks = -1)
        u1 = ds;
        k1 = ks;
        if (ds <= dbest) { dbest = ds; mbest = ms; jbest = js; kbest = ks; }
    }
    (void)kbest;
    int i = 0;
    while (i < P.n_nodes) {
        const V3 lo = v3(nodes[i].lo[0], nodes[i].lo[1], nodes[i].lo[2]);
        const V3 hi = v3(nodes[i].hi[0], nodes[i].hi[1], nodes[i].hi[2]);
        const int count = nodes[i].count, skip = nodes[i].skip;
        const V3 q = vmax0(vmax(lo - p, p - hi));
        const float lb2 = dot(q, q);
        const float t = fmaxf(dbest + fmaf(fabsf(dbest), 0x1p-18f, P.bvh_margin), P.bvh_margin);
        const bool need = !(lb2 > t * t);   // NaN p: lb2 NaN -> needed
        if (!__ballot(need)) {
            // every primitive below is >= the node box distance - bvh_margin (map_bvh's culling rule)
            lbs = fminf(lbs, fmaf(__builtin_amdgcn_sqrtf(lb2), 1.0f - 0x1p-20f, -P.bvh_margin));
            i = skip;
            continue;
        }
        if (count == 0) { i++; continue; }
        const int first = nodes[i].first;
        for (int k = first; k < first + count; k++) {
            const int tw = pr[k].type;
            const int type = tw & 0xff, j = tw >> 8;
            const V3 c = v3(pr[k].c[0], pr[k].c[1], pr[k].c[2]);
            const V3 r = v3(pr[k].r[0], pr[k].r[1], pr[k].r[2]);
            const float mid = pr[k].mat_id;
            if (k == ks) continue;   // the seed, already folded in
            const float dj = (type == RMR_PRIM_BOX) ? sd_box(p, c, r) : sd_sphere(p, c, r.x);
            if (count) RMR_COUNT(P.counters, active_lanes(), (type == RMR_PRIM_BOX ? 22 : 10) + 2, 1);
            // insert dj into (u1, u2, u3): u3' = med3(u2, dj, u3), u2' = med3(u1, dj, u2), u1' = min
            const bool lt1 = dj < u1, lt2 = dj < u2;
            u3 = __builtin_amdgcn_fmed3f(u2, dj, u3);
            u2 = __builtin_amdgcn_fmed3f(u1, dj, u2);
            k2 = lt1 ? k1 : (lt2 ? k : k2);
            k1 = lt1 ? k : k1;
            u1 = fminf(u1, dj);
            if (dj < dbest || (dj == dbest && j > jbest)) { dbest = dj; mbest = mid; jbest = j; kbest = k; }
            if (dj != dj && j > jnan) { jnan = j; mnan = mid; }
        }
        i = skip;
    }
    // the cache is the set {k1, k2} (the fold's own minimiser is one of them when the bound holds)
    // and the bound covers exactly the primitives outside it
    kw = (jnan >= 0 || jbest < 0 || k1 < 0) ? -1 : k1;
    if (RMR_NPC_K >= 2 && k2 >= 0) {
        kw2 = k2;
        sb = fminf(u3, lbs);
    } else {
        kw2 = k1;
        sb = fminf(u2, lbs);
    }
    return v2(dbest, jnan > jbest ? mnan : mbest);
}

// The same traversal on approximate distances (am_* above: bare v_sqrt_f32, |a - d| <= 2^-21 (|a| +
// R) + 2^-40), without the exact fold's minimum / tie / NaN bookkeeping, then the minimiser's exact
// distance once. Where the two smallest approximate values are separated by am_unique's margin the
// approximate minimiser is the exact fold's unique minimiser, so the result is opU((maxDist, -1),
// d_w, id_w) (closed form, as am_result) and the cache is {k1, k2} as in map_bvh_npc_exact; the
// bound sb takes the third-smallest approximate value minus twice its error bound (or a skipped
// node's bound). The culling radius is an upper bound of the exact running minimum (the approximate
// one plus twice its error bound), so no node the exact traversal needs is skipped, and a skipped
// node's primitives stay strictly above the exact minimum. Lanes without that separation (near
// ties, NaN or infinite points) run map_bvh_npc_exact: the results are the exact traversal's.
RMR_D float am_prim(int type, V3 p, V3 c, V3 r) {
    if (type == RMR_PRIM_BOX) {
        const V3 q = vabs(p - c) - r;
        const float k = fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f);
        const V3 o = vmax0(q);
        return k + __builtin_amdgcn_sqrtf(dot(o, o));
    }
    const V3 v = p - c;
    return __builtin_amdgcn_sqrtf(dot(v, v)) - r.x;
}
RMR_D V2 map_bvh_npc(const KParams& P, V3 p, int& kw, int& kw2, float& sb, int ks, int js, float ds, float ms) {
    typedef const __attribute__((address_space(4))) BvhNode CNode;
    CNode* nodes = (CNode*)P.bvh;
    CDPrim* pr = (CDPrim*)P.dprims;
    const float R2 = P.am_r2;
    // the three smallest approximate distances (u1 <= u2 <= u3), the leaf indices of the first two,
    // and the smallest skipped-node bound; the seed's distance is exact
    float u1 = __builtin_inff(), u2 = __builtin_inff(), u3 = __builtin_inff(), lbs = __builtin_inff();
    int k1 = -1, k2 = -1;
    if (ks >= 0) {
        u1 = ds;
        k1 = ks;
    }
    // culling radius^2 from the running minimum: a function of u1 alone, so it is recomputed only
    // where u1 changes (after a leaf); skipped nodes keep only their smallest lb2 (the bound below is
    // monotonic in it, so one sqrt at the end gives the same lower bound up to v_sqrt's ulp, which
    // the 1 - 2^-20 factor covers)
    auto radius2 = [&](float u) {
        const float ub = fminf(P.max_dist, u + fmaf(fabsf(u) + R2, 0x1p-20f, 0x1p-39f));   // >= the exact minimum
        const float t = fmaxf(ub + fmaf(fabsf(ub), 0x1p-18f, P.bvh_margin), P.bvh_margin);
        return t * t;
    };
    float t2 = radius2(u1), lbs2 = __builtin_inff();
    int i = 0;
#ifdef RMR_NPC_VISITS   // diagnostics: wave-level node tests / prim evaluations vs the per-lane need
    uint32_t v_tests = 0, v_prims = 0, own_int = 0, own_prims = 0;
#endif
    while (i < P.n_nodes) {
        const V3 lo = v3(nodes[i].lo[0], nodes[i].lo[1], nodes[i].lo[2]);
        const V3 hi = v3(nodes[i].hi[0], nodes[i].hi[1], nodes[i].hi[2]);
        const int count = nodes[i].count, skip = nodes[i].skip;
        const V3 q = vmax0(vmax(lo - p, p - hi));
        const float lb2 = dot(q, q);
        const bool need = !(lb2 > t2);
#ifdef RMR_NPC_VISITS
        v_tests++;
        if (need) { if (nodes[i].count == 0) own_int++; else own_prims += (uint32_t)nodes[i].count; }
        if (__ballot(need) && nodes[i].count != 0) v_prims += (uint32_t)nodes[i].count;
#endif
        if (!__ballot(need)) {
            lbs2 = fminf(lbs2, lb2);
            i = skip;
            continue;
        }
        if (count == 0) { i++; continue; }
        const int first = nodes[i].first;
        for (int k = first; k < first + count; k++) {
            const int type = pr[k].type & 0xff;
            const V3 c = v3(pr[k].c[0], pr[k].c[1], pr[k].c[2]);
            const V3 r = v3(pr[k].r[0], pr[k].r[1], pr[k].r[2]);
            if (k == ks) continue;
            const float a = am_prim(type, p, c, r);
            RMR_COUNT(P.counters, active_lanes(), (type == RMR_PRIM_BOX ? 22 : 10) + 2, 1);
            const bool lt1 = a < u1, lt2 = a < u2;
            u3 = __builtin_amdgcn_fmed3f(u2, a, u3);
            u2 = __builtin_amdgcn_fmed3f(u1, a, u2);
            k2 = lt1 ? k1 : (lt2 ? k : k2);
            k1 = lt1 ? k : k1;
            u1 = fminf(u1, a);
        }
        t2 = radius2(u1);
        i = skip;
    }
    lbs = fmaf(__builtin_amdgcn_sqrtf(lbs2), 1.0f - 0x1p-20f, -P.bvh_margin);
    #ifdef RMR_NPC_VISITS
    {
        uint32_t mt = 1u + 2u * own_int, mp = own_prims;
        for (int o = 32; o > 0; o >>= 1) {
            mt = max(mt, (uint32_t)__shfl_xor((int)mt, o));
            mp = max(mp, (uint32_t)__shfl_xor((int)mp, o));
        }
        if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) {
            atomicAdd(P.counters + 4, (unsigned long long)v_tests);
            atomicAdd(P.counters + 5, (unsigned long long)v_prims);
            atomicAdd(P.counters + 6, (unsigned long long)mt);
            atomicAdd(P.counters + 7, (unsigned long long)mp);
            atomicAdd(P.counters + 9, 1ull);
        }
    }
#endif
    const float margin = fmaf(fabsf(u1) + fabsf(u2) + R2, 0x1p-20f, 0x1p-39f);
    // no runner-up evaluated (u2 = +inf): every other primitive sits in a skipped node, strictly
    // above the exact minimum (finite u1: a finite point)
    const bool alone = (u2 == __builtin_inff()) && (u1 < __builtin_inff());
    const bool uniq = (alone || u2 - u1 > margin) && k1 >= 0;
    V2 d = v2(P.max_dist, -1.0f);
    if (uniq) {
        float mid;
        int j;
        const float dw = (k1 == ks) ? ds : prim_dist(P, k1, p, mid, j);
        if (k1 == ks) mid = ms;
        opu(d, dw, mid);
        kw = (dw > P.max_dist) ? -1 : k1;   // (the exact fold: no primitive at or below maxDist)
        // lower bound of an approximate value's exact distance (twice the error bound)
        const float v = (RMR_NPC_K >= 2 && k2 >= 0) ? u3 : u2;
        const float vlb = v - fmaf(fabsf(v) + R2, 0x1p-20f, 0x1p-39f);
        kw2 = (RMR_NPC_K >= 2 && k2 >= 0) ? k2 : k1;
        sb = fminf(vlb, lbs);
    }
    const uint64_t amb = __ballot(!uniq);
#ifdef RMR_NPC_AMBCOUNT   // diagnostics (RMR_JIT_OPTS=-DRMR_NPC_AMBCOUNT): fallback lanes [9], batches [10]
    if (amb && __lane_id() == __ffsll((unsigned long long)amb) - 1) {
        atomicAdd(P.counters + 9, (unsigned long long)__popcll(amb));
        atomicAdd(P.counters + 10, 1ull);
    }
#endif
    if (amb) {
        if (!uniq) d = map_bvh_npc_exact(P, p, kw, kw2, sb, ks, js, ds, ms, false);   // (re-evaluation: not counted)
    }
    return d;
}

// map_bvh_npc through the candidate grid (P.grid, built on the host: rmr_api.cpp build_grid). A cell
// C lists every small primitive whose distance lower bound over C is <= U(C) + margin, U(C) = the
// smallest distance upper bound over C of any primitive (large ones included), margin >= twice the
// float evaluation error; so at any point of C every unlisted primitive's float distance is strictly
// above the exact fold's minimum, and the fold's closed form over (large primitives, listed ones,
// the seed) is the full fold's (map_bvh). Cells are inflated past the rounding of the cell index.
// Each lane evaluates its own cell's list (per-lane loads, as many passes as the longest list of the
// batch) instead of the wave's union of BVH nodes; the approximate fold, the uniqueness test and the
// exact fallback are map_bvh_npc's, and the cache bound also takes the cell's bound of the unlisted
// primitives. Lanes outside the grid (or in a cell without a list) take map_bvh_npc.
RMR_D void npc_insert(float a, int k, float& u1, float& u2, float& u3, int& k1, int& k2) {
    const bool lt1 = a < u1, lt2 = a < u2;
    u3 = __builtin_amdgcn_fmed3f(u2, a, u3);
    u2 = __builtin_amdgcn_fmed3f(u1, a, u2);
    k2 = lt1 ? k1 : (lt2 ? k : k2);
    k1 = lt1 ? k : k1;
    u1 = fminf(u1, a);
}
// approximate distance of leaf-order primitive k (per-lane index; am_prim's value: a sphere is the
// box of half-extent 0 minus its radius, as prim_dist_at)
RMR_D float am_prim_at(const float4* q, V3 p) {
    const float4 a = q[0], b = q[kTabHi];   // c.xyz r.x | r.yz type|index<<8 mat_id (table entry)
    const bool box = (__float_as_int(b.z) & 0xff) == RMR_PRIM_BOX;
    const V3 h = box ? v3(a.w, b.x, b.y) : v3s(0.0f);
    const V3 qq = vabs(p - v3(a.x, a.y, a.z)) - h;
    const float k0 = fminf(fmaxf(qq.x, fmaxf(qq.y, qq.z)), 0.0f);
    const V3 o = vmax0(qq);
    return (k0 + __builtin_amdgcn_sqrtf(dot(o, o))) - (box ? 0.0f : a.w);
}
// am_prim_at for a primitive known to be a sphere: one float4 (c.xyz, r), the sphere distance. For a
// sphere am_prim_at computes the same value: q = |p - c| (h = 0), k0 = +0, max(q, 0) = q, and
// |v_i| |v_i| = v_i v_i, so (0 + sqrt(len2)) - r = sqrt(len2) - r bit for bit.
RMR_D float am_sphere_at(const float4* q, V3 p) {
    const float4 a = q[0];
    const V3 v = p - v3(a.x, a.y, a.z);
    return __builtin_amdgcn_sqrtf(dot(v, v)) - a.w;
}
#ifndef RMR_NPC_SPHERES
#define RMR_NPC_SPHERES 0   // 1: every primitive a grid cell lists is a sphere (rmr_jit.cpp)
#endif
// am_prim_at on the packed LDS table (kNpcPacked)
RMR_D float am_prim_packed(const float4* q, V3 p) {
    const float4 a = q[0], b = q[kTabHi];
    const V3 qq = vabs(p - v3(a.x, a.y, a.z)) - v3(b.x, b.y, b.z);
    const float k0 = fminf(fmaxf(qq.x, fmaxf(qq.y, qq.z)), 0.0f);
    const V3 o = vmax0(qq);
    return (k0 + __builtin_amdgcn_sqrtf(dot(o, o))) - a.w;
}
#define RMR_AM_LISTED(q, p) (RMR_NPC_SPHERES ? am_sphere_at((q), (p)) : (kNpcPacked ? am_prim_packed((q), (p)) : am_prim_at((q), (p))))
// dtab: the leaf-ordered primitive table as float4 pairs (the LDS copy of trace_main when it has one)
RMR_D V2 map_grid_npc(const KParams& P, V3 p, int& kw, int& kw2, float& sb, int ks, int js, float ds, float ms,
                      const float4* dtab) {
    const float R2 = P.am_r2;
    const float fx = floorf((p.x - P.grid_lo[0]) * P.grid_inv);
    const float fy = floorf((p.y - P.grid_lo[1]) * P.grid_inv);
    const float fz = floorf((p.z - P.grid_lo[2]) * P.grid_inv);
    bool in = fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < P.grid_dimf[0] && fy < P.grid_dimf[1] &&
              fz < P.grid_dimf[2];   // NaN: false
    // the cell record is loaded without a branch (cell 0 for lanes outside the grid, unused) and
    // first read after the large primitives' fold below, so its latency overlaps that work
    // 32-bit index arithmetic: the host builds grids of fewer than 2^31 cells (build_grid)
    const uint32_t ci = in ? ((uint32_t)fz * (uint32_t)P.grid_dim[1] + (uint32_t)fy) * (uint32_t)P.grid_dim[0] + (uint32_t)fx
                           : 0u;
    const uint4 cell = P.grid[ci];
    // the seed and the large primitives, every lane (approximate fold, am_*)
    float u1 = __builtin_inff(), u2 = __builtin_inff(), u3 = __builtin_inff();
    int k1 = -1, k2 = -1;
    if (ks >= 0) {
        u1 = ds;
        k1 = ks;
    }
    CDPrim* pr = (CDPrim*)P.dprims;
    for (int k = 0; k < P.grid_n_large; k++) {   // wave-uniform: scalar loads
        const int type = pr[k].type & 0xff;
        const V3 c = v3(pr[k].c[0], pr[k].c[1], pr[k].c[2]);
        const V3 r = v3(pr[k].r[0], pr[k].r[1], pr[k].r[2]);
        if (k == ks) continue;
        npc_insert(am_prim(type, p, c, r), k, u1, u2, u3, k1, k2);
    }
    in = in && (cell.x >> 24) != 255u;   // (count 255: a cell without a list)
    // lower bound of every unlisted primitive's float distance: the cell's, or outside the grid the
    // distance to the small primitives' box (each small primitive lies in it; its float distance is
    // >= the Euclidean distance to its own box minus npc_eps) — there a lane whose seed / large minimum
    // is below it needs no list at all ("far": the distant ground plane, the sky)
    float bout = __uint_as_float(cell.y);
    bool use = in;
    if (!in) {
        const V3 q = vmax0(vmax(v3(P.grid_sbox[0], P.grid_sbox[1], P.grid_sbox[2]) - p,
                                p - v3(P.grid_sbox[3], P.grid_sbox[4], P.grid_sbox[5])));
        bout = fmaf(__builtin_amdgcn_sqrtf(dot(q, q)), 1.0f - 0x1p-20f, -npc_eps(P, p));
        const float sum = p.x + p.y + p.z;
        use = (sum == sum) && bout > u1 + fmaf(fabsf(u1) + R2, 0x1p-20f, 0x1p-39f);
    }
    V2 d = v2(P.max_dist, -1.0f);
#ifdef RMR_GRID_STATS
    {
        const uint64_t outm = __ballot(!use), farm = __ballot(use && !in);
        if (__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) {
            atomicAdd(P.counters + 9, (unsigned long long)__popcll(outm));   // lanes taking the BVH
            atomicAdd(P.counters + 10, outm ? 1ull : 0ull);                  // batches with a BVH part
            atomicAdd(P.counters + 12, (unsigned long long)__popcll(farm));  // lanes outside, no list needed
        }
    }
#endif
    if (__ballot(!use)) {
        if (!use) d = map_bvh_npc(P, p, kw, kw2, sb, ks, js, ds, ms);
    }
    if (!__ballot(use)) return d;
    bool uniq = false;
    if (use) {
        const uint32_t n = in ? cell.x >> 24 : 0u, off = cell.x & 0xffffffu;
#ifdef RMR_GRID_STATS   // diagnostics (RMR_JIT_OPTS=-DRMR_GRID_STATS, tools/grid_stats.py)
        {
            uint32_t mx = n, sm = n;
            for (int o = 32; o > 0; o >>= 1) {
                mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
                sm += (uint32_t)__shfl_xor((int)sm, o);
            }
            const uint64_t lanes = __ballot(1);
            if (__lane_id() == __ffsll((unsigned long long)lanes) - 1) {
                atomicAdd(P.counters + 4, 1ull);                                 // grid batches
                atomicAdd(P.counters + 5, (unsigned long long)mx);               // longest list per batch
                atomicAdd(P.counters + 6, (unsigned long long)sm);               // listed primitives (lanes)
                atomicAdd(P.counters + 7, (unsigned long long)__popcll(lanes));  // lanes in grid batches
            }
        }
#endif
        // the list's first four entries are inline in the cell (no dependent load), the rest in
        // the list; the same order either way
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const int k = (int)(((i < 2 ? cell.z : cell.w) >> (16 * (i & 1))) & 0xffffu);
            if (i < n && k != ks) npc_insert(RMR_AM_LISTED(dtab + kTabStep * k, p), k, u1, u2, u3, k1, k2);
        }
        for (uint32_t i = 4; i < n; i++) {
            const int k = (int)P.grid_list[off + i];
            if (k == ks) continue;
            npc_insert(RMR_AM_LISTED(dtab + kTabStep * k, p), k, u1, u2, u3, k1, k2);
        }
        RMR_COUNT(P.counters, active_lanes(), 12, 1);   // (the count build prices a listed primitive as a sphere)
        const float margin = fmaf(fabsf(u1) + fabsf(u2) + R2, 0x1p-20f, 0x1p-39f);
        const bool alone = (u2 == __builtin_inff()) && (u1 < __builtin_inff());
        uniq = (alone || u2 - u1 > margin) && k1 >= 0;
        if (uniq) {
            float mid;
            int j;
            const float dw = (k1 == ks) ? ds : prim_dist_tab(dtab + kTabStep * k1, p, mid, j);
            if (k1 == ks) mid = ms;
            opu(d, dw, mid);
            kw = (dw > P.max_dist) ? -1 : k1;
            const float v = (RMR_NPC_K >= 2 && k2 >= 0) ? u3 : u2;
            const float vlb = v - fmaf(fabsf(v) + R2, 0x1p-20f, 0x1p-39f);
            kw2 = (RMR_NPC_K >= 2 && k2 >= 0) ? k2 : k1;
            sb = fminf(vlb, bout);
        }
    }
    if (__ballot(use && !uniq)) {
        if (use && !uniq) d = map_bvh_npc_exact(P, p, kw, kw2, sb, ks, js, ds, ms, false);
    }
    return d;
}

template <int NP>
struct TableMap {
    // NP == -3: the BVH map with the nearest-primitive cache (trace_main's kCache path)
    static constexpr bool kCache = (NP == -3);
    // eval_c certifies the hit primitive's getNormal probes (am_normal_cert; generated maps only)
    static constexpr bool kCert = false;
    static RMR_D V2 eval_c(const KParams& P, V3 p, int& w, bool& cert) {
        w = 0;
        cert = false;
        return eval(P, p);
    }
    // the map counts its own executed work (BVH traversals skip primitives; see RMR_COUNT_FLOPS)
    static constexpr bool kCounts = (NP == -2 || NP == -3);
    static constexpr bool kStepped = false;
    static RMR_D V2 eval(const KParams& P, V3 p) {
        if constexpr (NP > 0) return map_fixed<NP>(P, p);
        else if constexpr (NP == 0) return map_loop(P, p);
        else if constexpr (NP == -2 || NP == -3) return map_bvh(P, p);
        else return map_general(P, p);
    }
    static RMR_D V2 full(const KParams& P, V3 p, int& kw, int& kw2, float& sb, int ks, int js, float ds, float ms,
                         const float4* dtab) {
        if (P.grid) return map_grid_npc(P, p, kw, kw2, sb, ks, js, ds, ms, dtab);
        return map_bvh_npc(P, p, kw, kw2, sb, ks, js, ds, ms);
    }
};

// ------------------------------------------------------------------------------------------
// path bookkeeping shared by the variants
// ------------------------------------------------------------------------------------------
RMR_D V3 channel_vec(int chan) {
    return chan < 0 ? v3s(1.0f) : v3(chan == 0 ? 1.0f : 0.0f, chan == 1 ? 1.0f : 0.0f, chan == 2 ? 1.0f : 0.0f);
}
// grayscale, RM1:306-309
RMR_D float gray_ch(V3 c, int chan) {
    V3 ch = channel_vec(chan);
    return (c.x + c.y + c.z) / (ch.x + ch.y + ch.z);
}

#define PH_DONE (-1)

// skyColor(dir), RM1:78-113 = RM2:84-107: constant 0.015, or with useEnvTex the equirectangular
// envTex lookup, texture2D restated as GL's bilinear filter at level 0 with CLAMP_TO_EDGE (same
// arithmetic as the oracle's sky_color; the reference driver's filter precision is its own).
RMR_D V3 sky_color(const KParams& P, V3 dir) {
    if (!P.use_env) return v3(P.sky[0], P.sky[1], P.sky[2]);
    const float PI = 3.141592653f;
    float phi = det_atan2(dir.z, dir.x);
    if (phi < 0.0f) phi += 2.0f * PI;
    const float s = phi / (2.0f * PI);
    const float t = 1.0f - (dir.y * 0.5f + 0.5f);
    const int W = P.env_w;
    // (float)W, (float)H, (float)(W - 1), (float)(H - 1) come converted from the host (kernel
    // arguments, scalar operands) instead of VALU conversions the allocator keeps live and spills
    const float fu = s * P.env_wf[0] - 0.5f, fv = t * P.env_wf[1] - 0.5f;
    const float i0f = floorf(fu), j0f = floorf(fv);
    const float a = fu - i0f, b = fv - j0f;
    const int i0 = (int)fminf(fmaxf(i0f, 0.0f), P.env_wf[2]), i1 = (int)fminf(fmaxf(i0f + 1.0f, 0.0f), P.env_wf[2]);
    const int j0 = (int)fminf(fmaxf(j0f, 0.0f), P.env_wf[3]), j1 = (int)fminf(fmaxf(j0f + 1.0f, 0.0f), P.env_wf[3]);
    const float4 t00 = P.env[(size_t)j0 * W + i0], t10 = P.env[(size_t)j0 * W + i1];
    const float4 t01 = P.env[(size_t)j1 * W + i0], t11 = P.env[(size_t)j1 * W + i1];
    const float ia = 1.0f - a, ib = 1.0f - b;
    const V3 top = v3(t00.x * ia + t10.x * a, t00.y * ia + t10.y * a, t00.z * ia + t10.z * a);
    const V3 bot = v3(t01.x * ia + t11.x * a, t01.y * ia + t11.y * a, t01.z * ia + t11.z * a);
    return v3(top.x * ib + bot.x * b, top.y * ib + bot.y * b, top.z * ib + bot.z * b);
}

// Escape bound (every kernel of a sphere/box/Mandelbulb scene, P.esc_on; RM2's shadow rays and the
// node-program-material kernels since round 3). esc_boxes are boxes whose union covers
// every primitive, each inflated by >= 0.001 + the float error of any distance at any point a march
// reaches + the rounding of the slab parameters below (host: launch setup; 0.002 + 2^-16 (|eye| +
// 2E + 3 maxDist)). ray_exit returns an upper bound of the last ray parameter at which the ray is
// inside any of them (-inf when it meets none ahead). Past it no march point can be within 0.001 of
// a primitive, so march() can only end in its miss (t = maxDist, the same state whichever step gets
// there): a march whose t passes texit ends as that miss at once. The reference marches on to
// t >= maxDist (up to maxSteps) with the same outcome; only the number of map() calls differs.
// Slab parameters use v_rcp (1 ulp): relative error < 2^-21, i.e. < 2^-21 x 3000 in space, far
// inside the inflation slack; d == +-0 gives +-inf (no constraint / never inside); 0 x inf = NaN,
// which the NaN-dropping fminf/fmaxf ignore (the ray then lies on a box face: >= the inflation
// from every primitive). A NaN origin or direction (e.g. randHemisphere about a normal of exactly
// (0,-1,0)) never escapes: the reference's map(NaN) "hits" at t = 0 (opU NaN rule).
// (oxy = o.x + o.y: primary rays pass the host's P.eye_xy, a value the kernel would otherwise keep in a
// VGPR for the whole launch)
// Slab parameters as one FMA each, B ix - o ix (o ix once per ray; RMR_ESC_FMA=0: (B - o) ix
// always, A/B). With ix = RN-ish(1/d_k) (v_rcp, <= 1 ulp) the parameter t' of a face B satisfies
// |(o + t' d)_k - B| <= 2^-22.4 |B - o_k| + 2^-24 |o_k| <= 2^-21 (|B| + |o|) whatever d_k is (t's
// error grows as 1 / |d_k|, the offset it causes along axis k shrinks as |d_k|): every point past a
// computed far face, or on a ray whose computed slab interval is empty, is outside the box shrunk
// by that much, far inside the inflation's 2^-16 (|eye| + 2E + 3 maxDist) term. The products stay
// finite: |B|, |o| < 2^60 (the host turns the bound off beyond) and |ix| <= 2^40; a wave with a lane
// whose direction has a component below ~2^-40 (its ix may be +-inf, and inf - inf a NaN on one
// side of a slab only) takes the (B - o) ix form, whose infinities carry the right signs.
#ifndef RMR_ESC_FMA
#define RMR_ESC_FMA 1
#endif
RMR_D void esc_box(float& last, float ax, float bx, float ay, float by, float az, float bz) {
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    // inside this box for t in [tn, tf] (nonempty and ahead): the ray may still hit its primitives
    if (!(tn > tf)) last = fmaxf(last, tf);
}
RMR_D float ray_exit(const KParams& P, V3 o, V3 d, float oxy) {
    const float chk = (oxy + (o.z + d.x)) + (d.y + d.z);   // NaN if any is NaN (or +-inf mix)
    if (!P.esc_on || !(chk == chk)) return __builtin_inff();
    const float ix = __builtin_amdgcn_rcpf(d.x), iy = __builtin_amdgcn_rcpf(d.y), iz = __builtin_amdgcn_rcpf(d.z);
    float last = -__builtin_inff();
    // wave-uniform box index, constant address space: scalar loads into SGPRs (a generic pointer
    // compiled to per-lane vector loads, one dependent L1 round trip per box)
#if RMR_ESC_FMA
    const float im = fmaxf(fmaxf(fabsf(ix), fabsf(iy)), fabsf(iz));
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(!(im <= 0x1p40f)) == 0, 1)) {
        const float ox = -(o.x * ix), oy = -(o.y * iy), oz = -(o.z * iz);
        for (int b = 0; b < P.n_esc; b++) {
            CFloat* B = (CFloat*)P.esc_boxes + 6 * b;
            esc_box(last, fmaf(B[0], ix, ox), fmaf(B[3], ix, ox), fmaf(B[1], iy, oy), fmaf(B[4], iy, oy),
                    fmaf(B[2], iz, oz), fmaf(B[5], iz, oz));
        }
    } else
#endif
    {
        for (int b = 0; b < P.n_esc; b++) {
            CFloat* B = (CFloat*)P.esc_boxes + 6 * b;
            esc_box(last, (B[0] - o.x) * ix, (B[3] - o.x) * ix, (B[1] - o.y) * iy, (B[4] - o.y) * iy,
                    (B[2] - o.z) * iz, (B[5] - o.z) * iz);
        }
    }
    // relative error < 2^-21: widen a positive bound
    return last > 0.0f ? fmaf(last, 1.0f + 0x1p-19f, 0x1p-60f) : last;
}
RMR_D float ray_exit(const KParams& P, V3 o, V3 d) { return ray_exit(P, o, d, o.x + o.y); }

// te_pre: the ray's escape bound when the caller has it (primary rays: computed full-width with the
// chunk's rays, chunk_ray; RM2's shadow rays: with the light-side bound); NaN = compute it here
#ifndef RMR_SHADOW_LIGHT_BOUND
#define RMR_SHADOW_LIGHT_BOUND 1   // (0: shadow rays with the escape bound alone, A/B)
#endif
template <bool HO>
RMR_D void start_march_te(const KParams& P, Lane& L, int phase_on_run, float texit) {
    L.t = 0.0f;
    L.ctr = 0;
    L.texit = texit;
    if (P.max_steps > 0 && !(L.texit < 0.0f)) {
        L.phase = phase_on_run;
    } else if (phase_on_run == PH_SHADOW) {  // march() falls out of its loop: miss
        L.t = P.max_dist;
        L.phase = PH_NEE;
    } else {
        L.t = P.max_dist;
        L.mid = -1.0f;
        if constexpr (!HO) hitref<HO>(L) = vfma(L.d, L.t, L.o);   // (HO: written at the shading batch)
        L.phase = PH_MISS;
    }
}
// every march from outside (primary, bounce, RM2's shadow rays) gets its escape bound; past it the
// march can only end as its miss, whose state (t = maxDist) is the same whichever step reaches it. An
// inside march (distMult = -1, RM1:498-505) does not: past its object's box the reference's next map()
// is positive, -map < 0.001, a hit — which a step longer than the distance to the surface
// (stepMultiply > 1) can reach in one step from inside
template <bool HO>
RMR_D void start_march(const KParams& P, Lane& L, int phase_on_run, float te_pre = __builtin_nanf("")) {
    const bool inside_march = L.inside && phase_on_run != PH_SHADOW;
    start_march_te<HO>(P, L, phase_on_run,
                       (te_pre == te_pre) ? te_pre : (inside_march ? __builtin_inff() : ray_exit(P, L.o, L.d)));
}

// trace() prologue: o = eye, d = dir, per-variant throughput init (RM1:485-492, RM2:422-429,
// RM3:349-355). Returns false if the trace has zero bounces (loop body never runs).
template <int VAR, bool HO>
RMR_D bool trace_prologue(const KParams& P, Lane& L, V3 dir, float te_pre = __builtin_nanf("")) {
    L.o = v3(P.eye[0], P.eye[1], P.eye[2]);
    L.d = dir;
    L.bounces = 0;
    L.inside = false;
    if (VAR == RMR_VARIANT_RM1) L.color = channel_vec(L.chan);
    if (VAR == RMR_VARIANT_RM2) { L.color = v3s(1.0f); L.fin = v3s(0.0f); }
    if (VAR == RMR_VARIANT_RM3) { L.wl = 0u; L.power = 1.0f; }
    if (L.bounces < P.max_bounces) {
        L.bounces = 1;
        // a primary ray's escape bound from the eye (o.x + o.y = the host's eye_xy, the same bits)
        start_march_te<HO>(P, L, PH_MARCH, (te_pre == te_pre) ? te_pre : ray_exit(P, L.o, dir, P.eye_xy));
        return true;
    }
    return false;
}

// unit -> (sample k, pixel); false if the pixel is outside the launch's clip rect
RMR_D bool unit_pixel(const KParams& P, uint32_t u, int& px, int& py, float& time) {
    const uint32_t per_k = (uint32_t)P.n_tiles * 64u;
    const uint32_t k = u / per_k;
    const uint32_t rem = u - k * per_k;
    const int tile = (int)(rem >> 6), lane = (int)(rem & 63u);
    const TileXY txy = P.tiles[tile];
    px = txy.x + (lane & 7);
    py = txy.y + (lane >> 3);
    time = P.nspp == 1u ? P.time1 : P.times[k];
    return !(px < P.x0 || py < P.y0 || px >= P.x1 || py >= P.y1);
}

// main(): jittered corner ray, RM1:569-584 (identical in RM2/RM3). The three rand() calls start
// the invocation's chain (randChange = 0); `rc` returns the chain state after them.
RMR_D V3 primary_dir(const KParams& P, int px, int py, float time, float& rc) {
    const float gxt = (float)px + time, gyt = (float)py + time;
    rc = 0.0f;
    const float W = P.Wf, H = P.Hf;   // (float)P.W, (float)P.H, converted on the host
    const float posx = (float)px / W, posy = (float)py / H;
    const float j1 = rand_step(gxt, gyt, rc, v2((float)px + time, (float)py + time));
    const float j2 = rand_step(gxt, gyt, rc, v2((float)px + time, (float)py + time));
    const float j3 = rand_step(gxt, gyt, rc, v2((float)py + time, (float)px + time));
    // mix(r00, r01, x) = fma(x, r01 - r00, r00) (rmr_math.h fmix): the differences r01 - r00 and
    // r11 - r10 come from the host (the same float subtraction; scalar operands here instead of
    // hoisted VGPRs the allocator spilled)
    const V3 r00 = v3(P.r00[0], P.r00[1], P.r00[2]), r10 = v3(P.r10[0], P.r10[1], P.r10[2]);
    const V3 d0 = v3(P.dr01[0], P.dr01[1], P.dr01[2]), d1 = v3(P.dr11[0], P.dr11[1], P.dr11[2]);
    const V3 top = vfma(d0, posx + j1 / W, r00);
    const V3 bot = vfma(d1, posx + j2 / W, r10);
    return normalize(vmix(top, bot, posy + j3 / H));
}

// a finished sample's plane store: write-once data the fold reads once. Nontemporal (streamed past the
// L2) where the hipRTC source asks for it (rmr_jit.cpp: RM2 +15%, C4's HBM traffic -37%; the L2 merges
// the lines' 16-B pieces better for the other classes); the fold's loads nontemporal measured neutral
// (r05_nt_planes_ab.log)
#ifndef RMR_NT_PLANES
#define RMR_NT_PLANES 0
#endif
RMR_D void store_sample(float4* p, float4 v) {
#if RMR_NT_PLANES
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (f4v*)p);
#else
    *p = v;
#endif
}

// End of trace(): store the channel result into the sample plane. Returns true when the sample
// is complete; otherwise (separateChannels, RM1:586-598) the lane is parked in PH_RESTART and the
// next channel's trace starts where new units start (one inlined copy of the ray setup).
template <int VAR, bool HO>
RMR_D bool finish_trace(const KParams& P, Lane& L) {
    {
        V3 res;
        if (VAR == RMR_VARIANT_RM1) res = L.color;
        if (VAR == RMR_VARIANT_RM2) {
            if (L.bounces != P.max_bounces) L.fin = L.fin + L.color;   // RM2:514-517
            res = L.fin;
        }
        if (VAR == RMR_VARIANT_RM3) {
            // wavelengthToColor(range) * power, RM3:447-522 / 540
            // wl is an integer: each quotient by a constant is the two-FMA form, equal to the IEEE one on
            // every numerator of its branch (tools/probes/wl_divconst_check.c)
            float wl = (float)L.wl, R, G, B, alpha;
            if (wl >= 380.0f && wl < 440.0f) { R = div_k(-1.0f * (wl - 440.0f), 60.0f); G = 0.0f; B = 1.0f; }
            else if (wl >= 440.0f && wl < 490.0f) { R = 0.0f; G = div_k(wl - 440.0f, 50.0f); B = 1.0f; }
            else if (wl >= 490.0f && wl < 510.0f) { R = 0.0f; G = 1.0f; B = div_k(-1.0f * (wl - 510.0f), 20.0f); }
            else if (wl >= 510.0f && wl < 580.0f) { R = div_k(wl - 510.0f, 70.0f); G = 1.0f; B = 0.0f; }
            else if (wl >= 580.0f && wl < 645.0f) { R = 1.0f; G = div_k(-1.0f * (wl - 645.0f), 65.0f); B = 0.0f; }
            else if (wl >= 645.0f && wl <= 780.0f) { R = 1.0f; G = 0.0f; B = 0.0f; }
            else { R = 0.0f; G = 0.0f; B = 0.0f; }
            if (wl > 780.0f || wl < 380.0f) alpha = 0.0f;
            else if (wl > 700.0f) alpha = div_k(780.0f - wl, 80.0f);
            else if (wl < 420.0f) alpha = div_k(wl - 380.0f, 40.0f);
            else alpha = 1.0f;
            const V3 c = (v3(R, G, B) * alpha) * L.power;
            store_sample(P.samp + L.unit, make_float4(c.x, c.y, c.z, 1.0f));
            return true;
        }
        if (L.chan < 0) {
#ifdef RMR_DIAG_NO_STORE   // timing experiment only (wrong planes): what the plane stores cost
            if (res.x == -1234.5f)
#endif
            store_sample(P.samp + L.unit, make_float4(res.x, res.y, res.z, 1.0f));
            return true;
        }
        // separateChannels: (r + g) + b, RM1:597; the partial sum lives in the sample plane
        V3 acc = res;
        if (L.chan != 0) {
            const float4 pv = P.samp[L.unit];
            acc = v3(pv.x, pv.y, pv.z) + res;
        }
        P.samp[L.unit] = make_float4(acc.x, acc.y, acc.z, 1.0f);
        if (L.chan == 2) return true;
        L.chan++;
        L.phase = PH_RESTART;
        return false;
    }
}

// `while (bounces < maxBounces) { bounces++; v = march(o, d, ...) ...}`: next march or trace end
template <int VAR, bool HO>
RMR_D void next_bounce(const KParams& P, Lane& L) {
    if (L.bounces < P.max_bounces) {
        // nearest-primitive cache: the new ray starts at t = 0 within NPC_BOUNCE_DELTA of the hit
        // (HO kernels: hit +- N 0.003 / 0.002); harmless where the cache is off
        L.cs -= NPC_BOUNCE_DELTA;
        L.cta = 0.0f;
        L.bounces++;
        start_march<HO>(P, L, PH_MARCH);   // march sign = inside ? -1 : 1
    } else if (finish_trace<VAR, HO>(P, L)) {
        L.phase = PH_DONE;
    }
}

// main(): jittered corner ray, RM1:569-584 (identical in RM2/RM3)
// (Re)start a trace: a fresh unit (fresh = true: pixel, seed chain, channel) or the next
// separateChannels pass of this lane's unit (same primary ray; the rand chain continues).
template <int VAR, bool HO>
RMR_D void begin_trace(const KParams& P, Lane& L, uint32_t u, bool fresh) {
    int px, py;
    float time, rc;
    const bool in_rect = unit_pixel(P, u, px, py, time);
    if (fresh && !in_rect) {
        L.phase = PH_IDLE;
        return;
    }
    const V3 dir = primary_dir(P, px, py, time, rc);
    L.cw = 0;
    L.cw2 = 0;
    L.cs = -__builtin_inff();
    if (fresh) {
        L.unit = u;
        L.time = time;
        L.gxt = (float)px + time;
        L.gyt = (float)py + time;
        L.rc = rc;
        L.chan = (VAR != RMR_VARIANT_RM3 && P.separate_channels != 0) ? 0 : -1;
    }
    for (;;) {  // a zero-bounce trace finishes at once (and may start the next channel)
        if (trace_prologue<VAR, HO>(P, L, dir)) return;
        if (finish_trace<VAR, HO>(P, L)) {
            L.phase = PH_DONE;
            return;
        }
    }
}

// Primary rays of a work chunk, computed full-width by the wave that fetches the chunk (instead of
// by the few lanes each refill starts) and kept in LDS: (dir.xyz, randChange after the 3 jitter
// rand() calls) and (gid.x + time, gid.y + time, time, escape bound of the primary ray or NaN
// outside the clip rect).
struct ChunkRay { float4 a, b; };
template <bool HO>
RMR_D ChunkRay chunk_ray(const KParams& P, uint32_t u) {
    int px, py;
    float time, rc = 0.0f;
    ChunkRay r;
    const bool in_rect = unit_pixel(P, u, px, py, time);
    V3 dir = v3s(0.0f);
    float te = __builtin_nanf("");
    if (in_rect) {
        dir = primary_dir(P, px, py, time, rc);
        te = ray_exit(P, v3(P.eye[0], P.eye[1], P.eye[2]), dir, P.eye_xy);   // never NaN
    }
    r.a = make_float4(dir.x, dir.y, dir.z, rc);
    r.b = make_float4((float)px + time, (float)py + time, time, te);
    return r;
}
// begin_trace for a fresh unit whose primary ray is in LDS
template <int VAR, bool HO>
RMR_D void begin_unit(const KParams& P, Lane& L, uint32_t u, float4 a, float4 b) {
    if (!(b.w == b.w)) {   // outside the clip rect
        L.phase = PH_IDLE;
        return;
    }
    L.cw = 0;
    L.cw2 = 0;
    L.cs = -__builtin_inff();
    L.unit = u;
    L.time = b.z;
    L.gxt = b.x;
    L.gyt = b.y;
    L.rc = a.w;
    L.chan = (VAR != RMR_VARIANT_RM3 && P.separate_channels != 0) ? 0 : -1;
    const V3 dir = v3(a.x, a.y, a.z);
    for (;;) {  // a zero-bounce trace finishes at once (and may start the next channel)
        if (trace_prologue<VAR, HO>(P, L, dir, b.w)) return;   // the escape bound from chunk_ray
        if (finish_trace<VAR, HO>(P, L)) {
            L.phase = PH_DONE;
            return;
        }
    }
}

// one map() result applied to a lane in PH_MARCH / PH_SHADOW (march(), RM1:233-257)
// distMult = inside ? -1 : 1 (RM1:498-505); m.x * -1.0f == -m.x exactly. Shadow rays use +1.
// cert / w (HO kernels whose map certifies its minimiser, MAP::kCert): a hit whose getNormal probes
// all have primitive w as their unique minimiser (am_normal_cert) skips the six probe iterations: it
// parks in PH_HIT with ctr = -1, and the shading batch evaluates the probes on w alone
// (cert_normals), the same six map() values
#ifndef RMR_CACHE_CERT
#define RMR_CACHE_CERT 1   // (0: the cache kernels probe in the march loop, A/B)
#endif
// p (cache kernels with one cached primitive): the march point, for the same certificate from the
// cache's bound — a hit whose six probes all stay within the cached primitive's validity (each probe
// would be served by the cache, F_w(probe) < cs - delta - eps) parks in PH_HIT with ctr = -1 too
template <bool HO, bool CACHE = false>
RMR_D void march_update(const KParams& P, Lane& L, V2 m, int w = 0, bool cert = false, V3 p = V3{0.0f, 0.0f, 0.0f}) {
    if constexpr (HO && !CACHE) {   // (cache kernels: A/B neutral-negative)
        // HO kernels (no shadow rays): the same state transitions as below as per-lane selects
        const float dist = L.inside ? -m.x : m.x;
        const bool hit0 = dist < 0.001f;
        const bool hit = hit0 && (L.t < P.max_dist);   // a far hit is trace()'s miss (see below)
        const bool past = L.t >= P.max_dist;
        const float tn = fmaf(dist, P.step_mult, L.t);
        const int cn = L.ctr + 1;
        const bool miss = hit0 ? !hit : (past || cn >= P.max_steps || tn > L.texit);
        const float tf = hit0 ? L.t : (miss ? P.max_dist : tn);
        const bool probe = hit && !cert;
        L.t = tf;   // (o stays the ray origin: the shading batch writes the point, init_probe)
        L.e = v3(probe ? 0.001f : L.e.x, probe ? 0.0f : L.e.y, probe ? 0.0f : L.e.z);
        L.mid = hit ? m.y : (miss ? -1.0f : L.mid);
        L.ctr = hit ? (cert ? -1 : 0) : cn;
        L.phase = hit ? (cert ? PH_HIT : PH_NORMAL) : (miss ? PH_MISS : L.phase);
        L.cw = cert ? w : L.cw;
        return;
    }
    const bool shadow = (L.phase == PH_SHADOW);
    const float dist = (L.inside && !shadow) ? -m.x : m.x;
    if (dist < 0.001f) {
        if (shadow) {          // sd = t; keep hit/mid/normal of the shaded point
            L.phase = PH_NEE;
        } else if (!(L.t < P.max_dist)) {
            // A far hit: march() returns its t as a hit even at t >= maxDist (its hit test comes
            // before the t >= maxDist test, RM1:240-251) — a step of stepMultiply > 1 can overshoot
            // into an object there — but trace() shades only `v.x < maxDist` (RM1:514, RM2:436,
            // RM3:368); otherwise its miss branch runs, with the point o + t d (RM3's rand seed)
            L.mid = -1.0f;
            if constexpr (!HO) hitref<HO>(L) = vfma(L.d, L.t, L.o);
            L.phase = PH_MISS;
        } else {
            bool c = false;
            if constexpr (CACHE) {
                L.cs -= (L.t - L.cta) * (1.0f + 0x1p-21f);   // cache now relative to the hit
                if constexpr (HO && RMR_NPC_K == 1 && RMR_CACHE_CERT) {
                    // every probe q is served by the cache when F_w(q) < cs - delta - eps(q); with
                    // F_w(q) <= F_w(p) + delta + 2 eps (1-Lipschitz, float error; F_w(p) = m.x, the
                    // cached or re-anchored minimiser's distance: cs = -inf without one) and eps the
                    // npc_eps bound over the probes' box: cs - 2 delta - 3 eps > m.x, with |cs| 2^-20 for
                    // this test's rounding (NaN / -inf: false)
                    const float ax = fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z)));
                    const float eps = fmaf(ax + 0.002f, 0x1p-17f, P.npc_eps0);
                    c = L.cs - fmaf(fabsf(L.cs), 0x1p-20f, fmaf(3.0f, eps, 2.0f * NPC_PROBE_DELTA)) > m.x;
                }
            }
            L.mid = m.y;
            if constexpr (HO) L.e = c ? L.e : v3(0.001f, 0.0f, 0.0f);   // first probe (init_probe)
            else hitref<HO>(L) = vfma(L.d, L.t, L.o);
            L.ctr = c ? -1 : 0;
            L.phase = c ? PH_HIT : PH_NORMAL;
        }
        return;
    }
    bool miss = L.t >= P.max_dist;
    if (!miss) {
        L.t = fmaf(dist, P.step_mult, L.t);
        L.ctr++;
        miss = (L.ctr >= P.max_steps);
        miss = miss || L.t > L.texit;   // escaped (ray_exit; shadow rays too)
    }
    if (miss) {
        L.t = P.max_dist;
        if (shadow) {
            L.phase = PH_NEE;
        } else {
            L.mid = -1.0f;
            if constexpr (!HO) hitref<HO>(L) = vfma(L.d, L.t, L.o);
            L.phase = PH_MISS;
        }
    }
}

// getNormal probe order: +x, -x, +y, -y, +z, -z (RM1:263-265).
// +probes add (+h, +0, +0); -probes add (-h, -0, -0): x + (-0) == x - 0 bit for bit, so this is
// exactly the oracle's p +- vec3(h,0,0) without a divergent switch (A/B: +10% vs a switch).
template <bool HO>
RMR_D V3 probe_point(const Lane& L) {
    const float h = 0.001f;
    const int ax = L.ctr >> 1;
    const bool neg = (L.ctr & 1) != 0;
    const float hs = neg ? -h : h, z0 = neg ? -0.0f : 0.0f;
    const V3 hp = hitref<HO>(L);
    return v3(hp.x + (ax == 0 ? hs : z0), hp.y + (ax == 1 ? hs : z0), hp.z + (ax == 2 ? hs : z0));
}
// The map() point of an active lane in HO kernels, without a divergent branch: fma(d, t, o) + e. A
// marching lane has e = -0 (init_probe): its march point fma(d, t, o) exactly. A probing lane has
// t = the hit's t, so fma(d, t, o) is the hit point, and e = probe_point's offset for ctr
// (normal_update): hit + e, the probe.
template <bool HO>
RMR_D V3 march_point(const Lane& L) {
    return vfma(L.d, L.t, L.o) + L.e;
}
// getNormal's differences map(p + h e_c) - map(p - h e_c) through a shift register: a + probe parks
// its value in nrm.z; a - probe forms the difference (the same one subtraction) and, for x and y,
// shifts it in (nrm.x <- nrm.y, nrm.y <- difference), for z leaves it in nrm.z. After the six probes
// nrm = (dx, dy, dz); one value per lane changes per probe instead of a per-axis select of all three.
RMR_D void normal_update(Lane& L, float m) {
    const bool plus = (L.ctr & 1) == 0;
    const bool last = L.ctr == 5;
    const float dv = L.nrm.z - m;
    const bool shift = !plus && !last;
    L.nrm.x = shift ? L.nrm.y : L.nrm.x;
    L.nrm.y = shift ? dv : L.nrm.y;
    L.nrm.z = plus ? m : (last ? dv : L.nrm.z);
    // next probe offset: after a + probe its negation (-h, -0, -0 for x), after a - probe the next
    // axis's + probe, (-e.z, -e.x, -e.y): (-h,-0,-0) -> (+0,+h,+0) -> (-0,-h,-0) -> (+0,+0,+h) ->
    // (-0,-0,-h) -> (+h,+0,+0), the first probe of the next normal. Signed zeros as probe_point's.
    L.e = plus ? -L.e : v3(-L.e.z, -L.e.x, -L.e.y);
    L.ctr++;
    if (L.ctr == 6) L.phase = PH_HIT;   // normalize() happens in the shading batch (shade())
}

// getNormal (RM1:259-268) of the hits certified by their march_update (cert, w; ctr = -1), at the
// shading batch and spread over the whole wave (ballot / prefix compaction): probe c of the certified
// lane of rank r (among the certified lanes, mbcnt) is evaluation g = 6 r + c, run by lane g mod 64 in
// pass g / 64, so a batch of n certified hits costs ceil(6 n / 64) evaluations per lane instead of six.
// The helper lane fetches the owner's hit point and primitive with ds_bpermute (the owner's lane from
// a per-wave LDS table of ranks), evaluates the probe hp + e_c (normal_update's offsets and signed
// zeros) on that primitive alone — each probe's map() is opU((maxDist, -1), F_w(probe), id_w) by the
// certificate, distance F_w or maxDist beyond it; F_w by prim_dist_at, bit-identical to sd_box /
// sd_sphere at points without NaN — and each owner gathers its six values back with ds_bpermute:
// nrm = (m0 - m1, m2 - m3, m4 - m5), normalised in shade() as every normal.
// Runs with every lane of the wave active (bpermute reads the owners' registers).
RMR_D void cert_normals(const KParams& P, Lane& L, bool mine, uint64_t cm, int* tab, const float4* dtab) {
    const int lane = (int)__lane_id();
    const int n = __popcll(cm);
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
    if (mine) tab[rank] = lane;
    __builtin_amdgcn_wave_barrier();
    const V3 hp = vfma(L.d, L.t, L.o);   // the hit point (HO: written at the shading batch, same bits)
    const int total = 6 * n;
    float v[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int g0 = 0; g0 < total; g0 += 64) {   // wave-uniform
        const int g = g0 + lane;
        const bool act = g < total;
        const int r = act ? g / 6 : 0;
        const int c = g - 6 * r;
        const int own = tab[r];
        const float hx = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * own, __float_as_int(hp.x)));
        const float hy = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * own, __float_as_int(hp.y)));
        const float hz = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * own, __float_as_int(hp.z)));
        const int w = __builtin_amdgcn_ds_bpermute(4 * own, L.cw);
        // e_c: (+h,+0,+0) (-h,-0,-0) (+0,+h,+0) (-0,-h,-0) (+0,+0,+h) (-0,-0,-h)
        const float sg = (c & 1) ? -1.0f : 1.0f;
        const int ax = c >> 1;
        const V3 e = v3(sg * (ax == 0 ? 0.001f : 0.0f), sg * (ax == 1 ? 0.001f : 0.0f), sg * (ax == 2 ? 0.001f : 0.0f));
        float mid;
        int j;
        const float F = prim_dist_tab(dtab + kTabStep * (act ? w : 0), v3(hx, hy, hz) + e, mid, j);
        const float val = (P.max_dist >= F) ? F : P.max_dist;   // opu(d = (maxDist, -1), F, .).x
#pragma unroll
        for (int k = 0; k < 6; k++) {   // owners collect the values of this pass
            const int gk = 6 * rank + k;
            const float got = __int_as_float(__builtin_amdgcn_ds_bpermute(4 * (gk & 63), __float_as_int(val)));
            if (mine && (gk >> 6) == (g0 >> 6)) v[k] = got;
        }
    }
    __builtin_amdgcn_wave_barrier();   // (tab is rewritten by the next batch)
    if (mine) L.nrm = v3(v[0] - v[1], v[2] - v[3], v[4] - v[5]);
}

// ------------------------------------------------------------------------------------------
// RM1 materials: mat_func_j bodies generated by Graphics.cpp:515-645 from v1 node lists
// ------------------------------------------------------------------------------------------
RMR_D V3 mat_opnd(const KParams& P, const VarFile& vf, int ref) {
    if (RMR_OPND_IS_CONST(ref)) return cvec(P, ref);
    if (ref >= 0) return vf.get(ref);
    return v3s(0.0f);
}

// One material node (RM1:313-479 shader / misc / math functions) for this lane; ray = (o, d, t,
// hit, inside), N = getNormal(hit). Shared by the table interpreter and the per-scene generated
// material functions (rmr_jit.cpp), which call it with a literal code.
RMR_D void mat_node(const KParams& P, Lane& L, int code, const V3* in, V3& o0, V3& o1, V3& o2, V3& o3) {
    const V3 N = L.nrm;
    const V3 ch = channel_vec(L.chan);
    o0 = v3s(0.0f); o1 = v3s(0.0f); o2 = v3s(0.0f); o3 = v3s(0.0f);
    switch (code) {
    case RMR_OP_M_FACING: {  // RM1:314-317
        const float sg = (float)((int)L.inside * 2 - 1);
        o0 = v3s(clampf(dot(L.d * sg, N), 0.0f, 1.0f));
        break;
    }
    case RMR_OP_M_INSIDE: o0 = v3s((float)(int)L.inside); break;
    case RMR_OP_M_ADD: o0 = in[0] + in[1]; break;
    case RMR_OP_M_SUB: o0 = in[0] - in[1]; break;
    case RMR_OP_M_MUL: o0 = in[0] * in[1]; break;
    case RMR_OP_M_DIV: o0 = in[0] / in[1]; break;
    case RMR_OP_M_MIX: {  // RM1:346-376
        const float r = lrand(L, v2(L.o.z, L.o.x));
        const float f = clampf(gray_ch(in[6] * ch, L.chan), 0.0f, 1.0f);
        bool second = r < f;
        if (f == 0.0f) second = false;
        else if (f == 1.0f) second = true;
        o0 = second ? in[3] : in[0];
        o1 = second ? in[4] : in[1];
        o2 = second ? in[5] : in[2];
        break;
    }
    case RMR_OP_M_DIFFUSE:  // RM1:378-387
        o0 = in[0];
        o1 = hemisphere(L, v2(L.hit.x, L.hit.y), v2(L.hit.z, L.hit.x), N);
        break;
    case RMR_OP_M_GLOSSY: {  // RM1:389-398
        o0 = in[0];
        const V3 hd = hemisphere(L, v2(L.hit.y, L.hit.x), v2(L.hit.x, L.hit.z), N);
        const float sg = -(float)((int)L.inside * 2 - 1);
        const V3 rf = reflect(L.d, N * sg);
        o1 = vmix(hd, rf, 1.0f - gray_ch(in[1] * ch, L.chan));
        break;
    }
    case RMR_OP_M_REFRACTION:  // RM1:400-427
        o0 = L.inside ? in[0] : v3s(1.0f);
        if (!L.inside) {
            o1 = normalize(refract(L.d, N, 1.0f / gray_ch(in[1] * ch, L.chan)));
            o2 = v3s(1.0f);
        } else {
            const V3 rdir = normalize(refract(L.d, -N, gray_ch(in[1] * ch, L.chan)));
            const V3 ddir = hemisphere(L, v2(L.hit.z, L.hit.y), v2(L.hit.y, L.hit.z), N);
            o1 = vmix(ddir, rdir, 1.0f - gray_ch(in[2] * ch, L.chan));
            o2 = v3s(0.0f);
        }
        break;
    case RMR_OP_M_VOLUME:  // RM1:429-474
        if (L.inside) {
            const float t = L.t;
            const float den = gray_ch(in[1] * ch, L.chan) / 20.0f;
            const int npts = (int)floorf(t * 100.0f);
            V3 hp = v3s(0.0f);
            for (int i = 0; i < npts; i++) {
                float r = lrand(L, v2(L.hit.x, L.hit.y));
                if (r < den) {
                    r = lrand(L, v2(L.hit.z, L.hit.y)) * t;
                    hp = vfma(L.d, r, L.o);
                    break;
                }
            }
            if (!is_zero(hp)) {
                o0 = in[0];
                o1 = hemisphere(L, v2(hp.x, hp.y), v2(hp.z, hp.y), v3s(0.0f));
                o2 = v3s(1.0f);
                o3 = hp;
            } else {
                o0 = v3s(1.0f); o1 = L.d; o2 = v3s(0.0f); o3 = v3s(0.0f);
            }
        } else {
            o0 = v3s(1.0f); o1 = L.d; o2 = v3s(1.0f); o3 = v3s(0.0f);
        }
        break;
    case RMR_OP_M_EMISSION:  // RM1:476-479
        o0 = in[0] * gray_ch(in[1] * ch, L.chan);
        break;
    default: break;
    }
}

// runs material `m` (wave-uniform) for this lane from the node tables
RMR_D void run_material_v1(const KParams& P, Lane& L, int m, V3& oc, V3& od, V3& oi, V3& oh) {
    CMat* mats = (CMat*)P.mats;
    COp* ops = (COp*)P.ops;
    VarFile vf;
    vf.clear();
    const int begin = mats[m].prog_begin, end = mats[m].prog_end;
    for (int k = begin; k < end; k++) {
        V3 in[7];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int ref = ops[k].in[i];
            in[i] = (ref == RMR_OPND_NONE) ? v3s(0.0f) : mat_opnd(P, vf, ref);
        }
        V3 o0, o1, o2, o3;
        mat_node(P, L, ops[k].code, in, o0, o1, o2, o3);
        const int w0 = ops[k].out[0], w1 = ops[k].out[1], w2 = ops[k].out[2], w3 = ops[k].out[3];
        if (w0 >= 0) vf.set(w0, o0);
        if (w1 >= 0) vf.set(w1, o1);
        if (w2 >= 0) vf.set(w2, o2);
        if (w3 >= 0) vf.set(w3, o3);
    }
    const int cv = mats[m].color_var, dv = mats[m].dir_var, iv = mats[m].inside_var, hv = mats[m].hit_var;
    if (cv >= 0) oc = vf.get(cv);
    if (dv >= 0) od = vf.get(dv);
    if (iv >= 0) oi = vf.get(iv);
    if (hv >= 0) oh = vf.get(hv);
}
// material policies of the trace kernel: table interpreter (ahead of time) or generated per scene
RMR_D void run_material_v2(const KParams& P, Lane& L, V3 pos, V3 pdir, V3 N, V3 t0, V3 t1, V3 t2,
                           V3& mat_color, V3& new_dir, bool& will_break);
// Material programs from the tables (node-program interpreters); the hipRTC kernels pass generated
// straight-line code instead (rmr_jit.cpp: JitMats for RM1 node programs, JitV2Mats for RM2's v2
// material, whose slots then live in registers rather than a scratch array)
struct TableMats {
    static RMR_D void run(const KParams& P, Lane& L, int m, V3& oc, V3& od, V3& oi, V3& oh) {
        run_material_v1(P, L, m, oc, od, oi, oh);
    }
    static RMR_D void run_v2(const KParams& P, Lane& L, V3 pos, V3 pdir, V3 N, V3 t0, V3 t1, V3 t2, V3& mat_color,
                             V3& new_dir, bool& will_break) {
        run_material_v2(P, L, pos, pdir, N, t0, t1, t2, mat_color, new_dir, will_break);
    }
};

// trace() hit tail, RM1:526-553
template <bool HO>
RMR_D void rm1_after_material(const KParams& P, Lane& L, V3 nc, V3 nd, V3 ni, V3 nh) {
    L.color = L.color * nc;
    L.inside = ni.x != 0.0f;
    if (is_zero(nd)) {
        if (finish_trace<RMR_VARIANT_RM1, HO>(P, L)) L.phase = PH_DONE;
        return;
    }
    const V3 hit = hitref<HO>(L);
    L.d = nd;
    if (is_zero(nh)) L.o = L.inside ? vfma(L.nrm, -0.002f, hit) : vfma(L.nrm, 0.003f, hit);
    else L.o = nh;
    next_bounce<RMR_VARIANT_RM1, HO>(P, L);
}

// ------------------------------------------------------------------------------------------
// RM2: NEE + v2 node material
// ------------------------------------------------------------------------------------------
RMR_D void make_tbn(V3 N, V3& c0, V3& c1, V3& c2) {  // makeTBN, RM2:211-229
    const V3 tangent = (N.x == 0.0f) ? v3(1.0f, 0.0f, 0.0f) : normalize(cross(v3(0.0f, 1.0f, 0.0f), N));
    c0 = normalize(cross(tangent, N));
    c1 = N;
    c2 = tangent;
}
RMR_D V3 diffuse_sample(Lane& L) {  // material_diffuse.samplePDF, RM2:279-290
    const float sin2 = lrand(L, v2(L.time, L.time));
    const float cos2 = 1.0f - sin2;
    const float st = sqrt_cr(sin2), ct = sqrt_cr(cos2);
    const float o = (lrand(L, v2(L.time, L.time)) * 2.0f) * PI_F;
    float so, co;
    det_sincos(o, so, co);
    return normalize(v3(st * co, ct, st * so));
}
RMR_D V3 glossy_sample(Lane& L, V3 wo, V3 n, float rough) {  // material_glossy.samplePDF, RM2:326-342
    if (rough == 0.0f) return reflect(wo, n);
    const float o = (lrand(L, v2(L.time, L.time)) * 2.0f) * PI_F;
    const float a = pow2(rough);
    const float r = lrand(L, v2(L.time, L.time));
    const float th = det_acos(sqrt_cr((1.0f - r) / ((a * a - 1.0f) * r + 1.0f)));
    float sth, cth, so, co;
    det_sincos(th, sth, cth);
    det_sincos(o, so, co);
    return normalize(v3(sth * co, cth, sth * so));
}
// the end of the generated mat_func_<id> (Graphics.cpp:724-736): slot 1 the reflectance, slot 0
// the new direction; shared by the interpreter below and the generated JitV2Mats
RMR_D void v2_tail(Lane& L, V3 pos, V3 refl, V3 dir, V3& mat_color, V3& new_dir, bool& will_break) {
    new_dir = dir;
    const float prob = fmaxf(refl.x, fmaxf(refl.y, refl.z));
    mat_color = L.color;
    if (lrand(L, v2(pos.z, pos.x)) <= 1.0f) {
        mat_color = mat_color * (refl / v3s(prob));
        will_break = false;
    } else {
        will_break = true;
    }
}
// generated mat_func_<id>, Graphics.cpp:705-739 + compileNode 412-463 (program is wave-uniform)
RMR_D void run_material_v2(const KParams& P, Lane& L, V3 pos, V3 pdir, V3 N, V3 t0, V3 t1, V3 t2,
                           V3& mat_color, V3& new_dir, bool& will_break) {
    COp* ops = (COp*)P.ops;
    VarFile vf;
    vf.clear();
    for (int k = P.v2_begin; k < P.v2_end; k++) {
        const int code = ops[k].code;
        if (code == RMR_OP_V2_DIFFUSE) {
            vf.set(ops[k].out[0], mat_mul(t0, t1, t2, diffuse_sample(L)));
            vf.set(ops[k].out[1], cvec(P, ops[k].in[0]));
        } else if (code == RMR_OP_V2_GLOSSY) {
            const float rough = cvec(P, ops[k].in[1]).x;
            vf.set(ops[k].out[0], mat_mul(t0, t1, t2, glossy_sample(L, pdir, N, rough)));
            vf.set(ops[k].out[1], cvec(P, ops[k].in[0]));
        } else if (code == RMR_OP_V2_FRESNEL) {
            vf.set(ops[k].out[0], v3s(pow5(1.0f - clampf(dot(N, pdir), 0.0f, 1.0f)) * 0.96f + 0.04f));
        } else if (code == RMR_OP_V2_MIX) {
            const float r = lrand(L, v2(pos.x, pos.z));
            const bool second = r <= vf.get(ops[k].in[4]).x;
            const V3 dsel = second ? vf.get(ops[k].in[2]) : vf.get(ops[k].in[0]);
            const V3 rsel = second ? vf.get(ops[k].in[3]) : vf.get(ops[k].in[1]);
            vf.set(ops[k].out[0], dsel);
            vf.set(ops[k].out[1], rsel);
        }
    }
    v2_tail(L, pos, vf.get(1), vf.get(0), mat_color, new_dir, will_break);
}
RMR_D V3 rm2_albedo(const KParams& P, int id) {
    if (id < 0 || id >= RMR_MAX_MATERIALS) return v3s(0.0f);
    const float* a = P.rm2->albedo[id];
    return v3(a[0], a[1], a[2]);
}

// ------------------------------------------------------------------------------------------
// RM3: spectral event (mat_func_k RM3:251-345, sky RM3:408-438)
// ------------------------------------------------------------------------------------------
RMR_D bool spectral_event(Lane& L, uint32_t mn, uint32_t mx, float pw, V2 seed) {
    if (L.wl == 0u) {
        float r = lrand(L, seed);
        r = r * (float)((mx - mn) / 5u);
        r = floorf(r) * 5.0f;
        L.wl = (uint32_t)(int)r + mn;
        L.power = L.power * pw;
        return false;
    }
    if (L.wl < mn || L.wl > mx) { L.wl = 0u; return true; }
    L.power = L.power * pw;
    return false;
}

// ------------------------------------------------------------------------------------------
// shading of the parked lanes
// ------------------------------------------------------------------------------------------
template <int VAR, bool PROG, class MATS, bool CERT = false>
RMR_D void shade(const KParams& P, Lane& L) {
    constexpr bool HO = hit_in_origin<VAR, PROG>();
    // (certified hits, CERT: L.nrm holds getNormal's differences from cert_normals)
    // getNormal's normalize (RM1:267), deferred from the last probe to the batch: the map loop then
    // carries no division/sqrt for the few lanes that finish a normal in a given iteration
    if (L.phase == PH_HIT) L.nrm = normalize(L.nrm);
    if (VAR == RMR_VARIANT_RM1) {
        const bool want = (L.phase == PH_HIT);
        const int id = want ? (int)L.mid : -1;
        int kind = MAT_NONE;
        DMat dm{};
        if (want && id >= 0 && id < P.n_mats) {
            dm = P.dmats[id];
            kind = dm.kind;
        }
        V3 nc = v3s(0.0f), nd = v3s(0.0f), ni = v3s(0.0f), nh = v3s(0.0f);
        if (kind == MAT_DIFFUSE) {          // shader_diffuse(ray, c, color, dir), RM1:378-387
            nc = v3(dm.c[0], dm.c[1], dm.c[2]);
            const V3 hp = hitref<HO>(L);
            nd = hemisphere(L, v2(hp.x, hp.y), v2(hp.z, hp.x), L.nrm);
        } else if (kind == MAT_EMISSION) {  // shader_emission(ray, c, p, color), RM1:476-479
            // gray_ch of p without separateChannels is a per-material constant (host, DMat.gray1)
            float g = dm.gray1;
            if (L.chan >= 0) g = gray_ch(v3(dm.p[0], dm.p[1], dm.p[2]) * channel_vec(L.chan), L.chan);
            nc = v3(dm.c[0], dm.c[1], dm.c[2]) * g;
        }
        if constexpr (PROG) {  // generic node programs, one wave-uniform material at a time
            const bool valid = (kind == MAT_PROGRAM);
            uint64_t pending = __ballot(valid);
            while (pending) {
                const int lead = __ffsll((unsigned long long)pending) - 1;
                const int m = __builtin_amdgcn_readlane(id, lead);
                const bool mine = valid && id == m;
                if (mine) MATS::run(P, L, m, nc, nd, ni, nh);
                pending &= ~__ballot(mine);
            }
        }
        if (want) rm1_after_material<HO>(P, L, nc, nd, ni, nh);
        if (L.phase == PH_MISS) {  // shader_emission(ray, skyColor(dir), vec3(1), emit), RM1:555-561
            // gray_ch of vec3(1) is (1 + 1 + 1) / (1 + 1 + 1) = 1 exactly without separateChannels
            // (chan < 0): the division runs only for channel passes
            float g = 1.0f;
            if (L.chan >= 0) g = gray_ch(v3s(1.0f) * channel_vec(L.chan), L.chan);
            const V3 emit = sky_color(P, L.d) * g;
            L.color = L.color * emit;
            if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
        }
    }
    if (VAR == RMR_VARIANT_RM2) {
        const V3 lp = v3(P.rm2_light[0], P.rm2_light[1], P.rm2_light[2]);
        if (L.phase == PH_HIT) {  // RM2:436-506
            const V3 pos = hitref<HO>(L), N = L.nrm, pdir = -L.d;
            const int id = (int)L.mid;
            if (id == P.rm2_node_id) {
                V3 t0, t1, t2;
                make_tbn(N, t0, t1, t2);
                V3 matc, nd;
                bool wb;
                MATS::run_v2(P, L, pos, pdir, N, t0, t1, t2, matc, nd, wb);
                L.color = L.color * matc;
                if (wb) {
                    L.color = v3s(0.0f);
                    if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
                } else {
                    L.o = vfma(N, 0.002f, pos);
                    L.d = nd;
                    next_bounce<VAR, HO>(P, L);
                }
            } else {  // light-march toward the point light, RM2:481
                L.o = vfma(N, 0.002f, pos);
                L.d = normalize(lp - pos);
                // Light-side bound: the NEE step reads this march only through sd >= len (RM2:482,
                // len = length(lightPos - pos), the same expression as there). t starts at 0 <= len and
                // a step adds dist * stepMultiply with dist >= 0.001, so t can pass len only with
                // stepMultiply > 0, and then never decreases: every ending after that gives sd >= len (a
                // hit returns its t > len; a miss or the step limit maxDist >= len). The march may then
                // end as its miss at once (t = maxDist), as past the escape bound; only the number of
                // map() calls differs.
                float te = __builtin_nanf("");   // (start_march: the escape bound alone)
#if RMR_SHADOW_LIGHT_BOUND
                const float len = length(lp - pos);
                if (P.esc_on && len <= P.max_dist) te = fminf(ray_exit(P, L.o, L.d), len);
#endif
                start_march<HO>(P, L, PH_SHADOW, te);   // hit/mid/nrm stay for the NEE step
            }
        } else if (L.phase == PH_NEE) {  // RM2:482-501
            const V3 pos = hitref<HO>(L), N = L.nrm;
            const float sd = L.t;
            const V3 mc = rm2_albedo(P, (int)L.mid);
            const V3 ld = normalize(lp - pos);
            const float len = length(lp - pos);
            if (sd >= len) {
                const V3 brdf = v3(mc.x / PI_F, mc.y / PI_F, mc.z / PI_F);
                V3 c = L.color * brdf;
                c = c * clampf(dot(ld, N), 0.0f, 1.0f);
                c = c * (P.rm2_light_power / pow2(len));
                L.fin = L.fin + c;
            }
            V3 t0, t1, t2;
            make_tbn(N, t0, t1, t2);
            const V3 nd = mat_mul(t0, t1, t2, diffuse_sample(L));
            const float prob = fmaxf(mc.x, fmaxf(mc.y, mc.z));
            if (lrand(L, v2(pos.z, pos.x)) <= prob) {
                L.color = L.color * (mc / v3s(prob));
                L.o = vfma(N, 0.002f, pos);
                L.d = nd;
                next_bounce<VAR, HO>(P, L);
            } else {
                L.color = v3s(0.0f);
                if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
            }
        } else if (L.phase == PH_MISS) {
            L.color = L.color * sky_color(P, L.d);   // RM2:509
            if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
        }
    }
    if (VAR == RMR_VARIANT_RM3) {
        if (L.phase == PH_HIT) {  // RM3:368-406
            const V3 pos = hitref<HO>(L), N = L.nrm;
            const int id = (int)L.mid;
            V3 nd = v3s(0.0f);
            bool stop = false;
            if (id >= 0 && id < P.n_mats && P.spec[id].defined) {
                const rmr_spectral s = P.spec[id];
                if (spectral_event(L, s.min_wave, s.max_wave, s.power, v2(pos.y, pos.x))) stop = true;
                else if (s.terminates) stop = true;
                else nd = hemisphere(L, v2(pos.x, pos.y), v2(pos.z, pos.y), N);
            }
            if (stop) {
                if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
            } else {
                L.o = vfma(N, 0.002f, pos);
                L.d = nd;
                next_bounce<VAR, HO>(P, L);
            }
        } else if (L.phase == PH_MISS) {  // RM3:408-438
            const V3 pos = hitref<HO>(L);
            spectral_event(L, P.spec_sky.min_wave, P.spec_sky.max_wave, P.spec_sky.power, v2(pos.y, pos.x));
            if (finish_trace<VAR, HO>(P, L)) L.phase = PH_DONE;
        }
    }
}

// Lane state that only shading, refills and the end of a trace read (RM1 throughput / RM3 power and
// hero wavelength, RNG chain, unit, channel, bounce count): parked in LDS, one word per lane per
// field (conflict-free), while the nearest-primitive cache's inner march loop runs.
constexpr int kColdWords = 8;
template <int VAR>
RMR_D void cold_put(float (*s)[256], int t, const Lane& L) {
    s[0][t] = __uint_as_float(L.unit);
    s[1][t] = L.gxt;
    s[2][t] = L.gyt;
    s[3][t] = L.rc;
    if constexpr (VAR == RMR_VARIANT_RM3) {
        s[4][t] = L.power;
        s[5][t] = __uint_as_float(L.wl);
    } else {
        s[4][t] = L.color.x;
        s[5][t] = L.color.y;
        s[6][t] = L.color.z;
    }
    s[7][t] = __int_as_float((L.chan + 1) | (L.bounces << 8));   // chan in [-1, 2], bounces >= 0
}
template <int VAR>
RMR_D void cold_get(float (*s)[256], int t, Lane& L) {
    L.unit = __float_as_uint(s[0][t]);
    L.gxt = s[1][t];
    L.gyt = s[2][t];
    L.rc = s[3][t];
    if constexpr (VAR == RMR_VARIANT_RM3) {
        L.power = s[4][t];
        L.wl = __float_as_uint(s[5][t]);
    } else {
        L.color = v3(s[4][t], s[5][t], s[6][t]);
    }
    const int cb = __float_as_int(s[7][t]);
    L.chan = (cb & 0xff) - 1;
    L.bounces = cb >> 8;
}

// The lane id where trace_main needs it (the work-queue fetch, counter flushes): recomputed at each
// use (two VALU) instead of a hoisted value the allocator keeps across the loop — at 8 waves / SIMD it
// spilled that register to scratch (the stepped Mandelbulb kernel)
RMR_D uint32_t lane_now() {
    uint32_t v;
    __asm__ volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}

// The nearest-primitive cache's state after a full map() at p: primitives kw, kw2 (kw < 0: none) and the
// lower bound s2 of every other primitive's distance (MAP::full); |s2| 2^-20: the rounding of the
// check's own subtractions
RMR_D void npc_apply(const KParams& P, Lane& L, V3 p, int kw, int kw2, float s2) {
    L.cw = kw >= 0 ? kw : 0;
    L.cw2 = kw >= 0 ? kw2 : 0;
    L.cs = kw >= 0 ? s2 - fmaf(fabsf(s2), 0x1p-20f, npc_eps(P, p)) - (L.phase == PH_NORMAL ? NPC_PROBE_DELTA : 0.0f)
                   : -__builtin_inff();
    L.cta = L.t;
}


// a defined value the compiler cannot see (no constant to propagate into the loop PHIs): trace_main's
// lane at kernel entry; the inline asm emits no instruction
RMR_D float opq() {
    float v;
    __asm__ volatile("; lane init %0" : "=v"(v));
    return v;
}
RMR_D V3 opq3() { return v3(opq(), opq(), opq()); }
RMR_D void lane_define(Lane& L) {
    L.unit = __float_as_uint(opq());
    L.gxt = opq(); L.gyt = opq(); L.rc = opq();
    L.o = opq3(); L.d = opq3();
    L.t = opq();
    L.ctr = __float_as_int(opq());
    L.hit = opq3();
    L.mid = opq();
    L.nrm = opq3();
    L.color = opq3();
    L.chan = __float_as_int(opq()); L.bounces = __float_as_int(opq());
    L.inside = false;
    L.time = opq();
    L.fin = opq3();
    L.wl = __float_as_uint(opq());
    L.power = opq();
    L.cw = __float_as_int(opq()); L.cw2 = __float_as_int(opq());
    L.cs = opq(); L.cta = opq(); L.texit = opq();
    L.e = opq3();
}
RMR_D bool is_active(int ph) { return (uint32_t)ph <= (uint32_t)PH_SHADOW; }   // PH_DONE (-1) is not
RMR_D bool is_shade(int ph) { return ph >= PH_HIT; }   // (PH_DONE, -1, is not)

// ------------------------------------------------------------------------------------------
// the trace kernel
// ------------------------------------------------------------------------------------------
// Occupancy target (waves per SIMD) for the fast specialisations: the kernel is latency-bound
// (scalar-load and dependent-chain stalls), and 8 waves/SIMD measured +8% over the 5 that the
// register allocator picks unconstrained. The general/interpreter kernels keep their registers.
#ifndef RMR_FAST_WAVES
#define RMR_FAST_WAVES 8
#endif
// waves/SIMD the register allocator targets for the general-map (node program, Mandelbulb) kernels
// without material programs (A/B on C3: 8 waves +8% over the allocator's free choice)
#ifndef RMR_GENERAL_WAVES
#define RMR_GENERAL_WAVES 8
#endif
// waves/SIMD of the nearest-primitive cache kernels (BVH scenes): at 8 the allocator spills hot march
// state (origin, escape bound) inside the cache loop, reloaded every iteration; at 6 it does not
// (csg256 8 spp: 8 / 7 / 6 / 5 waves -> 25.3 / 23.5 / 22.2 (64-unit chunks) / 24.3 ms)
#ifndef RMR_CACHE_WAVES
#define RMR_CACHE_WAVES 6
#endif
// waves/SIMD target of the kernels with node-program materials (1 = none: the allocator's choice, 4-6
// waves at 79-120 VGPRs; the hipRTC kernels set 6, rmr_jit.cpp). Until round 5 the 6 / 7-wave builds of
// glass_test.scene rendered wrong samples: `Lane L;` left lane fields undefined, the IR carried undef
// PHIs into the persistent loop, and the allocator's live-range splitting dropped the prologue's
// throughput on some refill paths (trace_main now defines every field: lane_define)
#ifndef RMR_PROG_WAVES
#define RMR_PROG_WAVES 1
#endif
// waves/SIMD target of the RM2 (next-event estimation) kernels: 1 = the allocator's choice (5 waves)
#ifndef RMR_RM2_WAVES
#define RMR_RM2_WAVES 1
#endif
template <int VAR, bool GENERAL, bool PROG>
constexpr int trace_waves() {
    return PROG ? RMR_PROG_WAVES
                : (VAR == RMR_VARIANT_RM2 ? RMR_RM2_WAVES : (GENERAL ? RMR_GENERAL_WAVES : RMR_FAST_WAVES));
}

// the map() point of an active lane: one select per component in HO kernels (A/B: C2 +1%; the RM2
// kernel was slower with it)
#define RMR_MARCH_POINT(L) (HO ? march_point<HO>(L) : ((L.phase == PH_NORMAL) ? probe_point<HO>(L) : vfma(L.d, L.t, L.o)))
#ifndef RMR_CHUNK
#define RMR_CHUNK 128   // units a wave takes from the work queue at a time (primary rays in LDS)
#endif
#ifndef RMR_QUEUE_PARTS
#define RMR_QUEUE_PARTS 32   // work-queue partitions (counters; rmr_internal.h kQueueBytes): 32 against
                             // 16, same process: RM3 -0.5 / -3.5% at 16 / 4 spp, RM2 -2%, C3 -1.2%, the
                             // rest within noise (r06z2_parts_ab.log, r06z4_parts_ab2.log)
#endif
#ifndef RMR_QUEUE_SEQ
#define RMR_QUEUE_SEQ 1   // small launches: partitions a wave tries in turn before it reads every counter
#endif
#define RMR_QUEUE_STRIDE 32   // 32-bit words between two partition counters (128 B)
static_assert(RMR_QUEUE_STRIDE == kQueueWordStride, "fold_main zeroes the counters at this stride");
static_assert(RMR_QUEUE_PARTS >= 1 && RMR_QUEUE_PARTS <= 64 && RMR_QUEUE_PARTS * RMR_QUEUE_STRIDE * 4 <= (int)kQueueBytes,
              "queue counters: one per lane of the scan");
#ifndef RMR_CHUNK_CACHE
#define RMR_CHUNK_CACHE 64   // the same for the nearest-primitive cache kernels (6 blocks per CU: 24 KiB of LDS each)
#endif
typedef uint32_t WCount;
template <int VAR, class MAP, bool PERSIST, bool PROG, class MATS = TableMats>
RMR_D void trace_main(const KParams& P) {
    constexpr bool HO = hit_in_origin<VAR, PROG>();
    // certified hits (march_update: ctr = -1) get getNormal's probes in the shading batch from one
    // primitive: the approximate sphere/box maps' certificate (MAP::kCert), the one-primitive cache's
    constexpr bool CERT = HO && (MAP::kCert || (MAP::kCache && RMR_NPC_K == 1 && RMR_CACHE_CERT));
    // Every lane field defined before the persistent loop. With `Lane L;` alone the optimised IR had
    // `phi [undef, %entry]` at the loop header for each field, and the allocator's live-range
    // splitting was then free to lose a lane's value on refill paths (the round-4 6 / 7-wave glass_test
    // miscompute; tests/test_kernel_ir.py, test_gpu_prog_waves.py). Opaque values (lane_define), not
    // `Lane L{}`: zeros give the optimiser constants to propagate through the loop PHIs, which cost
    // the Cornell-5 kernel 20 spilled VGPRs (C2 +0.8%, C3 +1.0%, same process)
    Lane L;
    lane_define(L);
    L.phase = PH_IDLE;
    init_probe(L);
    MBStep mbs{};   // stepped map() state (MAP::kStepped); i < 0: no map() in progress
    mbs.i = -1;
    mbs.fin = false;
    // per-wave event counters, 32-bit (wave-uniform: SGPRs; 64-bit ones cost the cache kernels
    // scratch round trips), flushed to the 64-bit global counters before any can pass 2^31
    WCount maps = 0, iters = 0, shades = 0, fulls = 0, shaded = 0, bmaps = 0;
    constexpr uint32_t CHUNK = MAP::kCache ? RMR_CHUNK_CACHE : RMR_CHUNK;
    const uint32_t n_units = (uint32_t)P.n_units;   // < 2^32 per launch (host chunking)
    // units per claim: the LDS ray buffer's CHUNK, or fewer for a small launch (the host's chunk_units)
    const uint32_t CK = P.chunk_units - 1u < CHUNK ? P.chunk_units : CHUNK;
    uint32_t rnext = 0, rend = 0;
    // The work queue in RMR_QUEUE_PARTS partitions of whole chunks, each with its own counter (128 B
    // apart): a wave starts on partition blockIdx % parts (with a multiple of 8 partitions, blocks of one XCD
    // under the round-robin block dispatch over the 8 XCDs) and moves on to the next partition when
    // its own is used up. One counter shared by every wave of the chip serialises its atomics: RM2's
    // short paths fetch ~80 chunks per microsecond, and one counter held its 1080p 16-spp frame at
    // 3.24 ms against 0.98 / 0.97 ms with 8 / 16 partitions (round 4; Cornell-5, RM3,
    // multilight, the Mandelbulb 1-2.5% faster with 16 than with one counter).
    const uint32_t n_chunks = (n_units + CK - 1) / CK;
    auto part_begin = [&](uint32_t q) -> uint32_t {   // first unit of partition q (q = parts: the end)
        return (uint32_t)(((uint64_t)n_chunks * q) / (uint32_t)RMR_QUEUE_PARTS) * CK;
    };
    uint32_t part = blockIdx.x % (uint32_t)RMR_QUEUE_PARTS, tried = 0;
    // small launches (fewer than 4 chunks per wave of the grid: C1's 256 x 256 frame) scan the counters
    // after the first used-up partition, where most waves find theirs used up at once; larger ones walk
    // the partitions in turn (RM2 1080p: 21.2 against 17.5-19.6 Gsamples/s with a scan)
    const uint32_t q_seq = n_chunks < gridDim.x * 16u ? (uint32_t)RMR_QUEUE_SEQ : (uint32_t)RMR_QUEUE_PARTS;
    bool exhausted = false;
    if (!PERSIST) {
        const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
        if (u < n_units) begin_trace<VAR, HO>(P, L, u, true);
        exhausted = true;
    }
    const int T = P.shade_threshold, TR = P.refill_threshold;
    // eye_map: every primary ray (a fresh unit, or a separateChannels restart) starts its march at
    // t = 0 from the eye, whose march point fma(dir, 0, eye) is the eye itself for a finite direction
    // (the host clears P.eye_step where an eye coordinate is -0 or not finite). Its map() is therefore
    // one value for the whole launch: evaluated here once by the wave (every lane the same point) and
    // applied as each primary ray's first step (march_update) instead of a map() iteration. On
    // Cornell-5 that point ties the two side walls exactly (x = 0), so it was also the approximate
    // map's most frequent exact-fold fallback.
    // (HO kernels: RM1 without node-program materials and RM3; the node-program-material kernels
    // measured 0.3-1% slower with it, RM2 neutral)
    const bool eye1 = HO && !MAP::kCache && P.eye_step != 0;
    V2 meye = v2(0.0f, 0.0f);
    if (eye1) {
        meye = MAP::eval(P, v3(P.eye[0], P.eye[1], P.eye[2]));
        meye = v2(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(meye.x))),
                  __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(meye.y))));
    }
#ifdef RMR_PROFILE
    uint64_t cyc[4] = {0, 0, 0, 0};   // refill, map() iterations, shading, cache kernels: full map() batches
    uint64_t full_lanes = 0;           // cache kernels: lanes in the full map() batches
    uint64_t cyc_claim = 0, cyc_rays = 0;   // refill: work-queue claims (atomics), chunk primary rays
    const uint64_t c_begin = __builtin_amdgcn_s_memtime();
#define RMR_STAMP(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define RMR_STAMP(v)
#endif
    __shared__ ChunkRay s_ray[4][CHUNK];   // per wave (256-thread blocks = 4 waves)
    __shared__ int s_tab[4][CERT ? 64 : 1];   // cert_normals: certified lanes by rank
    // cache kernels: the lane's shading-only state during the inner march loop (cold_put / cold_get)
    constexpr bool kStash = MAP::kCache && HO;
    __shared__ float s_cold[kStash ? kColdWords : 1][kStash ? 256 : 1];
    // the cached primitives' table in LDS (per-lane reads of the cache path)
    __shared__ float4 s_dp[MAP::kCache ? 2 * RMR_NPC_LDS_MAX : 1];
    // the stepped Mandelbulb kernel (8 waves / SIMD, 20 KiB of LDS per block): the RNG state (seeds
    // gx + time, gy + time and the chain value randChange), which only shading reads and advances,
    // waits in LDS between shading batches instead of in registers the allocator spilled to scratch
#ifndef RMR_SEED_LDS
#define RMR_SEED_LDS 1
#endif
    constexpr bool kSeeds = MAP::kStepped && PERSIST && RMR_SEED_LDS;
    __shared__ float s_rng[kSeeds ? 3 : 1][4][kSeeds ? 64 : 1];
    const bool dp_lds = MAP::kCache && (RMR_NPC_DP_LDS >= 0 ? RMR_NPC_DP_LDS == 1 : P.n_prims <= RMR_NPC_LDS_MAX);
    if (dp_lds) {
        if constexpr (kNpcPacked) {
            for (int i = (int)threadIdx.x; i < P.n_prims; i += (int)blockDim.x) {
                float4 a = ((const float4*)P.dprims)[2 * i], b = ((const float4*)P.dprims)[2 * i + 1];
                npc_pack_entry(a, b);
                s_dp[kTabStep * i] = a;
                s_dp[kTabStep * i + kTabHi] = b;
            }
        } else {
            for (int i = (int)threadIdx.x; i < 2 * P.n_prims; i += (int)blockDim.x)
                s_dp[kTabStep * (i >> 1) + (i & 1) * kTabHi] = ((const float4*)P.dprims)[i];
        }
        __syncthreads();
    }
#define RMR_PRIM_DIST(k, p, mid, j) (dp_lds ? prim_dist_tab(s_dp + kTabStep * (k), p, mid, j) : prim_dist(P, k, p, mid, j))
    static_assert(!RMR_NPC_TAB_SOA || MAP::kCache, "an SoA table kernel reads dtab as the LDS copy only");
#define RMR_DTAB (dp_lds ? (const float4*)s_dp : (const float4*)P.dprims)
    const int wv = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 3);   // the wave's index in its block (an SGPR)
    uint32_t chunk_base = 0;
#ifdef RMR_WAVE_TIMES   // counters [9] ~min start, [11] ~min / [10] max queue exhaustion, [12] ~min /
                        // [13] max end, [15] sum over waves of end - exhaustion (s_memrealtime ticks)
    unsigned long long t_exh = 0;
    if (lane_now() == 0) atomicMax(P.counters + 9, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
    for (;;) {
        RMR_STAMP(c0);
        bool fresh = false;
        uint32_t fu = 0;
        if (PERSIST && !exhausted) {
            uint64_t idle = __ballot(L.phase == PH_IDLE);
            uint64_t act0 = __ballot(is_active(L.phase));
            if (idle && (__popcll(idle) >= TR || act0 == 0)) {
                if (rnext >= rend) {
                    // the next chunk of the wave's work partition; once that one is used up, of the next
                    // partitions in turn, and after RMR_QUEUE_SEQ used-up ones of the next partition (in
                    // cyclic order) whose counter says it has work left — all counters read at once, one
                    // per lane — until none has (the launch's work is all handed out)
                    unsigned int base = 0;
#ifdef RMR_PROFILE
                    const uint64_t q0 = __builtin_amdgcn_s_memtime();
#endif
                    for (;;) {
                        const uint32_t pb = part_begin(part), pe = part_begin(part + 1);
                        unsigned int off = 0;
                        if (lane_now() == 0) off = atomicAdd((unsigned int*)P.queue + RMR_QUEUE_STRIDE * part, CK);
                        off = __builtin_amdgcn_readfirstlane(off);
                        if (off < pe - pb) {
                            base = pb + off;
                            rend = n_units - base > CK ? base + CK : n_units;
                            break;
                        }
                        // the next few partitions in turn (one atomic each), then a scan of all counters
                        if (++tried < q_seq) {
                            part = part + 1 == (uint32_t)RMR_QUEUE_PARTS ? 0 : part + 1;
                            continue;
                        }
                        if (q_seq >= (uint32_t)RMR_QUEUE_PARTS) {
                            exhausted = true;
                            break;
                        }
                        const uint32_t q = lane_now();
                        bool left = false;
                        if (q < (uint32_t)RMR_QUEUE_PARTS) {
                            const unsigned int c = __hip_atomic_load((unsigned int*)P.queue + RMR_QUEUE_STRIDE * q,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            left = c < part_begin(q + 1) - part_begin(q);
                        }
                        const uint64_t lm = __ballot(left);
                        if (lm == 0) {
                            exhausted = true;
                            break;
                        }
                        // one of the partitions with work left, spread over the waves (the k-th, k from
                        // the wave's index): piling every wave onto the same one serialises its counter
                        uint64_t m = lm;
                        for (int k = (int)((blockIdx.x * 4u + (uint32_t)wv + tried) % (uint32_t)__popcll(lm)); k > 0; k--)
                            m &= m - 1;
                        part = (uint32_t)__builtin_ctzll(m);
                    }
                    rnext = base;
#ifdef RMR_PROFILE
                    const uint64_t q1 = __builtin_amdgcn_s_memtime();
                    cyc_claim += q1 - q0;
#endif
#ifdef RMR_WAVE_TIMES   // diagnostics (tools/wave_times.py): when each wave finds the queue empty
                    if (exhausted && lane_now() == 0) {
                        const unsigned long long te = __builtin_amdgcn_s_memrealtime();
                        t_exh = te;
                        atomicMax(P.counters + 11, ~te);
                        atomicMax(P.counters + 10, te);
                    }
#endif
                    if (!exhausted) {  // the chunk's primary rays, all 64 lanes at once
                        chunk_base = base;
                        for (uint32_t sl = lane_now(); sl < CK; sl += 64) {
                            if (base + sl < rend) s_ray[wv][sl] = chunk_ray<HO>(P, base + sl);
                        }
                        __builtin_amdgcn_wave_barrier();
#ifdef RMR_PROFILE
                        cyc_rays += __builtin_amdgcn_s_memtime() - q1;
#endif
                    }
                }
                if (!exhausted) {
                    const uint32_t avail = rend - rnext;
                    const uint32_t nidle = (uint32_t)__popcll(idle);
                    const uint32_t take = avail < nidle ? avail : nidle;
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    if (L.phase == PH_IDLE && rank < take) {
                        fresh = true;
                        fu = rnext + rank;
                    }
                    rnext += take;
                }
            }
        }
        const bool restart = (L.phase == PH_RESTART);
        if (PERSIST) {
            if (__ballot(fresh)) {
                if (fresh) {
                    const ChunkRay cr = s_ray[wv][fu - chunk_base];
                    if constexpr (kSeeds) {
                        const uint32_t ln = lane_now();
                        s_rng[0][wv][ln] = cr.b.x;
                        s_rng[1][wv][ln] = cr.b.y;
                        s_rng[2][wv][ln] = cr.a.w;
                    }
                    begin_unit<VAR, HO>(P, L, fu, cr.a, cr.b);
                }
            }
            if (__ballot(restart)) {
                if (restart) begin_trace<VAR, HO>(P, L, L.unit, false);
            }
        } else if (__ballot(restart)) {
            if (restart) begin_trace<VAR, HO>(P, L, L.unit, false);
        }
        if (eye1) {   // primary rays' first march step (eye_map above)
            const float dsum = (L.d.x + L.d.y) + L.d.z;   // NaN for a NaN / infinite direction
            const bool first = (fresh || restart) && L.phase == PH_MARCH && (dsum - dsum == 0.0f);
            if (__ballot(first)) {
                if (first) march_update<HO>(P, L, meye);
            }
        }
        RMR_STAMP(c1);
        const bool act = is_active(L.phase);
        const uint64_t amask = __ballot(act);
        if constexpr (MAP::kCache && HO) {   // HO kernels only: normalized directions, fixed bounce offsets
            // the shading-only lane state waits in LDS during the inner march loop: its registers are
            // then free for the map, where the compiler would otherwise spill the lane to scratch at
            // every loop entry (C4: ~0.5 TB of scratch writes per launch)
            if constexpr (kStash) {
                if (amask) {
                    cold_put<VAR>(s_cold, (int)threadIdx.x, L);
                    __asm__ volatile("" ::: "memory");
                }
            }
            for (bool go = amask != 0; go;) {   // inner march loop (see the non-cache path)
                const bool act1 = is_active(L.phase);
                // nearest-primitive cache: one primitive where the bound holds; lanes where it does not
                // wait for a full map() batch (>= full_threshold lanes, or no lane could use the cache)
                V3 p = v3s(0.0f);
                V2 m = v2(P.max_dist, -1.0f);
                bool ok = false;
                float F = 0.0f, mid = -1.0f;
                int jw = 0;
                bool pfin = false;   // a point without NaN (and without +-inf of both signs)
                if (act1) {
                    p = RMR_MARCH_POINT(L);
                    F = RMR_PRIM_DIST(L.cw, p, mid, jw);
                    float Fm = F;
                    if (RMR_NPC_K >= 2) {
                        // both cached primitives, folded in scene order: opU's closed form over the
                        // pair (every other primitive is strictly farther when the bound holds)
                        float mid2;
                        int jw2;
                        const float F2 = RMR_PRIM_DIST(L.cw2, p, mid2, jw2);
                        if (jw2 < jw) {
                            opu(m, F2, mid2);
                            opu(m, F, mid);
                        } else {
                            opu(m, F, mid);
                            opu(m, F2, mid2);
                        }
                        Fm = fminf(F, F2);
                    } else {
                        opu(m, F, mid);
                    }
#ifdef RMR_COUNT_FLOPS
                    {   // the cached primitives evaluated here (types per lane: the leaf table's)
                        const int t1 = __float_as_int(((const float4*)(P.dprims + L.cw))[1].z) & 0xff;
                        const int t2 = __float_as_int(((const float4*)(P.dprims + L.cw2))[1].z) & 0xff;
                        const uint64_t nb = (uint64_t)__popcll(__ballot(t1 == RMR_PRIM_BOX)) +
                                            (RMR_NPC_K >= 2 ? (uint64_t)__popcll(__ballot(t2 == RMR_PRIM_BOX)) : 0);
                        const uint64_t n = active_lanes() * (RMR_NPC_K >= 2 ? 2 : 1);
                        RMR_COUNT(P.counters, n - nb, 10 + 2, 1);
                        RMR_COUNT(P.counters, nb, 22 + 2, 1);
                    }
#endif
                    const float delta = (L.phase == PH_NORMAL) ? NPC_PROBE_DELTA : (L.t - L.cta) * (1.0f + 0x1p-21f);
                    const float sum = p.x + p.y + p.z;   // NaN for a NaN (or +-inf mixed) point
                    pfin = sum == sum;
                    ok = pfin && (L.cs - delta - npc_eps(P, p) > Fm);
                }
                const uint64_t okm = __ballot(act1 && ok);
                const uint64_t fm = __ballot(act1 && !ok);
                bool done = ok;
                const int nf = __popcll(fm), nok = __popcll(okm);
                const int ft = P.full_threshold & 0xff, fr = P.full_threshold >> 8;
                if (fm && (okm == 0 || nf >= ft || nf * fr >= 8 * nok)) {
                    RMR_STAMP(f0);
                    if (act1 && !ok) {
                        int kw = -1, kw2 = 0;   // (written by every path of MAP::full: defined for the compiler too)
                        float s2 = -__builtin_inff();
                        // seeded with the cached primitive only at a finite point: prim_dist's box form
                        // of a sphere drops a NaN coordinate (fmaxf / fminf) where sd_sphere keeps it
                        m = MAP::full(P, p, kw, kw2, s2, (pfin && F == F) ? L.cw : -1, jw, F, mid, RMR_DTAB);
                        npc_apply(P, L, p, kw, kw2, s2);
                        done = true;
                    }
                    fulls++;
#ifdef RMR_PROFILE
                    RMR_STAMP(f1);
                    cyc[3] += f1 - f0;
                    full_lanes += (uint64_t)nf;
#endif
                }
#ifdef RMR_NPC_CHECK   // diagnostics (RMR_JIT_OPTS=-DRMR_NPC_CHECK): every cached map() against the exact fold
                if (done) {
                    const V2 ex = map_bvh(P, p);
                    if (__float_as_uint(ex.x) != __float_as_uint(m.x) || __float_as_uint(ex.y) != __float_as_uint(m.y))
                        printf("NPC mismatch unit %u ph %d ctr %d t %a cta %a p (%a %a %a) m (%a %a) exact (%a %a) ok %d "
                               "cw %d cw2 %d F %a cs %a\n",
                               L.unit, L.phase, L.ctr, L.t, L.cta, p.x, p.y, p.z, m.x, m.y, ex.x, ex.y, (int)ok, L.cw, L.cw2,
                               F, L.cs);
                }
#endif
                if (done) {
                    if (L.phase == PH_NORMAL) normal_update(L, m.x);
                    else march_update<HO, true>(P, L, m, 0, false, p);
                }
                const uint64_t dm = __ballot(done);
                maps += (WCount)__popcll(dm);
                iters += dm ? 1 : 0;
                const uint64_t sm = __ballot(is_shade(L.phase));
                go = __ballot(is_active(L.phase)) && __popcll(sm) < T;
            }
            if constexpr (kStash) {
                if (amask) {
                    __asm__ volatile("" ::: "memory");
                    cold_get<VAR>(s_cold, (int)threadIdx.x, L);
                }
            }
        } else if constexpr (MAP::kStepped) {
          if (amask) {
            // stepped map() (scenes with one Mandelbulb, MBStep): every pass runs one estimator
            // iteration for the lanes whose estimator is still running; once RMR_MB_FIN lanes have
            // finished theirs (or none is running), those lanes complete their map() (the other
            // primitives, the estimate and the fold: MAP::finish), apply it and begin their next one.
            // Same operations per lane as MAP::eval, so the same bits.
            if (is_active(L.phase) && mbs.i < 0) MAP::begin(P, RMR_MARCH_POINT(L), mbs);
            uint32_t lmaps = 0, liters = 0;
            for (;;) {
                if (is_active(L.phase) && !mbs.fin) mbs.fin = MAP::step(P, mbs);
                liters++;
                const uint64_t fm = __ballot(is_active(L.phase) && mbs.fin);
                const uint64_t rm = __ballot(is_active(L.phase) && !mbs.fin);
                if (fm && (!rm || __popcll(fm) >= RMR_MB_FIN)) {
#ifdef RMR_MB_STATS   // diagnostics: estimator iterations per finished map, march steps vs normal probes
                    {
                        const bool fin_l = is_active(L.phase) && mbs.fin;
                        const bool nrm_l = L.phase == PH_NORMAL;
                        uint32_t it_m = (fin_l && !nrm_l) ? (uint32_t)mbs.i : 0u, it_n = (fin_l && nrm_l) ? (uint32_t)mbs.i : 0u;
                        for (int o = 32; o > 0; o >>= 1) {
                            it_m += (uint32_t)__shfl_xor((int)it_m, o);
                            it_n += (uint32_t)__shfl_xor((int)it_n, o);
                        }
                        const uint64_t bm_ = __ballot(fin_l && !nrm_l), bn_ = __ballot(fin_l && nrm_l);
                        if (lane_now() == 0) {
                            atomicAdd(P.counters + 9, (unsigned long long)__popcll(bm_));
                            atomicAdd(P.counters + 10, (unsigned long long)it_m);
                            atomicAdd(P.counters + 12, (unsigned long long)__popcll(bn_));
                            atomicAdd(P.counters + 13, (unsigned long long)it_n);
                            atomicAdd(P.counters + 11, (unsigned long long)liters);   // passes up to this batch
                            atomicAdd(P.counters + 15, 1ull);                         // finishing batches
                        }
                        liters = 0;
                    }
#endif
                    if (is_active(L.phase) && mbs.fin) {
                        if constexpr (!MAP::kCounts)
                            RMR_COUNT(P.counters, active_lanes(), (uint64_t)P.flops_static, (uint64_t)P.transc_static);
                        const V2 m = MAP::finish(P, RMR_MARCH_POINT(L), mbs);
                        if (L.phase == PH_NORMAL) normal_update(L, m.x);
                        else march_update<HO>(P, L, m);
                        mbs.i = -1;
                        if (is_active(L.phase)) MAP::begin(P, RMR_MARCH_POINT(L), mbs);
                    }
                    lmaps += (uint32_t)__popcll(fm);
                    const uint64_t sm = __ballot(is_shade(L.phase));
                    const uint64_t am = __ballot(is_active(L.phase));
                    if (!am || __popcll(sm) >= T) break;
                }
            }
            maps += (WCount)__builtin_amdgcn_readfirstlane(lmaps);
            iters += (WCount)__builtin_amdgcn_readfirstlane(liters);
          }
        } else if (amask) {
            // map() steps back to back until a shading batch is due or no lane is active: idle lanes
            // only appear in shading and refill, so the refill / restart checks can wait until then
            uint64_t am = amask;
            // the loop's own counts (scalar registers; the wave counters were carried in VGPRs here)
            uint32_t lmaps = 0, liters = 0;
            for (;;) {
                if (is_active(L.phase)) {
                    const V3 p = RMR_MARCH_POINT(L);
                    if constexpr (!MAP::kCounts)   // every primitive of the fold (Mandelbulb iterations: inside)
                        RMR_COUNT(P.counters, active_lanes(), (uint64_t)P.flops_static, (uint64_t)P.transc_static);
                    if constexpr (MAP::kCert && HO) {
                        int w;
                        bool cert;
                        const V2 m = MAP::eval_c(P, p, w, cert);
                        if (L.phase == PH_NORMAL) normal_update(L, m.x);
                        else march_update<HO>(P, L, m, w, cert);
                    } else {
                        const V2 m = MAP::eval(P, p);
                        if (L.phase == PH_NORMAL) normal_update(L, m.x);
                        else march_update<HO>(P, L, m);
                    }
                }
                lmaps += (uint32_t)__popcll(am);
                liters++;
                const uint64_t sm = __ballot(is_shade(L.phase));
                am = __ballot(is_active(L.phase));
                if (!am || __popcll(sm) >= T) break;
            }
            maps += (WCount)__builtin_amdgcn_readfirstlane(lmaps);
            iters += (WCount)__builtin_amdgcn_readfirstlane(liters);
        }
        RMR_STAMP(c2);
        const uint64_t smask = __ballot(is_shade(L.phase));
        const uint64_t amask2 = __ballot(is_active(L.phase));
        if (smask && (__popcll(smask) >= T || amask2 == 0)) {
            shades++;
            shaded += (WCount)__popcll(smask);
            if constexpr (CERT) {   // the certified hits' getNormal probes, spread over the wave
                const bool mine = L.phase == PH_HIT && L.ctr < 0;
                const uint64_t cm = __ballot(mine);
                if (cm) cert_normals(P, L, mine, cm, s_tab[wv], RMR_DTAB);
                maps += (WCount)(6 * __popcll(cm));
                bmaps += (WCount)(6 * __popcll(cm));
#ifdef RMR_COUNT_FLOPS
                const uint64_t bm = __ballot(L.phase == PH_HIT && L.ctr < 0 &&
                                             (__float_as_int(((const float4*)(P.dprims + L.cw))[1].z) & 0xff) == RMR_PRIM_BOX);
                RMR_COUNT(P.counters, (uint64_t)__popcll(bm), 6 * (22 + 2), 6);
                RMR_COUNT(P.counters, (uint64_t)__popcll(cm & ~bm), 6 * (10 + 2), 6);
#endif
            }
            if (is_shade(L.phase)) {
                uint32_t ln = 0;
                if constexpr (kSeeds) {
                    ln = lane_now();
                    L.gxt = s_rng[0][wv][ln];
                    L.gyt = s_rng[1][wv][ln];
                    L.rc = s_rng[2][wv][ln];
                }
                if constexpr (HO) {   // the finished march's point (init_probe); the next march's e
                    L.o = vfma(L.d, L.t, L.o);
                    L.e = v3s(-0.0f);
                }
                shade<VAR, PROG, MATS, CERT>(P, L);
                if constexpr (kSeeds) s_rng[2][wv][ln] = L.rc;   // the chain continues at the next hit
            }
        }
        // finished samples have stored their radiance (finish_trace): the lane is free
        if (L.phase == PH_DONE) L.phase = PH_IDLE;
#ifdef RMR_PROFILE
        RMR_STAMP(c3);
        cyc[0] += c1 - c0;
        cyc[1] += c2 - c1;
        cyc[2] += c3 - c2;
#endif
        const uint64_t live = __ballot(L.phase != PH_IDLE);
        const bool last = live == 0 && exhausted;
        // (an inner loop adds at most 64 x its iterations to `maps`; a flush every 2^30 keeps every
        // 32-bit counter far from wrapping between two checks)
        if (last || ((maps | shaded) >> 30) != 0) {
            if (lane_now() == 0) {
                atomicAdd(P.counters + 0, (unsigned long long)maps);     // lane-level map() evaluations
                atomicAdd(P.counters + 1, (unsigned long long)iters);    // wave-level map() iterations
                atomicAdd(P.counters + 2, (unsigned long long)shades);   // wave-level shading batches
                if (MAP::kCache) atomicAdd(P.counters + 3, (unsigned long long)fulls);   // full map() batches
                atomicAdd(P.counters + 8, (unsigned long long)shaded);   // lane-level shading events
                // map() evaluations of the shading batches (certified getNormal probes; in [0] too)
                if (CERT) atomicAdd(P.counters + 14, (unsigned long long)bmaps);
            }
            maps = iters = shades = fulls = shaded = bmaps = 0;
        }
        if (last) break;
    }
#ifdef RMR_WAVE_TIMES
    if (lane_now() == 0) {
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
        atomicMax(P.counters + 12, ~tn);
        atomicMax(P.counters + 13, tn);
        if (t_exh) atomicAdd(P.counters + 15, tn - t_exh);
    }
#endif
    if (lane_now() == 0) {
#ifdef RMR_PROFILE
        atomicAdd(P.counters + 4, (unsigned long long)cyc[0]);
        atomicAdd(P.counters + 5, (unsigned long long)cyc[1]);
        atomicAdd(P.counters + 6, (unsigned long long)cyc[2]);
        if (MAP::kCache) {
            atomicAdd(P.counters + 9, (unsigned long long)cyc[3]);
            atomicAdd(P.counters + 10, (unsigned long long)full_lanes);
        }
        atomicAdd(P.counters + 11, (unsigned long long)cyc_claim);
        atomicAdd(P.counters + 12, (unsigned long long)cyc_rays);
        atomicAdd(P.counters + 7, (unsigned long long)(__builtin_amdgcn_s_memtime() - c_begin));
#endif
    }
}


// Running mean of main(), RM1:600-612: new = c/(n+1) + old*n/(n+1), sample order k = 0..nspp-1.
RMR_D void fold_main(const KParams& P) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    // the trace launch before this fold (same stream) is complete: zero its work-queue counters (every
    // one of the 64 the queue has room for) for the next launch (rmr_internal.h kQueueBytes)
    if (gid < (int)(kQueueBytes / (4 * kQueueWordStride))) ((uint32_t*)P.queue)[gid * kQueueWordStride] = 0u;
    const int tile = gid >> 6, lane = gid & 63;
    if (tile >= P.n_tiles) return;
    const TileXY txy = P.tiles[tile];
    const int px = txy.x + (lane & 7), py = txy.y + (lane >> 3);
    if (px < P.x0 || py < P.y0 || px >= P.x1 || py >= P.y1) return;
    float4* ap = P.accum + (size_t)py * P.W + px;
    float4 acc = *ap;
    const size_t plane = (size_t)P.n_tiles * 64;
    for (uint32_t k = 0; k < P.nspp; k++) {
        const float4 c = P.samp[(size_t)k * plane + (size_t)tile * 64 + lane];
        const uint32_t n = P.first_sample + k;
        if (n != 0u) {
            const float f1 = 1.0f / (float)(n + 1u);
            const float f2 = (float)n / (float)(n + 1u);
            acc.x = c.x * f1 + acc.x * f2;
            acc.y = c.y * f1 + acc.y * f2;
            acc.z = c.z * f1 + acc.z * f2;
        } else {
            acc.x = c.x; acc.y = c.y; acc.z = c.z;
        }
        acc.w = 1.0f;
    }
    *ap = acc;
}

}  // namespace rmr

