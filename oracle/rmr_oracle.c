/*
 * oracle/rmr_oracle.c — TEST INFRASTRUCTURE: CPU restatement of the reference hot path.
 *
 * This file is the checker for the HIP kernels and the CPU baseline of bench.py; it is never part
 * of the product path (librmr.so does not link it). Every function cites the reference GLSL it
 * restates ("RM1" = RayMarch.glsl, "RM2" = RayMarch2.glsl, "RM3" = RayMarch3.glsl, all under
 * /root/reference/RayMarch Renderer/). Float semantics follow oracle/detmath.h.
 *
 * Generated code is restated from the code generator that produces it: the v1 object/material
 * functions (Graphics.cpp:513-703, commented out in the reference but the only producer of RM1's
 * //#OBJINSERT / //#CASEINSERT bodies) and the v2 material function (Graphics.cpp:392-509,
 * 705-739). The scene arrives as rmr tables compiled by oracle/scene_compile.py.
 */
#include "rmr_oracle.h"
#include "detmath.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_F 3.14159274101257324219f /* float(3.1415926535897932384626433832795), RM2:3 */

/* ------------------------------------------------------------------------------------------ */
/* per-invocation state                                                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct lane {
    const oracle_job* job;
    const rmr_scene* sc;
    float max_dist, step_mult;
    int max_steps, max_bounces;
    float gxt, gyt;      /* float(gl_GlobalInvocationID.xy) + time                            */
    float time;
    float rc;            /* randChange, RM1:43                                               */
    o_v3 channels;       /* RM1:32                                                            */
    uint64_t maps;
} lane;

/* rand(co), RM1:44-57 (= RM2:50-63 = RM3:48-61) */
static float o_rand(lane* L, o_v2 co) {
    co.x = fmaf(L->gxt, L->rc, co.x);
    co.y = fmaf(L->gyt, L->rc, co.y);
    float dt = v_dot2(co, o2(12.9898f, 78.233f));
    float sn = f_mod(dt, 3.14f);
    L->rc = f_fract(det_sin(sn) * 43758.5453f);
    return L->rc;
}

/* ------------------------------------------------------------------------------------------ */
/* scene SDF                                                                                   */
/* ------------------------------------------------------------------------------------------ */
static o_v3 cvec(const rmr_scene* sc, int k) {
    const float* c = sc->consts + 3 * k;
    return o3(c[0], c[1], c[2]);
}

/* map_sphere RM1:170-174 (RM2/RM3:115-120 take a float radius = r.x) */
static float sd_sphere(o_v3 p, o_v3 c, float r) { return v_length(v_sub(p, c)) - r; }
/* map_box RM1:176-180 */
static float sd_box(o_v3 p, o_v3 c, o_v3 r) {
    o_v3 q = v_sub(v_abs(v_sub(p, c)), r);
    return fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f) + v_length(v_max0(q));
}
/* power 8 without transcendentals (csrc/rmr_trace.h mb_iter8, the same operations): cos/sin of
 * theta = acos(z.z/r) and phi = atan2(z.y, z.x) from the components, 8 theta / 8 phi by three angle
 * doublings, r^8 and r^7 by products */
static void mb_iter8(o_v3* z, float* dr, o_v3 p0, float r) {
    float ct = z->z / r;
    float st = sqrtf(fmaxf(fmaf(-ct, ct, 1.0f), 0.0f));
    const float rho2 = fmaf(z->x, z->x, z->y * z->y);
    float cp = 1.0f, sp = 0.0f;
    if (rho2 > 0.0f) {
        const float inv = 1.0f / sqrtf(rho2);
        cp = z->x * inv;
        sp = z->y * inv;
    }
    for (int k = 0; k < 3; k++) {
        const float st2 = (2.0f * st) * ct, ct2 = fmaf(ct, ct, -(st * st));
        const float sp2 = (2.0f * sp) * cp, cp2 = fmaf(cp, cp, -(sp * sp));
        st = st2; ct = ct2; sp = sp2; cp = cp2;
    }
    const float r2 = r * r, r4 = r2 * r2, r8 = r4 * r4, r7 = (r4 * r2) * r;
    *dr = fmaf(8.0f * r7, *dr, 1.0f);
    *z = v_fma(o3(st * cp, sp * st, ct), r8, p0);
}
/* power 8 as complex powers (csrc/rmr_trace.h mb_iter8_poly, the same operations): (z.z + i sqrt(a))^8
 * and (z.x + i z.y)^8 by two squarings each in a = x^2 + y^2, b = z^2; mb_iter8 near the z axis */
static void mb_iter8_poly(o_v3* z, float* dr, o_v3 p0, float r) {
    const float c = z->x * z->x, d = z->y * z->y, b = z->z * z->z;
    const float a = c + d;
    if (!(a >= 0x1p-30f)) {
        mb_iter8(z, dr, p0, r);
        return;
    }
    const float bma = b - a;
    const float ab4 = (4.0f * a) * b;
    const float re4 = fmaf(bma, bma, -ab4);
    const float re8 = fmaf(re4, re4, -((4.0f * ab4) * (bma * bma)));
    const float cmd = c - d;
    const float re4p = fmaf(cmd, cmd, -((4.0f * c) * d));
    const float im4p = ((4.0f * z->x) * z->y) * cmd;
    const float re8p = fmaf(re4p, re4p, -(im4p * im4p));
    const float im8p = (2.0f * re4p) * im4p;
    const float a2 = a * a;
    const float w = sqrtf(a) / (a2 * a2);
    const float t = (((8.0f * z->z) * bma) * re4) * w;
    const float r2 = r * r, r4 = r2 * r2, r7 = (r4 * r2) * r;
    *dr = fmaf(8.0f * r7, *dr, 1.0f);
    *z = v_add(o3(t * re8p, t * im8p, re8), p0);
}
#ifndef RMR_MB_POLY
#define RMR_MB_POLY 1
#endif
/* map_mandelbulb — new node: power-N bulb, distance 0.5*log(r)*r/dr */
static float sd_mandelbulb(o_v3 p, o_v3 c, o_v3 prm) {
    o_v3 p0 = v_sub(p, c);
    o_v3 z = p0;
    float power = prm.x, bail = prm.z;
    int iters = (int)prm.y;
    float dr = 1.0f, r = 0.0f;
    for (int i = 0; i < iters; i++) {
        r = v_length(z);
        if (r > bail) break;
        if (power == 8.0f) {
            if (RMR_MB_POLY) mb_iter8_poly(&z, &dr, p0, r);
            else mb_iter8(&z, &dr, p0, r);
            continue;
        }
        float theta = det_acos(z.z / r);
        float phi = det_atan2(z.y, z.x);
        dr = fmaf(det_pow(r, power - 1.0f) * power, dr, 1.0f);
        float zr = det_pow(r, power);
        theta = theta * power;
        phi = phi * power;
        float st = det_sin(theta);
        z = v_fma(o3(st * det_cos(phi), det_sin(phi) * st, det_cos(theta)), zr, p0);
    }
    return 0.5f * det_log(r) * r / dr;
}

static o_v3 opnd_obj(const rmr_scene* sc, const o_v3* vars, o_v3 p, int ref) {
    if (ref == RMR_OPND_P) return p;
    if (RMR_OPND_IS_CONST(ref)) return cvec(sc, RMR_OPND_CONST_INDEX(ref));
    return vars[ref];
}

/* obj_func_j(p, d): generated by Graphics.cpp:648-702 from the object's node list */
static float obj_program(const rmr_scene* sc, const rmr_prim* pr, o_v3 p) {
    o_v3 vars[RMR_MAX_VARS];
    for (int i = 0; i < RMR_MAX_VARS; i++) vars[i] = o3s(0.0f);
    for (int k = pr->prog_begin; k < pr->prog_end; k++) {
        const rmr_op* op = &sc->ops[k];
        o_v3 a = o3s(0), b = o3s(0), c = o3s(0), r = o3s(0);
        if (op->in[0] != RMR_OPND_NONE) a = opnd_obj(sc, vars, p, op->in[0]);
        if (op->in[1] != RMR_OPND_NONE) b = opnd_obj(sc, vars, p, op->in[1]);
        if (op->in[2] != RMR_OPND_NONE) c = opnd_obj(sc, vars, p, op->in[2]);
        switch (op->code) {
        case RMR_OP_GET_X: r = o3s(a.x); break;                         /* RM1:122-125 */
        case RMR_OP_GET_Y: r = o3s(a.y); break;                         /* RM1:127-130 */
        case RMR_OP_GET_Z: r = o3s(a.z); break;                         /* RM1:132-135 */
        case RMR_OP_ADD: r = v_add(a, b); break;                        /* RM1:138-141 */
        case RMR_OP_SUB: r = v_sub(a, b); break;                        /* RM1:143-146 */
        case RMR_OP_MUL: r = v_mul(a, b); break;                        /* RM1:148-151 */
        case RMR_OP_DIV: r = v_div(a, b); break;                        /* RM1:154-157 */
        case RMR_OP_SIN: r = o3(det_sin(a.x), det_sin(a.y), det_sin(a.z)); break; /* RM1:159 */
        case RMR_OP_COS: r = o3(det_cos(a.x), det_cos(a.y), det_cos(a.z)); break; /* RM1:164 */
        case RMR_OP_MAP_SPHERE: r = o3s(sd_sphere(a, b, c.x)); break;   /* RM1:170-174 */
        case RMR_OP_MAP_BOX: r = o3s(sd_box(a, b, c)); break;           /* RM1:176-180 */
        case RMR_OP_UNION: r = v_min(a, b); break;                      /* RM1:183-186 */
        case RMR_OP_SUBTRACT: r = v_max(a, v_neg(b)); break;            /* RM1:188-191 */
        case RMR_OP_INTERSECT: r = v_max(a, b); break;                  /* RM1:193-196 */
        case RMR_OP_DOMAIN_REPEAT:                                      /* RM1:199-215 */
            r = a;
            if (b.x != 0.0f) r.x = f_mod(a.x, b.x) - b.x * 0.5f;
            if (b.y != 0.0f) r.y = f_mod(a.y, b.y) - b.y * 0.5f;
            if (b.z != 0.0f) r.z = f_mod(a.z, b.z) - b.z * 0.5f;
            break;
        case RMR_OP_MAP_MANDELBULB: r = o3s(sd_mandelbulb(a, b, c)); break;
        default: break;
        }
        vars[op->out[0]] = r;
    }
    return vars[pr->dist_var].x;
}

static float prim_dist(const rmr_scene* sc, const rmr_prim* pr, o_v3 p) {
    switch (pr->type) {
    case RMR_PRIM_SPHERE: return sd_sphere(p, o3(pr->c[0], pr->c[1], pr->c[2]), pr->r[0]);
    case RMR_PRIM_BOX: return sd_box(p, o3(pr->c[0], pr->c[1], pr->c[2]), o3(pr->r[0], pr->r[1], pr->r[2]));
    case RMR_PRIM_MANDELBULB:
        return sd_mandelbulb(p, o3(pr->c[0], pr->c[1], pr->c[2]), o3(pr->r[0], pr->r[1], pr->r[2]));
    default: return obj_program(sc, pr, p);
    }
}

/* map(p), RM1:224-231 with the //#OBJINSERT body of Graphics.cpp:107-112:
 *   d = vec2(maxDist,-1); for j: d = opU(d, vec2(dj.x, matID_j)); opU = a.x < b.x ? a : b
 * NaN distances (a ray direction that normalize(vec3(0)) made NaN after total internal reflection):
 * the reference as compiled by Mesa llvmpipe evaluates opU per component — distance min(a.x, b.x)
 * ignoring a NaN operand, id (a.x < b.x ? a.y : b.y) (probed: tests/golden/kat_nan.npz). So a NaN
 * object never becomes the distance but does take the id. Identical to the plain select for every
 * non-NaN input, signed zeros included; d.x can never become NaN (it starts at maxDist). */
static o_v2 o_map(const rmr_scene* sc, float max_dist, o_v3 p) {
    o_v2 d = o2(max_dist, -1.0f);
    for (int j = 0; j < sc->n_prims; j++) {
        float dj = prim_dist(sc, &sc->prims[j], p);
        if (!(d.x < dj)) d.y = sc->prims[j].mat_id;
        if (d.x >= dj) d.x = dj;
    }
    return d;
}
static o_v2 L_map(lane* L, o_v3 p) { L->maps++; return o_map(L->sc, L->max_dist, p); }

/* march(origin, dir, distMult), RM1:233-257 = RM2:174-198 = RM3:145-169 */
static o_v2 o_march(lane* L, o_v3 o, o_v3 d, float dist_mult) {
    float t = 0.0f;
    for (int i = 0; i < L->max_steps; i++) {
        o_v2 m = L_map(L, v_fma(d, t, o));
        m.x = m.x * dist_mult;
        if (m.x < 0.001f) { m.x = t; return m; }
        if (t >= L->max_dist) return o2(L->max_dist, -1.0f);
        t = fmaf(m.x, L->step_mult, t);
    }
    return o2(L->max_dist, -1.0f);
}

/* getNormal(p), RM1:259-268 (= RM2:200-209 = RM3:171-180) */
static o_v3 o_normal(lane* L, o_v3 p) {
    const float h = 0.001f;
    o_v3 n;
    n.x = L_map(L, o3(p.x + h, p.y + 0.0f, p.z + 0.0f)).x - L_map(L, o3(p.x - h, p.y - 0.0f, p.z - 0.0f)).x;
    n.y = L_map(L, o3(p.x + 0.0f, p.y + h, p.z + 0.0f)).x - L_map(L, o3(p.x - 0.0f, p.y - h, p.z - 0.0f)).x;
    n.z = L_map(L, o3(p.x + 0.0f, p.y + 0.0f, p.z + h)).x - L_map(L, o3(p.x - 0.0f, p.y - 0.0f, p.z - h)).x;
    return v_normalize(n);
}

/* randHemisphere(s1, s2, normal), RM1:270-304 */
/* RMR_HEMI_ALGEBRAIC (default, csrc/rmr_trace.h hemisphere): cos(acos(u)) = u and
 * sin(acos(u)) = sqrt(1 - u^2) >= 0 taken algebraically instead of through det_acos / det_sin / det_cos:
 * the same direction, rounded differently (pinned by the distribution and PSNR tests) */
#ifndef RMR_HEMI_ALGEBRAIC
#define RMR_HEMI_ALGEBRAIC 1
#endif
static o_v3 o_hemisphere(lane* L, o_v2 s1, o_v2 s2, o_v3 n) {
    float theta = 6.28318548202514648438f * o_rand(L, s1); /* 2 * 3.141592653 */
    float sp, cp;
    if (RMR_HEMI_ALGEBRAIC) {
        const float u = 2.0f * o_rand(L, s2) - 1.0f;
        cp = u;
        sp = sqrtf(fmaxf(fmaf(-u, u, 1.0f), 0.0f));
    } else {
        float phi = det_acos(2.0f * o_rand(L, s2) - 1.0f);
        sp = det_sin(phi);
        cp = det_cos(phi);
    }
    o_v3 b = v_normalize(o3(sp * det_cos(theta), cp, sp * det_sin(theta)));
    if (!v_is_zero(n)) {
        if (b.z < 0.0f) b = v_neg(b);
        o_v3 lx;
        if (v_eq(n, o3(0.0f, 1.0f, 0.0f))) lx = v_normalize(v_cross(n, o3(0.0f, 0.0f, 1.0f)));
        else lx = v_normalize(v_cross(n, o3(0.0f, 1.0f, 0.0f)));
        o_v3 ly = v_normalize(v_cross(n, lx));
        b = m_mul(lx, ly, n, b);
    }
    return b;
}

/* grayscale RM1:306-309 (channel-normalised) */
static float gray1(const lane* L, o_v3 c) {
    return (c.x + c.y + c.z) / (L->channels.x + L->channels.y + L->channels.z);
}

/* ------------------------------------------------------------------------------------------ */
/* RM1: node-graph materials                                                                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct ray_data { o_v3 origin, hit, dir; float t; int inside; } ray_data; /* RM1:34-41 */

static o_v3 opnd_mat(const rmr_scene* sc, const o_v3* vars, int ref) {
    if (RMR_OPND_IS_CONST(ref)) return cvec(sc, RMR_OPND_CONST_INDEX(ref));
    if (ref >= 0) return vars[ref];
    return o3s(0.0f);
}

/* mat_func_j(ray, outColor, outDir, outInside, outHit), Graphics.cpp:515-645. getNormal(ray.hit)
 * is a pure function of ray.hit, so the value is computed once per hit and reused. */
static void mat_v1(lane* L, const rmr_material* m, const ray_data* ray, o_v3 N,
                   o_v3* out_color, o_v3* out_dir, o_v3* out_inside, o_v3* out_hit) {
    const rmr_scene* sc = L->sc;
    o_v3 vars[RMR_MAX_VARS];
    for (int i = 0; i < RMR_MAX_VARS; i++) vars[i] = o3s(0.0f);
    const o_v3 ch = L->channels;
    for (int k = m->prog_begin; k < m->prog_end; k++) {
        const rmr_op* op = &sc->ops[k];
        o_v3 in[7];
        for (int i = 0; i < 7; i++) in[i] = (op->in[i] == RMR_OPND_NONE) ? o3s(0.0f) : opnd_mat(sc, vars, op->in[i]);
        o_v3 o0 = o3s(0), o1 = o3s(0), o2v = o3s(0), o3v = o3s(0);
        switch (op->code) {
        case RMR_OP_M_FACING: { /* RM1:314-317 */
            float sg = (float)(ray->inside * 2 - 1);
            o0 = o3s(f_clamp(v_dot(v_scale(ray->dir, sg), N), 0.0f, 1.0f));
            break;
        }
        case RMR_OP_M_INSIDE: o0 = o3s((float)ray->inside); break;          /* RM1:319-322 */
        case RMR_OP_M_ADD: o0 = v_add(in[0], in[1]); break;                 /* RM1:325-328 */
        case RMR_OP_M_SUB: o0 = v_sub(in[0], in[1]); break;
        case RMR_OP_M_MUL: o0 = v_mul(in[0], in[1]); break;
        case RMR_OP_M_DIV: o0 = v_div(in[0], in[1]); break;
        case RMR_OP_M_MIX: { /* RM1:346-376 */
            float r = o_rand(L, o2(ray->origin.z, ray->origin.x));
            float f = f_clamp(gray1(L, v_mul(in[6], ch)), 0.0f, 1.0f);
            int second = r < f;
            if (f == 0.0f) second = 0;
            else if (f == 1.0f) second = 1;
            o0 = second ? in[3] : in[0];
            o1 = second ? in[4] : in[1];
            o2v = second ? in[5] : in[2];
            break;
        }
        case RMR_OP_M_DIFFUSE: /* RM1:378-387 */
            o0 = in[0];
            o1 = o_hemisphere(L, o2(ray->hit.x, ray->hit.y), o2(ray->hit.z, ray->hit.x), N);
            break;
        case RMR_OP_M_GLOSSY: { /* RM1:389-398 */
            o0 = in[0];
            o_v3 hd = o_hemisphere(L, o2(ray->hit.y, ray->hit.x), o2(ray->hit.x, ray->hit.z), N);
            float sg = -(float)(ray->inside * 2 - 1);
            o_v3 rf = v_reflect(ray->dir, v_scale(N, sg));
            o1 = v_mix(hd, rf, 1.0f - gray1(L, v_mul(in[1], ch)));
            break;
        }
        case RMR_OP_M_REFRACTION: /* RM1:400-427 */
            o0 = ray->inside ? in[0] : o3s(1.0f);
            if (!ray->inside) {
                o1 = v_normalize(v_refract(ray->dir, N, 1.0f / gray1(L, v_mul(in[1], ch))));
                o2v = o3s(1.0f);
            } else {
                o_v3 rdir = v_normalize(v_refract(ray->dir, v_neg(N), gray1(L, v_mul(in[1], ch))));
                o_v3 ddir = o_hemisphere(L, o2(ray->hit.z, ray->hit.y), o2(ray->hit.y, ray->hit.z), N);
                o1 = v_mix(ddir, rdir, 1.0f - gray1(L, v_mul(in[2], ch)));
                o2v = o3s(0.0f);
            }
            break;
        case RMR_OP_M_VOLUME: /* RM1:429-474 */
            if (ray->inside) {
                float t = ray->t;
                float den = gray1(L, v_mul(in[1], ch)) / 20.0f;
                int npts = (int)floorf(t * 100.0f);
                o_v3 hp = o3s(0.0f);
                for (int i = 0; i < npts; i++) {
                    float r = o_rand(L, o2(ray->hit.x, ray->hit.y));
                    if (r < den) {
                        r = o_rand(L, o2(ray->hit.z, ray->hit.y)) * t;
                        hp = v_fma(ray->dir, r, ray->origin);
                        break;
                    }
                }
                if (!v_is_zero(hp)) {
                    o0 = in[0];
                    o1 = o_hemisphere(L, o2(hp.x, hp.y), o2(hp.z, hp.y), o3s(0.0f));
                    o2v = o3s(1.0f);
                    o3v = hp;
                } else {
                    o0 = o3s(1.0f); o1 = ray->dir; o2v = o3s(0.0f); o3v = o3s(0.0f);
                }
            } else {
                o0 = o3s(1.0f); o1 = ray->dir; o2v = o3s(1.0f); o3v = o3s(0.0f);
            }
            break;
        case RMR_OP_M_EMISSION: /* RM1:476-479 */
            o0 = v_scale(in[0], gray1(L, v_mul(in[1], ch)));
            break;
        default: break;
        }
        if (op->out[0] >= 0) vars[op->out[0]] = o0;
        if (op->out[1] >= 0) vars[op->out[1]] = o1;
        if (op->out[2] >= 0) vars[op->out[2]] = o2v;
        if (op->out[3] >= 0) vars[op->out[3]] = o3v;
    }
    if (m->color_var >= 0) *out_color = vars[m->color_var];
    if (m->dir_var >= 0) *out_dir = vars[m->dir_var];
    if (m->inside_var >= 0) *out_inside = vars[m->inside_var];
    if (m->hit_var >= 0) *out_hit = vars[m->hit_var];
}

/* skyColor(dir), RM1:78-113 = RM2:84-107. With useEnvTex: equirectangular lookup
 * uv = (atan(z, x) / 2pi wrapped to [0,1), 1 - (y/2 + 1/2)) and texture2D on envTex, restated as
 * GL's bilinear filter (GL 4.5 §8.14.2) at level 0 (compute shaders have no derivatives) with
 * CLAMP_TO_EDGE; the filter arithmetic below is rmr's definition (the driver's filter precision is
 * implementation-defined, so parity with the reference there is statistical). */
static o_v3 sky_color(const lane* L, o_v3 dir) {
    const oracle_job* job = L->job;
    const rmr_scene* sc = L->sc;
    if (!job->params.use_env_tex || !job->env) return o3(sc->sky[0], sc->sky[1], sc->sky[2]);
    const float PI = 3.141592653f;
    float phi = det_atan2(dir.z, dir.x);
    if (phi < 0.0f) phi += 2.0f * PI;
    const float s = phi / (2.0f * PI);
    const float t = 1.0f - (dir.y * 0.5f + 0.5f);
    const int W = job->env_w, H = job->env_h;
    const float fu = s * (float)W - 0.5f, fv = t * (float)H - 0.5f;
    const float i0f = floorf(fu), j0f = floorf(fv);
    const float a = fu - i0f, b = fv - j0f;
    /* CLAMP_TO_EDGE (fmaxf/fminf also send NaN coordinates to texel 0) */
    const int i0 = (int)fminf(fmaxf(i0f, 0.0f), (float)(W - 1)), i1 = (int)fminf(fmaxf(i0f + 1.0f, 0.0f), (float)(W - 1));
    const int j0 = (int)fminf(fmaxf(j0f, 0.0f), (float)(H - 1)), j1 = (int)fminf(fmaxf(j0f + 1.0f, 0.0f), (float)(H - 1));
    const float* T = job->env;
    o_v3 c;
    float* cc = &c.x;
    for (int k = 0; k < 3; k++) {
        const float t00 = T[4 * ((size_t)j0 * W + i0) + k], t10 = T[4 * ((size_t)j0 * W + i1) + k];
        const float t01 = T[4 * ((size_t)j1 * W + i0) + k], t11 = T[4 * ((size_t)j1 * W + i1) + k];
        const float top = t00 * (1.0f - a) + t10 * a, bot = t01 * (1.0f - a) + t11 * a;
        cc[k] = top * (1.0f - b) + bot * b;
    }
    return c;
}

/* trace, RM1:483-565 */
static o_v3 trace_rm1(lane* L, o_v3 origin, o_v3 dir) {
    const rmr_scene* sc = L->sc;
    o_v3 color = L->channels;
    o_v3 o = origin, d = dir;
    int inside = 0;
    int bounces = 0;
    while (bounces < L->max_bounces) {
        bounces++;
        o_v2 v = o_march(L, o, d, inside ? -1.0f : 1.0f);
        ray_data ray;
        ray.origin = o; ray.dir = d; ray.t = v.x; ray.hit = v_fma(d, v.x, o); ray.inside = inside;
        if (ray.t < L->max_dist) {
            o_v3 nc = o3s(0), nd = o3s(0), ni = o3s(0), nh = o3s(0);
            o_v3 N = o_normal(L, ray.hit);
            int id = (int)v.y;
            if (id >= 0 && id < sc->n_materials && sc->materials[id].defined)
                mat_v1(L, &sc->materials[id], &ray, N, &nc, &nd, &ni, &nh);
            color = v_mul(color, nc);
            inside = ni.x != 0.0f;
            if (v_is_zero(nd)) break;
            d = nd;
            if (v_is_zero(nh)) o = inside ? v_fma(N, -0.002f, ray.hit) : v_fma(N, 0.003f, ray.hit);
            else o = nh;
        } else {
            /* shader_emission(ray, skyColor(dir), vec3(1), emit) */
            o_v3 emit = v_scale(sky_color(L, ray.dir), gray1(L, v_mul(o3s(1.0f), L->channels)));
            color = v_mul(color, emit);
            break;
        }
    }
    return color;
}

/* ------------------------------------------------------------------------------------------ */
/* RM2: NEE path tracer with a v2 node material                                               */
/* ------------------------------------------------------------------------------------------ */
typedef struct point_data { o_v3 pos, dir, normal, tb, tn, tt; } point_data; /* RM2:33-39 */

/* makeTBN(p) RM2:211-229 given N = getNormal(p) */
static void make_tbn(o_v3 N, o_v3* c0, o_v3* c1, o_v3* c2) {
    o_v3 tangent = (N.x == 0.0f) ? o3(1.0f, 0.0f, 0.0f) : v_normalize(v_cross(o3(0.0f, 1.0f, 0.0f), N));
    o_v3 bitangent = v_normalize(v_cross(tangent, N));
    *c0 = bitangent; *c1 = N; *c2 = tangent;
}
/* material_diffuse.samplePDF RM2:279-290 */
static o_v3 diffuse_sample(lane* L) {
    float sin2 = o_rand(L, o2(L->time, L->time));
    float cos2 = 1.0f - sin2;
    float st = sqrtf(sin2), ct = sqrtf(cos2);
    float o = (o_rand(L, o2(L->time, L->time)) * 2.0f) * PI_F;
    return v_normalize(o3(st * det_cos(o), ct, st * det_sin(o)));
}
/* material_glossy.samplePDF RM2:326-342 */
static o_v3 glossy_sample(lane* L, o_v3 wo, o_v3 n, float rough) {
    if (rough == 0.0f) return v_reflect(wo, n);
    float o = (o_rand(L, o2(L->time, L->time)) * 2.0f) * PI_F;
    float a = f_pow2(rough);
    float r = o_rand(L, o2(L->time, L->time));
    float th = det_acos(sqrtf((1.0f - r) / ((a * a - 1.0f) * r + 1.0f)));
    float s = det_sin(th);
    return v_normalize(o3(s * det_cos(o), det_cos(th), s * det_sin(o)));
}

/* generated mat_func_<id>(point, color, matData), Graphics.cpp:705-739 + compileNode 412-463 */
static void mat_v2(lane* L, const point_data* pt, o_v3 color, o_v3* mat_color, o_v3* new_dir, int* will_break) {
    const rmr_scene* sc = L->sc;
    o_v3 slot[RMR_MAX_VARS];
    for (int i = 0; i < RMR_MAX_VARS; i++) slot[i] = o3s(0.0f);
    for (int k = sc->v2_prog_begin; k < sc->v2_prog_end; k++) {
        const rmr_op* op = &sc->ops[k];
        switch (op->code) {
        case RMR_OP_V2_DIFFUSE:
            slot[op->out[0]] = m_mul(pt->tb, pt->tn, pt->tt, diffuse_sample(L));
            slot[op->out[1]] = cvec(sc, RMR_OPND_CONST_INDEX(op->in[0]));
            break;
        case RMR_OP_V2_GLOSSY: {
            float rough = cvec(sc, RMR_OPND_CONST_INDEX(op->in[1])).x;
            slot[op->out[0]] = m_mul(pt->tb, pt->tn, pt->tt, glossy_sample(L, pt->dir, pt->normal, rough));
            slot[op->out[1]] = cvec(sc, RMR_OPND_CONST_INDEX(op->in[0]));
            break;
        }
        case RMR_OP_V2_FRESNEL: /* Graphics.cpp:461 */
            slot[op->out[0]] = o3s(f_pow5(1.0f - f_clamp(v_dot(pt->normal, pt->dir), 0.0f, 1.0f)) * 0.96f + 0.04f);
            break;
        case RMR_OP_V2_MIX: { /* Graphics.cpp:447-457 */
            float r = o_rand(L, o2(pt->pos.x, pt->pos.z));
            int second = r <= slot[op->in[4]].x;
            o_v3 dsel = second ? slot[op->in[2]] : slot[op->in[0]];
            o_v3 rsel = second ? slot[op->in[3]] : slot[op->in[1]];
            slot[op->out[0]] = dsel;
            slot[op->out[1]] = rsel;
            break;
        }
        default: break;
        }
    }
    o_v3 refl = slot[1];
    *new_dir = slot[0];
    float prob = fmaxf(refl.x, fmaxf(refl.y, refl.z));
    *mat_color = color;
    if (o_rand(L, o2(pt->pos.z, pt->pos.x)) <= 1.0f) {
        *mat_color = v_mul(*mat_color, v_div(refl, o3s(prob)));
        *will_break = 0;
    } else {
        *will_break = 1;
    }
}

/* trace, RM2:420-520 */
static o_v3 trace_rm2(lane* L, o_v3 origin, o_v3 dir) {
    const rmr_scene* sc = L->sc;
    const rmr_rm2_consts* k = sc->rm2;
    o_v3 final_color = o3s(0.0f);
    o_v3 color = o3s(1.0f);
    o_v3 o = origin, d = dir;
    int bounces = 0;
    while (bounces < L->max_bounces) {
        bounces++;
        o_v2 v = o_march(L, o, d, 1.0f);
        if (v.x < L->max_dist) {
            point_data pt;
            pt.pos = v_fma(d, v.x, o);
            pt.dir = v_neg(d);
            pt.normal = o_normal(L, pt.pos);
            make_tbn(pt.normal, &pt.tb, &pt.tn, &pt.tt);
            int id = (int)v.y;
            o_v3 mc = o3s(0.0f);
            if (id >= 0 && id < RMR_MAX_MATERIALS) mc = o3(k->albedo[id][0], k->albedo[id][1], k->albedo[id][2]);
            o_v3 lp = o3(k->light_pos[0], k->light_pos[1], k->light_pos[2]);
            o_v3 ld = v_normalize(v_sub(lp, pt.pos));
            o_v3 nd;
            if (id == k->node_mat_id) {
                o_v3 matc; int wb;
                mat_v2(L, &pt, color, &matc, &nd, &wb);
                color = v_mul(color, matc);
                if (wb) { color = o3s(0.0f); break; }
            } else {
                o_v2 sd = o_march(L, v_fma(pt.normal, 0.002f, pt.pos), ld, 1.0f);
                float len = v_length(v_sub(lp, pt.pos));
                if (sd.x >= len) {
                    o_v3 brdf = o3(mc.x / PI_F, mc.y / PI_F, mc.z / PI_F); /* color / PI, RM2:276 */
                    o_v3 c = v_mul(color, brdf);
                    c = v_scale(c, f_clamp(v_dot(ld, pt.normal), 0.0f, 1.0f));
                    c = v_scale(c, k->light_power / f_pow2(len));
                    final_color = v_add(final_color, c);
                }
                nd = m_mul(pt.tb, pt.tn, pt.tt, diffuse_sample(L));
                o_v3 refl = mc;
                float prob = fmaxf(refl.x, fmaxf(refl.y, refl.z));
                if (o_rand(L, o2(pt.pos.z, pt.pos.x)) <= prob) color = v_mul(color, v_div(refl, o3s(prob)));
                else { color = o3s(0.0f); break; }
            }
            o = v_fma(pt.normal, 0.002f, pt.pos);
            d = nd;
        } else {
            color = v_mul(color, sky_color(L, d));   /* RM2:509 */
            break;
        }
    }
    if (bounces != L->max_bounces) final_color = v_add(final_color, color);
    return final_color;
}

/* ------------------------------------------------------------------------------------------ */
/* RM3: spectral hero wavelength                                                              */
/* ------------------------------------------------------------------------------------------ */
/* mat_func_k body, RM3:251-345 (and the sky block 408-438). returns 1 = willBreak */
static int spectral_event(lane* L, const rmr_spectral* m, o_v2 seed, uint32_t* color, float* power) {
    if (*color == 0u) {
        float r = o_rand(L, seed);
        r = r * (float)((m->max_wave - m->min_wave) / 5u);
        r = floorf(r) * 5.0f;
        *color = (uint32_t)(int)r + m->min_wave;
        *power = *power * m->power;
        return 0;
    }
    if (*color < m->min_wave || *color > m->max_wave) { *color = 0u; return 1; }
    *power = *power * m->power;
    return 0;
}

/* trace, RM3:347-444 */
static uint32_t trace_rm3(lane* L, o_v3 origin, o_v3 dir, float* light_power) {
    const rmr_scene* sc = L->sc;
    uint32_t color = 0u;
    float power = 1.0f;
    o_v3 o = origin, d = dir;
    int bounces = 0;
    while (bounces < L->max_bounces) {
        bounces++;
        o_v2 v = o_march(L, o, d, 1.0f);
        o_v3 pos = v_fma(d, v.x, o);
        if (v.x < L->max_dist) {
            /* getNormal/makeTBN of RM3:365-366 are only consumed on this branch */
            o_v3 N = o_normal(L, pos);
            int id = (int)v.y;
            o_v3 nd = o3s(0.0f);
            if (id >= 0 && id < sc->n_materials && sc->spectral[id].defined) {
                const rmr_spectral* m = &sc->spectral[id];
                if (spectral_event(L, m, o2(pos.y, pos.x), &color, &power)) break;
                if (m->terminates) break;
                nd = o_hemisphere(L, o2(pos.x, pos.y), o2(pos.z, pos.y), N);
            }
            o = v_fma(N, 0.002f, pos);
            d = nd;
        } else {
            spectral_event(L, &sc->spectral_sky, o2(pos.y, pos.x), &color, &power);
            break;
        }
    }
    *light_power = power;
    return color;
}

/* wavelengthToColor, RM3:447-522 */
static o_v3 wl2rgb(uint32_t wavelength) {
    float wl = (float)wavelength;
    float R, G, B, alpha;
    if (wl >= 380.0f && wl < 440.0f) { R = (-1.0f * (wl - 440.0f)) / 60.0f; G = 0.0f; B = 1.0f; }
    else if (wl >= 440.0f && wl < 490.0f) { R = 0.0f; G = (wl - 440.0f) / 50.0f; B = 1.0f; }
    else if (wl >= 490.0f && wl < 510.0f) { R = 0.0f; G = 1.0f; B = (-1.0f * (wl - 510.0f)) / 20.0f; }
    else if (wl >= 510.0f && wl < 580.0f) { R = (wl - 510.0f) / 70.0f; G = 1.0f; B = 0.0f; }
    else if (wl >= 580.0f && wl < 645.0f) { R = 1.0f; G = (-1.0f * (wl - 645.0f)) / 65.0f; B = 0.0f; }
    else if (wl >= 645.0f && wl <= 780.0f) { R = 1.0f; G = 0.0f; B = 0.0f; }
    else { R = 0.0f; G = 0.0f; B = 0.0f; }
    if (wl > 780.0f || wl < 380.0f) alpha = 0.0f;
    else if (wl > 700.0f) alpha = (780.0f - wl) / 80.0f;
    else if (wl < 420.0f) alpha = (wl - 380.0f) / 40.0f;
    else alpha = 1.0f;
    return v_scale(o3(R, G, B), alpha);
}

/* ------------------------------------------------------------------------------------------ */
/* main(): jittered corner-ray interpolation + trace, RM1:567-598 / RM2:522-553 / RM3:524-540   */
/* ------------------------------------------------------------------------------------------ */
static void lane_init(lane* L, const oracle_job* job, int px, int py, float time) {
    L->job = job;
    L->sc = job->scene;
    L->max_dist = job->params.max_dist;
    L->step_mult = job->params.step_multiply;
    L->max_steps = job->params.max_steps;
    L->max_bounces = job->params.max_bounces;
    L->time = time;
    L->gxt = (float)px + time;
    L->gyt = (float)py + time;
    L->rc = 0.0f;
    L->channels = o3s(1.0f);
    L->maps = 0;
}

static o_v3 sample_rgb(lane* L, int px, int py) {
    const oracle_job* job = L->job;
    const float* V = job->view;
    o_v3 eye = o3(V[0], V[1], V[2]);
    o_v3 r00 = o3(V[3], V[4], V[5]), r01 = o3(V[6], V[7], V[8]);
    o_v3 r10 = o3(V[9], V[10], V[11]), r11 = o3(V[12], V[13], V[14]);
    float W = (float)job->W, H = (float)job->H;
    float posx = (float)px / W, posy = (float)py / H;
    float t = L->time;
    float j1 = o_rand(L, o2((float)px + t, (float)py + t));
    float j2 = o_rand(L, o2((float)px + t, (float)py + t));
    float j3 = o_rand(L, o2((float)py + t, (float)px + t));
    o_v3 top = v_mix(r00, r01, posx + j1 / W);
    o_v3 bot = v_mix(r10, r11, posx + j2 / W);
    o_v3 dir = v_normalize(v_mix(top, bot, posy + j3 / H));
    int variant = job->scene->variant;
    if (variant == RMR_VARIANT_RM3) {
        float power;
        uint32_t range = trace_rm3(L, eye, dir, &power);
        return v_scale(wl2rgb(range), power);
    }
    o_v3 (*tr)(lane*, o_v3, o_v3) = (variant == RMR_VARIANT_RM2) ? trace_rm2 : trace_rm1;
    if (job->params.separate_channels == 0) {
        L->channels = o3s(1.0f);
        return tr(L, eye, dir);
    }
    L->channels = o3(1.0f, 0.0f, 0.0f);
    o_v3 r = tr(L, eye, dir);
    L->channels = o3(0.0f, 1.0f, 0.0f);
    o_v3 g = tr(L, eye, dir);
    L->channels = o3(0.0f, 0.0f, 1.0f);
    o_v3 b = tr(L, eye, dir);
    return v_add(v_add(r, g), b);
}

void oracle_sample(const oracle_job* job, int px, int py, float time, float out[3], uint64_t* map_evals) {
    lane L;
    lane_init(&L, job, px, py, time);
    o_v3 c = sample_rgb(&L, px, py);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
    if (map_evals) *map_evals += L.maps;
}

/* running mean of main(), RM1:600-612 */
static void fold(float* acc, const float c[3], uint32_t n) {
    if (n != 0u) {
        float f1 = 1.0f / (float)(n + 1u);
        float f2 = (float)n / (float)(n + 1u);
        for (int i = 0; i < 3; i++) acc[i] = c[i] * f1 + acc[i] * f2;
    } else {
        for (int i = 0; i < 3; i++) acc[i] = c[i];
    }
    acc[3] = 1.0f;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

void oracle_render(const oracle_job* job, const float* times, int x0, int y0, int x1, int y1,
                   uint32_t first_sample, uint32_t nspp, float* accum, int nthreads, uint64_t* map_evals) {
    x0 = clampi(x0, 0, job->W); x1 = clampi(x1, 0, job->W);
    y0 = clampi(y0, 0, job->H); y1 = clampi(y1, 0, job->H);
    int w = x1 - x0, h = y1 - y0;
    if (w <= 0 || h <= 0 || nspp == 0) return;
    long npix = (long)w * h;
    uint64_t total = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
#endif
    for (long i = 0; i < npix; i++) {
        int px = x0 + (int)(i % w), py = y0 + (int)(i / w);
        float* acc = accum + 4 * ((long)py * job->W + px);
        for (uint32_t k = 0; k < nspp; k++) {
            lane L;
            lane_init(&L, job, px, py, times[k]);
            o_v3 c = sample_rgb(&L, px, py);
            float cc[3] = {c.x, c.y, c.z};
            fold(acc, cc, first_sample + k);
            total += L.maps;
        }
    }
    if (map_evals) *map_evals += total;
}

void oracle_trace_samples(const oracle_job* job, const float* times, int x0, int y0, int x1, int y1,
                          uint32_t nspp, float* out, int nthreads, uint64_t* map_evals) {
    int w = x1 - x0, h = y1 - y0;
    if (w <= 0 || h <= 0 || nspp == 0) return;
    long npix = (long)w * h;
    uint64_t total = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : total)
#endif
    for (long i = 0; i < npix * (long)nspp; i++) {
        long k = i / npix, pi = i % npix;
        int px = x0 + (int)(pi % w), py = y0 + (int)(pi / w);
        lane L;
        lane_init(&L, job, px, py, times[k]);
        o_v3 c = sample_rgb(&L, px, py);
        float* o = out + 4 * i;
        o[0] = c.x; o[1] = c.y; o[2] = c.z; o[3] = 1.0f;
        total += L.maps;
    }
    if (map_evals) *map_evals += total;
}

/* ---- KAT hooks ---- */
float oracle_det_sin(float x) { return det_sin(x); }
float oracle_det_cos(float x) { return det_cos(x); }
float oracle_det_acos(float x) { return det_acos(x); }
float oracle_det_log(float x) { return det_log(x); }
float oracle_det_exp(float x) { return det_exp(x); }
float oracle_det_atan2(float y, float x) { return det_atan2(y, x); }

void oracle_map(const rmr_scene* sc, float max_dist, const float p[3], float out[2]) {
    o_v2 d = o_map(sc, max_dist, o3(p[0], p[1], p[2]));
    out[0] = d.x; out[1] = d.y;
}
static void kat_lane(lane* L, const rmr_scene* sc, const rmr_params* prm) {
    memset(L, 0, sizeof(*L));
    L->sc = sc;
    L->max_dist = prm ? prm->max_dist : 1000.0f;
    L->step_mult = prm ? prm->step_multiply : 0.5f;
    L->max_steps = prm ? prm->max_steps : 512;
    L->max_bounces = prm ? prm->max_bounces : 16;
    L->channels = o3s(1.0f);
}
/* trace(o, d) of RM1/RM2 for the invocation at gid (gx, gy) with seed `time`, channels = 1 */
void oracle_trace(const oracle_job* job, int gx, int gy, float time, const float o[3], const float d[3],
                  float out[3]) {
    lane L;
    lane_init(&L, job, gx, gy, time);
    L.channels = o3s(1.0f);
    o_v3 (*tr)(lane*, o_v3, o_v3) = (job->scene->variant == RMR_VARIANT_RM2) ? trace_rm2 : trace_rm1;
    o_v3 c = tr(&L, o3(o[0], o[1], o[2]), o3(d[0], d[1], d[2]));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
void oracle_march(const rmr_scene* sc, const rmr_params* prm, const float o[3], const float d[3],
                  float dist_mult, float out[2]) {
    lane L; kat_lane(&L, sc, prm);
    o_v2 v = o_march(&L, o3(o[0], o[1], o[2]), o3(d[0], d[1], d[2]), dist_mult);
    out[0] = v.x; out[1] = v.y;
}
void oracle_normal(const rmr_scene* sc, float max_dist, const float p[3], float out[3]) {
    lane L; kat_lane(&L, sc, NULL); L.max_dist = max_dist;
    o_v3 n = o_normal(&L, o3(p[0], p[1], p[2]));
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
}
void oracle_rand_chain(int gx, int gy, float time, const float* co_xy, int n, float* out) {
    lane L; memset(&L, 0, sizeof(L));
    L.gxt = (float)gx + time; L.gyt = (float)gy + time; L.time = time;
    for (int i = 0; i < n; i++) out[i] = o_rand(&L, o2(co_xy[2 * i], co_xy[2 * i + 1]));
}
void oracle_hemisphere(int gx, int gy, float time, float rc0, const float s1[2], const float s2[2],
                       const float normal[3], float out[3]) {
    lane L; memset(&L, 0, sizeof(L));
    L.gxt = (float)gx + time; L.gyt = (float)gy + time; L.time = time; L.rc = rc0;
    o_v3 b = o_hemisphere(&L, o2(s1[0], s1[1]), o2(s2[0], s2[1]), o3(normal[0], normal[1], normal[2]));
    out[0] = b.x; out[1] = b.y; out[2] = b.z;
}
void oracle_wl2rgb(uint32_t wl, float out[3]) {
    o_v3 c = wl2rgb(wl);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
