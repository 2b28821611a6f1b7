/*
 * oracle/rmr_oracle.h — TEST INFRASTRUCTURE. CPU restatement of the reference's per-pixel hot path
 * (RayMarch.glsl, RayMarch2.glsl, RayMarch3.glsl) over rmr scene tables.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so —
 * as the checker / CPU baseline, never as the product path.
 *
 * Parity pinning: the restatement is checked against outputs of the reference GLSL itself, run
 * headless on Mesa llvmpipe in the survey container (oracle/glsl_ref/, fixtures in tests/golden/):
 * deterministic functions (map / march / getNormal / wavelengthToColor) within float tolerance,
 * whole images statistically (the reference's sin-hash RNG stream is driver-defined).
 */
#ifndef RMR_ORACLE_H
#define RMR_ORACLE_H

#include <stdint.h>
#include "../include/rmr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* view = eye, ray00, ray01, ray10, ray11 in shader-uniform order (15 floats). */
typedef struct oracle_job {
    const rmr_scene* scene;
    rmr_params params;
    float view[15];
    int W, H;
    /* envTex (used when params.use_env_tex != 0): env_w x env_h RGBA texels as floats, row 0 = t 0,
     * i.e. the RGBA8 texture's c / 255 (GL unorm conversion) */
    const float* env;
    int env_w, env_h;
} oracle_job;

/* Radiance of one sample of pixel (px,py) at seed `time` — RayMarch*.glsl main() minus the
 * accumulator update. Returns RGB in out[3]; *map_evals (optional) += map() calls. */
void oracle_sample(const oracle_job* job, int px, int py, float time, float out[3], uint64_t* map_evals);

/* nspp running-mean samples (first_sample ...) of every pixel of [x0,x1)x[y0,y1) into accum
 * (W*H*4 floats, in/out), exactly as nspp Graphics::Render dispatches. nthreads <= 0: all. */
void oracle_render(const oracle_job* job, const float* times, int x0, int y0, int x1, int y1,
                   uint32_t first_sample, uint32_t nspp, float* accum, int nthreads, uint64_t* map_evals);

/* Per-sample radiance planes: out[k][pixel in rect, row-major][4] (alpha = 1). */
void oracle_trace_samples(const oracle_job* job, const float* times, int x0, int y0, int x1, int y1,
                          uint32_t nspp, float* out, int nthreads, uint64_t* map_evals);

/* ---- function-level known-answer hooks ---- */
float oracle_det_sin(float x);
float oracle_det_cos(float x);
float oracle_det_acos(float x);
float oracle_det_log(float x);
float oracle_det_exp(float x);
float oracle_det_atan2(float y, float x);
/* trace(o, d) (RM1/RM2) for the invocation at gid (gx, gy), seed `time`, channels = 1 */
void oracle_trace(const oracle_job* job, int gx, int gy, float time, const float o[3], const float d[3],
                  float out[3]);
/* map(p) -> (dist, id) */
void oracle_map(const rmr_scene* sc, float max_dist, const float p[3], float out[2]);
/* march(o,d,distMult) -> (t, id) */
void oracle_march(const rmr_scene* sc, const rmr_params* prm, const float o[3], const float d[3],
                  float dist_mult, float out[2]);
void oracle_normal(const rmr_scene* sc, float max_dist, const float p[3], float out[3]);
/* n successive rand(co) calls from randChange = 0 with gid/time; writes n values */
void oracle_rand_chain(int gx, int gy, float time, const float* co_xy, int n, float* out);
/* randHemisphere(s1,s2,normal) from randChange = rc0 */
void oracle_hemisphere(int gx, int gy, float time, float rc0, const float s1[2], const float s2[2],
                       const float normal[3], float out[3]);
void oracle_wl2rgb(uint32_t wl, float out[3]);

#ifdef __cplusplus
}
#endif
#endif
