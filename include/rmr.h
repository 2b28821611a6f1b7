/*
 * rmr.h — C ABI of the MI355X-native SDF ray-march path tracer (librmr.so).
 *
 * This is the drop-in boundary for the reference's render backend, the static C++ class
 * `Graphics` (RayMarch Renderer/Graphics.h:15-134, Graphics.cpp:215-835), which had no FFI of its
 * own. Each entry point names the reference member it replaces. Conventions:
 *   - plain C, opaque handle, int status (RMR_OK = 0, negative = error), message through
 *     rmr_last_error(ctx); nothing throws across the boundary;
 *   - caller-owned host buffers, library-owned device memory (or caller-bound device memory via
 *     rmr_bind_accum), one context per thread;
 *   - calls are asynchronous w.r.t. the GPU exactly like the reference's glDispatchCompute;
 *     rmr_sync / rmr_read_accum / rmr_save_bmp synchronise.
 * INTEGRATION.md shows the binding a maintainer adds on the reference side.
 */
#ifndef RMR_H
#define RMR_H

#include <stddef.h>
#include <stdint.h>
#include "rmr_tables.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RMR_OK          0
#define RMR_E_INVALID  (-1) /* bad argument                                                  */
#define RMR_E_HIP      (-2) /* HIP runtime error / no device                                  */
#define RMR_E_SCENE    (-3) /* scene does not compile (the reference's shader compile error)  */
#define RMR_E_IO       (-4) /* file I/O                                                        */
#define RMR_E_STATE    (-5) /* call out of order (e.g. render before a scene is loaded)        */
#define RMR_E_NOMEM    (-6)
#define RMR_E_UNSUPPORTED (-7)

typedef struct rmr_ctx rmr_ctx;

/* Render parameters. Defaults = the constants Graphics::Render uploads (Graphics.cpp:326-340). */
typedef struct rmr_params {
    float   max_dist;          /* 1000                                                        */
    int32_t max_steps;         /* 512                                                         */
    int32_t max_bounces;       /* 16                                                          */
    float   step_multiply;     /* 0.5                                                         */
    int32_t separate_channels; /* 0                                                           */
    int32_t use_env_tex;       /* 0 (Graphics.cpp:338); 1 = skyColor from the env map          */
} rmr_params;

/* Kernel statistics for the roofline (accumulated since the last rmr_reset_stats). */
typedef struct rmr_stats {
    uint64_t map_evals;      /* scene-SDF evaluations (the algorithmic work unit)  */
    uint64_t samples;        /* pixel samples traced                                           */
    uint64_t trace_launches; /* trace-kernel launches                                          */
    double   trace_ms;       /* summed trace-kernel time measured with HIP events              */
    double   fold_ms;        /* summed accumulate-kernel time                                  */
    double   flops_per_map;  /* algorithmic flops of one map() for the loaded scene            */
    uint64_t map_iters;      /* wave-level map() iterations: map_evals/(64*map_iters) = lane use */
    uint64_t shade_batches;  /* wave-level deferred-shading batches                             */
    uint64_t jit_launches;   /* trace launches that ran the hipRTC scene-specialised kernel     */
} rmr_stats;

/* ---- lifetime --------------------------------------------------------------------------- */
/* Graphics::Init (Graphics.cpp:263-300): select device, create streams; no GL context needed. */
int  rmr_create(rmr_ctx** out, int device);
void rmr_destroy(rmr_ctx* ctx);
const char* rmr_last_error(const rmr_ctx* ctx);
/* Compile-time kernel configuration string (variants, wave size, build flags). */
const char* rmr_build_info(void);

/* Run kernels on a caller stream (a hipStream_t passed as void*). NULL gives the context a new
 * library-owned non-blocking stream (it does NOT select the legacy null stream): work the caller
 * orders on its own streams (zeroing the accumulator, a collective over it) must then be ordered
 * with rmr_sync, so pass the caller's stream whenever it shares buffers with the renderer. */
int rmr_set_stream(rmr_ctx* ctx, void* hip_stream);

/* ---- image / view / params ------------------------------------------------------------- */
/* Graphics::setImageSize / getImageSize (Graphics.cpp:817-825). The reference applies a new size
 * at the next Init/Reload (Graphics.cpp:744-745); rmr_reload does the same here. */
int rmr_set_image_size(rmr_ctx* ctx, int w, int h);
int rmr_get_image_size(const rmr_ctx* ctx, int* w, int* h);

int rmr_set_params(rmr_ctx* ctx, const rmr_params* p);
int rmr_get_params(const rmr_ctx* ctx, rmr_params* p);
void rmr_default_params(rmr_params* p);

/* Graphics::setView (Graphics.cpp:827-835), arguments in *shader-uniform* order. Note the
 * reference camera calls setView(eye, ray00, ray10, ray01, ray11) (Camera.cpp:101), so its
 * uniform "ray01" holds the camera's ray10. rmr_camera_view() below already applies that swap. */
int rmr_set_view(rmr_ctx* ctx, const float eye[3], const float ray00[3], const float ray01[3],
                 const float ray10[3], const float ray11[3]);

/* Camera::calculateRays (Camera.cpp:25-102) restated: eye/dir/aspect/fov -> the five uniforms in
 * shader order (eye, ray00, ray01, ray10, ray11), i.e. after the setView argument swap. */
void rmr_camera_view(const double eye[3], const double dir[3], float aspect, float fov,
                     float out_eye[3], float out_ray00[3], float out_ray01[3],
                     float out_ray10[3], float out_ray11[3]);

/* ---- scene ------------------------------------------------------------------------------- */
/* Graphics::clearScene/addMaterial/addObject + Reload's code generator (Graphics.cpp:392-752,
 * 801-815): parse a reference scene file (v1 or v2 format, App. C of SURVEY) for `variant` and
 * compile it into tables. Errors the reference would hit as a GLSL compile error (stale arity,
 * unknown node, bad var index) return RMR_E_SCENE with the message in rmr_last_error. */
int rmr_load_scene_json(rmr_ctx* ctx, int variant, const char* json, size_t len);
/* Context-free scene compilation (no GPU needed): compile to a library-owned table set, view it
 * as an rmr_scene, free it. On RMR_E_SCENE the reason is written to err (if errlen > 0). */
typedef struct rmr_scene_blob rmr_scene_blob;
int rmr_scene_compile(int variant, const char* json, size_t len, rmr_scene_blob** out, char* err, size_t errlen);
int rmr_scene_view(const rmr_scene_blob* blob, rmr_scene* out);
void rmr_scene_free(rmr_scene_blob* blob);
/* Load precompiled tables (copied). */
int rmr_load_scene_tables(rmr_ctx* ctx, const rmr_scene* scene);
/* The built-in scenes that the reference hard-codes in its shaders: RM2's one-sphere map
 * (RayMarch2.glsl:133-172, needs a v2 material for id 1 via rmr_load_scene_json) and RM3's
 * three-primitive spectral scene (RayMarch3.glsl:132-143, 251-345). */
int rmr_load_builtin_scene(rmr_ctx* ctx, int variant);

/* Graphics::Reload tail (Graphics.cpp:741-751): apply the pending image size and clear the
 * accumulator to (0,0,0,0). */
int rmr_reload(rmr_ctx* ctx);

/* ---- render ------------------------------------------------------------------------------ */
/* Graphics::Render (Graphics.cpp:314-354): add ONE sample to every pixel with
 * min <= pix < max, as the running mean of RayMarch*.glsl main() using `current_sample` (0
 * overwrites). `time` is the rand() seed uniform. */
int rmr_render(rmr_ctx* ctx, float time, float min_x, float min_y, float max_x, float max_y,
               uint32_t current_sample);
/* Call batching of rmr_render (the reference calls Graphics::Render once per tile and sample,
 * Program.cpp:232-284; one such launch renders one sample of a tile and is bound by its longest path,
 * not by the chip). With batching on, rmr_render records the call (checking its state errors at once)
 * and launches nothing; consecutive samples of a rect, and rects holding the same samples, go out
 * together as one launch when any other entry point is called (rmr_sync, rmr_read_accum, rmr_save_bmp,
 * rmr_display, a setter, ...; rmr_accum_device_ptr included), when an overlapping rect or a
 * non-consecutive sample of a held rect arrives, or when 2^28 units are held. Bitwise equal to
 * unbatched calls (each pixel's samples, their seeds and their running-mean order are the same). Like
 * GL, which also queues the reference's dispatches until something reads their results, the work
 * starts at the next flush: a caller that orders its own stream work on the context's accumulator
 * without calling into rmr must flush first (rmr_sync). mode 1 on, 0 off, -1 auto (default): on while
 * the context owns its stream and its accumulator (no rmr_set_stream / rmr_bind_accum), since only
 * then are all readers inside rmr. rmr_destroy drops calls still held. */
int rmr_set_call_batching(rmr_ctx* ctx, int mode);
/* Launch overlap: n >= 2 (default 2; 4 with 8 or more hardware queues) puts consecutive trace launches round-robin on n private
 * streams, each with its own sample planes and work queue, so one launch's drain (its last long paths)
 * overlaps the next launch's start; n = 0 or 1 runs every launch on the context's stream. Each
 * launch's fold stays on the context's stream, after its trace and in call order, so results are
 * bitwise the same, and work the caller orders after a call on that stream still sees the call's
 * samples. Costs one sample-plane buffer per stream; launches whose planes exceed the plane budget / n
 * run on the context's stream. At most 4. Several contexts that already overlap each other's frames
 * (multi_gpu.FrameRenderer, the device group) set 0: their streams would exceed the GPU's hardware
 * queues (4 per process) and serialise. */
int rmr_set_launch_streams(rmr_ctx* ctx, int n);
/* The context's launch streams (rmr_create's default: 2, or 4 where the process has 8 or more hardware
 * queues, GPU_MAX_HW_QUEUES); -1 for a null context. */
int rmr_get_launch_streams(const rmr_ctx* ctx);
/* Batched fast path: samples first_sample .. first_sample+nspp-1 of every pixel in the integer
 * rect [x0,x1)x[y0,y1), sample k seeded with times[k]. Bitwise equal to nspp rmr_render calls
 * with the same times. */
int rmr_render_spp(rmr_ctx* ctx, const float* times, int x0, int y0, int x1, int y1,
                   uint32_t first_sample, uint32_t nspp);
/* Same as rmr_render_spp but over an explicit tile list (tile_size x tile_size tiles, given as
 * (tx,ty) pairs): the multi-GPU partition unit. Each (tx,ty) may appear at most once (a repeated or
 * negative tile is RMR_E_INVALID: two threads would fold into the same pixel). */
int rmr_render_tiles(rmr_ctx* ctx, const float* times, const int32_t* tiles_xy, int n_tiles,
                     int tile_size, uint32_t first_sample, uint32_t nspp);

/* ---- output ------------------------------------------------------------------------------ */
/* Accumulator as RGBA32F, row 0 = image row 0 (= the top edge). */
int rmr_read_accum(rmr_ctx* ctx, float* rgba, size_t bytes);
int rmr_write_accum(rmr_ctx* ctx, const float* rgba, size_t bytes); /* checkpoint resume */
/* Device pointer of the accumulator (float4 per pixel) for collectives (RCCL reduce). */
void* rmr_accum_device_ptr(rmr_ctx* ctx);
/* Render into caller-owned device memory of w*h*16 bytes instead (e.g. a torch tensor). */
int rmr_bind_accum(rmr_ctx* ctx, void* device_ptr, size_t bytes);
/* Graphics::SaveImage (Graphics.cpp:754-799): 24-bit BMP with the reference's quirks
 * (u8 round, 1.055*c^(1/2.4) without -0.055, truncation, SOIL pink background for alpha 0). */
int rmr_save_bmp(rmr_ctx* ctx, const char* path);
/* The same encoding from a host RGBA32F buffer (no context needed). */
int rmr_encode_bmp(const float* rgba, int w, int h, const char* path);
/* Raw float accumulator checkpoint: "RMRACC1\0", w, h, samples, then RGBA32F. */
int rmr_save_accum(rmr_ctx* ctx, const char* path, uint32_t samples_done);
int rmr_load_accum(rmr_ctx* ctx, const char* path, uint32_t* samples_done);

int rmr_sync(rmr_ctx* ctx);
int rmr_get_stats(rmr_ctx* ctx, rmr_stats* out);
int rmr_reset_stats(rmr_ctx* ctx);
/* Profiling builds only (librmr compiled with -DRMR_PROFILE; zeros otherwise): per-wave shader-clock
 * cycles summed over all waves since rmr_reset_stats, split into [0] refill/ray setup, [1] map()
 * iterations, [2] shading batches, [3] whole trace loop. */
int rmr_get_section_cycles(rmr_ctx* ctx, uint64_t out[4]);
/* Raw kernel counters (diagnostics): [0] map evals, [1] map iterations, [2] shading batches,
 * [3] full map() batches of the nearest-primitive cache, [8] lanes shaded (lane-level shading events),
 * [14] map evals in shading batches (certified getNormal probes, rmr_trace.h cert_normals; part of [0]),
 * [4..7] the section cycles above (or the RMR_JIT_AMBCOUNT fallback counts, tools/amb_rate.py). */
int rmr_get_counters(rmr_ctx* ctx, uint64_t out[16]);
/* Select kernel implementation (0 = persistent wavefront kernel, 1 = one launch-thread per path). */
int rmr_set_kernel(rmr_ctx* ctx, int kernel);
/* envTex of skyColor (RM1:78-113, RM2:84-107; the reference loads veranda_1k.hdr through SOIL as
 * an RGBA8 texture, Graphics.cpp:287): w x h RGBA8 texels, row 0 = texture coordinate t = 0 (the
 * direction +y). Used when params.use_env_tex != 0; NULL removes it. Sampling: bilinear, level 0,
 * CLAMP_TO_EDGE. */
int rmr_set_env_map(rmr_ctx* ctx, const uint8_t* rgba8, int w, int h);

/* ---- display ---------------------------------------------------------------------------- */
/* Graphics::Display(centre, zoom, min, max) (Graphics.cpp:356-390 with createFQ 227-258 and
 * FullQuad.vs / FullQuad.fs), headless: draws the accumulator into a screen_w x screen_h RGBA8 image
 * (row 0 = top, the window's coordinates; Screen::getScreenSize() is the image size) the way the
 * reference's textured quad does: quad [centre - size/2 zoom, centre + size/2 zoom), nearest texel
 * (GL_NEAREST, Graphics.h:90-91), alpha 1 inside [min, max] and 0 elsewhere, GL_FRAMEBUFFER_SRGB
 * encode (byte = round(255 srgb(clamp(c, 0, 1))), exact; rmr_srgb_thresholds) and the
 * SRC_ALPHA / ONE_MINUS_SRC_ALPHA blend: pixels drawn with alpha 1 are replaced, every other pixel
 * keeps the caller's content (the GUI behind the image). rgba8 is a host buffer (in/out) of nbytes
 * bytes; RMR_E_INVALID unless nbytes >= screen_w * screen_h * 4. */
int rmr_display(rmr_ctx* ctx, float centre_x, float centre_y, float zoom, float min_x, float min_y, float max_x,
                float max_y, int screen_w, int screen_h, uint8_t* rgba8, size_t nbytes);
/* The same into a device buffer of nbytes bytes (e.g. a torch uint8 tensor or an interop surface), on
 * the context's stream, without host copies or a sync. */
int rmr_display_device(rmr_ctx* ctx, float centre_x, float centre_y, float zoom, float min_x, float min_y,
                       float max_x, float max_y, int screen_w, int screen_h, void* rgba8_dev, size_t nbytes);
/* The 256 sRGB decision points rmr_display uses: out[k] = the smallest float c with byte(c) >= k. */
int rmr_srgb_thresholds(float out[256]);
/* Test hook, no GPU needed: the candidate grid a context builds for a BVH scene's nearest-primitive
 * cache (rmr_trace.h map_grid_npc). prims: n rows of 8 floats in leaf order (c.xyz, r.xyz, type
 * RMR_PRIM_SPHERE / RMR_PRIM_BOX as a float value, mat_id); rows [0, n_large) are evaluated everywhere
 * (large primitives), the rest are gridded. E = max |c|_inf + |r|_inf over the scene. target / pad:
 * cell count / region growth (<= 0: the context's defaults). Out: idims = (dim.xyz, list length,
 * built 0/1); geom = (lo.xyz, 1 / cell size, small-primitive box lo.xyz hi.xyz, eps, margin); cells:
 * 2 words per cell (offset | count << 24, bound bits); list: leaf indices. Returns RMR_E_INVALID with
 * idims filled when cells_cap (words) or list_cap is too small. */
int rmr_candidate_grid(const float* prims, int n, int n_large, double E, double target, double pad, int32_t idims[5],
                       float geom[12], uint32_t* cells, size_t cells_cap, uint16_t* list, size_t list_cap);
/* Per-scene kernel specialisation (the reference recompiles its shader per scene, Graphics::Reload):
 * the scene's map() is generated as HIP source with the primitives as literals and compiled by
 * hipRTC for gfx950 at the first render that uses it (code objects cached in-process and under
 * $RMR_JIT_CACHE or ~/.cache/rmr-jit). Results are bit-identical to the table-driven kernels.
 * mode 0 = off, 1 = always (errors are returned), 2 = auto (default: launches of >= 2^16 units;
 * a failed compile falls back to the table-driven kernel). (The diagnostic build librmr_diag.so also
 * reads env RMR_JIT at rmr_create; the release librmr.so reads no environment but RMR_JIT_CACHE.) */
int rmr_set_jit(rmr_ctx* ctx, int mode);
/* Exact work-skipping in the trace kernels (all results bit-identical; only the count of map()
 * calls changes), default all on (librmr_diag.so: env RMR_ESC=0 / RMR_NPC=0 / RMR_JIT_APPROX=0 /
 * RMR_EYE=0 clear a bit at rmr_create):
 *   RMR_CULL_ESCAPE: a march past the exit of the inflated scene box ends as its miss
 *   RMR_CULL_NPC:    nearest-primitive cache of the BVH map (scenes of > 32 spheres/boxes)
 *   RMR_CULL_APPROX: approximate-then-exact map() of sphere/box scenes (one exact sqrt)
 *   RMR_CULL_EYE:    every primary ray's first march step is map(eye): evaluated once per wave
 *                    (RM1 sphere/box/Mandelbulb kernels and RM3) */
#define RMR_CULL_ESCAPE 1
#define RMR_CULL_NPC 2
#define RMR_CULL_APPROX 4
#define RMR_CULL_EYE 8
int rmr_set_culling(rmr_ctx* ctx, int flags);
/* Instrumented specialised kernels (measurement only; the images are the same bits):
 *   RMR_INSTR_COUNT_FLOPS: the hipRTC kernel built with -DRMR_COUNT_FLOPS (rmr_trace.h count_work):
 *     executed SDF flops / transcendentals per map() into rmr_get_counters [11] / [12] / [13], one
 *     atomic per wave and counted event (so it is slower; bench.py's count pass, never timed).
 * Applies to the hipRTC kernels (rmr_set_jit 1); 0 restores the production kernel. */
#define RMR_INSTR_COUNT_FLOPS 1
int rmr_set_instrument(rmr_ctx* ctx, int flags);
/* Compile the specialised kernel of a scene without a GPU (json NULL = the variant's built-in
 * scene). On success `log` receives the code-object key, otherwise the compiler log. */
int rmr_jit_compile_scene(int variant, const char* json, size_t len, char* log, size_t loglen);
/* Tuning knobs (<= 0 / < 0 keeps the current value): deferred-shading batch size in lanes (1..64),
 * persistent workgroups per CU (0 = occupancy), per-launch sample-plane budget in bytes. Until a
 * batch size is set (here, or by env RMR_SHADE_T in librmr_diag.so) it is chosen per kernel: 8 for general maps
 * without material programs, 16 otherwise. Results do not depend on any of these (scheduling only). */
int rmr_set_tuning(rmr_ctx* ctx, int shade_threshold, int grid_per_cu, long long samp_budget_bytes);
/* (shade_threshold bits 8..15, when non-zero, set the refill threshold separately: idle lanes a
 * wave collects before it fetches new units; default (and when zero) = half the shading
 * threshold, at least 2.) */
/* Persistent-grid reserve: the trace launch leaves `blocks` workgroups of its occupancy grid
 * unlaunched (default 0; the grid stays >= 1 workgroup). For two contexts that alternate frames on
 * one GPU (multi_gpu.FrameRenderer): a persistent trace kernel holds every slot it gets until its
 * queue runs out, so the other context's running-mean fold (and the next frame's zeroing) would
 * wait for that trace's drain, and the next trace behind them; a few free slots let them run beside
 * it. Scheduling only: results do not depend on it. RMR_E_INVALID for blocks < 0. */
int rmr_set_grid_reserve(rmr_ctx* ctx, int blocks);
/* Test hook: per-sample radiance (before the running mean) of the integer rect, written as
 * out[k][y-y0][x-x0][4]; sample k is seeded with times[k]. The accumulator is left unchanged. */
int rmr_trace_samples(rmr_ctx* ctx, const float* times, int x0, int y0, int x1, int y1, uint32_t nspp, float* out);
/* sizeof of the ABI structs (prim, op, material, spectral, rm2_consts, scene, params, stats). */
int rmr_abi_sizes(int32_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* RMR_H */
