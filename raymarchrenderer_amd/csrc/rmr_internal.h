// rmr_internal.h — kernel launch parameters shared by the host API (rmr_api.cpp) and the kernels.
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif
#include "../../include/rmr_tables.h"

namespace rmr {

// One 8x8 pixel tile = one wave's initial 64 paths (the reference RM1 workgroup shape,
// RayMarch.glsl:11). tiles[] holds the tile origin (x, y) in pixels.
struct TileXY { int32_t x, y; };

// Packed primitive for the sphere/box fast paths: one s_load_dwordx8 per prim.
struct DPrim {
    float c[3];
    float r[3];
    int32_t type;  // RMR_PRIM_SPHERE / RMR_PRIM_BOX; 0 = padding (never evaluated)
    float mat_id;
};

// Material shading kind, precomputed on the host from the v1 node program (rmr_material).
enum MatKind : int32_t {
    MAT_NONE = 0,      // no `case` for this id: outputs stay vec3(0) -> path ends black
    MAT_DIFFUSE = 1,   // single shader_diffuse(literal) node, color/dir wired straight out
    MAT_EMISSION = 2,  // single shader_emission(literal, literal) node, dir not written
    MAT_PROGRAM = 3,   // anything else: the generic node interpreter
};
struct DMat {
    int32_t kind;
    float c[3];   // diffuse / emission color literal
    float p[3];   // emission power literal
    float gray1;  // gray_ch(p, -1) = ((p.x + p.y) + p.z) / 3 (host, same float operations)
};

// Bounding-volume node of the exact culling map (NP = -2, scenes of more than 32 spheres/boxes).
// Nodes are in depth-first pre-order: the first child of an internal node is the next node,
// `skip` is the node after the whole subtree. Leaves hold `count` primitives starting at `first`
// in the leaf-ordered DPrim array (DPrim.type carries the original scene index in bits 8..31).
struct BvhNode {
    float lo[3];
    int32_t first;
    float hi[3];
    int32_t count;   // 0 = internal node
    int32_t skip;
    int32_t pad[3];
};

// the trace kernel's work-queue counters (rmr_trace.h RMR_QUEUE_PARTS partitions, 128 B apart; room
// for 64): zero when a trace launch starts. Zeroed once at rmr_create (and at a launch slot's creation),
// then by each launch's fold (fold_main, ordered after its trace) for the next launch on the same queue,
// so a launch costs no separate memset dispatch (the reference's one-sample Graphics::Render calls: one
// dispatch fewer per call)
constexpr size_t kQueueBytes = 8192;
constexpr int kQueueWordStride = 32;   // 32-bit words between two partition counters

struct KParams {
    // ---- scene tables (device pointers, read-only) ----
    const rmr_prim* prims;
    const rmr_op* ops;
    const float* consts;
    const rmr_material* mats;
    const rmr_spectral* spec;
    const rmr_rm2_consts* rm2;
    const DPrim* dprims;        // packed prims (fast map paths)
    const DMat* dmats;          // per-id shading kind (RM1)
    const BvhNode* bvh;         // NP = -2: node array (n_nodes), prims in dprims in leaf order
    int32_t n_nodes;
    // candidate grid of the nearest-primitive cache's full map() (rmr_trace.h map_grid_npc; null =
    // none): per cell x = list offset | count << 24 (count 255: no list, take the BVH), y = float bits
    // of a lower bound of every non-listed primitive's float distance in the cell, z / w = the list's
    // first four leaf indices (16 bits each, z low first), inline; lists of leaf indices; leaf indices
    // [0, grid_n_large) are evaluated everywhere (large primitives)
    const uint4* grid;
    const uint16_t* grid_list;
    float grid_lo[3];
    float grid_inv;             // 1 / cell size
    int32_t grid_dim[3];
    float grid_dimf[3];         // the same as floats (the kernel's range test compares against SGPR
                                // operands instead of converted values the allocator would spill)
    int32_t grid_n_large;
    float grid_sbox[6];         // box of the small primitives (lo.xyz, hi.xyz), rounded outward
    float bvh_margin;           // absolute part of the culling margin (scales with the scene extent)
    float am_r2;                // 2 x the largest |sphere radius| (approximate-then-exact map, rmr_trace.h)
    float npc_eps0;             // nearest-primitive cache: 2^-17 E + 2^-60 (rmr_trace.h npc_eps)
    float cert_k;               // certified getNormal probes: the bound of rmr_trace.h am_normal_cert
    int32_t esc_on;             // escape bound (rmr_trace.h ray_exit): sphere/box scenes
    int32_t eye_step;           // primary rays' first march step from map(eye) (rmr_trace.h eye_map)
    const float* esc_boxes;     // n_esc inflated boxes (lo.xyz, hi.xyz) covering every primitive
    int32_t n_esc;
    int32_t full_threshold;     // nearest-primitive cache: bits 0-7 lanes per full map() batch; bits 8-15 R:
                                // also a batch once waiting lanes x R >= 8 x cache-served lanes
    int32_t n_prims;
    int32_t n_mats;
    int32_t v2_begin, v2_end;
    rmr_spectral spec_sky;
    float sky[3];
    const float4* env;          // envTex texels (c / 255, RGBA), row 0 = t 0; used when use_env
    int32_t env_w, env_h, use_env;
    float rm2_light[3];
    float rm2_light_power;
    int32_t rm2_node_id;
    // ---- render parameters (Graphics::Render uniforms) ----
    float max_dist, step_mult;
    int32_t max_steps, max_bounces, separate_channels;
    // ---- view (setView uniforms, shader order) ----
    float eye[3], r00[3], r01[3], r10[3], r11[3];
    int32_t W, H;
    // host-computed uniforms the kernels would otherwise derive per wave with VALU ops (whose results
    // the allocator keeps in VGPRs for the whole kernel, and spills): r01 - r00, r11 - r10 (float
    // subtraction, the same bits), (float)W, (float)H, and the env map's (float) w, h, w - 1, h - 1
    float dr01[3], dr11[3];
    float Wf, Hf;
    float env_wf[4];
    float eye_xy;               // eye.x + eye.y (the first sum of a primary ray's ray_exit NaN check)
    // ---- work ----
    int32_t x0, y0, x1, y1;     // clip rect (pixels inside = rendered)
    const TileXY* tiles;        // n_tiles tiles
    int32_t n_tiles;
    uint32_t nspp;              // samples in this launch
    uint32_t first_sample;      // running-mean index of sample 0
    const float* times;         // [nspp] rand() seed per sample (null when nspp == 1: time1)
    float time1;                // the seed of a one-sample launch, as a kernel argument (no copy)
    uint64_t n_units;           // nspp * n_tiles * 64
    uint32_t chunk_units;       // units a wave takes per claim (0: the kernel's chunk; smaller for small
                                // launches, so they spread over every CU, rmr_api.cpp render_tiles)
    float4* samp;               // [nspp][n_tiles][64] per-sample radiance
    float4* accum;              // W*H running mean
    unsigned long long* queue;  // persistent work counters (kQueueBytes: one per partition, 128 B apart)
    unsigned long long* counters; // [0] map evals, [1] samples traced
    int32_t flops_static;       // count builds (RMR_COUNT_FLOPS): flops of one map() fold without the
    int32_t transc_static;      //   Mandelbulb iterations, and its transcendentals (scene.cpp)
    int32_t shade_threshold;    // deferred-shading batch size (lanes)
    int32_t refill_threshold;   // idle lanes before a wave fetches new units
};

}  // namespace rmr
