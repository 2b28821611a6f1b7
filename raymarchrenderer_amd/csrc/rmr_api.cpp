// rmr_api.cpp — the C ABI of librmr.so (include/rmr.h): the drop-in replacement for the
// reference's static `Graphics` backend (Graphics.h:15-134, Graphics.cpp:215-835).
//
// Ownership: the context owns its HIP stream, the scene tables in HBM, the per-sample radiance
// planes and (unless rmr_bind_accum is used) the RGBA32F accumulator. Host buffers passed in are
// caller-owned and copied. No exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <new>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rmr.h"
#include "rmr_internal.h"
#include "grid.hpp"
#include "rmr_jit.hpp"
#include "scene.hpp"

namespace rmr {
hipError_t launch_trace(const KParams& P, int variant, int np, bool prog, bool persistent, int grid, hipStream_t s);
hipError_t launch_fold(const KParams& P, hipStream_t s);
hipError_t launch_ray_exit(const KParams& P, const float* rays, float* out, int n, hipStream_t s);
hipError_t launch_display(const float4* accum, int img_w, int img_h, float cx, float cy, float zoom, float min_x,
                          float min_y, float max_x, float max_y, int scr_w, int scr_h, uint32_t* rgba8,
                          const float* thr, hipStream_t s);
int trace_occupancy(int variant, int np, bool prog, int* blocks_per_cu);
}  // namespace rmr

using rmr::CompiledScene;
using rmr::KParams;
using rmr::TileXY;

struct EventPair { hipEvent_t a, b, c; };

constexpr int kSlotGridReserve = 32;   // workgroups a slotted launch leaves free for the previous fold

struct rmr_ctx {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int W = 1024, H = 1024;               // GUI.cpp:201-208 defaults (Graphics.cpp:6 is overridden)
    int pend_W = 1024, pend_H = 1024;
    rmr_params params{};
    float view[15];
    bool view_set = false;
    CompiledScene scene;
    bool scene_loaded = false;
    // device tables
    rmr_prim* d_prims = nullptr;
    rmr_op* d_ops = nullptr;
    float* d_consts = nullptr;
    rmr_material* d_mats = nullptr;
    rmr_spectral* d_spec = nullptr;
    rmr_rm2_consts* d_rm2 = nullptr;
    rmr::DPrim* d_dprims = nullptr;
    rmr::DMat* d_dmats = nullptr;
    rmr::BvhNode* d_bvh = nullptr;
    // escape bound (rmr_trace.h ray_exit): <= kMaxEscBoxes boxes covering every primitive (lo.xyz,
    // hi.xyz), uploaded inflated by esc_infl (which depends on the view and maxDist)
    std::vector<float> esc_raw;
    std::vector<rmr::BvhNode> bvh_host;   // host copy of the BVH (escape-box cut)
    std::vector<int> bvh_order;           // leaf-order -> scene index
    float* d_esc = nullptr;
    double esc_infl_dev = -1.0;
    float4* d_env = nullptr;              // envTex (rmr_set_env_map)
    float* d_srgb_thr = nullptr;          // rmr_display: sRGB decision points (256 floats)
    uint32_t* d_screen = nullptr;         // rmr_display: staging of a host screen image
    size_t screen_cap = 0;
    int env_w = 0, env_h = 0;
    int n_bvh = 0;
    float bvh_margin = 1e-4f;
    // candidate grid of the cache's full map() (build_grid; BVH scenes)
    uint4* d_grid = nullptr;
    uint16_t* d_grid_list = nullptr;
    bool grid_on = false;
    bool grid_small_spheres = false;   // every primitive a cell can list is a sphere (rmr_jit.cpp)
    float grid_lo[3] = {0, 0, 0}, grid_inv = 1.0f, grid_sbox[6] = {0, 0, 0, 0, 0, 0};
    int grid_dim[3] = {0, 0, 0}, grid_n_large = 0;
    int map_np = -1;  // map() specialisation: 4/8 unrolled, 0 loop, -1 general
    bool has_prog = true;  // RM1 scene has materials needing the generic node interpreter
    // buffers
    float4* d_accum = nullptr;
    bool accum_external = false;
    float4* d_samp = nullptr;
    size_t samp_cap = 0;
    // Launch slots (rmr_set_launch_streams): trace launches go round-robin to private streams, each with
    // its own sample planes and work queue, so a launch's drain (its last long paths on a nearly idle
    // chip) overlaps the next launch's start. Every fold stays on the context's stream, after its trace's
    // `done` event, in call order: a sync of the context's stream covers every trace queued before it,
    // and the accumulator sees the same running-mean order. A slot's planes and queue are reused once
    // the fold that read them (`freed`) is done.
    struct Slot {
        hipStream_t s = nullptr;
        float4* samp = nullptr;
        size_t cap = 0;
        unsigned long long* queue = nullptr;
        bool queue_dirty = true;
        hipEvent_t done = nullptr, freed = nullptr;
        bool in_use = false;
    };
    std::vector<Slot> slots;
    int launch_streams = 2;       // fewer than 2: every launch on the context's stream (rmr_create: 4 with
                                  // 8 or more hardware queues)
    int slot_reserve = kSlotGridReserve;   // workgroups a slotted launch leaves free (RMR_SLOT_RESERVE)
    size_t next_slot = 0;
    float4* last_samp = nullptr;  // the last launch's planes (rmr_trace_samples)
    hipEvent_t trace_end = nullptr;   // after the last trace launch, on its stream
    // device tile lists by content (tile_list): a list is uploaded once and reused by every later launch
    // with the same tiles (the reference's per-tile, per-sample calls; a rank's share each frame) with no
    // copy and no stream sync; least recently used entries go beyond kTileCacheEntries
    struct TileList { std::vector<TileXY> host; TileXY* dev; uint64_t hash; uint64_t used; };
    std::vector<TileList> tile_cache;
    uint64_t tile_clock = 0;
    // seeds of launches of more than one sample: a pinned host ring and its device twin, so the copy is
    // asynchronous (from the caller's pageable array hipMemcpyAsync had waited for the copy, i.e. for the
    // work queued before it); a one-sample launch passes its seed as a kernel argument (KParams::time1)
    float* d_times = nullptr;
    float* h_times = nullptr;
    size_t times_cap = 0, times_pos = 0;
    bool queue_dirty = false;   // a trace launch went out without the fold that zeroes the queue after it
    // deferred one-sample calls (rmr_render, the reference's Graphics::Render pattern): per pixel rect
    // the consecutive samples requested so far, launched together at the next call of any other entry
    // point (flush_calls); rmr_set_call_batching: -1 auto (on while the context owns its stream and its
    // accumulator), 0 off, 1 on
    struct Deferred { int x0, y0, x1, y1; uint32_t s0; std::vector<float> times; };
    std::vector<Deferred> deferred;
    uint64_t deferred_units = 0;
    int call_batching = -1;
    unsigned long long* d_queue = nullptr;
    unsigned long long* d_counters = nullptr;
    // timing
    std::vector<EventPair> pending, pool;
    rmr_stats stats{};
    int kernel_mode = 0;  // 0 persistent, 1 thread-per-path
    int shade_threshold = 16;   // explicit (env RMR_SHADE_T / rmr_set_tuning) or, with shade_auto, per kernel:
    bool shade_auto = true;     // per specialised kernel (ensure_jit: 20 / 8 / 16), 16 for the table kernels
    // idle lanes before a refill: -1 = half the shading threshold, at least 2 (round 2: T/2 = 8 at T = 16:
    // Cornell-5 -0.4%, RM3 -1.2%, default -2% against 2; Mandelbulb T = 8: 4 best); 0 = the shading
    // threshold; refills are cheap with the LDS chunk rays
    int refill_threshold = -1;
    // nearest-primitive cache: 40 lanes per full map() batch, or once waiting lanes >= cache-served ones
    // (R = 8; csg256 with the candidate grid: 15.7 -> 14.8 ms per 4 spp against R = 2)
    int full_threshold = 40 | (8 << 8);
    int cull = RMR_CULL_ESCAPE | RMR_CULL_NPC | RMR_CULL_APPROX | RMR_CULL_EYE;   // rmr_set_culling
    int instrument = 0;   // RMR_INSTR_* (rmr_set_instrument): instrumented specialised kernels
    int grid_per_cu = 0;  // 0 = occupancy
    int grid_reserve = 0;  // persistent grid: workgroups left free of the occupancy grid (rmr_set_grid_reserve)
    bool diag_no_fold = false;   // RMR_DIAG_NO_FOLD (diagnostic library, timing only): no k_fold launch
    int small_chunk = 64;  // fewest units per work claim when a launch is too small to fill every wave (0: off)
    // hipRTC per-scene specialisation (rmr_jit.hpp): 0 off, 1 always, 2 auto (launches of
    // >= jit_min_units units; smaller renders use the ahead-of-time kernels). 2^16: C1's 256x256
    // 1-spp frame is 65536 units and runs 0.157 -> 0.106 ms per launch specialised (the compile,
    // ~1 s once per scene and process, is cached)
    int jit_mode = 2;
    uint64_t jit_min_units = (uint64_t)1 << 16;
    bool jit_ready = false;     // `jit` matches the loaded scene
    bool jit_failed = false;    // compile/load failed for the loaded scene (auto mode falls back)
    rmr::JitKernel jit;
    std::string jit_struct_src;  // structure-only source of the last specialised scene
    std::vector<rmr_prim> jit_base;   // primitive values the specialised kernel was baked with
    std::vector<char> jit_live;       // primitives that moved since: loaded, not literals
    std::vector<rmr::JitKernel> jit_loaded;  // modules loaded by this context (unloaded at destroy)
    // sample planes per launch (bytes): 48 GiB, at most a quarter of the device's memory (rmr_create).
    // 288 GB of HBM hold a whole C4 frame (3840x2160 x 256 spp: 34 GB) in one launch, so the frame
    // pays one persistent-kernel drain instead of one per 8 GiB
    size_t samp_budget = (size_t)48 << 30;
    std::string err;
    // capacity of each table buffer (keyed by the address of its device-pointer member): a reload of
    // the same scene layout (an animation frame) copies into the buffers it has, ordered on the
    // context's stream, instead of hipFree + hipMalloc, which wait for the whole device — including
    // another context's frame still rendering (FrameRenderer's two overlapping contexts)
    std::unordered_map<const void*, size_t> dev_caps;
};

namespace {

// the kernel's refill threshold from the context setting (rmr_ctx::refill_threshold) and the
// shading threshold in effect
int refill_for(int setting, int shade_t) {
    if (setting > 0) return setting;
    if (setting == 0) return shade_t;
    return std::max(2, shade_t / 2);
}

int fail(rmr_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}
#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(ctx, RMR_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// Host -> device table upload, ordered on the context's stream: kernels of this context launched
// before it have read the old contents, those launched after read the new. A buffer is reallocated
// only when it must grow. The call returns once this context's stream has completed the copy (the
// source may be a temporary); another context's work on its own stream is not waited for.
template <class T>
int dev_upload(rmr_ctx* c, T** dst, const T* src, size_t n) {
    const size_t bytes = std::max<size_t>(1, n) * sizeof(T);
    size_t& cap = c->dev_caps[(const void*)dst];
    if (!*dst || cap < bytes) {
        if (*dst) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            (void)hipFree(*dst);
            *dst = nullptr;
        }
        HIPCHK(c, hipMalloc((void**)dst, bytes));
        cap = bytes;
    }
    if (n) {
        HIPCHK(c, hipMemcpyAsync(*dst, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return RMR_OK;
}

int alloc_accum(rmr_ctx* c) {
    if (!c->accum_external && c->d_accum) { (void)hipFree(c->d_accum); c->d_accum = nullptr; }
    c->accum_external = false;
    const size_t bytes = (size_t)c->W * c->H * sizeof(float4);
    HIPCHK(c, hipMalloc((void**)&c->d_accum, bytes));
    HIPCHK(c, hipMemsetAsync(c->d_accum, 0, bytes, c->stream));
    return RMR_OK;
}

void default_view(rmr_ctx* c) {
    // Program.cpp:102: Camera((0,4,-6), normalized(0,-3,6), W/H, PI/4), PI = 3.141592653f
    const double m = std::sqrt(0.0 + 9.0 + 36.0);
    const double eye[3] = {0.0, 4.0, -6.0};
    const double dir[3] = {0.0, -3.0 / m, 6.0 / m};
    const float pi = 3.141592653f;
    rmr_camera_view(eye, dir, (float)((double)c->W / (double)c->H), pi / 4.0f, c->view, c->view + 3, c->view + 6,
                    c->view + 9, c->view + 12);
    c->view_set = true;
}

// Scenes of more than kMaxLoopPrims spheres/boxes use the exact-culling BVH map (map_bvh in
// rmr_trace.h): median-split hierarchy over the primitives' boxes, leaves of <= 4, pre-order with
// skip links; the primitives are stored in leaf order with their scene index (the id tie-break).
constexpr size_t kMaxLoopPrims = 32;

int upload_bvh(rmr_ctx* c);

// Escape boxes: each primitive's box for scenes of <= kMaxEscBoxes primitives; for BVH scenes a cut
// of the hierarchy (the always-visited large primitives individually, then the node with the most
// primitives split until kMaxEscBoxes boxes). Their union covers every primitive.
constexpr size_t kMaxEscBoxesDefault = 32;
size_t max_esc_boxes() {   // env RMR_ESC_BOXES (experiments), read at scene upload
    if (const char* e = RMR_ENV("RMR_ESC_BOXES")) return (size_t)std::max(1, std::min(64, std::atoi(e)));
    return kMaxEscBoxesDefault;
}
// A Mandelbulb primitive (sd_mandelbulb) takes part when it iterates at least once with a bailout
// >= 1.5: at |p - c| > bailout its loop stops at once with r = |p - c|, dr = 1, so its distance is
// 0.5 log(r) r >= 0.30 — the box c +- bailout then bounds everything within 0.001 of it.
bool escape_prim(const rmr_prim& q) {
    if (q.type == RMR_PRIM_SPHERE || q.type == RMR_PRIM_BOX) return true;
    return q.type == RMR_PRIM_MANDELBULB && q.r[1] >= 1.0f && q.r[2] >= 1.5f && std::isfinite(q.r[2]);
}
float escape_halfwidth(const rmr_prim& q, int k) {
    if (q.type == RMR_PRIM_SPHERE) return std::fabs(q.r[0]);
    if (q.type == RMR_PRIM_MANDELBULB) return q.r[2];
    return std::fabs(q.r[k]);
}
void build_escape_boxes(rmr_ctx* c, bool simple) {
    const CompiledScene& s = c->scene;
    c->esc_raw.clear();
    bool ok = !s.prims.empty();
    for (const rmr_prim& q : s.prims) ok = ok && escape_prim(q);
    const size_t kMaxEscBoxes = max_esc_boxes();
    if (!ok || (!simple && s.prims.size() > kMaxEscBoxes)) return;
    auto prim_box = [&](const rmr_prim& q, float* b) {
        for (int k = 0; k < 3; k++) {
            const float h = escape_halfwidth(q, k);
            b[k] = q.c[k] - h;
            b[3 + k] = q.c[k] + h;
        }
    };
    float b[6];
    if (c->map_np != -2 || s.prims.size() <= kMaxEscBoxes) {   // one box per primitive
        for (const rmr_prim& q : s.prims) {
            prim_box(q, b);
            c->esc_raw.insert(c->esc_raw.end(), b, b + 6);
        }
        return;
    }
    // BVH scene: nodes are in pre-order (first child = next node, second child = that node's skip);
    // leaves of the always-visited list have infinite bounds: use their primitives' own boxes
    std::vector<int> cut;
    for (size_t i = 0; i < c->bvh_host.size();) {
        const rmr::BvhNode& nd = c->bvh_host[i];
        if (nd.lo[0] <= -1e38f) {   // always-visited leaf of large primitives
            for (int k = nd.first; k < nd.first + nd.count; k++) {
                prim_box(s.prims[(size_t)(c->bvh_order[(size_t)k])], b);
                c->esc_raw.insert(c->esc_raw.end(), b, b + 6);
            }
            i = (size_t)nd.skip;
            continue;
        }
        cut.push_back((int)i);   // root of the remaining hierarchy
        break;
    }
    while (!cut.empty() && c->esc_raw.size() / 6 + cut.size() < kMaxEscBoxes) {
        // split the internal node of the cut with the largest box
        int best = -1;
        float bestv = -1.0f;
        for (size_t q = 0; q < cut.size(); q++) {
            const rmr::BvhNode& nd = c->bvh_host[(size_t)cut[q]];
            if (nd.count != 0) continue;
            const float v = (nd.hi[0] - nd.lo[0]) * (nd.hi[1] - nd.lo[1]) * (nd.hi[2] - nd.lo[2]);
            if (v > bestv) { bestv = v; best = (int)q; }
        }
        if (best < 0) break;
        const int i = cut[(size_t)best];
        cut[(size_t)best] = i + 1;
        cut.push_back(c->bvh_host[(size_t)(i + 1)].skip);
    }
    for (int i : cut) {
        const rmr::BvhNode& nd = c->bvh_host[(size_t)i];
        for (int k = 0; k < 3; k++) { b[k] = nd.lo[k]; b[3 + k] = nd.hi[k]; }
        c->esc_raw.insert(c->esc_raw.end(), b, b + 6);
    }
}

// Shading kinds of the RM1 materials: the single-node diffuse / emission materials run the fast
// shading path, every other defined material its node program (has_prog). Shared by upload_scene and
// rmr_jit_compile_scene, so both pick the same kernel class.
std::vector<rmr::DMat> shading_kinds(const CompiledScene& s) {
    std::vector<rmr::DMat> dm(std::max<size_t>(1, s.materials.size()));
    for (size_t i = 0; i < s.materials.size(); i++) {
        const rmr_material& m = s.materials[i];
        rmr::DMat d{};
        d.kind = m.defined ? rmr::MAT_PROGRAM : rmr::MAT_NONE;
        if (m.defined && m.prog_end - m.prog_begin == 1 && m.inside_var < 0 && m.hit_var < 0) {
            const rmr_op& op = s.ops[(size_t)m.prog_begin];
            auto lit = [&](int ref, float* out) {
                if (!RMR_OPND_IS_CONST(ref)) return false;
                const int k = RMR_OPND_CONST_INDEX(ref);
                for (int j = 0; j < 3; j++) out[j] = s.consts[3 * (size_t)k + j];
                return true;
            };
            if (op.code == RMR_OP_M_DIFFUSE && m.color_var == op.out[0] && m.dir_var == op.out[1] &&
                op.out[0] != op.out[1] && lit(op.in[0], d.c))
                d.kind = rmr::MAT_DIFFUSE;
            else if (op.code == RMR_OP_M_EMISSION && m.color_var == op.out[0] && m.dir_var < 0 &&
                     lit(op.in[0], d.c) && lit(op.in[1], d.p)) {
                d.kind = rmr::MAT_EMISSION;
                // grayscale of p * vec3(1) without separateChannels (rmr_trace.h gray_ch, RM1:306-309):
                // x * 1 is exact, so this is the kernel's ((p.x + p.y) + p.z) / (1 + 1 + 1)
                const float sum = (d.p[0] + d.p[1]) + d.p[2];
                d.gray1 = sum / 3.0f;
            }
        }
        dm[i] = d;
    }
    return dm;
}
bool any_program(const std::vector<rmr::DMat>& dm) {
    for (const auto& d : dm)
        if (d.kind == rmr::MAT_PROGRAM) return true;
    return false;
}

int free_slots(rmr_ctx* c);

int upload_scene(rmr_ctx* c) {
    const CompiledScene& s = c->scene;
    int r;
    if ((r = dev_upload(c, &c->d_prims, s.prims.data(), s.prims.size()))) return r;
    if ((r = dev_upload(c, &c->d_ops, s.ops.data(), s.ops.size()))) return r;
    if ((r = dev_upload(c, &c->d_consts, s.consts.data(), s.consts.size()))) return r;
    if ((r = dev_upload(c, &c->d_mats, s.materials.data(), s.materials.size()))) return r;
    if ((r = dev_upload(c, &c->d_spec, s.spectral.data(), s.spectral.size()))) return r;
    if ((r = dev_upload(c, &c->d_rm2, &s.rm2, 1))) return r;
    const std::vector<rmr::DMat> dm = shading_kinds(s);
    c->has_prog = any_program(dm);
    if ((r = dev_upload(c, &c->d_dmats, dm.data(), dm.size()))) return r;
    // packed prims + map() specialisation
    bool simple = true;
    for (const auto& p : s.prims) simple = simple && (p.type == RMR_PRIM_SPHERE || p.type == RMR_PRIM_BOX);
    const size_t n = s.prims.size();
    c->map_np = !simple || n == 0 ? -1 : (n <= 4 ? 4 : (n <= 8 ? 8 : (n <= kMaxLoopPrims ? 0 : -2)));
    if (c->map_np == -2) {
        if ((r = upload_bvh(c))) return r;
    } else {
        std::vector<rmr::DPrim> dp(std::max<size_t>(n, 8));
        for (size_t i = 0; i < dp.size(); i++) {
            rmr::DPrim q{};
            if (i < n) {
                const rmr_prim& p = s.prims[i];
                for (int k = 0; k < 3; k++) { q.c[k] = p.c[k]; q.r[k] = p.r[k]; }
                q.type = p.type;
                q.mat_id = p.mat_id;
            }
            dp[i] = q;
        }
        if ((r = dev_upload(c, &c->d_dprims, dp.data(), dp.size()))) return r;
        c->n_bvh = 0;
        c->grid_on = false;
    }
    build_escape_boxes(c, simple);
    c->esc_infl_dev = -1.0;
    if (const char* e = RMR_ENV("RMR_FULL_T"))   // (experiments; read per scene load)
        c->full_threshold = (c->full_threshold & ~0xff) | std::max(1, std::min(64, std::atoi(e)));
    if (const char* e = RMR_ENV("RMR_FULL_R"))
        c->full_threshold = (c->full_threshold & 0xff) | (std::max(0, std::min(255, std::atoi(e))) << 8);
    if (const char* e = RMR_ENV("RMR_SMALL_CHUNK")) c->small_chunk = std::max(0, std::atoi(e));
    c->diag_no_fold = false;
    if (const char* e = RMR_ENV("RMR_DIAG_NO_FOLD")) c->diag_no_fold = std::atoi(e) != 0;
    if (const char* e = RMR_ENV("RMR_SLOT_RESERVE")) c->slot_reserve = std::max(0, std::atoi(e));
    if (const char* e = RMR_ENV("RMR_LAUNCH_STREAMS")) {   // (experiments; the slots go at the next launch)
        (void)free_slots(c);
        c->launch_streams = std::max(0, std::min(4, std::atoi(e)));
    }
    c->scene_loaded = true;
    c->jit_ready = false;
    c->jit_failed = false;
    c->stats.flops_per_map = s.flops_per_map();
    return RMR_OK;
}

// Compile (or fetch from the cache) and load the specialised trace kernel of the loaded scene.
int ensure_jit(rmr_ctx* c) {
    if (c->jit_ready) return RMR_OK;
    // animation: same structure as the last specialised scene, different numbers -> the primitives
    // that changed since the kernel's baked values become loads ("live"), the others stay literals:
    // one compile when the motion starts, then the same kernel every frame
    const std::string struct_src = rmr::jit_source(c->scene, c->has_prog, false, c->cull);
    const auto& prims = c->scene.prims;
    if (struct_src != c->jit_struct_src || c->jit_base.size() != prims.size()) {   // new layout
        c->jit_base = prims;
        c->jit_live.assign(prims.size(), 0);
    } else {
        for (size_t j = 0; j < prims.size(); j++)
            if (std::memcmp(&prims[j], &c->jit_base[j], sizeof(rmr_prim)) != 0) c->jit_live[j] = 1;
    }
    c->jit_struct_src = struct_src;
    // one cached primitive when the cache's full map() runs through the candidate grid (csg256: 21.5 ->
    // 17.4 ms per 4 spp against two); two with the BVH full map
    int npc_k = (c->map_np == -2 && c->grid_on) ? 1 : 2;
    if (const char* e = RMR_ENV("RMR_NPC_KSEL")) npc_k = std::atoi(e) == 1 ? 1 : 2;   // (experiments)
    const bool npc_spheres = c->map_np == -2 && c->grid_on && c->grid_small_spheres;
    rmr::JitFacts facts;
    const std::string src = rmr::jit_source(c->scene, c->has_prog, true, c->cull, &c->jit_live, npc_k, npc_spheres, &facts);
    std::vector<char> code;
    std::string key, log;
    std::vector<std::string> opts;
    if (c->instrument & RMR_INSTR_COUNT_FLOPS) opts.push_back("-DRMR_COUNT_FLOPS");
    if (!rmr::jit_compile(src, code, key, log, opts)) {
        c->jit_failed = true;
        return fail(c, RMR_E_HIP, "hipRTC specialisation failed: " + log.substr(0, 2000));
    }
    for (const auto& k : c->jit_loaded) {
        if (k.key == key) {
            c->jit = k;
            c->jit_ready = true;
            return RMR_OK;
        }
    }
    rmr::JitKernel k;
    k.key = key;
    // a code object that does not load (e.g. a stale disk-cache entry) marks the scene as failed, so
    // auto mode falls back to the ahead-of-time kernels instead of retrying every launch
    if (hipModuleLoadData(&k.module, code.data()) != hipSuccess) {
        c->jit_failed = true;
        return fail(c, RMR_E_HIP, "hipModuleLoadData of the specialised kernel failed (key " + key + ")");
    }
    if (hipModuleGetFunction(&k.fn, k.module, "rmr_jit_trace") != hipSuccess) {
        (void)hipModuleUnload(k.module);
        c->jit_failed = true;
        return fail(c, RMR_E_HIP, "rmr_jit_trace missing from the specialised code object (key " + key + ")");
    }
    k.block = 256;
    k.chunk = facts.chunk();
    int b = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&b, k.fn, k.block, 0) != hipSuccess || b <= 0) b = 4;
    k.blocks_per_cu = b;
    // shading batch per kernel class (rmr_jit.hpp JitFacts::shade_t). Measured: the Mandelbulb 10 (8
    // until round 5's early bailout made the passes cheaper: 10 -0.6%, csg_nodes -0.5%); RM1 inline sphere/box maps 16 (20 until the map() loop lost ~12% of its instructions in
    // round 2; then 14-16 best on Cornell-5, 20 -> 16: -2.4%, multilight -4%, default +1.2%); node-program
    // materials 20 (round 4, 1080p 16 spp: default.scene 27.9 -> 26.9 ms, multilight 13.41 -> 13.24; 24:
    // -6% / +1.4%); the cache kernels 20 (csg256 1080p 8 spp: 16.83 -> 16.68 ms; 24: 16.81); the
    // certified sphere/box kernels at 7 waves 20 (Cornell-5 1080p 64 spp: 47.17 -> 46.63 ms; 18: 46.77,
    // 14: 47.92)
    k.shade_t = facts.shade_t();
    c->jit_loaded.push_back(k);
    c->jit = k;
    c->jit_ready = true;
    return RMR_OK;
}

namespace {
struct BvhItem {
    float lo[3], hi[3], cen[3];
    int idx;
};
int bvh_leaf_size() {   // primitives per BVH leaf (env RMR_BVH_LEAF: experiments), read at scene upload
    if (const char* e = RMR_ENV("RMR_BVH_LEAF")) return std::max(1, std::min(16, std::atoi(e)));
    return 8;   // csg256 4 spp: 2 / 3 / 4 / 6 / 8 / 12 / 16 -> 37.0 / 36.1 / 34.1 / 33.3 / 32.9 / 33.1 / 33.6 ms
}
void bvh_build(std::vector<BvhItem>& it, int l, int r, std::vector<rmr::BvhNode>& nodes, std::vector<int>& order) {
    const int me = (int)nodes.size();
    nodes.push_back(rmr::BvhNode{});
    rmr::BvhNode nd{};
    for (int k = 0; k < 3; k++) { nd.lo[k] = 3.0e38f; nd.hi[k] = -3.0e38f; }
    float clo[3] = {3.0e38f, 3.0e38f, 3.0e38f}, chi[3] = {-3.0e38f, -3.0e38f, -3.0e38f};
    for (int i = l; i < r; i++)
        for (int k = 0; k < 3; k++) {
            nd.lo[k] = std::min(nd.lo[k], it[i].lo[k]);
            nd.hi[k] = std::max(nd.hi[k], it[i].hi[k]);
            clo[k] = std::min(clo[k], it[i].cen[k]);
            chi[k] = std::max(chi[k], it[i].cen[k]);
        }
    if (r - l <= bvh_leaf_size()) {
        std::sort(it.begin() + l, it.begin() + r, [](const BvhItem& a, const BvhItem& b) { return a.idx < b.idx; });
        nd.first = (int)order.size();
        nd.count = r - l;
        for (int i = l; i < r; i++) order.push_back(it[i].idx);
    } else {
        int ax = 0;
        for (int k = 1; k < 3; k++)
            if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
        const int mid = (l + r) / 2;
        std::nth_element(it.begin() + l, it.begin() + mid, it.begin() + r,
                         [ax](const BvhItem& a, const BvhItem& b) { return a.cen[ax] < b.cen[ax]; });
        nd.first = -1;
        nd.count = 0;
        bvh_build(it, l, mid, nodes, order);
        bvh_build(it, mid, r, nodes, order);
    }
    nd.skip = (int)nodes.size();
    nodes[(size_t)me] = nd;
}
}  // namespace

// Candidate grid over the small primitives (leaf order [n_large, n)) of a BVH scene, for the nearest-
// primitive cache's full map() (rmr_trace.h map_grid_npc). Per cell C (inflated past the kernel's
// rounding of the cell index): U = the smallest distance upper bound over C of any primitive (box and
// sphere SDFs are convex: the maximum is at a corner); the list = the small primitives whose distance
// lower bound over C is <= U + margin (margin = 4 x the float evaluation error bound of a distance
// anywhere in the grid, so an unlisted primitive's float distance is strictly above the minimum's);
// the cell's bound = the smallest lower bound of an unlisted one, minus that error bound. Exact
// arithmetic in double; cells of more than 254 candidates keep the BVH (count 255).
// Env (experiments): RMR_GRID=0 off, RMR_GRID_CELLS (target cell count), RMR_GRID_PAD (region pad).
// The construction is host code (grid.cpp, build_candidate_grid); this uploads it.
int build_grid(rmr_ctx* c, const std::vector<rmr::DPrim>& dp, int n_large, double E) {
    c->grid_on = false;
    if (const char* e = RMR_ENV("RMR_GRID")) if (std::atoi(e) == 0) return RMR_OK;
    // 2^20 cells (round 3; csg256 1080p 8 spp, same process: 2^18 21.1, 2^19 20.2, 2^20 19.9 ms,
    // flat beyond; 16 MB of cell records, ~0.4 s to build on 16 host threads)
    double target = 1048576.0, pad = 0.5;
    if (const char* e = RMR_ENV("RMR_GRID_CELLS")) target = std::max(1.0, std::atof(e));
    if (const char* e = RMR_ENV("RMR_GRID_PAD")) pad = std::max(0.0, std::atof(e));
    rmr::CandidateGrid g;
    if (!rmr::build_candidate_grid(dp, n_large, E, target, pad, g)) return RMR_OK;
    int r;
    // device cells: the host record (offset | count, bound) plus the list's first four entries
    // inline, so most full-map lanes read their candidates without a dependent list load
    const size_t ncell = g.cells.size() / 2;
    if (ncell >= ((size_t)1 << 31)) return RMR_OK;   // the kernel's cell index is 32-bit (map_grid_npc)
    std::vector<uint4> cells4(ncell);
    for (size_t i = 0; i < ncell; i++) {
        const uint32_t x = g.cells[2 * i], off = x & 0xffffffu, cnt = x >> 24;
        uint32_t e[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < 4 && cnt != 255u && k < cnt; k++) e[k] = g.list[off + k];
        cells4[i] = make_uint4(x, g.cells[2 * i + 1], e[0] | (e[1] << 16), e[2] | (e[3] << 16));
    }
    if ((r = dev_upload(c, &c->d_grid, cells4.data(), cells4.size()))) return r;
    if ((r = dev_upload(c, &c->d_grid_list, g.list.data(), g.list.size()))) return r;
    for (int k = 0; k < 3; k++) { c->grid_lo[k] = g.lo[k]; c->grid_dim[k] = g.dim[k]; }
    for (int k = 0; k < 6; k++) c->grid_sbox[k] = g.sbox[k];
    c->grid_inv = g.inv;
    c->grid_n_large = n_large;
    c->grid_small_spheres = true;
    for (size_t k = (size_t)n_large; k < dp.size(); k++)
        c->grid_small_spheres = c->grid_small_spheres && (dp[k].type & 0xff) == RMR_PRIM_SPHERE;
    c->grid_on = true;
    return RMR_OK;
}

// Bounding boxes of a BVH scene's primitives, and which are "large": primitives much larger than the
// typical one (ground planes, walls) would make every box above them cover the scene, so they go
// first, in an always-visited leaf (infinite bounds), which also gives the running minimum a small
// value early; the candidate grid lists only the others. Shared by upload_bvh and
// rmr_jit_compile_scene (the cache kernel's RMR_NPC_SPHERES depends on the split).
std::vector<BvhItem> bvh_items(const CompiledScene& s, std::vector<char>& is_large, float& extent) {
    std::vector<BvhItem> items;
    extent = 0.0f;
    for (size_t i = 0; i < s.prims.size(); i++) {
        const rmr_prim& p = s.prims[i];
        BvhItem b{};
        for (int k = 0; k < 3; k++) {
            const float h = (p.type == RMR_PRIM_SPHERE) ? std::fabs(p.r[0]) : std::fabs(p.r[k]);
            b.lo[k] = p.c[k] - h;
            b.hi[k] = p.c[k] + h;
            b.cen[k] = p.c[k];
            extent = std::max(extent, std::fabs(p.c[k]) + h);
        }
        b.idx = (int)i;
        items.push_back(b);
    }
    std::vector<float> ext;
    for (const auto& b : items) ext.push_back(std::max({b.hi[0] - b.lo[0], b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]}));
    std::vector<float> sorted_ext = ext;
    is_large.assign(items.size(), 0);
    if (items.empty()) return items;
    std::nth_element(sorted_ext.begin(), sorted_ext.begin() + sorted_ext.size() / 2, sorted_ext.end());
    const float big = 8.0f * sorted_ext[sorted_ext.size() / 2];
    for (size_t i = 0; i < items.size(); i++) is_large[i] = ext[i] > big;
    return items;
}

int upload_bvh(rmr_ctx* c) {
    const CompiledScene& s = c->scene;
    std::vector<char> is_large;
    float extent = 0.0f;
    const std::vector<BvhItem> items = bvh_items(s, is_large, extent);
    std::vector<BvhItem> small, large;
    for (size_t i = 0; i < items.size(); i++) (is_large[i] ? large : small).push_back(items[i]);
    std::vector<rmr::BvhNode> nodes;
    std::vector<int> order;
    if (!large.empty()) {
        for (size_t at = 0; at < large.size(); at += 4) {  // leaves of <= 4, all always visited
            rmr::BvhNode nd{};
            for (int k = 0; k < 3; k++) { nd.lo[k] = -3.0e38f; nd.hi[k] = 3.0e38f; }
            nd.first = (int)order.size();
            nd.count = (int)std::min<size_t>(4, large.size() - at);
            for (int i = 0; i < nd.count; i++) order.push_back(large[at + (size_t)i].idx);
            nd.skip = (int)nodes.size() + 1;
            nodes.push_back(nd);
        }
    }
    if (!small.empty()) bvh_build(small, 0, (int)small.size(), nodes, order);
    std::vector<rmr::DPrim> dp(order.size());
    for (size_t k = 0; k < order.size(); k++) {
        const rmr_prim& p = s.prims[(size_t)order[k]];
        rmr::DPrim q{};
        for (int i = 0; i < 3; i++) { q.c[i] = p.c[i]; q.r[i] = p.r[i]; }
        q.type = p.type | (order[k] << 8);
        q.mat_id = p.mat_id;
        dp[k] = q;
    }
    int r;
    if ((r = dev_upload(c, &c->d_dprims, dp.data(), dp.size()))) return r;
    if ((r = dev_upload(c, &c->d_bvh, nodes.data(), nodes.size()))) return r;
    c->bvh_host = nodes;
    c->bvh_order = order;
    c->n_bvh = (int)nodes.size();
    c->bvh_margin = 1e-4f + extent * 0x1p-16f;
    double E = 0.0;   // max |c|_inf + |r|_inf (as render_tiles' npc_eps0)
    for (const rmr_prim& q : s.prims) {
        const double rr = q.type == RMR_PRIM_SPHERE ? std::fabs(q.r[0])
                                                    : std::max({std::fabs(q.r[0]), std::fabs(q.r[1]), std::fabs(q.r[2])});
        E = std::max(E, std::max({std::fabs((double)q.c[0]), std::fabs((double)q.c[1]), std::fabs((double)q.c[2])}) + rr);
    }
    int n_large = 0;
    for (const rmr::BvhNode& nd : nodes) {   // the always-visited leaves come first (leaf order 0 ..)
        if (nd.lo[0] > -1e38f) break;
        n_large += nd.count;
    }
    return build_grid(c, dp, n_large, E);
}

int validate_scene(rmr_ctx* c, const CompiledScene& s) {
    for (const auto& p : s.prims) {
        if (p.type < RMR_PRIM_SPHERE || p.type > RMR_PRIM_MANDELBULB) return fail(c, RMR_E_SCENE, "bad prim type");
        if (p.type == RMR_PRIM_PROGRAM) {
            if (p.prog_begin < 0 || p.prog_end > (int)s.ops.size() || p.prog_begin > p.prog_end)
                return fail(c, RMR_E_SCENE, "prim program range out of bounds");
            if (p.dist_var < 0 || p.dist_var >= RMR_MAX_VARS) return fail(c, RMR_E_SCENE, "bad dist_var");
        }
    }
    const int nconst = (int)(s.consts.size() / 3);
    for (const auto& o : s.ops) {
        for (int i = 0; i < 7; i++) {
            const int r = o.in[i];
            if (r == RMR_OPND_NONE || r == RMR_OPND_P) continue;
            if (RMR_OPND_IS_CONST(r)) {
                if (RMR_OPND_CONST_INDEX(r) >= nconst) return fail(c, RMR_E_SCENE, "constant index out of range");
            } else if (r < 0 || r >= RMR_MAX_VARS) {
                return fail(c, RMR_E_SCENE, "var index out of range");
            }
        }
        for (int i = 0; i < 4; i++)
            if (o.out[i] >= RMR_MAX_VARS) return fail(c, RMR_E_SCENE, "var index out of range");
    }
    for (const auto& m : s.materials)
        if (m.defined && (m.prog_begin < 0 || m.prog_end > (int)s.ops.size())) return fail(c, RMR_E_SCENE, "material program range");
    if (s.variant == RMR_VARIANT_RM2 && (s.v2_begin < 0 || s.v2_end > (int)s.ops.size()))
        return fail(c, RMR_E_SCENE, "v2 program range");
    return RMR_OK;
}

int ensure_samp(rmr_ctx* c, size_t n) {
    if (n <= c->samp_cap) return RMR_OK;
    if (c->d_samp) { (void)hipFree(c->d_samp); c->d_samp = nullptr; c->samp_cap = 0; }
    HIPCHK(c, hipMalloc((void**)&c->d_samp, n * sizeof(float4)));
    c->samp_cap = n;
    return RMR_OK;
}


// Create every launch slot's stream, events and work queue (rmr_create, rmr_set_launch_streams: a
// stream created at a slot's first launch cost that launch ~6 ms, r06s_timeline_full_ls2.txt).
int make_slots(rmr_ctx* c) {
    c->slots.resize(c->launch_streams >= 2 ? (size_t)c->launch_streams : 0);
    c->next_slot = 0;
    for (auto& S : c->slots) {
        if (S.s) continue;
        HIPCHK(c, hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&S.freed, hipEventDisableTiming));
        HIPCHK(c, hipMalloc((void**)&S.queue, rmr::kQueueBytes));
        S.queue_dirty = true;
    }
    return RMR_OK;
}

// The next launch slot, for `units` sample-plane entries. Planes grow for every slot at once (the
// launches that follow are the same size: no allocation inside a run of them), each once the fold
// that last read it is done; the slot's stream then waits for that fold.
int slot_prepare(rmr_ctx* c, size_t units, rmr_ctx::Slot** out) {
    int r;
    if (c->slots.empty() || !c->slots[0].s) {
        if ((r = make_slots(c))) return r;
    }
    if (units > c->slots[c->next_slot].cap) {
        for (auto& T : c->slots) {
            if (units <= T.cap) continue;
            if (T.samp) {
                if (T.in_use) HIPCHK(c, hipEventSynchronize(T.freed));
                (void)hipFree(T.samp);
                T.samp = nullptr;
                T.cap = 0;
            }
            HIPCHK(c, hipMalloc((void**)&T.samp, units * sizeof(float4)));
            T.cap = units;
        }
    }
    rmr_ctx::Slot& S = c->slots[c->next_slot];
    c->next_slot = (c->next_slot + 1) % c->slots.size();
    if (S.in_use) HIPCHK(c, hipStreamWaitEvent(S.s, S.freed, 0));
    *out = &S;
    return RMR_OK;
}

// Release the launch slots (the context's stream synced first: every trace queued is done).
int free_slots(rmr_ctx* c) {
    if (c->slots.empty() && !c->trace_end) return RMR_OK;
    const hipError_t e = c->stream ? hipStreamSynchronize(c->stream) : hipSuccess;
    for (auto& S : c->slots) {
        if (S.s) {
            (void)hipStreamSynchronize(S.s);
            (void)hipStreamDestroy(S.s);
        }
        if (S.done) (void)hipEventDestroy(S.done);
        if (S.freed) (void)hipEventDestroy(S.freed);
        if (S.samp) (void)hipFree(S.samp);
        if (S.queue) (void)hipFree(S.queue);
    }
    c->slots.clear();
    c->next_slot = 0;
    if (c->trace_end) (void)hipEventDestroy(c->trace_end);
    c->trace_end = nullptr;
    c->last_samp = c->d_samp;
    if (e != hipSuccess) return fail(c, RMR_E_HIP, std::string("launch slots: ") + hipGetErrorString(e));
    return RMR_OK;
}

constexpr size_t kTileCacheEntries = 64;

uint64_t tiles_hash(const std::vector<TileXY>& t) {
    uint64_t h = 1469598103934665603ull ^ t.size();
    for (const TileXY& v : t) {
        h = (h ^ (uint32_t)v.x) * 1099511628211ull;
        h = (h ^ (uint32_t)v.y) * 1099511628211ull;
    }
    return h;
}

// The device copy of a tile list (cached by content, see rmr_ctx::tile_cache).
int tile_list(rmr_ctx* c, const std::vector<TileXY>& t, const TileXY** out) {
    const uint64_t h = tiles_hash(t);
    auto same = [](const TileXY& a, const TileXY& b) { return a.x == b.x && a.y == b.y; };
    for (auto& e : c->tile_cache)
        if (e.hash == h && e.host.size() == t.size() && std::equal(t.begin(), t.end(), e.host.begin(), same)) {
            e.used = ++c->tile_clock;
            *out = e.dev;
            return RMR_OK;
        }
    if (c->tile_cache.size() >= kTileCacheEntries) {
        auto lru = std::min_element(c->tile_cache.begin(), c->tile_cache.end(),
                                    [](const rmr_ctx::TileList& a, const rmr_ctx::TileList& b) { return a.used < b.used; });
        HIPCHK(c, hipStreamSynchronize(c->stream));   // launches queued before may still read it
        (void)hipFree(lru->dev);
        c->tile_cache.erase(lru);
    }
    rmr_ctx::TileList e{t, nullptr, h, ++c->tile_clock};
    HIPCHK(c, hipMalloc((void**)&e.dev, std::max<size_t>(1, t.size()) * sizeof(TileXY)));
    // a new buffer no queued launch reads: a plain synchronous copy, no wait for the stream
    const hipError_t er = hipMemcpy(e.dev, t.data(), t.size() * sizeof(TileXY), hipMemcpyHostToDevice);
    if (er != hipSuccess) {
        (void)hipFree(e.dev);
        return fail(c, RMR_E_HIP, std::string("tile list upload: ") + hipGetErrorString(er));
    }
    c->tile_cache.push_back(std::move(e));
    *out = c->tile_cache.back().dev;
    return RMR_OK;
}

// The launch's seeds on the device (launches of more than one sample; see rmr_ctx::h_times).
int stage_times(rmr_ctx* c, const float* times, uint32_t n, const float** out, hipStream_t st = nullptr) {
    if (!st) st = c->stream;
    if (n > c->times_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_times) (void)hipFree(c->d_times);
        if (c->h_times) (void)hipHostFree(c->h_times);
        c->d_times = nullptr;
        c->h_times = nullptr;
        c->times_cap = c->times_pos = 0;
        const size_t cap = std::max<size_t>(n, (size_t)1 << 16);
        HIPCHK(c, hipMalloc((void**)&c->d_times, cap * sizeof(float)));
        HIPCHK(c, hipHostMalloc((void**)&c->h_times, cap * sizeof(float), hipHostMallocDefault));
        c->times_cap = cap;
    }
    if (c->times_pos + n > c->times_cap) {   // wrap: every copy and launch that used the ring is done
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->times_pos = 0;
    }
    float* h = c->h_times + c->times_pos;
    float* d = c->d_times + c->times_pos;
    std::memcpy(h, times, n * sizeof(float));
    // (on a slot's stream, the copy is covered by the context stream's syncs above: the slot's trace
    // follows it there, and the trace's fold on the context stream waits for the trace)
    HIPCHK(c, hipMemcpyAsync(d, h, n * sizeof(float), hipMemcpyHostToDevice, st));
    c->times_pos += n;
    *out = d;
    return RMR_OK;
}

EventPair get_events(rmr_ctx* c) {
    if (!c->pool.empty()) {
        EventPair e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    EventPair e;
    (void)hipEventCreate(&e.a);
    (void)hipEventCreate(&e.b);
    (void)hipEventCreate(&e.c);
    return e;
}

int collect_timing(rmr_ctx* c) {
    for (auto& e : c->pending) {
        HIPCHK(c, hipEventSynchronize(e.c));
        float t1 = 0, t2 = 0;
        (void)hipEventElapsedTime(&t1, e.a, e.b);
        (void)hipEventElapsedTime(&t2, e.b, e.c);
        c->stats.trace_ms += t1;
        c->stats.fold_ms += t2;
        c->pool.push_back(e);
    }
    c->pending.clear();
    return RMR_OK;
}

// The launch's escape bound (rmr_trace.h ray_exit): the escape boxes inflated by 0.002 + 2^-16 (|eye| +
// 2E + 3 maxDist) >= 0.001 + 8 x the float error of a distance at any point a march reaches
// (|p| <= |eye| + E + 3 maxDist) + the rounding of the slab parameters
int escape_params(rmr_ctx* c, KParams& P) {
    const CompiledScene& s = c->scene;
    bool simple = !s.prims.empty();
    double E = 0.0;
    for (const rmr_prim& q : s.prims) {
        simple = simple && escape_prim(q);
        if (!escape_prim(q)) continue;
        for (int k = 0; k < 3; k++) E = std::max(E, std::fabs((double)q.c[k]) + (double)escape_halfwidth(q, k));
    }
    double eye = 0.0;
    for (int k = 0; k < 3; k++) eye = std::max(eye, std::fabs((double)c->view[k]));
    const double infl = 0.002 + std::ldexp(eye + 2.0 * E + 3.0 * std::fabs((double)c->params.max_dist), -16);
    // (infl < 2^44: |eye|, E, maxDist < 2^60, the range ray_exit's FMA slab form is exact in)
    P.esc_on = (c->cull & RMR_CULL_ESCAPE) && simple && infl < 0x1p44 && !c->esc_raw.empty() ? 1 : 0;
    if (P.esc_on && infl != c->esc_infl_dev) {
        std::vector<float> bx(c->esc_raw.size());
        for (size_t i = 0; i < bx.size(); i++)   // outward in double, then to float
            bx[i] = (float)((double)c->esc_raw[i] + ((i % 6) < 3 ? -infl : infl));
        int rr;
        if ((rr = dev_upload(c, &c->d_esc, bx.data(), bx.size()))) return rr;
        c->esc_infl_dev = infl;
    }
    P.esc_boxes = c->d_esc;
    P.n_esc = (int)(c->esc_raw.size() / 6);
    return RMR_OK;
}

// Core: nspp samples over an 8x8 tile list, clipped to [x0,x1)x[y0,y1).
int render_tiles(rmr_ctx* c, const std::vector<TileXY>& tiles, int x0, int y0, int x1, int y1,
                 const float* times, uint32_t first_sample, uint32_t nspp) {
    if (!c->scene_loaded) return fail(c, RMR_E_STATE, "no scene loaded (call rmr_load_scene_json / rmr_load_builtin_scene)");
    if (c->params.use_env_tex && !c->d_env) return fail(c, RMR_E_STATE, "useEnvTex != 0 but no env map (rmr_set_env_map)");
    if (tiles.empty() || nspp == 0) return RMR_OK;
    if (!c->view_set) default_view(c);
    int r;
    const TileXY* d_tiles = nullptr;
    if ((r = tile_list(c, tiles, &d_tiles))) return r;
    const size_t plane = tiles.size() * 64;
    size_t chunk = std::max<size_t>(1, c->samp_budget / (plane * sizeof(float4)));
    chunk = std::min<size_t>(chunk, nspp);
    // the trace kernel indexes units with 32 bits (atomic work counter included): < 2^31 per launch
    chunk = std::max<size_t>(1, std::min<size_t>(chunk, ((size_t)1 << 31) / plane));
    // slots for launches whose planes fit the budget shared between the slots (larger ones, C4's 34-GB
    // 4K 256-spp frame, run on the context's stream: one plane buffer of them is enough)
    const bool slotted = c->launch_streams >= 2 && plane * chunk * sizeof(float4) <= c->samp_budget / (size_t)c->launch_streams;
    if (slotted && c->slots.size() != (size_t)c->launch_streams) {
        if ((r = free_slots(c)) || (r = make_slots(c))) return r;
    }
    const float* d_times = nullptr;

    const CompiledScene& s = c->scene;
    KParams P{};
    P.prims = c->d_prims; P.ops = c->d_ops; P.consts = c->d_consts; P.mats = c->d_mats;
    P.spec = c->d_spec; P.rm2 = c->d_rm2;
    P.dprims = c->d_dprims; P.dmats = c->d_dmats;
    P.bvh = c->d_bvh; P.n_nodes = c->n_bvh; P.bvh_margin = c->bvh_margin;
    if (c->grid_on && c->map_np == -2) {
        P.grid = c->d_grid; P.grid_list = c->d_grid_list; P.grid_inv = c->grid_inv; P.grid_n_large = c->grid_n_large;
        for (int k = 0; k < 3; k++) {
            P.grid_lo[k] = c->grid_lo[k];
            P.grid_dim[k] = c->grid_dim[k];
            P.grid_dimf[k] = (float)c->grid_dim[k];
        }
        for (int k = 0; k < 6; k++) P.grid_sbox[k] = c->grid_sbox[k];
    }
    P.n_prims = (int)s.prims.size();
    P.am_r2 = 2.0f * rmr::max_sphere_radius(s);
    {
        float E = 0.0f;   // max |c|_inf + |r|_inf: scale of the float error of a box/sphere distance
        for (const rmr_prim& q : s.prims) {
            const float rr = q.type == RMR_PRIM_SPHERE ? std::fabs(q.r[0])
                                                       : std::max({std::fabs(q.r[0]), std::fabs(q.r[1]), std::fabs(q.r[2])});
            E = std::max(E, std::max({std::fabs(q.c[0]), std::fabs(q.c[1]), std::fabs(q.c[2])}) + rr);
        }
        P.npc_eps0 = E * 0x1p-17f + 0x1p-60f;
        // rmr_trace.h am_normal_cert: (0.002 + 2R) 2^-20 + 2^-39 + 4 eps + 2 delta with eps the npc_eps
        // bound at |p|_inf <= E + 0.005 (a hit's probes), in double, widened by 2^-20 for the kernel
        // fma's rounding and rounded up to float
        const double eps = ((double)E + 0.005) * 0x1p-17 + (double)P.npc_eps0;
        const double k0 = (0.002 + (double)P.am_r2) * 0x1p-20 + 0x1p-39 + 4.0 * eps + 2.0 * 0.0010001;
        P.cert_k = std::nextafter((float)(k0 * (1.0 + 0x1p-20)), INFINITY);
    }
    P.full_threshold = c->full_threshold;
    {
        int rr;
        if ((rr = escape_params(c, P))) return rr;
    }
    {
        // primary rays' first march step from the eye (rmr_trace.h eye_map): the march point
        // fma(dir, 0, eye) is the eye itself for every finite direction unless an eye coordinate is
        // -0 (then it is +-0 by the direction's sign), so that case keeps the per-lane step
        bool neg0 = false;
        for (int k = 0; k < 3; k++)
            neg0 = neg0 || (c->view[k] == 0.0f && std::signbit(c->view[k])) || !std::isfinite(c->view[k]);
        P.eye_step = (c->cull & RMR_CULL_EYE) && !neg0 ? 1 : 0;
    }
    P.n_mats = (int)(s.variant == RMR_VARIANT_RM3 ? s.spectral.size() : s.materials.size());
    P.v2_begin = s.v2_begin; P.v2_end = s.v2_end;
    P.spec_sky = s.spectral_sky;
    P.env = c->d_env; P.env_w = c->env_w; P.env_h = c->env_h;
    P.use_env = (c->params.use_env_tex != 0 && c->d_env) ? 1 : 0;
    for (int i = 0; i < 3; i++) { P.sky[i] = s.sky[i]; P.rm2_light[i] = s.rm2.light_pos[i]; }
    P.rm2_light_power = s.rm2.light_power;
    P.rm2_node_id = s.rm2.node_mat_id;
    P.max_dist = c->params.max_dist; P.step_mult = c->params.step_multiply;
    P.max_steps = c->params.max_steps; P.max_bounces = c->params.max_bounces;
    P.separate_channels = c->params.separate_channels;
    for (int i = 0; i < 3; i++) {
        P.eye[i] = c->view[i]; P.r00[i] = c->view[3 + i]; P.r01[i] = c->view[6 + i];
        P.r10[i] = c->view[9 + i]; P.r11[i] = c->view[12 + i];
    }
    P.W = c->W; P.H = c->H;
    for (int i = 0; i < 3; i++) {
        P.dr01[i] = P.r01[i] - P.r00[i];   // float subtraction: the bits fmix's y - x gives
        P.dr11[i] = P.r11[i] - P.r10[i];
    }
    P.Wf = (float)c->W; P.Hf = (float)c->H;
    P.env_wf[0] = (float)c->env_w; P.env_wf[1] = (float)c->env_h;
    P.env_wf[2] = (float)(c->env_w - 1); P.env_wf[3] = (float)(c->env_h - 1);
    P.eye_xy = P.eye[0] + P.eye[1];
    P.x0 = x0; P.y0 = y0; P.x1 = x1; P.y1 = y1;
    P.tiles = d_tiles;
    P.n_tiles = (int)tiles.size();
    P.samp = c->d_samp;
    P.accum = c->d_accum;
    P.queue = c->d_queue;
    P.counters = c->d_counters;
    P.flops_static = (int32_t)s.flops_per_map();
    P.transc_static = (int32_t)s.transc_per_map();
    P.shade_threshold = c->shade_threshold;
    P.refill_threshold = refill_for(c->refill_threshold, c->shade_threshold);

    // hipRTC specialisation for large launches (always when jit_mode == 1)
    bool use_jit = false;
    if (c->kernel_mode == 0 && c->jit_mode != 0 && !(c->jit_mode == 2 && c->jit_failed)) {
        const uint64_t units = (uint64_t)std::min<size_t>(chunk, nspp) * plane;
        if (c->jit_mode == 1 || units >= c->jit_min_units) {
            const int jr = ensure_jit(c);
            if (jr == RMR_OK) use_jit = true;
            else if (c->jit_mode == 1) return jr;
        }
    }
    int bpc = c->grid_per_cu;
    if (bpc <= 0) {
        if (use_jit) bpc = c->jit.blocks_per_cu;
        else if (rmr::trace_occupancy(s.variant, c->map_np, c->has_prog, &bpc) != 0 || bpc <= 0) bpc = 4;
    }
    const int full_grid = c->n_cu * bpc;
    for (uint32_t k0 = 0; k0 < nspp; k0 += (uint32_t)chunk) {
        const uint32_t n = (uint32_t)std::min<size_t>(chunk, nspp - k0);
        // a slot only while the previous trace is still running (something to overlap); otherwise the
        // context's stream, with no stream hop (one launch per frame, then a sync: r06t_slot_ab.log)
        rmr_ctx::Slot* S = nullptr;
        if (slotted && c->trace_end && hipEventQuery(c->trace_end) == hipErrorNotReady) {
            if ((r = slot_prepare(c, plane * n, &S))) return r;
            P.samp = S->samp;
            P.queue = S->queue;
        } else {
            if ((r = ensure_samp(c, plane * n))) return r;
            P.samp = c->d_samp;
            P.queue = c->d_queue;
        }
        d_times = nullptr;
        if (n > 1 && (r = stage_times(c, times + k0, n, &d_times, S ? S->s : c->stream))) return r;
        c->last_samp = P.samp;
        P.nspp = n;
        P.first_sample = first_sample + k0;
        P.times = d_times;
        P.time1 = times[k0];   // the seed when this launch has one sample (unit_pixel)
        P.n_units = (uint64_t)n * plane;
        // a persistent grid no larger than the launch's work: one work chunk per wave at most (a
        // 256x256 1-spp launch (C1) on the full grid: 0.47 ms, almost all of it waves that find no
        // work; the per-path kernel takes one wave per 64 units as it is). Waves per block and units
        // per chunk of the kernel that runs.
        // A launch with less work than one chunk per wave of the grid (a tile of one sample: the
        // reference's Graphics::Render call) takes smaller claims instead, down to small_chunk units,
        // so its paths spread over more CUs rather than running after one another in a few waves.
        // 480x270 tiles of one sample, same process (r06m_small_chunk.log), 64 against 128 units:
        // Cornell-5 -21%, RM3 -7%, Mandelbulb -18%; 32 / 16 slower again. Single-bounce paths are too
        // short for it (C1's 256x256 frame +6%): those launches keep the kernel's chunk.
        int grid = full_grid;
        P.chunk_units = 0;
        if (c->kernel_mode == 0 && c->grid_per_cu <= 0) {
            const uint64_t wpb = (uint64_t)((use_jit ? c->jit.block : 256) / 64), kchunk = use_jit ? c->jit.chunk : 128;
            // slotted launches leave workgroups free for the previous launch's fold, which waits behind
            // the next trace's persistent workgroups otherwise (and the slot's reuse behind that fold)
            const int reserve = (S && c->grid_reserve == 0) ? c->slot_reserve : c->grid_reserve;
            const uint64_t avail = (uint64_t)std::max(1, full_grid - reserve);
            uint64_t ck = kchunk;
            if (c->small_chunk > 0 && P.max_bounces >= 2 && P.n_units < avail * wpb * kchunk)
                ck = std::min(kchunk, std::max<uint64_t>((uint64_t)c->small_chunk, (P.n_units + avail * wpb - 1) / (avail * wpb)));
            if (ck < kchunk) P.chunk_units = (uint32_t)ck;
            const uint64_t want = (P.n_units + wpb * ck - 1) / (wpb * ck);
            grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(avail, want));
        }
        // tuned shading batch size of the kernel that runs (measured: C2 +2% at 20; the Mandelbulb
        // and the cached BVH map -1..2%)
        if (c->shade_auto) {
            P.shade_threshold = use_jit ? c->jit.shade_t : 16;
            P.refill_threshold = refill_for(c->refill_threshold, P.shade_threshold);
        }
        const hipStream_t ts = S ? S->s : c->stream;   // the trace's stream
        bool& qdirty = S ? S->queue_dirty : c->queue_dirty;
        if (qdirty) HIPCHK(c, hipMemsetAsync(P.queue, 0, rmr::kQueueBytes, ts));
        qdirty = true;   // until the fold that zeroes it is queued
        EventPair ev = get_events(c);
        HIPCHK(c, hipEventRecord(ev.a, ts));
        hipError_t le;
        if (use_jit) {
            void* args[] = {&P};
            le = hipModuleLaunchKernel(c->jit.fn, (unsigned)grid, 1, 1, (unsigned)c->jit.block, 1, 1, 0, ts, args, nullptr);
            if (le == hipSuccess) c->stats.jit_launches++;
        } else {
            le = rmr::launch_trace(P, s.variant, c->map_np, c->has_prog, c->kernel_mode == 0, grid, ts);
        }
        if (le == hipSuccess) le = hipEventRecord(ev.b, ts);
        if (le == hipSuccess && c->launch_streams >= 2) {
            if (!c->trace_end) le = hipEventCreateWithFlags(&c->trace_end, hipEventDisableTiming);
            if (le == hipSuccess) le = hipEventRecord(c->trace_end, ts);
        }
        if (S) {
            // the context's stream waits for the trace before its fold (and before anything after it)
            if (le == hipSuccess) le = hipEventRecord(S->done, ts);
            if (le == hipSuccess) le = hipStreamWaitEvent(c->stream, S->done, 0);
            if (le != hipSuccess) (void)hipStreamSynchronize(ts);   // nothing of this slot left running
        }
        if (le != hipSuccess) return fail(c, RMR_E_HIP, std::string("trace launch: ") + hipGetErrorString(le));
        // (RMR_DIAG_NO_FOLD: what the fold costs the frame, a timing experiment with a wrong accumulator;
        // the next launch then zeroes the queue with a memset)
        if (!c->diag_no_fold) {
            HIPCHK(c, rmr::launch_fold(P, c->stream));
            qdirty = false;
        }
        if (S) {
            HIPCHK(c, hipEventRecord(S->freed, c->stream));
            S->in_use = true;
        }
        HIPCHK(c, hipEventRecord(ev.c, c->stream));
        c->pending.push_back(ev);
        c->stats.trace_launches++;
        c->stats.samples += (uint64_t)n * plane;  // upper bound; exact count below
    }
    return RMR_OK;
}

std::vector<TileXY> rect_tiles(int x0, int y0, int x1, int y1) {
    std::vector<TileXY> t;
    for (int y = y0; y < y1; y += 8)
        for (int x = x0; x < x1; x += 8) t.push_back(TileXY{x, y});
    return t;
}

int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

bool batching_on(const rmr_ctx* c) {
    return c->call_batching > 0 || (c->call_batching < 0 && c->own_stream && !c->accum_external);
}

// deferred units beyond which rmr_render launches what it holds (2^28 units: 4 GiB of sample planes)
constexpr uint64_t kDeferredUnitsMax = (uint64_t)1 << 28;
constexpr size_t kDeferredRectsMax = 4096;

// Launch the deferred one-sample calls. Rects holding the same samples (same first index, same seeds)
// whose union is a rectangle go out as one launch over that rectangle (the reference's 4x4 grid, fixed
// or progressive: the whole grid in one launch); any other rect goes out as a launch of its own (a
// launch clips to one rect: a tile of a rect whose edge is off the 8-pixel grid reaches into its
// neighbour). Bitwise equal to the calls made one by one: each pixel gets the same samples with the same
// seeds in the same order, and the held rects are disjoint (rmr_render flushes before an overlapping
// call).
int flush_calls(rmr_ctx* c) {
    if (c->deferred.empty()) return RMR_OK;
    std::vector<rmr_ctx::Deferred> d;
    d.swap(c->deferred);
    c->deferred_units = 0;
    std::vector<char> done(d.size(), 0);
    for (size_t i = 0; i < d.size(); i++) {
        if (done[i]) continue;
        std::vector<size_t> grp;
        int bx0 = d[i].x0, by0 = d[i].y0, bx1 = d[i].x1, by1 = d[i].y1;
        uint64_t area = 0;
        for (size_t j = i; j < d.size(); j++) {
            if (done[j] || d[j].s0 != d[i].s0 || d[j].times.size() != d[i].times.size() ||
                std::memcmp(d[j].times.data(), d[i].times.data(), d[i].times.size() * sizeof(float)) != 0)
                continue;
            grp.push_back(j);
            done[j] = 1;
            bx0 = std::min(bx0, d[j].x0); by0 = std::min(by0, d[j].y0);
            bx1 = std::max(bx1, d[j].x1); by1 = std::max(by1, d[j].y1);
            area += (uint64_t)(d[j].x1 - d[j].x0) * (uint64_t)(d[j].y1 - d[j].y0);
        }
        const uint32_t n = (uint32_t)d[i].times.size();
        if (area == (uint64_t)(bx1 - bx0) * (uint64_t)(by1 - by0)) {   // disjoint rects filling their box
            const int r = render_tiles(c, rect_tiles(bx0, by0, bx1, by1), bx0, by0, bx1, by1, d[i].times.data(), d[i].s0, n);
            if (r) return r;
            continue;
        }
        for (size_t j : grp) {
            const int r = render_tiles(c, rect_tiles(d[j].x0, d[j].y0, d[j].x1, d[j].y1), d[j].x0, d[j].y0, d[j].x1,
                                       d[j].y1, d[j].times.data(), d[j].s0, n);
            if (r) return r;
        }
    }
    return RMR_OK;
}

}  // namespace

// every entry point but rmr_render (and the pure getters) first launches the deferred calls, so that
// whatever it reads, changes or orders sees them done in call order
#define RMR_FLUSH(c)                                                   \
    do {                                                               \
        if (!(c)->deferred.empty()) {                                  \
            const int rf_ = flush_calls(c);                            \
            if (rf_) return rf_;                                       \
        }                                                              \
    } while (0)

extern "C" {

const char* rmr_build_info(void) {
    return "rmr gfx950 (CDNA4): variants RM1/RM2/RM3; wave64 persistent path-state kernel; "
           "scalar-cached scene tables; -ffp-contract=off deterministic math";
}

void rmr_default_params(rmr_params* p) {
    if (!p) return;
    p->max_dist = 1000.0f;  // Graphics.cpp:326
    p->max_steps = 512;     // Graphics.cpp:327
    p->max_bounces = 16;    // Graphics.cpp:328
    p->step_multiply = 0.5f;  // Graphics.cpp:329
    p->separate_channels = 0; // Graphics.cpp:340
    p->use_env_tex = 0;       // Graphics.cpp:338
}

int rmr_create(rmr_ctx** out, int device) {
    if (!out) return RMR_E_INVALID;
    *out = nullptr;
    rmr_ctx* c = new (std::nothrow) rmr_ctx();
    if (!c) return RMR_E_NOMEM;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
        delete c;
        return RMR_E_HIP;
    }
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) { delete c; return RMR_E_HIP; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        c->n_cu = prop.multiProcessorCount;
        if (prop.totalGlobalMem > 0) c->samp_budget = std::min(c->samp_budget, (size_t)prop.totalGlobalMem / 4);
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return RMR_E_HIP; }
    c->own_stream = true;
    rmr_default_params(&c->params);
    if (hipMalloc((void**)&c->d_queue, rmr::kQueueBytes) != hipSuccess ||
        hipMalloc((void**)&c->d_counters, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_counters, 0, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_queue, 0, rmr::kQueueBytes) != hipSuccess) {   // then each fold zeroes it
        rmr_destroy(c);
        return RMR_E_HIP;
    }
    if (const char* e = RMR_ENV("RMR_SHADE_T")) {
        c->shade_threshold = std::max(1, std::atoi(e));
        c->shade_auto = false;
    }
    if (const char* e = RMR_ENV("RMR_REFILL_T")) c->refill_threshold = std::max(0, std::atoi(e));
    if (const char* e = RMR_ENV("RMR_ESC")) if (std::atoi(e) == 0) c->cull &= ~RMR_CULL_ESCAPE;
    if (const char* e = RMR_ENV("RMR_NPC")) if (std::atoi(e) == 0) c->cull &= ~RMR_CULL_NPC;
    if (const char* e = RMR_ENV("RMR_JIT_APPROX")) if (std::atoi(e) == 0) c->cull &= ~RMR_CULL_APPROX;
    if (const char* e = RMR_ENV("RMR_EYE")) if (std::atoi(e) == 0) c->cull &= ~RMR_CULL_EYE;
    if (const char* e = RMR_ENV("RMR_GRID_PER_CU")) c->grid_per_cu = std::max(0, std::atoi(e));
    if (const char* e = RMR_ENV("RMR_GRID_RESERVE")) c->grid_reserve = std::max(0, std::atoi(e));
    if (const char* e = RMR_ENV("RMR_JIT")) c->jit_mode = std::max(0, std::min(2, std::atoi(e)));
    // launch slots: 2 within HIP's default 4 hardware queues per process (the context's stream, two
    // slots, the caller's default stream); 4 where the process has 8 or more (GPU_MAX_HW_QUEUES, the
    // variable HIP reads): the per-call loop then runs at 511 against 356 Msamples/s (r06ze_api_ls.log)
    if (const char* e = std::getenv("GPU_MAX_HW_QUEUES"))
        if (std::atoi(e) >= 8) c->launch_streams = 4;
    if (alloc_accum(c) != RMR_OK || make_slots(c) != RMR_OK) { rmr_destroy(c); return RMR_E_HIP; }
    *out = c;
    return RMR_OK;
}

void rmr_destroy(rmr_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)free_slots(c);
    for (auto& e : c->pending) c->pool.push_back(e);
    for (auto& e : c->pool) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); (void)hipEventDestroy(e.c); }
    void* bufs[] = {c->d_prims, c->d_ops, c->d_consts, c->d_mats, c->d_spec, c->d_rm2, c->d_dprims, c->d_dmats, c->d_bvh, c->d_esc, c->d_env, c->d_samp,
                    c->d_times, c->d_queue, c->d_counters, c->d_srgb_thr, c->d_screen, c->d_grid, c->d_grid_list};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& e : c->tile_cache) (void)hipFree(e.dev);
    if (c->h_times) (void)hipHostFree(c->h_times);
    if (c->d_accum && !c->accum_external) (void)hipFree(c->d_accum);
    for (auto& k : c->jit_loaded)
        if (k.module) (void)hipModuleUnload(k.module);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rmr_last_error(const rmr_ctx* c) { return c ? c->err.c_str() : "null context"; }

int rmr_set_stream(rmr_ctx* c, void* s) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int r = free_slots(c);   // (every queued trace done)
    if (r) return r;
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    if (s) {
        c->stream = (hipStream_t)s;
        c->own_stream = false;
    } else {
        HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    // the slots' streams again, created after the context's stream (HIP hands out its hardware queues
    // in creation order: r06v_set_stream_slots.log)
    return make_slots(c);
}

int rmr_set_image_size(rmr_ctx* c, int w, int h) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (w <= 0 || h <= 0 || w > 32768 || h > 32768) return fail(c, RMR_E_INVALID, "bad image size");
    c->pend_W = w;
    c->pend_H = h;
    return RMR_OK;
}

int rmr_get_image_size(const rmr_ctx* c, int* w, int* h) {
    if (!c || !w || !h) return RMR_E_INVALID;
    *w = c->W;
    *h = c->H;
    return RMR_OK;
}

int rmr_set_params(rmr_ctx* c, const rmr_params* p) {
    if (!c || !p) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (p->max_steps < 0 || p->max_bounces < 0 || !(p->max_dist > 0.0f)) return fail(c, RMR_E_INVALID, "bad params");
    c->params = *p;
    return RMR_OK;
}

int rmr_get_params(const rmr_ctx* c, rmr_params* p) {
    if (!c || !p) return RMR_E_INVALID;
    *p = c->params;
    return RMR_OK;
}

int rmr_set_view(rmr_ctx* c, const float eye[3], const float r00[3], const float r01[3], const float r10[3],
                 const float r11[3]) {
    if (!c || !eye || !r00 || !r01 || !r10 || !r11) return RMR_E_INVALID;
    RMR_FLUSH(c);
    for (int i = 0; i < 3; i++) {
        c->view[i] = eye[i]; c->view[3 + i] = r00[i]; c->view[6 + i] = r01[i];
        c->view[9 + i] = r10[i]; c->view[12 + i] = r11[i];
    }
    c->view_set = true;
    return RMR_OK;
}

int rmr_load_scene_json(rmr_ctx* c, int variant, const char* json, size_t len) {
    if (!c || !json) return RMR_E_INVALID;
    RMR_FLUSH(c);
    try {
        CompiledScene s = rmr::compile_scene(std::string(json, len), variant);
        int r = validate_scene(c, s);
        if (r) return r;
        c->scene = std::move(s);
    } catch (const rmr::SceneError& e) {
        return fail(c, RMR_E_SCENE, e.what());
    } catch (const std::exception& e) {
        return fail(c, RMR_E_SCENE, e.what());
    }
    HIPCHK(c, hipSetDevice(c->device));
    return upload_scene(c);
}

int rmr_load_scene_tables(rmr_ctx* c, const rmr_scene* s) {
    if (!c || !s) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (s->variant < RMR_VARIANT_RM1 || s->variant > RMR_VARIANT_RM3) return fail(c, RMR_E_INVALID, "bad variant");
    if (s->n_prims < 0 || s->n_prims > RMR_MAX_PRIMS || s->n_ops < 0 || s->n_ops > RMR_MAX_OPS ||
        s->n_consts < 0 || s->n_consts > RMR_MAX_CONSTS || s->n_materials < 0 || s->n_materials > RMR_MAX_MATERIALS)
        return fail(c, RMR_E_INVALID, "table sizes out of range");
    CompiledScene cs;
    cs.from_tables(*s);
    int r = validate_scene(c, cs);
    if (r) return r;
    c->scene = std::move(cs);
    HIPCHK(c, hipSetDevice(c->device));
    return upload_scene(c);
}

int rmr_load_builtin_scene(rmr_ctx* c, int variant) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (variant == RMR_VARIANT_RM2) return fail(c, RMR_E_SCENE, "RayMarch2.glsl needs a v2 scene for mat_func_1; use rmr_load_scene_json");
    try {
        c->scene = rmr::builtin_scene(variant);
    } catch (const std::exception& e) {
        return fail(c, RMR_E_SCENE, e.what());
    }
    HIPCHK(c, hipSetDevice(c->device));
    return upload_scene(c);
}

int rmr_reload(rmr_ctx* c) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->accum_external && (c->pend_W != c->W || c->pend_H != c->H))
        return fail(c, RMR_E_STATE, "bound accumulator cannot be resized");
    const bool resize = (c->pend_W != c->W || c->pend_H != c->H);
    c->W = c->pend_W;
    c->H = c->pend_H;
    if (resize) {
        if (c->view_set) { /* caller's view is kept (reference: camera.calculateRays after Reload) */ }
        int r = alloc_accum(c);
        if (r) return r;
    } else {
        HIPCHK(c, hipMemsetAsync(c->d_accum, 0, (size_t)c->W * c->H * sizeof(float4), c->stream));
    }
    return RMR_OK;
}

int rmr_render(rmr_ctx* c, float time, float min_x, float min_y, float max_x, float max_y, uint32_t current_sample) {
    if (!c) return RMR_E_INVALID;
    // pix >= bounds.xy && pix < bounds.zw for integer pix (RM1:572) <=> pix in [ceil(min), ceil(max))
    const int x0 = clampi((int)std::ceil(min_x), 0, c->W), y0 = clampi((int)std::ceil(min_y), 0, c->H);
    const int x1 = clampi((int)std::ceil(max_x), 0, c->W), y1 = clampi((int)std::ceil(max_y), 0, c->H);
    if (x1 <= x0 || y1 <= y0) return RMR_OK;
    if (!batching_on(c)) {
        RMR_FLUSH(c);
        return render_tiles(c, rect_tiles(x0, y0, x1, y1), x0, y0, x1, y1, &time, current_sample, 1);
    }
    // deferred (rmr_set_call_batching): the errors the launch would give now come at the call
    if (!c->scene_loaded) return fail(c, RMR_E_STATE, "no scene loaded (call rmr_load_scene_json / rmr_load_builtin_scene)");
    if (c->params.use_env_tex && !c->d_env) return fail(c, RMR_E_STATE, "useEnvTex != 0 but no env map (rmr_set_env_map)");
    rmr_ctx::Deferred* same = nullptr;
    bool overlap = false;
    for (auto& e : c->deferred) {
        if (e.x0 == x0 && e.y0 == y0 && e.x1 == x1 && e.y1 == y1) same = &e;
        else if (x0 < e.x1 && e.x0 < x1 && y0 < e.y1 && e.y0 < y1) overlap = true;
    }
    if (overlap || (same && current_sample != same->s0 + (uint32_t)same->times.size()) ||
        (!same && c->deferred.size() >= kDeferredRectsMax)) {
        RMR_FLUSH(c);
        same = nullptr;
    }
    if (same) same->times.push_back(time);
    else c->deferred.push_back(rmr_ctx::Deferred{x0, y0, x1, y1, current_sample, std::vector<float>(1, time)});
    c->deferred_units += (uint64_t)((x1 - x0 + 7) / 8) * ((y1 - y0 + 7) / 8) * 64;
    if (c->deferred_units >= kDeferredUnitsMax) RMR_FLUSH(c);
    return RMR_OK;
}

int rmr_set_call_batching(rmr_ctx* c, int mode) {
    if (!c || mode < -1 || mode > 1) return RMR_E_INVALID;
    RMR_FLUSH(c);
    c->call_batching = mode;
    return RMR_OK;
}

int rmr_set_launch_streams(rmr_ctx* c, int n) {
    if (!c || n < 0 || n > 4) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (n == c->launch_streams) return RMR_OK;
    int r = free_slots(c);   // (syncs the context's stream: every queued trace is done)
    c->launch_streams = n;
    return r ? r : make_slots(c);
}

int rmr_get_launch_streams(const rmr_ctx* c) { return c ? c->launch_streams : -1; }

int rmr_render_spp(rmr_ctx* c, const float* times, int x0, int y0, int x1, int y1, uint32_t first_sample, uint32_t nspp) {
    if (!c || (!times && nspp)) return RMR_E_INVALID;
    RMR_FLUSH(c);
    x0 = clampi(x0, 0, c->W); x1 = clampi(x1, 0, c->W);
    y0 = clampi(y0, 0, c->H); y1 = clampi(y1, 0, c->H);
    if (x1 <= x0 || y1 <= y0) return RMR_OK;
    return render_tiles(c, rect_tiles(x0, y0, x1, y1), x0, y0, x1, y1, times, first_sample, nspp);
}

int rmr_render_tiles(rmr_ctx* c, const float* times, const int32_t* tiles_xy, int n_tiles, int tile_size,
                     uint32_t first_sample, uint32_t nspp) {
    if (!c || (!times && nspp) || (!tiles_xy && n_tiles) || tile_size <= 0 || (tile_size % 8) != 0)
        return fail(c, RMR_E_INVALID, "tile_size must be a positive multiple of 8");
    RMR_FLUSH(c);
    // every (tx, ty) at most once: k_fold gives each pixel of a launch one thread, and a repeated
    // tile would have two threads read-modify-write the same accumulator pixel
    std::vector<std::pair<int, int>> seen;
    seen.reserve((size_t)n_tiles);
    for (int i = 0; i < n_tiles; i++) {
        if (tiles_xy[2 * i] < 0 || tiles_xy[2 * i + 1] < 0) return fail(c, RMR_E_INVALID, "negative tile index");
        seen.emplace_back(tiles_xy[2 * i], tiles_xy[2 * i + 1]);
    }
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end())
        return fail(c, RMR_E_INVALID, "duplicate tile in rmr_render_tiles");
    std::vector<TileXY> t;
    t.reserve((size_t)n_tiles * (tile_size / 8) * (tile_size / 8));
    for (int i = 0; i < n_tiles; i++) {
        const int bx = tiles_xy[2 * i] * tile_size, by = tiles_xy[2 * i + 1] * tile_size;
        for (int y = by; y < std::min(by + tile_size, c->H); y += 8)
            for (int x = bx; x < std::min(bx + tile_size, c->W); x += 8) t.push_back(TileXY{x, y});
    }
    if (t.empty()) return RMR_OK;
    return render_tiles(c, t, 0, 0, c->W, c->H, times, first_sample, nspp);
}

int rmr_read_accum(rmr_ctx* c, float* rgba, size_t bytes) {
    if (!c || !rgba) return RMR_E_INVALID;
    RMR_FLUSH(c);
    const size_t need = (size_t)c->W * c->H * sizeof(float4);
    if (bytes < need) return fail(c, RMR_E_INVALID, "buffer too small");
    HIPCHK(c, hipMemcpyAsync(rgba, c->d_accum, need, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RMR_OK;
}

int rmr_write_accum(rmr_ctx* c, const float* rgba, size_t bytes) {
    if (!c || !rgba) return RMR_E_INVALID;
    RMR_FLUSH(c);
    const size_t need = (size_t)c->W * c->H * sizeof(float4);
    if (bytes < need) return fail(c, RMR_E_INVALID, "buffer too small");
    HIPCHK(c, hipMemcpyAsync(c->d_accum, rgba, need, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RMR_OK;
}

void* rmr_accum_device_ptr(rmr_ctx* c) {
    if (!c) return nullptr;
    if (!c->deferred.empty() && flush_calls(c) != RMR_OK) return nullptr;   // the pointer's contents include them
    return (void*)c->d_accum;
}

int rmr_bind_accum(rmr_ctx* c, void* ptr, size_t bytes) {
    if (!c || !ptr) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (bytes < (size_t)c->W * c->H * sizeof(float4)) return fail(c, RMR_E_INVALID, "bound accumulator too small");
    if (c->d_accum && !c->accum_external) {  // the context's own buffer: free it once idle
        HIPCHK(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_accum);
    }
    // (an external buffer is only swapped: launches already queued keep the pointer they captured)
    c->d_accum = (float4*)ptr;
    c->accum_external = true;
    return RMR_OK;
}

int rmr_save_bmp(rmr_ctx* c, const char* path) {
    if (!c || !path) return RMR_E_INVALID;
    RMR_FLUSH(c);
    std::vector<float> host((size_t)c->W * c->H * 4);
    int r = rmr_read_accum(c, host.data(), host.size() * sizeof(float));
    if (r) return r;
    r = rmr_encode_bmp(host.data(), c->W, c->H, path);
    if (r) return fail(c, r, std::string("cannot write ") + path);
    return RMR_OK;
}

int rmr_save_accum(rmr_ctx* c, const char* path, uint32_t samples_done) {
    if (!c || !path) return RMR_E_INVALID;
    RMR_FLUSH(c);
    std::vector<float> host((size_t)c->W * c->H * 4);
    int r = rmr_read_accum(c, host.data(), host.size() * sizeof(float));
    if (r) return r;
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(c, RMR_E_IO, std::string("cannot open ") + path);
    const char magic[8] = {'R', 'M', 'R', 'A', 'C', 'C', '1', 0};
    const uint32_t hdr[3] = {(uint32_t)c->W, (uint32_t)c->H, samples_done};
    bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(hdr, 4, 3, f) == 3 &&
              std::fwrite(host.data(), sizeof(float), host.size(), f) == host.size();
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RMR_OK : fail(c, RMR_E_IO, "write failed");
}

int rmr_load_accum(rmr_ctx* c, const char* path, uint32_t* samples_done) {
    if (!c || !path) return RMR_E_INVALID;
    RMR_FLUSH(c);
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(c, RMR_E_IO, std::string("cannot open ") + path);
    char magic[8];
    uint32_t hdr[3];
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, "RMRACC1", 8) != 0 || std::fread(hdr, 4, 3, f) != 3) {
        std::fclose(f);
        return fail(c, RMR_E_IO, "not an rmr accumulator file");
    }
    if ((int)hdr[0] != c->W || (int)hdr[1] != c->H) {
        std::fclose(f);
        return fail(c, RMR_E_STATE, "accumulator size does not match the image size");
    }
    std::vector<float> host((size_t)c->W * c->H * 4);
    const bool ok = std::fread(host.data(), sizeof(float), host.size(), f) == host.size();
    std::fclose(f);
    if (!ok) return fail(c, RMR_E_IO, "truncated accumulator file");
    if (samples_done) *samples_done = hdr[2];
    return rmr_write_accum(c, host.data(), host.size() * sizeof(float));
}

int rmr_sync(rmr_ctx* c) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return collect_timing(c);
}

int rmr_get_stats(rmr_ctx* c, rmr_stats* out) {
    if (!c || !out) return RMR_E_INVALID;
    RMR_FLUSH(c);
    int r = rmr_sync(c);
    if (r) return r;
    unsigned long long cnt[16];
    HIPCHK(c, hipMemcpy(cnt, c->d_counters, sizeof cnt, hipMemcpyDeviceToHost));
    c->stats.map_evals = cnt[0];
    c->stats.map_iters = cnt[1];
    c->stats.shade_batches = cnt[2];
    *out = c->stats;
    return RMR_OK;
}

int rmr_get_section_cycles(rmr_ctx* c, uint64_t out[4]) {
    if (!c || !out) return RMR_E_INVALID;
    RMR_FLUSH(c);
    int r = rmr_sync(c);
    if (r) return r;
    unsigned long long cnt[8];
    HIPCHK(c, hipMemcpy(cnt, c->d_counters, sizeof cnt, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; i++) out[i] = cnt[4 + i];
    return RMR_OK;
}

int rmr_get_counters(rmr_ctx* c, uint64_t out[16]) {
    if (!c || !out) return RMR_E_INVALID;
    RMR_FLUSH(c);
    int r = rmr_sync(c);
    if (r) return r;
    unsigned long long cnt[16];
    HIPCHK(c, hipMemcpy(cnt, c->d_counters, sizeof cnt, hipMemcpyDeviceToHost));
    for (int i = 0; i < 16; i++) out[i] = cnt[i];
    return RMR_OK;
}

int rmr_reset_stats(rmr_ctx* c) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    int r = rmr_sync(c);
    if (r) return r;
    const double fpm = c->stats.flops_per_map;
    c->stats = rmr_stats{};
    c->stats.flops_per_map = fpm;
    HIPCHK(c, hipMemset(c->d_counters, 0, 16 * sizeof(unsigned long long)));
    return RMR_OK;
}

int rmr_set_kernel(rmr_ctx* c, int kernel) {
    if (!c || kernel < 0 || kernel > 1) return RMR_E_INVALID;
    RMR_FLUSH(c);
    c->kernel_mode = kernel;
    return RMR_OK;
}

// The candidate grid a context builds for a BVH scene, on the host (contract: rmr.h; construction:
// grid.cpp build_candidate_grid).
int rmr_candidate_grid(const float* prims, int n, int n_large, double E, double target, double pad, int32_t idims[5],
                       float geom[12], uint32_t* cells, size_t cells_cap, uint16_t* list, size_t list_cap) {
    if (!prims || n <= 0 || n_large < 0 || n_large > n || !idims || !geom) return RMR_E_INVALID;
    std::vector<rmr::DPrim> dp((size_t)n);
    for (int i = 0; i < n; i++) {
        const float* r = prims + 8 * (size_t)i;
        rmr::DPrim q{};
        for (int k = 0; k < 3; k++) { q.c[k] = r[k]; q.r[k] = r[3 + k]; }
        q.type = (int32_t)r[6] | (i << 8);
        q.mat_id = r[7];
        dp[(size_t)i] = q;
    }
    rmr::CandidateGrid g;
    const bool built = rmr::build_candidate_grid(dp, n_large, E, target > 0.0 ? target : 1048576.0,
                                                 pad > 0.0 ? pad : 0.5, g);
    for (int k = 0; k < 5; k++) idims[k] = 0;
    for (int k = 0; k < 12; k++) geom[k] = 0.0f;
    idims[4] = built ? 1 : 0;
    if (!built) return RMR_OK;
    for (int k = 0; k < 3; k++) { idims[k] = g.dim[k]; geom[k] = g.lo[k]; }
    idims[3] = (int32_t)g.list.size();
    geom[3] = g.inv;
    for (int k = 0; k < 6; k++) geom[4 + k] = g.sbox[k];
    geom[10] = (float)g.eps;
    geom[11] = (float)g.margin;
    if (!cells || !list || cells_cap < g.cells.size() || list_cap < g.list.size()) return RMR_E_INVALID;
    std::memcpy(cells, g.cells.data(), g.cells.size() * sizeof(uint32_t));
    std::memcpy(list, g.list.data(), g.list.size() * sizeof(uint16_t));
    return RMR_OK;
}

// sRGB decision points of Graphics::Display's GL_FRAMEBUFFER_SRGB write: byte(c) = round(255 srgb(c))
// for c in [0, 1] (srgb: 12.92 c below 0.0031308, else 1.055 c^(1/2.4) - 0.055), so byte(c) >= k
// <=> srgb(c) >= (k - 1/2) / 255 <=> c >= linear((k - 1/2) / 255); out[k] is that bound rounded up to
// a float (for a float c the comparison is then exact), out[0] = 0.
int rmr_srgb_thresholds(float out[256]) {
    if (!out) return RMR_E_INVALID;
    out[0] = 0.0f;
    for (int k = 1; k < 256; k++) {
        const double y = (k - 0.5) / 255.0;
        const double lin = (y <= 0.04045) ? y / 12.92 : std::pow((y + 0.055) / 1.055, 2.4);
        float f = (float)lin;
        if ((double)f < lin) f = std::nextafter(f, 2.0f);
        out[k] = f;
    }
    return RMR_OK;
}

namespace {
int display_common(rmr_ctx* c, float cx, float cy, float zoom, float min_x, float min_y, float max_x, float max_y,
                   int sw, int sh, uint32_t* dev) {
    if (!c->d_srgb_thr) {
        float t[256];
        rmr_srgb_thresholds(t);
        int r = dev_upload(c, &c->d_srgb_thr, t, 256);
        if (r) return r;
    }
    HIPCHK(c, rmr::launch_display(c->d_accum, c->W, c->H, cx, cy, zoom, min_x, min_y, max_x, max_y, sw, sh, dev,
                                  c->d_srgb_thr, c->stream));
    return RMR_OK;
}
}  // namespace

int rmr_display(rmr_ctx* c, float centre_x, float centre_y, float zoom, float min_x, float min_y, float max_x,
                float max_y, int screen_w, int screen_h, uint8_t* rgba8, size_t nbytes) {
    if (!c || !rgba8 || screen_w <= 0 || screen_h <= 0 || screen_w > 32768 || screen_h > 32768)
        return fail(c, RMR_E_INVALID, "rmr_display: bad screen image");
    if (nbytes < (size_t)screen_w * screen_h * 4)
        return fail(c, RMR_E_INVALID, "rmr_display: screen buffer smaller than screen_w * screen_h * 4 bytes");
    RMR_FLUSH(c);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t n = (size_t)screen_w * screen_h;
    if (n > c->screen_cap) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->d_screen) (void)hipFree(c->d_screen);
        c->d_screen = nullptr;
        c->screen_cap = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_screen, n * sizeof(uint32_t)));
        c->screen_cap = n;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_screen, rgba8, n * 4, hipMemcpyHostToDevice, c->stream));
    int r = display_common(c, centre_x, centre_y, zoom, min_x, min_y, max_x, max_y, screen_w, screen_h, c->d_screen);
    if (r) return r;
    HIPCHK(c, hipMemcpyAsync(rgba8, c->d_screen, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RMR_OK;
}

int rmr_display_device(rmr_ctx* c, float centre_x, float centre_y, float zoom, float min_x, float min_y, float max_x,
                       float max_y, int screen_w, int screen_h, void* rgba8_dev, size_t nbytes) {
    if (!c || !rgba8_dev || screen_w <= 0 || screen_h <= 0 || screen_w > 32768 || screen_h > 32768)
        return fail(c, RMR_E_INVALID, "rmr_display_device: bad screen image");
    if (nbytes < (size_t)screen_w * screen_h * 4)
        return fail(c, RMR_E_INVALID, "rmr_display_device: screen buffer smaller than screen_w * screen_h * 4 bytes");
    RMR_FLUSH(c);
    HIPCHK(c, hipSetDevice(c->device));
    return display_common(c, centre_x, centre_y, zoom, min_x, min_y, max_x, max_y, screen_w, screen_h,
                          (uint32_t*)rgba8_dev);
}

int rmr_set_env_map(rmr_ctx* c, const uint8_t* rgba8, int w, int h) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (!rgba8) {
        if (c->d_env) (void)hipFree(c->d_env);
        c->d_env = nullptr;
        c->env_w = c->env_h = 0;
        return RMR_OK;
    }
    if (w <= 0 || h <= 0 || (size_t)w * h > ((size_t)1 << 26)) return fail(c, RMR_E_INVALID, "bad env map size");
    std::vector<float4> t((size_t)w * h);
    for (size_t i = 0; i < t.size(); i++)  // GL unorm8 -> float: c / 255
        t[i] = make_float4((float)rgba8[4 * i] / 255.0f, (float)rgba8[4 * i + 1] / 255.0f,
                           (float)rgba8[4 * i + 2] / 255.0f, (float)rgba8[4 * i + 3] / 255.0f);
    int r;
    if ((r = dev_upload(c, &c->d_env, t.data(), t.size()))) return r;
    c->env_w = w;
    c->env_h = h;
    return RMR_OK;
}

int rmr_set_jit(rmr_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 2) return RMR_E_INVALID;
    RMR_FLUSH(c);
    c->jit_mode = mode;
    c->jit_failed = false;
    return RMR_OK;
}

int rmr_set_culling(rmr_ctx* c, int flags) {
    if (!c || (flags & ~(RMR_CULL_ESCAPE | RMR_CULL_NPC | RMR_CULL_APPROX | RMR_CULL_EYE))) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (flags != c->cull) c->jit_ready = false;   // the specialised kernel depends on it
    c->cull = flags;
    return RMR_OK;
}

int rmr_jit_compile_scene(int variant, const char* json, size_t len, char* log, size_t loglen) {
    std::string lg;
    try {
        CompiledScene s = (json && len) ? rmr::compile_scene(std::string(json, len), variant) : rmr::builtin_scene(variant);
        // the kernel class as a context picks it: node-program materials by upload_scene's rule
        // (shading_kinds), the cache's primitives per lane and the sphere-only candidates as
        // ensure_jit for BVH scenes, whose full map() runs through the candidate grid (assumed built,
        // as it is unless the grid would exceed 2^31 cells)
        const bool prog = any_program(shading_kinds(s));
        bool simple = true;
        for (const auto& q : s.prims) simple = simple && (q.type == RMR_PRIM_SPHERE || q.type == RMR_PRIM_BOX);
        const bool bvh = simple && s.prims.size() > (size_t)kMaxLoopPrims;
        bool npc_spheres = bvh;
        if (bvh) {
            std::vector<char> is_large;
            float extent = 0.0f;
            (void)bvh_items(s, is_large, extent);
            for (size_t i = 0; i < s.prims.size(); i++)
                npc_spheres = npc_spheres && (is_large[i] || s.prims[i].type == RMR_PRIM_SPHERE);
        }
        std::vector<char> code;
        std::string key;
        const bool ok = rmr::jit_compile(
            rmr::jit_source(s, prog, true, RMR_CULL_ESCAPE | RMR_CULL_NPC | RMR_CULL_APPROX | RMR_CULL_EYE, nullptr,
                            bvh ? 1 : 2, npc_spheres),
            code, key, lg);
        if (log && loglen) std::snprintf(log, loglen, "%s", ok ? key.c_str() : lg.c_str());
        return ok ? RMR_OK : RMR_E_HIP;
    } catch (const std::exception& e) {
        if (log && loglen) std::snprintf(log, loglen, "%s", e.what());
        return RMR_E_SCENE;
    }
}

int rmr_set_instrument(rmr_ctx* c, int flags) {
    if (!c || (flags & ~RMR_INSTR_COUNT_FLOPS)) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (flags != c->instrument) {
        c->instrument = flags;
        c->jit_ready = false;   // another code object (its own cache key)
        c->jit_failed = false;
    }
    return RMR_OK;
}

int rmr_set_tuning(rmr_ctx* c, int shade_threshold, int grid_per_cu, long long samp_budget_bytes) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (shade_threshold > 0) {
        c->shade_threshold = std::max(1, std::min(64, shade_threshold & 0xff));
        c->shade_auto = false;
        const int tr = (shade_threshold >> 8) & 0xff;
        c->refill_threshold = tr ? std::min(64, tr) : -1;   // unset: half the shading threshold
    }
    if (grid_per_cu >= 0) c->grid_per_cu = grid_per_cu;
    if (samp_budget_bytes > 0) c->samp_budget = (size_t)samp_budget_bytes;
    return RMR_OK;
}

int rmr_set_grid_reserve(rmr_ctx* c, int blocks) {
    if (!c || blocks < 0) return RMR_E_INVALID;
    RMR_FLUSH(c);
    c->grid_reserve = blocks;
    return RMR_OK;
}

// Per-sample radiance planes for parity tests: out[k][y-y0][x-x0][4] for the rect.
int rmr_trace_samples(rmr_ctx* c, const float* times, int x0, int y0, int x1, int y1, uint32_t nspp, float* out) {
    if (!c || !times || !out) return RMR_E_INVALID;
    RMR_FLUSH(c);
    x0 = clampi(x0, 0, c->W); x1 = clampi(x1, 0, c->W);
    y0 = clampi(y0, 0, c->H); y1 = clampi(y1, 0, c->H);
    if (x1 <= x0 || y1 <= y0 || nspp == 0) return RMR_OK;
    std::vector<TileXY> tiles = rect_tiles(x0, y0, x1, y1);
    const size_t saved_budget = c->samp_budget;
    const size_t plane = tiles.size() * 64;
    c->samp_budget = std::max(saved_budget, plane * nspp * sizeof(float4));  // one chunk
    // render into a scratch accumulator region: trace writes samp planes; fold into accum is harmless
    std::vector<float> keep((size_t)c->W * c->H * 4);
    int r = rmr_read_accum(c, keep.data(), keep.size() * sizeof(float));
    if (!r) r = render_tiles(c, tiles, x0, y0, x1, y1, times, 0, nspp);
    c->samp_budget = saved_budget;
    if (r) return r;
    std::vector<float4> h(plane * nspp);
    HIPCHK(c, hipMemcpyAsync(h.data(), c->last_samp, h.size() * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int w = x1 - x0, hh = y1 - y0;
    const int tx = (w + 7) / 8;
    for (uint32_t k = 0; k < nspp; k++)
        for (int y = 0; y < hh; y++)
            for (int x = 0; x < w; x++) {
                const size_t tile = (size_t)(y / 8) * tx + (x / 8);
                const size_t lane = (size_t)(y % 8) * 8 + (x % 8);
                const float4 v = h[(size_t)k * plane + tile * 64 + lane];
                float* o = out + (((size_t)k * hh + y) * w + x) * 4;
                o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
            }
    return rmr_write_accum(c, keep.data(), keep.size() * sizeof(float));
}

#if RMR_DIAG
// Diagnostic library only (not in include/rmr.h): the escape bound ray_exit at n given rays (rays:
// o.xyz, d.xyz per ray) with the context's scene, view and maxDist, as a launch would use it; out[i]
// = the bound (+inf: none). boxes (optional, 6 floats per box, up to max_boxes) receives the inflated
// escape boxes the kernel read, *n_boxes their number (0: the bound is off for this scene).
int rmr_diag_ray_exit(rmr_ctx* c, const float* rays, int n, float* out, float* boxes, int max_boxes, int* n_boxes) {
    if (!c) return RMR_E_INVALID;
    RMR_FLUSH(c);
    if (!c->scene_loaded) return fail(c, RMR_E_STATE, "no scene loaded");
    if (n < 0 || (n > 0 && (!rays || !out))) return fail(c, RMR_E_INVALID, "bad rays / out");
    if (!c->view_set) default_view(c);
    KParams P{};
    int rr;
    if ((rr = escape_params(c, P))) return rr;
    if (n_boxes) *n_boxes = P.esc_on ? P.n_esc : 0;
    if (boxes && P.esc_on && max_boxes > 0) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(boxes, c->d_esc, sizeof(float) * 6 * (size_t)std::min(max_boxes, P.n_esc), hipMemcpyDeviceToHost));
    }
    if (n == 0) return RMR_OK;
    float *d_rays = nullptr, *d_out = nullptr;
    HIPCHK(c, hipMalloc((void**)&d_rays, sizeof(float) * 6 * (size_t)n));
    HIPCHK(c, hipMalloc((void**)&d_out, sizeof(float) * (size_t)n));
    hipError_t e = hipMemcpyAsync(d_rays, rays, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = rmr::launch_ray_exit(P, d_rays, d_out, n, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_rays);
    (void)hipFree(d_out);
    HIPCHK(c, e);
    return RMR_OK;
}
#endif

int rmr_abi_sizes(int32_t* out, int n) {
    const int32_t s[] = {(int32_t)sizeof(rmr_prim), (int32_t)sizeof(rmr_op), (int32_t)sizeof(rmr_material),
                         (int32_t)sizeof(rmr_spectral), (int32_t)sizeof(rmr_rm2_consts), (int32_t)sizeof(rmr_scene),
                         (int32_t)sizeof(rmr_params), (int32_t)sizeof(rmr_stats)};
    const int m = (int)(sizeof s / sizeof s[0]);
    for (int i = 0; i < n && i < m; i++) out[i] = s[i];
    return m;
}

}  // extern "C"
