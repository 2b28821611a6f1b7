// rmr_group.cpp — librmr_group.so: one host process drives every GPU of the node (include/rmr_group.h).
//
// The frame's tiles are dealt round-robin to the members; each member renders its tiles through two
// ordinary rmr contexts (the single-GPU C ABI, librmr.so) on two HIP streams of its device, into the
// contexts' own accumulators, zeroed per frame; one ncclReduce(SUM) per frame, issued for all members
// inside ncclGroupStart/End on the frame's streams, assembles the image on member 0. Frame f's zeroing,
// render and reduce are ordered on stream f % 2 of each member, so the two frames in flight overlap
// (one process, one stream per GPU, ncclCommInitAll; §8e: tile partition + one reduce).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rmr_group.h"

namespace {

// workgroups each trace launch leaves free for the other frame's fold, zeroing and reduce
// (multi_gpu.OVERLAP_GRID_RESERVE; rmr.h rmr_set_grid_reserve)
constexpr int kGridReserve = 64;

struct Member {
    int device = 0;
    rmr_ctx* ctx[2] = {nullptr, nullptr};
    hipStream_t stream[2] = {nullptr, nullptr};
    ncclComm_t comm = nullptr;
    std::vector<int32_t> tiles;   // (tx, ty) pairs of this member's share
};

}  // namespace

struct rmr_group {
    std::vector<Member> m;
    int W = 1024, H = 1024, pend_W = 1024, pend_H = 1024;   // rmr_create's defaults
    int tile = 32;
    bool reloaded = false;
    uint64_t frames = 0;
    std::string err;
};

namespace {

int gfail(rmr_group* g, int code, const std::string& msg) {
    if (g) g->err = msg;
    return code;
}

// a member context's failure, with its message
int cfail(rmr_group* g, int code, int member, rmr_ctx* c, const char* what) {
    return gfail(g, code, std::string(what) + " (member " + std::to_string(member) + "): " + rmr_last_error(c));
}

#define GHIP(g, expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return gfail(g, RMR_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define GNCCL(g, expr)                                                                              \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) return gfail(g, RMR_E_HIP, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)

// apply f(ctx) to both contexts of every member, on that member's device
template <class F>
int each_ctx(rmr_group* g, const char* what, F f) {
    if (!g) return RMR_E_INVALID;
    for (size_t i = 0; i < g->m.size(); i++)
        for (int k = 0; k < 2; k++) {
            GHIP(g, hipSetDevice(g->m[i].device));
            const int r = f(g->m[i].ctx[k]);
            if (r != RMR_OK) return cfail(g, r, (int)i, g->m[i].ctx[k], what);
        }
    return RMR_OK;
}

void partition(int w, int h, int tile, int member, int n, std::vector<int32_t>& out) {
    out.clear();
    const int tw = (w + tile - 1) / tile, th = (h + tile - 1) / tile;
    long idx = 0;
    for (int ty = 0; ty < th; ty++)
        for (int tx = 0; tx < tw; tx++, idx++)
            if (idx % n == member) {
                out.push_back(tx);
                out.push_back(ty);
            }
}

}  // namespace

extern "C" {

int rmr_group_partition(int w, int h, int tile_size, int member, int n, int32_t* tiles_xy, int cap) {
    if (w <= 0 || h <= 0 || tile_size <= 0 || n <= 0 || member < 0 || member >= n || cap < 0 || (!tiles_xy && cap))
        return RMR_E_INVALID;
    std::vector<int32_t> t;
    partition(w, h, tile_size, member, n, t);
    const int count = (int)(t.size() / 2);
    std::memcpy(tiles_xy, t.data(), sizeof(int32_t) * 2 * (size_t)std::min(count, cap));
    return count;
}

int rmr_group_create(rmr_group** out, const int* devices, int n) {
    if (!out || !devices || n <= 0) return RMR_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RMR_E_HIP;
    for (int i = 0; i < n; i++) {
        if (devices[i] < 0 || devices[i] >= ndev) return RMR_E_INVALID;
        for (int j = 0; j < i; j++)
            if (devices[j] == devices[i]) return RMR_E_INVALID;   // RCCL: one rank per device
    }
    rmr_group* g = new (std::nothrow) rmr_group();
    if (!g) return RMR_E_NOMEM;
    g->m.resize((size_t)n);
    for (int i = 0; i < n; i++) {
        Member& mb = g->m[(size_t)i];
        mb.device = devices[i];
        for (int k = 0; k < 2; k++) {
            if (rmr_create(&mb.ctx[k], mb.device) != RMR_OK || hipSetDevice(mb.device) != hipSuccess ||
                hipStreamCreateWithFlags(&mb.stream[k], hipStreamNonBlocking) != hipSuccess ||
                rmr_set_stream(mb.ctx[k], (void*)mb.stream[k]) != RMR_OK ||
                rmr_set_grid_reserve(mb.ctx[k], kGridReserve) != RMR_OK ||
                // the two contexts overlap each other's frames: no launch slots of their own
                // (rmr.h rmr_set_launch_streams: 2 x 3 streams would exceed the hardware queues)
                rmr_set_launch_streams(mb.ctx[k], 0) != RMR_OK) {
                rmr_group_destroy(g);
                return RMR_E_HIP;
            }
        }
    }
    std::vector<ncclComm_t> comms((size_t)n);
    if (ncclCommInitAll(comms.data(), n, devices) != ncclSuccess) {
        rmr_group_destroy(g);
        return RMR_E_HIP;
    }
    for (int i = 0; i < n; i++) g->m[(size_t)i].comm = comms[(size_t)i];
    *out = g;
    return RMR_OK;
}

void rmr_group_destroy(rmr_group* g) {
    if (!g) return;
    for (Member& mb : g->m) {
        (void)hipSetDevice(mb.device);
        for (int k = 0; k < 2; k++)
            if (mb.stream[k]) (void)hipStreamSynchronize(mb.stream[k]);
        if (mb.comm) (void)ncclCommDestroy(mb.comm);
        for (int k = 0; k < 2; k++) {
            if (mb.ctx[k]) rmr_destroy(mb.ctx[k]);   // its stream is ours: destroyed below
            if (mb.stream[k]) (void)hipStreamDestroy(mb.stream[k]);
        }
    }
    delete g;
}

const char* rmr_group_last_error(const rmr_group* g) { return g ? g->err.c_str() : "null group"; }

int rmr_group_size(const rmr_group* g) { return g ? (int)g->m.size() : 0; }

rmr_ctx* rmr_group_context(rmr_group* g, int member, int k) {
    if (!g || member < 0 || member >= (int)g->m.size() || k < 0 || k > 1) return nullptr;
    return g->m[(size_t)member].ctx[k];
}

int rmr_group_set_image_size(rmr_group* g, int w, int h) {
    const int r = each_ctx(g, "set_image_size", [&](rmr_ctx* c) { return rmr_set_image_size(c, w, h); });
    if (r == RMR_OK) { g->pend_W = w; g->pend_H = h; }
    return r;
}

int rmr_group_set_params(rmr_group* g, const rmr_params* p) {
    return each_ctx(g, "set_params", [&](rmr_ctx* c) { return rmr_set_params(c, p); });
}

int rmr_group_set_view(rmr_group* g, const float eye[3], const float ray00[3], const float ray01[3],
                       const float ray10[3], const float ray11[3]) {
    return each_ctx(g, "set_view", [&](rmr_ctx* c) { return rmr_set_view(c, eye, ray00, ray01, ray10, ray11); });
}

int rmr_group_load_scene_json(rmr_group* g, int variant, const char* json, size_t len) {
    return each_ctx(g, "load_scene_json", [&](rmr_ctx* c) { return rmr_load_scene_json(c, variant, json, len); });
}

int rmr_group_load_builtin_scene(rmr_group* g, int variant) {
    return each_ctx(g, "load_builtin_scene", [&](rmr_ctx* c) { return rmr_load_builtin_scene(c, variant); });
}

int rmr_group_set_env_map(rmr_group* g, const uint8_t* rgba8, int w, int h) {
    return each_ctx(g, "set_env_map", [&](rmr_ctx* c) { return rmr_set_env_map(c, rgba8, w, h); });
}

int rmr_group_set_tile_size(rmr_group* g, int tile_size) {
    if (!g) return RMR_E_INVALID;
    if (tile_size <= 0 || tile_size % 8) return gfail(g, RMR_E_INVALID, "tile_size must be a positive multiple of 8");
    g->tile = tile_size;
    g->reloaded = false;   // the partition follows at rmr_group_reload
    return RMR_OK;
}

int rmr_group_reload(rmr_group* g) {
    if (!g) return RMR_E_INVALID;
    int r = rmr_group_sync(g);
    if (r) return r;
    r = each_ctx(g, "reload", [&](rmr_ctx* c) { return rmr_reload(c); });
    if (r) return r;
    g->W = g->pend_W;
    g->H = g->pend_H;
    const int n = (int)g->m.size();
    for (int i = 0; i < n; i++) partition(g->W, g->H, g->tile, i, n, g->m[(size_t)i].tiles);
    g->reloaded = true;
    return RMR_OK;
}

int rmr_group_render_frame(rmr_group* g, const float* times, uint32_t nspp) {
    if (!g || (!times && nspp)) return RMR_E_INVALID;
    if (!g->reloaded) return gfail(g, RMR_E_STATE, "call rmr_group_reload first (image size and tile partition)");
    const int k = (int)(g->frames & 1);
    const size_t count = (size_t)g->W * g->H * 4;   // floats
    std::vector<void*> acc(g->m.size());
    for (size_t i = 0; i < g->m.size(); i++) {
        Member& mb = g->m[i];
        GHIP(g, hipSetDevice(mb.device));
        acc[i] = rmr_accum_device_ptr(mb.ctx[k]);
        if (!acc[i]) return cfail(g, RMR_E_STATE, (int)i, mb.ctx[k], "accumulator");
        // the zeroing waits (stream order) for this buffer's previous reduce, two frames back
        GHIP(g, hipMemsetAsync(acc[i], 0, count * sizeof(float), mb.stream[k]));
        if (!mb.tiles.empty()) {
            const int r = rmr_render_tiles(mb.ctx[k], times, mb.tiles.data(), (int)(mb.tiles.size() / 2), g->tile, 0, nspp);
            if (r) return cfail(g, r, (int)i, mb.ctx[k], "render_tiles");
        }
    }
    // the frame's one collective: every member's frame summed onto member 0 (in place there)
    GNCCL(g, ncclGroupStart());
    for (size_t i = 0; i < g->m.size(); i++)
        GNCCL(g, ncclReduce(acc[i], acc[i], count, ncclFloat32, ncclSum, 0, g->m[i].comm, g->m[i].stream[k]));
    GNCCL(g, ncclGroupEnd());
    g->frames++;
    return RMR_OK;
}

int rmr_group_sync(rmr_group* g) {
    if (!g) return RMR_E_INVALID;
    for (size_t i = 0; i < g->m.size(); i++)
        for (int k = 0; k < 2; k++) {
            const int r = rmr_sync(g->m[i].ctx[k]);   // its stream: renders, zeroing and reduces
            if (r) return cfail(g, r, (int)i, g->m[i].ctx[k], "sync");
        }
    return RMR_OK;
}

int rmr_group_read_frame(rmr_group* g, float* rgba, size_t bytes) {
    if (!g || !rgba) return RMR_E_INVALID;
    if (!g->frames) return gfail(g, RMR_E_STATE, "no frame rendered");
    int r = rmr_group_sync(g);
    if (r) return r;
    Member& m0 = g->m[0];
    GHIP(g, hipSetDevice(m0.device));
    rmr_ctx* c = m0.ctx[(g->frames - 1) & 1];
    r = rmr_read_accum(c, rgba, bytes);
    return r ? cfail(g, r, 0, c, "read_frame") : RMR_OK;
}

int rmr_group_save_bmp(rmr_group* g, const char* path) {
    if (!g || !path) return RMR_E_INVALID;
    std::vector<float> host((size_t)g->W * g->H * 4);
    int r = rmr_group_read_frame(g, host.data(), host.size() * sizeof(float));
    if (r) return r;
    r = rmr_encode_bmp(host.data(), g->W, g->H, path);
    return r ? gfail(g, r, std::string("cannot write ") + path) : RMR_OK;
}

int rmr_group_get_stats(rmr_group* g, int member, rmr_stats* out) {
    if (!g || !out || member < 0 || member >= (int)g->m.size()) return RMR_E_INVALID;
    rmr_stats s[2];
    for (int k = 0; k < 2; k++) {
        const int r = rmr_get_stats(g->m[(size_t)member].ctx[k], &s[k]);
        if (r) return cfail(g, r, member, g->m[(size_t)member].ctx[k], "get_stats");
    }
    *out = s[0];
    out->map_evals += s[1].map_evals;
    out->samples += s[1].samples;
    out->trace_launches += s[1].trace_launches;
    out->trace_ms += s[1].trace_ms;
    out->fold_ms += s[1].fold_ms;
    out->map_iters += s[1].map_iters;
    out->shade_batches += s[1].shade_batches;
    out->jit_launches += s[1].jit_launches;
    return RMR_OK;
}

int rmr_group_reset_stats(rmr_group* g) {
    return each_ctx(g, "reset_stats", [&](rmr_ctx* c) { return rmr_reset_stats(c); });
}

}  // extern "C"
