// rmr_jit.hpp — per-scene specialisation of the trace kernel with hipRTC.
//
// The reference recompiles its compute shader whenever the scene changes: Graphics::Reload
// generates GLSL for every object and material and hands it to the GL driver (Graphics.cpp:
// 392-752). rmr does the MI355X equivalent: the scene's map() is emitted as straight-line HIP with
// every primitive's centre, size and material id as literals, compiled by hipRTC for gfx950 against
// the same device code as the ahead-of-time kernels (rmr_trace.h), and launched in their place. The
// arithmetic is the same expression for expression, so the results are bit-identical; what goes
// away is the per-primitive scalar loads and type branches (measured +14% on Cornell-5).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "scene.hpp"

// Environment switches (RMR_GRID, RMR_JIT_OPTS, RMR_JIT_BAKE, ...: A/B experiments, tools/) exist only
// in the diagnostic build librmr_diag.so (`make diag`, -DRMR_DIAG=1). The release librmr.so reads no
// environment variable but RMR_JIT_CACHE (and HOME for its default): a drop-in renderer's results and
// kernels do not depend on an inherited environment. RMR_ENV("X") is nullptr there, and the name
// does not reach the binary.
#ifndef RMR_DIAG
#define RMR_DIAG 0
#endif
#if RMR_DIAG
#define RMR_ENV(name) std::getenv(name)
#else
#define RMR_ENV(name) ((const char*)nullptr)
#endif

namespace rmr {

struct JitKernel {
    std::string key;            // hash of source + options
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
    int blocks_per_cu = 0;
    int shade_t = 16;           // default shading batch size for this kernel (rmr_api.cpp)
    int block = 256;            // workgroup size
    int chunk = 128;            // units a wave takes from the work queue at a time (rmr_trace.h
                                // RMR_CHUNK; the nearest-primitive cache kernels: RMR_CHUNK_CACHE)
};

// What jit_source decided about the kernel class (the launch settings follow from these, not from
// the text of the source): the nearest-primitive cache map (TableMap<-3>: 64-unit chunks), a general
// map (Mandelbulb / node-program objects), node-program materials, certified getNormal probes.
struct JitFacts {
    int variant = 0;
    bool cache = false, general = false, prog = false, cert = false;
    int chunk() const { return cache ? 64 : 128; }   // rmr_trace.h RMR_CHUNK_CACHE / RMR_CHUNK
    // default shading batch: general maps without material programs, whose map() dwarfs the shading
    // (the Mandelbulb): 10 (C3: 8 / 12 within 0.6%, 6 / 16 +3%, profiles/r05_c3_shade_ab.log); node-program materials, the cache kernels and the certified
    // sphere/box kernels (their batches run the certified probes): 20; otherwise 16 (rmr_api.cpp)
    int shade_t() const {
        if (variant == RMR_VARIANT_RM1 && general && !prog) return 10;
        if (prog || cache || cert) return 20;
        return 16;
    }
};

// HIP source of the specialised trace kernel for `s` (entry point "rmr_jit_trace"). bake: the
// primitives' numbers are literals (fastest: +6-12% over loading them); otherwise only the scene's
// structure is compiled and the numbers are scalar loads, so a scene that only moves (an animation)
// reuses one kernel instead of recompiling per frame.
// cull: RMR_CULL_* bits of the context (rmr.h): approximate-then-exact map, nearest-primitive cache.
// live (with bake): primitives j with live[j] != 0 are loaded even so (an animation's moving
// primitives; the rest stay literals).
// npc_k: primitives per lane in the nearest-primitive cache (RMR_NPC_K: 1 or 2) of BVH scenes.
// npc_spheres: every primitive the candidate grid lists is a sphere (RMR_NPC_SPHERES: the full
// map's candidates take the sphere distance, the same value as the general form for a sphere).
// facts (optional): the kernel class, for the launch settings.
std::string jit_source(const CompiledScene& s, bool prog, bool bake = true, int cull = 7,
                       const std::vector<char>* live = nullptr, int npc_k = 2, bool npc_spheres = false,
                       JitFacts* facts = nullptr);
// Compile `src` for gfx950 (no GPU needed). Code-object cache: in-process, then the directory
// $RMR_JIT_CACHE (default $HOME/.cache/rmr-jit). Returns false with the compiler log in `log`.
// opts: further compiler options, part of the key (the instrumented build of rmr_set_instrument:
// -DRMR_COUNT_FLOPS).
bool jit_compile(const std::string& src, std::vector<char>& code, std::string& key, std::string& log,
                 const std::vector<std::string>& opts = {});

}  // namespace rmr
