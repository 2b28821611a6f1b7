// rmr_kernels.hip — ahead-of-time gfx950 kernels of the rmr SDF ray-march path tracer: the
// table-driven trace kernel k_trace<VARIANT, NP, PERSIST, PROG> (device code in rmr_trace.h), the
// running-mean fold k_fold, and their host launchers. Scenes can additionally be specialised at
// load time by hipRTC (rmr_jit.cpp), which reuses rmr_trace.h with the scene's map() baked in.
#include <hip/hip_runtime.h>
#include "rmr_trace.h"

namespace rmr {

template <int VAR, int NP, bool PERSIST, bool PROG>
__global__ __launch_bounds__(256, (trace_waves<VAR, (NP == -1), PROG>())) void k_trace(KParams P) {
    trace_main<VAR, TableMap<NP>, PERSIST, PROG>(P);
}

__global__ __launch_bounds__(256) void k_fold(KParams P) { fold_main(P); }

}  // namespace rmr

// ---- host-side launchers (C++ linkage, used by rmr_api.cpp) ----------------------------------
namespace rmr {
#define RMR_TRACE_SWITCH(V, NPV, PERS, PRG, CALL)        \
    switch (NPV) {                                          \
    case 4: CALL(V, 4, PERS, PRG); break;                   \
    case 8: CALL(V, 8, PERS, PRG); break;                   \
    case 0: CALL(V, 0, PERS, PRG); break;                   \
    case -2: CALL(V, -2, PERS, PRG); break;                 \
    default: CALL(V, -1, PERS, PRG); break;                 \
    }
#define RMR_LAUNCH(V, NPV, PERS, PRG) k_trace<V, NPV, PERS, PRG><<<g, block, 0, s>>>(P)

hipError_t launch_trace(const KParams& P, int variant, int np, bool prog, bool persistent, int grid, hipStream_t s) {
    dim3 block(256);
    unsigned g = (unsigned)grid;
    if (persistent) {
        switch (variant) {
        case RMR_VARIANT_RM1:
            if (prog) { RMR_TRACE_SWITCH(RMR_VARIANT_RM1, np, true, true, RMR_LAUNCH); }
            else { RMR_TRACE_SWITCH(RMR_VARIANT_RM1, np, true, false, RMR_LAUNCH); }
            break;
        case RMR_VARIANT_RM2: RMR_TRACE_SWITCH(RMR_VARIANT_RM2, np, true, false, RMR_LAUNCH); break;
        default: RMR_TRACE_SWITCH(RMR_VARIANT_RM3, np, true, false, RMR_LAUNCH); break;
        }
    } else {
        g = (unsigned)((P.n_units + 255) / 256);
        switch (variant) {
        case RMR_VARIANT_RM1: RMR_LAUNCH(RMR_VARIANT_RM1, -1, false, true); break;
        case RMR_VARIANT_RM2: RMR_LAUNCH(RMR_VARIANT_RM2, -1, false, false); break;
        default: RMR_LAUNCH(RMR_VARIANT_RM3, -1, false, false); break;
        }
    }
    return hipGetLastError();
}
// ray_exit at given rays (o.xyz, d.xyz per ray), with the launch's escape boxes: the diagnostic
// library's rmr_diag_ray_exit (tests/test_gpu_escape_bound.py checks the bound's validity)
__global__ void k_ray_exit(KParams P, const float* rays, float* out, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) {
        const float* r = rays + 6 * (size_t)i;
        out[i] = ray_exit(P, v3(r[0], r[1], r[2]), v3(r[3], r[4], r[5]));
    }
}
hipError_t launch_ray_exit(const KParams& P, const float* rays, float* out, int n, hipStream_t s) {
    k_ray_exit<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(P, rays, out, n);
    return hipGetLastError();
}
hipError_t launch_fold(const KParams& P, hipStream_t s) {
    const uint64_t threads = (uint64_t)P.n_tiles * 64;
    k_fold<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(P);
    return hipGetLastError();
}
#define RMR_OCC(V, NPV, PERS, PRG) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_trace<V, NPV, PERS, PRG>, 256, 0)
int trace_occupancy(int variant, int np, bool prog, int* blocks_per_cu) {
    int b = 0;
    hipError_t e = hipSuccess;
    switch (variant) {
    case RMR_VARIANT_RM1:
        if (prog) { RMR_TRACE_SWITCH(RMR_VARIANT_RM1, np, true, true, RMR_OCC); }
        else { RMR_TRACE_SWITCH(RMR_VARIANT_RM1, np, true, false, RMR_OCC); }
        break;
    case RMR_VARIANT_RM2: RMR_TRACE_SWITCH(RMR_VARIANT_RM2, np, true, false, RMR_OCC); break;
    default: RMR_TRACE_SWITCH(RMR_VARIANT_RM3, np, true, false, RMR_OCC); break;
    }
    *blocks_per_cu = b;
    return e == hipSuccess ? 0 : -1;
}
}  // namespace rmr
