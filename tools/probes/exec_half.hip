// Does a wave64 VALU instruction cost less when whole groups of lanes are masked off by EXEC?
// Each lane runs 8 independent v_fma_f32 chains inside `if (mask bit of its lane)`: the loop issues
// with EXEC = the mask. Masks: all 64 lanes, the low 32, the low 16, lane 0 only, the even lanes
// (32 lanes spread over both halves), lanes 0-7 of each 16-lane group. If the SIMD skipped the
// passes of lane groups with no active lane, the low-32 / low-16 masks would run faster than all 64.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/probes/exec_half.hip -o tools/probes/exec_half
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

__global__ __launch_bounds__(256, 8) void k_masked(float* out, float a, float b, uint64_t mask) {
    const int lane = __lane_id();
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    if ((mask >> lane) & 1) {
        for (int i = 0; i < kIters; i++) {
            x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
            x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 8 * 4;
    float* out = nullptr;
    hipMalloc((void**)&out, (size_t)blocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct M { const char* name; uint64_t m; } masks[] = {
        {"all64", ~0ull},
        {"low32", 0xffffffffull},
        {"high32", 0xffffffff00000000ull},
        {"low16", 0xffffull},
        {"lane0", 1ull},
        {"even32", 0x5555555555555555ull},
        {"first8_of_16", 0x00ff00ff00ff00ffull},
        {"low48", 0xffffffffffffull},
        {"all64_again", ~0ull},
    };
    for (const M& mk : masks) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(e0);
            k_masked<<<blocks, 256>>>(out, 0.999f, 0.001f, mk.m);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        printf("{\"mask\": \"%s\", \"ms\": %.3f}\n", mk.name, best);
    }
    hipFree(out);
    return 0;
}
