// Follow-up of exec_half.hip (a wave whose EXEC holds <= 16 lanes ran an FMA loop ~2.9x slower than
// one with 17-64 lanes, profiles/r03e_exec_half_probe.log): is it a cost to the SIMD (other waves
// slowed too) or to the wave itself? Variants, each over the same grid and loop:
//   waves8_all / waves8_one   : 8 waves per SIMD, every wave 64 / 1 active lanes
//   waves8_mix                : 8 waves per SIMD, odd waves 1 lane, even waves 64
//   waves1_all / waves1_one   : 1 wave per SIMD (one block of 64 threads per SIMD slot)
//   chain1_all / chain1_one   : 8 waves per SIMD, ONE dependent FMA chain per lane (latency-bound)
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/probes/exec_mix.hip -o tools/probes/exec_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

// mode 0: every wave mask m0; mode 1: waves with odd wave index use m1
__global__ __launch_bounds__(256) void k_mix(float* out, float a, float b, uint64_t m0, uint64_t m1, int mode) {
    const int lane = __lane_id();
    const int wv = (int)(threadIdx.x >> 6);
    const uint64_t mask = (mode == 1 && (wv & 1)) ? m1 : m0;
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    if ((mask >> lane) & 1) {
        for (int i = 0; i < kIters; i++) {
            x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
            x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

__global__ __launch_bounds__(256) void k_chain(float* out, float a, float b, uint64_t m0) {
    const int lane = __lane_id();
    float x0 = threadIdx.x;
    if ((m0 >> lane) & 1) {
        for (int i = 0; i < 8 * kIters; i++) x0 = fmaf(x0, a, b);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0;
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float* out = nullptr;
    hipMalloc((void**)&out, (size_t)cus * 32 * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        printf("{\"case\": \"%s\", \"ms\": %.3f}\n", name, best);
    };
    const uint64_t ALL = ~0ull, ONE = 1ull;
    const int b8 = cus * 8;   // 8 blocks of 4 waves per CU = 8 waves per SIMD (one round)
    timeit("waves8_all", [&] { k_mix<<<b8, 256>>>(out, 0.999f, 0.001f, ALL, ALL, 0); });
    timeit("waves8_one", [&] { k_mix<<<b8, 256>>>(out, 0.999f, 0.001f, ONE, ONE, 0); });
    timeit("waves8_mix", [&] { k_mix<<<b8, 256>>>(out, 0.999f, 0.001f, ALL, ONE, 1); });
    timeit("waves4_all", [&] { k_mix<<<cus * 4, 256>>>(out, 0.999f, 0.001f, ALL, ALL, 0); });
    timeit("waves4_one", [&] { k_mix<<<cus * 4, 256>>>(out, 0.999f, 0.001f, ONE, ONE, 0); });
    timeit("waves1_all", [&] { k_mix<<<cus, 256>>>(out, 0.999f, 0.001f, ALL, ALL, 0); });
    timeit("waves1_one", [&] { k_mix<<<cus, 256>>>(out, 0.999f, 0.001f, ONE, ONE, 0); });
    timeit("chain1_all", [&] { k_chain<<<b8, 256>>>(out, 0.999f, 0.001f, ALL); });
    timeit("chain1_one", [&] { k_chain<<<b8, 256>>>(out, 0.999f, 0.001f, ONE); });
    timeit("chain1_17", [&] { k_chain<<<b8, 256>>>(out, 0.999f, 0.001f, 0x1ffffull); });
    hipFree(out);
    return 0;
}
