// FP32 vector peak of this MI355X, measured ("verify with a microbenchmark on the box"):
// every lane runs 8 independent FMA chains, scalar v_fma_f32 or packed v_pk_fma_f32 (two FMAs per
// instruction), on a full grid at 8 waves per SIMD. Prints TFLOP/s (FMA = 2 flops) for both forms.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/probes/fma_peak.hip -o tools/probes/fma_peak
// (-fno-slp-vectorize: otherwise the scalar kernel is compiled to packed FMAs as well)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

constexpr int kIters = 4096;

__global__ __launch_bounds__(256, 8) void k_scalar(float* out, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < kIters; i++) {
        x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
        x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

__global__ __launch_bounds__(256, 8) void k_packed(float* out, float a, float b) {
    const float2v av = {a, a}, bv = {b, b};
    float2v x0 = {(float)threadIdx.x, 1.0f}, x1 = x0 + 1.0f, x2 = x0 + 2.0f, x3 = x0 + 3.0f;
    float2v x4 = x0 + 4.0f, x5 = x0 + 5.0f, x6 = x0 + 6.0f, x7 = x0 + 7.0f;
    for (int i = 0; i < kIters; i++) {
        x0 = __builtin_elementwise_fma(x0, av, bv); x1 = __builtin_elementwise_fma(x1, av, bv);
        x2 = __builtin_elementwise_fma(x2, av, bv); x3 = __builtin_elementwise_fma(x3, av, bv);
        x4 = __builtin_elementwise_fma(x4, av, bv); x5 = __builtin_elementwise_fma(x5, av, bv);
        x6 = __builtin_elementwise_fma(x6, av, bv); x7 = __builtin_elementwise_fma(x7, av, bv);
    }
    const float2v s = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 8 * 4;   // 8 blocks of 4 waves per CU = 8 waves per SIMD, 4 rounds
    float* out = nullptr;
    hipMalloc((void**)&out, (size_t)blocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int form = 0; form < 2; form++) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(e0);
            if (form == 0) k_scalar<<<blocks, 256>>>(out, 0.999f, 0.001f);
            else k_packed<<<blocks, 256>>>(out, 0.999f, 0.001f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        const double fmas = (double)blocks * 256 * kIters * 8 * (form ? 2 : 1);
        printf("{\"form\": \"%s\", \"cus\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", form ? "v_pk_fma_f32" : "v_fma_f32",
               cus, best, 2.0 * fmas / (best * 1e-3) / 1e12);
    }
    hipFree(out);
    return 0;
}
