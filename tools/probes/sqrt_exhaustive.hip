// Exhaustive check: is gfx950's v_sqrt_f32 (no fix-up sequence) correctly rounded?
// Compares __builtin_amdgcn_sqrtf(x) with the IEEE-correct sqrtf(x) (hipcc's default lowering)
// for every non-negative finite float bit pattern, split by input range.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint32_t base, unsigned long long* cnt) {
    uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= 0x7f800000u) return;
    float x = __uint_as_float(u);
    float a = __builtin_amdgcn_sqrtf(x);
    float b = sqrtf(x);
    unsigned long long bad = (__float_as_uint(a) != __float_as_uint(b)) ? 1ull : 0ull;
    int bucket = (u < 0x00800000u) ? 0 : (u < 0x0f800000u ? 1 : 2);  // denormal / < 2^-96 / rest
    if (bad) atomicAdd(cnt + bucket, 1ull);
    // reciprocal: v_rcp_f32 vs 1/x
    float r1 = __builtin_amdgcn_rcpf(x);
    float r2 = 1.0f / x;
    if (__float_as_uint(r1) != __float_as_uint(r2)) atomicAdd(cnt + 3 + bucket, 1ull);
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8 * sizeof(unsigned long long));
    hipMemset(d, 0, 8 * sizeof(unsigned long long));
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < 0x7f800000ull; base += chunk) k<<<chunk / 256, 256>>>((uint32_t)base, d);
    unsigned long long h[8];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("sqrt mismatches: denormal=%llu tiny(<2^-96)=%llu normal=%llu\n", h[0], h[1], h[2]);
    printf("rcp  mismatches: denormal=%llu tiny(<2^-96)=%llu normal=%llu\n", h[3], h[4], h[5]);
    return 0;
}
