// Exhaustive checks on gfx950 over all 2^32 float bit patterns:
//  (1) is v_sqrt_f32 / v_rcp_f32 correctly rounded?  (no: hipcc's IEEE lowering adds a fix-up)
//  (2) is rmr::sqrt_cr (v_sqrt_f32 + one-ulp fix-up, divergent sqrtf() for 0 < x < 2^-96) bitwise
//      equal to sqrtf() for every input (NaN compared as NaN)?  The kernels rely on it.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/sqrt_exhaustive.hip -o tools/probes/sqrt_exhaustive
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../raymarchrenderer_amd/csrc/rmr_math.h"

__global__ void k(uint32_t base, unsigned long long* cnt) {
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(u);
    const float b = sqrtf(x);
    const uint32_t a = u & 0x7fffffffu;
    if (u < 0x7f800000u) {
        const int bucket = (u < 0x00800000u) ? 0 : (u < 0x0f800000u ? 1 : 2);  // denormal / < 2^-96 / rest
        if (__float_as_uint(__builtin_amdgcn_sqrtf(x)) != __float_as_uint(b)) atomicAdd(cnt + bucket, 1ull);
        if (__float_as_uint(__builtin_amdgcn_rcpf(x)) != __float_as_uint(1.0f / x)) atomicAdd(cnt + 3 + bucket, 1ull);
    }
    const float f = rmr::sqrt_cr(x);
    const bool both_nan = (f != f) && (b != b);
    if (!both_nan && __float_as_uint(f) != __float_as_uint(b)) atomicAdd(cnt + 6, 1ull);
    if (a > 0x7f800000u && !(f != f)) atomicAdd(cnt + 7, 1ull);  // NaN in, non-NaN out
}

int main() {
    unsigned long long* d;
    if (hipMalloc(&d, 8 * sizeof(unsigned long long)) != hipSuccess) return 1;
    if (hipMemset(d, 0, 8 * sizeof(unsigned long long)) != hipSuccess) return 1;
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < 0x100000000ull; base += chunk) k<<<chunk / 256, 256>>>((uint32_t)base, d);
    unsigned long long h[8];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("v_sqrt_f32 mismatches vs IEEE: denormal=%llu tiny(<2^-96)=%llu normal=%llu\n", h[0], h[1], h[2]);
    printf("v_rcp_f32  mismatches vs IEEE: denormal=%llu tiny(<2^-96)=%llu normal=%llu\n", h[3], h[4], h[5]);
    printf("rmr::sqrt_cr mismatches vs sqrtf over all 2^32 inputs: %llu ; NaN lost: %llu\n", h[6], h[7]);
    return (h[6] == 0 && h[7] == 0) ? 0 : 3;
}
