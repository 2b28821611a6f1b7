// Exhaustive check on gfx950: is q = fma(fma(-x, r, 1), r, r) with r = v_rcp_f32(x) (one Newton
// step) bitwise equal to the IEEE 1.0f / x? Mismatches are histogrammed by the input's exponent.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint32_t base, unsigned long long* cnt) {
    const uint32_t u = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(u);
    const float b = 1.0f / x;
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r, 1.0f);
    const float q = fmaf(e, r, r);
    const bool both_nan = (q != q) && (b != b);
    if (!both_nan && __float_as_uint(q) != __float_as_uint(b)) atomicAdd(cnt + ((u >> 23) & 0xff), 1ull);
}

int main() {
    unsigned long long* d;
    if (hipMalloc(&d, 256 * sizeof(unsigned long long)) != hipSuccess) return 1;
    if (hipMemset(d, 0, 256 * sizeof(unsigned long long)) != hipSuccess) return 1;
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < 0x100000000ull; base += chunk) k<<<chunk / 256, 256>>>((uint32_t)base, d);
    unsigned long long h[256];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    unsigned long long tot = 0;
    for (int e = 0; e < 256; e++) {
        if (h[e]) printf("biased exponent %3d: %llu mismatches\n", e, h[e]);
        tot += h[e];
    }
    printf("total mismatches: %llu\n", tot);
    return 0;
}
