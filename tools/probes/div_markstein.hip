// Checks on gfx950 that Markstein's division (y = one-Newton reciprocal, q = a y, one residual
// correction) is bitwise the IEEE quotient a / b:
//   (1) exhaustively for the Mandelbulb iteration's w = sqrt(a) / (a^2 a^2), every float a in
//       [2^-30, 2^31] (rmr_math.h div_mk in mb_iter8_poly);
//   (2) the reciprocal itself for every normal b with |b| in [2^-125, 2^125];
//   (3) 2^34 pseudo-random pairs with |a|, |b| in [2^-60, 2^60) (quotient and residual normal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../raymarchrenderer_amd/csrc/rmr_math.h"

using namespace rmr;

__global__ void k_mb(uint32_t lo, uint32_t n, unsigned long long* cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = __uint_as_float(lo + i);
    const float s = sqrt_cr(a), a2 = a * a, b = a2 * a2;
    if (__float_as_uint(div_mk(s, b)) != __float_as_uint(s / b)) atomicAdd(cnt + 0, 1ull);
}

__global__ void k_rcp(uint32_t lo, uint32_t n, unsigned long long* cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float b = __uint_as_float(lo + i);
    if (__float_as_uint(rcp_cr(b)) != __float_as_uint(1.0f / b)) atomicAdd(cnt + 1, 1ull);
    if (__float_as_uint(rcp_cr(-b)) != __float_as_uint(1.0f / -b)) atomicAdd(cnt + 1, 1ull);
}

__device__ uint32_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}
__global__ void k_rand(uint64_t base, unsigned long long* cnt) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = mix(2 * i), v = mix(2 * i + 1);
    // exponent fields: a, b in [2^-60, 2^60); random mantissas and signs
    const uint32_t ea = 127 - 60 + (u >> 24) % 120, eb = 127 - 60 + (v >> 24) % 120;
    const float a = __uint_as_float((u & 0x807fffffu) | (ea << 23));
    const float b = __uint_as_float((v & 0x807fffffu) | (eb << 23));
    if (__float_as_uint(div_mk(a, b)) != __float_as_uint(a / b)) atomicAdd(cnt + 2, 1ull);
}

int main() {
    unsigned long long* d;
    if (hipMalloc(&d, 4 * sizeof(unsigned long long)) != hipSuccess) return 1;
    if (hipMemset(d, 0, 4 * sizeof(unsigned long long)) != hipSuccess) return 1;
    const uint32_t lo = __builtin_bit_cast(uint32_t, 0x1p-30f), hi = __builtin_bit_cast(uint32_t, 0x1p31f);
    k_mb<<<(hi - lo + 256) / 256, 256>>>(lo, hi - lo + 1, d);
    const uint32_t rlo = __builtin_bit_cast(uint32_t, 0x1p-125f), rhi = __builtin_bit_cast(uint32_t, 0x1p125f);
    k_rcp<<<(rhi - rlo + 256) / 256, 256>>>(rlo, rhi - rlo + 1, d);
    const uint64_t chunk = 1ull << 30;
    for (uint64_t base = 0; base < (1ull << 34); base += chunk) k_rand<<<(uint32_t)(chunk / 256), 256>>>(base, d);
    unsigned long long h[4];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("mandelbulb w = sqrt(a)/a^4, a in [2^-30, 2^31]: %llu mismatches of %u\n", h[0], hi - lo + 1);
    printf("reciprocal, |b| in [2^-125, 2^125]: %llu mismatches of %u\n", h[1], 2 * (rhi - rlo + 1));
    printf("random pairs: %llu mismatches of %llu\n", h[2], 1ull << 34);
    return (h[0] || h[1] || h[2]) ? 3 : 0;
}
