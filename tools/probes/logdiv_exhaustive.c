/* Exhaustive check (CPU) of det_log's s = f / (2 + f) by Markstein's correction (rmr_math.h div_mk,
 * RMR_LOG_DIVMK) for every positive finite float x that reaches it: f = m - 1 of det_log's
 * reduction (m in [sqrt(1/2), sqrt(2)), so only the 2^24-odd distinct m matter, but every x is run).
 * rcp_cr(b) is RN(1 / b) on the device for |b| in [2^-125, 2^125] (rcp_exhaustive.hip), so here
 * y = 1 / b (IEEE). Prints the number of mismatches against the IEEE quotient.
 * Build: gcc -O2 -mfma -fopenmp -ffp-contract=off logdiv_exhaustive.c -o logdiv -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(void) {
    unsigned long long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(static)
    for (long long i = 1; i < 0x7f800000LL; i++) {   // every positive finite x (denormals included)
        float x = u2f((uint32_t)i);
        uint32_t u = f2u(x);
        if (u < 0x00800000u) { x = x * 16777216.0f; u = f2u(x); }
        u += 0x3f800000u - 0x3f3504f3u;
        u = (u & 0x007fffffu) + 0x3f3504f3u;
        const float f = u2f(u) - 1.0f;
        const float b = 2.0f + f;
        const float ref = f / b;
        const float y = 1.0f / b;
        const float q = f * y;
        const float s = fmaf(fmaf(-b, q, f), y, q);
        n++;
        if (f2u(s) != f2u(ref)) bad++;
    }
    printf("inputs=%llu mismatches=%llu\n", n, bad);
    return bad != 0;
}
