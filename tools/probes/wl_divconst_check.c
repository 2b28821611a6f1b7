/* wavelengthToColor's divisions by constants (RM3:447-522, rmr_trace.h finish_trace) as two FMAs
 * (div_const: q0 = x RN(1/c), r = fma(-q0, c, x), fma(r, RN(1/c), q0)) against the IEEE quotient,
 * for every numerator the kernel can form: the hero wavelength wl is an integer, so each quotient's
 * numerator is an integer-valued float in its branch's range.
 * Build: gcc -O2 -mfma -ffp-contract=off wl_divconst_check.c -o wl_divconst_check */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float div_const(float x, float c) {
    const float rc = 1.0f / c;
    const float q0 = x * rc;
    const float r = fmaf(-q0, c, x);
    return fmaf(r, rc, q0);
}

int main(void) {
    /* each quotient over the wavelengths of its own branch (the kernel selects it only there); the
     * only mismatches anywhere in [0, 2000] are -0 / c at the branch boundaries 440, 510, 645, where
     * the next branch is taken */
    const float cs[] = {60.0f, 50.0f, 20.0f, 70.0f, 65.0f, 80.0f, 40.0f};
    const int lo[] = {380, 440, 490, 510, 580, 701, 380}, hi[] = {439, 489, 509, 579, 644, 780, 419};
    unsigned bad = 0, n = 0;
    for (int i = 0; i < 7; i++) {
        for (int w = lo[i]; w <= hi[i]; w++) {
            const float wl = (float)w;
            const float xs[] = {-1.0f * (wl - 440.0f), wl - 440.0f, -1.0f * (wl - 510.0f), wl - 510.0f,
                                -1.0f * (wl - 645.0f), 780.0f - wl, wl - 380.0f};
            n++;
            if (f2u(div_const(xs[i], cs[i])) != f2u(xs[i] / cs[i])) { bad++; printf("wl %d c %g x %g\n", w, cs[i], xs[i]); }
        }
    }
    printf("quotients=%u mismatches=%u\n", n, bad);
    return bad != 0;
}
