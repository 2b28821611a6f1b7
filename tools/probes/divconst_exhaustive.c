/* Exhaustive check (all 2^32 float inputs, CPU) of division by a constant with two FMAs:
 *     q0 = x * rc;  r = fma(-q0, y, x);  q1 = fma(r, rc, q0)      rc = RN(1 / y)
 * against the IEEE quotient x / y. Usage: divconst_exhaustive 3.14
 * Prints the number of mismatching inputs by class (finite / inf-nan) and the smallest and
 * largest |x| of a finite mismatch. Build: gcc -O2 -mfma -fopenmp -ffp-contract=off */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    const float y = argc > 1 ? strtof(argv[1], NULL) : 3.14f;
    const float rc = 1.0f / y;
    unsigned long long bad_fin = 0, bad_inf = 0;
    float lo = INFINITY, hi = 0.0f;
#pragma omp parallel for reduction(+ : bad_fin, bad_inf) reduction(min : lo) reduction(max : hi) schedule(static)
    for (long long i = 0; i < (1LL << 32); i++) {
        const float x = u2f((uint32_t)i);
        const float ref = x / y;
        const float q0 = x * rc;
        const float r = fmaf(-q0, y, x);
        const float q1 = fmaf(r, rc, q0);
        const int same = (f2u(q1) == f2u(ref)) || (isnan(q1) && isnan(ref));
        if (!same) {
            if (isfinite(x)) {
                bad_fin++;
                const float ax = fabsf(x);
                if (ax < lo) lo = ax;
                if (ax > hi) hi = ax;
            } else {
                bad_inf++;
            }
        }
    }
    printf("y=%a rc=%a finite_mismatch=%llu nonfinite_mismatch=%llu min|x|=%a max|x|=%a\n", y, rc, bad_fin, bad_inf,
           lo, hi);
    return 0;
}
