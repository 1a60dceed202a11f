/* Exhaustive check that  q = fma(fma(-q0, d, a), y, q0),  q0 = a*y,  y = 1/d (f32)
 * equals the correctly rounded a/d for every non-negative finite f32 a and each small
 * integer divisor d used by the harmonic-mask moving average (window lengths M+1 .. 2M+1).
 * gcc -O2 -ffp-contract=off -march=x86-64-v3 -fopenmp tools/check_div.c -lm */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    int lo = argc > 1 ? atoi(argv[1]) : 1, hi = argc > 2 ? atoi(argv[2]) : 64;
    for (int di = lo; di <= hi; di++) {
        const float d = (float)di, y = 1.0f / d;
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static, 1 << 20)
        for (long long u = 0; u < 0x7f800000LL; u++) {
            const float a = fb((uint32_t)u);
            const float q0 = a * y;
            const float r = fmaf(-q0, d, a);
            const float q = fmaf(r, y, q0);
            if (bf(q) != bf(a / d)) bad++;
        }
        printf("d=%d bad=%lld\n", di, bad);
        fflush(stdout);
    }
    return 0;
}
