/* Exhaustive check: sd_logf_ge1_t2 (two-column table, no m / c formed) against sd_logf_ge1 on
 * every f32 >= 1 (finite, +inf) and a NaN.  gcc -O2 -ffp-contract=off -march=x86-64-v3 -fopenmp */
#include <stdio.h>
#include <stdint.h>
#include "../include/sdsp_libm.h"

int main(void) {
    sd_logtab2_t t2[128];
    for (int i = 0; i < 128; i++) t2[i] = sd_logtab2_from(SD_LOGTAB_H, i);
    long long diff = 0, n = 0;
    uint32_t first = 0;
#pragma omp parallel for reduction(+ : diff, n) schedule(static, 1 << 20)
    for (long long u = 0x3f800000LL; u <= 0x7fc00000LL; u++) {
        const float x = sd_from_bits_f((uint32_t)u);
        const float a = sd_logf_ge1(x, SD_LOGTAB_H), b = sd_logf_ge1_t2(x, t2);
        n++;
        if (sd_bits_f(a) != sd_bits_f(b)) {
            diff++;
            first = (uint32_t)u;
        }
    }
    printf("f32 >= 1: %lld inputs, %lld differ (last 0x%08x)\n", n, diff, first);
    return diff != 0;
}
