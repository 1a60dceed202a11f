/* Exhaustive checks: sd_logf_ge1_t2 (two-column table, no m / c formed) against sd_logf_ge1 on
 * every f32 >= 1 (finite, +inf) and a NaN; sd_ln1p_max0_t2(v) against
 * sd_logf_ge1_t2(1 + sd_maxf(v, 0)) on all 2^32 bit patterns of v; and (round 5) the 9-bit-table,
 * degree-4 sd_ln1p_x_t9_finite against sd_logf_ge1 on every finite f32 >= 1.
 * gcc -O2 -ffp-contract=off -march=x86-64-v3 -fopenmp */
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
    long long diff2 = 0, n2 = 0;
    uint32_t first2 = 0;
#pragma omp parallel for reduction(+ : diff2, n2) schedule(static, 1 << 20)
    for (long long u = 0; u <= 0xffffffffLL; u++) {
        const float v = sd_from_bits_f((uint32_t)u);
        const float a = sd_logf_ge1_t2(1.0f + sd_maxf(v, 0.0f), t2), b = sd_ln1p_max0_t2(v, t2);
        n2++;
        if (sd_bits_f(a) != sd_bits_f(b)) {
            diff2++;
            first2 = (uint32_t)u;
        }
    }
    printf("ln(1 + max(v, 0)), all v: %lld inputs, %lld differ (last 0x%08x)\n", n2, diff2, first2);
    sd_ln2tab_t et[129];
    for (int e = 0; e < 129; e++) et[e] = sd_ln2tab_from(e);
    long long diff3 = 0, n3 = 0;
    uint32_t first3 = 0;
#pragma omp parallel for reduction(+ : diff3, n3) schedule(static, 1 << 20)
    for (long long u = 0x3f800000LL; u < 0x7f800000LL; u++) {
        const float x = sd_from_bits_f((uint32_t)u);
        const float a = sd_logf_ge1(x, SD_LOGTAB_H), b = sd_ln1p_x_t9_finite(x, SD_LOGTAB9_H, et);
        n3++;
        if (sd_bits_f(a) != sd_bits_f(b)) {
            diff3++;
            first3 = (uint32_t)u;
        }
    }
    printf("9-bit table, degree 4, finite f32 >= 1: %lld inputs, %lld differ (last 0x%08x)\n", n3, diff3, first3);
    return diff != 0 || diff2 != 0 || diff3 != 0;
}
