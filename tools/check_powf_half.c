/* Exhaustive check of sd_sqrt_is_powf_half (include/sdsp_libm.h): on every non-negative f32 x
 * (+0 .. +inf), sqrtf(x) where the test admits it equals sd_powf(x, 0.5f) bit for bit.
 * gcc -O2 -ffp-contract=off -march=x86-64-v3 -fopenmp tools/check_powf_half.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include "../include/sdsp_libm.h"

int main(void) {
    long long diff = 0, n = 0, slow = 0, plain = 0;
    uint32_t last = 0;
#pragma omp parallel for reduction(+ : diff, n, slow, plain) schedule(static, 1 << 20)
    for (long long u = 0; u <= 0x7f800000LL; u++) {
        const float x = sd_from_bits_f((uint32_t)u);
        const float s = sqrtf(x), p = sd_powf(x, 0.5f);
        const int ok = sd_sqrt_is_powf_half(x, s);
        n++;
        slow += !ok;
        plain += sd_bits_f(s) != sd_bits_f(p);
        if (ok && sd_bits_f(s) != sd_bits_f(p)) {
            diff++;
            last = (uint32_t)u;
        }
    }
    printf("x^0.5 by sqrtf where admitted: %lld inputs, %lld differ (last 0x%08x); %lld take sd_powf; "
           "sqrtf alone would differ on %lld\n", n, diff, last, slow, plain);
    return diff != 0;
}
