/* Exhaustive check of sd_logf (include/sdsp_libm.h) over every positive finite f32:
 * against the correctly rounded value (x87 logl rounded to f32) and against the previous
 * double-series algorithm.  gcc -O2 -ffp-contract=off -march=x86-64-v3 -fopenmp */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include "../include/sdsp_libm.h"

int main(void) {
    long long bad_cr = 0, diff_old = 0;
    uint32_t first_bad = 0;
#pragma omp parallel for reduction(+ : bad_cr, diff_old) schedule(static, 1 << 20)
    for (long long u = 1; u < 0x7f800000LL; u++) {
        const float x = sd_from_bits_f((uint32_t)u);
        const float got = sd_logf(x);
        const float cr = (float)logl((long double)x);
        const float old = (float)sd_log_d((double)x);
        if (sd_bits_f(got) != sd_bits_f(cr)) {
            bad_cr++;
            first_bad = (uint32_t)u;
        }
        if (sd_bits_f(got) != sd_bits_f(old)) diff_old++;
    }
    printf("positive finite f32: %lld differ from correctly rounded (logl), %lld differ from the old series; last bad 0x%08x\n",
           bad_cr, diff_old, first_bad);
    return 0;
}
