// Checks the reciprocal-correction division used by k_features2's staging against IEEE division:
//   y = RN(1/b), q = RN(a*y), r = fma(-q, b, a), q' = fma(r, y, q)  ==  RN(a/b) ?
// for a in [0, b] (the normalised magnitudes x / max with x <= max).  b: 4096 random f32 plus
// significands at the binade edges (1.0, 1.000..01, 1.111..1, 1.111..10), over exponents
// -100..100; a: every f32 with the 2^20 significands nearest each binade edge of [b*2^-24, b]
// plus 2^22 random ones.  With the kernel's guard (a or the quotient below 2^-100 -> IEEE
// division) there must be no mismatch; without it the fast path errs only in the subnormal range.  Prints the mismatch count; -ffp-contract=off, fmaf is exact.
// gcc -O2 -march=x86-64-v3 -ffp-contract=off -o check_div_rcp check_div_rcp.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t rng = 88172645463325252ull;
static uint64_t xs(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

static long check(float b, long* n) {
    const float y = 1.0f / b;
    long bad = 0;
    const uint32_t ub = bf(b);
    for (long i = 0; i < (1l << 22); i++) {
        uint32_t ua;
        if (i < (1l << 21)) ua = ub - (uint32_t)(i % (1 << 21));          // just below b, down ~2 binades' worth
        else ua = (uint32_t)(xs() % (uint64_t)ub);                      // anywhere in [0, b)
        const float a = fb(ua);
        if (!(a >= 0.0f) || a > b) continue;
        const float q = a * y;
        const float r = fmaf(-q, b, a);
        float q2 = fmaf(r, y, q);
        if (q2 < 0x1p-100f || a < 0x1p-100f) q2 = a / b;  // the kernel's guard: small operands take IEEE division
        const float ref = a / b;
        (*n)++;
        if (bf(q2) != bf(ref)) {
            if (bad < 5) printf("mismatch a=%a b=%a got %a want %a\n", a, b, q2, ref);
            bad++;
        }
    }
    return bad;
}

int main(void) {
    long bad = 0, n = 0;
    const uint32_t sig[] = {0x000000, 0x000001, 0x7FFFFF, 0x7FFFFE, 0x400000, 0x2AAAAB, 0x555555};
    for (int e = -100; e <= 100; e += 7)
        for (unsigned s = 0; s < sizeof sig / sizeof sig[0]; s++) bad += check(fb(((uint32_t)(e + 127) << 23) | sig[s]), &n);
    for (int k = 0; k < 600; k++) {
        const uint32_t e = 127 - 60 + (uint32_t)(xs() % 120);
        bad += check(fb((e << 23) | (uint32_t)(xs() & 0x7FFFFF)), &n);
    }
    printf("checked %ld quotients, %ld mismatches\n", n, bad);
    return bad != 0;
}
