// Exhaustive check: for every integer window size b in [B_LO, B_HI] and every fp32 a in
// [2^-40, 2^16), is fma(fma(-q0, b, a), y, q0) with y = RN(1/b), q0 = RN(a*y) equal to the
// correctly rounded a / b?  (Aggregation's "C /= windowSize", ADCensus.cpp:743-749.)
// Also a = 0.  Build: gcc -O3 -march=native -fopenmp -ffp-contract=off div_check.c -lm
// B_HI = 6561 = 81 x 81 covers every window of arms up to 40 (maxLength1 <= 41: the
// streamers' limit); the run over [1, 4489] is the default parameters' 67 x 67.
#ifndef B_LO
#define B_LO 1
#endif
#ifndef B_HI
#define B_HI 6561
#endif
#ifndef LO_BITS
#define LO_BITS 0x2b800000u  /* 2^-40 */
#endif
#ifndef HI_BITS
#define HI_BITS 0x47800000u  /* 2^16 */
#endif
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
int main(void) {
    const uint32_t lo = LO_BITS;
    const uint32_t hi = HI_BITS;
    long long bad = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : bad)
    for (int b = B_LO; b <= B_HI; ++b) {
        const float fb = (float)b;
        const float y = 1.0f / fb;
        long long nb = 0;
        for (uint32_t u = lo; u < hi; ++u) {
            const float a = bits2f(u);
            const float q0 = a * y;
            const float r = fmaf(-q0, fb, a);
            const float q = fmaf(r, y, q0);
            const float ref = a / fb;
            nb += (q != ref);
        }
        if (nb) {
#pragma omp critical
            printf("b=%d mismatches=%lld\n", b, nb);
        }
        bad += nb;
    }
    printf("total mismatches: %lld\n", bad);
    return bad != 0;
}
