// Exhaustive check of acnet_kernels.hip div_tenth(): q = x * 10, r = fma(-q, 0.1f, x), y = fma(r, 10, q) equals the
// IEEE quotient x / 0.1f for every finite f32 x with |x| >= 2^-100 whose quotient is finite (tinier nonzero x take
// the division in the kernel).  ~1.5 min on one core.
//   gcc -O2 -o /tmp/div_tenth scripts/micro/div_tenth.c -lm && /tmp/div_tenth
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    long bad = 0, tot = 0;
    for (uint64_t u = 0; u < 0x100000000ull; ++u) {
        const uint32_t b = (uint32_t)u;
        float x;
        memcpy(&x, &b, 4);
        if (!isfinite(x) || fabsf(x) < 0x1p-100f) continue;
        const float ref = x / 0.1f;
        if (!isfinite(ref)) continue;
        const float q = x * 10.0f, r = fmaf(-q, 0.1f, x), y = fmaf(r, 10.0f, q);
        uint32_t a1, a2;
        memcpy(&a1, &ref, 4);
        memcpy(&a2, &y, 4);
        ++tot;
        if (a1 != a2) {
            if (bad < 5) printf("x=%a ref=%a got=%a\n", x, ref, y);
            ++bad;
        }
    }
    printf("checked %ld, mismatches %ld\n", tot, bad);
    return bad != 0;
}
