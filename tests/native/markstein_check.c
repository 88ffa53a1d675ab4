/* markstein_check.c -- div_known (csrc/pd_physics.h) against IEEE division, on the host.
 *
 * The step kernel divides by literals and per-handle constants through their correctly rounded
 * reciprocals rb = RN(1/b): q = RN(a rb), r = fma(-b, q, a), then (for a divisor whose
 * eps = b rb - 1 exceeds 2^-(p+1) in magnitude, times 0.99) one more correction
 * q = -fma(-r, rb, -q), r = fma(-b, q, a), and the result -fma(-r, rb, -q).  Both the host's fma
 * and gfx950's v_fma_f64 / v_fma_f32 are IEEE fused multiply-adds, so the host sees the device's
 * bits.  eps is exact here: fma(b, rb, -1) has at most 53 (24) significant bits.
 *   markstein_check classify b1 b2 ...        per divisor: "b one_step64 one_step32"
 *   markstein_check sample N b1 b2 ...        N random numerators per divisor, binary64 and binary32
 *   markstein_check mantissas32 b1 b2 ...     every signed binary32 mantissa at exponents -99, -40, 0, 40,
 *                                             100 (q, r and the corrections scale exactly by 2^e while
 *                                             no intermediate leaves the normal range, so this covers
 *                                             the exhaustive check's domain; seconds instead of minutes)
 *   markstein_check exhaustive32 b1 b2 ...    every binary32 numerator of magnitude 0 or >= 2^-100 with
 *                                             a finite quotient of magnitude 0 or >= 2^-100 (below, the
 *                                             remainder a - b q is subnormal and the theorem does not
 *                                             apply; no quantity of the step is that small)
 * The check modes print "<mismatches> <numerators tried>" and exit 1 on any mismatch.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {   /* splitmix64 */
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int one_step_d(double b, double rb) { const double e = fma(b, rb, -1.0); return fabs(e) <= 0.99 * 0x1p-54; }
static int one_step_f(float b, float rb) { const float e = fmaf(b, rb, -1.0f); return fabsf(e) <= 0.99f * 0x1p-25f; }

static double div_known(double a, double b, double rb, int two) {
    double q = a * rb;
    double r = fma(-b, q, a);
    if (two) { q = -fma(-r, rb, -q); r = fma(-b, q, a); }
    return -fma(-r, rb, -q);
}
static float div_known_f(float a, float b, float rb, int two) {
    float q = a * rb;
    float r = fmaf(-b, q, a);
    if (two) { q = -fmaf(-r, rb, -q); r = fmaf(-b, q, a); }
    return -fmaf(-r, rb, -q);
}

static int same_d(double x, double y) { return memcmp(&x, &y, sizeof x) == 0; }
static int same_f(float x, float y) { return memcmp(&x, &y, sizeof x) == 0; }

static int sample(long n, int nb, char** bs) {
    long bad = 0, tried = 0;
    for (int k = 0; k < nb; ++k) {
        const double b = strtod(bs[k], NULL);
        const double rb = 1.0 / b;
        const int two = !one_step_d(b, rb);
        const float bf = (float)b, rbf = 1.0f / bf;
        const int twof = !one_step_f(bf, rbf);
        for (long i = 0; i < n; ++i) {
            const uint64_t u = next();
            double a;
            switch (i & 7) {
                case 0: a = ldexp((double)(u >> 11) * 0x1p-53 + 0.5, (int)(u % 121) - 60); break;  /* wide exponents */
                case 1: a = (double)(int64_t)(u % 2000001) - 1000000.0; break;                      /* integers */
                case 2: a = b * (double)(int64_t)(u % 20001 - 10000); break;                        /* multiples of b */
                case 3: a = ldexp(1.0, (int)(u % 81) - 40) * (1.0 + ((u >> 20) % 5 - 2) * 0x1p-52); break;  /* near 2^k */
                case 4: { /* quotients at the top of a binade, where RN(a rb) may be 1.5 ulp off */
                    const double m = 2.0 - (double)(u % 4096) * 0x1p-52;
                    a = ldexp(m, (int)((u >> 16) % 41) - 20) * b;
                    break;
                }
                default: { double m = (double)(u >> 11) * 0x1p-53; a = (m - 0.5) * 2e6; }                   /* physics range */
            }
            if (i == 0) a = 0.0;
            if (i == 1) a = -0.0;
            if ((u >> 63) && (i & 7) != 1) a = -a;
            ++tried;
            if (!same_d(div_known(a, b, rb, two), a / b)) {
                if (bad < 10) fprintf(stderr, "f64 b=%.17g a=%.17g: %.17g vs %.17g\n", b, a, div_known(a, b, rb, two), a / b);
                ++bad;
            }
            const float af = (float)a;
            if (!same_f(div_known_f(af, bf, rbf, twof), af / bf)) {
                if (bad < 10) fprintf(stderr, "f32 b=%.9g a=%.9g: %.9g vs %.9g\n", bf, af, div_known_f(af, bf, rbf, twof), af / bf);
                ++bad;
            }
        }
    }
    printf("%ld %ld\n", bad, tried);
    return bad ? 1 : 0;
}

static int exhaustive32(int nb, char** bs) {
    long long bad = 0, tried = 0;
    for (int k = 0; k < nb; ++k) {
        const float b = (float)strtod(bs[k], NULL), rb = 1.0f / b;
        const int two = !one_step_f(b, rb);
        long long kb = 0, kt = 0;
#pragma omp parallel for reduction(+ : kb, kt) schedule(static)
        for (long long w = 0; w < (1ll << 32); ++w) {
            const uint32_t bits = (uint32_t)w;
            float a;
            memcpy(&a, &bits, 4);
            const float q = a / b;
            /* finite numerators, zero or of magnitude >= 2^-100, whose quotient is finite and zero or
             * >= 2^-100: Markstein's remainder r ~ a 2^-24 must not be subnormal */
            if (!isfinite(a) || !isfinite(q)) continue;
            if (a != 0.0f && (fabsf(a) < 0x1p-100f || fabsf(q) < 0x1p-100f)) continue;
            ++kt;
            if (!same_f(div_known_f(a, b, rb, two), q)) ++kb;
        }
        if (kb) fprintf(stderr, "f32 b=%.9g: %lld mismatches\n", b, kb);
        bad += kb;
        tried += kt;
    }
    printf("%lld %lld\n", bad, tried);
    return bad ? 1 : 0;
}

static int mantissas32(int nb, char** bs) {
    static const int ex[5] = {-99, -40, 0, 40, 100};
    long long bad = 0, tried = 0;
    for (int k = 0; k < nb; ++k) {
        const float b = (float)strtod(bs[k], NULL), rb = 1.0f / b;
        const int two = !one_step_f(b, rb);
        long long kb = 0, kt = 0;
#pragma omp parallel for reduction(+ : kb, kt) schedule(static)
        for (long long w = 0; w < 5ll << 24; ++w) {
            const int e = ex[w >> 24];
            const uint32_t m = (uint32_t)w & 0x7fffffu, sg = ((uint32_t)w >> 23) & 1u;
            const uint32_t bits = (sg << 31) | ((uint32_t)(e + 127) << 23) | m;
            float a;
            memcpy(&a, &bits, 4);
            const float q = a / b;
            if (!isfinite(q) || fabsf(q) < 0x1p-100f) continue;
            ++kt;
            if (!same_f(div_known_f(a, b, rb, two), q)) ++kb;
        }
        if (kb) fprintf(stderr, "f32 b=%.9g: %lld mismatches\n", b, kb);
        bad += kb;
        tried += kt;
    }
    printf("%lld %lld\n", bad, tried);
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc >= 3 && !strcmp(argv[1], "classify")) {
        for (int k = 2; k < argc; ++k) {
            const double b = strtod(argv[k], NULL);
            const float bf = (float)b;
            printf("%.17g %d %d\n", b, one_step_d(b, 1.0 / b), one_step_f(bf, 1.0f / bf));
        }
        return 0;
    }
    if (argc >= 4 && !strcmp(argv[1], "sample")) return sample(atol(argv[2]), argc - 3, argv + 3);
    if (argc >= 3 && !strcmp(argv[1], "exhaustive32")) return exhaustive32(argc - 2, argv + 2);
    if (argc >= 3 && !strcmp(argv[1], "mantissas32")) return mantissas32(argc - 2, argv + 2);
    fprintf(stderr, "usage: %s classify|sample N|mantissas32|exhaustive32 b1 [b2 ...]\n", argv[0]);
    return 2;
}
