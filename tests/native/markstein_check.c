/* markstein_check.c -- div_known (csrc/pd_physics.h) against IEEE division, on the host.
 *
 * The step kernel divides by literals and per-handle constants through their correctly rounded
 * reciprocals rb = RN(1/b): q = RN(a rb), r = fma(-b, q, a), result -fma(-r, rb, -q).  Both the
 * host's fma and gfx950's v_fma_f64 / v_fma_f32 are IEEE fused multiply-adds, so the host sees
 * the device's bits.  For every divisor given on the command line this checks, in binary64 and in
 * binary32, random numerators over a wide exponent range (and signed zeros, integers, values
 * near powers of two and the divisor's own multiples) bit for bit against a / b.
 *   markstein_check N b1 b2 ...     (prints the number of mismatches; exit 1 on any)
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

static double div_known(double a, double b, double rb) {
    const double q = a * rb;
    const double r = fma(-b, q, a);
    return -fma(-r, rb, -q);
}
static float div_known_f(float a, float b, float rb) {
    const float q = a * rb;
    const float r = fmaf(-b, q, a);
    return -fmaf(-r, rb, -q);
}

static int same_d(double x, double y) { return memcmp(&x, &y, sizeof x) == 0; }
static int same_f(float x, float y) { return memcmp(&x, &y, sizeof x) == 0; }

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s N b1 [b2 ...]\n", argv[0]); return 2; }
    const long n = atol(argv[1]);
    long bad = 0, tried = 0;
    for (int k = 2; k < argc; ++k) {
        const double b = strtod(argv[k], NULL);
        const double rb = 1.0 / b;
        const float bf = (float)b, rbf = 1.0f / bf;
        for (long i = 0; i < n; ++i) {
            const uint64_t u = next();
            double a;
            switch (i & 7) {
                case 0: a = ldexp((double)(u >> 11) * 0x1p-53 + 0.5, (int)(u % 121) - 60); break;  /* wide exponents */
                case 1: a = (double)(int64_t)(u % 2000001) - 1000000.0; break;                      /* integers */
                case 2: a = b * (double)(int64_t)(u % 20001 - 10000); break;                        /* multiples of b */
                case 3: a = ldexp(1.0, (int)(u % 81) - 40) * (1.0 + ((u >> 20) % 5 - 2) * 0x1p-52); break;  /* near 2^k */
                default: { double m = (double)(u >> 11) * 0x1p-53; a = (m - 0.5) * 2e6; }                   /* physics range */
            }
            if (i == 0) a = 0.0;
            if (i == 1) a = -0.0;
            if ((u >> 63) && (i & 7) != 1) a = -a;
            ++tried;
            if (!same_d(div_known(a, b, rb), a / b)) {
                if (bad < 10) fprintf(stderr, "f64 b=%.17g a=%.17g: %.17g vs %.17g\n", b, a, div_known(a, b, rb), a / b);
                ++bad;
            }
            const float af = (float)a;
            if (!same_f(div_known_f(af, bf, rbf), af / bf)) {
                if (bad < 10) fprintf(stderr, "f32 b=%.9g a=%.9g: %.9g vs %.9g\n", bf, af, div_known_f(af, bf, rbf), af / bf);
                ++bad;
            }
        }
    }
    printf("%ld %ld\n", bad, tried);
    return bad ? 1 : 0;
}
