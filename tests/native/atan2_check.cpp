// Host check of atan2_fd (csrc/pd_common.h) against glibc's atan2 (what the reference's
// math.atan2 / np.arctan2 call): the largest difference in units in the last place, and how many
// results differ at all, over random arguments -- the descent's velocity range (vx, vy), all four
// quadrants at log-uniform magnitudes, and ratios at the reduction intervals' edges.
#include "pd_common.h"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
using namespace pd;

static uint64_t st = 0x243F6A8885A308D3ull;
static uint64_t nx() {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01() { return (double)(nx() >> 11) * 0x1p-53; }
static int64_t ord(double v) {   // monotone integer image of a double
    int64_t i;
    std::memcpy(&i, &v, 8);
    return i < 0 ? INT64_MIN - i : i;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    long diff = 0, total = 0;
    int64_t worst = 0;
    double wy = 0, wx = 0;
    const double edges[] = {0.4375, 0.6875, 1.1875, 2.4375};
    for (long i = 0; i < 4 * n; ++i) {
        double y, x;
        const int kind = (int)(i % 4);
        if (kind == 0) { x = -300.0 + 350.0 * u01(); y = -1100.0 + 1110.0 * u01(); }             // descent vx, vy
        else if (kind == 1) {
            x = std::exp((u01() - 0.5) * 46.0) * ((nx() & 1) ? -1.0 : 1.0);                    // 1e-10 .. 1e10
            y = std::exp((u01() - 0.5) * 46.0) * ((nx() & 1) ? -1.0 : 1.0);
        } else if (kind == 2) {
            x = std::exp((u01() - 0.5) * 20.0) * ((nx() & 1) ? -1.0 : 1.0);
            const double e = edges[nx() % 4] * (1.0 + (u01() - 0.5) * 1e-6);                  // interval edges
            y = std::fabs(x) * e * ((nx() & 1) ? -1.0 : 1.0);
        } else { x = (u01() - 0.5) * 2.0; y = (u01() - 0.5) * 2.0; }
        if (x == 0.0 || y == 0.0) continue;
        const double a = atan2_fd(y, x), b = std::atan2(y, x);
        ++total;
        const int64_t d = ord(a) > ord(b) ? ord(a) - ord(b) : ord(b) - ord(a);
        if (d) ++diff;
        if (d > worst) { worst = d; wy = y; wx = x; }
    }
    std::printf("total %ld differ %ld worst_ulp %lld at y=%.17g x=%.17g\n", total, diff, (long long)worst, wy, wx);
    return worst <= 1 ? 0 : 1;
}
