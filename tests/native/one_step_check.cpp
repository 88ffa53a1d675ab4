// The step kernel's own divisor classification (pd::one_step_ok, csrc/pd_physics.h: the compiler
// folds it for literal divisors, pd_create evaluates it for the handle's) on the host, for
// tests/test_markstein.py to compare with the exact rule.  Prints "b one_step64 one_step32".
#include <cstdio>
#include <cstdlib>

#include "pd_physics.h"

int main(int argc, char** argv) {
    for (int k = 1; k < argc; ++k) {
        const double b = std::strtod(argv[k], nullptr);
        const float bf = (float)b;
        std::printf("%.17g %d %d\n", b, (int)pd::one_step_ok<double>(b, 1.0 / b), (int)pd::one_step_ok<float>(bf, 1.0f / bf));
    }
    return 0;
}
