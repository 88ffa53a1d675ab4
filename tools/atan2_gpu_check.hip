// atan2 on the device against glibc's on the host: the device library's atan2 (ocml) and
// atan2_fd (pd_common.h) over the arguments of tests/native/atan2_check.cpp's descent range and
// all four quadrants.  Prints, for each, how many results differ from glibc and the worst ulp;
// and whether atan2_fd gives the same bits on the device as on the host.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I psso-sac-for-powered-descent_amd/csrc \
//         tools/atan2_gpu_check.hip -o tools/bin/atan2_gpu_check
#include "pd_common.h"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
using namespace pd;

__global__ void k_atan2(const double* y, const double* x, double* lib, double* fd, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { lib[i] = atan2(y[i], x[i]); fd[i] = atan2_fd(y[i], x[i]); }
}

static uint64_t st = 0x243F6A8885A308D3ull;
static uint64_t nx() {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01() { return (double)(nx() >> 11) * 0x1p-53; }
static int64_t ord(double v) { int64_t i; std::memcpy(&i, &v, 8); return i < 0 ? INT64_MIN - i : i; }

int main() {
    const int n = 1 << 22;
    std::vector<double> y(n), x(n), lib(n), fd(n);
    for (int i = 0; i < n; ++i) {
        if (i & 1) { x[i] = -300.0 + 350.0 * u01(); y[i] = -1100.0 + 1110.0 * u01(); }
        else { x[i] = std::exp((u01() - 0.5) * 20.0) * ((nx() & 1) ? -1.0 : 1.0);
               y[i] = std::exp((u01() - 0.5) * 20.0) * ((nx() & 1) ? -1.0 : 1.0); }
        if (x[i] == 0.0) x[i] = 1.0;
        if (y[i] == 0.0) y[i] = 1.0;
    }
    double *dy, *dx, *dl, *df;
    if (hipMalloc(&dy, n * 8) || hipMalloc(&dx, n * 8) || hipMalloc(&dl, n * 8) || hipMalloc(&df, n * 8)) return 2;
    hipMemcpy(dy, y.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_atan2, dim3(n / 256), dim3(256), 0, 0, dy, dx, dl, df, n);
    hipMemcpy(lib.data(), dl, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(fd.data(), df, n * 8, hipMemcpyDeviceToHost);
    long dlib[2] = {0, 0}, dfd[2] = {0, 0}, hostfd = 0, cnt[2] = {0, 0};
    int64_t wlib = 0, wfd = 0;
    for (int i = 0; i < n; ++i) {
        const double g = std::atan2(y[i], x[i]);
        const int k = i & 1;
        ++cnt[k];
        const int64_t a = std::llabs(ord(lib[i]) - ord(g)), b = std::llabs(ord(fd[i]) - ord(g));
        dlib[k] += a != 0; dfd[k] += b != 0;
        wlib = a > wlib ? a : wlib; wfd = b > wfd ? b : wfd;
        hostfd += ord(fd[i]) != ord(atan2_fd(y[i], x[i]));
    }
    std::printf("{\"n\": %d, \"ocml_differ_frac_quadrants\": %.6f, \"ocml_differ_frac_descent\": %.6f, "
                "\"ocml_worst_ulp\": %lld, \"fd_differ_frac_quadrants\": %.6f, \"fd_differ_frac_descent\": %.6f, "
                "\"fd_worst_ulp\": %lld, \"fd_device_vs_host_bits_differ\": %ld}\n",
                n, (double)dlib[0] / cnt[0], (double)dlib[1] / cnt[1], (long long)wlib, (double)dfd[0] / cnt[0],
                (double)dfd[1] / cnt[1], (long long)wfd, hostfd);
    return 0;
}
