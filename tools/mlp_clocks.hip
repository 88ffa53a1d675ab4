// mlp_clocks.hip -- section clocks of the SAC actor tile (csrc/pd_sac_mlp.h sac_mlp_tile) at
// c5's size: 4 096 envs, the reference Actor 2-256-256-1 (256 workgroups of 16 envs, one per
// CU).  Every wave's lane 0 stamps clock64() at the tile's start and at each phase's end (layer
// 1, the hidden layer, the heads); the program prints the medians over the waves of each phase's
// cycles and the event-timed kernel duration (median of 200 launches), and the heads' largest relative
// difference from a host binary64 forward pass (a variant that computes wrong values shows).
// Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mlp_clocks.hip -o mlp_clocks && ./mlp_clocks
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <random>
#include <vector>

// (-DMLP_H='"file"': another version of the tile, with the same mark hook, for a comparison)
#ifdef MLP_H
#include MLP_H
#else
#include "../psso-sac-for-powered-descent_amd/csrc/pd_sac_mlp.h"
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kPh = 4;   // start, layer 1, hidden layer, heads

template <int H>
__global__ __launch_bounds__(pd::kSacBlock) void k_clk(pd::SacMlp a, int64_t n, float* heads, long long* clk) {
    __shared__ __attribute__((aligned(16))) float hb[pd::sac_mlp_lds_floats<H>()];
    const int64_t e0 = (int64_t)blockIdx.x * pd::kSacTile;
#ifdef MLP_TWICE
    // (a first, unstamped pass: the stamped one then runs with warm instruction and data caches)
    pd::sac_mlp_tile<H>(a, n, e0, hb, [&](int e, int o, float v) {
        if (e0 + e < n) heads[(e0 + e) * 2 * a.A + o] = v;
    });
    __syncthreads();
#endif
    long long t0 = clock64(), t1 = 0, t2 = 0, t3 = 0;
    pd::sac_mlp_tile<H>(
        a, n, e0, hb,
        [&](int e, int o, float v) {
            const int64_t ge = e0 + e;
            if (ge < n) heads[ge * 2 * a.A + o] = v;
        },
        [&](int k) {
            const long long c = clock64();
            if (k == 0) t1 = c;
            else if (k == 1) t2 = c;
            else t3 = c;
        });
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (pd::kSacBlock / 64) + (threadIdx.x >> 6);
        clk[(size_t)w * kPh] = t0; clk[(size_t)w * kPh + 1] = t1;
        clk[(size_t)w * kPh + 2] = t2; clk[(size_t)w * kPh + 3] = t3;
    }
}

int main(int argc, char** argv) {
    constexpr int S = 2, H = 256, L = 2, A = 1;
    const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;   // (fewer envs: fewer workgroups per XCD)
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> u(-0.1f, 0.1f);
    std::vector<std::vector<float>> host;   // (every parameter, for the host reference below)
    auto dev = [&](size_t cnt) {
        std::vector<float> h(cnt);
        for (auto& x : h) x = u(rng);
        host.push_back(h);
        float* d = nullptr;
        if (hipMalloc(&d, cnt * 4) != hipSuccess) return (float*)nullptr;
        if (hipMemcpy(d, h.data(), cnt * 4, hipMemcpyHostToDevice) != hipSuccess) return (float*)nullptr;
        return d;
    };
    pd::SacMlp a{};
    a.S = S; a.L = L; a.A = A; a.H = H;
    a.obs = dev((size_t)n * S);
    a.w[0] = dev((size_t)H * S); a.b[0] = dev(H);
    a.w[1] = dev((size_t)H * H); a.b[1] = dev(H);
    a.wm = dev((size_t)A * H); a.bm = dev(A); a.ws = dev((size_t)A * H); a.bs = dev(A);
    float* heads = nullptr;
    long long* clk = nullptr;
    const unsigned grid = (unsigned)(n / pd::kSacTile);
    const int waves = (int)grid * (pd::kSacBlock / 64);
    CK(hipMalloc(&heads, (size_t)n * 2 * A * 4));
    CK(hipMalloc(&clk, (size_t)waves * kPh * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int r = 0; r < 220; ++r) {
        CK(hipEventRecord(e0, nullptr));
        hipLaunchKernelGGL(k_clk<H>, dim3(grid), dim3(pd::kSacBlock), 0, nullptr, a, n, heads, clk);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float t = 0.f;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (r >= 20) ms.push_back(t);
    }
    // the heads against a host binary64 forward pass of the same parameters (order: obs, w0, b0,
    // w1, b1, wm, bm, ws, bs)
    std::vector<float> hd((size_t)n * 2 * A);
    CK(hipMemcpy(hd.data(), heads, hd.size() * 4, hipMemcpyDeviceToHost));
    double max_err = 0.0;
    {
        const auto &ob = host[0], &w0 = host[1], &b0 = host[2], &w1 = host[3], &b1 = host[4];
        const auto &wm = host[5], &bm = host[6], &ws = host[7], &bs = host[8];
        std::vector<double> x1(H), x2(H);
        for (int64_t e = 0; e < n; ++e) {
            for (int j = 0; j < H; ++j) {
                double t = b0[j];
                for (int k = 0; k < S; ++k) t += (double)ob[e * S + k] * w0[j * S + k];
                x1[j] = t > 0 ? t : 0;
            }
            for (int j = 0; j < H; ++j) {
                double t = b1[j];
                for (int k = 0; k < H; ++k) t += x1[k] * w1[(size_t)j * H + k];
                x2[j] = t > 0 ? t : 0;
            }
            for (int o = 0; o < 2 * A; ++o) {
                const auto& w = o < A ? wm : ws;
                double t = o < A ? bm[o] : bs[o - A];
                for (int k = 0; k < H; ++k) t += x2[k] * w[(size_t)(o % A) * H + k];
                const double d = hd[e * 2 * A + o];
                max_err = std::max(max_err, std::fabs(d - t) / (std::fabs(t) + 1e-3));
            }
        }
    }
    std::vector<long long> c((size_t)waves * kPh);
    CK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
    std::sort(ms.begin(), ms.end());
    printf("{\"envs\": %lld, \"hidden\": %d, \"kernel_us_med\": %.2f, \"kernel_us_min\": %.2f", (long long)n, H,
           1e3 * ms[ms.size() / 2], 1e3 * ms[0]);
    const char* name[kPh - 1] = {"layer1", "hidden", "heads"};
    for (int k = 1; k < kPh; ++k) {
        std::vector<long long> d(waves);
        for (int w = 0; w < waves; ++w) d[w] = c[(size_t)w * kPh + k] - c[(size_t)w * kPh + k - 1];
        std::sort(d.begin(), d.end());
        printf(", \"%s_cycles\": {\"p10\": %lld, \"med\": %lld, \"p90\": %lld}", name[k - 1], d[waves / 10], d[waves / 2],
               d[waves * 9 / 10]);
    }
    std::vector<long long> tot(waves);
    for (int w = 0; w < waves; ++w) tot[w] = c[(size_t)w * kPh + kPh - 1] - c[(size_t)w * kPh];
    std::sort(tot.begin(), tot.end());
    printf(", \"tile_cycles_med\": %lld, \"tile_cycles_max\": %lld, \"heads_max_rel_err\": %.3g}\n", tot[waves / 2],
           tot[waves - 1], max_err);
    return 0;
}
