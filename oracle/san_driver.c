/* Host sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).  Built with
 * -fsanitize=address,undefined by `make -C oracle sanitize`; reads an orc_params image written
 * by tests/test_oracle_golden.py::test_oracle_under_asan_ubsan and exercises the restatement:
 * KAT grids of the atmosphere and the aero tables, Philox/Box-Muller draws, episodes of both
 * landing phases with wind, tilt and auto-reset, and a multi-threaded rollout. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "pd_oracle.h"

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: san_driver params.bin\n"); return 2; }
    orc_params* P = (orc_params*)calloc(1, sizeof(orc_params));
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(P, sizeof(orc_params), 1, f) != 1) { fprintf(stderr, "bad params image\n"); return 2; }
    fclose(f);
    double acc = 0.0;
    for (int k = 0; k <= 400; ++k) {
        double rho, p, a;
        orc_atmosphere(P, -500.0 + 250.0 * k, &rho, &p, &a);
        acc += rho + p * 1e-5 + a * 1e-3 + orc_gravity(P, 250.0 * k);
    }
    for (int i = 0; i <= 40; ++i)
        for (int j = -12; j <= 12; ++j) {
            double M = 0.25 * i, al = j * 0.0004;
            acc += orc_CD(P, M, al) + orc_CL(P, M, al) + orc_Ca(P, M) + orc_Cn(P, M, al);
            acc += orc_rbf(P, 0, M, j * 2.5) + orc_rbf(P, 1, M, j * 2.5);
        }
    for (uint32_t c = 0; c < 256; ++c) {
        orc_u32x4 ctr = {c, c ^ 7u, c * 3u, 16u};
        double z0, z1;
        orc_gauss_pair(orc_philox(ctr, 5u, 0u), &z0, &z1);
        acc += z0 + z1;
    }
    const int n = 16, T = 120;
    float* A = (float*)malloc(sizeof(float) * (size_t)T * n * 4);
    for (int i = 0; i < T * n * 4; ++i) A[i] = (float)(((i * 2654435761u) % 2001u) / 1000.0 - 1.0);
    double* rew = (double*)calloc((size_t)T * n, sizeof(double));
    unsigned char* dn = (unsigned char*)calloc((size_t)T * n, 1);
    unsigned char* tr = (unsigned char*)calloc((size_t)T * n, 1);
    signed char* tid = (signed char*)calloc((size_t)T * n, 1);
    double* obs = (double*)calloc((size_t)T * n * 8, sizeof(double));
    double* sf = (double*)calloc((size_t)n * 11, sizeof(double));
    uint64_t* g = (uint64_t*)malloc(sizeof(uint64_t) * n);
    uint32_t* ep = (uint32_t*)calloc(n, sizeof(uint32_t));
    for (int i = 0; i < n; ++i) g[i] = (uint64_t)i * 977u;
    int64_t steps = 0;
    for (int phase = ORC_PHASE_PURE_THROTTLE; phase <= ORC_PHASE_SUPERSONIC; ++phase)
        for (int rtd = ORC_RTD_RL; rtd <= ORC_RTD_NONE; ++rtd)
            acc += orc_rollout_philox(P, phase, rtd, n, g, ep, T, A, 1, 1, 1, rtd == ORC_RTD_PSO ? 38 : -1, 0.01745, 7,
                                      rew, dn, tr, (int8_t*)tid, obs, 8, sf, 4, &steps);
    acc += orc_rollout_mt(P, ORC_PHASE_PURE_THROTTLE, ORC_RTD_RL, n, 100, A, 1, 1, 0.01745, 3, 3, &steps);
    for (int phase = ORC_PHASE_PURE_THROTTLE; phase <= ORC_PHASE_LANDING_BURN; ++phase) {
        const int np_ = orc_actor_params(phase), m = 6;
        float* w = (float*)malloc(sizeof(float) * (size_t)np_ * m);
        for (int i = 0; i < np_ * m; ++i) w[i] = (float)((((unsigned)i * 40503u) % 1001u) / 1000.0 - 0.5);
        double fit[6];
        int32_t len[6];
        orc_rollout_policy(P, phase, m, w, 200, fit, len);
        for (int i = 0; i < m; ++i) acc += fit[i] * 1e-6 + len[i];
        free(w);
    }
    printf("ok %.6e %lld\n", acc, (long long)steps);
    free(A); free(rew); free(dn); free(tr); free(tid); free(obs); free(sf); free(g); free(ep); free(P);
    return isfinite(acc) ? 0 : 1;
}
