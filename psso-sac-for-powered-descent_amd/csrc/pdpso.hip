// pdpso.hip -- device-side particle-swarm update of the PSO driver.
//
// One generation's particle update of ParticleSubswarmOptimisation.run
// (src/particle_swarm_optimisation/particle_swarm_optimisation.py):
//   personal best            if fitness < best_fitness: best_position = position      (:437-441)
//   update_velocity_with_local_best                                                   (:515-519)
//     v = w v + c1 r1 (best_position - x) + c2 r2 (subswarm_best - x)
//     with ONE uniform r1 and ONE r2 per particle and call (np.random.rand(), not per dimension)
//   update_position          x += v, clipped to the bounds                            (:112-118)
// Everything is binary64 as NumPy computes it, operation by operation (left-to-right
// products, (inertia + cognitive) + social), so a NumPy restatement with the same r1, r2 is
// bit-identical.  Layout is parameter-major [D][P] (lane = particle): every access coalesces,
// and the float32 copy written alongside is exactly the [P_params][N] weight layout that
// pd_rollout_policy reads.  HBM-bound: 52 B per (particle, parameter).
#include <hip/hip_runtime.h>

#include "../../include/pdenv.h"
#include "pd_common.h"

namespace {

using namespace pd;

constexpr uint32_t kTagPso = 32;
constexpr int kPsoBlock = 256;

__global__ __launch_bounds__(kPsoBlock) void k_pso_step(
    int64_t P, int D, const double* __restrict__ fit, const double* __restrict__ pbf, double* __restrict__ x,
    double* __restrict__ v, double* __restrict__ pb, const double* __restrict__ sb, const int32_t* __restrict__ swarm,
    const double* __restrict__ lo, const double* __restrict__ hi, double w, double c1, double c2, uint32_t seed_lo,
    uint32_t seed_hi, uint32_t gen, uint64_t p_offset, float* __restrict__ x32) {
    const int d = blockIdx.y;
    const int64_t p = (int64_t)blockIdx.x * kPsoBlock + threadIdx.x;
    if (p >= P) return;
    const int64_t e = (int64_t)d * P + p;
    const double xv = x[e];
    double pbv;
    if (fit[p] < pbf[p]) { pbv = xv; pb[e] = xv; }
    else pbv = pb[e];
    const uint64_t g = p_offset + (uint64_t)p;
    u32x4 r = philox({(uint32_t)g, (uint32_t)(g >> 32), gen, kTagPso}, seed_lo, seed_hi);
    const double r1 = u01(r.x, r.y), r2 = u01(r.z, r.w);
    const double inertia = w * v[e];
    const double cognitive = c1 * r1 * (pbv - xv);
    const double social = c2 * r2 * (sb[(int64_t)swarm[p] * D + d] - xv);
    const double vn = inertia + cognitive + social;
    double xn = xv + vn;
    if (xn < lo[d]) xn = lo[d];
    else if (xn > hi[d]) xn = hi[d];
    v[e] = vn;
    x[e] = xn;
    if (x32) x32[e] = (float)xn;
}

__global__ __launch_bounds__(kPsoBlock) void k_pso_best(int64_t P, const double* __restrict__ fit,
                                                        double* __restrict__ pbf) {
    const int64_t p = (int64_t)blockIdx.x * kPsoBlock + threadIdx.x;
    if (p < P && fit[p] < pbf[p]) pbf[p] = fit[p];
}

}  // namespace

namespace pd {
pd_status set_error(pd_status s, const char* m);   // pdenv.hip: the pd_last_error() message
}

extern "C" {

pd_status pd_pso_step(int64_t n_particles, int32_t dim, const double* fitness, double* best_fitness, double* position,
                      double* velocity, double* best_position, const double* swarm_best, const int32_t* swarm,
                      const double* lower, const double* upper, double w, double c1, double c2, uint64_t seed,
                      uint32_t generation, uint64_t particle_offset, float* position_f32, void* stream) {
    if (n_particles <= 0 || dim <= 0 || dim > 65535 || !fitness || !best_fitness || !position || !velocity ||
        !best_position || !swarm_best || !swarm || !lower || !upper)
        return set_error(PD_ERR_INVALID, "pd_pso_step: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    dim3 grid((unsigned)((n_particles + kPsoBlock - 1) / kPsoBlock), (unsigned)dim);
    hipLaunchKernelGGL(k_pso_step, grid, dim3(kPsoBlock), 0, s, n_particles, dim, fitness, best_fitness, position,
                       velocity, best_position, swarm_best, swarm, lower, upper, w, c1, c2, (uint32_t)seed,
                       (uint32_t)(seed >> 32), generation, particle_offset, position_f32);
    hipLaunchKernelGGL(k_pso_best, dim3((unsigned)((n_particles + kPsoBlock - 1) / kPsoBlock)), dim3(kPsoBlock), 0, s,
                       n_particles, fitness, best_fitness);
    if (hipGetLastError() != hipSuccess) return set_error(PD_ERR_HIP, "pd_pso_step: launch failed");
    return PD_OK;
}

}  // extern "C"
