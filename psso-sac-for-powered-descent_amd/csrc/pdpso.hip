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
// and the float32 copy written alongside is the [P_params][N] weight layout that
// pd_rollout_policy reads, or (pd_pso_step_chunked, k_pso_step4) the chunked layout
// [ceil(P_params/4)][N][4] that the step kernel's actor reads, so a rollout makes no copy pass.
// HBM-bound: 44 B per (particle, parameter).
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

// pd_pso_step_chunked: thread (chunk c, particle p) updates parameters 4c .. 4c+3 of particle p
// with k_pso_step's operations in its order (one Philox draw, reused for the four: r1, r2 are per
// particle), and stores their float32 copy as one 16-byte chunk of [ceil(D/4)][P][4], the layout
// the step kernel's actor reads (pd_step_impl.h actor_forward), zeros past D.
__global__ __launch_bounds__(kPsoBlock) void k_pso_step4(
    int64_t P, int D, const double* __restrict__ fit, const double* __restrict__ pbf, double* __restrict__ x,
    double* __restrict__ v, double* __restrict__ pb, const double* __restrict__ sb, const int32_t* __restrict__ swarm,
    const double* __restrict__ lo, const double* __restrict__ hi, double w, double c1, double c2, uint32_t seed_lo,
    uint32_t seed_hi, uint32_t gen, uint64_t p_offset, float4* __restrict__ x32c) {
    // (grid: the particle range fastest, as k_pso_step's.  Chunk-major and tiled orders keep the
    // range's fit / pbf / swarm words in L2 across its chunks, 0.4 GB fewer fetches at 262 144
    // particles, and measured 5-8 % slower: tools/pso_grid_ab.py, profiles/r06_exp_pso_chunked.jsonl)
    const int c = blockIdx.y;
    const int64_t p = (int64_t)blockIdx.x * kPsoBlock + threadIdx.x;
    if (p >= P) return;
    const bool better = fit[p] < pbf[p];
    const uint64_t g = p_offset + (uint64_t)p;
    u32x4 r = philox({(uint32_t)g, (uint32_t)(g >> 32), gen, kTagPso}, seed_lo, seed_hi);
    const double r1 = u01(r.x, r.y), r2 = u01(r.z, r.w);
    const double* sbp = sb + (int64_t)swarm[p] * D;
    // every load of the four parameters first (the update of one does not wait on the stores of
    // the one before), then the arithmetic in k_pso_step's order, then the stores
    double xv[4], vv[4], pbv[4], sv[4], lv[4], hv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int d = 4 * c + k < D ? 4 * c + k : D - 1;   // (past D: a valid address, result unused)
        const int64_t e = (int64_t)d * P + p;
        xv[k] = x[e]; vv[k] = v[e];
        pbv[k] = better ? 0.0 : pb[e];
        sv[k] = sbp[d]; lv[k] = lo[d]; hv[k] = hi[d];
    }
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int d = 4 * c + k;
        o[k] = 0.f;
        if (d < D) {
            const int64_t e = (int64_t)d * P + p;
            if (better) { pbv[k] = xv[k]; pb[e] = xv[k]; }
            const double inertia = w * vv[k];
            const double cognitive = c1 * r1 * (pbv[k] - xv[k]);
            const double social = c2 * r2 * (sv[k] - xv[k]);
            const double vn = inertia + cognitive + social;
            double xn = xv[k] + vn;
            if (xn < lv[k]) xn = lv[k];
            else if (xn > hv[k]) xn = hv[k];
            v[e] = vn;
            x[e] = xn;
            o[k] = (float)xn;
        }
    }
    x32c[(int64_t)c * P + p] = make_float4(o[0], o[1], o[2], o[3]);
}

__global__ __launch_bounds__(kPsoBlock) void k_pso_best(int64_t P, const double* __restrict__ fit,
                                                        double* __restrict__ pbf) {
    const int64_t p = (int64_t)blockIdx.x * kPsoBlock + threadIdx.x;
    if (p < P && fit[p] < pbf[p]) pbf[p] = fit[p];
}

// The reference's sequential rule (:437-441): `if fitness < subswarm_best`, particle by particle,
// so a NaN fitness never wins (every comparison with it is false) and on ties the first particle
// stays.  Here: a NaN loses to anything, else the smaller value, ties to the lower index.
__device__ __forceinline__ bool argmin_better(double a, int64_t ia, double b, int64_t ib) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return !na && nb;
    return a < b || (a == b && ia < ib);
}

// Block-wide argmin of (f, i) pairs (i < 0: none), LDS tree with the rule above; every thread
// gets the winner.
__device__ __forceinline__ void block_argmin(double& f, int64_t& i, double* sf, int64_t* si) {
    sf[threadIdx.x] = f; si[threadIdx.x] = i;
    __syncthreads();
    for (int o = kPsoBlock / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            const double f2 = sf[threadIdx.x + o];
            const int64_t i2 = si[threadIdx.x + o];
            if (i2 >= 0 && (si[threadIdx.x] < 0 || argmin_better(f2, i2, sf[threadIdx.x], si[threadIdx.x]))) {
                sf[threadIdx.x] = f2; si[threadIdx.x] = i2;
            }
        }
        __syncthreads();
    }
    f = sf[0]; i = si[0];
    __syncthreads();
}

// Segmented argmin in two passes (the subswarm minima of :437-441).  Pass 1: block b takes
// particles [b C, (b + 1) C) (C = kMinChunk, four per thread, coalesced) and writes, per subswarm
// s, its first particle of minimal non-NaN fitness (index -1: none) to part[b][s].
constexpr int kMinPer = 4;
constexpr int kMinChunk = kMinPer * kPsoBlock;
__global__ __launch_bounds__(kPsoBlock) void k_swarm_minima_part(int64_t P, int S, const double* __restrict__ fit,
                                                                 const int32_t* __restrict__ swarm,
                                                                 double* __restrict__ part_f,
                                                                 int64_t* __restrict__ part_i) {
    __shared__ double sf[kPsoBlock];
    __shared__ int64_t si[kPsoBlock];
    const int64_t base = (int64_t)blockIdx.x * kMinChunk + threadIdx.x;
    double f[kMinPer];
    int32_t sw[kMinPer];
#pragma unroll
    for (int k = 0; k < kMinPer; ++k) {
        const int64_t p = base + (int64_t)k * kPsoBlock;
        sw[k] = p < P ? swarm[p] : -1;
        f[k] = p < P ? fit[p] : 0.0;
    }
    for (int s = 0; s < S; ++s) {
        double bf = 0.0;
        int64_t bi = -1;
#pragma unroll
        for (int k = 0; k < kMinPer; ++k)   // (increasing index: strictly better replaces)
            if (sw[k] == s && f[k] == f[k] && (bi < 0 || f[k] < bf)) { bf = f[k]; bi = base + (int64_t)k * kPsoBlock; }
        block_argmin(bf, bi, sf, si);
        if (threadIdx.x == 0) { part_f[(int64_t)blockIdx.x * S + s] = bf; part_i[(int64_t)blockIdx.x * S + s] = bi; }
    }
}

// Pass 2, one workgroup per subswarm s: the winner over the G pass-1 blocks (lower block = lower
// index, so the rule above keeps the first particle), its fitness and position; +inf and a zero
// position when no particle of s has a non-NaN fitness (the reference then keeps its best).
__global__ __launch_bounds__(kPsoBlock) void k_swarm_minima_final(int64_t P, int D, int S, int64_t G,
                                                                  const double* __restrict__ part_f,
                                                                  const int64_t* __restrict__ part_i,
                                                                  const double* __restrict__ x, double* __restrict__ min_f,
                                                                  double* __restrict__ min_pos) {
    __shared__ double sf[kPsoBlock];
    __shared__ int64_t si[kPsoBlock];
    const int s = blockIdx.x;
    double bf = 0.0;
    int64_t bi = -1;
    for (int64_t b = threadIdx.x; b < G; b += kPsoBlock) {
        const int64_t i2 = part_i[b * S + s];
        const double f2 = part_f[b * S + s];
        if (i2 >= 0 && (bi < 0 || argmin_better(f2, i2, bf, bi))) { bf = f2; bi = i2; }
    }
    block_argmin(bf, bi, sf, si);
    if (threadIdx.x == 0) min_f[s] = bi >= 0 ? bf : __builtin_inf();
    for (int d = threadIdx.x; d < D; d += kPsoBlock) min_pos[(int64_t)s * D + d] = bi >= 0 ? x[(int64_t)d * P + bi] : 0.0;
}

// :442-444 and :474-477 (one workgroup): subswarm s takes a strictly better minimum; then the
// first subswarm holding the smallest best replaces the global best if strictly better.
__global__ __launch_bounds__(kPsoBlock) void k_update_bests(int S, int D, const double* __restrict__ min_f,
                                                            const double* __restrict__ min_pos, double* __restrict__ sbf,
                                                            double* __restrict__ sb, double* __restrict__ gbf,
                                                            double* __restrict__ gb) {
    for (int s = 0; s < S; ++s) {
        const bool better = min_f[s] < sbf[s];
        if (better)
            for (int d = threadIdx.x; d < D; d += kPsoBlock) sb[(int64_t)s * D + d] = min_pos[(int64_t)s * D + d];
        __syncthreads();
        if (better && threadIdx.x == 0) sbf[s] = min_f[s];
        __syncthreads();
    }
    int j = 0;
    for (int s = 1; s < S; ++s) if (sbf[s] < sbf[j]) j = s;
    if (sbf[j] < *gbf) {
        for (int d = threadIdx.x; d < D; d += kPsoBlock) gb[d] = sb[(int64_t)j * D + d];
        __syncthreads();
        if (threadIdx.x == 0) *gbf = sbf[j];
    }
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

pd_status pd_pso_step_chunked(int64_t n_particles, int32_t dim, const double* fitness, double* best_fitness,
                              double* position, double* velocity, double* best_position, const double* swarm_best,
                              const int32_t* swarm, const double* lower, const double* upper, double w, double c1,
                              double c2, uint64_t seed, uint32_t generation, uint64_t particle_offset,
                              float* position_f32_chunked, void* stream) {
    if (n_particles <= 0 || dim <= 0 || dim > 65535 || !fitness || !best_fitness || !position || !velocity ||
        !best_position || !swarm_best || !swarm || !lower || !upper || !position_f32_chunked ||
        (uintptr_t)position_f32_chunked % 16 != 0)
        return set_error(PD_ERR_INVALID, "pd_pso_step_chunked: bad arguments (the chunked copy is required, 16-byte aligned)");
    hipStream_t s = (hipStream_t)stream;
    dim3 grid((unsigned)((n_particles + kPsoBlock - 1) / kPsoBlock), (unsigned)((dim + 3) / 4));
    hipLaunchKernelGGL(k_pso_step4, grid, dim3(kPsoBlock), 0, s, n_particles, dim, fitness, best_fitness, position,
                       velocity, best_position, swarm_best, swarm, lower, upper, w, c1, c2, (uint32_t)seed,
                       (uint32_t)(seed >> 32), generation, particle_offset, (float4*)position_f32_chunked);
    hipLaunchKernelGGL(k_pso_best, dim3((unsigned)((n_particles + kPsoBlock - 1) / kPsoBlock)), dim3(kPsoBlock), 0, s,
                       n_particles, fitness, best_fitness);
    if (hipGetLastError() != hipSuccess) return set_error(PD_ERR_HIP, "pd_pso_step_chunked: launch failed");
    return PD_OK;
}

size_t pd_pso_swarm_minima_scratch_bytes(int64_t n_particles, int32_t n_swarms) {
    const int64_t G = n_particles > 0 ? (n_particles + kMinChunk - 1) / kMinChunk : 1;
    return (size_t)G * (size_t)(n_swarms > 0 ? n_swarms : 1) * (sizeof(double) + sizeof(int64_t));
}

pd_status pd_pso_swarm_minima(int64_t n_particles, int32_t dim, int32_t n_swarms, const double* fitness,
                              const int32_t* swarm, const double* position, double* min_fitness, double* min_position,
                              void* scratch, size_t scratch_bytes, void* stream) {
    if (n_particles < 0 || dim <= 0 || n_swarms <= 0 || n_swarms > 65535 || !min_fitness || !min_position ||
        (n_particles > 0 && (!fitness || !swarm || !position)))
        return set_error(PD_ERR_INVALID, "pd_pso_swarm_minima: bad arguments");
    // pass-1 partials in the caller's scratch: [G][n_swarms] doubles, then [G][n_swarms] indices
    const int64_t G = (n_particles + kMinChunk - 1) / kMinChunk;
    const size_t need = pd_pso_swarm_minima_scratch_bytes(n_particles, n_swarms);
    if (!scratch || scratch_bytes < need || (uintptr_t)scratch % 8 != 0)
        return set_error(PD_ERR_INVALID, "pd_pso_swarm_minima: scratch missing, too small or misaligned");
    double* part_f = (double*)scratch;
    int64_t* part_i = (int64_t*)((char*)scratch + (size_t)(G > 0 ? G : 1) * (size_t)n_swarms * sizeof(double));
    hipStream_t s = (hipStream_t)stream;
    if (G > 0)
        hipLaunchKernelGGL(k_swarm_minima_part, dim3((unsigned)G), dim3(kPsoBlock), 0, s, n_particles, n_swarms,
                           fitness, swarm, part_f, part_i);
    hipLaunchKernelGGL(k_swarm_minima_final, dim3((unsigned)n_swarms), dim3(kPsoBlock), 0, s, n_particles, dim,
                       n_swarms, G, part_f, part_i, position, min_fitness, min_position);
    if (hipGetLastError() != hipSuccess) return set_error(PD_ERR_HIP, "pd_pso_swarm_minima: launch failed");
    return PD_OK;
}

pd_status pd_pso_update_bests(int32_t n_swarms, int32_t dim, const double* min_fitness, const double* min_position,
                              double* swarm_best_fitness, double* swarm_best, double* global_best_fitness,
                              double* global_best, void* stream) {
    if (n_swarms <= 0 || dim <= 0 || !min_fitness || !min_position || !swarm_best_fitness || !swarm_best ||
        !global_best_fitness || !global_best)
        return set_error(PD_ERR_INVALID, "pd_pso_update_bests: bad arguments");
    hipLaunchKernelGGL(k_update_bests, dim3(1), dim3(kPsoBlock), 0, (hipStream_t)stream, n_swarms, dim, min_fitness,
                       min_position, swarm_best_fitness, swarm_best, global_best_fitness, global_best);
    if (hipGetLastError() != hipSuccess) return set_error(PD_ERR_HIP, "pd_pso_update_bests: launch failed");
    return PD_OK;
}

}  // extern "C"
