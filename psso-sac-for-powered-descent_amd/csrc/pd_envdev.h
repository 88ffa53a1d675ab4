// pd_envdev.h -- device helpers shared by the step kernel and the small per-env kernels:
// global-address-space per-env accessors, the constant-address-space parameter view, and the
// reset of one env (base_environment.py:80-97) computed into registers.
#pragma once
#include "pd_step.h"

namespace pd {

// Per-env element `i` of a wave-uniform base pointer, addressed as base + zero-extended 32-bit
// byte offset in the global address space: the base stays in SGPRs (global_load ... saddr) and
// the offset is one VGPR per lane.
template <typename T> __device__ __forceinline__ PD_AS1 T& ev(T* base, uint32_t i) {
    using B = typename std::conditional<std::is_const<T>::value, const PD_AS1 char, PD_AS1 char>::type;
    return *(PD_AS1 T*)((B*)(uint64_t)base + (uint32_t)(i * (uint32_t)sizeof(T)));
}
template <typename T> __device__ __forceinline__ T ldv(const T* base, uint32_t i) { return ev(base, i); }

// The Philox key (the handle's seed) through an opaque copy at each draw: otherwise the compiler
// precomputes the 10-round key schedule once (20 uniform values) and holds it in scalar
// registers for the whole launch -- spilled into VGPR lanes.  Recomputing it is 20 SALU adds.
__device__ __forceinline__ u32x4 philox_k(u32x4 ctr, uint32_t k0, uint32_t k1) {
    asm volatile("" : "+s"(k0), "+s"(k1));
    return philox(ctr, k0, k1);
}

// The handle's parameter block through a constant-address-space pointer laundered into SGPRs:
// uniform fields are scalar loads, and a fresh laundered copy per sub-step keeps the compiler
// from holding ~150 parameters live across the loop (they are re-read from the scalar cache).
template <typename R> __device__ __forceinline__ DP<R>* params(uint64_t p) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (DP<R>*)(((uint64_t)hi << 32) | lo);
}

// The step kernel's arguments through a laundered pointer into its kernarg segment (the by-value
// StepArgs is the kernel's only explicit argument: offset 0).  A scope that launders it anew loads
// the fields it uses there (scalar loads) instead of the compiler loading every field in the
// prologue and holding them across the loops (spilled into VGPR lanes)
template <typename R> using SA = const PD_AS4 StepArgs<R>;
template <typename R> __device__ __forceinline__ SA<R>& kargs() {
    const uint64_t p = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
    asm volatile("" : "+s"(lo), "+s"(hi));
    return *(SA<R>*)(((uint64_t)hi << 32) | lo);
}

// The per-env state a launch keeps in registers (the g-load ring lives in LDS meanwhile).
template <typename R> struct EnvRegs {
    R s[11];
    R vprev;
    int glen, ghead;
    R act0, act1, act2;            // landing_burn gimbal deg + fin commands; flip-over gimbal
    R fu0, fu1, fv0, fv1, sgu, sgv;
    int prof;
    uint32_t ep, ts;
    int tid;
};

// base_environment.py:80-97 (reset) with the build's perturbations, for env g in episode
// `episode`: the initial state (load_initial_states.py:56-62) + pitch tilt N(0, tilt_sigma)
// (Philox tag kTagTilt, alpha = theta - gamma); actuator memory, g-load window and wind filters
// zeroed; sigma_u, sigma_v ~ U (VKDisturbanceGenerator._new_filters, vonkarman.py:60-66) from
// Philox tag kTagReset, and the percentile randint(50, 99) (WindModel.compile_horizontal_fixed_wind,
// full_wind_model.py:27-33) from its own draw, tag kTagProf (the reference draws the three from
// independent np.random calls).  invc/logc: the log_tab cells (element
// stride S: 2 for the step kernel's interleaved LDS copy).
template <typename R, int S = 1, typename AT>
__device__ __forceinline__ void reset_values(DP<R>& P, const AT& a, uint64_t g, uint32_t episode,
                                             const double* invc, const double* logc, EnvRegs<R>& e) {
#pragma unroll
    for (int k = 0; k < 11; ++k) e.s[k] = P.state0[k];
    if (a.use_tilt) {
        u32x4 r = philox_k({(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, kTagTilt}, a.seed_lo, a.seed_hi);
        double z0, z1;
        gauss_pair<S>(r, invc, logc, z0, z1);
        e.s[4] = e.s[4] + (R)(a.tilt_sigma * z0);
        e.s[7] = e.s[4] - e.s[6];
    }
    e.vprev = sqrt(e.s[2] * e.s[2] + e.s[3] * e.s[3]);
    e.glen = 0; e.ghead = 0;
    e.act0 = R(0); e.act1 = R(0); e.act2 = R(0);
    e.tid = 0;
    e.ep = episode; e.ts = 0;
    // the sigmas' draw and the percentile's draw: one Philox instance for both (register pressure)
    double su = 0.0, sv = 0.0;
    uint32_t pw = 0u;
#pragma unroll 1
    for (int t = 0; t < 2; ++t) {
        const u32x4 r = philox_k({(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, t ? kTagProf : kTagReset}, a.seed_lo, a.seed_hi);
        if (t == 0) {
            su = P.sigma_u_lo + (P.sigma_u_hi - P.sigma_u_lo) * u01(r.x, r.y);
            sv = P.sigma_v_lo + (P.sigma_v_hi - P.sigma_v_lo) * u01(r.z, r.w);
        } else {
            pw = r.x;
        }
    }
    e.fu0 = R(0); e.fu1 = R(0); e.fv0 = R(0); e.fv1 = R(0);
    e.sgu = (R)su; e.sgv = (R)sv;
    e.prof = a.fixed_prof >= 0 ? a.fixed_prof : prof_draw(pw);
}

}  // namespace pd
