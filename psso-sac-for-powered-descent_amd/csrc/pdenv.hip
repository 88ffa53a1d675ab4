// pdenv.hip -- MI355X (gfx950) kernels and C ABI of the vectorised powered-descent env.
//
// Layout in HBM: struct-of-arrays, one lane per env.  A step launch reads each env's state
// (11 words), its g-load window and caches, runs the 4 physics sub-steps of
// rocket_environment_pre_wrap.step in registers, and writes state + outputs once.
// Parameter tables are staged into LDS per workgroup; scalar parameters are uniform loads
// from a per-handle parameter block.  See DESIGN.md for the roofline of each kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pdenv.h"
#include "pd_physics.h"

using namespace pd;

namespace pd {
// the thread-local message behind pd_last_error(), shared by every source of the library
thread_local std::string g_err;
pd_status set_error(pd_status s, const char* m) { g_err = m; return s; }
}  // namespace pd

namespace {

pd_status fail(pd_status s, const std::string& m) { g_err = m; return s; }

#define PD_HIP(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(PD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kBlock = 256;
// k_step workgroup: its LDS tables (~63 KB) are shared by all its waves, so the size sets how
// many waves per SIMD the LDS admits (two workgroups per CU)
#ifndef PD_STEP_BLOCK
#define PD_STEP_BLOCK 256
#endif
constexpr int kStepBlock = PD_STEP_BLOCK;
constexpr int kScratch = kSys * kSys + kSys + 3 * kNbr + kPay;   // doubles per wave
constexpr int kPendingCap = 1024;
constexpr int kGridExact = 1 << 30;   // grid_slot flag: every point of the cell has its key

// ---------------------------------------------------------------- per-env device buffers
template <typename R> struct EnvBufs {
    R* st;            // [11][N]
    R* vprev;         // [N]   |v| of the previous state (base_environment.py:137-139)
    R* gwin;          // [10][N] g-load ring
    uint8_t* ghead;   // [N]
    uint8_t* glen;    // [N]
    R* act;           // [3][N] landing_burn actuator memory
    R* wind;          // [6][N] fu0 fu1 fv0 fv1 sigma_u sigma_v
    uint8_t* wprof;   // [N] wind profile (percentile-50)
    unsigned long long* key;   // [2][N] cached neighbourhood keys (cd, cl)
    int* slot;                 // [2][N] cached table slots
    int8_t* tid;      // [N] truncation id
    uint32_t* epi;    // [N] episode counter
    uint32_t* tstep;  // [N] step within episode
    uint8_t* fin;     // [N] episode finished (policy rollouts: the env is frozen until reset)
};

struct Pending {
    unsigned long long* count;   // [1] entries appended this launch
    unsigned long long* keys;    // [cap] (table id in bit 63)
    double* pay;                 // [cap][kPay]
    unsigned long long* stats;   // [4] misses, nan events, inserted cd, inserted cl
};

template <typename R> struct StepArgs {
    const DevParams<R>* P;
    EnvBufs<R> b;
    Pending pend;
    int64_t n;
    uint64_t env_offset;
    uint32_t seed_lo, seed_hi;
    int act_f64, auto_reset, stochastic, fixed_prof, use_tilt;
    double tilt_sigma;
    const void* actions;
    R* obs; R* reward; uint8_t* done; uint8_t* trunc; int8_t* trunc_id;
    const double* noise;
    R* info;
    R* reward_sum;
    const float* policy_w;           // policy rollouts: actor parameters [P][N] float32
    // policy rollouts: the live envs as a compacted index list; a launch steps list_in[0, *cnt_in)
    // and appends the envs whose episode goes on to list_out (wave ballot + prefix count, one
    // atomic per wave), then the next launch steps those only (triple-buffered counts: this
    // launch also zeroes the count the launch after next appends to)
    const int32_t* list_in; int32_t* list_out;
    const uint32_t* cnt_in; uint32_t* cnt_out; uint32_t* cnt_zero;
    int use_list;   // step list_in (else all N envs, finished ones skipped by their fin flag)
    double dt_aux;                   // physics dt of phases 2..6 (compile_physics(dt, phase))
    int rtd_none;                    // PD_RTD_NONE: physics stepping only (reward/done/trunc 0)
    int n_fused;                     // env-steps per launch (actions/outputs: [n_fused][N] rows)
};

// Per-env element `i` of a wave-uniform base pointer, addressed as base + zero-extended 32-bit
// byte offset: the compiler keeps the bases in SGPRs (global_load ... saddr) instead of one
// 64-bit VGPR address per SoA field.
template <typename T> __device__ __forceinline__ T& ev(T* base, uint32_t i) {
    using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
    return *(T*)((B*)base + (uint32_t)(i * (uint32_t)sizeof(T)));
}

// Streamed per-env fields of the step kernel: read once and written once per launch, so with
// PD_NT they bypass the caches' retention (nontemporal) and leave L2 to the aero tables.
template <typename T> __device__ __forceinline__ T ldv(const T* base, uint32_t i) {
#ifdef PD_NT
    return __builtin_nontemporal_load(&ev(base, i));
#else
    return ev(base, i);
#endif
}
template <typename T> struct StRef {
    T* p;
    __device__ __forceinline__ void operator=(T v) const {
#ifdef PD_NT
        __builtin_nontemporal_store(v, p);
#else
        *p = v;
#endif
    }
};
template <typename T> __device__ __forceinline__ StRef<T> stv(T* base, uint32_t i) { return {&ev(base, i)}; }

// ---------------------------------------------------------------- reset of one env
template <typename R>
__device__ void reset_env(const StepArgs<R>& a, int64_t i, uint32_t episode, bool reset_cache) {
    const DevParams<R>& P = *a.P;
    const int64_t N = a.n;
    uint32_t ui = (uint32_t)i;
    asm volatile("" : "+v"(ui));   // addresses recomputed here, not kept live by the caller
    R s[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) s[k] = P.state0[k];
    uint64_t g = a.env_offset + (uint64_t)i;
    if (a.use_tilt) {
        u32x4 r = philox({(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, kTagTilt}, a.seed_lo, a.seed_hi);
        double u1 = 1.0 - u01(r.x, r.y), u2 = u01(r.z, r.w);
        double z = sqrt(-2.0 * log(u1)) * cos(2.0 * kPi * u2);
        s[4] = s[4] + (R)(a.tilt_sigma * z);
        s[7] = s[4] - s[6];
    }
#pragma unroll
    for (int k = 0; k < 11; ++k) ev(a.b.st + (k) * N, ui) = s[k];
    ev(a.b.vprev, ui) = sqrt(s[2] * s[2] + s[3] * s[3]);
    ev(a.b.ghead, ui) = 0; ev(a.b.glen, ui) = 0;
    ev(a.b.act, ui) = R(0); ev(a.b.act + N, ui) = R(0); ev(a.b.act + (2) * N, ui) = R(0);
    ev(a.b.tid, ui) = 0;
    ev(a.b.epi, ui) = episode; ev(a.b.tstep, ui) = 0;
    ev(a.b.fin, ui) = 0;
    // wind: VKDisturbanceGenerator._new_filters (vonkarman.py:60-66): sigmas drawn per reset,
    // filter state zeroed; WindModel.compile_horizontal_fixed_wind: percentile per reset
    u32x4 r = philox({(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, kTagReset}, a.seed_lo, a.seed_hi);
    double su = P.sigma_u_lo + (P.sigma_u_hi - P.sigma_u_lo) * u01(r.x, r.y);
    double sv = P.sigma_v_lo + (P.sigma_v_hi - P.sigma_v_lo) * u01(r.z, r.w);
    ev(a.b.wind, ui) = R(0); ev(a.b.wind + N, ui) = R(0); ev(a.b.wind + (2) * N, ui) = R(0); ev(a.b.wind + (3) * N, ui) = R(0);
    ev(a.b.wind + (4) * N, ui) = (R)su; ev(a.b.wind + (5) * N, ui) = (R)sv;
    ev(a.b.wprof, ui) = a.fixed_prof >= 0 ? (uint8_t)a.fixed_prof : (uint8_t)((r.x ^ r.w) % 49u);  // randint(50, 99)
    if (reset_cache) {   // any valid 50-set is a correct start for the swap search
        ev(a.b.key, ui) = P.init_key_cd; ev(a.b.key + N, ui) = P.init_key_cl;
        ev(a.b.slot, ui) = -1; ev(a.b.slot + N, ui) = -1;
    }
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_reset(StepArgs<R> a, const uint8_t* mask) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    if (mask && !mask[i]) return;
    uint32_t ep = a.b.epi[i] + 1;
    reset_env(a, i, ep, true);
}

// Opaque copy of a uniform pointer: loads through it cannot be hoisted above this point.
// The step kernel re-launders its parameter block per sub-step, so that the ~150 uniform
// parameters are re-read (scalar loads, cheap) instead of being kept live in registers
// across the whole kernel (which cost >200 VGPRs and occupancy).
template <typename T> __device__ __forceinline__ const T* launder(const T* p) {
    uint64_t v = (uint64_t)p;
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (const T*)(((uint64_t)hi << 32) | lo);
}

// ---------------------------------------------------------------- RBF lookup + evaluation
// Lanes-per-env (LPE) decomposition: with LPE = 1 one lane evaluates both tables; with
// LPE = 2 lane role 0 owns C_D and role 1 owns C_L; with LPE = 4/8 each table is owned by a
// pair/quad of lanes that split its 50-term thin-plate sum (terms k = part, part + nparts..).
template <typename R> struct TabView {
    const R* smach;
    const R* saoa;             // per-point AoA (LDS)
    const int* start;
    const int* n;
    const R* aoa;
    const unsigned long long* keys;
    const R* pay;
    int logcap;
    int line0;                 // index of this table's first clamped line (0: C_D, 2: C_L)
    const unsigned long long* grid_key;
    const int* grid_slot;
    int grid_nm, grid_na;
    R grid_a0, grid_inv_da, grid_inv_dm;
};

// Per-workgroup LDS scratch for the rare exact on-device neighbourhood solve, guarded by a
// spin lock taken by lane 0 of the solving wave (a wave never waits on itself: it releases the
// lock before its next miss).
struct SolveLds {
    double work[kScratch];
    int lock;
};

// LDS copy of the clamped-line interval tables
template <typename R> struct LineLds {
    R bp[4][kLineMax];
    int slot[4][kLineMax + 1];
    unsigned long long key[4][kLineMax + 1];
    R a[4];
    int nbp[4];
};

template <typename R>
__device__ __forceinline__ TabView<R> tab_view(const DevParams<R>& P, const R* s_cd, const R* s_cl, int table) {
    TabView<R> t;
    t.smach = table ? s_cl : s_cd;
    t.saoa = (table ? s_cl : s_cd) + 512;   // Lds: kCdA = kCd + 512, kClA = kCl + 512
    t.start = table ? P.cl_start : P.cd_start;
    t.n = table ? P.cl_len : P.cd_len;
    t.aoa = table ? P.cl_aoa : P.cd_aoa;
    t.keys = table ? P.keys_cl : P.keys_cd;
    t.pay = table ? P.pay_cl : P.pay_cd;
    t.logcap = table ? P.logcap_cl : P.logcap_cd;
    t.line0 = table ? 2 : 0;
    t.grid_key = P.grid_key[table];
    t.grid_slot = P.grid_slot[table];
    t.grid_nm = P.grid_nm[table];
    t.grid_na = P.grid_na[table];
    t.grid_a0 = P.grid_a0[table];
    t.grid_inv_da = P.grid_inv_da[table];
    t.grid_inv_dm = P.grid_inv_dm[table];
    return t;
}

// This lane's share of sum_j c_j phi(|x - y_j|) + poly of one neighbourhood payload.
// phi(r) = r^2 log r = d2 log(d2) / 2 with d2 = |x - y|^2 (thin_plate_spline, phi(0) = 0).
// The payload names each term's table point by a byte index, whose (Mach, AoA) sit in LDS; the
// terms are evaluated in chunks of 10 independent terms so that the loads of a chunk are in
// flight together and the 10 log chains interleave.
template <typename R>
__device__ __forceinline__ R rbf_eval(const R* __restrict__ pay, const R* smach, const R* saoa, R M, R a,
                                      int part, int nparts) {
    const uint8_t* ib = (const uint8_t*)(pay + kPayIdx);
    R s0 = R(0), s1 = R(0);
#ifndef PD_CHUNK
#define PD_CHUNK 10
#endif
    constexpr int kChunk = PD_CHUNK;
    // fully unrolled: the scheduler issues a later chunk's loads under an earlier chunk's
    // arithmetic (c3 f64 0.089 -> 0.085 ms; tools/sweep.py, profiles/r01_experiments.json)
#ifdef PD_RBF_NO_UNROLL
#pragma unroll 1
#else
#pragma unroll
#endif
    for (int j0 = part; j0 < kNbr; j0 += kChunk * nparts) {
        R mm[kChunk], aa[kChunk], pp[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; ++u) {
            int j = j0 + u * nparts;
            bool ok = j < kNbr;
            int jj = ok ? j : 0;
            int ix = ib[jj];
            mm[u] = smach[ix];
            aa[u] = saoa[ix];
            pp[u] = ok ? pay[jj] : R(0);
        }
#pragma unroll
        for (int u = 0; u < kChunk; ++u) {
            R dm = M - mm[u], da = a - aa[u];
            R d2 = dm * dm + da * da;
            // c_j d2 log(d2) accumulated (the 1/2 of phi is applied once below); d2 = 0 (query
            // on a table point) contributes c_j * 0 * finite = 0
            R w = d2 * pp[u];
#ifdef PD_EXP_NOLOG
            R l = d2;
#elif defined(PD_EXP_LIBLOG)
            R l = log(d2 > R(0) ? d2 : R(1));
#else
            R l = eval_log<R>(sizeof(R) == 8 ? d2 : (d2 > R(1e-30) ? d2 : R(1e-30)));
#endif
            if (u & 1) s1 = fma(w, l, s1); else s0 = fma(w, l, s0);
        }
    }
    R s = R(0.5) * (s0 + s1);
    if (part == 0) {
        s += R(1) * pay[kNbr];
        s += (M - pay[kSys + 0]) / pay[kSys + 2] * pay[kNbr + 1];
        s += (a - pay[kSys + 1]) / pay[kSys + 3] * pay[kNbr + 2];
    }
    return s;
}

// slow path: the neighbourhood is not in the table -> solve it here, exactly, on one lane
// (rare: the table is pre-enumerated over the reachable domain), and queue it for insertion.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Wave-cooperative exact solve of one neighbourhood into the workgroup's LDS scratch: lane r
// owns row r of the 53x53 system; LU with partial pivoting (pivot by a wave max-reduction,
// smallest row index on ties) and column-oriented back substitution -- the operations and
// their order per element are those of solve_neighbourhood(), so the payload is bit-identical
// to the host-built one.  Must be called by a converged wave (all 64 lanes active).
template <typename R>
__device__ __noinline__ void solve_wave(const DevParams<R>& P, int table, unsigned long long key, SolveLds* sl) {
    const int lane = (int)__lane_id();
    double* A = sl->work;
    double* b = A + kSys * kSys;
    double* ym = b + kSys;
    double* ya = ym + kNbr;
    double* yd = ya + kNbr;
    double* pay = sl->work + (kScratch - kPay);
    const double* mach = table ? P.cl_mach_d : P.cd_mach_d;
    const double* coef = table ? P.cl_coef_d : P.cd_coef_d;
    const int* start = table ? P.cl_start : P.cd_start;
    const double* aoa = table ? P.cl_aoa_d : P.cd_aoa_d;
    int lo[kCols], len[kCols];
    key_unpack(key, lo, len);
    int my_idx = 0;
    if (lane < kNbr) {
        int c = 0, off = lane, acc = 0;
#pragma unroll
        for (int q = 0; q < kCols; ++q) {
            if (lane >= acc && lane < acc + len[q]) { c = q; off = lane - acc; }
            acc += len[q];
        }
        int idx = start[c] + lo[c] + off;
        my_idx = idx;
        ym[lane] = mach[idx]; ya[lane] = aoa[c]; yd[lane] = coef[idx];
    }
    lds_sync();
    double mn0 = ym[0], mx0 = ym[0], mn1 = ya[0], mx1 = ya[0];
    for (int j = 1; j < kNbr; ++j) {
        double u = ym[j], w = ya[j];
        mn0 = u < mn0 ? u : mn0; mx0 = u > mx0 ? u : mx0;
        mn1 = w < mn1 ? w : mn1; mx1 = w > mx1 ? w : mx1;
    }
    double sh0 = (mx0 + mn0) / 2, sc0 = (mx0 - mn0) / 2, sh1 = (mx1 + mn1) / 2, sc1 = (mx1 - mn1) / 2;
    if (sc0 == 0.0) sc0 = 1.0;
    if (sc1 == 0.0) sc1 = 1.0;
    if (lane < kNbr) {
        double yi = ym[lane], ai = ya[lane];
        for (int j = 0; j < kNbr; ++j) {
            double d0 = yi - ym[j], d1 = ai - ya[j];
            A[lane * kSys + j] = tps(sqrt(d0 * d0 + d1 * d1));
        }
        A[lane * kSys + kNbr] = 1.0;
        A[lane * kSys + kNbr + 1] = (yi - sh0) / sc0;
        A[lane * kSys + kNbr + 2] = (ai - sh1) / sc1;
        b[lane] = yd[lane];
    } else if (lane < kSys) {
        for (int j = 0; j < kNbr; ++j)
            A[lane * kSys + j] = lane == kNbr ? 1.0 : (lane == kNbr + 1 ? (ym[j] - sh0) / sc0 : (ya[j] - sh1) / sc1);
        for (int j = kNbr; j < kSys; ++j) A[lane * kSys + j] = 0.0;
        b[lane] = 0.0;
    }
    lds_sync();
    bool singular = false;
    for (int k = 0; k < kSys; ++k) {
        double v = (lane >= k && lane < kSys) ? fabs(A[lane * kSys + k]) : -1.0;
        int p = lane;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            double ov = __shfl_xor(v, o);
            int op = __shfl_xor(p, o);
            if (ov > v || (ov == v && op < p)) { v = ov; p = op; }
        }
        if (v == 0.0) { singular = true; break; }
        if (p != k) {
            if (lane < kSys) { double t = A[k * kSys + lane]; A[k * kSys + lane] = A[p * kSys + lane]; A[p * kSys + lane] = t; }
            if (lane == 0) { double t = b[k]; b[k] = b[p]; b[p] = t; }
            lds_sync();
        }
        double r = 1.0 / A[k * kSys + k];
        if (lane > k && lane < kSys) {
            double l = A[lane * kSys + k] * r;
            if (l != 0.0)
                for (int j = k + 1; j < kSys; ++j) A[lane * kSys + j] -= l * A[k * kSys + j];
            b[lane] -= l * b[k];
        }
        lds_sync();
    }
    if (!singular) {
        for (int i = kSys - 1; i >= 0; --i) {
            double xi = b[i] / A[i * kSys + i];
            lds_sync();
            if (lane == i) b[i] = xi;
            if (lane < i) b[lane] -= A[lane * kSys + i] * xi;
            lds_sync();
        }
    }
    if (lane < kSys) pay[lane] = singular ? (double)NAN : b[lane];
    else if (lane == kSys) pay[kSys] = sh0;
    else if (lane == kSys + 1) pay[kSys + 1] = sh1;
    else if (lane == kSys + 2) pay[kSys + 2] = sc0;
    else if (lane == kSys + 3) pay[kSys + 3] = sc1;
    else if (lane < kPay) pay[lane] = 0.0;
    lds_sync();
    if (lane < kNbr) ((uint8_t*)(pay + kPayIdx))[lane] = (uint8_t)my_idx;
    lds_sync();
    // payload in the kernel's precision, in the (now free) matrix area (pay_store, by lanes)
    R* pr = (R*)sl->work;
    if (lane < kPayIdx) pr[lane] = (R)pay[lane];
    else if (lane < pay_stride<R>()) pr[lane] = R(0);
    lds_sync();
    if (lane < kNbr) ((uint8_t*)(pr + kPayIdx))[lane] = (uint8_t)my_idx;
    lds_sync();
}

// Each distinct (table, key) missed by the wave is solved cooperatively into the workgroup's LDS
// scratch (under its lock), evaluated by the lanes that need it, and queued for insertion into
// the device table (pd_flush_misses).  Called by the converged wave.
template <typename R>
__device__ __forceinline__ R rbf_miss_wave(const StepArgs<R>& a, SolveLds* sl, int table, const R* smach,
                                        const R* saoa, unsigned long long key, R M, R aq,
                                        int part, int nparts, bool need) {
    R val = R(0);
    unsigned long long mm = __ballot(need);
    while (mm) {
        int leader = __ffsll((long long)mm) - 1;
        unsigned long long lk = ((unsigned long long)(unsigned int)__shfl((int)(key >> 32), leader) << 32) |
                                (unsigned int)__shfl((int)key, leader);
        int lt = __shfl(table, leader);
        if (__lane_id() == 0) {
            while (atomicCAS(&sl->lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        solve_wave<R>(*a.P, lt, lk, sl);
        if (need && key == lk && table == lt) {
            val = rbf_eval<R>((const R*)sl->work, smach, saoa, M, aq, part, nparts);
            need = false;
        }
        if ((int)__lane_id() == leader) {
            atomicAdd(&a.pend.stats[0], 1ull);
            unsigned long long idx = atomicAdd(a.pend.count, 1ull);
            const double* pay = sl->work + (kScratch - kPay);
            if (idx < (unsigned long long)kPendingCap) {
                for (int j = 0; j < kPay; ++j) a.pend.pay[idx * kPay + j] = pay[j];
                a.pend.keys[idx] = lk | ((unsigned long long)lt << 63);
            }
        }
        lds_sync();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (__lane_id() == 0) atomicExch(&sl->lock, 0);
        mm = __ballot(need);
    }
    return val;
}

// This lane's share of the RBF value of `table` at (M, aq).
// Candidate neighbourhood: on a clamped query line (the common case: |alpha_eff| > 0.003 rad
// clamps both tables) the interval table of that line (binary search over <= 96 Mach
// breakpoints in LDS); elsewhere the env's cached set.  Either way the candidate is VERIFIED
// (and repaired by the swap search) against the exact distances before it is used.
template <typename R>
__device__ __forceinline__ R rbf(const StepArgs<R>& a, SolveLds* sl, int table, const TabView<R>& t,
                                 const LineLds<R>& ln, RbfCache<R>& cache, R M, R aq, int part, int nparts) {
    unsigned long long ckey = cache.key;
    int cslot = cache.slot;
    int li = aq == ln.a[t.line0] ? t.line0 : (aq == ln.a[t.line0 + 1] ? t.line0 + 1 : -1);
    bool trusted = false;
    if (li >= 0 && ln.nbp[li] >= 0) {
        const int nb = ln.nbp[li];
        int l = 0, h = nb;
        while (l < h) { int mid = (l + h) >> 1; if (ln.bp[li][mid] < M) l = mid + 1; else h = mid; }
        ckey = ln.key[li][l];
        cslot = ln.slot[li][l];
        // The host split the line at EVERY pairwise bisector, so the 50-NN set is constant
        // strictly between breakpoints: the interval's key is exact unless M lies within
        // rounding distance of a breakpoint (then the search below verifies it).
        const R eps = sizeof(R) == 8 ? R(1e-9) : R(1e-4);
        const R blo = l > 0 ? ln.bp[li][l - 1] : R(-1);
        const R bhi = l < nb ? ln.bp[li][l] : R(1e30);
        trusted = cslot >= 0 && (M - blo > eps) && (bhi - M > eps);
    } else if (t.grid_key) {
        R fm = M * t.grid_inv_dm, fa = (aq - t.grid_a0) * t.grid_inv_da;
        int im = fm < R(0) ? 0 : (fm >= R(t.grid_nm) ? t.grid_nm - 1 : (int)fm);
        int ia = fa < R(0) ? 0 : (fa >= R(t.grid_na) ? t.grid_na - 1 : (int)fa);
        if (!(fm == fm) || !(fa == fa)) { im = 0; ia = 0; }   // NaN queries
        int cell = im * t.grid_na + ia;
        ckey = t.grid_key[cell];
        const int gsl = t.grid_slot[cell];
        cslot = gsl < 0 ? -1 : (gsl & (kGridExact - 1));
        // every point of an exact cell has the cell's key (convexity of 50-NN regions); the
        // rounding margin keeps queries on a cell edge on the verified path
        const R eps = sizeof(R) == 8 ? R(1e-9) : R(1e-4);
        trusted = gsl >= 0 && (gsl & kGridExact) && fm - (R)im > eps && (R)(im + 1) - fm > eps &&
                  fa - (R)ia > eps && (R)(ia + 1) - fa > eps;
    }
    unsigned long long key = ckey;
    int slot = cslot;
#ifdef PD_EXP_TRUSTCHECK
    const bool check_trusted = trusted;
    trusted = false;
#endif
    if (!trusted) {
        int lo[kCols], len[kCols];
        key_unpack(ckey, lo, len);
        // keys store lo=0 for empty columns; knn_windows uses insertion points for those
#ifndef PD_EXP_NOKNN
#ifdef PD_EXP_COUNT
        int iters = knn_windows<R>(t.smach, t.start, t.n, t.aoa, M, aq, lo, len);
        atomicAdd(&a.pend.stats[4], 1ull);
        atomicAdd(&a.pend.stats[5], (unsigned long long)(li >= 0));
        atomicAdd(&a.pend.stats[6], (unsigned long long)iters);
#else
        knn_windows<R>(t.smach, t.start, t.n, t.aoa, M, aq, lo, len);
#endif
#endif
        key = key_pack(lo, len);
        slot = key == ckey ? cslot : -1;
#ifdef PD_EXP_TRUSTCHECK
        atomicAdd(&a.pend.stats[4], (unsigned long long)check_trusted);
        atomicAdd(&a.pend.stats[7], (unsigned long long)(check_trusted && key != ckey));
#endif
    }
    if (slot < 0) {
        uint32_t mask = (1u << t.logcap) - 1u;
        uint32_t h = key_hash(key, t.logcap);
        for (uint32_t probe = 0; probe <= mask; ++probe) {
            unsigned long long k = t.keys[h];
            if (k == key) { slot = (int)h; break; }
            if (k == kEmptyKey) break;
            h = (h + 1) & mask;
        }
    }
    cache.key = key;
    cache.slot = slot;
    R val = R(0);
    if (slot >= 0) val = rbf_eval<R>(t.pay + (int64_t)slot * pay_stride<R>(), t.smach, t.saoa, M, aq, part, nparts);
    // Misses (a neighbourhood outside the pre-enumerated tables) take the wave-cooperative
    // exact solve; the loop in rbf_miss_wave runs only when some lane of the wave missed
    if (__ballot(slot < 0)) {
        R mv = rbf_miss_wave<R>(a, sl, table, t.smach, t.saoa, key, M, aq, part, nparts, slot < 0);
        if (slot < 0) val = mv;
    }
    return val;
}

// rocket_CD query: CD_func = rocket_CD(M, degrees(alpha)); clamp of the DEGREE value at
// +-radians(10) (rockets_physics.py:712, aerodynamic_coefficients.py:105-115)
template <typename R> __device__ __forceinline__ R cd_query(R ae) {
    R aoa = ae * Cst<R>::rad2deg;
    const R r10 = (R)(10.0 * kDeg2Rad);
    if (aoa > r10) aoa = r10;
    else if (aoa < (R)(-10.0 * kDeg2Rad)) aoa = (R)(-10.0 * kDeg2Rad);
    return aoa;
}
// rocket_CL query: degrees applied twice (rockets_physics.py:711 + aerodynamic_coefficients.py:117-132)
// returns the RBF abscissa, the sign to apply, and whether C_L is exactly 0
template <typename R> __device__ __forceinline__ R cl_query(R ae, R& sgn, bool& zero) {
    R aq = (ae * Cst<R>::rad2deg) * Cst<R>::rad2deg;
    sgn = R(1);
    zero = false;
    if (aq > R(10)) aq = R(10);
    else if (aq < R(-10)) aq = R(-10);
    else if (fabs(aq) < R(1e-6)) zero = true;
    else if (aq < R(0)) { aq = fabs(aq); sgn = R(-1); }
    return aq;
}

// ---------------------------------------------------------------- the step kernel
// simple_actor.forward (env_wrapped_ea.py:18-44): Linear(IN,8)-ReLU-[Linear(8,8)-ReLU]xNL-
// Linear(8,OUT)-Tanh in binary32 on the float32-cast observation.  Parameters are in
// named_parameters() order (weight [out][in] row-major, then bias, layer by layer), stored
// parameter-major [P][N] so that every load is coalesced across the envs of a wave.
// Each output is the sequential sum over inputs (no FMA) plus the bias; tanh is evaluated in
// binary64 and rounded (the oracle restates the same order: oracle/pd_oracle.c orc_actor).
template <int IN, int NL, int OUT>
__device__ __forceinline__ void actor_forward(const float* __restrict__ W, int64_t N, uint32_t ui,
                                              const float* x, float* y) {
    constexpr int H = 8;
    float h[H], g[H];
    int64_t p = 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < IN; ++k) acc = acc + ev(W + (p + j * IN + k) * N, ui) * x[k];
        acc = acc + ev(W + (p + H * IN + j) * N, ui);
        h[j] = acc < 0.f ? 0.f : acc;
    }
    p += H * IN + H;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < H; ++k) acc = acc + ev(W + (p + j * H + k) * N, ui) * h[k];
            acc = acc + ev(W + (p + H * H + j) * N, ui);
            g[j] = acc < 0.f ? 0.f : acc;
        }
#pragma unroll
        for (int j = 0; j < H; ++j) h[j] = g[j];
        p += H * H + H;
    }
#pragma unroll
    for (int j = 0; j < OUT; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < H; ++k) acc = acc + ev(W + (p + j * H + k) * N, ui) * h[k];
        acc = acc + ev(W + (p + H * OUT + j) * N, ui);
        y[j] = (float)tanh((double)acc);
    }
}

// PD_STAMP (diagnostic builds only): per-wave shader-clock sections of k_step, summed into
// pend.stats[8..15] (staging, loads, pre-aero, aero tables, post-aero, rtd, outputs, waves)
#ifdef PD_STAMP
#define PD_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PD_ACC(k, d) acc_[k] += (d)
#else
#define PD_T(v)
#define PD_ACC(k, d)
#endif

template <bool WIND> struct Lds {
    // table Mach values and, 512 further on, each point's AoA (tab_view relies on that offset)
    static constexpr int kCd = 0, kCl = 256, kCdA = 512, kClA = 768, kCaX = 1024, kCaY = 1088, kCnX = 1152,
                         kCnY = 1216, kWAlt = 1280, kWSp = kWAlt + 800, kTotal = WIND ? kWSp + 800 : kWAlt;
};

template <typename R, int PHASE, int RTD, bool WIND, int LPE, int POL = 0>
// waves_per_eu(2): caps VGPR+AGPR at 256 so the f64 kernel keeps two waves per SIMD (without it
// the allocator spilled into AGPRs and ran one wave per SIMD, 20% slower on the c3 workload).
#ifndef PD_WPE
#define PD_WPE 2
#endif
__global__ __launch_bounds__(kStepBlock) __attribute__((amdgpu_waves_per_eu(PD_WPE))) void k_step(StepArgs<R> a) {
    using L = Lds<WIND>;
#ifdef PD_STAMP
    unsigned long long acc_[7] = {0, 0, 0, 0, 0, 0, 0};
#endif
    PD_T(t_start);
    __shared__ R lds[L::kTotal];
    __shared__ LineLds<R> lines;
    __shared__ SolveLds solve;
    const DevParams<R>& P = *a.P;
    // envs this launch steps: all N, or (POL) the compacted live list; a workgroup past its end
    // leaves before staging the tables (workgroup-uniform)
    int64_t n_act = a.n;
    if constexpr (POL) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *a.cnt_zero = 0u;
        if (a.use_list) {
            n_act = (int64_t)*a.cnt_in;
            if ((int64_t)blockIdx.x * (kStepBlock / LPE) >= n_act) return;
        }
    }
    for (int t = threadIdx.x; t < 256; t += kStepBlock) {
        lds[L::kCd + t] = P.cd_mach[t]; lds[L::kCl + t] = P.cl_mach[t];
        lds[L::kCdA + t] = P.cd_pt_aoa[t]; lds[L::kClA + t] = P.cl_pt_aoa[t];
    }
    if (threadIdx.x < 64) {
        lds[L::kCaX + threadIdx.x] = P.ca_x[threadIdx.x]; lds[L::kCaY + threadIdx.x] = P.ca_y[threadIdx.x];
        lds[L::kCnX + threadIdx.x] = P.cn_x[threadIdx.x]; lds[L::kCnY + threadIdx.x] = P.cn_y[threadIdx.x];
    }
    if constexpr (WIND) {
        for (int t = threadIdx.x; t < 800; t += kStepBlock) {
            lds[L::kWAlt + t] = (&P.wind_alt_km[0][0])[t];
            lds[L::kWSp + t] = (&P.wind_speed[0][0])[t];
        }
    }
    for (int t = threadIdx.x; t < 4 * kLineMax; t += kStepBlock) (&lines.bp[0][0])[t] = (&P.line_bp[0][0])[t];
    for (int t = threadIdx.x; t < 4 * (kLineMax + 1); t += kStepBlock) {
        (&lines.slot[0][0])[t] = (&P.line_slot[0][0])[t];
        (&lines.key[0][0])[t] = (&P.line_key[0][0])[t];
    }
    if (threadIdx.x < 4) { lines.a[threadIdx.x] = P.line_a[threadIdx.x]; lines.nbp[threadIdx.x] = P.line_nbp[threadIdx.x]; }
    if (threadIdx.x == 0) solve.lock = 0;
    for (int t = threadIdx.x; t < kLogCells; t += kStepBlock) {
        s_logtab[t] = P.logtab.invc[t]; s_logtab[kLogCells + t] = P.logtab.logc[t];
    }
    __syncthreads();
    PD_T(t_staged);
    PD_ACC(0, t_staged - t_start);
    const int64_t N = a.n;
    const int64_t gt = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
    // every lane stays active (the cooperative miss solve needs converged waves): lanes past
    // the end recompute the last env and write nothing
    const bool valid = gt / LPE < n_act;
    const int64_t e_act = valid ? gt / LPE : n_act - 1;
    const int64_t i = (POL && a.use_list) ? (int64_t)a.list_in[e_act] : e_act;
    const int role = (int)(gt % LPE);
    const uint32_t ui = (uint32_t)i;   // N <= 2^25 (validated): 32-bit per-lane byte offsets
    // POL (policy rollout): with the list, only live envs are stepped; without it, finished
    // envs stay frozen and a wave with none left exits (wave-uniform, after the only barrier)
    bool live_ = valid;
    if constexpr (POL) {
        if (!a.use_list) {
            live_ = live_ && ev(a.b.fin, ui) == 0;
            if (__ballot(live_) == 0) return;
        }
    }
    const bool live = live_;
    // role -> (table, part): LPE 1: both tables on one lane; else table = role / (LPE/2)
    constexpr int nparts = LPE >= 2 ? LPE / 2 : 1;
    const int my_table = LPE >= 2 ? role / nparts : 0;   // 0 = C_D, 1 = C_L
    const int part = LPE >= 2 ? role % nparts : 0;
    const int gbase = (int)__lane_id() & ~(LPE - 1);
    const R* s_cd = lds + L::kCd;
    const R* s_cl = lds + L::kCl;

    // Fused launches (pd_step_n, pd_rollout): n_fused consecutive env-steps of the same envs,
    // each the body below with its own action row and output rows.  The per-env state goes
    // through memory between them exactly as between launches; the lanes that store a field
    // and the lanes that load it next are in the same wave, so a workgroup-scope fence (a
    // wait on the outstanding stores) orders them.  Saves the table staging and the launch
    // tail per step, and lets each wave run ahead of the slowest (e.g. a miss-solving) one.
    const int nf = POL ? 1 : a.n_fused;
#pragma unroll 1
    for (int f = 0; f < nf; ++f) {
    if (f > 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const size_t fo = (size_t)f * (size_t)N;

    R s[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) s[k] = ldv(a.b.st + (k) * N, ui);
    RbfCache<R> cA, cB;   // LPE 1: A = C_D, B = C_L; LPE >= 2: A = own table
    cA.key = ldv(a.b.key + (my_table) * N, ui); cA.slot = ldv(a.b.slot + (my_table) * N, ui);
    if constexpr (LPE == 1) { cB.key = ldv(a.b.key + N, ui); cB.slot = ldv(a.b.slot + N, ui); }
    else { cB.key = 0; cB.slot = -1; }
    R gprev = R(0), dlprev = R(0), drprev = R(0);
    if constexpr (PHASE == 1) { gprev = ldv(a.b.act, ui); dlprev = ldv(a.b.act + N, ui); drprev = ldv(a.b.act + (2) * N, ui); }
    // PHASE 2 = the other compile_physics phases, chosen at run time by P.phase (wave-uniform)
    const int aux = PHASE == 2 ? a.P->phase : PHASE;
    const bool ascent = PHASE == 2 && (aux == PD_PHASE_SUBSONIC || aux == PD_PHASE_SUPERSONIC);
    if constexpr (PHASE == 2) gprev = ldv(a.b.act, ui);   // flip-over gimbal memory
    R fu0 = R(0), fu1 = R(0), fv0 = R(0), fv1 = R(0), sgu = R(0), sgv = R(0);
    int prof = 0;
    if constexpr (WIND) {
        fu0 = ldv(a.b.wind, ui); fu1 = ldv(a.b.wind + N, ui); fv0 = ldv(a.b.wind + (2) * N, ui); fv1 = ldv(a.b.wind + (3) * N, ui);
        sgu = ldv(a.b.wind + (4) * N, ui); sgv = ldv(a.b.wind + (5) * N, ui);
        prof = ldv(a.b.wprof, ui);
    }
    const uint32_t ep = ldv(a.b.epi, ui), ts = ldv(a.b.tstep, ui);
    const uint64_t g = a.env_offset + (uint64_t)i;

    // actions (float32 unless act_f64)
    constexpr int A = PHASE == 0 ? 1 : (PHASE == 1 ? 4 : 2);
    const int AD = PHASE == 2 ? (ascent ? 2 : 1) : A;   // row stride of the action array
    float uf[A];
    double ud[A];
#pragma unroll
    for (int k = 0; k < A; ++k) { uf[k] = 0.f; ud[k] = 0.0; }
    if constexpr (POL) {
        // pso_wrapper.augment_state (env_wrapped_ea.py:97-123) of the current state in the
        // handle's precision, cast to float32 (simple_actor.forward), then the actor
        const DevParams<R>& Q = *a.P;
        if constexpr (PHASE == 0) {
            float x[2] = {(float)(s[1] / Q.norm_y), (float)(s[3] / Q.norm_vy)};
            actor_forward<2, 3, 1>(a.policy_w, N, ui, x, uf);
        } else {
            float x[5] = {(float)(s[0] / Q.norm_x), (float)(s[1] / Q.norm_y), (float)(s[2] / Q.norm_vx),
                          (float)(s[3] / Q.norm_vy), (float)tanh(Q.k_theta_pso * (s[4] - Cst<R>::pi / R(2)))};
            actor_forward<5, 4, 4>(a.policy_w, N, ui, x, uf);
        }
    } else if (a.act_f64) {
#pragma unroll
        for (int k = 0; k < A; ++k) if (k < AD) ud[k] = ldv((const double*)a.actions + fo * AD + k, ui * AD);
    } else {
#pragma unroll
        for (int k = 0; k < A; ++k) if (k < AD) uf[k] = ldv((const float*)a.actions + fo * AD + k, ui * AD);
    }

    // pure throttle 4 x 0.025 s, landing_burn 4 x 0.1 s (actuators 0.025 s); the other phases
    // one call of rocket_physics_fcn at dt, actuators at the same dt (rockets_physics.py:728-997)
    constexpr int NSUB = PHASE == 2 ? 1 : 4;
    const R dt = PHASE == 0 ? R(0.025) : (PHASE == 1 ? R(0.1) : (R)a.dt_aux);
    const R dt_act = PHASE == 2 ? dt : R(0.025);
    R gdeg_out = gprev, dcmdl_out = dlprev, dcmdr_out = drprev;
    bool nan_hit = false;

    PD_T(t_loaded);
    PD_ACC(1, t_loaded - t_staged);
#pragma unroll 1
    for (int sub = 0; sub < NSUB; ++sub) {
        PD_T(t_sub);
        const DevParams<R>& P = *launder(a.P);
        R x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], thd = s[5], ga = s[6], al = s[7];
        R m = s[8], mp = s[9];
        // rocket_physics_fcn (rockets_physics.py:455-704)
        R rho, patm, asnd;
        atmosphere<R>(P, y, rho, patm, asnd);
        R speed = sqrt(vx * vx + vy * vy);
        R mach = R(0);
        if (asnd != R(0)) { R mr = speed / asnd; mach = (R(10) < mr) ? R(10) : mr; }
        R q = R(0.5) * rho * (speed * speed);
        R fpc = (P.m_prop0 - mp) / P.m_prop0;
        if (fpc == R(0)) fpc = R(1e-6);
        R x_cog, I;
        // subrocket_0 (full rocket) closures for the ascent, subrocket_2 after (:748-750, :772-774)
        if (ascent) inertia_full<R>(P, R(1) - fpc, x_cog, I);
        else inertia<R>(P, R(1) - fpc, x_cog, I);
        R d_thrust = x_cog + P.engine_height;
        R ae = (vy < R(0)) ? ga - th - Cst<R>::pi : al;
        R d_cp_cg = x_cog - (ascent ? P.cop_ascent : P.cop);
        R ug = R(0), vg = R(0);
        if constexpr (WIND) {
            // WindModel.__call__ (full_wind_model.py:35-43)
            const R* walt = lds + L::kWAlt + prof * 16;
            const R* wsp = lds + L::kWSp + prof * 16;
            R km = y / R(1000);
            int wn = P.wind_n[prof];
            ug = np_interp<R>(walt, wsp, wn, km);
            if (y < P.vk_y_threshold && a.stochastic) {
                double w0, w1;
                if (a.noise) { w0 = ev(a.noise + 2 * sub, ui * 8); w1 = ev(a.noise + 2 * sub + 1, ui * 8); }
                else {
                    u32x4 r = philox({(uint32_t)g, (uint32_t)(g >> 32) ^ ep, ts, kTagWindSub + (uint32_t)sub},
                                     a.seed_lo, a.seed_hi);
                    // Box-Muller in binary32 on 24-bit uniforms (hardware log2 and sin/cos of 2*pi*u):
                    // the gust normals are random variates, their last bits carry no physics
                    float u1 = 1.0f - (float)(r.x >> 8) * 0x1p-24f, u2 = (float)(r.z >> 8) * 0x1p-24f;
                    float rad = sqrtf(-1.38629436112f * __builtin_amdgcn_logf(u1));
                    w0 = (double)(rad * __builtin_amdgcn_cosf(u2)); w1 = (double)(rad * __builtin_amdgcn_sinf(u2));
                }
                // vonkarman.py:33-36: state = Ad @ state + Bd * w  (Bd = sigma * Bd(sigma=1))
                R n0 = (P.vk_Ad_u[0] * fu0 + P.vk_Ad_u[1] * fu1) + (sgu * P.vk_Bd_u[0]) * (R)w0;
                R n1 = (P.vk_Ad_u[2] * fu0 + P.vk_Ad_u[3] * fu1) + (sgu * P.vk_Bd_u[1]) * (R)w0;
                fu0 = n0; fu1 = n1;
                n0 = (P.vk_Ad_v[0] * fv0 + P.vk_Ad_v[1] * fv1) + (sgv * P.vk_Bd_v[0]) * (R)w1;
                n1 = (P.vk_Ad_v[2] * fv0 + P.vk_Ad_v[3] * fv1) + (sgv * P.vk_Bd_v[1]) * (R)w1;
                fv0 = n0; fv1 = n1;
                ug = ug + fu1;
                vg = fv1;
            }
        }
        R Fwx = R(0.5) * rho * (ug * ug) * P.A_front * P.C_gust_x;
        R Fwy = R(0.5) * rho * (vg * vg) * P.A_front * P.C_gust_y;
        R Mw = -d_cp_cg * Fwy;
        R CL = R(0), CD = R(0);
        PD_T(t_aero0);
        PD_ACC(2, t_aero0 - t_sub);
#ifndef PD_EXP_NORBF
        {
            // evaluated convergently by every lane; results of lanes that need none (speed of
            // sound 0 above 81 km, |deg(deg(alpha))| < 1e-6 for C_L) are discarded
            R cl_sgn; bool cl_zero;
            R aq_cl = cl_query<R>(ae, cl_sgn, cl_zero);
            R aq_cd = cd_query<R>(ae);
            const bool have = asnd != R(0);
            if constexpr (LPE == 1) {
                R v = rbf<R>(a, &solve, 1, tab_view<R>(P, s_cd, s_cl, 1), lines, cB, mach, aq_cl, 0, 1);
                CL = (!have || cl_zero) ? R(0) : (cl_sgn < R(0) ? -v : v);
                R w = rbf<R>(a, &solve, 0, tab_view<R>(P, s_cd, s_cl, 0), lines, cA, mach, aq_cd, 0, 1);
                CD = have ? w : R(0);
            } else {
                R v = rbf<R>(a, &solve, my_table, tab_view<R>(P, s_cd, s_cl, my_table), lines, cA, mach,
                             my_table ? aq_cl : aq_cd, part, nparts);
                if constexpr (nparts >= 2) v += __shfl_xor(v, 1);
                if constexpr (nparts >= 4) v += __shfl_xor(v, 2);
                if constexpr (nparts >= 8) v += __shfl_xor(v, 4);
                R vcd = __shfl(v, gbase);
                R vcl = __shfl(v, gbase + nparts);
                CD = have ? vcd : R(0);
                CL = (!have || cl_zero) ? R(0) : (cl_sgn < R(0) ? -vcl : vcl);
            }
        }
#endif
        PD_T(t_aero1);
        PD_ACC(3, t_aero1 - t_aero0);
        R drag = R(0.5) * rho * (speed * speed) * CD * P.A_front;
        R lift = R(0.5) * rho * (speed * speed) * CL * P.A_front;
        R sae, cae;
        pd_sincos<R>(ae, sae, cae);
        R apar, aperp;
        if (vy >= R(0)) { apar = lift * sae - drag * cae; aperp = -lift * cae - drag * sae; }
        else { apar = drag * cae - lift * sae; aperp = -drag * sae - lift * cae; }
        R sth, cth;
        pd_sincos<R>(th, sth, cth);
        R aero_x = apar * cth + aperp * sth;
        R aero_y = apar * sth - aperp * cth;
        R aero_m = aperp * d_cp_cg;
        if (PHASE == 2 && aux == PD_PHASE_FLIP_OVER) { aero_x = R(0); aero_y = R(0); aero_m = R(0); }   // :548-551

        R T_full = P.T_e + (P.p_e - patm) * P.A_e;
        R qS = q * P.S_gf;
        R Ca = grid_fin_ca<R>(P, lds + L::kCaX, lds + L::kCaY, mach);
        R cfp, cfperp, cm, mdot_dt, md_info, thr_info;
        // binary32 control forces (ascent, float32 actions): the force sums then stay binary32,
        // the aero terms being Python floats (weak under NEP 50, rockets_physics.py:608-616)
        bool f32_forces = false;
        float cfp_f = 0.f, cfperp_f = 0.f;
        if constexpr (PHASE == 2) {
            if (aux == PD_PHASE_PCONTROL) {
                // force_moment_decomposer_landing_burn_throttle_PID (:402-451): throttle from
                // v_ref - speed (Kp -0.08, clip [0, 1]) into throttle_only as a list (binary64)
                R u0;
                if (a.act_f64) {
                    R nt = ((R)ud[0] - speed) * P.kp_pc;
                    nt = nt < R(0) ? R(0) : (nt > R(1) ? R(1) : nt);
                    u0 = R(2) * (nt - R(0.5));
                } else {
                    float nt = (uf[0] - (float)speed) * P.f_kp_pc;
                    nt = nt < 0.f ? 0.f : (nt > 1.f ? 1.f : nt);
                    u0 = (R)(2.0f * (nt - 0.5f));
                }
                R thr = (u0 + R(1)) / R(2) * P.one_minus_nom_pt + P.nom_pt;
                R tg = T_full * (R)P.n_eng * thr;
                R md = P.Te_over_vex * (tg / T_full);
                cfp = tg + qS * (Ca * R(4)); cfperp = R(0); cm = R(0);   // ACS, zero deflection
                mdot_dt = md * dt; md_info = md; thr_info = thr;
            } else if (aux == PD_PHASE_BALLISTIC_ARC) {
                // RCS (:149-166): moment only, promoted to binary64 by x_cog; no mass flow
                R tf = a.act_f64 ? P.rcs_force * (R)ud[0] : (R)(P.f_rcs_force * uf[0]);
                cfp = R(0); cfperp = R(0);
                cm = -tf * (x_cog - P.rcs_d_bottom) + tf * (P.rcs_d_top - x_cog);
                mdot_dt = R(0); md_info = R(0); thr_info = R(0);
            } else if (aux == PD_PHASE_FLIP_OVER) {
                // force_moment_decomposer_flipoverboostbackburn (:63-92): gimbal low-pass (tau 1,
                // dt), full throttle; the filtered angle keeps the action's dtype
                R gd;
                if (a.act_f64) gd = gprev + dt * ((-gprev + (R)ud[0] * R(10)) / R(1));
                else { float x0 = (float)gprev; gd = (R)(x0 + (float)dt * ((-x0 + uf[0] * 10.0f) / 1.0f)); }
                R grad = gd * Cst<R>::deg2rad;
                R tg = T_full * (R)P.n_eng;
                R cg = cos(grad), sg = sin(grad);
                R tpar = tg * cg, tperp = -tg * sg;
                cfp = tpar; cfperp = tperp; cm = -tg * sg * d_thrust;
                R md = P.Te_over_vex * (sqrt(tpar * tpar + tperp * tperp) / T_full);
                mdot_dt = md * dt; md_info = md; thr_info = R(1);
                gdeg_out = gd; gprev = gd;
            } else {
                // force_moment_decomposer_ascent (:17-56): 16 gimballed + 26 fixed, nominal 0.5,
                // gimbal radians(7)
                const R ng = (R)P.n_eng, nng = (R)(P.n_eng_stage1 - P.n_eng);
                if (a.act_f64) {
                    R grad = (R)ud[0] * P.mg_ascent;
                    R thr = ((R)ud[1] + R(1)) / R(2) * R(0.5) + R(0.5);
                    R tg = T_full * ng * thr, tng = T_full * nng * thr;
                    R cg = cos(grad), sg = sin(grad);
                    R tpar = tng + tg * cg, tperp = -tg * sg;
                    cfp = tpar; cfperp = tperp; cm = -tg * sg * d_thrust;
                    R md = P.Te_over_vex * (sqrt(tpar * tpar + tperp * tperp) / T_full);
                    mdot_dt = md * dt; md_info = md; thr_info = thr;
                    gdeg_out = grad * Cst<R>::rad2deg;
                } else {
                    float grad = uf[0] * P.f_mg_ascent;
                    float nnt = (uf[1] + 1.0f) / 2.0f;
                    float thr = nnt * 0.5f + 0.5f;
                    float tg = (float)(T_full * ng) * thr, tng = (float)(T_full * nng) * thr;
                    float cg = (float)cos((R)grad), sg = (float)sin((R)grad);
                    float tpar = tng + tg * cg, tperp = (-tg) * sg;
                    float tot = sqrtf(tpar * tpar + tperp * tperp);
                    float mdf = P.f_Te_over_vex * (tot / (float)T_full);
                    cfp_f = tpar; cfperp_f = tperp; f32_forces = true;
                    cfp = (R)tpar; cfperp = (R)tperp; cm = (R)((-tg) * sg) * d_thrust;
                    mdot_dt = (R)(mdf * (float)dt); md_info = (R)mdf; thr_info = (R)thr;
                    gdeg_out = (R)grad * Cst<R>::rad2deg;
                }
            }
        } else if constexpr (PHASE == 0) {
            // force_moment_decomposer_landing_burn_throttle_only (:340-400); ACS with zero
            // deflection: F_perp = M = 0 exactly, F_par = qS * (Ca * (2 + 1 + 1))
            R acs_par = qS * (Ca * R(4));
            if (a.act_f64) {
                R u0 = (R)ud[0];
                R nnt = (u0 + R(1)) / R(2);
                R thr = nnt * P.one_minus_nom_pt + P.nom_pt;
                R tg = T_full * (R)P.n_eng * thr;
                R md = P.Te_over_vex * (tg / T_full);
                cfp = tg + acs_par; mdot_dt = md * dt; md_info = md; thr_info = thr;
            } else {
                float nnt = (uf[0] + 1.0f) / 2.0f;
                float thr = nnt * P.f_one_minus_nom_pt + P.f_nom_pt;
                float tg = (float)(T_full * (R)P.n_eng) * thr;
                float md = P.f_Te_over_vex * (tg / (float)T_full);
                cfp = (R)tg + acs_par; mdot_dt = (R)(md * P.f_dt_pt); md_info = (R)md; thr_info = (R)thr;
            }
            cfperp = R(0); cm = R(0);
        } else {
            // force_moment_decomposer_landing_burn_gimballed (:168-269)
            R gdeg_cmd, tpar, tperp, tmz, cmd_l, cmd_r, md, thr;
            R gd;
            if (a.act_f64) {
                R grad = (R)ud[0] * P.max_gimbal_rad;
                gdeg_cmd = grad * Cst<R>::rad2deg;
                gd = gprev + dt_act * ((-gprev + gdeg_cmd) / R(1));
                gd = gd < -P.max_gimbal_deg ? -P.max_gimbal_deg : gd;
                gd = gd > P.max_gimbal_deg ? P.max_gimbal_deg : gd;
                R grad2 = gd * Cst<R>::deg2rad;
                R nnt = ((R)ud[1] + R(1)) / R(2);
                thr = nnt * P.one_minus_nom_lb + P.nom_lb;
                R tg = T_full * (R)(P.n_eng + 2) * thr;
                R cg, sg;
                pd_sincos<R>(grad2, sg, cg);
                tpar = tg * cg; tperp = -tg * sg; tmz = -tg * sg * d_thrust;
                R tot = sqrt(tpar * tpar + tperp * tperp);
                md = P.Te_over_vex * (tot / T_full);
                gdeg_out = grad2 * Cst<R>::rad2deg;
                cmd_l = (R)ud[2] * P.max_defl_rad * R(60); cmd_r = (R)ud[3] * P.max_defl_rad * R(60);
                mdot_dt = md * dt;
            } else {
                float grad = uf[0] * P.f_max_gimbal_rad;
                gdeg_cmd = (R)grad * Cst<R>::rad2deg;
                gd = gprev + dt_act * ((-gprev + gdeg_cmd) / R(1));
                gd = gd < -P.max_gimbal_deg ? -P.max_gimbal_deg : gd;
                gd = gd > P.max_gimbal_deg ? P.max_gimbal_deg : gd;
                R grad2 = gd * Cst<R>::deg2rad;
                float nnt = (uf[1] + 1.0f) / 2.0f;
                float thrf = nnt * P.f_one_minus_nom_lb + P.f_nom_lb;
                float tg = (float)(T_full * (R)(P.n_eng + 2)) * thrf;
                float cg = (float)cos(grad2), sg = (float)sin(grad2);
                float fpar = tg * cg, fperp = (-tg) * sg, fm = (-tg) * sg;
                float tot = sqrtf(fpar * fpar + fperp * fperp);
                float mdf = P.f_Te_over_vex * (tot / (float)T_full);
                tpar = (R)fpar; tperp = (R)fperp; tmz = (R)fm * d_thrust;   // d_thrust_cg is float64
                md = (R)mdf; thr = (R)thrf;
                gdeg_out = grad2 * Cst<R>::rad2deg;
                float dlf = uf[2] * P.f_max_defl_rad, drf = uf[3] * P.f_max_defl_rad;
                cmd_l = (R)(dlf * 60.0f); cmd_r = (R)(drf * 60.0f);
                mdot_dt = (R)(mdf * P.f_dt_lb);
            }
            // ACS (acs_model.py:13-87)
            R dcl = cmd_l * Cst<R>::deg2rad, dcr = cmd_r * Cst<R>::deg2rad;
            R dl = dlprev + dt_act * ((-dlprev + dcl) / R(0.5));
            R dr = drprev + dt_act * ((-drprev + dcr) / R(0.5));
            R cna = grid_fin_cn_alpha<R>(P, lds + L::kCnX, lds + L::kCnY, mach);
            R CnL = cna * ((ae - dl) * Cst<R>::rad2deg);
            R CnR = cna * ((ae - dr) * Cst<R>::rad2deg);
            R cl_, cr_, sl_, sr_;
            pd_sincos<R>(dl, sl_, cl_);
            pd_sincos<R>(dr, sr_, cr_);
            R f_perp = qS * (CnR * cr_ - CnL * cl_ - Ca * (sl_ - sr_));
            R f_par = qS * (Ca * (R(2) + cl_ + cr_) - CnL * sl_ + CnR * sr_);
            R m_z = -(P.d_base_gf - x_cog) * f_perp + P.R_rocket * qS * (Ca * (sr_ - sl_) - CnL * cl_ + CnR * cr_);
            cfp = tpar + f_par; cfperp = tperp + f_perp; cm = tmz + m_z;
            dcmdl_out = dcl; dcmdr_out = dcr;
            md_info = md; thr_info = thr;
        }
        // NaN guard (rockets_physics.py:599-607), an elif chain
        if (isnan(cfp)) { cfp = R(0); nan_hit = true; }
        else if (isnan(cfperp)) { cfperp = R(0); nan_hit = true; }
        else if (isnan(cm)) { cm = R(0); nan_hit = true; }
        R gr = gravity<R>(P, y);
        R fx, fy;
        if (PHASE == 2 && f32_forces) {
            // float32 control forces join the Python-float aero terms in binary32; with wind on
            // F_wind_x is a numpy float64 (interp1d output) and promotes the last sum
            if (isnan(cfp_f)) cfp_f = 0.f;
            else if (isnan(cfperp_f)) cfperp_f = 0.f;
            float c = (float)cth, sn = (float)sth;
            float cx = cfp_f * c + cfperp_f * sn, cy = cfp_f * sn - cfperp_f * c;
            float sx = (float)aero_x + cx, sy = (float)aero_y + cy;
            fx = WIND ? (R)sx + Fwx : (R)(sx + (float)Fwx);
            fy = (R)(sy + (float)Fwy);
        } else {
            R cfx = cfp * cth + cfperp * sth;
            R cfy = cfp * sth - cfperp * cth;
            fx = aero_x + cfx + Fwx; fy = aero_y + cfy + Fwy;
        }
        R vxd = fx / m, vyd = fy / m - gr;
        vx += vxd * dt; vy += vyd * dt; x += vx * dt; y += vy * dt;
        R thdd = (cm + aero_m + Mw) / I;
        thd += thdd * dt; th += thd * dt;
        ga = atan2(vy, vx);
        if (th > Cst<R>::two_pi) th -= Cst<R>::two_pi;
        if (ga < R(0)) ga = Cst<R>::two_pi + ga;
        al = th - ga;
        mp -= mdot_dt; m -= mdot_dt;
        s[0] = x; s[1] = y; s[2] = vx; s[3] = vy; s[4] = th; s[5] = thd; s[6] = ga; s[7] = al;
        s[8] = m; s[9] = mp; s[10] = s[10] + dt;
        PD_T(t_subend);
        PD_ACC(4, t_subend - t_aero1);
        if (sub == NSUB - 1 && a.info && role == 0 && live) {   // info of the last sub-step (rockets_physics.py:649-702)
            R vals[PD_N_INFO - 1] = {rho, patm, asnd, mach, q, CL, CD, md_info, x_cog, I, ae, thr_info, ug, vg, gdeg_out};
#pragma unroll
            for (int k = 0; k < PD_N_INFO - 1; ++k) ev(a.info + ((k < PD_INFO_GLOAD ? k : k + 1)) * N, ui) = vals[k];
        }
    }
    if (nan_hit && role == 0 && live) atomicAdd(&a.pend.stats[1], 1ull);
    PD_T(t_loop);

    // ---- g-load window (base_environment.py:136-149): ring of 10, Python sum() from the oldest
    const DevParams<R>& P2 = *launder(a.P);
    R v = sqrt(s[2] * s[2] + s[3] * s[3]);
    R vp = ldv(a.b.vprev, ui);
    R gl_new = fabs(v - vp) / R(0.1) * R(1) / R(9.81);
    int glen = ldv(a.b.glen, ui), ghead = ldv(a.b.ghead, ui);
    int wslot;
    if (glen < 10) { wslot = glen; glen += 1; }
    else { wslot = ghead; ghead = ghead == 9 ? 0 : ghead + 1; }
    // the window's slots in summation order (oldest first); their addresses are known up front,
    // so the (at most 9) loads are issued together instead of one round trip per term
    const int gstart = glen < 10 ? 0 : ghead;
    R gv[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        int p = gstart + k;
        p = p >= 10 ? p - 10 : p;
        gv[k] = (k < glen && p != wslot) ? ldv(a.b.gwin + (p) * N, ui) : gl_new;
    }
    R gsum = R(0);
#pragma unroll
    for (int k = 0; k < 10; ++k)
        if (k < glen) gsum += gv[k];
    R gl = gsum / R(10);

    // ---- truncated -> done -> reward (rtd_rl.py:190-336 / rtd_pso.py:172-317)
    R x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], ga = s[6], mp = s[9];
    R rho, pa_, as_;
    atmosphere<R>(P2, y, rho, pa_, as_);
    R speed = v;
    R q = R(0.5) * rho * (speed * speed);
    int tr = 0, id = 0, dn = 0;
    R rew = R(0);
    const R r2 = (R)(2.0 * kDeg2Rad);
    if constexpr (RTD == 0 && PHASE != 2) {
        // landing burns: truncated/done shared by both RL flavours (rtd_rl.py:194-240)
        if (y < R(-10)) { tr = 1; id = 1; }
        else if (mp <= R(0)) { tr = 1; id = 2; }
        else if (th > Cst<R>::pi + r2) { tr = 1; id = 3; }
        else if (q > R(65000)) { tr = 1; id = 4; }
        else if (gl > R(6)) { tr = 1; id = 5; }
        else if (vy > R(0)) { tr = 1; id = 6; }
        else if (vx > R(0.01)) { tr = 1; id = 7; }
        dn = (y > R(0) && y < R(1) && speed < R(5));
        if constexpr (PHASE == 0) {   // pure-throttle reward (rtd_rl.py:272-336)
            R sp = hypot(vx, vy);
            R qr = R(0.5) * rho * (sp * sp);
            if (qr > R(60000)) { R e = (qr - R(60000)) / (R(65000) - R(60000)); R e2 = e * e; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            if (gl > R(5.5)) { R e = (gl - R(5.5)) / (R(6) - R(5.5)); R e2 = e * e; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            R prog = (P2.y0_rl - y) / P2.y0_rl;
            R wp = (qr <= R(60000) && gl <= R(5.5)) ? R(0.5) : R(0.5) * R(0.1);
            rew += wp * prog;
            if (y < R(100)) rew += R(5.5) * (R(1) - fabs(vy) / R(50));
            if (dn && !tr) rew += R(400) * mp / P2.m0_rl;
            else if (tr && y > R(0)) rew -= R(50) * (fabs(y) / P2.y0_rl);
            else if (tr && y < R(0)) rew -= R(50) * (fabs(vy) / R(10));
            if (!dn || !(tr && y < R(0))) rew = rew < R(-10) ? R(-10) : (rew > R(10) ? R(10) : rew);
        } else {                      // landing_burn / ACS reward (rtd_rl.py:243-269), u0 = actions[0]
            R ae = fabs(ga - th - Cst<R>::pi);
            R lead = R(1.5) - log(R(1) + ae) / P2.log_1p_max_ae;
            R X;
            if (a.act_f64) X = lead - ((R)ud[0] + R(1)) / R(2) * R(0.5);
            else X = (R)((float)lead - ((uf[0] + 1.0f) / 2.0f) * 0.5f);
            rew = X * (R(1) - y / P2.y0_rl) * R(2) / R(3);
            if (y < R(100)) rew += R(1) - tanh((speed - R(15)) / R(15));
            if (tr && y < R(5)) rew += R(1) - tanh((speed - R(5)) / R(5));
            if (dn) rew += R(5);
            rew *= P2.rl_scale;
        }
        if (a.rtd_none) { tr = 0; id = 0; dn = 0; rew = R(0); }
    } else if constexpr (RTD == 0) {
        const int ph = P2.phase;
        if (ph == PD_PHASE_PCONTROL) {
            // compile_rtd_rl_landing_burn_PDcontrol (rtd_rl.py:353-401) + the reward that rebinds
            // the first (:479-531); v_ref = actions[0]
            if (y < R(-10)) { tr = 1; id = 1; }
            else if (mp <= R(0)) { tr = 1; id = 2; }
            else if (th > Cst<R>::pi + r2) { tr = 1; id = 3; }
            else if (q > R(65000)) { tr = 1; id = 4; }
            else if (gl > R(6)) { tr = 1; id = 5; }
            else if (vy > R(0)) { tr = 1; id = 6; }
            dn = (y > R(0) && y < R(5) && speed < R(1));
            R sp = hypot(vx, vy);
            R qr = R(0.5) * rho * (sp * sp);
            if (qr > R(60000)) { R e = (qr - R(60000)) / (R(65000) - R(60000)); R e2 = e * e; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            if (gl > R(5.5)) { R e = (gl - R(5.5)) / (R(6) - R(5.5)); R e2 = e * e; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            R prog = (P2.y0_rl - y) / P2.y0_rl;
            R vt;
            if (a.act_f64) { R t = R(1) - fabs(sp - (R)ud[0]) / R(10); vt = t > R(0) ? t : R(0); }
            else { float t = 1.0f - fabsf((float)sp - uf[0]) / 10.0f; vt = t > 0.f ? (R)t : R(0); }
            R wp = (qr <= R(60000) && gl <= R(5.5)) ? R(0.5) : R(0.5) * R(0.1);
            rew += wp * prog * vt;
            if (y < R(100)) { R t = R(1) - fabs(vy - R(0)) / R(50); rew += R(0.5) * (t > R(0) ? t : R(0)); }
            rew += P2.alive_bonus;
            if (dn && !tr) { rew += R(5); R used = P2.y0_rl * R(0) + (P2.m0_rl - s[8]); R u = R(0.1) * used; rew -= u < R(1) ? u : R(1); }
            else if (tr) { R u = R(4) * (y / P2.y0_rl) * (fabs(vy) / R(100)); rew -= u < R(5) ? u : R(5); }
            rew = rew < R(-10) ? R(-10) : (rew > R(10) ? R(10) : rew);
        } else if (ph == PD_PHASE_BALLISTIC_ARC) {
            // compile_rtd_rl_ballistic_arc_descent (rtd_rl.py:153-188)
            R ae = fabs(ga - th - Cst<R>::pi);
            dn = (q > R(10000) && ae < (R)(3.0 * kDeg2Rad));
            if (q > R(10000 - 2000) && ae > (R)(5.0 * kDeg2Rad)) { tr = 1; id = 1; }
            rew = (Cst<R>::pi - ae) / Cst<R>::pi;
            if (dn) rew += R(3.5);
            rew /= R(100);
        } else if (ph == PD_PHASE_SUBSONIC || ph == PD_PHASE_SUPERSONIC) {
            // compile_rtd_rl_ascent (rtd_rl.py:11-114) over the ascent reference trajectory
            bool nan_ = false;
#pragma unroll
            for (int k = 0; k < 11; ++k) nan_ |= isnan(s[k]);
            if (nan_) { tr = 1; id = 0; }
            else {
                R mach = (speed != R(0) && as_ != R(0)) ? speed / as_ : R(0);
                R mx = hyper_interp<R>(P2, 1, mach), mvy = hyper_interp<R>(P2, 2, mach);
                R mvx = hyper_interp<R>(P2, 3, mach), mal = hyper_interp<R>(P2, 4, mach);
                int n = P2.n_ref;
                R xr = interp1d_ext<R>(P2.ref_y, P2.ref_x, n, y), vxr = interp1d_ext<R>(P2.ref_y, P2.ref_vx, n, y);
                R vyr = interp1d_ext<R>(P2.ref_y, P2.ref_vy, n, y);
                R al = s[7];
                dn = (mp >= R(0) && mach > P2.terminal_mach);
                if (mp <= R(0)) { tr = 1; id = 1; }
                else if (mach > P2.terminal_mach + R(0.09)) { tr = 1; id = 2; }
                else if (fabs(x - xr) > mx) { tr = 1; id = 3; }
                else if (y < R(0)) { tr = 1; id = 4; }
                else if (fabs(al) > mal * Cst<R>::deg2rad) { tr = 1; id = 5; }
                else if (fabs(vx - vxr) > mvx) { tr = 1; id = 6; }
                else if (fabs(vy - vyr) > mvy) { tr = 1; id = 7; }
                if (!(y < R(0))) {
                    R d = vx - vxr; rew += exp(R(-4) * (d * d) / (mvx * mvx)) * hyper_interp<R>(P2, 8, mach);
                    d = vy - vyr; rew += exp(R(-4) * (d * d) / (mvy * mvy)) * hyper_interp<R>(P2, 7, mach);
                    d = x - xr; rew += exp(R(-4) * (d * d) / (mx * mx)) * hyper_interp<R>(P2, 6, mach);
                    d = al * Cst<R>::rad2deg; rew += exp(R(-4) * (d * d) / (mal * mal)) * hyper_interp<R>(P2, 5, mach);
                    if (dn) rew += R(2.5);
                    rew /= R(10000);
                }
            }
        }
        if (a.rtd_none || ph == PD_PHASE_FLIP_OVER) { tr = 0; id = 0; dn = 0; rew = R(0); }
    } else {
        if constexpr (PHASE == 0) {
            if (y < R(0)) { tr = 1; id = 1; }
            else if (mp <= R(0)) { tr = 1; id = 2; }
            else if (th > Cst<R>::pi + r2) { tr = 1; id = 3; }
            else if (q > R(65000)) { tr = 1; id = 4; }
            else if (vy > R(0)) { tr = 1; id = 6; }
            else if (gl > R(6)) { tr = 1; id = 7; }
            dn = (y > R(0) && y < R(1) && speed < R(5.5));
            if (tr && y > R(0)) rew = -fabs(y);
            else if (tr && y < R(0)) rew = R(200) - fabs(speed);
            else if (dn) rew = mp;
        } else {
            R dist = sqrt(x * x + y * y);
            R over;
            if (x < R(0) && y < R(0)) over = sqrt(x * x + y * y);
            else if (x < R(0)) over = -x;
            else if (y < R(0)) over = -y;
            else over = R(0);
            R aeff = (vy < R(0)) ? fabs(ga - th - Cst<R>::pi) : fabs(th - ga);
            if (over > R(0.5)) { tr = 1; id = 1; }
            else if (mp <= R(0)) { tr = 1; id = 2; }
            else if (aeff > (R)(10.0 * kDeg2Rad)) { tr = 1; id = 3; }
            else if (q > R(65000)) { tr = 1; id = 4; }
            else if (vy > R(0)) { tr = 1; id = 6; }
            else if (gl > R(6)) { tr = 1; id = 7; }
            else if (y > R(1000) && vx > R(0)) { tr = 1; id = 8; }
            dn = (dist > R(0) && dist < R(1) && speed < R(2.5));
            if (tr && over < R(0.5)) rew = -fabs(dist);
            else if (tr) rew = R(200) - fabs(speed);
            else if (dn) rew = mp;
        }
    }

    PD_T(t_rtd);
    PD_ACC(5, t_rtd - t_loop);
    // ---- outputs (role 0 of the env's lane group)
    // fresh copy of the offset: the store addresses are recomputed here from the SGPR bases
    // instead of keeping the load addresses live (spilled) across the sub-step loop
    uint32_t ui_out = ui;
    asm volatile("" : "+v"(ui_out));
    const bool ended = !POL && a.auto_reset && (dn || tr);
    if (role == 0 && live) {
        if (a.obs) {
            // the wrappers' observation (obs_write kinds); compile-time for the landing burns
            constexpr int kind = RTD == 1 ? (PHASE == 0 ? 1 : 2) : (PHASE == 0 ? 0 : (PHASE == 1 ? 3 : -1));
            const int ok = kind >= 0 ? kind : P2.obs_kind;
            obs_write<R>(P2, ok, s, a.obs + fo * obs_dim(ok), ui_out);
        }
        if (a.reward) stv(a.reward + fo, ui_out) = rew;
        if constexpr (POL) {
            // objective_function: episode_reward -= reward until done or truncated (env_wrapped_ea.py:200-222)
            ev(a.reward_sum, ui_out) -= rew;
            if (dn || tr) stv(a.b.fin, ui_out) = 1;
        } else if (a.reward_sum) {
            ev(a.reward_sum, ui_out) += rew;
        }
        if (a.done) stv(a.done + fo, ui_out) = (uint8_t)dn;
        if (a.trunc) stv(a.trunc + fo, ui_out) = (uint8_t)tr;
        if (a.trunc_id) stv(a.trunc_id + fo, ui_out) = (int8_t)id;
        if (a.info) stv(a.info + (PD_INFO_GLOAD) * N, ui_out) = gl;
        if (ended) {
            reset_env(a, i, ep + 1, false);
        } else {
            stv(a.b.vprev, ui_out) = v;
            stv(a.b.gwin + (wslot) * N, ui_out) = gl_new;
            stv(a.b.glen, ui_out) = (uint8_t)glen; stv(a.b.ghead, ui_out) = (uint8_t)ghead;
            stv(a.b.tid, ui_out) = (int8_t)id;
            stv(a.b.tstep, ui_out) = ts + 1;
            if constexpr (PHASE == 1) { stv(a.b.act, ui_out) = gdeg_out; stv(a.b.act + N, ui_out) = dcmdl_out; stv(a.b.act + (2) * N, ui_out) = dcmdr_out; }
            if constexpr (PHASE == 2) { if (aux == PD_PHASE_FLIP_OVER) stv(a.b.act, ui_out) = gdeg_out; }
            if constexpr (WIND) {
                stv(a.b.wind, ui_out) = fu0; stv(a.b.wind + N, ui_out) = fu1; stv(a.b.wind + (2) * N, ui_out) = fv0; stv(a.b.wind + (3) * N, ui_out) = fv1;
            }
        }
    }
    if constexpr (POL) {
        // done-mask compaction: the envs whose episode goes on, in lane order, appended to the
        // next launch's list at a base taken by one atomic per wave (the count also tells the
        // host when every episode has ended)
        const bool cont = role == 0 && live && !(dn || tr);
        const unsigned long long m = __ballot(cont);
        if (m) {
            const int lane = (int)__lane_id();
            const int leader = __ffsll((long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.cnt_out, (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, leader);
            if (cont) a.list_out[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (int32_t)i;
        }
    }
    // neighbourhood caches survive resets (any valid 50-set is a correct start)
    if (part == 0 && live) {
        stv(a.b.key + (my_table) * N, ui_out) = cA.key; stv(a.b.slot + (my_table) * N, ui_out) = cA.slot;
        if constexpr (LPE == 1) { stv(a.b.key + N, ui_out) = cB.key; stv(a.b.slot + N, ui_out) = cB.slot; }
    }
    if (!ended && live) {
#pragma unroll
        for (int k = 0; k < 11; ++k)
            if (k % LPE == role) stv(a.b.st + (k) * N, ui_out) = s[k];
    }
    }   // fused steps
#ifdef PD_STAMP
    PD_T(t_end);
    PD_ACC(6, t_end - t_rtd);
    if (__lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 7; ++k) atomicAdd(&a.pend.stats[8 + k], acc_[k]);
        atomicAdd(&a.pend.stats[15], 1ull);
    }
#endif
}

// Insert the neighbourhoods solved on device during the last launch (single block; the only
// writer of the tables, stream-ordered between step launches, so readers never race it).
template <typename R>
__global__ void k_insert(Pending pend, unsigned long long* keys_cd, R* pay_cd, int lc_cd,
                         unsigned long long* keys_cl, R* pay_cl, int lc_cl) {
    __shared__ int s_slot;
    unsigned long long cnt = *pend.count;
    if (cnt == 0) return;
    if (cnt > (unsigned long long)kPendingCap) cnt = kPendingCap;
    for (unsigned long long e = 0; e < cnt; ++e) {
        if (threadIdx.x == 0) {
            unsigned long long kk = pend.keys[e];
            int table = (int)(kk >> 63);
            unsigned long long key = kk & ~(1ull << 63);
            unsigned long long* keys = table ? keys_cl : keys_cd;
            int lc = table ? lc_cl : lc_cd;
            uint32_t mask = (1u << lc) - 1u, h = key_hash(key, lc);
            int slot = -1;
            uint32_t used = 0;
            for (uint32_t p = 0; p <= mask; ++p) {
                unsigned long long k = keys[h];
                if (k == key) { slot = -1; break; }
                if (k == kEmptyKey) { slot = (int)h; break; }
                h = (h + 1) & mask; ++used;
            }
            // keep the load factor <= 1/2
            if (slot >= 0 && pend.stats[2 + table] * 2 + 2 > (1ull << lc)) slot = -1;
            if (slot >= 0) { pend.stats[2 + table] += 1; }
            s_slot = slot >= 0 ? (slot | (table << 30)) : -1;
            if (slot >= 0) keys[slot] = key;
        }
        __syncthreads();
        int sl = s_slot;
        if (sl >= 0) {
            int table = sl >> 30, slot = sl & ((1 << 30) - 1);
            R* pay = (table ? pay_cl : pay_cd) + (int64_t)slot * pay_stride<R>();
            if (threadIdx.x == 0) pay_store<R>(pend.pay + e * kPay, pay);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *pend.count = 0;
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_observe(StepArgs<R> a, int obs_kind) {
    const DevParams<R>& P = *a.P;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t N = a.n;
    if (i >= N) return;
    R s[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) s[k] = a.b.st[k * N + i];
    obs_write<R>(P, obs_kind, s, a.obs, (uint32_t)i);
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_set_sigmas(StepArgs<R> a, const double* sig) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    a.b.wind[4 * a.n + i] = (R)sig[i];
    a.b.wind[5 * a.n + i] = (R)sig[a.n + i];
}

// ---------------------------------------------------------------- host side
int log2ceil(int64_t v) { int l = 0; while ((1ll << l) < v) ++l; return l; }

template <typename R> struct Table {
    int logcap = 0;
    std::vector<unsigned long long> keys;
    std::vector<R> pay;
    int64_t entries = 0;
};

// brute-force 50-NN key at a query (host), used for the initial cache and key checks
uint64_t host_knn_key(const pd_aero_table& t, double M, double a) {
    std::vector<std::pair<double, int>> d;
    for (int c = 0; c < t.n_cols; ++c)
        for (int k = 0; k < t.col_len[c]; ++k) {
            double dm = M - t.mach[t.col_start[c] + k], da = a - t.col_aoa[c];
            d.push_back({dm * dm + da * da, t.col_start[c] + k});
        }
    std::stable_sort(d.begin(), d.end(), [](auto& x, auto& y) { return x.first < y.first; });
    int lo[kCols], hi[kCols];
    for (int c = 0; c < kCols; ++c) { lo[c] = 1 << 20; hi[c] = -1; }
    for (int j = 0; j < kNbr; ++j) {
        int p = d[j].second, c = 0;
        while (c + 1 < t.n_cols && p >= t.col_start[c + 1]) ++c;
        int k = p - t.col_start[c];
        lo[c] = std::min(lo[c], k); hi[c] = std::max(hi[c], k);
    }
    int L[kCols], N[kCols];
    for (int c = 0; c < kCols; ++c) {
        if (hi[c] < 0) { L[c] = 0; N[c] = 0; } else { L[c] = lo[c]; N[c] = hi[c] - lo[c] + 1; }
    }
    return key_pack(L, N);
}

template <typename R>
int table_insert(const pd_aero_table& t, Table<R>& T, uint64_t key, std::vector<double>& work, std::vector<double>& pay) {
    int64_t cap = 1ll << T.logcap;
    uint32_t mask = (uint32_t)(cap - 1), h = key_hash(key, T.logcap);
    while (T.keys[h] != kEmptyKey && T.keys[h] != key) h = (h + 1) & mask;
    if (T.keys[h] == key) return (int)h;
    double aoa[kCols];
    for (int c = 0; c < kCols; ++c) aoa[c] = t.col_aoa[c];
    if (solve_neighbourhood(t.mach, t.coef, t.col_start, aoa, key, work.data(), pay.data()) != 0) return -1;
    if ((T.entries + 1) * 2 > cap) return -1;
    T.keys[h] = key;
    pay_store<R>(pay.data(), T.pay.data() + h * pay_stride<R>());
    ++T.entries;
    return (int)h;
}

template <typename R>
pd_status build_table(const pd_aero_table& t, const uint64_t* keys, int64_t nk, Table<R>& T) {
    int64_t cap_need = std::max<int64_t>(4 * std::max<int64_t>(nk, 64), 1024);
    T.logcap = log2ceil(cap_need);
    int64_t cap = 1ll << T.logcap;
    T.keys.assign(cap, kEmptyKey);
    T.pay.assign(cap * pay_stride<R>(), R(0));
    std::vector<double> work(kScratch), pay(kPay);
    for (int64_t e = 0; e < nk; ++e)
        if (table_insert<R>(t, T, keys[e], work, pay) < 0)
            return fail(PD_ERR_INVALID, "invalid/singular neighbourhood key in param pack");
    return PD_OK;
}

// Exact neighbourhood intervals along one horizontal query line a = const: the 50-NN set only
// changes where two points swap distance order, i.e. at pair-bisector crossings; evaluate the
// set between consecutive crossings and merge equal neighbours.  (The device still verifies
// every looked-up set, so a query exactly on a breakpoint stays exact.)
template <typename R>
pd_status build_line(const pd_aero_table& t, double a, Table<R>& T, int li, DevParams<R>& D) {
    std::vector<double> m(t.n_pts), dz(t.n_pts);
    for (int c = 0; c < kCols; ++c)
        for (int k = 0; k < t.col_len[c]; ++k) {
            m[t.col_start[c] + k] = t.mach[t.col_start[c] + k];
            double da = a - t.col_aoa[c];
            dz[t.col_start[c] + k] = da * da;
        }
    std::vector<double> xs;
    for (int i = 0; i < t.n_pts; ++i)
        for (int j = i + 1; j < t.n_pts; ++j) {
            double den = 2.0 * (m[j] - m[i]);
            if (den == 0.0) continue;
            double x = (m[j] * m[j] - m[i] * m[i] + dz[j] - dz[i]) / den;
            if (x > 0.0 && x < 10.0) xs.push_back(x);
        }
    std::sort(xs.begin(), xs.end());
    xs.erase(std::unique(xs.begin(), xs.end()), xs.end());
    std::vector<double> bps;
    bps.push_back(0.0);
    bps.insert(bps.end(), xs.begin(), xs.end());
    bps.push_back(10.0);
    std::vector<double> B;
    std::vector<uint64_t> K;
    for (size_t k = 0; k + 1 < bps.size(); ++k) {
        uint64_t key = host_knn_key(t, 0.5 * (bps[k] + bps[k + 1]), a);
        if (K.empty()) K.push_back(key);
        else if (key != K.back()) { B.push_back(bps[k]); K.push_back(key); }
    }
    D.line_a[li] = (R)a;
    if ((int)B.size() > kLineMax) { D.line_nbp[li] = -1; return PD_OK; }   // too fine: cache path only
    std::vector<double> work(kScratch), pay(kPay);
    D.line_nbp[li] = (int)B.size();
    for (size_t k = 0; k < B.size(); ++k) D.line_bp[li][k] = (R)B[k];
    for (size_t k = 0; k < K.size(); ++k) {
        D.line_key[li][k] = K[k];
        D.line_slot[li][k] = table_insert<R>(t, T, K[k], work, pay);
    }
    return PD_OK;
}

// Candidate grid over the interior query domain [0, 10] Mach x [a0, a1]: the 50-NN key at
// every cell centre (brute force), inserted into the table.  A 50-NN region is an intersection
// of half-planes (order-k Voronoi cell), hence convex: when all four corners of a cell carry
// the centre's key, the whole cell does, and the slot is flagged kGridExact so that device
// lookups skip the verification.  Other cells' keys are candidates the device verifies.
template <typename R>
pd_status build_grid(const pd_aero_table& t, double a0, double a1, int nm, int na, Table<R>& T,
                     std::vector<unsigned long long>& gk, std::vector<int>& gs) {
    gk.assign((size_t)nm * na, 0); gs.assign((size_t)nm * na, -1);
    std::vector<double> work(kScratch), pay(kPay);
    double dm = 10.0 / nm, da = (a1 - a0) / na;
    std::vector<uint64_t> corner((size_t)(nm + 1) * (na + 1));
    for (int im = 0; im <= nm; ++im)
        for (int ia = 0; ia <= na; ++ia)
            corner[(size_t)im * (na + 1) + ia] = host_knn_key(t, im * dm, a0 + ia * da);
    for (int im = 0; im < nm; ++im)
        for (int ia = 0; ia < na; ++ia) {
            uint64_t key = host_knn_key(t, (im + 0.5) * dm, a0 + (ia + 0.5) * da);
            gk[(size_t)im * na + ia] = key;
            int slot = table_insert<R>(t, T, key, work, pay);
            bool exact = slot >= 0;
            for (int c = 0; c < 4 && exact; ++c)
                exact = corner[(size_t)(im + (c >> 1)) * (na + 1) + ia + (c & 1)] == key;
            gs[(size_t)im * na + ia] = slot < 0 ? -1 : (slot | (exact ? kGridExact : 0));
        }
    return PD_OK;
}

}  // namespace

// ---------------------------------------------------------------- the handle
struct pd_env {
    pd_config cfg{};
    int device = 0;
    int obs_dim = 2, act_dim = 1;
    size_t rsize = 8;
    void* dparams = nullptr;
    std::vector<void*> allocs;
    // per-env buffers (typed views in the precision of the handle)
    void* st = nullptr; void* vprev = nullptr; void* gwin = nullptr; void* act = nullptr; void* wind = nullptr;
    uint8_t *ghead = nullptr, *glen = nullptr, *wprof = nullptr;
    unsigned long long* key = nullptr; int* slot = nullptr;
    int8_t* tid = nullptr; uint32_t *epi = nullptr, *tstep = nullptr;
    uint8_t* fin = nullptr;
    int32_t* live[2] = {nullptr, nullptr};   // policy rollouts: compacted live-env lists
    uint32_t* live_cnt = nullptr;            // [3] their lengths (triple-buffered)
    uint32_t* host_cnt = nullptr;            // [2] pinned host copies of checked lengths
    hipEvent_t cnt_ev[2] = {nullptr, nullptr};
    Pending pend{};
    unsigned long long *keys_cd = nullptr, *keys_cl = nullptr;
    void *pay_cd = nullptr, *pay_cl = nullptr;
    int logcap_cd = 0, logcap_cl = 0;
    int64_t entries_cd = 0, entries_cl = 0;
    int lpe = 2;   // lanes per env of the step kernel
    int obs_kind = 0;   // obs_write layout of the handle's observation
};

namespace {
// observation layout (obs_write) and widths of a (phase, rtd) pair
int obs_kind_of(int phase, int rtd) {
    if (rtd == PD_RTD_PSO) return phase == PD_PHASE_PURE_THROTTLE ? 1 : 2;
    switch (phase) {
        case PD_PHASE_PURE_THROTTLE: return 0;
        case PD_PHASE_LANDING_BURN: return 3;
        case PD_PHASE_PCONTROL: return 4;
        case PD_PHASE_BALLISTIC_ARC: return 5;
        case PD_PHASE_FLIP_OVER: return 6;
        default: return 7;
    }
}
int act_dim_of(int phase) {
    return phase == PD_PHASE_LANDING_BURN ? 4 : ((phase == PD_PHASE_SUBSONIC || phase == PD_PHASE_SUPERSONIC) ? 2 : 1);
}
}  // namespace

namespace {

pd_status dalloc(pd_env* e, void** p, size_t bytes) {
    if (bytes == 0) bytes = 8;
    PD_HIP(hipMalloc(p, bytes));
    e->allocs.push_back(*p);
    return PD_OK;
}

template <typename R> StepArgs<R> make_args(pd_env* e) {
    StepArgs<R> a{};
    a.P = (const DevParams<R>*)e->dparams;
    a.b.st = (R*)e->st; a.b.vprev = (R*)e->vprev; a.b.gwin = (R*)e->gwin; a.b.ghead = e->ghead; a.b.glen = e->glen;
    a.b.act = (R*)e->act; a.b.wind = (R*)e->wind; a.b.wprof = e->wprof; a.b.key = e->key; a.b.slot = e->slot;
    a.b.tid = e->tid; a.b.epi = e->epi; a.b.tstep = e->tstep; a.b.fin = e->fin;
    a.pend = e->pend;
    a.n = e->cfg.n_envs;
    a.env_offset = e->cfg.env_offset;
    a.seed_lo = (uint32_t)e->cfg.seed; a.seed_hi = (uint32_t)(e->cfg.seed >> 32);
    a.act_f64 = e->cfg.action_f64;
    a.auto_reset = e->cfg.auto_reset;
    a.stochastic = e->cfg.stochastic_wind;
    a.fixed_prof = e->cfg.wind_percentile >= 50 ? e->cfg.wind_percentile - 50 : -1;
    a.use_tilt = e->cfg.tilt_sigma_rad > 0.0;
    a.tilt_sigma = e->cfg.tilt_sigma_rad;
    a.dt_aux = e->cfg.dt > 0.0 ? e->cfg.dt : 0.1;
    a.rtd_none = e->cfg.rtd == PD_RTD_NONE;
    a.n_fused = 1;
    return a;
}

template <typename R> void fill_params(const pd_params* p, const pd_config* c, DevParams<R>& D) {
    std::memset(&D, 0, sizeof(D));
    D.T_e = (R)p->thrust_per_engine; D.p_e = (R)p->nozzle_exit_pressure; D.A_e = (R)p->nozzle_exit_area;
    D.v_ex = (R)p->v_exhaust; D.S_gf = (R)p->grid_fin_area; D.d_base_gf = (R)p->d_base_grid_fin;
    D.R_rocket = (R)p->rocket_radius; D.A_front = (R)p->frontal_area; D.m_prop0 = (R)p->m_prop0;
    D.C_gust_x = (R)p->C_gust_x; D.C_gust_y = (R)p->C_gust_y; D.n_eng = p->n_engines_gimballed;
    // compile_physics constants (rockets_physics.py:808-835, 914-916), in binary64 as Python does
    double nom_pt = (0 * 0.4) / (double)p->n_engines_gimballed;
    double nom_lb = (3 * 0.4) / (double)p->n_engines_gimballed;
    double te_vex = p->thrust_per_engine / p->v_exhaust;
    double mg = 5.0 * kDeg2Rad, md = 20.0 * kDeg2Rad;
    D.f_Te_over_vex = (float)te_vex; D.f_one_minus_nom_pt = (float)(1 - nom_pt); D.f_nom_pt = (float)nom_pt;
    D.f_one_minus_nom_lb = (float)(1 - nom_lb); D.f_nom_lb = (float)nom_lb; D.f_dt_pt = (float)0.025;
    D.f_dt_lb = (float)0.1; D.f_max_gimbal_rad = (float)mg; D.f_max_defl_rad = (float)md;
    D.Te_over_vex = (R)te_vex; D.one_minus_nom_pt = (R)(1 - nom_pt); D.nom_pt = (R)nom_pt;
    D.one_minus_nom_lb = (R)(1 - nom_lb); D.nom_lb = (R)nom_lb; D.max_gimbal_rad = (R)mg;
    D.max_gimbal_deg = (R)(mg * kRad2Deg); D.max_defl_rad = (R)md;
    D.h_ox = (R)p->h_ox; D.h_f = (R)p->h_f; D.m_ox = (R)p->m_ox; D.m_f = (R)p->m_f; D.h_lower = (R)p->h_lower;
    D.m_dry = (R)p->m_dry; D.x_dry = (R)p->x_dry; D.I_dry = (R)p->I_dry; D.engine_height = (R)p->engine_height;
    D.cop = (R)p->cop;
    for (int k = 0; k < 9; ++k) {
        double b = p->isa_beta[k], Tb = p->isa_Tb[k];
        D.isa_Hb[k] = (R)p->isa_Hb[k]; D.isa_Tb[k] = (R)Tb; D.isa_beta[k] = (R)b; D.isa_pb[k] = (R)p->isa_pb[k];
        D.isa_bt[k] = (R)(b / Tb);
        D.isa_ex[k] = (R)(b != 0.0 ? -p->isa_g0 / (b * p->isa_R) : 0.0);
        D.isa_iso[k] = (R)(-p->isa_g0 / (p->isa_R * Tb));
    }
    D.isa_r = (R)p->isa_r; D.isa_R = (R)p->isa_R; D.isa_kappaR = (R)(p->isa_kappa * p->isa_R);
    D.isa_alt_max = (R)p->isa_alt_max; D.grav_R = (R)p->grav_R; D.grav_g0 = (R)p->grav_g0;
    for (int cc = 0; cc < kCols; ++cc) {
        D.cd_start[cc] = p->cd.col_start[cc]; D.cd_len[cc] = p->cd.col_len[cc]; D.cd_aoa[cc] = (R)p->cd.col_aoa[cc];
        D.cl_start[cc] = p->cl.col_start[cc]; D.cl_len[cc] = p->cl.col_len[cc]; D.cl_aoa[cc] = (R)p->cl.col_aoa[cc];
        D.cd_aoa_d[cc] = p->cd.col_aoa[cc]; D.cl_aoa_d[cc] = p->cl.col_aoa[cc];
    }
    D.cd_n = p->cd.n_pts; D.cl_n = p->cl.n_pts;
    for (int cc = 0; cc < kCols; ++cc) {
        for (int k = 0; k < p->cd.col_len[cc]; ++k) D.cd_pt_aoa[p->cd.col_start[cc] + k] = (R)p->cd.col_aoa[cc];
        for (int k = 0; k < p->cl.col_len[cc]; ++k) D.cl_pt_aoa[p->cl.col_start[cc] + k] = (R)p->cl.col_aoa[cc];
    }
    for (int k = 0; k < 256; ++k) {
        D.cd_mach[k] = (R)p->cd.mach[k]; D.cl_mach[k] = (R)p->cl.mach[k];
        D.cd_mach_d[k] = p->cd.mach[k]; D.cl_mach_d[k] = p->cl.mach[k];
        D.cd_coef_d[k] = p->cd.coef[k]; D.cl_coef_d[k] = p->cl.coef[k];
    }
    D.ca_n = p->ca_n; D.cn_n = p->cn_n;
    for (int k = 0; k < 64; ++k) {
        D.ca_x[k] = (R)p->ca_x[k]; D.ca_y[k] = (R)p->ca_y[k]; D.cn_x[k] = (R)p->cn_x[k]; D.cn_y[k] = (R)p->cn_y[k];
    }
    D.ca_min_mach = (R)p->ca_min_mach; D.ca_min_val = (R)p->ca_min_val;
    D.cn_min_mach = (R)p->cn_min_mach; D.cn_max_mach = (R)p->cn_max_mach; D.cn_min_val = (R)p->cn_min_val;
    D.cn_max_val = (R)p->cn_max_val; D.cn_slope = (R)p->cn_slope;
    for (int w = 0; w < 50; ++w) {
        D.wind_n[w] = p->wind_n[w];
        for (int k = 0; k < 16; ++k) { D.wind_alt_km[w][k] = (R)p->wind_alt_km[w][k]; D.wind_speed[w][k] = (R)p->wind_speed[w][k]; }
    }
    for (int k = 0; k < 4; ++k) { D.vk_Ad_u[k] = (R)p->vk_Ad_u[k]; D.vk_Ad_v[k] = (R)p->vk_Ad_v[k]; }
    for (int k = 0; k < 2; ++k) { D.vk_Bd_u[k] = (R)p->vk_Bd_u[k]; D.vk_Bd_v[k] = (R)p->vk_Bd_v[k]; }
    D.vk_y_threshold = (R)p->vk_y_threshold;
    D.sigma_u_lo = p->sigma_u_lo; D.sigma_u_hi = p->sigma_u_hi; D.sigma_v_lo = p->sigma_v_lo; D.sigma_v_hi = p->sigma_v_hi;
    for (int k = 0; k < 11; ++k) { D.state0[k] = (R)p->state0[k]; D.state0_d[k] = p->state0[k]; }
    D.norm_y = (R)p->norm_y; D.norm_vy = (R)p->norm_vy; D.norm_x = (R)p->norm_x; D.norm_vx = (R)p->norm_vx;
    D.k_theta_pso = (R)(std::atanh(0.75) / (25.0 * kDeg2Rad));
    log_table_fill(D.logtab);
    D.y0_rl = (R)p->state0[1]; D.m0_rl = (R)p->state0[8];
    // ---- phase of the handle: its initial state, observation, and the constants of the
    // other compile_physics phases (rockets_physics.py:17-166,402-451,728-802,959-997)
    D.phase = c->phase;
    D.obs_kind = obs_kind_of(c->phase, c->rtd);
    if (c->phase >= PD_PHASE_PCONTROL)
        for (int k = 0; k < 11; ++k) { D.state0[k] = (R)p->state0_phase[c->phase][k]; D.state0_d[k] = p->state0_phase[c->phase][k]; }
    for (int k = 0; k < 13; ++k) D.fr[k] = (R)p->full_rocket[k];
    D.cop_ascent = (R)p->cop_ascent; D.n_eng_stage1 = p->n_engines_stage1;
    double mg_ascent = 7.0 * kDeg2Rad;
    D.mg_ascent = (R)mg_ascent; D.f_mg_ascent = (float)mg_ascent;
    D.kp_pc = (R)-0.08; D.f_kp_pc = (float)-0.08;
    D.rcs_force = (R)p->rcs_force; D.f_rcs_force = (float)p->rcs_force;
    D.rcs_d_bottom = (R)p->rcs_d_bottom; D.rcs_d_top = (R)p->rcs_d_top;
    // rl_wrapped_env_pytorch.augment_state (env_wrapped_rl_pytorch.py:178-194) constants
    D.f_k_theta_rl = (float)(std::atanh(0.75) / (5.0 * kDeg2Rad));
    D.f_k_thetad_rl = (float)(std::atanh(0.75) / 0.01);
    D.f_k_gamma_rl = (float)(std::atanh(0.75) / (5.0 * kDeg2Rad));
    D.f_pi_2 = (float)(kPi / 2); D.f_pi_3_2 = (float)(3.0 / 2 * kPi);
    for (int k = 0; k < 8; ++k) D.norm_ph[k] = (R)p->norm_phase[c->phase][k];
    int which = c->phase == PD_PHASE_SUPERSONIC ? 1 : 0;
    for (int r = 0; r < 12; ++r) for (int f = 0; f < 9; ++f) D.hyper[r][f] = (R)p->hyper[which][r][f];
    D.terminal_mach = (R)p->terminal_mach[which];
    D.n_ref = p->n_ref;
    // rtd_rl.py:267 (n-step scale, Python float ** int -> C pow), :472 (alive bonus), :250
    double g = c->discount_factor;
    D.rl_scale = (R)((1 - g) / (1 - std::pow(g, (double)c->trajectory_length)));
    D.alive_bonus = (R)(0.01 * (1 - g));
    D.log_1p_max_ae = (R)std::log(1 + 20.0 * kDeg2Rad);
}

pd_status validate(const pd_params* p, const pd_config* c) {
    if (!p || !c) return fail(PD_ERR_INVALID, "null params/config");
    // per-lane byte offsets in k_step are 32-bit (largest per-env row: noise, 64 B)
    if (c->n_envs <= 0 || c->n_envs > (int64_t)1 << 25) return fail(PD_ERR_INVALID, "n_envs out of range (1 .. 2^25 per handle)");
    if (c->phase < 0 || c->phase > PD_PHASE_LANDING_BURN_ACS) return fail(PD_ERR_INVALID, "bad phase");
    if (c->rtd != PD_RTD_RL && c->rtd != PD_RTD_PSO && c->rtd != PD_RTD_NONE) return fail(PD_ERR_INVALID, "bad rtd");
    if (c->phase == PD_PHASE_LANDING_BURN_ACS)
        return fail(PD_ERR_UNSUPPORTED, "landing_burn_ACS: the reference raises TypeError at its first step "
                                        "(rockets_physics.py:867-891 passes ACS arguments to the gimballed decomposer; "
                                        "base_environment.py:126-130 passes two prevs to a three-prev lambda)");
    if (c->rtd == PD_RTD_RL && c->phase == PD_PHASE_FLIP_OVER)
        return fail(PD_ERR_UNSUPPORTED, "flip_over_boostbackburn with rtd RL: the reference raises TypeError at its first "
                                        "step (rtd_rl.py:134 truncated_func(state) called with three arguments, "
                                        "base_environment.py:150); use PD_RTD_NONE for physics stepping");
    if (c->rtd == PD_RTD_PSO && c->phase > PD_PHASE_LANDING_BURN)
        return fail(PD_ERR_UNSUPPORTED, "rtd PSO exists for the two landing burns only: the other rtd_pso functions take "
                                        "(state) / (state, done, truncated) and raise TypeError when the env calls them "
                                        "(rtd_pso.py:38,63,107,120,141,157 vs base_environment.py:150-152)");
    if (c->dt < 0.0) return fail(PD_ERR_INVALID, "dt must be >= 0");
    if (c->rtd == PD_RTD_RL && (c->phase == PD_PHASE_LANDING_BURN || c->phase == PD_PHASE_PCONTROL) &&
        (c->trajectory_length < 1 || !(c->discount_factor > 0.0 && c->discount_factor < 1.0)))
        return fail(PD_ERR_INVALID, "this RL reward needs discount_factor in (0, 1) and trajectory_length >= 1");
    if (c->phase == PD_PHASE_SUBSONIC || c->phase == PD_PHASE_SUPERSONIC) {
        if (!p->ref_y || !p->ref_x || !p->ref_vx || !p->ref_vy || p->n_ref < 2)
            return fail(PD_ERR_INVALID, "ascent phases need the reference trajectory (ref_y/x/vx/vy, n_ref >= 2)");
    }
    if (c->precision != PD_F64 && c->precision != PD_F32) return fail(PD_ERR_INVALID, "bad precision");
    if (c->action_f64 && c->precision != PD_F64) return fail(PD_ERR_INVALID, "f64 actions need PD_F64");
    if (c->enable_wind && !(c->wind_percentile == -1 || (c->wind_percentile >= 50 && c->wind_percentile <= 99)))
        return fail(PD_ERR_INVALID, "wind_percentile must be 50..99 or -1");
    const pd_aero_table* ts[2] = {&p->cd, &p->cl};
    for (auto t : ts) {
        if (t->n_cols != kCols || t->n_pts < kNbr || t->n_pts > PD_MAX_PTS) return fail(PD_ERR_INVALID, "aero table shape");
        int s = 0;
        for (int k = 0; k < kCols; ++k) {
            if (t->col_start[k] != s || t->col_len[k] < 1 || t->col_len[k] >= (1 << kKeyLoBits))
                return fail(PD_ERR_INVALID, "aero column layout");
            s += t->col_len[k];
        }
        if (s != t->n_pts) return fail(PD_ERR_INVALID, "aero column count");
    }
    if (p->ca_n < 2 || p->ca_n > PD_MAX_TAB || p->cn_n < 2 || p->cn_n > PD_MAX_TAB) return fail(PD_ERR_INVALID, "grid fin tables");
    for (int w = 0; w < PD_N_WIND_PROFILES; ++w)
        if (c->enable_wind && (p->wind_n[w] < 1 || p->wind_n[w] > PD_MAX_WIND)) return fail(PD_ERR_INVALID, "wind profile");
    return PD_OK;
}

template <typename R> pd_status create_impl(const pd_params* p, const pd_config* c, pd_env* e) {
    const int64_t N = c->n_envs;
    DevParams<R> D;
    fill_params<R>(p, c, D);
    Table<R> tcd, tcl;
    pd_status st;
    if ((st = build_table<R>(p->cd, p->keys_cd, p->n_keys_cd, tcd)) != PD_OK) return st;
    if ((st = build_table<R>(p->cl, p->keys_cl, p->n_keys_cl, tcl)) != PD_OK) return st;
    // clamped query lines: C_D at +-radians(10) (aerodynamic_coefficients.py:108-114), C_L at
    // +-10 (:122-125); the device computes these abscissae with the same expressions
    if ((st = build_line<R>(p->cd, 10.0 * kDeg2Rad, tcd, 0, D)) != PD_OK) return st;
    if ((st = build_line<R>(p->cd, -10.0 * kDeg2Rad, tcd, 1, D)) != PD_OK) return st;
    if ((st = build_line<R>(p->cl, 10.0, tcl, 2, D)) != PD_OK) return st;
    if ((st = build_line<R>(p->cl, -10.0, tcl, 3, D)) != PD_OK) return st;
    // interior candidate grids: C_D abscissa in [-radians(10), radians(10)], C_L in [0, 10]
    std::vector<unsigned long long> gk[2];
    std::vector<int> gs[2];
    int gnm[2] = {400, 400}, gna[2] = {16, 200};
    if (const char* g = getenv("PDENV_GRID")) {   // experiments: "nm_cd,na_cd,nm_cl,na_cl"
        int v[4];
        if (sscanf(g, "%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3]) == 4 && v[0] > 0 && v[1] > 0 && v[2] > 0 && v[3] > 0) {
            gnm[0] = v[0]; gna[0] = v[1]; gnm[1] = v[2]; gna[1] = v[3];
        }
    }
    const double ga0[2] = {-10.0 * kDeg2Rad, 0.0}, ga1[2] = {10.0 * kDeg2Rad, 10.0};
    if ((st = build_grid<R>(p->cd, ga0[0], ga1[0], gnm[0], gna[0], tcd, gk[0], gs[0])) != PD_OK) return st;
    if ((st = build_grid<R>(p->cl, ga0[1], ga1[1], gnm[1], gna[1], tcl, gk[1], gs[1])) != PD_OK) return st;
    for (int tb = 0; tb < 2; ++tb) {
        void *dk, *ds;
        if ((st = dalloc(e, &dk, gk[tb].size() * 8)) || (st = dalloc(e, &ds, gs[tb].size() * 4))) return st;
        PD_HIP(hipMemcpy(dk, gk[tb].data(), gk[tb].size() * 8, hipMemcpyHostToDevice));
        PD_HIP(hipMemcpy(ds, gs[tb].data(), gs[tb].size() * 4, hipMemcpyHostToDevice));
        D.grid_key[tb] = (const unsigned long long*)dk; D.grid_slot[tb] = (const int*)ds;
        D.grid_nm[tb] = gnm[tb]; D.grid_na[tb] = gna[tb]; D.grid_a0[tb] = (R)ga0[tb];
        D.grid_inv_da[tb] = (R)(gna[tb] / (ga1[tb] - ga0[tb])); D.grid_inv_dm[tb] = (R)(gnm[tb] / 10.0);
    }
    e->logcap_cd = tcd.logcap; e->logcap_cl = tcl.logcap;
    e->entries_cd = tcd.entries; e->entries_cl = tcl.entries;
    if ((st = dalloc(e, (void**)&e->keys_cd, tcd.keys.size() * 8)) || (st = dalloc(e, &e->pay_cd, tcd.pay.size() * sizeof(R))) ||
        (st = dalloc(e, (void**)&e->keys_cl, tcl.keys.size() * 8)) || (st = dalloc(e, &e->pay_cl, tcl.pay.size() * sizeof(R))))
        return st;
    PD_HIP(hipMemcpy(e->keys_cd, tcd.keys.data(), tcd.keys.size() * 8, hipMemcpyHostToDevice));
    PD_HIP(hipMemcpy(e->pay_cd, tcd.pay.data(), tcd.pay.size() * sizeof(R), hipMemcpyHostToDevice));
    PD_HIP(hipMemcpy(e->keys_cl, tcl.keys.data(), tcl.keys.size() * 8, hipMemcpyHostToDevice));
    PD_HIP(hipMemcpy(e->pay_cl, tcl.pay.data(), tcl.pay.size() * sizeof(R), hipMemcpyHostToDevice));
    D.keys_cd = e->keys_cd; D.keys_cl = e->keys_cl; D.pay_cd = (const R*)e->pay_cd; D.pay_cl = (const R*)e->pay_cl;
    D.logcap_cd = tcd.logcap; D.logcap_cl = tcl.logcap;
    // initial neighbourhood caches: the 50-NN at the initial state's clamped query points
    // (any valid 50-set works; the in-kernel swap search repairs it)
    D.init_key_cd = host_knn_key(p->cd, 3.0, 0.0);
    D.init_key_cl = host_knn_key(p->cl, 3.0, 10.0);
    if (c->phase == PD_PHASE_SUBSONIC || c->phase == PD_PHASE_SUPERSONIC) {
        // ascent reference trajectory, in the handle's precision (binary-searched per env-step)
        const double* src[4] = {p->ref_y, p->ref_x, p->ref_vx, p->ref_vy};
        const R** dst[4] = {&D.ref_y, &D.ref_x, &D.ref_vx, &D.ref_vy};
        std::vector<R> buf((size_t)p->n_ref);
        for (int k = 0; k < 4; ++k) {
            void* d;
            if ((st = dalloc(e, &d, buf.size() * sizeof(R)))) return st;
            for (int32_t r = 0; r < p->n_ref; ++r) buf[r] = (R)src[k][r];
            PD_HIP(hipMemcpy(d, buf.data(), buf.size() * sizeof(R), hipMemcpyHostToDevice));
            *dst[k] = (const R*)d;
        }
    }
    if ((st = dalloc(e, &e->dparams, sizeof(D)))) return st;
    PD_HIP(hipMemcpy(e->dparams, &D, sizeof(D), hipMemcpyHostToDevice));
    size_t R_ = sizeof(R);
    if ((st = dalloc(e, &e->st, 11 * N * R_)) || (st = dalloc(e, &e->vprev, N * R_)) ||
        (st = dalloc(e, &e->gwin, 10 * N * R_)) || (st = dalloc(e, &e->act, 3 * N * R_)) ||
        (st = dalloc(e, &e->wind, 6 * N * R_)) || (st = dalloc(e, (void**)&e->ghead, N)) ||
        (st = dalloc(e, (void**)&e->glen, N)) || (st = dalloc(e, (void**)&e->wprof, N)) ||
        (st = dalloc(e, (void**)&e->key, 2 * N * 8)) || (st = dalloc(e, (void**)&e->slot, 2 * N * 4)) ||
        (st = dalloc(e, (void**)&e->tid, N)) || (st = dalloc(e, (void**)&e->epi, N * 4)) ||
        (st = dalloc(e, (void**)&e->tstep, N * 4)) || (st = dalloc(e, (void**)&e->fin, N)) ||
        (st = dalloc(e, (void**)&e->live[0], N * 4)) ||
        (st = dalloc(e, (void**)&e->live[1], N * 4)) || (st = dalloc(e, (void**)&e->live_cnt, 3 * 4)))
        return st;
    PD_HIP(hipMemset(e->gwin, 0, 10 * N * R_));
    PD_HIP(hipMemset(e->epi, 0xff, N * 4));   // first reset -> episode 0
    if ((st = dalloc(e, (void**)&e->pend.count, 8)) || (st = dalloc(e, (void**)&e->pend.keys, kPendingCap * 8)) ||
        (st = dalloc(e, (void**)&e->pend.pay, (size_t)kPendingCap * kPay * 8)) || (st = dalloc(e, (void**)&e->pend.stats, 16 * 8)))
        return st;
    PD_HIP(hipMemset(e->pend.count, 0, 8));
    unsigned long long stats0[16] = {0, 0, (unsigned long long)tcd.entries, (unsigned long long)tcl.entries};
    PD_HIP(hipMemcpy(e->pend.stats, stats0, sizeof(stats0), hipMemcpyHostToDevice));
    StepArgs<R> a = make_args<R>(e);
    unsigned grid = (unsigned)((N + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_reset<R>, dim3(grid), dim3(kBlock), 0, 0, a, (const uint8_t*)nullptr);
    PD_HIP(hipGetLastError());
    PD_HIP(hipDeviceSynchronize());
    return PD_OK;
}

template <typename R, int PH, int RT, bool W, int LPE> void launch_step(const StepArgs<R>& a, hipStream_t s) {
    unsigned grid = (unsigned)((a.n * LPE + kStepBlock - 1) / kStepBlock);
    hipLaunchKernelGGL((k_step<R, PH, RT, W, LPE>), dim3(grid), dim3(kStepBlock), 0, s, a);
}

template <typename R, int PH, int RT, bool W> void launch_lpe(int lpe, const StepArgs<R>& a, hipStream_t s) {
    switch (lpe) {
        case 1: launch_step<R, PH, RT, W, 1>(a, s); break;
        case 2: launch_step<R, PH, RT, W, 2>(a, s); break;
        case 8: launch_step<R, PH, RT, W, 8>(a, s); break;
        case 16: launch_step<R, PH, RT, W, 16>(a, s); break;
        default: launch_step<R, PH, RT, W, 4>(a, s); break;
    }
}

template <typename R> void dispatch_step(const pd_env* e, const StepArgs<R>& a, hipStream_t s) {
    int ph = e->cfg.phase, l = e->lpe;
    bool pso = e->cfg.rtd == PD_RTD_PSO;   // RL and NONE share the RL instantiation (NONE zeroes the rtd)
    bool w = e->cfg.enable_wind != 0;
    if (ph == 0 && !pso) { if (w) launch_lpe<R, 0, 0, true>(l, a, s); else launch_lpe<R, 0, 0, false>(l, a, s); }
    else if (ph == 0) { if (w) launch_lpe<R, 0, 1, true>(l, a, s); else launch_lpe<R, 0, 1, false>(l, a, s); }
    else if (ph == 1 && pso) { if (w) launch_lpe<R, 1, 1, true>(l, a, s); else launch_lpe<R, 1, 1, false>(l, a, s); }
    else if (ph == 1) { if (w) launch_lpe<R, 1, 0, true>(l, a, s); else launch_lpe<R, 1, 0, false>(l, a, s); }
    else { if (w) launch_lpe<R, 2, 0, true>(l, a, s); else launch_lpe<R, 2, 0, false>(l, a, s); }
}

template <typename R, int PH, bool W, int LPE> void launch_policy_lpe(const StepArgs<R>& a, int64_t n_launch,
                                                                      hipStream_t s) {
    unsigned grid = (unsigned)((n_launch * LPE + kStepBlock - 1) / kStepBlock);
    hipLaunchKernelGGL((k_step<R, PH, 1, W, LPE, 1>), dim3(grid), dim3(kStepBlock), 0, s, a);
}
template <typename R, int PH, bool W> void launch_policy(const StepArgs<R>& a, int lpe, int64_t n_launch, hipStream_t s) {
    if (lpe >= 8) launch_policy_lpe<R, PH, W, 8>(a, n_launch, s);
    else if (lpe == 4) launch_policy_lpe<R, PH, W, 4>(a, n_launch, s);
    else launch_policy_lpe<R, PH, W, 2>(a, n_launch, s);
}

template <typename R> void launch_insert(pd_env* e, hipStream_t s) {
    hipLaunchKernelGGL(k_insert<R>, dim3(1), dim3(kPay), 0, s, e->pend, e->keys_cd, (R*)e->pay_cd, e->logcap_cd,
                       e->keys_cl, (R*)e->pay_cl, e->logcap_cl);
}

template <typename R>
pd_status step_impl(pd_env* e, const void* actions, void* obs, void* reward, uint8_t* done, uint8_t* trunc,
                    int8_t* tid, const double* noise, void* info, void* reward_sum, hipStream_t s,
                    int n_fused = 1) {
    StepArgs<R> a = make_args<R>(e);
    a.actions = actions; a.obs = (R*)obs; a.reward = (R*)reward; a.done = done; a.trunc = trunc; a.trunc_id = tid;
    a.noise = noise; a.info = (R*)info; a.reward_sum = (R*)reward_sum;
    a.n_fused = n_fused;
    dispatch_step<R>(e, a, s);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

// policy rollouts: every env live, in index order
__global__ __launch_bounds__(kBlock) void k_live_init(int32_t* list, uint32_t* cnt, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) list[i] = (int32_t)i;
    if (i < 3) cnt[i] = i == 0 ? (uint32_t)n : 0u;
}

template <typename R>
pd_status rollout_policy_impl(pd_env* e, const float* w, int32_t max_steps, void* fitness, int32_t* steps,
                              int32_t check_every, hipStream_t s) {
    const int64_t N = e->cfg.n_envs;
    unsigned grid = (unsigned)((N + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_reset<R>, dim3(grid), dim3(kBlock), 0, s, make_args<R>(e), (const uint8_t*)nullptr);
    PD_HIP(hipMemsetAsync(fitness, 0, (size_t)N * sizeof(R), s));
    hipLaunchKernelGGL(k_live_init, dim3(grid), dim3(kBlock), 0, s, e->live[0], e->live_cnt, N);
    StepArgs<R> a = make_args<R>(e);
    a.policy_w = w; a.reward_sum = (R*)fitness; a.auto_reset = 0;
    const bool wind = e->cfg.enable_wind != 0;
    // launch t steps live[t & 1][0, live_cnt[t % 3]) and appends the survivors to the other list;
    // the grid covers the live count last read back (a workgroup past the device count leaves
    // at once), so the launches shrink with the swarm's live envs.  Checks are one interval
    // behind: at a check the count is copied to pinned memory under an event, and the host
    // waits for the PREVIOUS check's event, with check_every launches still queued behind it
    // (no bubble); at most 2 * check_every nearly empty launches run after the last episode.
    if (check_every > 0 && !e->host_cnt) {
        PD_HIP(hipHostMalloc((void**)&e->host_cnt, 2 * sizeof(uint32_t), hipHostMallocDefault));
        for (hipEvent_t& ev : e->cnt_ev) PD_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    // The list pays off once the grid no longer fits the chip in one round (a launch then costs
    // the rounds its waves need); below that the launch time is one wave's, and reading the
    // state and actor weights through the list (gathers) only costs.  PDENV_COMPACT=0/1 forces.
    int dev_cus = 256;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, e->device);
    const char* force = getenv("PDENV_COMPACT");
    a.use_list = force && *force ? (atoi(force) != 0) : (N * e->lpe > (int64_t)dev_cus * 512);
    int64_t n_launch = N;
    int checks = 0;
    for (int32_t t = 0; t < max_steps; ++t) {
        a.list_in = e->live[t & 1]; a.list_out = e->live[(t + 1) & 1];
        a.cnt_in = e->live_cnt + t % 3; a.cnt_out = e->live_cnt + (t + 1) % 3; a.cnt_zero = e->live_cnt + (t + 2) % 3;
        if (e->cfg.phase == PD_PHASE_PURE_THROTTLE) { if (wind) launch_policy<R, 0, true>(a, e->lpe, n_launch, s); else launch_policy<R, 0, false>(a, e->lpe, n_launch, s); }
        else { if (wind) launch_policy<R, 1, true>(a, e->lpe, n_launch, s); else launch_policy<R, 1, false>(a, e->lpe, n_launch, s); }
        PD_HIP(hipGetLastError());
        if ((t & 15) == 15) launch_insert<R>(e, s);
        if (check_every > 0 && (t + 1) % check_every == 0 && t + 1 < max_steps) {
            const int k = checks & 1;
            PD_HIP(hipMemcpyAsync(e->host_cnt + k, e->live_cnt + (t + 1) % 3, 4, hipMemcpyDeviceToHost, s));
            PD_HIP(hipEventRecord(e->cnt_ev[k], s));
            if (checks > 0) {
                PD_HIP(hipEventSynchronize(e->cnt_ev[k ^ 1]));
                const uint32_t live = ((volatile uint32_t*)e->host_cnt)[k ^ 1];
                if (live == 0) break;
                if (a.use_list) n_launch = live;
            }
            ++checks;
        }
    }
    launch_insert<R>(e, s);
    if (steps) PD_HIP(hipMemcpyAsync(steps, e->tstep, (size_t)N * 4, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipGetLastError());
    return PD_OK;
}

// Steps per fused launch: the miss flush runs between launches, so a neighbourhood solved on
// device is re-solved at most this many steps before it is in the tables (PDENV_FUSE overrides).
int fuse_chunk() {
    const char* s = getenv("PDENV_FUSE");
    int k = s && *s ? atoi(s) : 16;
    return k < 1 ? 1 : (k > 256 ? 256 : k);
}

// n_steps env-steps in launches of fuse_chunk() fused steps, each followed by the miss flush.
// Row t of every [n_steps][N...] array belongs to step t; NULL outputs are not written.
pd_status step_n_impl(pd_env* e, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                      uint8_t* trunc, int8_t* tid, void* reward_sum, hipStream_t s) {
    const size_t N = (size_t)e->cfg.n_envs;
    const size_t sa = N * e->act_dim * (e->cfg.action_f64 ? 8 : 4), so = N * e->obs_dim * e->rsize;
    const size_t sr = N * e->rsize;
    const int K = fuse_chunk();
    for (int32_t t = 0; t < n_steps; t += K) {
        const int k = n_steps - t < K ? n_steps - t : K;
        auto at = [&](void* p, size_t stride) { return p ? (void*)((char*)p + stride * t) : nullptr; };
        const void* act = (const char*)actions + sa * t;
        pd_status st = e->rsize == 8
            ? step_impl<double>(e, act, at(obs, so), at(reward, sr), (uint8_t*)at(done, N), (uint8_t*)at(trunc, N),
                                (int8_t*)at(tid, N), nullptr, nullptr, reward_sum, s, k)
            : step_impl<float>(e, act, at(obs, so), at(reward, sr), (uint8_t*)at(done, N), (uint8_t*)at(trunc, N),
                               (int8_t*)at(tid, N), nullptr, nullptr, reward_sum, s, k);
        if (st != PD_OK) return st;
        if ((st = pd_flush_misses(e, s)) != PD_OK) return st;
    }
    return PD_OK;
}

}  // namespace

// ================================================================ C ABI
extern "C" {

int pd_abi_version(void) { return PD_ABI_VERSION; }
size_t pd_sizeof_params(void) { return sizeof(pd_params); }
size_t pd_sizeof_config(void) { return sizeof(pd_config); }
const char* pd_last_error(void) { return g_err.c_str(); }

int pd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

pd_status pd_create(const pd_params* params, const pd_config* cfg, pd_env** out) {
    if (!out) return fail(PD_ERR_INVALID, "out is null");
    *out = nullptr;
    pd_status st = validate(params, cfg);
    if (st != PD_OK) return st;
    int ndev = pd_device_count();
    if (ndev <= 0) return fail(PD_ERR_HIP, "no HIP device visible");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(PD_ERR_INVALID, "device ordinal out of range");
    PD_HIP(hipSetDevice(cfg->device));
    pd_env* e = new pd_env();
    e->cfg = *cfg;
    e->device = cfg->device;
    e->act_dim = act_dim_of(cfg->phase);
    e->obs_kind = obs_kind_of(cfg->phase, cfg->rtd);
    e->obs_dim = obs_dim(e->obs_kind);
    e->rsize = cfg->precision == PD_F64 ? 8 : 4;
    // default lanes per env: about one wave per SIMD (n_envs x LPE ~ 65 536 lanes), at least 2.
    // Below ~64k envs the step is bound by one wave's latency, and splitting each RBF over more
    // lanes shortens it (measured, f64 ms/step: 4 096 envs LPE 16 0.049, 8 0.054, 2 0.071;
    // 16 384 LPE 4 0.066, 8 0.067, 16 0.105; 32 768 LPE 2 0.072, 4 0.075; 65 536 LPE 2 best)
    e->lpe = cfg->lanes_per_env != 0 ? cfg->lanes_per_env
                                     : (cfg->n_envs <= 4096 ? 16 : (cfg->n_envs <= 8192 ? 8 : (cfg->n_envs <= 16384 ? 4 : 2)));
    if (e->lpe != 1 && e->lpe != 2 && e->lpe != 4 && e->lpe != 8 && e->lpe != 16) { delete e; return fail(PD_ERR_INVALID, "lanes_per_env must be 0, 1, 2, 4, 8 or 16"); }
    st = cfg->precision == PD_F64 ? create_impl<double>(params, cfg, e) : create_impl<float>(params, cfg, e);
    if (st != PD_OK) { pd_destroy(e); return st; }
    *out = e;
    return PD_OK;
}

pd_status pd_destroy(pd_env* e) {
    if (!e) return PD_OK;
    (void)hipSetDevice(e->device);
    for (void* p : e->allocs) (void)hipFree(p);
    if (e->host_cnt) (void)hipHostFree(e->host_cnt);
    for (hipEvent_t ev : e->cnt_ev) if (ev) (void)hipEventDestroy(ev);
    delete e;
    return PD_OK;
}

pd_status pd_reset(pd_env* e, const uint8_t* mask, void* obs, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    unsigned grid = (unsigned)((e->cfg.n_envs + kBlock - 1) / kBlock);
    if (e->rsize == 8) hipLaunchKernelGGL(k_reset<double>, dim3(grid), dim3(kBlock), 0, s, make_args<double>(e), mask);
    else hipLaunchKernelGGL(k_reset<float>, dim3(grid), dim3(kBlock), 0, s, make_args<float>(e), mask);
    PD_HIP(hipGetLastError());
    if (obs) return pd_observe(e, obs, stream);
    return PD_OK;
}

pd_status pd_step(pd_env* e, const void* actions, void* obs, void* reward, uint8_t* done, uint8_t* truncated,
                  int8_t* trunc_id, const double* noise, void* info, void* stream) {
    if (!e || !actions) return fail(PD_ERR_INVALID, "null env/actions");
    PD_HIP(hipSetDevice(e->device));
    if (e->rsize == 8)
        return step_impl<double>(e, actions, obs, reward, done, truncated, trunc_id, noise, info, nullptr, (hipStream_t)stream);
    return step_impl<float>(e, actions, obs, reward, done, truncated, trunc_id, noise, info, nullptr, (hipStream_t)stream);
}

pd_status pd_step_n(pd_env* e, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                    uint8_t* truncated, int8_t* trunc_id, void* stream) {
    if (!e || !actions || n_steps < 0) return fail(PD_ERR_INVALID, "bad step_n args");
    if (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN)
        return fail(PD_ERR_UNSUPPORTED, "pd_step_n: landing-burn phases only (use pd_step)");
    PD_HIP(hipSetDevice(e->device));
    return step_n_impl(e, actions, n_steps, obs, reward, done, truncated, trunc_id, nullptr, (hipStream_t)stream);
}

pd_status pd_rollout(pd_env* e, const void* actions, int32_t n_steps, void* reward_sum, void* stream) {
    if (!e || !actions || n_steps < 0) return fail(PD_ERR_INVALID, "bad rollout args");
    PD_HIP(hipSetDevice(e->device));
    if (e->cfg.phase == PD_PHASE_PURE_THROTTLE || e->cfg.phase == PD_PHASE_LANDING_BURN)
        return step_n_impl(e, actions, n_steps, nullptr, nullptr, nullptr, nullptr, nullptr, reward_sum,
                           (hipStream_t)stream);
    size_t stride = (size_t)e->cfg.n_envs * e->act_dim * (e->cfg.action_f64 ? 8 : 4);
    for (int32_t t = 0; t < n_steps; ++t) {
        const void* at = (const char*)actions + stride * t;
        pd_status st = e->rsize == 8
            ? step_impl<double>(e, at, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, reward_sum, (hipStream_t)stream)
            : step_impl<float>(e, at, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, reward_sum, (hipStream_t)stream);
        if (st != PD_OK) return st;
        if ((t & 15) == 15 || t + 1 == n_steps) { if ((st = pd_flush_misses(e, stream)) != PD_OK) return st; }
    }
    return PD_OK;
}

pd_status pd_rollout_policy(pd_env* e, const float* weights, int32_t n_params, int32_t max_steps, void* fitness,
                            int32_t* steps, int32_t check_every, void* stream) {
    if (!e || !weights || !fitness || max_steps < 0) return fail(PD_ERR_INVALID, "bad policy rollout args");
    if (e->cfg.rtd != PD_RTD_PSO) return fail(PD_ERR_UNSUPPORTED, "policy rollouts need rtd = PD_RTD_PSO");
    int want = e->cfg.phase == PD_PHASE_PURE_THROTTLE ? PD_ACTOR_PARAMS_PURE_THROTTLE : PD_ACTOR_PARAMS_LANDING_BURN;
    if (n_params != want) return fail(PD_ERR_INVALID, "n_params does not match the phase's actor");
    PD_HIP(hipSetDevice(e->device));
    return e->rsize == 8 ? rollout_policy_impl<double>(e, weights, max_steps, fitness, steps, check_every, (hipStream_t)stream)
                         : rollout_policy_impl<float>(e, weights, max_steps, fitness, steps, check_every, (hipStream_t)stream);
}

pd_status pd_flush_misses(pd_env* e, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    if (e->rsize == 8) launch_insert<double>(e, (hipStream_t)stream);
    else launch_insert<float>(e, (hipStream_t)stream);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

pd_status pd_observe(pd_env* e, void* obs, void* stream) {
    if (!e || !obs) return fail(PD_ERR_INVALID, "null env/obs");
    PD_HIP(hipSetDevice(e->device));
    int kind = e->obs_kind;
    unsigned grid = (unsigned)((e->cfg.n_envs + kBlock - 1) / kBlock);
    hipStream_t s = (hipStream_t)stream;
    if (e->rsize == 8) { auto a = make_args<double>(e); a.obs = (double*)obs; hipLaunchKernelGGL(k_observe<double>, dim3(grid), dim3(kBlock), 0, s, a, kind); }
    else { auto a = make_args<float>(e); a.obs = (float*)obs; hipLaunchKernelGGL(k_observe<float>, dim3(grid), dim3(kBlock), 0, s, a, kind); }
    PD_HIP(hipGetLastError());
    return PD_OK;
}

pd_status pd_get_state(pd_env* e, void* state, void* stream) {
    if (!e || !state) return fail(PD_ERR_INVALID, "null env/state");
    PD_HIP(hipSetDevice(e->device));
    PD_HIP(hipMemcpyAsync(state, e->st, 11 * e->cfg.n_envs * e->rsize, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return PD_OK;
}

pd_status pd_set_state(pd_env* e, const void* state, void* stream) {
    if (!e || !state) return fail(PD_ERR_INVALID, "null env/state");
    PD_HIP(hipSetDevice(e->device));
    PD_HIP(hipMemcpyAsync(e->st, state, 11 * e->cfg.n_envs * e->rsize, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return PD_OK;
}

pd_status pd_get_actuators(pd_env* e, void* act, void* stream) {
    if (!e || !act) return fail(PD_ERR_INVALID, "null env/act");
    PD_HIP(hipSetDevice(e->device));
    PD_HIP(hipMemcpyAsync(act, e->act, 3 * e->cfg.n_envs * e->rsize, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return PD_OK;
}

pd_status pd_set_actuators(pd_env* e, const void* act, void* stream) {
    if (!e || !act) return fail(PD_ERR_INVALID, "null env/act");
    PD_HIP(hipSetDevice(e->device));
    PD_HIP(hipMemcpyAsync(e->act, act, 3 * e->cfg.n_envs * e->rsize, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return PD_OK;
}

pd_status pd_set_gload_window(pd_env* e, const void* vprev, const void* window, const uint8_t* len, void* stream) {
    if (!e || !vprev || !window || !len) return fail(PD_ERR_INVALID, "null env/vprev/window/len");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    PD_HIP(hipMemcpyAsync(e->vprev, vprev, N * e->rsize, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipMemcpyAsync(e->gwin, window, 10 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipMemcpyAsync(e->glen, len, N, hipMemcpyDeviceToDevice, s));
    PD_HIP(hipMemsetAsync(e->ghead, 0, N, s));   // oldest entry in slot 0
    return PD_OK;
}

pd_status pd_set_wind_sigmas(pd_env* e, const double* sig, void* stream) {
    if (!e || !sig) return fail(PD_ERR_INVALID, "null env/sig");
    PD_HIP(hipSetDevice(e->device));
    unsigned grid = (unsigned)((e->cfg.n_envs + kBlock - 1) / kBlock);
    hipStream_t s = (hipStream_t)stream;
    if (e->rsize == 8) hipLaunchKernelGGL(k_set_sigmas<double>, dim3(grid), dim3(kBlock), 0, s, make_args<double>(e), sig);
    else hipLaunchKernelGGL(k_set_sigmas<float>, dim3(grid), dim3(kBlock), 0, s, make_args<float>(e), sig);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

pd_status pd_counters(pd_env* e, int64_t* misses, int64_t* ecd, int64_t* ecl, int64_t* nans) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    unsigned long long st[16];
    PD_HIP(hipMemcpy(st, e->pend.stats, sizeof(st), hipMemcpyDeviceToHost));
    if (getenv("PDENV_DEBUG_COUNTERS")) {
        fprintf(stderr, "[pdenv] knn calls %llu line-candidates %llu iterations %llu probes %llu\n", st[4], st[5], st[6], st[7]);
        if (st[15])
            fprintf(stderr, "[pdenv] k_step wave clocks (mean per wave): staging %.0f loads %.0f pre-aero %.0f aero %.0f "
                    "post-aero %.0f rtd %.0f outputs %.0f (waves %llu)\n", (double)st[8] / st[15], (double)st[9] / st[15],
                    (double)st[10] / st[15], (double)st[11] / st[15], (double)st[12] / st[15], (double)st[13] / st[15],
                    (double)st[14] / st[15], st[15]);
    }
    if (misses) *misses = (int64_t)st[0];
    if (nans) *nans = (int64_t)st[1];
    if (ecd) *ecd = (int64_t)st[2];
    if (ecl) *ecl = (int64_t)st[3];
    return PD_OK;
}

int pd_obs_dim(const pd_env* e) { return e ? e->obs_dim : 0; }
int pd_action_dim(const pd_env* e) { return e ? e->act_dim : 0; }

}  // extern "C"
