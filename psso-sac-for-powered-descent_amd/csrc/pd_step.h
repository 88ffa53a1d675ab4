// pd_step.h -- the step kernel of libpdenv: declarations shared by the host translation unit
// (pdenv.hip) and the kernel translation units (kstep_*.hip, which include pd_step_impl.h).
//
// Layout in HBM: struct-of-arrays, one env per group of LPE lanes.  A launch loads each env's
// state once into registers (its g-load ring into LDS), runs F consecutive env-steps of
// rocket_environment_pre_wrap.step (4 physics sub-steps, g-load window, truncated -> done ->
// reward, observation, in-register auto-reset), writes each step's outputs, and stores the
// state once at the end.  See DESIGN.md for the roofline of each kernel.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pdenv.h"
#include "pd_physics.h"
#include "pd_sac_mlp.h"

namespace pd {

constexpr int kBlock = 256;
constexpr int kStepBlock = 256;
constexpr int kScratch = kSys * kSys + kSys + 3 * kNbr + kPay;   // doubles per solve slot
constexpr int kPendingCap = 4096;     // device-solved neighbourhoods queued per launch
constexpr int kSolveSlots = 1024;     // global-memory LU scratch slots (one per workgroup, modulo)
constexpr int kGridExact = 1 << 30;   // grid_slot flag: every point of the cell has its key
constexpr int kGridRefine = 1 << 29;  // grid_slot flag: the cell is refined, low bits = its sub-grid
constexpr int kGridBisect = 1 << 28;  // sub_slot flag: two regions split by one bisector, low bits = its record
constexpr int kGridPiece = 1 << 27;   // grid_slot flag (exact cells of binary64 handles): the cell has its cell piece
// Fine index (binary64 handles with cell pieces): one word per sub-cell of every cell (kGridSub x
// kGridSub per cell, Mach-major over the whole grid), read in place of the cell record: a piece
// the sub-cell's points all use, or the bisector record splitting it; 0: the cell/sub-cell records
constexpr uint32_t kFinePiece = 1u << 30;
constexpr uint32_t kFineBisect = 1u << 29;
constexpr uint32_t kFineRefined = 1u << 28;    // (the sub-cell belongs to a refined cell: workload counters)
constexpr uint32_t kFineIndex = kFineRefined - 1u;

// Cell pieces (binary64 handles): the thin-plate sum of one neighbourhood over one interior grid
// cell as a polynomial of total degree kCellDeg in the cell coordinates (u, v) in [-1, 1]^2 plus
// its kCellExact terms nearest to the cell (pdenv.hip build_cell_pieces).  Record: the
// coefficients row by row (u^i, i = kCellDeg .. 0; within a row v^j, j = kCellDeg - i .. 0), then
// per exact term (Mach, coefficient / 8, AoA), then the neighbourhood's key (its bits), padded to 16
// bytes.
#ifndef PD_CELL_DEG
#define PD_CELL_DEG 8
#endif
#ifndef PD_CELL_EXACT
#define PD_CELL_EXACT 4
#endif
constexpr int kCellDeg = PD_CELL_DEG;
constexpr int kCellCoef = (kCellDeg + 1) * (kCellDeg + 2) / 2;
constexpr int kCellExact = PD_CELL_EXACT;
constexpr int kCellKey = kCellCoef + 3 * kCellExact;
constexpr int kCellStride = (kCellKey + 2) & ~1;
// binary32 handles: the same record in floats, the key's 8 bytes at an 8-byte aligned float index,
// the stride a multiple of 4 floats (16 bytes)
constexpr int kCellKeyF = (kCellKey + 1) & ~1;
constexpr int kCellStrideF = (kCellKeyF + 2 + 3) & ~3;
template <typename R> constexpr int cell_stride() { return sizeof(R) == 8 ? kCellStride : kCellStrideF; }
template <typename R> constexpr int cell_key() { return sizeof(R) == 8 ? kCellKey : kCellKeyF; }

// A sub-cell holding two 50-NN regions A, B whose keys differ by one point swap (p in A, q in B):
// s(x) = n . x - c < 0 on A's side (p nearer than q).  Each side's slot carries kGridExact only if
// the host checked that the side's part of the sub-cell, kept tau off the bisector, has that key
// everywhere (its clipped polygon's vertices carry it; regions are convex); |s| <= 3 tau: verified.
struct GridBisect {
    double nx, ny, c, tau;
    unsigned long long key_a, key_b;
    int slot_a, slot_b;
    int piece_a, piece_b;   // each side's cell piece (binary64 handles; -1: none)
};
#ifndef PD_GRID_SUB
#define PD_GRID_SUB 8
#endif
constexpr int kGridSub = PD_GRID_SUB;   // sub-cells per refined cell side
constexpr int kStats = 48;            // pend.stats words (see Stat)

// pend.stats[] words
enum Stat {
    kStMisses = 0, kStNan = 1, kStInsCd = 2, kStInsCl = 3,
    kStStamp = 8,                                                 // 8..15, 22..31: PD_STAMP section clocks
    kStDropped = 16,
    // workload counters of the step kernel (launches with counting on, pd_count_work: per-wave
    // sums in LDS, one atomic per counter and wave at the end): what the launches did
    kStWork = 32,
    kStGust = kStWork + 0,       // env sub-steps inside the gust band (stochastic wind, y < vk_y_threshold)
    kStResets = kStWork + 1,     // in-kernel auto-resets
    kStQLine = kStWork + 2,      // LPE 2 table queries on a clamped line (|alpha_eff| clamps the table)
    kStQVerify = kStWork + 3,    // LPE 2 queries whose candidate neighbourhood the swap search verified
    kStQTaylor = kStWork + 4,    // LPE 2 queries evaluated from a Taylor piece
    kStQBal = kStWork + 5,       // LPE 2 queries evaluated by the balanced chunk sums
    kStQMiss = kStWork + 6,      // LPE 2 queries whose neighbourhood was not in the tables (device solve)
    kStBalRounds = kStWork + 7,  // balanced-sum rounds (per wave and call: ceil(5 n / 64))
    kStQRefined = kStWork + 8,   // LPE 2 interior queries in a refined grid cell (a dependent sub-cell load)
    kStQBisect = kStWork + 9,    // ... whose sub-cell is split by a bisector (a third dependent load)
    kStWRefined = kStWork + 10,  // wave sub-steps with at least one refined-cell query
    kStWBisect = kStWork + 11,   // wave sub-steps with at least one bisector query
    kStQCell = kStWork + 12,     // LPE 2 queries evaluated from a cell piece
    kStWMixed = kStWork + 13,    // wave sub-steps holding both clamped-line and interior queries
    kNWork = 14
};

// Per-wave workload counts in LDS (nullptr: counting off, the launch pays one scalar branch per
// site).  Every update is the popcount of a ballot, added by lane 0 of the converged wave.
struct WaveCount {
    uint32_t* w;
    __device__ __forceinline__ void add(int k, bool pred) {
        if (w) {
            const uint32_t v = (uint32_t)__popcll(__ballot(pred));
            if (__lane_id() == 0) w[k] += v;
        }
    }
    __device__ __forceinline__ void add_n(int k, uint32_t v) {
        if (w && __lane_id() == 0) w[k] += v;
    }
};

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
    unsigned long long* stats;   // [kStats]
    double* solve_ws;            // [kSolveSlots][kScratch] exact-solve scratch (global memory)
    int* solve_lock;             // [kSolveSlots]
};

template <typename R> struct StepArgs {
    uint64_t P;                      // const DevParams<R>* (read through a constant-AS view)
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
    R* info;                         // [PD_N_INFO][N] (single-step launches)
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
    int count_work;                  // workload counters on (pd_count_work; diagnostic launches)
    // pd_step_sac (single-step launches): the action sampled from the actor's heads in the kernel,
    // tanh(mean + exp(clamp(log_std, lo, hi)) eps) max (eps NULL: tanh(mean) max), and float32
    // outputs: the action, the transition row [N][2S + A + 2] and the next observation [N][S]
    const float* sac_mean; const float* sac_logstd; const float* sac_eps;
    float sac_lo, sac_hi, sac_max;
    uint32_t sac_hs;                 // row stride of mean / log_std in floats (both heads in one [N][2A] array: 2A)
    float* sac_act; float* slab; float* obs32;
    // pd_step_sac_ring: eps drawn in the kernel (Philox tag kTagSacEps; sac_eps then NULL), written
    // to sac_eps_out when given; the transition rows into a replay ring of ring_cap rows at
    // (ring_state[0] + i) mod ring_cap with prio[row] = *max_prio, and the launch's last workgroup
    // advancing ring_state (0 position, 1 size, 2 the workgroup ticket); ring_state NULL: slab rows
    // at i (pd_step_sac's layout)
    int sac_draw;
    float* sac_eps_out;
    int64_t ring_cap;
    long long* ring_state;
    float* prio;
    const float* max_prio;
    // pd_step_sac_fused (16 lanes per env): the actor's forward pass for the workgroup's 16 envs
    // in the kernel prologue (pd_sac_mlp.h sac_mlp_tile) on obs32 as the previous step left it, the
    // heads into LDS (and into sac_heads_out [N][2A] when given); sac_mlp.H = 0: heads from
    // sac_mean / sac_logstd
    SacMlp sac_mlp;
    float* sac_heads_out;
    // list launches of a policy rollout: the live envs' parameters in list order, [P][N] (the
    // launch copies them there once, so that its fused steps read them coalesced, not gathered)
    float* policy_wc;
};

// Kernel launchers, explicitly instantiated in the kstep_*.hip translation units.
template <typename R, int PH, int RT, bool W, int LPE, bool RK = false> void launch_step(const StepArgs<R>& a, hipStream_t s);
template <typename R, int PH, bool W, int LPE> void launch_policy_lpe(const StepArgs<R>& a, int64_t n_launch,
                                                                      hipStream_t s);

}  // namespace pd
