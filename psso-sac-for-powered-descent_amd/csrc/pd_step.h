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

#include <cstring>

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
// (degree 7 and 3 exact terms were measured in round 3 and dropped: DESIGN.md s9)
constexpr int kCellDeg = 8;
constexpr int kCellCoef = (kCellDeg + 1) * (kCellDeg + 2) / 2;
constexpr int kCellExact = 4;
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
constexpr int kGridSub = 8;   // sub-cells per refined cell side
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

// the clamped query lines' breakpoints, interval keys/slots and search buckets (staged into LDS)
template <typename R> struct LineLds {
    R bp[4][kLineMax];
    int slot[4][kLineMax + 1];
    unsigned long long key[4][kLineMax + 1];
    R a[4];
    int nbp[4];
    int tay_off[4];
    uint16_t lb[4][kLineBuckets];
};

// The tables every step workgroup stages into LDS, in the layout of its LDS (StepLds derives from
// it): the handle keeps an image of it in HBM (pd_create, fill_step_static) and the kernel
// prologue copies it with 16-byte loads.
template <typename R, bool WIND> struct alignas(16) StepStatic {
    // table points as (Mach_p, Mach_p+1) entries, C_D's 256 then C_L's: one 16-byte LDS read per
    // payload pair slot (smach[2p] is point p's Mach for the neighbourhood search)
    alignas(16) R tab[1024];
    R gf[256];                    // grid fins: ca_x, ca_y, cn_x, cn_y (64 each)
    R gfs[128];                   // their interval slopes: C_a at the upper index, C_n at the lower
    uint16_t ca_lb[64];           // C_a search buckets
    R isa[9 * kIsaCols];          // ISA layers
    R walt[WIND ? 800 : 1];       // wind profiles [50][16]: altitude km, speed
    R wsp[WIND ? 800 : 1];
    LineLds<R> lines;
};

// The image's contents from the handle's parameter block (host): what the kernel prologue staged
// field by field before round 5, the same values; the grid-fin interval slopes are the division
// grid_fin_ca / np_interp would do, on the same operands (IEEE on host and device: same bits)
template <typename R, bool WIND> void fill_step_static(const DevParams<R>& P, StepStatic<R, WIND>& L) {
    std::memset(&L, 0, sizeof(L));
    for (int t = 0; t < 256; ++t) {
        L.tab[2 * t] = P.cd_mach[t]; L.tab[2 * t + 1] = t < 255 ? P.cd_mach[t + 1] : R(0);
        L.tab[512 + 2 * t] = P.cl_mach[t]; L.tab[513 + 2 * t] = t < 255 ? P.cl_mach[t + 1] : R(0);
    }
    for (int i = 0; i < 64; ++i) {
        L.gf[i] = P.ca_x[i]; L.gf[64 + i] = P.ca_y[i]; L.gf[128 + i] = P.cn_x[i]; L.gf[192 + i] = P.cn_y[i];
        L.ca_lb[i] = P.ca_lb[i];
        // (entries past a table's end are never read)
        L.gfs[i] = i >= 1 ? (P.ca_y[i] - P.ca_y[i - 1]) / (P.ca_x[i] - P.ca_x[i - 1]) : R(0);
        L.gfs[64 + i] = i < 63 ? (P.cn_y[i + 1] - P.cn_y[i]) / (P.cn_x[i + 1] - P.cn_x[i]) : R(0);
    }
    for (int k = 0; k < 9; ++k) {
        R* r = L.isa + k * kIsaCols;
        r[0] = P.isa_Hb[k]; r[1] = P.isa_Tb[k]; r[2] = P.isa_beta[k]; r[3] = P.isa_pb[k];
        r[4] = P.isa_bt[k]; r[5] = P.isa_ex[k]; r[6] = P.isa_iso[k]; r[7] = R(0);
    }
    if (WIND)
        for (int t = 0; t < 800; ++t) { L.walt[t] = (&P.wind_alt_km[0][0])[t]; L.wsp[t] = (&P.wind_speed[0][0])[t]; }
    for (int t = 0; t < 4 * kLineMax; ++t) (&L.lines.bp[0][0])[t] = (&P.line_bp[0][0])[t];
    for (int t = 0; t < 4 * (kLineMax + 1); ++t) {
        (&L.lines.slot[0][0])[t] = (&P.line_slot[0][0])[t];
        (&L.lines.key[0][0])[t] = (&P.line_key[0][0])[t];
    }
    for (int k = 0; k < 4; ++k) { L.lines.a[k] = P.line_a[k]; L.lines.nbp[k] = P.line_nbp[k]; L.lines.tay_off[k] = P.tay_off[k]; }
    for (int t = 0; t < 4 * kLineBuckets; ++t) (&L.lines.lb[0][0])[t] = (&P.line_lb[0][0])[t];
}

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
    unsigned int* ticket;        // [1] workgroups of the step launch that have finished (0 between launches)
};

// Insert the queued neighbourhoods into the device tables and empty the queue; one thread, with
// nothing else reading the tables (k_insert after a launch, or the last workgroup of a step launch
// once every other workgroup has finished).  Open addressing, load factor <= 1/2; a key already
// present is skipped.
template <typename R>
__device__ void insert_pending(unsigned long long* count, const unsigned long long* pkeys, const double* ppay,
                               unsigned long long* stats, unsigned long long* keys_cd, R* pay_cd, int lc_cd,
                               unsigned long long* keys_cl, R* pay_cl, int lc_cl) {
    unsigned long long cnt = *count;
    if (cnt == 0) return;
    if (cnt > (unsigned long long)kPendingCap) cnt = kPendingCap;
    for (unsigned long long e = 0; e < cnt; ++e) {
        const unsigned long long kk = pkeys[e];
        const int table = (int)(kk >> 63);
        const unsigned long long key = kk & ~(1ull << 63);
        unsigned long long* keys = table ? keys_cl : keys_cd;
        const int lc = table ? lc_cl : lc_cd;
        uint32_t mask = (1u << lc) - 1u, h = key_hash(key, lc);
        int slot = -1;
        for (uint32_t p = 0; p <= mask; ++p) {
            const unsigned long long k = keys[h];
            if (k == key) { slot = -1; break; }
            if (k == kEmptyKey) { slot = (int)h; break; }
            h = (h + 1) & mask;
        }
        if (slot >= 0 && stats[kStInsCd + table] * 2 + 2 > (1ull << lc)) slot = -1;
        if (slot < 0) continue;
        stats[kStInsCd + table] += 1;
        keys[slot] = key;
        pay_store<R>(ppay + e * kPay, (table ? pay_cl : pay_cd) + (int64_t)slot * pay_stride<R>());
    }
    *count = 0;
}

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
    R* info;                         // [n_fused][nsel][N]: the info fields of info_mask, in pd_info_field order
    uint64_t info_mask;              // (pd_step: every field, nsel = PD_N_INFO)
    int info_nsel;
    R* reward_sum;
    const float* policy_w;           // policy rollouts: actor parameters in chunks of four, [ceil(P/4)][N][4] float32
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
    // refill rollouts (pd_tuning.policy_refill): the grid holds refill_base env slots; an env whose
    // episode ends (or reaches refill_max steps) is stored and its lanes wait for the next particle,
    // which a wave hands out once `refill` of its slots wait (or none is live): refill_base + the
    // launch's count of handed-out particles so far (*refill_next, one atomic per hand-out), until
    // every particle of the swarm has run
    uint32_t* refill_next;
    int refill, refill_base, refill_max;
    int refill_slots, refill_q;   // (the slots; particles of a wave's own range, [w Q, (w + 1) Q))
};

// Kernel launchers, explicitly instantiated in the kstep_*.hip translation units.
template <typename R, int PH, int RT, bool W, int LPE, bool RK = false> void launch_step(const StepArgs<R>& a, hipStream_t s);
template <typename R, int PH, bool W, int LPE> void launch_policy_lpe(const StepArgs<R>& a, int64_t n_launch,
                                                                      hipStream_t s);

}  // namespace pd
