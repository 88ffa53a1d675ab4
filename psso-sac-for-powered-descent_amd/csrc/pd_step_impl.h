// pd_step_impl.h -- the step kernel k_step and its launchers (included by the kstep_*.hip
// translation units, each of which instantiates a subset; pdenv.hip sees pd_step.h only).
#pragma once
#include "pd_envdev.h"

namespace pd {

// ---------------------------------------------------------------- lane pairs
// Value of the partner lane (2k <-> 2k+1) by a DPP quad permutation [1,0,3,2] (no LDS
// crossbar).  Only at converged points of the wave.
__device__ __forceinline__ int dpp_swap1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ float pair_swap(float v) { return __int_as_float(dpp_swap1(__float_as_int(v))); }
__device__ __forceinline__ double pair_swap(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)dpp_swap1((int)(uint32_t)b), hi = (uint32_t)dpp_swap1((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// sin/cos of two angles of one env; with LPE >= 2 the env's even lane evaluates x0 and its odd
// lane x1 (one pass of the instruction stream for both), then they swap.
template <int LPE, typename R>
__device__ __forceinline__ void sincos_pair(R x0, R x1, int role, R& s0, R& c0, R& s1, R& c1) {
    if constexpr (LPE >= 2) {
        const bool odd = role & 1;
        R s, c;
        pd_sincos<R>(odd ? x1 : x0, s, c);
        const R so = pair_swap(s), co = pair_swap(c);
        s0 = odd ? so : s; c0 = odd ? co : c;
        s1 = odd ? s : so; c1 = odd ? c : co;
    } else {
        pd_sincos<R>(x0, s0, c0);
        pd_sincos<R>(x1, s1, c1);
    }
}
// a0 / b0 and a1 / b1 as one division per lane pair (LPE >= 2)
template <int LPE, typename R>
__device__ __forceinline__ void div_pair(R a0, R b0, R a1, R b1, int role, R& q0, R& q1) {
    if constexpr (LPE >= 2) {
        const bool odd = role & 1;
        const R q = (odd ? a1 : a0) / (odd ? b1 : b0);
        const R qo = pair_swap(q);
        q0 = odd ? qo : q; q1 = odd ? q : qo;
    } else {
        q0 = a0 / b0; q1 = a1 / b1;
    }
}

// ---------------------------------------------------------------- RBF lookup + evaluation
// Lanes-per-env (LPE) decomposition: with LPE = 1 one lane evaluates both tables; with
// LPE = 2 lane role 0 owns C_D and role 1 owns C_L; with LPE = 4/8/16 each table is owned by
// LPE/2 lanes that split its 50-term thin-plate sum (terms k = part, part + nparts, ..).
template <typename R> struct TabView {
    const R* smach;            // LDS: entry p = (Mach_p, Mach_p+1); smach[2p] = point p's Mach
    const PD_AS4 int* start;   // column geometry (uniform: scalar loads)
    const PD_AS4 int* n;
    const PD_AS4 R* aoa;
    const PD_AS1 unsigned long long* keys;
    const PD_AS1 R* pay;
    int logcap;
    int line0;                 // index of this table's first clamped line (0: C_D, 2: C_L)
    const PD_AS1 unsigned long long* grid_key;
    const PD_AS1 int* grid_slot;
    const PD_AS1 unsigned long long* sub_key;
    const PD_AS1 int* sub_slot;
    const PD_AS1 GridBisect* sub_bis;
    const PD_AS1 R* cell_pc;        // cell pieces (cell_stride<R>() words each; nullptr: none)
    const PD_AS1 int* sub_piece;
    const PD_AS1 uint32_t* fine;    // fine index (nullptr: none)
    int grid_nm, grid_na;
    R grid_a0, grid_inv_da, grid_inv_dm;
};

// LDS copy of the clamped-line interval tables

// One chunk (five pair slots, ten terms) of sum_j c_j phi(|x - y_j|), phi(r) = r^2 log r =
// d2 log(d2) / 2 with d2 = |x - y|^2 (thin_plate_spline, phi(0) = 0), times 8: the lane-
// independent unit of every evaluation order below, so that its bits do not depend on which lane
// computes it.  pp: the chunk's ten coefficients, w: its three index words.  Terms come in pair
// slots (pd_common.h): one 16-byte LDS read gives the Mach values of a slot's two consecutive
// table points, whose column AoA (an integer, in the slot's AoA byte) gives one d_a^2 for both.
// Binary64 evaluates in phases (five pair reads, ten d2, ten log-cell reads, ten finishes) so
// that the reads are in flight together and the ten log chains interleave.  d2 = 0 (query on a
// table point) contributes c_j * 0 * finite = 0, as do padding terms (c_j = 0).
template <typename R, typename R2>
__device__ __forceinline__ R chunk_sum(const R pp[10], const uint32_t w[3], const R2* pt, R M, R a) {
    R s0 = R(0), s1 = R(0);
    if constexpr (sizeof(R) == 8) {
        R2 v[5];
        R da2[6];
        R m5;     // the general slot's (u = 4) second point: its own entry and AoA
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const uint32_t h = w[u >> 1] >> (16 * (u & 1));
            if (u < 5) v[u] = pt[h & 0xffu]; else m5 = pt[h & 0xffu].x;
            const R da = a - (R)((h >> 8) & 0xffu);
            da2[u] = da * da;
        }
        R d2[10];
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const R dm0 = M - v[u].x, dm1 = M - (u == 4 ? m5 : v[u].y);
            d2[2 * u] = fma(dm0, dm0, da2[u]);
            d2[2 * u + 1] = fma(dm1, dm1, da2[u == 4 ? 5 : u]);
        }
        LogPart lp[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) lp[k] = log_start(d2[k]);
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const R wk = d2[k] * pp[k];
            if (k & 1) s1 = fma(wk, log4_finish(lp[k]), s1); else s0 = fma(wk, log4_finish(lp[k]), s0);
        }
    } else {
        const uint32_t h5 = w[2] >> 16;           // the general slot's second point
        const R m5 = pt[h5 & 0xffu].x;
        const R da5 = a - (R)((h5 >> 8) & 0xffu);
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const uint32_t h = w[u >> 1] >> (16 * (u & 1));
            const R2 v = pt[h & 0xffu];
            const R da = a - (R)((h >> 8) & 0xffu);
            const R da2 = da * da;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const R dm = M - (i ? (u == 4 ? m5 : v.y) : v.x);
                const R d2 = fma(dm, dm, (u == 4 && i) ? da5 * da5 : da2);
                const R l = eval_log4<R>(sizeof(R) == 8 ? d2 : (d2 > R(1e-30) ? d2 : R(1e-30)));
                if (i) s1 = fma(d2 * pp[2 * u + 1], l, s1); else s0 = fma(d2 * pp[2 * u], l, s0);
            }
        }
    }
    return s0 + s1;
}

// One parity half of chunk_sum: h = 0 its even terms (each slot's first point), h = 1 its odd
// terms (second points; the general slot's from its own entry), accumulated in chunk_sum's order
// with the same operations, so that chunk_sum(...) == chunk_half(.., 0) + chunk_half(.., 1) bit
// for bit (the balanced sums' last round deals half-chunks when it is at most half full).
template <typename R, typename R2>
__device__ __forceinline__ R chunk_half(const R pp[10], const uint32_t w[3], const R2* pt, R M, R a, int h) {
    R s = R(0);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        const uint32_t hw = w[u >> 1] >> (16 * (u & 1));
        const uint32_t hs = (h && u == 4) ? (w[2] >> 16) : hw;          // the general slot's second point
        const R2 v = pt[hs & 0xffu];
        const R m = (h && u < 4) ? v.y : v.x;
        const R da = a - (R)((hs >> 8) & 0xffu);
        const R dm = M - m;
        const R d2 = fma(dm, dm, da * da);
        if constexpr (sizeof(R) == 8) s = fma(d2 * pp[2 * u + h], log4_finish(log_start(d2)), s);
        else s = fma(d2 * pp[2 * u + h], eval_log4<R>(d2 > R(1e-30) ? d2 : R(1e-30)), s);
    }
    return s;
}

// The payload's degree-1 polynomial added to the scaled kernel sum (the same order everywhere);
// f: the payload's fields [kPayPoly, kPayPoly + 7) (poly coefficients, shifts, scales)
template <typename R>
__device__ __forceinline__ R rbf_finish_f(const R f[7], R tot, R M, R a) {
    R s = R(0.125) * tot;
    s += R(1) * f[0];
    s += (M - f[3]) / f[5] * f[1];
    s += (a - f[4]) / f[6] * f[2];
    return s;
}
template <typename R>
__device__ __forceinline__ R rbf_finish(const PD_AS1 R* __restrict__ pay, R tot, R M, R a) {
    R f[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) f[u] = pay[kPayPoly + u];
    return rbf_finish_f<R>(f, tot, M, a);
}

// This lane's share of sum_j c_j phi(|x - y_j|) + poly of one neighbourhood payload.
// nparts = 1 (the lane owns the query): the six chunks in order, each chunk_sum'd, the next
// chunk's coefficients and index words requested before the current one computes; the same
// bits as rbf_balanced's distributed evaluation.  nparts > 1 (LPE >= 4): the lane's slots are
// part, part + nparts, ... (summed by the caller's shuffles).
template <typename R>
__device__ __forceinline__ R rbf_eval(const PD_AS1 R* __restrict__ pay, const R* spt, R M, R a,
                                      int part, int nparts) {
    using R2 = typename std::conditional<sizeof(R) == 8, double2, float2>::type;
    const R2* pt = (const R2*)spt;
    const PD_AS1 uint32_t* iw = (const PD_AS1 uint32_t*)(pay + kPayIdx);
    if (nparts == 1) {
        R pn[10];
        uint32_t wn[3];
#pragma unroll
        for (int u = 0; u < 10; ++u) pn[u] = pay[u];
#pragma unroll
        for (int u = 0; u < 3; ++u) wn[u] = iw[u];
        R tot = R(0);
#pragma unroll 1
        for (int c = 0; c < kChunks; ++c) {
            R pp[10];
            uint32_t w[3];
            const int cn = c + 1 < kChunks ? c + 1 : c;   // (the last chunk reloads itself)
#pragma unroll
            for (int u = 0; u < 10; ++u) { pp[u] = pn[u]; pn[u] = pay[10 * cn + u]; }
#pragma unroll
            for (int u = 0; u < 3; ++u) { w[u] = wn[u]; wn[u] = iw[3 * cn + u]; }
            const R cs = chunk_sum<R, R2>(pp, w, pt, M, a);
            tot = c == 0 ? cs : tot + cs;
        }
        return rbf_finish<R>(pay, tot, M, a);
    }
    // LPE >= 4: this lane's chunks part, part + nparts, ... (the chunk sums of the LPE 2 path;
    // the caller adds the parts with shuffles)
    R tot = R(0);
#pragma unroll 1
    for (int c = part; c < kChunks; c += nparts) {
        R pp[10];
        uint32_t w[3];
#pragma unroll
        for (int u = 0; u < 10; ++u) pp[u] = pay[10 * c + u];
#pragma unroll
        for (int u = 0; u < 3; ++u) w[u] = iw[3 * c + u];
        tot = tot + chunk_sum<R, R2>(pp, w, pt, M, a);
    }
    if (part == 0) return rbf_finish<R>(pay, tot, M, a);
    return R(0.125) * tot;
}

// Orders this wave's global-memory accesses (the solve scratch is written and read back by the
// same wave: same CU, so an s_waitcnt on its stores is all the ordering it needs).
__device__ __forceinline__ void wave_mem_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Wave-cooperative exact solve of one neighbourhood into a global-memory scratch slot: lane r
// owns row r of the 53x53 system; LU with partial pivoting (pivot by a wave max-reduction,
// smallest row index on ties) and column-oriented back substitution -- the operations and
// their order per element are those of solve_neighbourhood(), so the payload is bit-identical
// to the host-built one.  Must be called by a converged wave (all 64 lanes active).  Leaves the
// binary64 payload at work + kScratch - kPay and the handle-precision payload at work.
template <typename R>
__device__ __forceinline__ void solve_wave(DP<R>& P, int table, unsigned long long key, PD_AS1 double* work) {
    const int lane = (int)__lane_id();
    PD_AS1 double* A = work;
    PD_AS1 double* b = A + kSys * kSys;
    PD_AS1 double* ym = b + kSys;
    PD_AS1 double* ya = ym + kNbr;
    PD_AS1 double* yd = ya + kNbr;
    PD_AS1 double* pay = work + (kScratch - kPay);
    const PD_AS4 double* mach = table ? P.cl_mach_d : P.cd_mach_d;
    const PD_AS4 double* coef = table ? P.cl_coef_d : P.cd_coef_d;
    const PD_AS4 int* start = table ? P.cl_start : P.cd_start;
    const PD_AS4 double* aoa = table ? P.cl_aoa_d : P.cd_aoa_d;
    int lo[kCols], len[kCols];
    key_unpack(key, lo, len);
    // lane < 50: term `lane` of the window order, column c, window offset off; its pair slot
    // my_slot and position my_pos (term_slot, the host packing's map)
    int my_idx = 0, my_c = 0, my_slot = 0, my_pos = 0;
    if (lane < kNbr) {
        int c = 0, off = lane, acc = 0;
#pragma unroll
        for (int q = 0; q < kCols; ++q) {
            if (lane >= acc && lane < acc + len[q]) { c = q; off = lane - acc; }
            acc += len[q];
        }
        int idx = start[c] + lo[c] + off;
        term_slot(len, lane, my_slot, my_pos);
        my_idx = idx; my_c = c;
        ym[lane] = mach[idx]; ya[lane] = aoa[c]; yd[lane] = coef[idx];
    }
    wave_mem_sync();
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
    wave_mem_sync();
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
            wave_mem_sync();
        }
        double r = 1.0 / A[k * kSys + k];
        if (lane > k && lane < kSys) {
            double l = A[lane * kSys + k] * r;
            if (l != 0.0)
                for (int j = k + 1; j < kSys; ++j) A[lane * kSys + j] -= l * A[k * kSys + j];
            b[lane] -= l * b[k];
        }
        wave_mem_sync();
    }
    if (!singular) {
        for (int i = kSys - 1; i >= 0; --i) {
            double xi = b[i] / A[i * kSys + i];
            wave_mem_sync();
            if (lane == i) b[i] = xi;
            if (lane < i) b[lane] -= A[lane * kSys + i] * xi;
            wave_mem_sync();
        }
    }
    // binary64 payload in the pair-slot layout of solve_neighbourhood (pd_common.h)
    for (int j = lane; j < kPay; j += 64) pay[j] = 0.0;
    wave_mem_sync();
    PD_AS1 uint8_t* ib = (PD_AS1 uint8_t*)(pay + kPayIdx);
    if (lane < kNbr) {
        pay[2 * my_slot + my_pos] = singular ? (double)NAN : b[lane];
        if (my_pos == 0) { ib[pair_entry_pos(my_slot)] = (uint8_t)my_idx; ib[pair_aoa_pos(my_slot)] = (uint8_t)aoa[my_c]; }
        else if (slot_general(my_slot)) { ib[second_entry_pos(my_slot)] = (uint8_t)my_idx; ib[second_aoa_pos(my_slot)] = (uint8_t)aoa[my_c]; }
    } else if (lane < kSys) {
        pay[kPayPoly + lane - kNbr] = singular ? (double)NAN : b[lane];
    } else if (lane == kSys) pay[kPaySS + 0] = sh0;
    else if (lane == kSys + 1) pay[kPaySS + 1] = sh1;
    else if (lane == kSys + 2) pay[kPaySS + 2] = sc0;
    else if (lane == kSys + 3) pay[kPaySS + 3] = sc1;
    wave_mem_sync();
    // payload in the kernel's precision, in the (now free) matrix area (pay_store, by lanes)
    PD_AS1 R* pr = (PD_AS1 R*)work;
    for (int j = lane; j < pay_stride<R>(); j += 64) pr[j] = j < kPayIdx ? (R)pay[j] : R(0);
    wave_mem_sync();
    for (int j = lane; j < kPayIdxBytes; j += 64) ((PD_AS1 uint8_t*)(pr + kPayIdx))[j] = ib[j];
    wave_mem_sync();
}

// Each distinct (table, key) missed by the wave is solved cooperatively into the workgroup's
// global scratch slot (under the slot's lock), evaluated by the lanes that need it, and queued
// for insertion into the device table (pd_flush_misses).  Called by the converged wave.
template <typename R, typename AT>
__device__ __forceinline__ R rbf_miss_wave(const AT& a, DP<R>& P, int table, const R* spt,
                                           unsigned long long key, R M, R aq,
                                           int part, int nparts, bool need) {
    R val = R(0);
    unsigned long long mm = __ballot(need);
    const unsigned slot = blockIdx.x % kSolveSlots;
    PD_AS1 double* work = gblw(a.pend.solve_ws) + (size_t)slot * kScratch;
    while (mm) {
        int leader = __ffsll((long long)mm) - 1;
        unsigned long long lk = ((unsigned long long)(unsigned int)__shfl((int)(key >> 32), leader) << 32) |
                                (unsigned int)__shfl((int)key, leader);
        int lt = __shfl(table, leader);
        if (__lane_id() == 0) {
            while (atomicCAS(&a.pend.solve_lock[slot], 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
        }
        wave_mem_sync();
        solve_wave<R>(P, lt, lk, work);
        if (need && key == lk && table == lt) {
            val = rbf_eval<R>((const PD_AS1 R*)work, spt, M, aq, part, nparts);
            need = false;
        }
        if ((int)__lane_id() == leader) {
            atomicAdd(&a.pend.stats[kStMisses], 1ull);
            unsigned long long idx = atomicAdd(a.pend.count, 1ull);
            const PD_AS1 double* pay = work + (kScratch - kPay);
            if (idx < (unsigned long long)kPendingCap) {
                for (int j = 0; j < kPay; ++j) a.pend.pay[idx * kPay + j] = pay[j];
                a.pend.keys[idx] = lk | ((unsigned long long)lt << 63);
                // (release, device scope: the entry reaches memory before this workgroup takes
                // its end-of-launch ticket, so the inserting workgroup on any XCD reads it)
                __threadfence();
            } else {
                atomicAdd(&a.pend.stats[kStDropped], 1ull);   // solved again until a later flush
            }
        }
        wave_mem_sync();
        if (__lane_id() == 0) atomicExch(&a.pend.solve_lock[slot], 0);
        mm = __ballot(need);
    }
    return val;
}

// The neighbourhood of `table` at (M, aq): its table slot (-1: not in the tables), the key in
// cache.key.  Candidate neighbourhood: on a clamped query line (the common case: |alpha_eff| > 0.003 rad
// clamps both tables) the interval table of that line (binary search over <= 96 Mach
// breakpoints in LDS); elsewhere the interior grid cell's, or the env's cached set.  Unless the
// candidate is trusted (strictly inside its interval/exact cell) it is VERIFIED (and repaired by
// the swap search) against the exact distances before it is used.
// A query's Taylor piece on a clamped line (rbf2): its record index and cell, piece < 0: none
// (line, verify, refined, bisect: the query was on a clamped line / its candidate was verified /
// it read a refined cell's sub-cell / a bisector record -- for the workload counters).  cp: a
// trusted interior query's cell piece (-1 none), cu, cv: its position in the cell, [0, 1); fine:
// the piece came from the fine index (the cached key is then the piece's)
struct TayRef { int piece, cell; bool line, verify, refined, bisect; int cp; double cu, cv; bool fine; };

struct NoPre { __device__ void operator()() const {} };


// pre(): the caller's work that does not depend on the tables, run while the grid loads are in
// flight
template <typename R, typename Pre = NoPre, typename AT>
__device__ __forceinline__ int rbf_lookup(const AT& a, DP<R>& P, int table, const TabView<R>& t,
                                          const LineLds<R>& ln, RbfCache<R>& cache, R M, R aq,
                                          TayRef* tay = nullptr, unsigned long long* st = nullptr,
                                          Pre&& pre = Pre()) {
#ifdef PD_STAMP
    unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#define PD_LST(k) if (st) { const unsigned long long ts1 = __builtin_amdgcn_s_memtime(); st[k] += ts1 - ts0; ts0 = ts1; }
#else
#define PD_LST(k)
#endif
    unsigned long long ckey = cache.key;
    int cslot = cache.slot;
    int li = aq == ln.a[t.line0] ? t.line0 : (aq == ln.a[t.line0 + 1] ? t.line0 + 1 : -1);
    bool trusted = false;
    const bool on_line = li >= 0 && ln.nbp[li] >= 0;
    // the interior grid cell's candidate is requested by every lane first (its global loads are
    // in flight during the line search; lanes on a line discard it)
    unsigned long long gkey = 0ull;
    int gsl0 = -1, gcell = 0;
    R um = R(0), ua = R(0);
    const bool use_grid = t.grid_key != nullptr;
    // handles with cell pieces read the query's sub-cell word of the fine index instead of the
    // cell record: one dependent load to the piece (or its bisector record) for refined cells
    // too; the cell / sub-cell records only when it does not settle the query
    const bool fine_path = tay != nullptr && t.fine != nullptr;
    uint32_t fe = 0u;
    R fsm = R(0), fsa = R(0);
    if (use_grid) {
        R fm = M * t.grid_inv_dm, fa = (aq - t.grid_a0) * t.grid_inv_da;
        int im = fm < R(0) ? 0 : (fm >= R(t.grid_nm) ? t.grid_nm - 1 : (int)fm);
        int ia = fa < R(0) ? 0 : (fa >= R(t.grid_na) ? t.grid_na - 1 : (int)fa);
        if (!(fm == fm) || !(fa == fa)) { im = 0; ia = 0; }   // NaN queries
        gcell = im * t.grid_na + ia;
        um = fm - (R)im; ua = fa - (R)ia;     // position in the cell, [0, 1)
        if (fine_path) {
            const R sm = um * R(kGridSub), sa = ua * R(kGridSub);
            int jm = (int)sm, ja = (int)sa;
            jm = jm < 0 ? 0 : (jm > kGridSub - 1 ? kGridSub - 1 : jm);
            ja = ja < 0 ? 0 : (ja > kGridSub - 1 ? kGridSub - 1 : ja);
            fe = t.fine[(uint32_t)(im * kGridSub + jm) * (uint32_t)(t.grid_na * kGridSub) + (uint32_t)(ia * kGridSub + ja)];
            fsm = sm - (R)jm; fsa = sa - (R)ja;
        } else {
            gkey = t.grid_key[gcell];
            gsl0 = t.grid_slot[gcell];
        }
    }
    pre();
    if (on_line) {
        const int nb = ln.nbp[li];
        // lower_bound of M over the breakpoints, within the bucket's range
        int bk = (int)(M * R(kLineBuckets / 10.0));
        bk = bk < 0 ? 0 : (bk > kLineBuckets - 1 ? kLineBuckets - 1 : bk);
        const uint32_t rg = ln.lb[li][bk];
        int l = (int)(rg & 0xffu), h = (int)(rg >> 8);
        if (!(M >= R(0) && M < R(10))) { l = 0; h = nb; }   // (outside the buckets: whole line)
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
        if (tay != nullptr && trusted && ln.tay_off[li] >= 0) {
            // strictly inside interval l: the piece of (cell, l), Mach in [0, 10]
            int cell = (int)(M * R(kTayCells / 10.0));
            cell = cell < 0 ? 0 : (cell > kTayCells - 1 ? kTayCells - 1 : cell);
            tay->piece = ln.tay_off[li] + cell + l;
            tay->cell = cell;
        }
        PD_LST(0);
    } else if (use_grid) {
        bool fast = false;
        if (fine_path) {
            // a piece every point of the sub-cell uses, or the side of its bisector, trusted off
            // the line.  The margin is the record path's, so that both paths trust the same
            // queries: a refined cell's sub-cell (and any bisector) in sub-cell coordinates, a
            // non-refined exact cell in cell coordinates (its sub-cell edges are no boundary).
            // Binary32 handles: 1e-4 cell widths as their record path, and 1e-3 sub-cell widths
            // (the binary32 position's rounding is ~5e-5 cell widths at the grid's far end)
            const R eps = sizeof(R) == 8 ? R(1e-9) : R(1e-4), eps_sub = sizeof(R) == 8 ? R(1e-9) : R(1e-3);
            const bool inside = (fe & kFineRefined)
                ? (fsm > eps_sub && R(1) - fsm > eps_sub && fsa > eps_sub && R(1) - fsa > eps_sub)
                : (um > eps && R(1) - um > eps && ua > eps && R(1) - ua > eps);
            int cpf = -1;
            if (fe & kFinePiece) cpf = (int)(fe & kFineIndex);
            else if (fe & kFineBisect) {
                const PD_AS1 GridBisect& b = t.sub_bis[fe & kFineIndex];
                const double sv = fma(b.nx, (double)M, fma(b.ny, (double)aq, -b.c));
                const int side = sv < 0.0 ? b.piece_a : b.piece_b;
                if (fabs(sv) > 3.0 * b.tau) cpf = side;
            }
            if (inside && cpf >= 0) {
                fast = true;
                trusted = true;
                cslot = -1;
                tay->cp = cpf; tay->cu = (double)um; tay->cv = (double)ua; tay->fine = true;
                tay->refined = (fe & kFineRefined) != 0u; tay->bisect = (fe & kFineBisect) != 0u;
            } else {
                gkey = t.grid_key[gcell];
                gsl0 = t.grid_slot[gcell];
            }
        }
        if (!fast) {
        ckey = gkey;
        int gsl = gsl0;
        // the cell piece (LPE 2 binary64 handles): an exact cell's own, else its sub-cell's
        const bool pieces = tay != nullptr && t.cell_pc != nullptr;
        const R cu = um, cv = ua;
        int cpc = pieces && gsl >= 0 && !(gsl & kGridRefine) && (gsl & kGridPiece) ? gcell : -1;
        if (sizeof(R) != 8 && gsl >= 0 && (gsl & kGridRefine)) gsl = -1;   // centre key, verified
        if (sizeof(R) == 8 && gsl >= 0 && (gsl & kGridRefine)) {
            // a cell that straddles neighbourhood regions: its sub-cell (binary64 handles; the
            // binary32 handle's rounding is too coarse for sub-cell margins and verifies instead)
            if (tay != nullptr) tay->refined = true;
            const int ref = gsl & (kGridRefine - 1);
            const R sm = um * R(kGridSub), sa = ua * R(kGridSub);
            int jm = (int)sm, ja = (int)sa;
            jm = jm < 0 ? 0 : (jm > kGridSub - 1 ? kGridSub - 1 : jm);
            ja = ja < 0 ? 0 : (ja > kGridSub - 1 ? kGridSub - 1 : ja);
            const int sc = (ref * kGridSub + jm) * kGridSub + ja;
            ckey = t.sub_key[sc];
            gsl = t.sub_slot[sc];
            if (pieces) cpc = t.sub_piece[sc];
            um = sm - (R)jm; ua = sa - (R)ja;
            if (gsl >= 0 && (gsl & kGridBisect)) {
                // two regions split by one bisector: the query's side (trusted off the line)
                if (tay != nullptr) tay->bisect = true;
                const PD_AS1 GridBisect& b = t.sub_bis[gsl & (kGridBisect - 1)];
                const double sv = fma(b.nx, (double)M, fma(b.ny, (double)aq, -b.c));
                const bool side_a = sv < 0.0;
                int sl = side_a ? b.slot_a : b.slot_b;
                ckey = side_a ? b.key_a : b.key_b;
                if (!(fabs(sv) > 3.0 * b.tau) && sl >= 0) sl &= ~kGridExact;
                gsl = sl;
                if (pieces) cpc = side_a ? b.piece_a : b.piece_b;
            }
        }
        cslot = gsl < 0 ? -1 : (gsl & (kGridPiece - 1));
        // every point of an exact cell has the cell's key (convexity of 50-NN regions); the
        // rounding margin keeps queries on a cell edge on the verified path
        const R eps = sizeof(R) == 8 ? R(1e-9) : R(1e-4);
        trusted = gsl >= 0 && (gsl & kGridExact) && um > eps && R(1) - um > eps && ua > eps && R(1) - ua > eps;
        if (pieces && trusted && cpc >= 0) { tay->cp = cpc; tay->cu = (double)cu; tay->cv = (double)cv; }
        }
    }
    PD_LST(1);
    unsigned long long key = ckey;
    int slot = cslot;
    if (tay != nullptr) { tay->line = on_line; tay->verify = !trusted; }
    if (!trusted) {
        int lo[kCols], len[kCols];
        key_unpack(ckey, lo, len);
        // keys store lo=0 for empty columns; knn_windows uses insertion points for those
        knn_windows<R>(t.smach, t.start, t.n, t.aoa, M, aq, lo, len);
        key = key_pack(lo, len);
        slot = key == ckey ? cslot : -1;
    }
    PD_LST(2);
    if (slot < 0 && !(tay != nullptr && tay->fine)) {   // (a fine-index piece needs no slot)
        uint32_t mask = (1u << t.logcap) - 1u;
        uint32_t h = key_hash(key, t.logcap);
        for (uint32_t probe = 0; probe <= mask; ++probe) {
            unsigned long long k = t.keys[h];
            if (k == key) { slot = (int)h; break; }
            if (k == kEmptyKey) break;
            h = (h + 1) & mask;
        }
    }
    PD_LST(3);
#undef PD_LST
    cache.key = key;
    cache.slot = slot;
    return slot;
}

// ---------------------------------------------------------------- LPE 2: Taylor lines + balanced sums
// A clamped-line query's value from its Taylor piece (pdenv.hip build_taylor): the degree-
// kTayDeg polynomial in M - (cell centre) plus the piece's exact terms.
template <typename R>
__device__ __forceinline__ R taylor_eval(const PD_AS1 R* __restrict__ rec, R M, int cell) {
    const R w = R(10.0 / kTayCells);
    const R t = M - fma((R)cell, w, R(0.5) * w);
    R c[kTayStride - 1];
#pragma unroll
    for (int n = 0; n < kTayStride - 1; ++n) c[n] = rec[n];
    R f = c[kTayDeg];
#pragma unroll
    for (int n = kTayDeg - 1; n >= 0; --n) f = fma(f, t, c[n]);
#pragma unroll
    for (int e = 0; e < kTayExact; ++e) {
        const R* x = c + kTayDeg + 1 + 3 * e;
        const R dm = M - x[0];
        const R d2 = fma(dm, dm, x[2]);
        f = fma(x[1] * d2, eval_log4<R>(sizeof(R) == 8 ? d2 : (d2 > R(1e-30) ? d2 : R(1e-30))), f);
    }
    return f;
}

// An interior query's value from its cell piece (pd_step.h kCellDeg, pdenv.hip
// build_cell_pieces): the polynomial in the cell coordinates u = 2 cu - 1, v = 2 cv - 1 (Horner
// in u over the rows' polynomials in v) plus the exact terms.  The host checks every piece at
// points of its cell in this order of operations.
// (binary32 handles: the same order in binary32 on the rounded records, host-checked against the
// binary64 pieces to 2e-6 of sum |c_j phi_j|; a zero distance is floored before the hardware log)
template <typename R>
__device__ __forceinline__ R cell_eval(const PD_AS1 R* __restrict__ rec, R M, R aq, R cu, R cv) {
    const R u = R(2) * cu - R(1), v = R(2) * cv - R(1);
    R f = R(0);
    int q = 0;
#pragma unroll
    for (int i = kCellDeg; i >= 0; --i) {
        R qi = rec[q++];
#pragma unroll
        for (int j = kCellDeg - i - 1; j >= 0; --j) qi = fma(qi, v, rec[q++]);
        f = i == kCellDeg ? qi : fma(f, u, qi);
    }
#pragma unroll
    for (int e = 0; e < kCellExact; ++e) {
        const PD_AS1 R* x = rec + kCellCoef + 3 * e;
        const R dm = M - x[0], da = aq - x[2];
        const R d2 = fma(dm, dm, da * da);
        f = fma(x[1] * d2, eval_log4<R>(sizeof(R) == 8 ? d2 : (d2 > R(1e-30) ? d2 : R(1e-30))), f);
    }
    return f;
}

// This lane's share of the RBF value of `table` at (M, aq): lookup, evaluation, and the
// wave-cooperative solve of missed neighbourhoods.
// Trusted clamped-line queries take their Taylor piece and trusted interior queries their cell
// piece (handles with pieces), as rbf2 does: every lane of the table's group evaluates the same
// piece (one pass of the instruction stream for all of them) and part 0 returns it, the other
// parts 0 -- the caller's shuffle sum then adds exact zeros.  The other queries split the payload
// sum over the parts.  PCS = false: payload sums for every hit (the kernels where the piece code
// would spill: wind, RK4, run-time-phase and landing-burn SAC instantiations).
template <bool PCS, typename R, typename AT>
__device__ __forceinline__ R rbf(const AT& a, DP<R>& P, int table, const TabView<R>& t, const LineLds<R>& ln,
                                 RbfCache<R>& cache, R M, R aq, int part, int nparts) {
    TayRef tr{-1, 0, false, false, false, false, -1, 0.0, 0.0, false};
    const int slot = rbf_lookup<R>(a, P, table, t, ln, cache, M, aq, PCS ? &tr : nullptr);
    const bool tay = tr.piece >= 0;
    const bool cel = tr.cp >= 0;
    R val = R(0);
    if (tay) val = taylor_eval<R>(gbl(P.tay) + (size_t)tr.piece * kTayStride, M, tr.cell);
    if (cel) {
        const PD_AS1 R* rec = t.cell_pc + (size_t)tr.cp * cell_stride<R>();
        val = cell_eval<R>(rec, M, aq, (R)tr.cu, (R)tr.cv);
        if (tr.fine) cache.key = *(const PD_AS1 unsigned long long*)(rec + cell_key<R>());
    }
    if ((tay || cel) && part != 0) val = R(0);
    if (!tay && !cel && slot >= 0) val = rbf_eval<R>(t.pay + (int64_t)slot * pay_stride<R>(), t.smach, M, aq, part, nparts);
    // Misses (a neighbourhood outside the pre-enumerated tables) take the wave-cooperative
    // exact solve; the loop in rbf_miss_wave runs only when some lane of the wave missed
    const bool miss = !tay && !cel && slot < 0;
    if (__ballot(miss)) {
        R mv = rbf_miss_wave<R>(a, P, table, t.smach, cache.key, M, aq, part, nparts, miss);
        if (miss) val = mv;
    }
    return val;
}

// Per-wave LDS of the balanced evaluation: the wave's payload queries by rank (Mach, AoA
// abscissa, table << 31 | slot) and the chunk sums of each
template <typename R> struct BalLds {
    alignas(16) R part[kChunks * 64];
    R qm[64];
    R qa[64];
    unsigned long long qp[64];   // payload address | table (bit 0)
    int wcnt[1];
};
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The payload sums of the wave's lanes with `mine` set, spread over all 64 lanes: the n queries'
// 6n chunks are numbered g = 6 rank + c and lane L computes chunks L, L + 64, ... (ceil(6n / 64)
// rounds instead of six per query); each chunk_sum goes to LDS and the query's lane adds its six
// in order -- the bits of rbf_eval (nparts = 1), whichever lanes computed the chunks.  `mid` runs
// once the first round's loads are in flight (the caller's own latency-bound work overlaps
// them).  Called by the converged wave.  (Dealing over the workgroup's four waves instead,
// with three workgroup barriers per call, measured 9 % slower: DESIGN.md s6.)
template <typename R, typename Mid>
__device__ __forceinline__ R rbf_balanced(DP<R>& P, BalLds<R>& B, const R* tab, bool mine, int table, int slot,
                                          R M, R aq, Mid&& mid) {
    using R2 = typename std::conditional<sizeof(R) == 8, double2, float2>::type;
    constexpr int NQ = 64;
    const unsigned long long mask = __ballot(mine);
    const int lane = (int)__lane_id();
    const int n = __popcll(mask);
    const int rank = __popcll(mask & ((1ull << lane) - 1ull));
    if (mask == 0ull) { mid(); return R(0); }
    const PD_AS1 R* pcd = gbl(P.pay_cd);
    const PD_AS1 R* pcl = gbl(P.pay_cl);
    const PD_AS1 R* own = (table ? pcl : pcd) + (size_t)(mine ? slot : 0) * pay_stride<R>();
    if (mine) { B.qm[rank] = M; B.qa[rank] = aq; B.qp[rank] = (unsigned long long)(uint64_t)own | (unsigned long long)table; }
    wave_lds_sync();
    const int total = kChunks * n;
    // full rounds of 64 chunks; a remainder of at most 32 chunks goes as 64 half-chunks in one
    // half-cost round (chunk_half, the same bits), a larger one as one more full round
    const int Kfull = total / NQ, rem = total - Kfull * NQ;
    const bool halfr = rem > 0 && rem <= NQ / 2;
    const int K = Kfull + (rem > NQ / 2 ? 1 : 0);
    // this lane's chunk in round r (round K: the half round's chunk, whose lane pair splits it)
    auto gidx = [&](int r) { return r < K ? r * NQ + lane : Kfull * NQ + (lane >> 1); };
    // chunk g's coefficients / index words / point table / query
    struct Buf { R pp[10]; uint32_t w[3]; const R2* pt; R M, a; };
    auto fetch = [&](int g, Buf& b) {
        const int gc = g < total ? g : total - 1;
        const int r = gc / kChunks, c = gc - kChunks * r;
        const unsigned long long q = B.qp[r];
        b.M = B.qm[r]; b.a = B.qa[r];
        const PD_AS1 R* pay = (const PD_AS1 R*)(uint64_t)(q & ~1ull) + 10 * c;
        const PD_AS1 uint32_t* iw = (const PD_AS1 uint32_t*)(pay + (kPayIdx - 10 * c)) + 3 * c;
#pragma unroll
        for (int u = 0; u < 10; ++u) b.pp[u] = pay[u];
#pragma unroll
        for (int u = 0; u < 3; ++u) b.w[u] = iw[u];
        b.pt = (const R2*)(tab + ((q & 1ull) ? 512 : 0));
    };
    auto run = [&](int g, const Buf& b) {
        const R cs = chunk_sum<R, R2>(b.pp, b.w, b.pt, b.M, b.a);
        if (g < total) B.part[g] = cs;
    };
    Buf b0, b1;
    fetch(gidx(0), b0);
    R pf[7];   // the own query's polynomial fields, requested with the first round
#pragma unroll
    for (int u = 0; u < 7; ++u) pf[u] = own[kPayPoly + u];
    mid();
    // two rounds per trip, ping-pong buffers: each round's loads are requested one round early
#pragma unroll 1
    for (int k = 0; k < K; k += 2) {
        const int g = k * NQ + lane;
        fetch(gidx(k + 1), b1);
        run(g, b0);
        if (k + 1 < K) {
            fetch(gidx(k + 2), b0);
            run(g + NQ, b1);
        }
    }
    if (halfr) {
        // the half round (its data fetched by the last full round, or up front): lane 2j + h
        // sums half h of chunk Kfull * 64 + j; the query abscissae B.qm are no longer read, so
        // they hold the halves until the pairs are added
        const bool odd = K & 1;     // (element-wise selects: a reference to b0 / b1 would put both in scratch)
        R hp[10];
        uint32_t hwd[3];
#pragma unroll
        for (int u = 0; u < 10; ++u) hp[u] = odd ? b1.pp[u] : b0.pp[u];
#pragma unroll
        for (int u = 0; u < 3; ++u) hwd[u] = odd ? b1.w[u] : b0.w[u];
        const R hsum = chunk_half<R, R2>(hp, hwd, odd ? b1.pt : b0.pt, odd ? b1.M : b0.M, odd ? b1.a : b0.a, lane & 1);
        wave_lds_sync();
        B.qm[lane] = hsum;
        wave_lds_sync();
        if (lane < rem) B.part[Kfull * NQ + lane] = B.qm[2 * lane] + B.qm[2 * lane + 1];
    }
    wave_lds_sync();
    R val = R(0);
    if (mine) {
        const R* pr = B.part + kChunks * rank;
        R tot = pr[0];
#pragma unroll
        for (int c = 1; c < kChunks; ++c) tot = tot + pr[c];
        val = rbf_finish_f<R>(pf, tot, M, aq);
    }
    // (B is reused by the next call)
    wave_lds_sync();
    return val;
}

// rbf() for LPE 2 (one query per lane): trusted clamped-line queries from their Taylor piece,
// the other table hits by the balanced payload sums, misses by the cooperative solve (whose
// evaluation, rbf_eval, has the balanced sums' bits).  Lanes with act = false (past the batch,
// frozen policy envs) only take part.
template <typename R, typename Pre, typename AT>
__device__ __forceinline__ R rbf2(const AT& a, DP<R>& P, int table, const TabView<R>& t, const LineLds<R>& ln,
                                  RbfCache<R>& cache, R M, R aq, bool act, BalLds<R>& B, const R* tab,
                                  WaveCount& wc, Pre&& pre, unsigned long long* stamp = nullptr) {
#ifdef PD_STAMP
    const unsigned long long s0 = __builtin_amdgcn_s_memtime();
#endif
    TayRef tr{-1, 0, false, false, false, false, -1, 0.0, 0.0, false};
    const int slot = rbf_lookup<R>(a, P, table, t, ln, cache, M, aq, &tr, stamp ? stamp + 2 : nullptr, pre);
#ifdef PD_STAMP
    const unsigned long long s1 = __builtin_amdgcn_s_memtime();
    stamp[0] += s1 - s0;
#endif
    const bool tay = act && tr.piece >= 0;
    const bool cel = act && tr.cp >= 0;   // (binary64 handles only)
    const bool full = act && !tay && !cel && slot >= 0;
    R vt = R(0);
    R vb;
    if (sizeof(R) == 8 || t.cell_pc != nullptr) {
        // with cell pieces the payload sums are rare (verified queries): the pieces first, then
        // the balanced sums of the lanes left, if any
        if (tay) vt = taylor_eval<R>(gbl(P.tay) + (size_t)tr.piece * kTayStride, M, tr.cell);
        if (cel) {
            const PD_AS1 R* rec = t.cell_pc + (size_t)tr.cp * cell_stride<R>();
            vt = cell_eval<R>(rec, M, aq, (R)tr.cu, (R)tr.cv);
            if (tr.fine) cache.key = *(const PD_AS1 unsigned long long*)(rec + cell_key<R>());
        }
        vb = rbf_balanced<R>(P, B, tab, full, table, slot, M, aq, []() {});
    } else {
        vb = rbf_balanced<R>(P, B, tab, full, table, slot, M, aq, [&]() {
            if (tay) vt = taylor_eval<R>(gbl(P.tay) + (size_t)tr.piece * kTayStride, M, tr.cell);
        });
    }
    R val = full ? vb : vt;
#ifdef PD_STAMP
    const unsigned long long s2 = __builtin_amdgcn_s_memtime();
    stamp[1] += s2 - s1;
#endif
    const bool miss = act && !tay && !cel && slot < 0;
    if (wc.w) {
        const int nf = __popcll(__ballot(full));
        wc.add(kStQLine - kStWork, act && tr.line);
        wc.add(kStQVerify - kStWork, act && tr.verify);
        wc.add(kStQTaylor - kStWork, tay);
        wc.add(kStQCell - kStWork, cel);
        wc.add_n(kStQBal - kStWork, nf);
        wc.add(kStQMiss - kStWork, miss);
        wc.add_n(kStBalRounds - kStWork, (kChunks * nf + 63) >> 6);
        wc.add(kStQRefined - kStWork, act && tr.refined);
        wc.add(kStQBisect - kStWork, act && tr.bisect);
        wc.add_n(kStWRefined - kStWork, __ballot(act && tr.refined) != 0ull);
        wc.add_n(kStWBisect - kStWork, __ballot(act && tr.bisect) != 0ull);
        wc.add_n(kStWMixed - kStWork, (__ballot(act && tr.line) != 0ull) && (__ballot(act && !tr.line) != 0ull));
    }
    if (__ballot(miss)) {
        R mv = rbf_miss_wave<R>(a, P, table, t.smach, cache.key, M, aq, 0, 1, miss);
        if (miss) val = mv;
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

// ---------------------------------------------------------------- the fused actor
// simple_actor.forward (env_wrapped_ea.py:18-44): Linear(IN,8)-ReLU-[Linear(8,8)-ReLU]xNL-
// Linear(8,OUT)-Tanh in binary32 on the float32-cast observation.  Parameters are in
// named_parameters() order (weight [out][in] row-major, then bias, layer by layer), stored
// parameter-major [P][N] so that every load is coalesced across the envs of a wave.
// Each output is the sequential sum over inputs (no FMA) plus the bias; tanh is evaluated in
// binary64 and rounded (the oracle restates the same order: oracle/pd_oracle.c orc_actor).
// The parameters are read in memory order through one running per-lane byte offset from the
// single SGPR base of W (weight q of this lane's particle at ui * 4 + q * 4 N; N * P * 4 < 2^32,
// validated by pd_rollout_policy), laundered after each step so that no offset is precomputed
// and held: with constant 64-bit addresses the compiler kept ~370 SGPR pairs live and spilled
// them.  Each output is still its own sequential sum plus the bias (the loads of a layer's
// weights come first, then its biases).
// SPLIT (LPE >= 2): the env's lane pair shares each layer -- lane half = 0 computes hidden units
// 0-3 and half = 1 units 4-7 (each unit the same sequential sum from the same loads), then one DPP
// swap per unit gives both lanes all eight; the output layer splits the same way when OUT is even.
// Half the loads and arithmetic per lane, the same bits (which lane sums a unit does not enter).
template <int IN, int NL, int OUT, bool SPLIT = false>
__device__ __forceinline__ void actor_forward(const float* __restrict__ W, int64_t N, uint32_t ui,
                                              int half, const float* x, float* y) {
    // W: the parameters in chunks of four, [ceil(P / 4)][N][4] (pdenv.hip k_wchunk): chunk c of
    // env ui holds parameters 4c .. 4c + 3 of its particle, 16 bytes, so one 16-byte load per lane
    // (512 contiguous bytes per wave) brings four parameters -- a quarter of the load instructions
    // of the parameter-major [P][N] layout, the same bytes.  Every block a lane reads starts at a
    // multiple of four parameters (the hidden rows are 8 long, the layer-1 blocks 4 IN, the biases
    // start at multiples of 4); the sums run in the same order as before: the same bits.
    constexpr int H = 8;
    constexpr int HS = SPLIT ? H / 2 : H;                          // hidden units per lane
    constexpr bool OSPLIT = SPLIT && OUT % 2 == 0;
    constexpr int OS = OSPLIT ? OUT / 2 : OUT;                     // outputs per lane
    static_assert((HS * IN) % 4 == 0 && (H * IN) % 4 == 0, "layer-1 blocks of whole chunks");
    using F4 = __attribute__((ext_vector_type(4))) float;
    float h[H], g[H];
    uint32_t sv = (uint32_t)N * 16u;                               // one chunk row
    uint32_t o0 = ui * 16u;
    uint32_t hv = SPLIT ? (uint32_t)half : 0u;
    asm volatile("" : "+v"(sv), "+v"(o0), "+v"(hv));
    // n parameters from parameter p (a multiple of 4) + this lane's half (`rows` parameters)
    auto load = [&](float* dst, int p, int rows, int n) {
        uint32_t off = o0 + (uint32_t)(p >> 2) * sv;
        if constexpr (SPLIT) off += hv * ((uint32_t)(rows >> 2) * sv);
        asm volatile("" : "+v"(off));
#pragma unroll
        for (int c = 0; c < (n + 3) / 4; ++c) {
            const F4 v = *(const PD_AS1 F4*)((const PD_AS1 char*)(uint64_t)W + off + (uint32_t)c * sv);
#pragma unroll
            for (int k = 0; k < 4; ++k) if (4 * c + k < n) dst[4 * c + k] = v[k];
        }
    };
    // both halves of a split layer on both lanes: own[j] is unit hs * HS + j of this lane's half
    auto gather = [&](const float* own, float* full, int n) {
#pragma unroll
        for (int j = 0; j < (SPLIT ? H / 2 : H); ++j) {
            if (j >= n) break;
            if constexpr (SPLIT) {
                const float oth = pair_swap(own[j]);
                full[j] = hv ? oth : own[j];
                full[n + j] = hv ? own[j] : oth;
            } else {
                full[j] = own[j];
            }
        }
    };
    int p = 0;
    float hs[HS];
    // layer 1: Linear(IN, 8)
    {
        float w[HS * IN], b[HS];
        load(w, p, HS * IN, HS * IN);
        load(b, p + H * IN, HS, HS);
#pragma unroll
        for (int j = 0; j < HS; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < IN; ++k) acc = acc + w[j * IN + k] * x[k];
            g[j] = acc;
        }
#pragma unroll
        for (int j = 0; j < HS; ++j) {
            const float acc = g[j] + b[j];
            hs[j] = acc < 0.f ? 0.f : acc;
        }
    }
    p += H * IN + H;
    if constexpr (SPLIT) gather(hs, h, HS);
    else {
#pragma unroll
        for (int j = 0; j < H; ++j) h[j] = hs[j];
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
#pragma unroll
        for (int j = 0; j < HS; ++j) {
            float w[H];
            load(w, p + j * H, HS * H, H);
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < H; ++k) acc = acc + w[k] * h[k];
            g[j] = acc;
        }
        float b[HS];
        load(b, p + H * H, HS, HS);
#pragma unroll
        for (int j = 0; j < HS; ++j) {
            const float acc = g[j] + b[j];
            hs[j] = acc < 0.f ? 0.f : acc;
        }
        p += H * H + H;
        if constexpr (SPLIT) gather(hs, h, HS);
        else {
#pragma unroll
            for (int j = 0; j < H; ++j) h[j] = hs[j];
        }
    }
    float o[OS], ys[OS];
#pragma unroll
    for (int j = 0; j < OS; ++j) {
        float w[H];
        load(w, p + j * H, OSPLIT ? OS * H : 0, H);
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < H; ++k) acc = acc + w[k] * h[k];
        o[j] = acc;
    }
    // the output biases: parameters p + OUT H + hv OS .. (+ OS), inside one chunk (OUT <= 4)
    {
        const int pb = p + OUT * H;
        float bb[4];
        load(bb, pb, 0, 4);
        const int sh = OSPLIT ? (int)hv * OS : 0;
#pragma unroll
        for (int j = 0; j < OS; ++j) ys[j] = (float)tanh((double)(o[j] + (sh ? bb[OS + j] : bb[j])));
    }
    if constexpr (OSPLIT) gather(ys, y, OS);
    else {
#pragma unroll
        for (int j = 0; j < OUT; ++j) y[j] = ys[j];
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

// ---------------------------------------------------------------- LDS of one step workgroup
// (the tables every workgroup stages come first: StepStatic, pd_step.h, copied from the handle's
// image of it)
template <typename R, bool WIND, int EPB, bool BAL = false> struct StepLds : StepStatic<R, WIND> {
    R gwin[10][EPB];              // the g-load ring of each env of the workgroup (register-resident launches)
    uint32_t work[kStepBlock / 64][kNWork];   // per-wave workload counts (counting launches)
    double wnx[WIND ? 2 : 1][WIND ? kStepBlock : 1];   // each lane's gust normals of the next (odd) sub-step
    BalLds<R> bal[BAL ? kStepBlock / 64 : 1];   // LPE 2: balanced-sum space per wave
    TabView<R> tdesc[2];          // each table's view, staged once: a lane's table is per lane
};

// A lane's table view from the workgroup's LDS copy (two entries; lanes of one wave read at most
// two addresses): its fields then come from LDS, not from lane-indexed global loads of the
// parameters at the head of every lookup
template <typename R>
__device__ __forceinline__ TabView<R> tab_view_lds(const TabView<R>* d, int table) { return d[table]; }
template <typename R>
__device__ __forceinline__ TabView<R> tab_view(DP<R>& P, const R* tab, int table) {
    TabView<R> t;
    t.smach = tab + (table ? 512 : 0);
    t.start = table ? &P.cl_start[0] : &P.cd_start[0];
    t.n = table ? &P.cl_len[0] : &P.cd_len[0];
    t.aoa = table ? &P.cl_aoa[0] : &P.cd_aoa[0];
    t.keys = gbl(table ? P.keys_cl : P.keys_cd);
    t.pay = gbl(table ? P.pay_cl : P.pay_cd);
    t.logcap = table ? P.logcap_cl : P.logcap_cd;
    t.line0 = table ? 2 : 0;
    t.grid_key = gbl(P.grid_key[table]);
    t.grid_slot = gbl(P.grid_slot[table]);
    t.sub_key = gbl(P.sub_key[table]);
    t.sub_slot = gbl(P.sub_slot[table]);
    t.sub_bis = gbl((const GridBisect*)P.sub_bis[table]);
    t.cell_pc = gbl(P.cell_pc[table]);
    t.sub_piece = gbl(P.sub_piece[table]);
    t.fine = gbl(P.fine[table]);
    t.grid_nm = P.grid_nm[table];
    t.grid_na = P.grid_na[table];
    t.grid_a0 = P.grid_a0[table];
    t.grid_inv_da = P.grid_inv_da[table];
    t.grid_inv_dm = P.grid_inv_dm[table];
    return t;
}

// ---------------------------------------------------------------- the step kernel
// One launch = n_fused consecutive env-steps of every env (or, POL, one policy step of the live
// envs).  The env's state is loaded once into registers (its g-load ring into LDS), the steps
// run in registers with their per-step outputs written as they go (row f of every [F][N]
// output), auto-reset happens in registers, and the state is stored once at the end.
// RK4 (pd_config.integrator = PD_INTEG_RK4, pure throttle without wind): NOT the reference's
// integrator -- BASELINE config c2's "RK4 dt=0.01 s", classical RK4 over (x, y, vx, vy, theta,
// theta_dot, m, m_prop) with rocket_physics_fcn's forces at each stage, 10 x 0.01 s per env step;
// the loop body below runs once per stage (oracle: orc_physics, ORC_INTEG_RK4, same order)
// CNT: the counting instantiation (pd_count_work; LPE 2 step kernels): without it every counting
// site folds away.  SAC: the pd_step_sac instantiation (RL landing burns): action sampling from
// the actor heads and the float32 transition-slab / next-observation epilogue
template <typename R, int PHASE, int RTD, bool WIND, int LPE, int POL = 0, bool RK4 = false, bool CNT = false,
          bool SAC = false>
// waves_per_eu(2): caps VGPR+AGPR at 256 so the f64 kernel keeps two waves per SIMD
__global__ __launch_bounds__(kStepBlock) __attribute__((amdgpu_waves_per_eu(2))) void k_step(StepArgs<R> a_) {
    SA<R>& a = kargs<R>();
    static_assert(sizeof(a_) > 0);
    constexpr int EPB = kStepBlock / LPE;   // envs per workgroup
    __shared__ StepLds<R, WIND, EPB, LPE == 2> L;
#ifdef PD_STAMP
    unsigned long long acc_[17] = {};   // [7], [8]: rbf2 lookup, evaluation; [9..12] lookup parts; [13..16] post-aero parts
#endif
    PD_T(t_start);
    // envs this launch steps: all N, or (POL) the compacted live list; a workgroup past its end
    // leaves before staging the tables (workgroup-uniform)
    int64_t n_act = a.n;
    // (refill rollouts in the windless policy kernels only: the windy ones have no registers to
    // spare for the particle reload; the host steps windy swarms by per-check launches)
    constexpr bool kRefill = POL && !WIND;
    // ring mode of pd_step_sac_ring: the ring position this launch writes at (every workgroup
    // reads it before the last one advances it, see the end of the kernel)
    int64_t ring_pos0 = 0;
    if constexpr (SAC) { if (a.ring_state) ring_pos0 = (int64_t)__atomic_load_n(a.ring_state, __ATOMIC_RELAXED); }
    if constexpr (POL) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *a.cnt_zero = 0u;
        // (refill: the grid's first refill_slots envs are the slots; the rest of its last
        // workgroup runs private copies, as past the end of any grid)
        if (kRefill && a.refill) n_act = a.refill_slots;
        if (a.use_list) {
            n_act = (int64_t)*a.cnt_in;
            if ((int64_t)blockIdx.x * EPB >= n_act) return;
        }
    }
    const int64_t N = a.n;
    const int64_t gt = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
    // Every lane stays active (the cooperative miss solve needs converged waves).  Lanes past the
    // end run a private copy of the initial state (no loads of another env's state, no stores).
    // (mutable: a refill rollout hands the lanes of an ended episode the next particle)
    bool valid = gt / LPE < n_act;
    const bool slot = valid;   // (refill: the lanes of one of the launch's env slots)
    bool drained = false;      // (refill: the swarm's particles all handed out; wave-uniform)
    int64_t e_act = valid ? gt / LPE : n_act - 1;
    // refill: wave w of the grid owns particles [w Q, (w + 1) Q) (refill_q = Q), its slots
    // starting on the first of them and taking the rest without any atomic; the particles from
    // refill_base on are the shared pool
    int rq_next = 0;   // (refill: this wave's next own particle, wave-uniform)
    if constexpr (kRefill) {
        if (a.refill && valid) {
            constexpr int kEpw = 64 / LPE;
            const int64_t gw = gt >> 6;
            e_act = gw * (int64_t)a.refill_q + (int64_t)(((int)gt & 63) / LPE);
            rq_next = kEpw;
        }
    }
    int64_t i = (POL && a.use_list) ? (int64_t)a.list_in[e_act] : e_act;
    const int role = (int)(gt % LPE);
    const int le = (int)threadIdx.x / LPE;   // the env's column of the workgroup's LDS g-load ring
    uint32_t ui = (uint32_t)i;   // N <= 2^25 (validated): 32-bit per-lane byte offsets
    // POL (policy rollout): with the list, only live envs are stepped; without it, finished
    // envs stay frozen and a wave with none left exits (wave-uniform, after the only barrier)
    bool live = valid;
    if constexpr (POL) {
        if (!a.use_list) live = live && ev(a.b.fin, ui) == 0;
    }
    // role -> (table, part): LPE 1: both tables on one lane; else table = role / (LPE/2)
    constexpr int nparts = LPE >= 2 ? LPE / 2 : 1;
    const int my_table = LPE >= 2 ? role / nparts : 0;   // 0 = C_D, 1 = C_L
    const int part = LPE >= 2 ? role % nparts : 0;
    const int gbase = (int)__lane_id() & ~(LPE - 1);
    uint64_t g = a.env_offset + (uint64_t)i;

    // ---- the env's state into registers (its g-load ring into LDS; the ring is not part of the
    // staged tables, so its stores may precede the staging barrier): requested ahead of the actor
    // prologue and the table staging, whose latencies then overlap it
    EnvRegs<R> e;
    RbfCache<R> cA, cB;   // LPE 1: A = C_D, B = C_L; LPE >= 2: A = own table
    auto load_env = [&]() {
        DP<R>& P = *params<R>(a.P);
#pragma unroll
        for (int k = 0; k < 11; ++k) e.s[k] = valid ? ldv(a.b.st + (k) * N, ui) : P.state0[k];
        e.vprev = valid ? ldv(a.b.vprev, ui) : sqrt(e.s[2] * e.s[2] + e.s[3] * e.s[3]);
        e.glen = valid ? (int)ldv(a.b.glen, ui) : 0;
        e.ghead = valid ? (int)ldv(a.b.ghead, ui) : 0;
#pragma unroll
        for (int k = 0; k < 10; ++k) L.gwin[k][le] = valid ? ldv(a.b.gwin + (k) * N, ui) : R(0);
        e.act0 = R(0); e.act1 = R(0); e.act2 = R(0);
        if constexpr (PHASE == 1 || PHASE == 2) e.act0 = valid ? ldv(a.b.act, ui) : R(0);
        if constexpr (PHASE == 1) {
            e.act1 = valid ? ldv(a.b.act + N, ui) : R(0);
            e.act2 = valid ? ldv(a.b.act + (2) * N, ui) : R(0);
        }
        e.fu0 = R(0); e.fu1 = R(0); e.fv0 = R(0); e.fv1 = R(0); e.sgu = R(0); e.sgv = R(0); e.prof = 0;
        if constexpr (WIND) {
            if (valid) {
                e.fu0 = ldv(a.b.wind, ui); e.fu1 = ldv(a.b.wind + N, ui);
                e.fv0 = ldv(a.b.wind + (2) * N, ui); e.fv1 = ldv(a.b.wind + (3) * N, ui);
                e.sgu = ldv(a.b.wind + (4) * N, ui); e.sgv = ldv(a.b.wind + (5) * N, ui);
                e.prof = ldv(a.b.wprof, ui);
            }
        }
        e.ep = valid ? ldv(a.b.epi, ui) : 0u;
        e.ts = valid ? ldv(a.b.tstep, ui) : 0u;
        e.tid = valid ? (int)ldv(a.b.tid, ui) : 0;
        cA.key = valid ? ldv(a.b.key + (my_table) * N, ui) : (my_table ? P.init_key_cl : P.init_key_cd);
        cA.slot = valid ? ldv(a.b.slot + (my_table) * N, ui) : -1;
        if constexpr (LPE == 1) { cB.key = valid ? ldv(a.b.key + N, ui) : P.init_key_cl; cB.slot = valid ? ldv(a.b.slot + N, ui) : -1; }
        else { cB.key = 0; cB.slot = -1; }
    };
    load_env();
    // the static tables: one 16-byte vector copy of the handle's image of them (pdenv.hip
    // fill_step_static: the same values, the grid-fin slopes by the same division), every load of
    // a thread issued here -- ahead of the SAC actor's prologue, whose first waits then cover
    // their latency -- and stored after it; then the eval_log cells
    constexpr int kImg = (int)(sizeof(StepStatic<R, WIND>) / 16);
    constexpr int kLog = (int)(sizeof(LogTableD) / 16);
    constexpr int kPer = (kImg + kLog + kStepBlock - 1) / kStepBlock;
    using V4 = __attribute__((ext_vector_type(4))) unsigned int;
    V4 stg[kPer];
    {
        DP<R>& P = *params<R>(a.P);
        const PD_AS1 V4* img = (const PD_AS1 V4*)P.stage_img;
        const PD_AS1 V4* lgt = (const PD_AS1 V4*)(uint64_t)&P.logtab_d.cell[0];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int t = threadIdx.x + k * kStepBlock;
            if (t < kImg) stg[k] = img[t];
            else if (t < kImg + kLog) stg[k] = lgt[t - kImg];
        }
    }
    // pd_step_sac_fused (16 lanes per env: the workgroup's 16 envs are one MLP tile): the actor's
    // heads of this step from the observation the previous step left in obs32, into s_sach (read
    // by the sampling below; the staging barrier orders them), before anything else of the step
    constexpr bool kSacMlp = SAC && LPE == 16;
    __shared__ __attribute__((aligned(16))) float s_mlp[kSacMlp ? sac_mlp_lds_floats<256>() : 1];
    __shared__ float s_sach[kSacMlp ? kSacTile * 16 : 1];
    if constexpr (kSacMlp) {
        const int H = a.sac_mlp.H;   // (grid-uniform: the barriers inside are reached by every thread)
        if (H) {
            const int64_t e0 = (int64_t)blockIdx.x * kSacTile;
            const int A2 = a.sac_mlp.A;
            auto put = [&](int e, int o, float v) {
                s_sach[e * 16 + (o < A2 ? o : 8 + o - A2)] = v;
                if (a.sac_heads_out && e0 + e < a.n) a.sac_heads_out[(e0 + e) * 2 * A2 + o] = v;
            };
            if (H == 128) sac_mlp_tile<128>(a.sac_mlp, a.n, e0, s_mlp, put);
            else sac_mlp_tile<256>(a.sac_mlp, a.n, e0, s_mlp, put);
            __syncthreads();   // (s_mlp is free again; the heads wait for the staging barrier)
        }
    }
    {
        DP<R>& P = *params<R>(a.P);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int t = threadIdx.x + k * kStepBlock;
            if (t < kImg) ((V4*)static_cast<StepStatic<R, WIND>*>(&L))[t] = stg[k];
            else if (t < kImg + kLog) ((V4*)s_logtab)[t - kImg] = stg[k];
        }
        if (threadIdx.x < (kStepBlock / 64) * kNWork) (&L.work[0][0])[threadIdx.x] = 0u;
        if (threadIdx.x < 2) L.tdesc[threadIdx.x] = tab_view<R>(P, L.tab, (int)threadIdx.x);
    }
    __syncthreads();
    PD_T(t_staged);
    PD_ACC(0, t_staged - t_start);
    if constexpr (POL) {
        // a wave whose envs have all finished leaves (wave-uniform, after the only barrier)
        if (!a.use_list && __ballot(live) == 0) return;
    }
    // PHASE 2 = the other compile_physics phases, chosen at run time by P.phase (wave-uniform)
    const int aux = PHASE == 2 ? params<R>(a.P)->phase : PHASE;
    const bool ascent = PHASE == 2 && (aux == PD_PHASE_SUBSONIC || aux == PD_PHASE_SUPERSONIC);
    constexpr int A = PHASE == 0 ? 1 : (PHASE == 1 ? 4 : 2);
    const int AD = PHASE == 2 ? (ascent ? 2 : 1) : A;   // row stride of the action array
    // pure throttle 4 x 0.025 s, landing_burn 4 x 0.1 s (actuators 0.025 s); the other phases
    // one call of rocket_physics_fcn at dt, actuators at the same dt (rockets_physics.py:728-997)
    static_assert(!RK4 || (PHASE == 0 && !WIND && !POL), "RK4: pure throttle, no wind, no policy");
    constexpr int NSUB = RK4 ? 40 : (PHASE == 2 ? 1 : 4);
    // LPE != 2: pieces for the trusted queries (rbf) where they fit the register file without
    // spilling (no wind, no RK4, not the landing-burn SAC kernel): c2, c5, the policy sweep
    // the tabulated atmosphere where it pays: binary32 handles and the windless kernels (c2, c4,
    // c5); the binary64 wind kernels (c3) keep the exact path (pd_physics.h atmosphere)
    constexpr bool kAtmTab = sizeof(R) == 4 || !WIND;
    // (LPE 16 measured 6 % slower with them: its split payload sum is as short as a piece)
    constexpr bool kPcs = !WIND && !RK4 && LPE <= 8 && (PHASE == 0 || (PHASE == 1 && !SAC));
    const R dt = RK4 ? R(0.01) : (PHASE == 0 ? R(0.025) : (PHASE == 1 ? R(0.1) : (R)a.dt_aux));
    const R dt_act = PHASE == 2 ? dt : R(0.025);
    PD_T(t_loaded);
    PD_ACC(1, t_loaded - t_staged);

    // The env's fields back to HBM (live lanes).  A fresh copy of the offset: the store
    // addresses are recomputed from the SGPR bases instead of being kept live from the loads
    auto store_all = [&]() {
    uint32_t uo = ui;
    asm volatile("" : "+v"(uo));
    if (live) {
        const uint32_t ui = uo;
#pragma unroll
        for (int k = 0; k < 11; ++k)
            if (k % LPE == role) ev(a.b.st + (k) * N, ui) = e.s[k];
        if (role == 0) {
            ev(a.b.vprev, ui) = e.vprev;
            ev(a.b.glen, ui) = (uint8_t)e.glen; ev(a.b.ghead, ui) = (uint8_t)e.ghead;
#pragma unroll
            for (int k = 0; k < 10; ++k) ev(a.b.gwin + (k) * N, ui) = L.gwin[k][le];
            ev(a.b.tid, ui) = (int8_t)e.tid;
            ev(a.b.epi, ui) = e.ep; ev(a.b.tstep, ui) = e.ts;
            if constexpr (PHASE == 1) { ev(a.b.act, ui) = e.act0; ev(a.b.act + N, ui) = e.act1; ev(a.b.act + (2) * N, ui) = e.act2; }
            if constexpr (PHASE == 2) { if (aux == PD_PHASE_FLIP_OVER) ev(a.b.act, ui) = e.act0; }
            if constexpr (WIND) {
                ev(a.b.wind, ui) = e.fu0; ev(a.b.wind + N, ui) = e.fu1; ev(a.b.wind + (2) * N, ui) = e.fv0; ev(a.b.wind + (3) * N, ui) = e.fv1;
                ev(a.b.wind + (4) * N, ui) = e.sgu; ev(a.b.wind + (5) * N, ui) = e.sgv;
                ev(a.b.wprof, ui) = (uint8_t)e.prof;
            }
        }
        // neighbourhood caches survive resets (any valid 50-set is a correct start); the table
        // row is laundered too (its 64-bit row offset would otherwise stay live from the loads)
        int mt = my_table;
        asm volatile("" : "+v"(mt));
        if (part == 0) {
            ev(a.b.key + (size_t)mt * (size_t)N, ui) = cA.key; ev(a.b.slot + (size_t)mt * (size_t)N, ui) = cA.slot;
            if constexpr (LPE == 1) { ev(a.b.key + N, ui) = cB.key; ev(a.b.slot + N, ui) = cB.slot; }
        }
    }
    };
    // policy rollouts stepping the live list: this launch's envs' actor parameters gathered once
    // into list order (policy_wc), so that every fused step reads them coalesced -- gathered per
    // step, the 372 scattered reads of each step cost more than the compaction saves
    const bool wcopy = POL && a.use_list && a.policy_wc != nullptr;
    if constexpr (POL) {
        if (wcopy) {
            // (the chunked layout of actor_forward: ceil(P / 4) rows of 16-byte chunks)
            constexpr int kC = ((PHASE == 0 ? PD_ACTOR_PARAMS_PURE_THROTTLE : PD_ACTOR_PARAMS_LANDING_BURN) + 3) / 4;
            using F4 = __attribute__((ext_vector_type(4))) float;
            uint32_t src = ui, dst = (uint32_t)e_act;
            asm volatile("" : "+v"(src), "+v"(dst));
#pragma unroll 8
            for (int q = 0; q < kC; ++q)
                ev((F4*)a.policy_wc + (size_t)q * (size_t)N, dst) = ldv((const F4*)a.policy_w + (size_t)q * (size_t)N, src);
        }
    }
    const int nf = a.n_fused;   // policy rollouts: finished envs freeze, stored at their last step
    WaveCount wc{CNT ? L.work[threadIdx.x >> 6] : nullptr};   // this wave's workload counts (CNT)
    // the atmosphere and speed of the state a sub-step ends in are computed right after its
    // integration (their work -- the table loads -- overlapping atan2's) and carried: to the next
    // sub-step, to the step's rtd after the last one, and on to the next step's first sub-step
    // unless the env reset (same y, vx, vy: bit-identical).  RK4: the rtd's only, carried to the
    // next step's first stage
    R k_rho = R(0), k_patm = R(0), k_asnd = R(0);
    double k_speed = 0.0;
    bool k_have = false;
    // The state chain of the sub-steps (position, velocity, pitch and its rate, flight-path angle,
    // alpha, masses, time) is integrated in binary64 in both precisions: a binary32 handle computes
    // its forces in binary32 but carries the chain in binary64 through the env-step (alpha_eff =
    // gamma - theta - pi, rockets_physics.py:498-501, is the difference of two O(1) angles: formed
    // from binary32 angles it lost ~1e-4 of itself, which the aerodynamic moment turned into
    // theta_dot) and rounds it to binary32 once, at the env-step's end -- the stored state, so
    // fused and per-step launches give the same bits.  Binary64 handles: xs is e.s itself.
    using RS = double;
    RS xs[sizeof(R) == 8 ? 1 : 11];
    auto SV = [&](int k) -> RS& {
        if constexpr (sizeof(R) == 8) return e.s[k];
        else return xs[k];
    };
#pragma unroll 1
    for (int f = 0; f < nf; ++f) {
    SA<R>& a = kargs<R>();
    const size_t fo = (size_t)f * (size_t)N;
    float uf[A];
    double ud[A];
#pragma unroll
    for (int k = 0; k < A; ++k) { uf[k] = 0.f; ud[k] = 0.0; }
    if constexpr (POL) {
        // pso_wrapper.augment_state (env_wrapped_ea.py:97-123) of the current state in the
        // handle's precision, cast to float32 (simple_actor.forward), then the actor
        DP<R>& Q = *params<R>(a.P);
        // the weights are the same every fused step: a laundered offset per step keeps their
        // 372 loads inside the loop (hoisted, they would be held in registers and spill)
        uint32_t uw = wcopy ? (uint32_t)e_act : ui;
        asm volatile("" : "+v"(uw));
        const float* W = wcopy ? a.policy_wc : a.policy_w;
        if constexpr (PHASE == 0) {
            float x[2] = {(float)(e.s[1] / Q.norm_y), (float)(e.s[3] / Q.norm_vy)};
            actor_forward<2, 3, 1, (LPE >= 2)>(W, N, uw, role & 1, x, uf);
        } else {
            float x[5] = {(float)(e.s[0] / Q.norm_x), (float)(e.s[1] / Q.norm_y), (float)(e.s[2] / Q.norm_vx),
                          (float)(e.s[3] / Q.norm_vy), (float)tanh(Q.k_theta_pso * (e.s[4] - Cst<R>::pi / R(2)))};
            actor_forward<5, 4, 4, (LPE >= 2)>(W, N, uw, role & 1, x, uf);
        }
    } else if constexpr (SAC) {
        // Actor.sample (sac_pytorch.py:161-179) on the caller's two heads, in binary32 as torch
        // computes it: log_std clamped (forward), std = exp, x = mean + std * eps (rsample),
        // action = tanh(x) * max_action; eps NULL: tanh(mean) * max_action (deterministic)
        // pd_step_sac_ring: eps ~ N(0, 1) drawn here (torch.randn's role), two components per
        // Philox block, keyed by (env, episode, step) like the gust draws: the same bits on
        // every lane of the env and in any launch order
        float ed[A];
#pragma unroll
        for (int k = 0; k < A; ++k) ed[k] = 0.f;
        if (a.sac_draw) {
            DP<R>& Q = *params<R>(a.P);
            const double* lic = (const double*)(uint64_t)&Q.logtab.invc[0];
            const double* llc = (const double*)(uint64_t)&Q.logtab.logc[0];
#pragma unroll
            for (int k = 0; k < A; k += 2) if (k < AD) {
                u32x4 r = philox_k({(uint32_t)g, (uint32_t)(g >> 32) ^ e.ep, e.ts, kTagSacEps + (uint32_t)(k >> 1)},
                                   a.seed_lo, a.seed_hi);
                double z0, z1;
                gauss_pair(r, lic, llc, z0, z1);
                ed[k] = (float)z0;
                if (k + 1 < A) ed[k + 1] = (float)z1;
            }
        }
        const bool mlp = kSacMlp && a.sac_mlp.H != 0;   // heads from the prologue's LDS rows
#pragma unroll
        for (int k = 0; k < A; ++k) if (k < AD) {
            const float m = mlp ? s_sach[le * 16 + k] : ldv(a.sac_mean + k, ui * a.sac_hs);
            float xk = m;
            if (a.sac_eps || a.sac_draw) {
                float ls = mlp ? s_sach[le * 16 + 8 + k] : ldv(a.sac_logstd + k, ui * a.sac_hs);
                ls = ls < a.sac_lo ? a.sac_lo : (ls > a.sac_hi ? a.sac_hi : ls);
                const float sd = expf(ls);
                const float ek = a.sac_draw ? ed[k] : ldv(a.sac_eps + k, ui * AD);
                xk = m + sd * ek;
                if (a.sac_eps_out && role == 0 && live) ev(a.sac_eps_out + k, ui * AD) = ek;
            }
            uf[k] = tanhf(xk) * a.sac_max;
            if (a.sac_act && role == 0 && live) ev(a.sac_act + k, ui * AD) = uf[k];
        }
    } else if (a.act_f64) {
#pragma unroll
        for (int k = 0; k < A; ++k) if (k < AD) ud[k] = ldv((const double*)a.actions + fo * AD + k, ui * AD);
    } else {
#pragma unroll
        for (int k = 0; k < A; ++k) if (k < AD) uf[k] = ldv((const float*)a.actions + fo * AD + k, ui * AD);
    }
    // pd_step_sac: the transition row of this step starts with the observation of its start state
    // (row srow: the env's, or in ring mode its row of the replay ring, (position + i) mod capacity)
    constexpr int kObsKind = RTD == 1 ? (PHASE == 0 ? 1 : 2) : (PHASE == 0 ? 0 : (PHASE == 1 ? 3 : -1));
    uint32_t srow = ui;
    if (SAC && a.ring_state) {
        const int64_t rp = ring_pos0 + (int64_t)i;
        srow = (uint32_t)(rp >= a.ring_cap ? rp - a.ring_cap : rp);
    }
    if (SAC && a.slab && role == 0 && live) {
        DP<R>& Q = *params<R>(a.P);
        const int ok = kObsKind >= 0 ? kObsKind : Q.obs_kind;
        const uint32_t W = 2u * (uint32_t)obs_dim(ok) + (uint32_t)AD + 2u;
        obs_eval<R>(Q, ok, e.s, [&](int k, R v) { ev(a.slab, srow * W + (uint32_t)k) = (float)v; });
        if (a.prio) ev(a.prio, srow) = *a.max_prio;
    }
    R gdeg_out = e.act0, dcmdl_out = e.act1, dcmdr_out = e.act2;
    const R gprev = e.act0, dlprev = e.act1, drprev = e.act2;
    bool nan_hit = false;
    // info tap: the last sub-step's quantities (rockets_physics.py:649-702) of the fields in
    // info_mask, row f of the [n_fused][nsel][N] array (pd_step: every field, one row)
    const bool tap = a.info != nullptr && role == 0 && live;
    // (the lane offset is laundered per use so that the 49 loop-invariant store addresses are
    // formed inside the taken branch, not hoisted out of the loops and kept live: 92 VGPRs)
    // (and the row base is laundered too: hoisted, the 49 uniform row bases a.info + k N were
    // kept in scalar registers -- spilled into VGPR lanes from the prologue on)
    auto info = [&](int k, R v) {
        const uint64_t m = a.info_mask;
        if (!((m >> k) & 1ull)) return;   // (uniform)
        const size_t row = (size_t)f * (size_t)a.info_nsel + (size_t)__popcll(m & ((1ull << k) - 1ull));
        uint32_t u = ui;
        uint32_t blo = (uint32_t)(uint64_t)a.info, bhi = (uint32_t)((uint64_t)a.info >> 32);
        asm volatile("" : "+v"(u), "+s"(blo), "+s"(bhi));
        R* base = (R*)(((uint64_t)bhi << 32) | blo);
        ev(base + row * (size_t)N, u) = v;
    };

    bool wpre = false;   // the odd sub-step's gust normals are in L.wnx (drawn with the even one's)
    RS rkb[8], rka[8];   // RK4: the 0.01 s step's base state and its k1 + 2 k2 + 2 k3 + k4
    if constexpr (sizeof(R) == 4) {
#pragma unroll
        for (int k = 0; k < 11; ++k) xs[k] = (RS)e.s[k];
    }
    // the sub-step's dt in binary64 (the reference's literals; the binary64 handle's dt bits)
    const RS dts = RK4 ? 0.01 : (PHASE == 0 ? 0.025 : (PHASE == 1 ? 0.1 : a.dt_aux));
#pragma unroll 1
    for (int sub = 0; sub < NSUB; ++sub) {
        PD_T(t_sub);
        const int stage = RK4 ? (sub & 3) : 0;
        SA<R>& a = kargs<R>();
        DP<R>& P = *params<R>(a.P);
        const bool tap_sub = tap && sub == NSUB - 1;
        RS x = SV(0), y = SV(1), vx = SV(2), vy = SV(3), th = SV(4), thd = SV(5), ga = SV(6), al = SV(7);
        RS m = SV(8), mp = SV(9);
        if constexpr (WIND) wc.add(kStGust - kStWork, role == 0 && live && a.stochastic && y < P.vk_y_threshold);
        // rocket_physics_fcn (rockets_physics.py:455-704)
        R rho, patm, asnd;
        RS speed;
        if (RK4 ? (sub == 0 && k_have) : k_have) { rho = k_rho; patm = k_patm; asnd = k_asnd; speed = k_speed; }
        else {
            atmosphere<R, kAtmTab>(P, L.isa, (R)y, rho, patm, asnd);
            speed = sqrt(vx * vx + vy * vy);
        }
        const R spR = (R)speed;
        R mach = R(0);
        if (asnd != R(0)) { R mr = spR / asnd; mach = (R(10) < mr) ? R(10) : mr; }
        // alpha_effective (rockets_physics.py:498-501) and Mach feed the aero tables; what the
        // tables do not need is computed after them (fewer values live across the RBF)
        const R ae = (R)((vy < RS(0)) ? ga - th - Cst<RS>::pi : al);
        // the horizontal wind and the gust filters (no table dependence): with LPE 2 run while
        // the aero lookup's grid loads are in flight, else after the tables
        R ug = R(0), vg = R(0);
        auto wind_block = [&]() {
            if constexpr (WIND) {
                // WindModel.__call__ (full_wind_model.py:35-43)
                const R* walt = L.walt + e.prof * 16;
                const R* wsp = L.wsp + e.prof * 16;
                R km = PD_DIVC(R, (R)y, 1000);
                int wn = P.wind_n[e.prof];
                ug = np_interp<R>(walt, wsp, wn, km);
                const bool gust = y < P.vk_y_threshold && a.stochastic;
                if (gust) {
                    double w0 = 0.0, w1 = 0.0;
                    // vonkarman.py:34: one np.random.randn() per filter step, u then v (gauss_pair:
                    // Philox counter (env, episode, step, sub-step), reproducible by the oracle)
                    const double* lic = (const double*)(uint64_t)&P.logtab.invc[0];
                    const double* llc = (const double*)(uint64_t)&P.logtab.logc[0];
                    bool drawn = false;
                    if (a.noise) { w0 = ev(a.noise + 2 * sub, ui * 8); w1 = ev(a.noise + 2 * sub + 1, ui * 8); drawn = true; }
                    else if constexpr (LPE >= 2 && NSUB == 4) {
                        if ((sub & 1) == 0) {
                            // the env's lane pair draws sub-steps sub and sub + 1 at once: the same
                            // code on two counters, results swapped (the same bits as one draw per
                            // sub-step; the odd sub-step's pair waits in LDS)
                            const int odd = role & 1;
                            u32x4 r = philox_k({(uint32_t)g, (uint32_t)(g >> 32) ^ e.ep, e.ts, kTagWindSub + (uint32_t)(sub + odd)},
                                             a.seed_lo, a.seed_hi);
                            double z0, z1;
                            gauss_pair(r, lic, llc, z0, z1);
                            const double o0 = pair_swap(z0), o1 = pair_swap(z1);
                            w0 = odd ? o0 : z0; w1 = odd ? o1 : z1;
                            L.wnx[0][threadIdx.x] = odd ? z0 : o0; L.wnx[1][threadIdx.x] = odd ? z1 : o1;
                            drawn = true;
                        } else if (wpre) {
                            w0 = L.wnx[0][threadIdx.x]; w1 = L.wnx[1][threadIdx.x];
                            drawn = true;
                        }
                    }
                    if (!drawn) {   // (one draw per sub-step; paired: an env that entered the band mid-pair)
                        u32x4 r = philox_k({(uint32_t)g, (uint32_t)(g >> 32) ^ e.ep, e.ts, kTagWindSub + (uint32_t)sub},
                                         a.seed_lo, a.seed_hi);
                        gauss_pair(r, lic, llc, w0, w1);
                    }
                    // vonkarman.py:33-36: state = Ad @ state + Bd * w  (Bd = sigma * Bd(sigma=1))
                    R n0 = (P.vk_Ad_u[0] * e.fu0 + P.vk_Ad_u[1] * e.fu1) + (e.sgu * P.vk_Bd_u[0]) * (R)w0;
                    R n1 = (P.vk_Ad_u[2] * e.fu0 + P.vk_Ad_u[3] * e.fu1) + (e.sgu * P.vk_Bd_u[1]) * (R)w0;
                    e.fu0 = n0; e.fu1 = n1;
                    n0 = (P.vk_Ad_v[0] * e.fv0 + P.vk_Ad_v[1] * e.fv1) + (e.sgv * P.vk_Bd_v[0]) * (R)w1;
                    n1 = (P.vk_Ad_v[2] * e.fv0 + P.vk_Ad_v[3] * e.fv1) + (e.sgv * P.vk_Bd_v[1]) * (R)w1;
                    e.fv0 = n0; e.fv1 = n1;
                    ug = ug + e.fu1;
                    vg = e.fv1;
                }
                wpre = gust && (sub & 1) == 0;
            }
        };
        R CL = R(0), CD = R(0);
        PD_T(t_aero0);
        PD_ACC(2, t_aero0 - t_sub);
        {
            // evaluated convergently by every lane; results of lanes that need none (speed of
            // sound 0 above 81 km, |deg(deg(alpha))| < 1e-6 for C_L) are discarded
            R cl_sgn; bool cl_zero;
            R aq_cl = cl_query<R>(ae, cl_sgn, cl_zero);
            R aq_cd = cd_query<R>(ae);
            const bool have = asnd != R(0);
            if constexpr (LPE == 1) {
                // (both sums interleaved in lockstep on one lane, 1 wave per SIMD with AGPR
                // spill space, measured 14 % slower than these two calls)
                R v = rbf<kPcs, R>(a, P, 1, tab_view_lds<R>(L.tdesc, 1), L.lines, cB, mach, aq_cl, 0, 1);
                R w = rbf<kPcs, R>(a, P, 0, tab_view_lds<R>(L.tdesc, 0), L.lines, cA, mach, aq_cd, 0, 1);
                CL = (!have || cl_zero) ? R(0) : (cl_sgn < R(0) ? -v : v);
                CD = have ? w : R(0);
            } else {
                R v;
                if constexpr (LPE == 2)
                    v = rbf2<R>(a, P, my_table, tab_view_lds<R>(L.tdesc, my_table), L.lines, cA, mach,
                                my_table ? aq_cl : aq_cd, live, L.bal[threadIdx.x >> 6], L.tab, wc, wind_block
#ifdef PD_STAMP
                                , acc_ + 7
#endif
                                );
                else
                    v = rbf<kPcs, R>(a, P, my_table, tab_view_lds<R>(L.tdesc, my_table), L.lines, cA, mach,
                                     my_table ? aq_cl : aq_cd, part, nparts);
                if constexpr (nparts >= 2) v += __shfl_xor(v, 1);
                if constexpr (nparts >= 4) v += __shfl_xor(v, 2);
                if constexpr (nparts >= 8) v += __shfl_xor(v, 4);
                R vcd, vcl;
                if constexpr (LPE == 2) {   // role 0 holds C_D, role 1 C_L: one DPP swap
                    const R vo = pair_swap(v);
                    vcd = role ? vo : v; vcl = role ? v : vo;
                } else {
                    vcd = __shfl(v, gbase);
                    vcl = __shfl(v, gbase + nparts);
                }
                CD = have ? vcd : R(0);
                CL = (!have || cl_zero) ? R(0) : (cl_sgn < R(0) ? -vcl : vcl);
            }
        }
        PD_T(t_aero1);
        PD_ACC(3, t_aero1 - t_aero0);
        R q = R(0.5) * rho * (spR * spR);
        R fpc = div_known<R>((R)(P.m_prop0 - mp), P.m_prop0, P.inv_m_prop0, P.div2 & kDiv2MProp0);
        if (fpc == R(0)) fpc = R(1e-6);
        R x_cog, I;
        // subrocket_0 (full rocket) closures for the ascent, subrocket_2 after (:748-750, :772-774)
        if (ascent) inertia_full<R>(P, R(1) - fpc, x_cog, I);
        else inertia<R>(P, R(1) - fpc, x_cog, I);
        R d_thrust = x_cog + P.engine_height;
        R d_cp_cg = x_cog - (ascent ? P.cop_ascent : P.cop);
        if constexpr (LPE != 2) wind_block();
#ifdef PD_STAMP
        PD_T(t_p1); acc_[9 + 4] += t_p1 - t_aero1;
#endif
        R Fwx = R(0.5) * rho * (ug * ug) * P.A_front * P.C_gust_x;
        R Fwy = R(0.5) * rho * (vg * vg) * P.A_front * P.C_gust_y;
        R Mw = -d_cp_cg * Fwy;
        if (tap_sub) {   // info of the last sub-step (rockets_physics.py:649-702), stored where computed
            const R mmax = asnd != R(0) ? sqrt(R(2) * R(30000) / rho) * R(1) / asnd : R(200);
            info(PD_INFO_AIR_DENSITY, rho); info(PD_INFO_PRESSURE, patm); info(PD_INFO_SPEED_OF_SOUND, asnd);
            info(PD_INFO_MACH, mach); info(PD_INFO_Q, q); info(PD_INFO_X_COG, x_cog); info(PD_INFO_INERTIA, I);
            info(PD_INFO_ALPHA_EFF, ae); info(PD_INFO_UG, ug); info(PD_INFO_VG, vg); info(PD_INFO_MACH_MAX, mmax);
            info(PD_INFO_D_CP_CG, d_cp_cg); info(PD_INFO_D_THRUST_CG, d_thrust); info(PD_INFO_FUEL_CONSUMED, fpc);
            info(PD_INFO_F_WIND_X, Fwx); info(PD_INFO_F_WIND_Y, Fwy); info(PD_INFO_M_WIND, Mw); info(PD_INFO_THETA_IN, (R)th);
        }
        R drag = R(0.5) * rho * (spR * spR) * CD * P.A_front;
        R lift = R(0.5) * rho * (spR * spR) * CL * P.A_front;
        R sae, cae, sth, cth;
        sincos_pair<LPE, R>(ae, (R)th, role, sae, cae, sth, cth);
        R apar, aperp;
        if (vy >= RS(0)) { apar = lift * sae - drag * cae; aperp = -lift * cae - drag * sae; }
        else { apar = drag * cae - lift * sae; aperp = -drag * sae - lift * cae; }
        R aero_x = apar * cth + aperp * sth;
        R aero_y = apar * sth - aperp * cth;
        R aero_m = aperp * d_cp_cg;
        if (PHASE == 2 && aux == PD_PHASE_FLIP_OVER) { aero_x = R(0); aero_y = R(0); aero_m = R(0); }   // :548-551

#ifdef PD_STAMP
        PD_T(t_p2); acc_[9 + 5] += t_p2 - t_p1;
#endif
        R T_full = P.T_e + (P.p_e - patm) * P.A_e;
        R qS = q * P.S_gf;
        R Ca = grid_fin_ca<R>(P, L.gf, L.gf + 64, mach, L.ca_lb, L.gfs);
        R cfp, cfperp, cm, mdot_dt, md_info, thr_info;
        // info of the grid-fin ACS (acs_model.py:62-86): deflections, C_n of both fins, forces
        R i_dl = R(0), i_dr = R(0), i_cnl = R(0), i_cnr = R(0), i_gfperp = R(0), i_gfpar = R(0), i_gfm = R(0);
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
                    R nt = ((R)ud[0] - spR) * P.kp_pc;
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
                i_gfpar = qS * (Ca * R(4));
                if (tap_sub) {   // C_n of the undeflected fins (acs_info only)
                    const R cna = grid_fin_cn_alpha<R>(P, L.gf + 128, L.gf + 192, mach, L.gfs + 64);
                    i_cnl = cna * (ae * Cst<R>::rad2deg); i_cnr = i_cnl;
                }
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
                gdeg_out = gd;
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
            i_gfpar = acs_par;
            if (tap_sub) {   // C_n of the undeflected fins (acs_info only)
                const R cna = grid_fin_cn_alpha<R>(P, L.gf + 128, L.gf + 192, mach, L.gfs + 64);
                i_cnl = cna * (ae * Cst<R>::rad2deg); i_cnr = i_cnl;
            }
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
            R cna = grid_fin_cn_alpha<R>(P, L.gf + 128, L.gf + 192, mach, L.gfs + 64);
            R CnL = cna * ((ae - dl) * Cst<R>::rad2deg);
            R CnR = cna * ((ae - dr) * Cst<R>::rad2deg);
            R cl_, cr_, sl_, sr_;
            sincos_pair<LPE, R>(dl, dr, role, sl_, cl_, sr_, cr_);
            R f_perp = qS * (CnR * cr_ - CnL * cl_ - Ca * (sl_ - sr_));
            R f_par = qS * (Ca * (R(2) + cl_ + cr_) - CnL * sl_ + CnR * sr_);
            R m_z = -(P.d_base_gf - x_cog) * f_perp + P.R_rocket * qS * (Ca * (sr_ - sl_) - CnL * cl_ + CnR * cr_);
            cfp = tpar + f_par; cfperp = tperp + f_perp; cm = tmz + m_z;
            dcmdl_out = dcl; dcmdr_out = dcr;
            md_info = md; thr_info = thr;
            i_dl = dl; i_dr = dr; i_cnl = CnL; i_cnr = CnR; i_gfperp = f_perp; i_gfpar = f_par; i_gfm = m_z;
        }
#ifdef PD_STAMP
        PD_T(t_p3); acc_[9 + 6] += t_p3 - t_p2;
#endif
        // NaN guard (rockets_physics.py:599-607), an elif chain
        if (isnan(cfp)) { cfp = R(0); nan_hit = true; }
        else if (isnan(cfperp)) { cfperp = R(0); nan_hit = true; }
        else if (isnan(cm)) { cm = R(0); nan_hit = true; }
        if (tap_sub) {
            info(PD_INFO_CL, CL); info(PD_INFO_CD, CD); info(PD_INFO_DRAG, drag); info(PD_INFO_LIFT, lift);
            info(PD_INFO_AERO_X, aero_x); info(PD_INFO_AERO_Y, aero_y); info(PD_INFO_AERO_MOMENT, aero_m);
            info(PD_INFO_MASS_FLOW, md_info); info(PD_INFO_THROTTLE, thr_info); info(PD_INFO_GIMBAL_DEG, gdeg_out);
            info(PD_INFO_CF_PAR, cfp); info(PD_INFO_CF_PERP, cfperp); info(PD_INFO_CONTROL_MOMENT, cm);
            info(PD_INFO_DCMD_L, dcmdl_out); info(PD_INFO_DCMD_R, dcmdr_out); info(PD_INFO_DELTA_L, i_dl);
            info(PD_INFO_DELTA_R, i_dr); info(PD_INFO_GF_CA, Ca); info(PD_INFO_GF_CN_L, i_cnl); info(PD_INFO_GF_CN_R, i_cnr);
            info(PD_INFO_GF_F_PERP, i_gfperp); info(PD_INFO_GF_F_PAR, i_gfpar); info(PD_INFO_GF_MZ, i_gfm);
        }
        R cfx, cfy;
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
            cfx = (R)cx; cfy = (R)cy;
        } else {
            cfx = cfp * cth + cfperp * sth;
            cfy = cfp * sth - cfperp * cth;
            fx = aero_x + cfx + Fwx; fy = aero_y + cfy + Fwy;
        }
        // vx_dot = F_x / m, vy_dot = F_y / m - g, theta_dot_dot = M_z / I, g = g0 (R/(R+y))^2:
        // three divisions as two lane-paired ones
        const R mz = cm + aero_m + Mw;
        R vxd, vyq, thdd, grq;
#ifdef PD_STAMP
        PD_T(t_p4); acc_[9 + 7] += t_p4 - t_p3;
#endif
        div_pair<LPE, R>(fx, (R)m, fy, (R)m, role, vxd, vyq);
        div_pair<LPE, R>(mz, I, P.grav_R, P.grav_R + (R)y, role, thdd, grq);
        const R gr = P.grav_g0 * (grq * grq);
        const R vyd = vyq - gr;
        if constexpr (RK4) {
            const RS kd[8] = {vx, vy, vxd, vyd, thd, thdd, -md_info, -md_info};
            RS sv[8] = {x, y, vx, vy, th, thd, m, mp};
            if (stage == 0) {
#pragma unroll
                for (int k = 0; k < 8; ++k) rkb[k] = sv[k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) rka[k] = stage == 0 ? kd[k] : (stage == 3 ? rka[k] + kd[k] : rka[k] + R(2) * kd[k]);
            const RS c = stage == 3 ? dts / RS(6) : (stage == 2 ? dts : RS(0.5) * dts);
#pragma unroll
            for (int k = 0; k < 8; ++k) sv[k] = rkb[k] + c * (stage == 3 ? rka[k] : kd[k]);
            x = sv[0]; y = sv[1]; vx = sv[2]; vy = sv[3]; th = sv[4]; thd = sv[5]; m = sv[6]; mp = sv[7];
            if (stage == 3 && th > Cst<RS>::two_pi) th -= Cst<RS>::two_pi;
            ga = pd_atan2<RS>(vy, vx);
            if (ga < RS(0)) ga = Cst<RS>::two_pi + ga;
            al = th - ga;
        } else {
        vx += (RS)vxd * dts; vy += (RS)vyd * dts; x += vx * dts; y += vy * dts;
        thd += (RS)thdd * dts; th += thd * dts;
        atmosphere<R, kAtmTab>(P, L.isa, (R)y, k_rho, k_patm, k_asnd);
        k_speed = sqrt(vx * vx + vy * vy);
        k_have = true;
        ga = pd_atan2<RS>(vy, vx);
        if (th > Cst<RS>::two_pi) th -= Cst<RS>::two_pi;
        if (ga < RS(0)) ga = Cst<RS>::two_pi + ga;
        al = th - ga;
        mp -= (RS)mdot_dt; m -= (RS)mdot_dt;
        }
        if (tap_sub) {
            info(PD_INFO_CF_X, cfx); info(PD_INFO_CF_Y, cfy); info(PD_INFO_GRAVITY, gr); info(PD_INFO_VX_DOT, vxd);
            info(PD_INFO_VY_DOT, vyd); info(PD_INFO_MOMENTS, mz); info(PD_INFO_THETA_DDOT, thdd);
        }
        SV(0) = x; SV(1) = y; SV(2) = vx; SV(3) = vy; SV(4) = th; SV(5) = thd; SV(6) = ga; SV(7) = al;
        SV(8) = m; SV(9) = mp;
        if (!RK4 || stage == 3) SV(10) = SV(10) + dts;
        PD_T(t_subend);
        PD_ACC(4, t_subend - t_aero1);
    }
    if (nan_hit && role == 0 && live) atomicAdd(&a.pend.stats[kStNan], 1ull);
    if constexpr (sizeof(R) == 4) {   // the env-step's state, rounded once
#pragma unroll
        for (int k = 0; k < 11; ++k) e.s[k] = (R)xs[k];
    }
    PD_T(t_loop);

    // ---- g-load window (base_environment.py:136-149): ring of 10 in LDS, Python sum() from the
    // oldest; the new entry is written first, then the window is read back in summation order
    DP<R>& P2 = *params<R>(a.P);
    const R* s = e.s;
    const RS v = RK4 ? sqrt(SV(2) * SV(2) + SV(3) * SV(3)) : k_speed;   // (the same expression's bits)
    R gl_new = (R)PD_DIVC(RS, PD_DIVC(RS, fabs(v - (RS)e.vprev), 0.1) * RS(1), 9.81);
    int glen = e.glen, ghead = e.ghead;
    int wslot;
    if (glen < 10) { wslot = glen; glen += 1; }
    else { wslot = ghead; ghead = ghead == 9 ? 0 : ghead + 1; }
    L.gwin[wslot][le] = gl_new;
    const int gstart = glen < 10 ? 0 : ghead;
    R gv[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        int p = gstart + k;
        p = p >= 10 ? p - 10 : p;
        gv[k] = L.gwin[p][le];
    }
    R gsum = R(0);
#pragma unroll
    for (int k = 0; k < 10; ++k)
        if (k < glen) gsum += gv[k];
    R gl = PD_DIVC(R, gsum, 10);

    // ---- truncated -> done -> reward (rtd_rl.py:190-336 / rtd_pso.py:172-317)
    R x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], ga = s[6], mp = s[9];
    R rho, pa_, as_;
    if constexpr (RK4) {
        atmosphere<R, kAtmTab>(P2, L.isa, y, rho, pa_, as_);
        k_rho = rho; k_patm = pa_; k_asnd = as_; k_speed = v;
    } else {
        rho = k_rho; pa_ = k_patm; as_ = k_asnd;   // (the last sub-step's, of this state)
    }
    R speed = (R)v;
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
            // (divisions by literals and by y0 / m0 through their reciprocals: div_known)
            if (qr > R(60000)) { R e_ = PD_DIVC(R, qr - R(60000), 5000); R e2 = e_ * e_; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            if (gl > R(5.5)) { R e_ = (gl - R(5.5)) / (R(6) - R(5.5)); R e2 = e_ * e_; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            R prog = div_known<R>(P2.y0_rl - y, P2.y0_rl, P2.inv_y0_rl, P2.div2 & kDiv2Y0);
            R wp = (qr <= R(60000) && gl <= R(5.5)) ? R(0.5) : R(0.5) * R(0.1);
            rew += wp * prog;
            if (y < R(100)) rew += R(5.5) * (R(1) - PD_DIVC(R, fabs(vy), 50));
            if (dn && !tr) rew += div_known<R>(R(400) * mp, P2.m0_rl, P2.inv_m0_rl, P2.div2 & kDiv2M0);
            else if (tr && y > R(0)) rew -= R(50) * div_known<R>(fabs(y), P2.y0_rl, P2.inv_y0_rl, P2.div2 & kDiv2Y0);
            else if (tr && y < R(0)) rew -= R(50) * PD_DIVC(R, fabs(vy), 10);
            if (!dn || !(tr && y < R(0))) rew = rew < R(-10) ? R(-10) : (rew > R(10) ? R(10) : rew);
        } else {                      // landing_burn / ACS reward (rtd_rl.py:243-269), u0 = actions[0]
            R aef = (R)fabs(SV(6) - SV(4) - Cst<RS>::pi);   // (the chain's binary64 angles)
            R lead = R(1.5) - log(R(1) + aef) / P2.log_1p_max_ae;
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
            if (qr > R(60000)) { R e_ = (qr - R(60000)) / (R(65000) - R(60000)); R e2 = e_ * e_; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
            if (gl > R(5.5)) { R e_ = (gl - R(5.5)) / (R(6) - R(5.5)); R e2 = e_ * e_; rew -= R(1) * (e2 > R(1) ? R(1) : e2); }
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
            R aef = (R)fabs(SV(6) - SV(4) - Cst<RS>::pi);
            dn = (q > R(10000) && aef < (R)(3.0 * kDeg2Rad));
            if (q > R(10000 - 2000) && aef > (R)(5.0 * kDeg2Rad)) { tr = 1; id = 1; }
            rew = (Cst<R>::pi - aef) / Cst<R>::pi;
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
                const PD_AS1 R* ry = gbl(P2.ref_y);
                R xr = interp1d_ext<R>(ry, gbl(P2.ref_x), n, y), vxr = interp1d_ext<R>(ry, gbl(P2.ref_vx), n, y);
                R vyr = interp1d_ext<R>(ry, gbl(P2.ref_vy), n, y);
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
            R aeff = (R)((vy < R(0)) ? fabs(SV(6) - SV(4) - Cst<RS>::pi) : fabs(SV(4) - SV(6)));
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
    // ---- outputs of step f (role 0 of the env's lane group)
    const bool ended = !POL && a.auto_reset && (dn || tr);
    wc.add(kStResets - kStWork, ended && role == 0 && live);
    k_have = !ended;
    // (binary32: the next step starts from the rounded state; its speed from the rounded velocity,
    // as a launch that loads it computes it; the atmosphere was evaluated at the rounded altitude)
    if constexpr (sizeof(R) == 4) k_speed = sqrt((RS)e.s[2] * (RS)e.s[2] + (RS)e.s[3] * (RS)e.s[3]);
    if (role == 0 && live) {
        // (loop-invariant addresses from a laundered offset: formed here, not held across the loop)
        uint32_t uo = ui;
        asm volatile("" : "+v"(uo));
        if (a.obs) {
            // the wrappers' observation (obs_write kinds); compile-time for the landing burns
            const int ok = kObsKind >= 0 ? kObsKind : P2.obs_kind;
            obs_write<R>(P2, ok, s, a.obs + fo * obs_dim(ok), uo);
        }
        if (a.reward) ev(a.reward + fo, ui) = rew;
        if constexpr (POL) {
            // objective_function: episode_reward -= reward until done or truncated (env_wrapped_ea.py:200-222)
            ev(a.reward_sum, uo) -= rew;
            if (dn || tr) ev(a.b.fin, uo) = 1;
        } else if (a.reward_sum) {
            ev(a.reward_sum, uo) += rew;
        }
        if (a.done) ev(a.done + fo, ui) = (uint8_t)dn;
        if (a.trunc) ev(a.trunc + fo, ui) = (uint8_t)tr;
        if (a.trunc_id) ev(a.trunc_id + fo, ui) = (int8_t)id;
        if (a.info) info(PD_INFO_GLOAD, gl);
        if (SAC && a.slab) {
            // state | action | reward | next_state (terminal, before any reset) | done: the
            // replay buffer's row (sac_pytorch.py:27-35; done without truncation, as the driver
            // stores it, sac_pytorch_powered_descent.py:170-176)
            const int ok = kObsKind >= 0 ? kObsKind : P2.obs_kind;
            const uint32_t S = (uint32_t)obs_dim(ok), W = 2u * S + (uint32_t)AD + 2u, r0 = srow * W;
#pragma unroll
            for (int k = 0; k < A; ++k) if (k < AD) ev(a.slab, r0 + S + (uint32_t)k) = uf[k];
            ev(a.slab, r0 + S + (uint32_t)AD) = (float)rew;
            obs_eval<R>(P2, ok, s, [&](int k, R v) { ev(a.slab, r0 + S + (uint32_t)AD + 1u + (uint32_t)k) = (float)v; });
            ev(a.slab, r0 + 2u * S + (uint32_t)AD + 1u) = (float)dn;
        }
    }
    // ---- the env's bookkeeping for the next step: auto-reset in registers, or carry on
    if (ended) {
        reset_values<R>(P2, a, g, e.ep + 1, (const double*)(uint64_t)&P2.logtab.invc[0],
                        (const double*)(uint64_t)&P2.logtab.logc[0], e);   // keeps the aero caches
    } else {
        e.vprev = (R)v;
        e.glen = glen; e.ghead = ghead;
        e.tid = id;
        e.ts = e.ts + 1;
        e.act0 = gdeg_out; e.act1 = dcmdl_out; e.act2 = dcmdr_out;
    }
    if (SAC && a.obs32 && role == 0 && live) {   // pd_step_sac: what the actor sees next (after any reset)
        const int ok = kObsKind >= 0 ? kObsKind : P2.obs_kind;
        const uint32_t S = (uint32_t)obs_dim(ok);
        obs_eval<R>(P2, ok, e.s, [&](int k, R v) { ev(a.obs32, ui * S + (uint32_t)k) = (float)v; });
    }
    if constexpr (POL) {
        // an episode that ended is stored now and its lanes freeze (they go on computing in step
        // with the wave, convergent for the cooperative miss solve, but write nothing)
        const bool ended_now = live && (dn || tr || (kRefill && a.refill && e.ts >= (uint32_t)a.refill_max));
        if (ended_now) { store_all(); live = false; }
        if (kRefill && a.refill && rq_next < a.refill_q) {
            // refill from the wave's own particles: every waiting slot at once, its rank in the
            // ballot (of its role-0 lane) the offset -- no atomic, no wait
            const unsigned long long mk = __ballot(slot && !live && role == 0);
            if (mk) {
                const int nw = __popcll(mk);
                const int take = nw < a.refill_q - rq_next ? nw : a.refill_q - rq_next;
                const int rank = __popcll(mk & ((1ull << gbase) - 1ull));
                if (slot && !live && rank < take) {
                    const int64_t nx = (gt >> 6) * (int64_t)a.refill_q + (int64_t)(rq_next + rank);
                    e_act = nx; i = nx; ui = (uint32_t)nx; g = a.env_offset + (uint64_t)nx; valid = true;
                    load_env();
                    live = true;
                    k_have = false;
                }
                rq_next += take;
            }
        }
        if (kRefill && a.refill && !drained && rq_next >= a.refill_q) {
            // then the shared pool: once `refill` of the wave's slots wait (or none is live), they
            // take its next particles, one atomic per hand-out and the ballot's prefix count per
            // env (its role-0 lane's rank); each loads the particle's reset state as the first
            // launch of a rollout does (same bits).  Batched, the pool's one counter sees a few
            // hand-outs per wave, not one per wave and step, and a wave pays the loads' latency
            // once per batch
            const unsigned long long mk = __ballot(slot && !live && role == 0);
            const int nw = __popcll(mk);
            if (nw >= a.refill || (nw > 0 && __ballot(live) == 0ull)) {
                const int lane = (int)__lane_id();
                const int leader = __ffsll((long long)mk) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(a.refill_next, (uint32_t)nw);
                base = (uint32_t)__shfl((int)base, leader);
                // (wave-uniform: once a hand-out reaches the swarm's end, no later one can start)
                drained = (int64_t)a.refill_base + (int64_t)base + nw >= N;
                const int64_t nx = (int64_t)a.refill_base + (int64_t)base + (int64_t)__popcll(mk & ((1ull << gbase) - 1ull));
                if (slot && !live && nx < N) {
                    e_act = nx; i = nx; ui = (uint32_t)nx; g = a.env_offset + (uint64_t)nx; valid = true;
                    load_env();
                    live = true;
                    k_have = false;
                }
            }
        }
        // a wave whose episodes have all ended leaves the launch's remaining steps (no barrier
        // follows; its lanes write nothing more): the launch then ends with its last live wave,
        // not F steps after the swarm's last episode
        if (__ballot(live) == 0ull) break;
    }
    }   // fused steps
    if constexpr (POL) {
        // done-mask compaction: the envs whose episode goes on, in lane order, appended to the
        // next launch's list at a base taken by one atomic per wave (the count also tells the
        // host when every episode has ended)
        const bool cont = role == 0 && live;
        const unsigned long long mk = __ballot(cont);
        if (mk) {
            const int lane = (int)__lane_id();
            const int leader = __ffsll((long long)mk) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.cnt_out, (uint32_t)__popcll(mk));
            base = (uint32_t)__shfl((int)base, leader);
            if (cont) a.list_out[base + (uint32_t)__popcll(mk & ((1ull << lane) - 1ull))] = (int32_t)i;
        }
    }

    // ---- the env's state back to HBM, once (policy rollouts: also when its episode ends)
    PD_T(t_store);
    store_all();
    if constexpr (SAC) {
        // ring mode: the launch's last workgroup (a ticket per workgroup, taken after all of its
        // ring rows are written and its position read) advances the ring's position and size
        if (a.ring_state) {
            __syncthreads();
            if (threadIdx.x == 0) {
                const unsigned long long t = atomicAdd((unsigned long long*)&a.ring_state[2], 1ull);
                if (t == (unsigned long long)gridDim.x - 1ull) {
                    const int64_t np = ring_pos0 + N, sz = (int64_t)a.ring_state[1] + N;
                    a.ring_state[0] = (long long)(np >= a.ring_cap ? np - a.ring_cap : np);
                    a.ring_state[1] = (long long)(sz > a.ring_cap ? a.ring_cap : sz);
                    a.ring_state[2] = 0;
                }
            }
        }
    }
    if constexpr (!POL) {
        // the launch's last workgroup inserts the neighbourhoods its launch solved (no k_insert
        // launch after every step launch): a ticket per workgroup, taken once all of its waves are
        // past their table reads; the other workgroups' queued entries were released by their
        // writers (rbf_miss_wave), the acquire below makes them visible here.  (Policy launches
        // have waves that leave early, so no workgroup barrier here: they keep k_insert.)
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned int t = atomicAdd(a.pend.ticket, 1u);
            if (t == gridDim.x - 1u) {
                __threadfence();
                DP<R>& P = *params<R>(a.P);
                insert_pending<R>(a.pend.count, a.pend.keys, a.pend.pay, a.pend.stats, (unsigned long long*)P.keys_cd, (R*)P.pay_cd, P.logcap_cd,
                                  (unsigned long long*)P.keys_cl, (R*)P.pay_cl, P.logcap_cl);
                *a.pend.ticket = 0u;
            }
        }
    }
    if (wc.w && __lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < kNWork; ++k)
            if (wc.w[k]) atomicAdd(&a.pend.stats[kStWork + k], (unsigned long long)wc.w[k]);
    }
#ifdef PD_STAMP
    PD_T(t_end);
    PD_ACC(6, t_end - t_store);
    if (__lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 7; ++k) atomicAdd(&a.pend.stats[kStStamp + k], acc_[k]);
        atomicAdd(&a.pend.stats[kStStamp + 7], 1ull);
        atomicAdd(&a.pend.stats[22], acc_[7]);
        atomicAdd(&a.pend.stats[23], acc_[8]);
        for (int k = 0; k < 4; ++k) atomicAdd(&a.pend.stats[24 + k], acc_[9 + k]);
        for (int k = 0; k < 4; ++k) atomicAdd(&a.pend.stats[28 + k], acc_[13 + k]);
    }
#endif
}

// ---------------------------------------------------------------- launchers
template <typename R, int PH, int RT, bool W, int LPE, bool RK> void launch_step(const StepArgs<R>& a, hipStream_t s) {
    unsigned grid = (unsigned)((a.n * LPE + kStepBlock - 1) / kStepBlock);
    // the SAC instantiation: heads from the caller (sac_mean) or from the kernel's own actor
    // prologue (sac_mlp.H, pd_step_sac_fused: sac_mean is then NULL and a.actions too)
    const bool sac = a.sac_mean != nullptr || a.sac_mlp.H != 0;
    if constexpr (LPE == 2 && !RK) {
        if (a.count_work && !sac) {
            hipLaunchKernelGGL((k_step<R, PH, RT, W, LPE, 0, RK, true>), dim3(grid), dim3(kStepBlock), 0, s, a);
            return;
        }
    }
    if constexpr (RT == 0 && PH <= 1 && !RK) {
        if (sac) {
            hipLaunchKernelGGL((k_step<R, PH, RT, W, LPE, 0, RK, false, true>), dim3(grid), dim3(kStepBlock), 0, s, a);
            return;
        }
    }
    if (sac) return;   // (no SAC instantiation for this kernel family: pdenv.hip refuses such handles first)
    hipLaunchKernelGGL((k_step<R, PH, RT, W, LPE, 0, RK>), dim3(grid), dim3(kStepBlock), 0, s, a);
}

template <typename R, int PH, bool W, int LPE> void launch_policy_lpe(const StepArgs<R>& a, int64_t n_launch,
                                                                      hipStream_t s) {
    unsigned grid = (unsigned)((n_launch * LPE + kStepBlock - 1) / kStepBlock);
    hipLaunchKernelGGL((k_step<R, PH, 1, W, LPE, 1>), dim3(grid), dim3(kStepBlock), 0, s, a);
}

}  // namespace pd
