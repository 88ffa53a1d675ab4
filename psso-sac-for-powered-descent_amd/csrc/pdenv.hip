// pdenv.hip -- host side and C ABI of libpdenv.so (MI355X / gfx950), plus its small kernels.
//
// The step kernel itself is k_step (pd_step_impl.h), instantiated in the kstep.hip translation
// units; this unit builds the per-handle parameter block and neighbourhood tables, owns the
// per-env SoA buffers in HBM, and launches.  See DESIGN.md for the roofline of each kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pdenv.h"
#include "pd_envdev.h"

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

// ---------------------------------------------------------------- per-env kernels
// The register state of one env written to its SoA slot (k_reset; the step kernel stores its
// own).  reset_cache: start the aero caches at the handle's initial keys.
template <typename R>
__device__ void store_env(const StepArgs<R>& a, DP<R>& P, uint32_t ui, const EnvRegs<R>& e, bool reset_cache) {
    const int64_t N = a.n;
#pragma unroll
    for (int k = 0; k < 11; ++k) ev(a.b.st + (k) * N, ui) = e.s[k];
    ev(a.b.vprev, ui) = e.vprev;
    ev(a.b.ghead, ui) = (uint8_t)e.ghead; ev(a.b.glen, ui) = (uint8_t)e.glen;
    ev(a.b.act, ui) = e.act0; ev(a.b.act + N, ui) = e.act1; ev(a.b.act + (2) * N, ui) = e.act2;
    ev(a.b.tid, ui) = (int8_t)e.tid;
    ev(a.b.epi, ui) = e.ep; ev(a.b.tstep, ui) = e.ts;
    ev(a.b.fin, ui) = 0;
    ev(a.b.wind, ui) = e.fu0; ev(a.b.wind + N, ui) = e.fu1; ev(a.b.wind + (2) * N, ui) = e.fv0; ev(a.b.wind + (3) * N, ui) = e.fv1;
    ev(a.b.wind + (4) * N, ui) = e.sgu; ev(a.b.wind + (5) * N, ui) = e.sgv;
    ev(a.b.wprof, ui) = (uint8_t)e.prof;
    if (reset_cache) {   // any valid 50-set is a correct start for the swap search
        ev(a.b.key, ui) = P.init_key_cd; ev(a.b.key + N, ui) = P.init_key_cl;
        ev(a.b.slot, ui) = -1; ev(a.b.slot + N, ui) = -1;
    }
}

// rocket_environment_pre_wrap.reset (base_environment.py:80-97) of every (masked) env
template <typename R>
__global__ __launch_bounds__(kBlock) void k_reset(StepArgs<R> a, const uint8_t* mask) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    if (mask && !mask[i]) return;
    DP<R>& P = *params<R>(a.P);
    const uint32_t ui = (uint32_t)i;
    EnvRegs<R> e;
    reset_values<R>(P, a, a.env_offset + (uint64_t)i, ev(a.b.epi, ui) + 1u,
                    (const double*)(uint64_t)&P.logtab.invc[0], (const double*)(uint64_t)&P.logtab.logc[0], e);
    store_env<R>(a, P, ui, e, true);
}

// Insert the neighbourhoods solved on device during the last launch (single thread; the only
// writer of the tables, stream-ordered between launches, so readers never race it).  The step
// launches insert their own (their last workgroup, k_step); this serves the policy rollouts and
// pd_flush_misses.
template <typename R>
__global__ void k_insert(Pending pend, unsigned long long* keys_cd, R* pay_cd, int lc_cd,
                         unsigned long long* keys_cl, R* pay_cl, int lc_cl) {
    if (threadIdx.x == 0) insert_pending<R>(pend.count, pend.keys, pend.pay, pend.stats, keys_cd, pay_cd, lc_cd, keys_cl, pay_cl, lc_cl);
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_observe(StepArgs<R> a, int obs_kind) {
    DP<R>& P = *params<R>(a.P);
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t N = a.n;
    if (i >= N) return;
    R s[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) s[k] = a.b.st[k * N + i];
    obs_write<R>(P, obs_kind, s, a.obs, (uint32_t)i);
}

// endo_atmospheric_model (atmosphere_dynamics.py:5-27) at n altitudes: out [3][n] = rho, p, a
template <typename R>
__global__ __launch_bounds__(kBlock) void k_atmosphere(StepArgs<R> a, const R* alt, R* out, int64_t n) {
    __shared__ R isa[9 * kIsaCols];
    DP<R>& P = *params<R>(a.P);
    if (threadIdx.x < 9) {
        const int k = threadIdx.x;
        R* r = isa + k * kIsaCols;
        r[0] = P.isa_Hb[k]; r[1] = P.isa_Tb[k]; r[2] = P.isa_beta[k]; r[3] = P.isa_pb[k];
        r[4] = P.isa_bt[k]; r[5] = P.isa_ex[k]; r[6] = P.isa_iso[k]; r[7] = R(0);
    }
    for (int t = threadIdx.x; t < 2 * kLogCellsD; t += kBlock) {
        s_logtab[t] = P.logtab_d.cell[t];
    }
    __syncthreads();
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    R rho, pr, as;
    atmosphere<R>(P, isa, alt[i], rho, pr, as);
    out[i] = rho; out[n + i] = pr; out[2 * n + i] = as;
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
    if ((T.entries + 1) * 2 > cap) return -1;   // full (load factor 1/2): no solve
    double aoa[kCols];
    for (int c = 0; c < kCols; ++c) aoa[c] = t.col_aoa[c];
    if (solve_neighbourhood(t.mach, t.coef, t.col_start, aoa, key, work.data(), pay.data()) != 0) return -1;
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
    // search buckets (pd_physics.h kLineBuckets), on the handle-precision breakpoints
    for (int b = 0; b < kLineBuckets; ++b) {
        const double w = 10.0 / kLineBuckets, lo = b * w - 1e-4, hi = (b + 1) * w + 1e-4;
        int nlo = 0, nhi = 0;
        for (size_t k = 0; k < B.size(); ++k) {
            nlo += (double)D.line_bp[li][k] < lo;
            nhi += (double)D.line_bp[li][k] < hi;
        }
        D.line_lb[li][b] = (uint16_t)(nlo | (nhi << 8));
    }
    for (size_t k = 0; k < K.size(); ++k) {
        D.line_key[li][k] = K[k];
        D.line_slot[li][k] = table_insert<R>(t, T, K[k], work, pay);
    }
    return PD_OK;
}

// Taylor pieces of clamped query line li (kTayCells cells of Mach [0, 10], one piece per (cell,
// neighbourhood interval) pair, piece index cell + l with l the interval's index -- the device's
// binary-search result -- so no piece table is needed).  Along the line a = const the thin-plate
// sum f(M) = sum_j c_j phi(|(M, a) - y_j|) + poly is analytic except at the points ON the line
// (d_a = 0, the C_L +10 line lies on the AoA-10 column): each term's singularities are at
// M = m_j +- i d_a.  A piece keeps the kTayExact terms whose singularity is nearest to its cell
// centre x0 as exact terms and expands the rest to degree kTayDeg in t = M - x0 (long double):
//   log((u0 + t)^2 + d^2) = log|z|^2 + sum_k 2 (-1)^(k+1) Re(z^-k) t^k / k,   z = u0 + i d,
//   times (|z|^2 + 2 u0 t + t^2), halved (phi = d2 log(d2) / 2), plus the degree-1 polynomial.
// The remaining singularities are >= 10x the cell half-width away (>= 0.17 on the C_D lines,
// >= 0.024 past the two nearest AoA-10 points), so the truncation is below binary64 rounding;
// every piece is checked at five points against the long double sum and a line whose worst
// error exceeds 1e-13 relative to sum |c_j phi_j| is left to the exact path (tay_off = -1).
// ---------------------------------------------------------------- smooth-function tables
// Least-squares fit of a degree-deg polynomial in t = x - c to f on [lo, hi] (c the centre), from
// 4 (deg + 1) Chebyshev nodes, in long double (monomials in s = t / h on [-1, 1]: well conditioned
// at these degrees); coefficients of t^k into out[0..deg].
template <typename F>
void fit_poly_ld(F&& f, long double lo, long double hi, int deg, long double* out) {
    const int M = 4 * (deg + 1), n = deg + 1;
    const long double c = (lo + hi) / 2, h = (hi - lo) / 2;
    long double A[12][12] = {}, b[12] = {};
    for (int m = 0; m < M; ++m) {
        const long double s = cosl(3.14159265358979323846264338327950288L * (m + 0.5L) / M);
        const long double v = f(c + h * s);
        long double pw[12];
        pw[0] = 1;
        for (int k = 1; k < n; ++k) pw[k] = pw[k - 1] * s;
        for (int i = 0; i < n; ++i) {
            b[i] += pw[i] * v;
            for (int j = 0; j < n; ++j) A[i][j] += pw[i] * pw[j];
        }
    }
    for (int k = 0; k < n; ++k) {   // Gaussian elimination with partial pivoting (normal equations)
        int pv = k;
        for (int i = k + 1; i < n; ++i) if (fabsl(A[i][k]) > fabsl(A[pv][k])) pv = i;
        for (int j = 0; j < n; ++j) std::swap(A[k][j], A[pv][j]);
        std::swap(b[k], b[pv]);
        for (int i = k + 1; i < n; ++i) {
            const long double l = A[i][k] / A[k][k];
            for (int j = k; j < n; ++j) A[i][j] -= l * A[k][j];
            b[i] -= l * b[k];
        }
    }
    long double x[12];
    for (int i = n - 1; i >= 0; --i) {
        long double s = b[i];
        for (int j = i + 1; j < n; ++j) s -= A[i][j] * x[j];
        x[i] = s / A[i][i];
    }
    long double hk = 1;
    for (int k = 0; k < n; ++k) { out[k] = x[k] / hk; hk *= h; }
}

// The device's Horner evaluation of coefficients q[0..deg] (in R) at t, in R
template <typename R> R horner_host(const R* q, int deg, R t) {
    R f = q[deg];
    for (int k = deg - 1; k >= 0; --k) f = (R)std::fma((double)f, (double)t, (double)q[k]);
    return f;
}

// The ISA atmosphere of atmosphere_dynamics.py:5-27 (ambiance restated, as the device's exact
// path and the oracle compute it) in long double, in layer i: rho, p, a at geometric altitude y
struct AtmLd { long double rho, p, a; };
AtmLd atm_exact_ld(const pd_params* P, int i, long double y) {
    const long double r = P->isa_r, R_ = P->isa_R, g0 = P->isa_g0;
    const long double H = r * y / (r + y), dH = H - (long double)P->isa_Hb[i];
    const long double Tb = P->isa_Tb[i], b = P->isa_beta[i], pb = P->isa_pb[i];
    const long double T = Tb + b * dH;
    const long double p = b != 0 ? pb * powl(1 + b / Tb * dH, -g0 / (b * R_)) : pb * expl(-g0 / (R_ * Tb) * dH);
    return {p / (R_ * T), p, sqrtl((long double)P->isa_kappa * R_ * T)};
}

// rho, p, a as piecewise polynomials in the geometric altitude (atmosphere_tab, pd_physics.h):
// cells of kAtmW metres over [0, isa_alt_max); a cell holds its piece and, past a layer boundary
// inside it (H = Hb: a kink of T, and a jump of p by the rounding of the tabulated pb), a second
// piece, with the boundary's Hb as the split (record word 1).  Every piece is
// checked at 33 points in R arithmetic (the device's Horner order) against the long double ISA;
// the worst relative error goes to max_rel (binary64: 2e-16 typical, 2e-15 at worst next to a
// layer boundary -- the closed form's own binary64 rounding is up to 5e-15 there, the pow of
// 1 + b/Tb dH rounded once amplified by its exponent, about 34).
template <typename R>
void build_atm_table(const pd_params* P, std::vector<R>& out, int& n_cells, double& max_rel) {
    const double w = kAtmW, top = P->isa_alt_max;
    n_cells = (int)std::ceil(top / w);
    out.assign((size_t)n_cells * kAtmStride, R(0));
    max_rel = 0;
    const long double r = P->isa_r;
    auto layer_of = [&](long double y) {
        const long double H = r * y / (r + y);
        int i = 0;
        for (int k = 0; k < 9; ++k) if ((long double)P->isa_Hb[k] <= H) i = k;
        return i;
    };
    for (int k = 0; k < n_cells; ++k) {
        const long double lo = (long double)k * w, hi = std::min<long double>((long double)(k + 1) * w, top);
        const int il = layer_of(lo), ih = layer_of(hi - 1e-9L);
        long double split = hi;
        if (ih != il) {   // the boundary y of H = Hb[ih]: y = r Hb / (r - Hb)
            const long double Hb = P->isa_Hb[ih];
            split = r * Hb / (r - Hb);
        }
        for (int half = 0; half < (ih != il ? 2 : 1); ++half) {
            const long double a0 = half ? split : lo, a1 = half ? hi : split;
            const int li = half ? ih : il;
            R* rec = out.data() + (size_t)k * kAtmStride + half * kAtmRec;
            long double q[3][kAtmDeg + 1];
            for (int fn = 0; fn < 3; ++fn)
                fit_poly_ld([&](long double y) { const AtmLd v = atm_exact_ld(P, li, y);
                                                 return fn == 0 ? v.p : (fn == 1 ? v.rho : v.a); },
                            a0, a1, kAtmDeg, q[fn]);
            const long double c = (a0 + a1) / 2;
            rec[0] = (R)c;
            // the split as the layer's base H: the device takes the upper piece where the exact path
            // takes the upper layer, Hb <= r alt / (r + alt) in R (the ISA's pb are rounded
            // constants: p jumps by ~4e-6 across 47 km, so the side must be the exact path's)
            rec[1] = half || ih == il ? (R)1e30 : (R)P->isa_Hb[ih];
            for (int fn = 0; fn < 3; ++fn)
                for (int j = 0; j <= kAtmDeg; ++j) rec[2 + fn * (kAtmDeg + 1) + j] = (R)q[fn][j];
            for (int m = 0; m <= 32; ++m) {
                const long double y = a0 + (a1 - a0) * (m == 0 ? 1e-6L : (m == 32 ? 0.999999L : m / 32.0L));
                const AtmLd v = atm_exact_ld(P, li, y);
                const R t = (R)y - rec[0];
                const long double ex[3] = {v.p, v.rho, v.a};
                for (int fn = 0; fn < 3; ++fn) {
                    const R f = horner_host<R>(rec + 2 + fn * (kAtmDeg + 1), kAtmDeg, t);
                    max_rel = std::max(max_rel, (double)(fabsl((long double)f - ex[fn]) / fabsl(ex[fn])));
                }
            }
        }
        if (ih == il) {   // (no second piece: the split never triggers; mirror the first anyway)
            R* rec = out.data() + (size_t)k * kAtmStride;
            std::copy(rec, rec + kAtmRec, rec + kAtmRec);
        }
    }
}

struct TayStats { double max_abs = 0, max_rel = 0; int64_t pieces = 0; };

template <typename R>
void build_taylor(const pd_aero_table& t, int li, DevParams<R>& D, std::vector<R>& out, TayStats& ts) {
    D.tay_off[li] = -1;
    const int nb = D.line_nbp[li];
    if (nb < 0) return;
    const long double a = (long double)D.line_a[li];
    const double w = 10.0 / kTayCells;
    std::vector<double> bp(nb);
    for (int k = 0; k < nb; ++k) bp[k] = (double)D.line_bp[li][k];
    auto count_below = [&](double x) { return (int)(std::lower_bound(bp.begin(), bp.end(), x) - bp.begin()); };
    // the binary64 payload of every interval (the same solve as the tables')
    std::vector<std::vector<double>> pays(nb + 1, std::vector<double>(kPay));
    std::vector<double> work(kScratch);
    std::vector<double> aoa(kCols);
    for (int c = 0; c < kCols; ++c) aoa[c] = t.col_aoa[c];
    for (int l = 0; l <= nb; ++l)
        if (solve_neighbourhood(t.mach, t.coef, t.col_start, aoa.data(), D.line_key[li][l], work.data(), pays[l].data()) != 0)
            return;
    const size_t base = out.size();
    out.resize(base + (size_t)(kTayCells + nb) * kTayStride, R(0));
    double worst_rel = 0.0;
    for (int cell = 0; cell < kTayCells; ++cell) {
        const double lo = cell * w, hi = (cell + 1) * w;
        const long double x0 = (long double)cell * w + 0.5L * w;
        for (int l = count_below(lo); l <= count_below(hi) && l <= nb; ++l) {
            const double* pay = pays[l].data();
            const uint8_t* ib = (const uint8_t*)(pay + kPayIdx);
            // the terms: Mach, d_a^2, coefficient
            long double m[2 * kPairs], dl2[2 * kPairs], cf[2 * kPairs], z2[2 * kPairs];
            int nt = 0;
            for (int k = 0; k < kPairs; ++k)
                for (int i = 0; i < 2; ++i) {
                    const double c = pay[2 * k + i];
                    if (c == 0.0) continue;
                    const bool g2 = i == 1 && slot_general(k);   // a general slot's second point
                    const int pidx = g2 ? ib[second_entry_pos(k)] : ib[pair_entry_pos(k)] + i;
                    const long double da = a - (long double)ib[g2 ? second_aoa_pos(k) : pair_aoa_pos(k)];
                    m[nt] = t.mach[pidx]; dl2[nt] = da * da; cf[nt] = c;
                    const long double u0 = x0 - m[nt];
                    z2[nt] = u0 * u0 + dl2[nt];
                    ++nt;
                }
            int ex[kTayExact];
            for (int e = 0; e < kTayExact; ++e) {
                int best = -1;
                for (int j = 0; j < nt; ++j) {
                    bool used = false;
                    for (int q = 0; q < e; ++q) used |= ex[q] == j;
                    if (!used && (best < 0 || z2[j] < z2[best])) best = j;
                }
                ex[e] = best;
            }
            long double B[kTayDeg + 1] = {};
            for (int j = 0; j < nt; ++j) {
                bool is_ex = false;
                for (int e = 0; e < kTayExact; ++e) is_ex |= ex[e] == j;
                if (is_ex) continue;
                const long double u0 = x0 - m[j], d = sqrtl(dl2[j]);
                // z^-k = conj(z)^k / |z|^(2k): real parts by the recurrence on (re, im)
                long double L[kTayDeg + 1];
                L[0] = logl(z2[j]);
                long double zr = 1.0L, zi = 0.0L;   // (conj(z) / |z|^2)^k
                const long double ir = u0 / z2[j], ii = -d / z2[j];
                for (int k = 1; k <= kTayDeg; ++k) {
                    const long double nr = zr * ir - zi * ii, ni = zr * ii + zi * ir;
                    zr = nr; zi = ni;
                    L[k] = 2.0L * ((k & 1) ? 1.0L : -1.0L) * zr / k;
                }
                const long double Q[3] = {z2[j], 2.0L * u0, 1.0L};
                for (int n = 0; n <= kTayDeg; ++n) {
                    long double b = 0.0L;
                    for (int q = 0; q < 3 && q <= n; ++q) b += Q[q] * L[n - q];
                    B[n] += 0.5L * cf[j] * b;
                }
            }
            const long double p0 = pay[kPayPoly], p1 = pay[kPayPoly + 1], p2 = pay[kPayPoly + 2];
            const long double sh0 = pay[kPaySS + 0], sh1 = pay[kPaySS + 1], sc0 = pay[kPaySS + 2], sc1 = pay[kPaySS + 3];
            B[0] += p0 + (x0 - sh0) / sc0 * p1 + (a - sh1) / sc1 * p2;
            B[1] += p1 / sc0;
            R* rec = out.data() + base + (size_t)(cell + l) * kTayStride;
            for (int n = 0; n <= kTayDeg; ++n) rec[n] = (R)B[n];
            for (int e = 0; e < kTayExact; ++e) {
                R* x = rec + kTayDeg + 1 + 3 * e;
                if (ex[e] < 0) { x[0] = R(0); x[1] = R(0); x[2] = R(1); continue; }
                x[0] = (R)m[ex[e]]; x[1] = (R)(cf[ex[e]] * 0.125L); x[2] = (R)dl2[ex[e]];
            }
            // check: five points of the piece's part of the cell
            const double plo = std::max(lo, l > 0 ? bp[l - 1] : lo), phi = std::min(hi, l < nb ? bp[l] : hi);
            for (int q = 0; q < 5; ++q) {
                const double M = plo + (phi - plo) * (0.02 + 0.24 * q);
                long double exact = p0 + ((long double)M - sh0) / sc0 * p1 + (a - sh1) / sc1 * p2, mag = 0.0L;
                for (int j = 0; j < nt; ++j) {
                    const long double dm = M - m[j], d2 = dm * dm + dl2[j];
                    const long double ph = d2 > 0 ? 0.5L * cf[j] * d2 * logl(d2) : 0.0L;
                    exact += ph; mag += fabsl(ph);
                }
                const double tt = M - (double)x0;
                double f = (double)rec[kTayDeg];
                for (int n = kTayDeg - 1; n >= 0; --n) f = std::fma(f, tt, (double)rec[n]);
                for (int e = 0; e < kTayExact; ++e) {
                    const R* x = rec + kTayDeg + 1 + 3 * e;
                    const double dm = M - (double)x[0], d2 = std::fma(dm, dm, (double)x[2]);
                    if (d2 > 0) f = std::fma((double)x[1] * d2, 4.0 * std::log(d2), f);
                }
                const double err = std::fabs(f - (double)exact);
                ts.max_abs = std::max(ts.max_abs, err);
                const double rel = err / (double)(mag + fabsl(exact) + 1e-300L);
                worst_rel = std::max(worst_rel, rel);
            }
            ++ts.pieces;
        }
    }
    ts.max_rel = std::max(ts.max_rel, worst_rel);
    const double lim = sizeof(R) == 8 ? 1e-13 : 1e-6;
    if (worst_rel > lim) { out.resize(base); return; }
    D.tay_off[li] = (int)(base / kTayStride);
}

// The same 50-NN key by selection instead of a full sort: the 50 smallest under the total order
// (distance, point index) are exactly stable_sort's first 50, so the key is host_knn_key's.
uint64_t knn_key_select(const pd_aero_table& t, double M, double a) {
    double d[PD_MAX_PTS];
    int id[PD_MAX_PTS], col[PD_MAX_PTS];
    int n = 0;
    for (int c = 0; c < t.n_cols; ++c)
        for (int k = 0; k < t.col_len[c]; ++k, ++n) {
            double dm = M - t.mach[t.col_start[c] + k], da = a - t.col_aoa[c];
            d[n] = dm * dm + da * da;
            id[n] = n;
            col[n] = c;
        }
    std::nth_element(id, id + (kNbr - 1), id + n, [&](int x, int y) { return d[x] < d[y] || (d[x] == d[y] && x < y); });
    int lo[kCols], hi[kCols];
    for (int c = 0; c < kCols; ++c) { lo[c] = 1 << 20; hi[c] = -1; }
    int base[kCols] = {0, 0, 0, 0, 0};
    for (int c = 1; c < t.n_cols; ++c) base[c] = base[c - 1] + t.col_len[c - 1];
    for (int j = 0; j < kNbr; ++j) {
        const int p = id[j], c = col[p], k = p - base[c];
        lo[c] = std::min(lo[c], k); hi[c] = std::max(hi[c], k);
    }
    int L[kCols], N[kCols];
    for (int c = 0; c < kCols; ++c) {
        if (hi[c] < 0) { L[c] = 0; N[c] = 0; } else { L[c] = lo[c]; N[c] = hi[c] - lo[c] + 1; }
    }
    return key_pack(L, N);
}

// Keys of one interior candidate grid: cell centres and corners, and for every cell whose
// corners disagree with its centre a kGridSub x kGridSub sub-grid (centres and corners).  Pure
// functions of the table, so they are computed once per process (threads over cells) and
// cached; slots are assigned per handle.
struct BisectHost { double nx, ny, c, tau; uint64_t key_a, key_b; bool ok_a, ok_b; };
struct GridKeys {
    int nm = 0, na = 0;
    std::vector<uint64_t> centre, corner;            // [nm][na], [nm + 1][na + 1]
    std::vector<int> refined;                        // cell index of each refined cell
    std::vector<uint64_t> sub_centre, sub_corner;    // [ref][S][S], [ref][S + 1][S + 1]
    std::vector<int> sub_bis;                        // [ref][S][S]: index into bis, -1 none
    std::vector<BisectHost> bis;
};

// The one point swap between two keys (A \ B = {p}, B \ A = {q}), as table point indices;
// false if the keys differ otherwise
bool single_swap(const pd_aero_table& t, uint64_t ka, uint64_t kb, int& p, int& q) {
    int la[kCols], na[kCols], lb[kCols], nb[kCols];
    key_unpack(ka, la, na);
    key_unpack(kb, lb, nb);
    int np = 0, nq = 0;
    p = q = -1;
    for (int c = 0; c < kCols; ++c) {
        for (int i = la[c]; i < la[c] + na[c]; ++i)
            if (!(nb[c] > 0 && i >= lb[c] && i < lb[c] + nb[c])) { ++np; p = t.col_start[c] + i; }
        for (int i = lb[c]; i < lb[c] + nb[c]; ++i)
            if (!(na[c] > 0 && i >= la[c] && i < la[c] + na[c])) { ++nq; q = t.col_start[c] + i; }
    }
    return np == 1 && nq == 1;
}
double point_aoa(const pd_aero_table& t, int idx) {
    int c = 0;
    while (c + 1 < t.n_cols && idx >= t.col_start[c + 1]) ++c;
    return t.col_aoa[c];
}

// Bisector record of a non-exact sub-cell [m0, m1] x [a0, a1] whose sample keys are {A, B} (see
// GridBisect): the bisector of the swapped points, and for each side whether its part of the
// cell, tau off the line, provably has the side's key (every vertex of the clipped polygon does).
bool make_bisect(const pd_aero_table& t, double m0, double m1, double a0, double a1, uint64_t ka, uint64_t kb,
                 BisectHost& out) {
    int p, q;
    if (!single_swap(t, ka, kb, p, q)) {
        if (!single_swap(t, kb, ka, p, q)) return false;
        std::swap(ka, kb);
    }
    const double pm = t.mach[p], pa = point_aoa(t, p), qm = t.mach[q], qa = point_aoa(t, q);
    out.nx = 2.0 * (qm - pm); out.ny = 2.0 * (qa - pa);
    out.c = (qm * qm + qa * qa) - (pm * pm + pa * pa);
    out.tau = 1e-9 * (std::fabs(out.nx) * 10.0 + std::fabs(out.ny) * 10.0 + std::fabs(out.c) + 1.0);
    out.key_a = ka; out.key_b = kb;
    auto side_ok = [&](double sign) {
        // the side's part of the cell kept 2 tau off the line (A: s <= -2 tau, B: s >= 2 tau) is
        // the convex polygon f <= 0; every vertex must carry the side's key (the device trusts
        // |s| > 3 tau, inside it)
        const double cx[4] = {m0, m1, m1, m0}, cy[4] = {a0, a0, a1, a1};
        std::vector<std::pair<double, double>> poly;
        auto f = [&](double x, double y) { return -sign * (out.nx * x + out.ny * y - out.c) + 2.0 * out.tau; };
        for (int k = 0; k < 4; ++k) {
            const int k1 = (k + 1) & 3;
            const double f0 = f(cx[k], cy[k]), f1 = f(cx[k1], cy[k1]);
            if (f0 <= 0) poly.push_back({cx[k], cy[k]});
            if ((f0 < 0) != (f1 < 0) && f0 != f1) {
                const double u = f0 / (f0 - f1);
                poly.push_back({cx[k] + u * (cx[k1] - cx[k]), cy[k] + u * (cy[k1] - cy[k])});
            }
        }
        if (poly.empty()) return false;
        const uint64_t want = sign < 0 ? ka : kb;
        for (auto& v : poly)
            if (knn_key_select(t, std::min(std::max(v.first, m0), m1), std::min(std::max(v.second, a0), a1)) != want)
                return false;
        return true;
    };
    out.ok_a = side_ok(-1.0);
    out.ok_b = side_ok(+1.0);
    return out.ok_a || out.ok_b;
}

template <typename F> void parallel_for(int64_t n, F f) {
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 64) nt = 1;
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; ++k)
        th.emplace_back([=] { for (int64_t i = (int64_t)k; i < n; i += nt) f(i); });
    for (auto& x : th) x.join();
}

const GridKeys& grid_keys(const pd_aero_table& t, double a0, double a1, int nm, int na) {
    static std::mutex mu;
    static std::map<uint64_t, GridKeys> cache;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; ++i) { h ^= ((const uint8_t*)p)[i]; h *= 1099511628211ull; }
    };
    mix(&t, sizeof(t)); mix(&a0, 8); mix(&a1, 8); mix(&nm, 4); mix(&na, 4);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(h);
    if (it != cache.end()) return it->second;
    GridKeys& g = cache[h];
    g.nm = nm; g.na = na;
    const double dm = 10.0 / nm, da = (a1 - a0) / na;
    const int S = kGridSub;
    g.corner.resize((size_t)(nm + 1) * (na + 1));
    g.centre.resize((size_t)nm * na);
    parallel_for(nm + 1, [&](int64_t im) {
        for (int ia = 0; ia <= na; ++ia) g.corner[(size_t)im * (na + 1) + ia] = knn_key_select(t, im * dm, a0 + ia * da);
        if (im < nm)
            for (int ia = 0; ia < na; ++ia)
                g.centre[(size_t)im * na + ia] = knn_key_select(t, (im + 0.5) * dm, a0 + (ia + 0.5) * da);
    });
    for (int im = 0; im < nm; ++im)
        for (int ia = 0; ia < na; ++ia) {
            const uint64_t key = g.centre[(size_t)im * na + ia];
            bool same = true;
            for (int c = 0; c < 4 && same; ++c) same = g.corner[(size_t)(im + (c >> 1)) * (na + 1) + ia + (c & 1)] == key;
            if (!same) g.refined.push_back(im * na + ia);
        }
    const int64_t nr = (int64_t)g.refined.size();
    g.sub_corner.resize((size_t)nr * (S + 1) * (S + 1));
    g.sub_centre.resize((size_t)nr * S * S);
    parallel_for(nr, [&](int64_t r) {
        const int im = g.refined[r] / na, ia = g.refined[r] % na;
        for (int jm = 0; jm <= S; ++jm)
            for (int ja = 0; ja <= S; ++ja) {
                g.sub_corner[((size_t)r * (S + 1) + jm) * (S + 1) + ja] =
                    knn_key_select(t, (im + (double)jm / S) * dm, a0 + (ia + (double)ja / S) * da);
                if (jm < S && ja < S)
                    g.sub_centre[((size_t)r * S + jm) * S + ja] =
                        knn_key_select(t, (im + (jm + 0.5) / S) * dm, a0 + (ia + (ja + 0.5) / S) * da);
            }
    });
    // non-exact sub-cells split by one bisector between two keys: records (threads per refined
    // cell, then gathered in order)
    g.sub_bis.assign((size_t)nr * S * S, -1);
    std::vector<std::vector<std::pair<int, BisectHost>>> found((size_t)nr);
    parallel_for(nr, [&](int64_t r) {
        const int im = g.refined[r] / na, ia = g.refined[r] % na;
        for (int jm = 0; jm < S; ++jm)
            for (int ja = 0; ja < S; ++ja) {
                const uint64_t kc = g.sub_centre[((size_t)r * S + jm) * S + ja];
                uint64_t other = kc;
                bool two = true, exact = true;
                for (int c = 0; c < 4 && two; ++c) {
                    const uint64_t k = g.sub_corner[((size_t)r * (S + 1) + jm + (c >> 1)) * (S + 1) + ja + (c & 1)];
                    if (k == kc) continue;
                    exact = false;
                    if (other == kc) other = k;
                    else if (k != other) two = false;
                }
                if (exact || !two) continue;
                BisectHost b;
                const double m0 = (im + (double)jm / S) * dm, m1 = (im + (double)(jm + 1) / S) * dm;
                const double c0 = a0 + (ia + (double)ja / S) * da, c1 = a0 + (ia + (double)(ja + 1) / S) * da;
                if (make_bisect(t, m0, m1, c0, c1, kc, other, b)) found[r].push_back({jm * S + ja, b});
            }
    });
    for (int64_t r = 0; r < nr; ++r)
        for (auto& fb : found[r]) {
            g.sub_bis[(size_t)r * S * S + fb.first] = (int)g.bis.size();
            g.bis.push_back(fb.second);
        }
    return g;
}

// Candidate grid over the interior query domain [0, 10] Mach x [a0, a1]: the 50-NN key at
// every cell centre, inserted into the table.  A 50-NN region is an intersection of
// half-planes (order-k Voronoi cell), hence convex: when all four corners of a cell carry the
// centre's key, the whole cell does, and the slot is flagged kGridExact so that device lookups
// skip the verification.  A cell whose corners disagree is refined into kGridSub x kGridSub
// sub-cells with the same construction (flagged kGridRefine, its sub-grid index in the low
// bits), so that only queries near a region boundary are verified on the device.
// The interior candidate grid of table tb (0: C_D, 1: C_L): Mach [0, 10] x AoA abscissa [a0, a1]
// (C_D in [-radians(10), radians(10)], C_L in [0, 10]) in nm x na cells.  800 x 32 / 800 x 400
// cells, refined cells in 8 x 8 sub-cells, two-region sub-cells split by their bisector: < 0.1 %
// of queries verified (measured against 400 x 200 and 1600 x 800)
void grid_geometry(int tb, int& nm, int& na, double& a0, double& a1) {
    const int d[4] = {800, 32, 800, 400};
    nm = d[2 * tb]; na = d[2 * tb + 1];
    a0 = tb ? 0.0 : -10.0 * kDeg2Rad;
    a1 = tb ? 10.0 : 10.0 * kDeg2Rad;
}

struct CellPieces;
bool cell_ok(const CellPieces* cp, int64_t cell, bool f32);
bool fine_is(const CellPieces* cp, int im, int ia, int jm, int ja, int na, uint32_t want, bool f32);
int cell_bis(const CellPieces* cp, int bi, bool side_b, bool f32);

template <typename R>
pd_status build_grid(const pd_aero_table& t, double a0, double a1, int nm, int na, Table<R>& T,
                     std::vector<unsigned long long>& gk, std::vector<int>& gs,
                     std::vector<unsigned long long>& sk, std::vector<int>& ss, std::vector<GridBisect>& bs,
                     const CellPieces* cp = nullptr) {
    const GridKeys& g = grid_keys(t, a0, a1, nm, na);
    const int S = kGridSub;
    const bool f32 = sizeof(R) == 4;
    gk.assign((size_t)nm * na, 0); gs.assign((size_t)nm * na, -1);
    std::vector<double> work(kScratch), pay(kPay);
    auto slot_of = [&](uint64_t key, bool exact) {
        int slot = table_insert<R>(t, T, key, work, pay);
        return slot < 0 ? -1 : (slot | (exact ? kGridExact : 0));
    };
    for (int im = 0; im < nm; ++im)
        for (int ia = 0; ia < na; ++ia) {
            const uint64_t key = g.centre[(size_t)im * na + ia];
            gk[(size_t)im * na + ia] = key;
            gs[(size_t)im * na + ia] = slot_of(key, true);   // refined cells overwritten below
            if (gs[(size_t)im * na + ia] >= 0 && cell_ok(cp, (int64_t)im * na + ia, f32)) gs[(size_t)im * na + ia] |= kGridPiece;
        }
    const int64_t nr = (int64_t)g.refined.size();
    if (nr >= kGridRefine) return fail(PD_ERR_INVALID, "too many refined grid cells");
    sk.assign((size_t)nr * S * S, 0); ss.assign((size_t)nr * S * S, -1);
    for (int64_t r = 0; r < nr; ++r) {
        gs[g.refined[r]] = kGridRefine | (int)r;
        for (int jm = 0; jm < S; ++jm)
            for (int ja = 0; ja < S; ++ja) {
                const size_t q = ((size_t)r * S + jm) * S + ja;
                const uint64_t key = g.sub_centre[q];
                bool exact = true;
                for (int c = 0; c < 4 && exact; ++c)
                    exact = g.sub_corner[((size_t)r * (S + 1) + jm + (c >> 1)) * (S + 1) + ja + (c & 1)] == key;
                sk[q] = key;
                ss[q] = slot_of(key, exact);
                const int bi = g.sub_bis[q];
                // (binary32 handles read the bisector records through the fine index only: their
                // record path verifies refined cells)
                if (!exact && bi >= 0 && (sizeof(R) == 8 || cp) && bs.size() < (size_t)kGridBisect) {
                    const BisectHost& h = g.bis[bi];
                    GridBisect b{};
                    b.nx = h.nx; b.ny = h.ny; b.c = h.c; b.tau = h.tau; b.key_a = h.key_a; b.key_b = h.key_b;
                    const int sa = table_insert<R>(t, T, h.key_a, work, pay), sb = table_insert<R>(t, T, h.key_b, work, pay);
                    b.slot_a = sa < 0 ? -1 : (sa | (h.ok_a ? kGridExact : 0));
                    b.slot_b = sb < 0 ? -1 : (sb | (h.ok_b ? kGridExact : 0));
                    b.piece_a = cell_bis(cp, bi, false, f32); b.piece_b = cell_bis(cp, bi, true, f32);
                    if (cp && !fine_is(cp, g.refined[r] / na, g.refined[r] % na, jm, ja, na,
                                       kFineBisect | kFineRefined | (uint32_t)bs.size(), f32))
                        return fail(PD_ERR_INVALID, "cell pieces: fine index does not match the bisector records");
                    ss[q] = kGridBisect | (int)bs.size();
                    bs.push_back(b);
                }
            }
    }
    return PD_OK;
}

// ---------------------------------------------------------------- cell pieces
// Interior queries of the binary64 handle are evaluated from cell pieces (pd_step.h kCellDeg):
// for every interior grid cell and every neighbourhood that owns part of it, the thin-plate sum
// s(x) = sum_j c_j phi(|x - y_j|) + poly(x) of that neighbourhood restricted to the cell.  s is
// analytic over the cell except at the table points themselves (phi = r^2 log r), so the
// kCellExact points nearest to the cell centre stay exact terms and the rest, with scipy's
// degree-1 polynomial, is a polynomial of total degree kCellDeg in the cell coordinates (u, v) in
// [-1, 1]^2 (the device's 2 (M inv_dm - im) - 1 and 2 ((a - a0) inv_da - ia) - 1): the least-
// squares fit (long double Householder QR, once) on the cell's 10 x 10 tensor Chebyshev grid of
// the far terms evaluated there.  Every piece is then evaluated as the device does (binary64
// Horner, exact terms) at 8 quasi-random points of the cell and compared with the long double
// sum of all 50 terms: a piece whose error exceeds kCellTol relative to sum |c_j phi_j| is not
// used (the query goes to the payload sum).  Pure functions of the table and the grid: built once
// per process (threads over pieces) and cached, like the grid keys.
constexpr double kCellTol = 1e-14;
constexpr int kCellNodes = 10;

struct CellPieces {
    std::vector<double> rec;          // [n][kCellStride]: exact cells at their cell index, then refined cells' pieces
    std::vector<uint8_t> cell_ok;     // [nm na] the exact cell's own piece is valid
    std::vector<int> sub_piece;       // [refined][S][S] piece of an exact sub-cell's key (-1 none)
    std::vector<int> bis_a, bis_b;    // per GridKeys bisector record: each trusted side's piece
    std::vector<uint32_t> fine;       // [nm S][na S] fine index (pd_step.h kFinePiece)
    double max_rel = 0, build_s = 0;
    int64_t pieces = 0, rejected = 0;
    std::vector<double> err;          // per piece: the binary64 check's error (INFINITY: unused slot)
    std::vector<double> scale;        // per piece: the largest sum |c_j phi_j| + |s| at its check points
    std::vector<int> cell_of;         // per piece: its grid cell
    // the fine index's inputs (kept for the binary32 variant)
    int nm = 0, na = 0;
    double a0 = 0, dm = 0, da = 0;
    std::vector<uint8_t> refined;
    std::vector<int> ridx;
    std::vector<int64_t> bs_of;
    // binary32 handles (ensure_f32): the records in floats (kCellStrideF), each checked in binary32
    // against its binary64 piece; validity, sub-cell pieces, bisector sides and fine index of
    // the pieces that pass
    bool have32 = false;
    std::vector<float> rec32;
    std::vector<uint8_t> cell_ok32;
    std::vector<int> sub_piece32, bis_a32, bis_b32;
    std::vector<uint32_t> fine32;
    double max_rel32 = 0;
    int64_t rejected32 = 0;
};
// binary32 pieces: error bound relative to sum |c_j phi_j| + |s| (the binary32 balanced payload
// sums, which these replace, round at ~50 eps_32 of the same scale)
constexpr double kCellTol32 = 2e-6;

// The fit operator: pinv[c][node] of the (node x coefficient) monomial design matrix, columns in
// record order (u^i v^j, i = kCellDeg .. 0, j = kCellDeg - i .. 0), nodes (k, l) -> (x_k, x_l)
const std::vector<long double>& cell_fit_operator() {
    static std::vector<long double> pinv;
    static std::once_flag once;
    std::call_once(once, [] {
        const int NN = kCellNodes * kCellNodes, NC = kCellCoef;
        long double x[kCellNodes];
        for (int k = 0; k < kCellNodes; ++k) x[k] = cosl((2 * k + 1) * 3.141592653589793238462643383279502884L / (2 * kCellNodes));
        std::vector<long double> A((size_t)NN * NC), Q((size_t)NN * NN, 0.0L);
        for (int k = 0; k < kCellNodes; ++k)
            for (int l = 0; l < kCellNodes; ++l) {
                int c = 0;
                for (int i = kCellDeg; i >= 0; --i)
                    for (int j = kCellDeg - i; j >= 0; --j) A[(size_t)(k * kCellNodes + l) * NC + c++] = powl(x[k], i) * powl(x[l], j);
            }
        for (int r = 0; r < NN; ++r) Q[(size_t)r * NN + r] = 1.0L;   // accumulates Q^T
        for (int c = 0; c < NC; ++c) {
            long double nrm = 0.0L;
            for (int r = c; r < NN; ++r) nrm += A[(size_t)r * NC + c] * A[(size_t)r * NC + c];
            nrm = sqrtl(nrm);
            const long double alpha = A[(size_t)c * NC + c] > 0 ? -nrm : nrm;
            std::vector<long double> v(NN, 0.0L);
            for (int r = c; r < NN; ++r) v[r] = A[(size_t)r * NC + c];
            v[c] -= alpha;
            long double vv = 0.0L;
            for (int r = c; r < NN; ++r) vv += v[r] * v[r];
            if (vv == 0.0L) continue;
            for (int cc = c; cc < NC; ++cc) {
                long double d = 0.0L;
                for (int r = c; r < NN; ++r) d += v[r] * A[(size_t)r * NC + cc];
                d = 2.0L * d / vv;
                for (int r = c; r < NN; ++r) A[(size_t)r * NC + cc] -= d * v[r];
            }
            for (int cc = 0; cc < NN; ++cc) {
                long double d = 0.0L;
                for (int r = c; r < NN; ++r) d += v[r] * Q[(size_t)r * NN + cc];
                d = 2.0L * d / vv;
                for (int r = c; r < NN; ++r) Q[(size_t)r * NN + cc] -= d * v[r];
            }
        }
        // R X = (Q^T)[0:NC]  ->  X = pinv
        pinv.assign((size_t)NC * NN, 0.0L);
        for (int cc = 0; cc < NN; ++cc)
            for (int c = NC - 1; c >= 0; --c) {
                long double s = Q[(size_t)c * NN + cc];
                for (int k = c + 1; k < NC; ++k) s -= A[(size_t)c * NC + k] * pinv[(size_t)k * NN + cc];
                pinv[(size_t)c * NN + cc] = s / A[(size_t)c * NC + c];
            }
    });
    return pinv;
}

// The terms of a neighbourhood's payload (Mach, AoA, coefficient) and its polynomial
struct NbrTerms {
    int nt = 0;
    double m[2 * kPairs], a[2 * kPairs], c[2 * kPairs];
    double p0 = 0, p1 = 0, p2 = 0, sh0 = 0, sh1 = 0, sc0 = 1, sc1 = 1;
    bool ok = false;
};
NbrTerms nbr_terms(const pd_aero_table& t, uint64_t key) {
    NbrTerms T;
    std::vector<double> work(kScratch), pay(kPay);
    double aoa[kCols];
    for (int c = 0; c < kCols; ++c) aoa[c] = t.col_aoa[c];
    if (solve_neighbourhood(t.mach, t.coef, t.col_start, aoa, key, work.data(), pay.data()) != 0) return T;
    const uint8_t* ib = (const uint8_t*)(pay.data() + kPayIdx);
    for (int k = 0; k < kPairs; ++k)
        for (int i = 0; i < 2; ++i) {
            const double c = pay[2 * k + i];
            if (c == 0.0) continue;
            const bool g2 = i == 1 && slot_general(k);
            T.m[T.nt] = t.mach[g2 ? ib[second_entry_pos(k)] : ib[pair_entry_pos(k)] + i];
            T.a[T.nt] = ib[g2 ? second_aoa_pos(k) : pair_aoa_pos(k)];
            T.c[T.nt] = c;
            ++T.nt;
        }
    T.p0 = pay[kPayPoly]; T.p1 = pay[kPayPoly + 1]; T.p2 = pay[kPayPoly + 2];
    T.sh0 = pay[kPaySS + 0]; T.sh1 = pay[kPaySS + 1]; T.sc0 = pay[kPaySS + 2]; T.sc1 = pay[kPaySS + 3];
    T.ok = true;
    return T;
}

// One piece: key's sum over cell (im, ia) into rec; returns the validation error (relative to
// sum |c_j phi_j|), or +inf if the neighbourhood did not solve
double make_cell_piece(const NbrTerms& T, int im, int ia, double dm, double da, double a0, double* rec,
                       double* scale = nullptr) {
    if (!T.ok) return INFINITY;
    const std::vector<long double>& pinv = cell_fit_operator();
    const double cm = (im + 0.5) * dm, ca = a0 + (ia + 0.5) * da, hm = 0.5 * dm, ha = 0.5 * da;
    // exact terms: the kCellExact nearest to the centre (ties by term order)
    int ex[kCellExact];
    bool is_ex[2 * kPairs] = {};
    for (int e = 0; e < kCellExact; ++e) {
        int best = -1;
        double bd = 0;
        for (int j = 0; j < T.nt; ++j) {
            if (is_ex[j]) continue;
            const double d = (cm - T.m[j]) * (cm - T.m[j]) + (ca - T.a[j]) * (ca - T.a[j]);
            if (best < 0 || d < bd) { best = j; bd = d; }
        }
        ex[e] = best;
        if (best >= 0) is_ex[best] = true;
    }
    const int NN = kCellNodes * kCellNodes;
    long double F[kCellNodes * kCellNodes];
    long double xn[kCellNodes];
    for (int k = 0; k < kCellNodes; ++k) xn[k] = cosl((2 * k + 1) * 3.141592653589793238462643383279502884L / (2 * kCellNodes));
    for (int k = 0; k < kCellNodes; ++k)
        for (int l = 0; l < kCellNodes; ++l) {
            const long double M = cm + xn[k] * hm, a = ca + xn[l] * ha;
            long double s = T.p0 + (M - T.sh0) / T.sc0 * T.p1 + (a - T.sh1) / T.sc1 * T.p2;
            for (int j = 0; j < T.nt; ++j) {
                if (is_ex[j]) continue;
                const long double dmj = M - T.m[j], daj = a - T.a[j], d2 = dmj * dmj + daj * daj;
                if (d2 > 0) s += 0.5L * T.c[j] * d2 * (long double)std::log((double)d2);
            }
            F[k * kCellNodes + l] = s;
        }
    for (int c = 0; c < kCellCoef; ++c) {
        long double s = 0.0L;
        for (int r = 0; r < NN; ++r) s += pinv[(size_t)c * NN + r] * F[r];
        rec[c] = (double)s;
    }
    for (int e = 0; e < kCellExact; ++e) {
        double* x = rec + kCellCoef + 3 * e;
        if (ex[e] < 0) { x[0] = 0.0; x[1] = 0.0; x[2] = 1e3; continue; }
        x[0] = T.m[ex[e]]; x[1] = T.c[ex[e]] * 0.125; x[2] = T.a[ex[e]];
    }
    for (int c = kCellCoef + 3 * kCellExact; c < kCellStride; ++c) rec[c] = 0.0;
    // validation: 8 Halton (2, 3) points of the cell, evaluated in the device's order
    double worst = 0.0;
    for (int q = 1; q <= 8; ++q) {
        double h2 = 0, h3 = 0, f2 = 0.5, f3 = 1.0 / 3;
        for (int n = q; n; n >>= 1, f2 *= 0.5) h2 += f2 * (n & 1);
        for (int n = q; n; n /= 3, f3 /= 3) h3 += f3 * (n % 3);
        const double u = 2 * h2 - 1, v = 2 * h3 - 1, M = cm + u * hm, a = ca + v * ha;
        double f = 0.0;
        int c = 0;
        for (int i = kCellDeg; i >= 0; --i) {
            double qi = rec[c++];
            for (int j = kCellDeg - i - 1; j >= 0; --j) qi = std::fma(qi, v, rec[c++]);
            f = i == kCellDeg ? qi : std::fma(f, u, qi);
        }
        for (int e = 0; e < kCellExact; ++e) {
            const double* x = rec + kCellCoef + 3 * e;
            const double dmx = M - x[0], dax = a - x[2], d2 = std::fma(dmx, dmx, dax * dax);
            if (d2 > 0) f = std::fma(x[1] * d2, 4.0 * std::log(d2), f);
        }
        long double exact = T.p0 + ((long double)M - T.sh0) / T.sc0 * T.p1 + ((long double)a - T.sh1) / T.sc1 * T.p2, mag = 0.0L;
        for (int j = 0; j < T.nt; ++j) {
            const long double dmj = M - T.m[j], daj = a - T.a[j], d2 = dmj * dmj + daj * daj;
            const long double ph = d2 > 0 ? 0.5L * T.c[j] * d2 * logl(d2) : 0.0L;
            exact += ph; mag += fabsl(ph);
        }
        worst = std::max(worst, (double)(fabsl((long double)f - exact) / (mag + fabsl(exact) + 1e-300L)));
        if (scale) *scale = std::max(*scale, (double)(mag + fabsl(exact)));
    }
    return worst;
}

// A piece record in binary32 (kCellStrideF floats, the key's bits at kCellKeyF) and its check:
// evaluated as the binary32 device does (Horner in fmaf, exact terms with the hardware log2) at
// the binary64 check's 8 points, against the binary64 record there; returns |error| / scale
double make_cell_piece_f32(const double* rec, int im, int ia, double dm, double da, double a0, double scale,
                           float* out) {
    for (int c = 0; c < kCellStrideF; ++c) out[c] = 0.0f;
    for (int c = 0; c < kCellKey; ++c) out[c] = (float)rec[c];
    std::memcpy(out + kCellKeyF, rec + kCellKey, 8);
    const double cm = (im + 0.5) * dm, ca = a0 + (ia + 0.5) * da, hm = 0.5 * dm, ha = 0.5 * da;
    double worst = 0.0;
    for (int q = 1; q <= 8; ++q) {
        double h2 = 0, h3 = 0, f2 = 0.5, f3 = 1.0 / 3;
        for (int n = q; n; n >>= 1, f2 *= 0.5) h2 += f2 * (n & 1);
        for (int n = q; n; n /= 3, f3 /= 3) h3 += f3 * (n % 3);
        const float u = (float)(2 * h2 - 1), v = (float)(2 * h3 - 1);
        const float M = (float)(cm + u * hm), a = (float)(ca + v * ha);
        float f = 0.0f;
        int c = 0;
        for (int i = kCellDeg; i >= 0; --i) {
            float qi = out[c++];
            for (int j = kCellDeg - i - 1; j >= 0; --j) qi = std::fma(qi, v, out[c++]);
            f = i == kCellDeg ? qi : std::fma(f, u, qi);
        }
        for (int e = 0; e < kCellExact; ++e) {
            const float* x = out + kCellCoef + 3 * e;
            const float dmx = M - x[0], dax = a - x[2], d2 = std::fma(dmx, dmx, dax * dax);
            f = std::fma(x[1] * d2, std::log2(d2 > 1e-30f ? d2 : 1e-30f) * (4.0f * 0.693147180559945309f), f);
        }
        // the binary64 record at the same point
        const double uu = u, vv = v, MM = M, aa = a;
        double g = 0.0;
        c = 0;
        for (int i = kCellDeg; i >= 0; --i) {
            double qi = rec[c++];
            for (int j = kCellDeg - i - 1; j >= 0; --j) qi = std::fma(qi, vv, rec[c++]);
            g = i == kCellDeg ? qi : std::fma(g, uu, qi);
        }
        for (int e = 0; e < kCellExact; ++e) {
            const double* x = rec + kCellCoef + 3 * e;
            const double dmx = MM - x[0], dax = aa - x[2], d2 = std::fma(dmx, dmx, dax * dax);
            if (d2 > 0) g = std::fma(x[1] * d2, 4.0 * std::log(d2), g);
        }
        worst = std::max(worst, std::fabs((double)f - g) / (scale + 1e-300));
    }
    return worst;
}

// The fine index of one precision's valid pieces (cell_ok, sub_piece) over the grid of cp
void build_fine(const CellPieces& cp, const std::vector<uint8_t>& cell_ok, const std::vector<int>& sub_piece,
                std::vector<uint32_t>& fine) {
    const int S = kGridSub, nm = cp.nm, na = cp.na;
    fine.assign((size_t)nm * S * na * S, 0u);
    parallel_for(nm, [&](int64_t im) {
        for (int ia = 0; ia < na; ++ia) {
            const int64_t c = im * na + ia;
            for (int jm = 0; jm < S; ++jm)
                for (int ja = 0; ja < S; ++ja) {
                    uint32_t e = 0u;
                    if (!cp.refined[c]) {
                        if (cell_ok[c]) e = kFinePiece | (uint32_t)c;
                    } else {
                        const size_t sq = (size_t)cp.ridx[c] * S * S + jm * S + ja;
                        if (sub_piece[sq] >= 0) e = kFinePiece | kFineRefined | (uint32_t)sub_piece[sq];
                        else if (cp.bs_of[sq] >= 0) e = kFineBisect | kFineRefined | (uint32_t)cp.bs_of[sq];
                    }
                    fine[(size_t)(im * S + jm) * ((size_t)na * S) + (size_t)ia * S + ja] = e;
                }
        }
    });
}

const CellPieces& cell_pieces(const pd_aero_table& t, double a0, double a1, int nm, int na) {
    static std::mutex mu;
    static std::map<uint64_t, CellPieces> cache;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; ++i) { h ^= ((const uint8_t*)p)[i]; h *= 1099511628211ull; }
    };
    mix(&t, sizeof(t)); mix(&a0, 8); mix(&a1, 8); mix(&nm, 4); mix(&na, 4);
    const GridKeys& g = grid_keys(t, a0, a1, nm, na);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(h);
    if (it != cache.end()) return it->second;
    const auto t0 = std::chrono::steady_clock::now();
    CellPieces& cp = cache[h];
    const int S = kGridSub;
    const double dm = 10.0 / nm, da = (a1 - a0) / na;
    const int64_t ncell = (int64_t)nm * na, nr = (int64_t)g.refined.size();
    // the pieces: (cell, key) pairs -- exact cells at their index, then each refined cell's keys
    // (its exact sub-cells' and trusted bisector sides'), one piece per distinct key
    std::vector<std::pair<int, uint64_t>> job((size_t)ncell);
    std::vector<uint8_t> refined(ncell, 0);
    for (int r : g.refined) refined[r] = 1;
    for (int64_t c = 0; c < ncell; ++c) job[c] = {(int)c, g.centre[c]};
    cp.sub_piece.assign((size_t)nr * S * S, -1);
    cp.bis_a.assign(g.bis.size(), -1);
    cp.bis_b.assign(g.bis.size(), -1);
    for (int64_t r = 0; r < nr; ++r) {
        std::map<uint64_t, int> own;
        auto piece_of = [&](uint64_t key) {
            auto f = own.find(key);
            if (f != own.end()) return f->second;
            const int p = (int)job.size();
            job.push_back({g.refined[r], key});
            own[key] = p;
            return p;
        };
        const int im = g.refined[r] / na, ia = g.refined[r] % na;
        (void)im; (void)ia;
        for (int q = 0; q < S * S; ++q) {
            const size_t sq = (size_t)r * S * S + q;
            const int jm = q / S, ja = q % S;
            const uint64_t key = g.sub_centre[sq];
            bool exact = true;
            for (int c = 0; c < 4 && exact; ++c)
                exact = g.sub_corner[((size_t)r * (S + 1) + jm + (c >> 1)) * (S + 1) + ja + (c & 1)] == key;
            if (exact) cp.sub_piece[sq] = piece_of(key);
            const int bi = g.sub_bis[sq];
            if (!exact && bi >= 0) {
                if (g.bis[bi].ok_a) cp.bis_a[bi] = piece_of(g.bis[bi].key_a);
                if (g.bis[bi].ok_b) cp.bis_b[bi] = piece_of(g.bis[bi].key_b);
            }
        }
    }
    // the neighbourhoods' terms, solved once per key
    std::map<uint64_t, int> kidx;
    std::vector<uint64_t> keys;
    for (auto& j : job)
        if (kidx.emplace(j.second, (int)keys.size()).second) keys.push_back(j.second);
    std::vector<NbrTerms> terms(keys.size());
    parallel_for((int64_t)keys.size(), [&](int64_t k) { terms[k] = nbr_terms(t, keys[k]); });
    cell_fit_operator();
    cp.rec.assign(job.size() * kCellStride, 0.0);
    cp.err.assign(job.size(), INFINITY);
    cp.scale.assign(job.size(), 0.0);
    cp.cell_of.resize(job.size());
    std::vector<double>& err = cp.err;
    parallel_for((int64_t)job.size(), [&](int64_t p) {
        const int c = job[p].first;
        cp.cell_of[p] = c;
        if (p < ncell && refined[c]) { err[p] = INFINITY; return; }   // (a refined cell's own index: unused)
        double* rec = cp.rec.data() + (size_t)p * kCellStride;
        err[p] = make_cell_piece(terms[kidx.at(job[p].second)], c / na, c % na, dm, da, a0, rec, &cp.scale[p]);
        const uint64_t key = job[p].second;
        std::memcpy(rec + kCellKey, &key, 8);
    });
    auto valid = [&](int p) { return p >= 0 && err[p] <= kCellTol; };
    cp.cell_ok.assign(ncell, 0);
    for (int64_t c = 0; c < ncell; ++c) cp.cell_ok[c] = !refined[c] && valid((int)c);
    for (auto& s : cp.sub_piece) if (!valid(s)) s = -1;
    for (auto& s : cp.bis_a) if (!valid(s)) s = -1;
    for (auto& s : cp.bis_b) if (!valid(s)) s = -1;
    for (size_t p = 0; p < job.size(); ++p) {
        if ((int64_t)p < ncell && refined[job[p].first]) continue;
        ++cp.pieces;
        if (err[p] <= kCellTol) cp.max_rel = std::max(cp.max_rel, err[p]);
        else ++cp.rejected;
    }
    // the fine index: per sub-cell of every cell the piece all its points use, or the bisector
    // record splitting it (numbered as build_grid numbers them: refined cells, then sub-cells in
    // order, every non-exact sub-cell with a bisector)
    cp.nm = nm; cp.na = na; cp.a0 = a0; cp.dm = dm; cp.da = da;
    cp.refined = refined;
    cp.ridx.assign(ncell, -1);
    for (int64_t r = 0; r < nr; ++r) cp.ridx[g.refined[r]] = (int)r;
    cp.bs_of.assign((size_t)nr * S * S, -1);
    {
        int64_t nbs = 0;
        for (int64_t r = 0; r < nr; ++r)
            for (int q = 0; q < S * S; ++q) {
                const size_t sq = (size_t)r * S * S + q;
                const int jm = q / S, ja = q % S;
                bool exact = true;
                for (int c = 0; c < 4 && exact; ++c)
                    exact = g.sub_corner[((size_t)r * (S + 1) + jm + (c >> 1)) * (S + 1) + ja + (c & 1)] == g.sub_centre[sq];
                if (!exact && g.sub_bis[sq] >= 0 && nbs < (int64_t)kGridBisect) cp.bs_of[sq] = nbs++;
            }
    }
    build_fine(cp, cp.cell_ok, cp.sub_piece, cp.fine);
    cp.build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return cp;
}
bool cell_ok(const CellPieces* cp, int64_t cell, bool f32) {
    return cp != nullptr && (f32 ? cp->cell_ok32[cell] : cp->cell_ok[cell]);
}
bool fine_is(const CellPieces* cp, int im, int ia, int jm, int ja, int na, uint32_t want, bool f32) {
    const int S = kGridSub;
    return (f32 ? cp->fine32 : cp->fine)[(size_t)(im * S + jm) * ((size_t)na * S) + (size_t)ia * S + ja] == want;
}
int cell_bis(const CellPieces* cp, int bi, bool side_b, bool f32) {
    if (cp == nullptr) return -1;
    if (f32) return side_b ? cp->bis_b32[bi] : cp->bis_a32[bi];
    return side_b ? cp->bis_b[bi] : cp->bis_a[bi];
}

// The binary32 variant of cp (once per process and table): every binary64-valid piece rounded to
// floats and checked in binary32 (make_cell_piece_f32); the pieces within kCellTol32 keep their
// places, the others drop out of the binary32 validity, sub-cell, bisector and fine-index tables
// (their queries take the record path: verified, payload sums)
void ensure_f32(CellPieces& cp) {
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (cp.have32) return;
    const int64_t np = (int64_t)cp.err.size();
    cp.rec32.assign((size_t)np * kCellStrideF, 0.0f);
    std::vector<double> e32(np, INFINITY);
    parallel_for(np, [&](int64_t p) {
        if (!(cp.err[p] <= kCellTol)) return;
        const int c = cp.cell_of[p];
        e32[p] = make_cell_piece_f32(cp.rec.data() + (size_t)p * kCellStride, c / cp.na, c % cp.na, cp.dm, cp.da,
                                     cp.a0, cp.scale[p], cp.rec32.data() + (size_t)p * kCellStrideF);
    });
    auto ok = [&](int p) { return p >= 0 && e32[p] <= kCellTol32; };
    const int64_t ncell = (int64_t)cp.cell_ok.size();
    cp.cell_ok32.assign(ncell, 0);
    for (int64_t c = 0; c < ncell; ++c) cp.cell_ok32[c] = cp.cell_ok[c] && ok((int)c);
    cp.sub_piece32 = cp.sub_piece; cp.bis_a32 = cp.bis_a; cp.bis_b32 = cp.bis_b;
    for (auto* v : {&cp.sub_piece32, &cp.bis_a32, &cp.bis_b32})
        for (auto& x : *v) if (!ok(x)) x = -1;
    for (int64_t p = 0; p < np; ++p) {
        if (!(cp.err[p] <= kCellTol)) continue;
        if (e32[p] <= kCellTol32) cp.max_rel32 = std::max(cp.max_rel32, e32[p]);
        else ++cp.rejected32;
    }
    build_fine(cp, cp.cell_ok32, cp.sub_piece32, cp.fine32);
    cp.have32 = true;
}

// The device copy of a table's cell pieces: one per device and process, shared read-only by the
// handles (never freed; ~0.2 GB of the 288 GB)
template <typename R>
pd_status cell_pieces_device(const CellPieces& cp, const R** rec, const int** sub, const uint32_t** fine) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, std::array<void*, 3>> m;
    const bool f32 = sizeof(R) == 4;
    const auto& rv = f32 ? (const void*)cp.rec32.data() : (const void*)cp.rec.data();
    const size_t rbytes = f32 ? cp.rec32.size() * 4 : cp.rec.size() * 8;
    const std::vector<int>& sp = f32 ? cp.sub_piece32 : cp.sub_piece;
    const std::vector<uint32_t>& fn = f32 ? cp.fine32 : cp.fine;
    int dev = 0;
    PD_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(mu);
    auto k = std::make_pair((const void*)(f32 ? (const void*)&cp.rec32 : (const void*)&cp.rec), dev);
    auto it = m.find(k);
    if (it == m.end()) {
        std::array<void*, 3> d{};
        const void* src[3] = {rv, sp.data(), fn.data()};
        const size_t nb[3] = {rbytes, sp.size() * 4, fn.size() * 4};
        for (int q = 0; q < 3; ++q) {
            PD_HIP(hipMalloc(&d[q], std::max<size_t>(nb[q], 8)));
            if (nb[q]) PD_HIP(hipMemcpy(d[q], src[q], nb[q], hipMemcpyHostToDevice));
        }
        it = m.emplace(k, d).first;
    }
    *rec = (const R*)it->second[0];
    *sub = (const int*)it->second[1];
    *fine = (const uint32_t*)it->second[2];
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
    int count_work = 0; // workload counters on (pd_count_work)
    float* sac_heads = nullptr;   // pd_step_sac_fused's two-launch path: the actor heads [N][2A]
    float* pol_w4 = nullptr;      // policy rollouts: the actor parameters in chunks of four ([P/4][N][4])
    float* pol_wc = nullptr;      // policy rollouts' list launches: the live envs' actor parameters
    pd_tuning tune{128, 64, 2, -1, 0.0, -1, 0, -1, 0};   // launch tuning (pd_set_tuning)
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
    a.P = (uint64_t)e->dparams;
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
    a.count_work = e->count_work;
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
    for (int b = 0; b < 64; ++b) {   // grid_fin_ca search buckets (handle-precision abscissae)
        const double w = 10.0 / 64, lo = b * w - 1e-4, hi = (b + 1) * w + 1e-4;
        int nlo = 0, nhi = 0;
        for (int k = 0; k < p->ca_n; ++k) { nlo += (double)D.ca_x[k] < lo; nhi += (double)D.ca_x[k] < hi; }
        D.ca_lb[b] = (uint16_t)(nlo | (nhi << 8));
    }
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
    log_table_fill(D.logtab_d);
    D.y0_rl = (R)p->state0[1]; D.m0_rl = (R)p->state0[8];
    // the divisors' correctly rounded reciprocals (div_known): one IEEE division each, in R
    D.inv_m_prop0 = R(1) / D.m_prop0; D.inv_y0_rl = R(1) / D.y0_rl; D.inv_m0_rl = R(1) / D.m0_rl;
    D.inv_norm_y = R(1) / D.norm_y; D.inv_norm_vy = R(1) / D.norm_vy; D.inv_norm_x = R(1) / D.norm_x;
    D.inv_norm_vx = R(1) / D.norm_vx;
    {
        const R b[7] = {D.m_prop0, D.y0_rl, D.m0_rl, D.norm_y, D.norm_vy, D.norm_x, D.norm_vx};
        const R rb[7] = {D.inv_m_prop0, D.inv_y0_rl, D.inv_m0_rl, D.inv_norm_y, D.inv_norm_vy, D.inv_norm_x, D.inv_norm_vx};
        D.div2 = 0;
        for (int k = 0; k < 7; ++k) if (!one_step_ok<R>(b[k], rb[k])) D.div2 |= 1u << k;
    }
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
    if (c->integrator != PD_INTEG_REFERENCE && c->integrator != PD_INTEG_RK4) return fail(PD_ERR_INVALID, "bad integrator");
    if (c->table_flags & ~(PD_TABLES_NO_CELL_PIECES | PD_TABLES_NO_FINE_INDEX | PD_TABLES_EXACT_ATMOSPHERE | PD_TABLES_VERBOSE))
        return fail(PD_ERR_INVALID, "unknown table_flags bits");
    if (c->integrator == PD_INTEG_RK4 && (c->phase != PD_PHASE_PURE_THROTTLE || c->enable_wind))
        return fail(PD_ERR_UNSUPPORTED, "the RK4 integrator (non-parity, BASELINE c2) exists for "
                                        "landing_burn_pure_throttle without wind only");
    // the neighbourhood payloads carry each pair slot's column AoA as a byte (pd_common.h)
    for (const pd_aero_table* t : {&p->cd, &p->cl})
        for (int k = 0; k < t->n_cols; ++k)
            if (!(t->col_aoa[k] >= 0.0 && t->col_aoa[k] <= 255.0 && t->col_aoa[k] == (double)(int)t->col_aoa[k]))
                return fail(PD_ERR_INVALID, "aero table column AoAs must be integers in [0, 255]");
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
    // Taylor pieces of the lines (evaluated instead of the payload sums by the LPE-2 kernels)
    std::vector<R> tay;
    TayStats tst;
    for (int li = 0; li < 4; ++li) build_taylor<R>(li < 2 ? p->cd : p->cl, li, D, tay, tst);
    const bool verbose = (c->table_flags & PD_TABLES_VERBOSE) != 0;
    if (verbose)
        fprintf(stderr, "pdenv taylor: %lld pieces, max abs err %.3g, max rel err %.3g, lines %d %d %d %d\n",
                (long long)tst.pieces, tst.max_abs, tst.max_rel, D.tay_off[0], D.tay_off[1], D.tay_off[2], D.tay_off[3]);
    {
        void* dt;
        if ((st = dalloc(e, &dt, std::max<size_t>(tay.size(), 1) * sizeof(R)))) return st;
        if (!tay.empty()) PD_HIP(hipMemcpy(dt, tay.data(), tay.size() * sizeof(R), hipMemcpyHostToDevice));
        D.tay = (const R*)dt;
    }
    // the atmosphere as piecewise polynomials (PD_TABLES_EXACT_ATMOSPHERE: the exact formulas on the device)
    if (!(c->table_flags & PD_TABLES_EXACT_ATMOSPHERE)) {
        std::vector<R> atm;
        int n_atm = 0;
        double err_atm = 0;
        build_atm_table<R>(p, atm, n_atm, err_atm);
        if (verbose) fprintf(stderr, "pdenv atmosphere table: %d cells, max rel err %.3g\n", n_atm, err_atm);
        // (else: the exact formulas; binary32: its y rounds by 8 mm at 80 km, 1e-6 of p)
        if (err_atm <= (sizeof(R) == 8 ? 1e-14 : 4e-6)) {
            void* da;
            if ((st = dalloc(e, &da, atm.size() * sizeof(R)))) return st;
            PD_HIP(hipMemcpy(da, atm.data(), atm.size() * sizeof(R), hipMemcpyHostToDevice));
            D.atm_tab = (const R*)da; D.atm_n = n_atm; D.atm_inv_w = (R)(1.0 / kAtmW);
        }
    }
    // interior candidate grids: C_D abscissa in [-radians(10), radians(10)], C_L in [0, 10]
    std::vector<unsigned long long> gk[2], sk[2];
    std::vector<int> gs[2], ss[2];
    std::vector<GridBisect> bs[2];
    int gnm[2], gna[2];
    double ga0[2], ga1[2];
    for (int tb = 0; tb < 2; ++tb) grid_geometry(tb, gnm[tb], gna[tb], ga0[tb], ga1[tb]);
    // cell pieces for the interior queries (PD_TABLES_NO_CELL_PIECES: payload sums only): binary64
    // records for binary64 handles, their binary32 roundings (each checked in binary32,
    // ensure_f32) for binary32 handles
    const CellPieces* cps[2] = {nullptr, nullptr};
    if (!(c->table_flags & PD_TABLES_NO_CELL_PIECES)) {
        CellPieces* c0 = const_cast<CellPieces*>(&cell_pieces(p->cd, ga0[0], ga1[0], gnm[0], gna[0]));
        CellPieces* c1 = const_cast<CellPieces*>(&cell_pieces(p->cl, ga0[1], ga1[1], gnm[1], gna[1]));
        if (sizeof(R) == 4) { ensure_f32(*c0); ensure_f32(*c1); }
        cps[0] = c0; cps[1] = c1;
    }
    if ((st = build_grid<R>(p->cd, ga0[0], ga1[0], gnm[0], gna[0], tcd, gk[0], gs[0], sk[0], ss[0], bs[0], cps[0])) != PD_OK) return st;
    if ((st = build_grid<R>(p->cl, ga0[1], ga1[1], gnm[1], gna[1], tcl, gk[1], gs[1], sk[1], ss[1], bs[1], cps[1])) != PD_OK) return st;
    // the fine index (PD_TABLES_NO_FINE_INDEX: cell and sub-cell records only)
    for (int tb = 0; tb < 2; ++tb) {
        D.cell_pc[tb] = nullptr; D.sub_piece[tb] = nullptr; D.fine[tb] = nullptr;
        if (cps[tb] && (st = cell_pieces_device<R>(*cps[tb], &D.cell_pc[tb], &D.sub_piece[tb], &D.fine[tb])) != PD_OK) return st;
        if (c->table_flags & PD_TABLES_NO_FINE_INDEX) D.fine[tb] = nullptr;
    }
    if (verbose)
        for (int tb = 0; tb < 2; ++tb) {
            int64_t nref = 0, nne = 0, nce = 0;
            for (int v : gs[tb]) { nref += v >= 0 && (v & kGridRefine); nce += v >= 0 && !(v & kGridRefine) && !(v & kGridExact); }
            int64_t nbs = 0, nbs2 = 0;
            for (int v : ss[tb]) nne += v < 0 || !(v & kGridExact);
            for (auto& b : bs[tb]) { nbs += 1; nbs2 += (b.slot_a >= 0 && (b.slot_a & kGridExact)) + (b.slot_b >= 0 && (b.slot_b & kGridExact)); }
            fprintf(stderr, "pdenv grid %d: %lld bisector sub-cells, %lld trusted sides\n", tb, (long long)nbs, (long long)nbs2);
            if (cps[tb]) fprintf(stderr, "pdenv grid %d: %lld cell pieces (%.1f MB), %lld rejected, max error %.2e of sum |c phi|, built in %.2f s\n", tb,
                                 (long long)cps[tb]->pieces, cps[tb]->rec.size() * 8e-6, (long long)cps[tb]->rejected, cps[tb]->max_rel, cps[tb]->build_s);
            fprintf(stderr, "pdenv grid %d: %d x %d cells, %lld refined, %lld non-exact cells, %lld of %zu sub-cells non-exact\n", tb,
                    gnm[tb], gna[tb], (long long)nref, (long long)nce, (long long)nne, ss[tb].size());
        }
    for (int tb = 0; tb < 2; ++tb) {
        void *dk, *ds, *dsk, *dss;
        const size_t nsub = std::max<size_t>(sk[tb].size(), 1);
        if ((st = dalloc(e, &dk, gk[tb].size() * 8)) || (st = dalloc(e, &ds, gs[tb].size() * 4)) ||
            (st = dalloc(e, &dsk, nsub * 8)) || (st = dalloc(e, &dss, nsub * 4)))
            return st;
        PD_HIP(hipMemcpy(dk, gk[tb].data(), gk[tb].size() * 8, hipMemcpyHostToDevice));
        PD_HIP(hipMemcpy(ds, gs[tb].data(), gs[tb].size() * 4, hipMemcpyHostToDevice));
        if (!sk[tb].empty()) {
            PD_HIP(hipMemcpy(dsk, sk[tb].data(), sk[tb].size() * 8, hipMemcpyHostToDevice));
            PD_HIP(hipMemcpy(dss, ss[tb].data(), ss[tb].size() * 4, hipMemcpyHostToDevice));
        }
        D.sub_key[tb] = (const unsigned long long*)dsk; D.sub_slot[tb] = (const int*)dss;
        void* dbs;
        if ((st = dalloc(e, &dbs, std::max<size_t>(bs[tb].size(), 1) * sizeof(GridBisect)))) return st;
        if (!bs[tb].empty()) PD_HIP(hipMemcpy(dbs, bs[tb].data(), bs[tb].size() * sizeof(GridBisect), hipMemcpyHostToDevice));
        D.sub_bis[tb] = dbs;
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
    {
        // the step kernels' LDS tables as one image (pd_step.h StepStatic), copied by their prologue
        void* img;
        const size_t nb = c->enable_wind ? sizeof(StepStatic<R, true>) : sizeof(StepStatic<R, false>);
        if ((st = dalloc(e, &img, nb))) return st;
        std::vector<uint8_t> h(nb);
        if (c->enable_wind) fill_step_static<R, true>(D, *(StepStatic<R, true>*)h.data());
        else fill_step_static<R, false>(D, *(StepStatic<R, false>*)h.data());
        PD_HIP(hipMemcpy(img, h.data(), nb, hipMemcpyHostToDevice));
        D.stage_img = img;
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
        (st = dalloc(e, (void**)&e->pend.pay, (size_t)kPendingCap * kPay * 8)) ||
        (st = dalloc(e, (void**)&e->pend.stats, kStats * 8)) ||
        (st = dalloc(e, (void**)&e->pend.solve_ws, (size_t)kSolveSlots * kScratch * 8)) ||
        (st = dalloc(e, (void**)&e->pend.solve_lock, (size_t)kSolveSlots * 4)) ||
        (st = dalloc(e, (void**)&e->pend.ticket, 4)))
        return st;
    PD_HIP(hipMemset(e->pend.count, 0, 8));
    PD_HIP(hipMemset(e->pend.ticket, 0, 4));
    PD_HIP(hipMemset(e->pend.solve_lock, 0, (size_t)kSolveSlots * 4));
    unsigned long long stats0[kStats] = {0, 0, (unsigned long long)tcd.entries, (unsigned long long)tcl.entries};
    PD_HIP(hipMemcpy(e->pend.stats, stats0, sizeof(stats0), hipMemcpyHostToDevice));
    // the policy rollouts' pinned live-count words and events, made here: a first pinned
    // allocation inside a timed rollout cost ~170 ms (the PSO driver's share handle)
    PD_HIP(hipHostMalloc((void**)&e->host_cnt, 2 * sizeof(uint32_t), hipHostMallocDefault));
    for (hipEvent_t& ev : e->cnt_ev) PD_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    StepArgs<R> a = make_args<R>(e);
    unsigned grid = (unsigned)((N + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_reset<R>, dim3(grid), dim3(kBlock), 0, 0, a, (const uint8_t*)nullptr);
    PD_HIP(hipGetLastError());
    PD_HIP(hipDeviceSynchronize());
    return PD_OK;
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
    if (e->cfg.integrator == PD_INTEG_RK4) {   // pure throttle, no wind (validated); LPE 2 or 16
        if (pso) { if (l <= 2) launch_step<R, 0, 1, false, 2, true>(a, s); else launch_step<R, 0, 1, false, 16, true>(a, s); }
        else { if (l <= 2) launch_step<R, 0, 0, false, 2, true>(a, s); else launch_step<R, 0, 0, false, 16, true>(a, s); }
        return;
    }
    if (ph == 0 && !pso) { if (w) launch_lpe<R, 0, 0, true>(l, a, s); else launch_lpe<R, 0, 0, false>(l, a, s); }
    else if (ph == 0) { if (w) launch_lpe<R, 0, 1, true>(l, a, s); else launch_lpe<R, 0, 1, false>(l, a, s); }
    else if (ph == 1 && pso) { if (w) launch_lpe<R, 1, 1, true>(l, a, s); else launch_lpe<R, 1, 1, false>(l, a, s); }
    else if (ph == 1) { if (w) launch_lpe<R, 1, 0, true>(l, a, s); else launch_lpe<R, 1, 0, false>(l, a, s); }
    else { if (w) launch_lpe<R, 2, 0, true>(l, a, s); else launch_lpe<R, 2, 0, false>(l, a, s); }
}

// Policy rollouts run at 2 lanes per env whatever the handle's step LPE: the per-lane actor and
// the LPE 2 table path (Taylor lines, cell pieces) fit 256 VGPRs without scratch.
// pd_tuning.policy_lanes 4/8 (the c4 lanes-per-env sweep) runs the LPE 4/8 instantiations, whose
// tables take the split payload sums.
template <typename R, int PH, bool W> void launch_policy(int lpe, const StepArgs<R>& a, int64_t n_launch, hipStream_t s) {
    switch (lpe) {
        case 4: launch_policy_lpe<R, PH, W, 4>(a, n_launch, s); break;
        case 8: launch_policy_lpe<R, PH, W, 8>(a, n_launch, s); break;
        default: launch_policy_lpe<R, PH, W, 2>(a, n_launch, s); break;
    }
}

template <typename R> void launch_insert(pd_env* e, hipStream_t s) {
    hipLaunchKernelGGL(k_insert<R>, dim3(1), dim3(64), 0, s, e->pend, e->keys_cd, (R*)e->pay_cd, e->logcap_cd,
                       e->keys_cl, (R*)e->pay_cl, e->logcap_cl);
}

// pd_step_sac's inputs and float32 outputs (see include/pdenv.h)
struct SacIO {
    const float *mean, *log_std, *eps;
    float lo, hi, max_action;
    float *action, *slab, *obs32;
    uint32_t head_stride;
    // pd_step_sac_ring
    int draw = 0;
    float* eps_out = nullptr;
    int64_t ring_cap = 0;
    long long* ring_state = nullptr;
    float* prio = nullptr;
    const float* max_prio = nullptr;
    // pd_step_sac_fused: the actor in the kernel prologue (mlp.H = 0: off)
    SacMlp mlp{};
    float* heads_out = nullptr;
};

template <typename R>
pd_status step_impl(pd_env* e, const void* actions, void* obs, void* reward, uint8_t* done, uint8_t* trunc,
                    int8_t* tid, const double* noise, void* info, void* reward_sum, hipStream_t s,
                    int n_fused = 1, const SacIO* sac = nullptr, uint64_t info_mask = (1ull << PD_N_INFO) - 1ull) {
    // every caller's launch needs its inputs: actions (plain steps), the heads or the actor (SAC);
    // the public entry points check them too, this keeps an internal caller from launching a
    // kernel that would read through a null pointer
    if (!sac && !actions) return fail(PD_ERR_INVALID, "step launch without actions");
    if (sac && sac->mlp.H == 0 && !sac->mean) return fail(PD_ERR_INVALID, "SAC step launch without heads or actor");
    if (sac && sac->mlp.H != 0 && (!sac->mlp.obs || !sac->mlp.wm || !sac->mlp.ws))
        return fail(PD_ERR_INVALID, "SAC step launch with an incomplete actor");
    if (sac && (e->cfg.rtd == PD_RTD_PSO || e->cfg.integrator != PD_INTEG_REFERENCE ||
                (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN)))
        return fail(PD_ERR_UNSUPPORTED, "SAC step launch on a handle without a SAC kernel");
    StepArgs<R> a = make_args<R>(e);
    a.actions = actions; a.obs = (R*)obs; a.reward = (R*)reward; a.done = done; a.trunc = trunc; a.trunc_id = tid;
    a.noise = noise; a.info = (R*)info; a.reward_sum = (R*)reward_sum;
    a.info_mask = info_mask; a.info_nsel = __builtin_popcountll(info_mask);
    a.n_fused = n_fused;
    if (sac) {
        a.sac_mean = sac->mean; a.sac_logstd = sac->log_std; a.sac_eps = sac->eps;
        a.sac_lo = sac->lo; a.sac_hi = sac->hi; a.sac_max = sac->max_action;
        a.sac_act = sac->action; a.slab = sac->slab; a.obs32 = sac->obs32;
        a.sac_hs = sac->head_stride;
        a.sac_draw = sac->draw; a.sac_eps_out = sac->eps_out;
        a.ring_cap = sac->ring_cap; a.ring_state = sac->ring_state; a.prio = sac->prio; a.max_prio = sac->max_prio;
        a.sac_mlp = sac->mlp; a.sac_heads_out = sac->heads_out;
    }
    dispatch_step<R>(e, a, s);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

// policy rollouts: the caller's parameter-major weights [P][N] in chunks of four parameters,
// [ceil(P / 4)][N][4] (zeros past P), the layout actor_forward reads with one 16-byte load per
// chunk (pd_step_impl.h)
__global__ __launch_bounds__(kBlock) void k_wchunk(const float* __restrict__ w, float4* __restrict__ out, int P,
                                                   int64_t N) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t C = (P + 3) / 4;
    if (t >= C * N) return;
    const int c = (int)(t / N);
    const int64_t i = t - (int64_t)c * N;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = 4 * c + k < P ? w[(int64_t)(4 * c + k) * N + i] : 0.f;
    out[t] = make_float4(v[0], v[1], v[2], v[3]);
}

// policy rollouts' prologue in one launch: k_reset of every env, its fitness zeroed, every env
// live in index order (the list, count 0 = n and the other two counts zero; refill: the three
// counts zero, the refill launch's hand-out counter among them) -- the four launches a rollout
// used to start with
template <typename R>
__global__ __launch_bounds__(kBlock) void k_policy_init(StepArgs<R> a, R* __restrict__ fitness, int32_t* list,
                                                        uint32_t* cnt, int refill) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < 3) cnt[i] = (i == 0 && !refill) ? (uint32_t)a.n : 0u;
    if (i >= a.n) return;
    list[i] = (int32_t)i;
    fitness[i] = R(0);
    DP<R>& P = *params<R>(a.P);
    const uint32_t ui = (uint32_t)i;
    EnvRegs<R> e;
    reset_values<R>(P, a, a.env_offset + (uint64_t)i, ev(a.b.epi, ui) + 1u,
                    (const double*)(uint64_t)&P.logtab.invc[0], (const double*)(uint64_t)&P.logtab.logc[0], e);
    store_env<R>(a, P, ui, e, true);
}

// policy rollouts' epilogue in one launch: k_insert (thread 0 of block 0) and the episode lengths
// copied to the caller's steps (the tstep words), which used a copy of its own
template <typename R>
__global__ __launch_bounds__(kBlock) void k_policy_finish(Pending pend, unsigned long long* keys_cd, R* pay_cd,
                                                          int lc_cd, unsigned long long* keys_cl, R* pay_cl, int lc_cl,
                                                          const uint32_t* __restrict__ tstep, int32_t* __restrict__ steps,
                                                          int64_t n) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
        insert_pending<R>(pend.count, pend.keys, pend.pay, pend.stats, keys_cd, pay_cd, lc_cd, keys_cl, pay_cl, lc_cl);
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (steps && i < n) steps[i] = (int32_t)tstep[i];
}

template <typename R> void launch_policy_finish(pd_env* e, int32_t* steps, hipStream_t s) {
    const int64_t N = e->cfg.n_envs;
    hipLaunchKernelGGL(k_policy_finish<R>, dim3((unsigned)((N + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, e->pend,
                       e->keys_cd, (R*)e->pay_cd, e->logcap_cd, e->keys_cl, (R*)e->pay_cl, e->logcap_cl,
                       (const uint32_t*)e->tstep, steps, N);
}

template <typename R>
pd_status rollout_policy_impl(pd_env* e, const float* w, int32_t max_steps, void* fitness, int32_t* steps,
                              int32_t check_every, hipStream_t s, bool chunked = false) {
    const int64_t N = e->cfg.n_envs;
    unsigned grid = (unsigned)((N + kBlock - 1) / kBlock);
    // the weights in the chunked layout of the step kernel's actor (one pass over them: 2 x 1.5 KB
    // per particle, against the 1.5 KB per policy step the rollout reads), unless the caller's
    // are chunked already (pd_rollout_policy_chunked: pd_pso_step_chunked writes that layout)
    const int P = e->cfg.phase == PD_PHASE_PURE_THROTTLE ? PD_ACTOR_PARAMS_PURE_THROTTLE : PD_ACTOR_PARAMS_LANDING_BURN;
    if (!chunked) {
        if (!e->pol_w4) {
            PD_HIP(hipMalloc((void**)&e->pol_w4, (size_t)PD_ACTOR_PARAMS_LANDING_BURN * (size_t)N * sizeof(float)));
            e->allocs.push_back(e->pol_w4);
        }
        const int64_t tot = (int64_t)((P + 3) / 4) * N;
        hipLaunchKernelGGL(k_wchunk, dim3((unsigned)((tot + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w,
                           (float4*)e->pol_w4, P, N);
    }
    StepArgs<R> a = make_args<R>(e);
    a.policy_w = chunked ? w : e->pol_w4; a.reward_sum = (R*)fitness; a.auto_reset = 0;
    const bool wind = e->cfg.enable_wind != 0;
    // launch t steps live[t & 1][0, live_cnt[t % 3]) and appends the survivors to the other list;
    // the grid covers the live count last read back (a workgroup past the device count leaves
    // at once), so the launches shrink with the swarm's live envs.  Checks are one interval
    // behind: at a check the count is copied to pinned memory under an event, and the host
    // waits for the PREVIOUS check's event, with check_every launches still queued behind it
    // (no bubble); at most 2 * check_every nearly empty launches run after the last episode.
    if (check_every > 0 && !e->host_cnt) return fail(PD_ERR_HIP, "policy rollout: no pinned live-count words");
    // The list pays off once the grid no longer fits the chip in one round (a launch then costs
    // the rounds its waves need); below that the launch time is one wave's, and reading the
    // state and actor weights through the list (gathers) only costs.  pd_tuning.policy_list forces.
    int dev_cus = 256;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, e->device);
    const int plpe = e->tune.policy_lanes;
    // refill: one launch of the chip's resident env slots (two waves per SIMD) steps the whole
    // swarm, the lanes of an ended episode taking the next particle -- the grid's lanes stay busy
    // until the swarm's last particles, where a launch per live-list check leaves most of a
    // workgroup's lanes idle behind its longest episode
    const int64_t cap = (int64_t)dev_cus * 512 / plpe;
    // (auto: a wave's slots are handed particles once three quarters of them wait -- 24 of the 32
    // at two lanes per env: c4 at 262 144 particles 4.71 ms a rollout, against 12.4 / 8.6 / 6.5 /
    // 5.5 / 5.0 / 5.0 ms at batches of 1 / 4 / 8 / 12 / 16 / 32 and 5.94 ms without refill)
    const int kRefillBatch = 48 / plpe;
    // (windless handles only: the windy policy kernels compile no refill, see pd_step_impl.h)
    // (and a swarm of at least one wave's slots: the slots are whole waves, none past the swarm).
    // Auto: every windless swarm -- beyond the resident slots for the refills, and within them for
    // the one launch without live-count reads (c4 at 32 768 particles: 1.452 ms a generation
    // against 1.476 with the per-check launches, profiles/r05_c4_refill.jsonl)
    // (auto refill yields to an explicit request for the per-check launches: policy_list >= 0 or
    // policy_list_at > 0 with policy_refill -1; check_every and the list apply to those only)
    const bool refill_on = e->tune.policy_refill > 0 ||
                           (e->tune.policy_refill < 0 && e->tune.policy_list < 0 && !(e->tune.policy_list_at > 0.0));
    const bool refill = !wind && N >= 64 / plpe && refill_on;
    // every env reset, fitness zeroed, the live list and counts initialised: one launch
    hipLaunchKernelGGL(k_policy_init<R>, dim3(grid), dim3(kBlock), 0, s, make_args<R>(e), (R*)fitness, e->live[0],
                       e->live_cnt, refill ? 1 : 0);
    if (refill) {
        // slots: whole waves (epw envs each), at most the swarm; wave w owns particles
        // [w Q, (w + 1) Q) -- its first epw are its slots' first episodes -- and takes them
        // without atomics; the rest, from waves x Q on, is the shared pool (batched hand-outs).
        // Q: policy_refill_own percent of the swarm over the waves, whole waves' worth of envs
        // (default 100: c4 at 262 144 particles, 128 per wave, no pool -- 3.97 ms a rollout against
        // 4.22 / 4.18 / 4.54 / 4.75 ms with 90 / 75 / 50 / 0 % own, the rest from the pool in
        // batches of 24: the pool's batching idles more lanes than the waves' uneven work does)
        const int64_t epw = 64 / plpe;
        int64_t slots = std::min<int64_t>(N, e->tune.policy_slots > 0 ? e->tune.policy_slots : cap);
        slots = std::max<int64_t>(epw, slots / epw * epw);   // (<= N: N >= epw)
        const int64_t waves = slots / epw;
        const int own = e->tune.policy_refill_own >= 0 ? e->tune.policy_refill_own : 100;
        int64_t q = (int64_t)((double)N * own / 100.0 / (double)waves) / epw * epw;
        q = std::max<int64_t>(epw, std::min<int64_t>(q, N / waves / epw * epw));   // (waves q <= N: N >= slots)
        a.use_list = 0; a.policy_wc = nullptr;
        a.refill = e->tune.policy_refill > 0 ? e->tune.policy_refill : kRefillBatch;
        a.refill_next = e->live_cnt; a.refill_max = max_steps;
        a.refill_slots = (int)slots; a.refill_q = (int)q; a.refill_base = (int)(waves * q);
        a.list_in = e->live[0]; a.list_out = e->live[1];
        a.cnt_in = e->live_cnt + 1; a.cnt_out = e->live_cnt + 1; a.cnt_zero = e->live_cnt + 2;
        // (a bound every wave reaches: a wave runs at most its own q particles and the pool's,
        // one of its slots live at every step until they are all handed out, each episode at most
        // max_steps steps; the waves leave when their lanes have none left)
        const int64_t bound = (int64_t)max_steps * (q + (N - waves * q) + 1);
        a.n_fused = (int)std::min<int64_t>(bound, INT32_MAX);
        if (e->cfg.phase == PD_PHASE_PURE_THROTTLE) { if (wind) launch_policy<R, 0, true>(plpe, a, slots, s); else launch_policy<R, 0, false>(plpe, a, slots, s); }
        else { if (wind) launch_policy<R, 1, true>(plpe, a, slots, s); else launch_policy<R, 1, false>(plpe, a, slots, s); }
        PD_HIP(hipGetLastError());
        launch_policy_finish<R>(e, steps, s);
        PD_HIP(hipGetLastError());
        return PD_OK;
    }
    a.use_list = e->tune.policy_list >= 0 ? e->tune.policy_list : (N * plpe > (int64_t)dev_cus * 512);
    // every launch appends its survivors to the next list, so the rollout can switch to the list
    // at any launch: once the live count read back falls to policy_list_at x N (default off), the
    // waves of the later launches hold live envs only
    const double compact_at = e->tune.policy_list_at;
    // the list launches' parameter copy (policy_wc, chunked as pol_w4): made at the first rollout
    if (!e->pol_wc) {
        PD_HIP(hipMalloc((void**)&e->pol_wc, (size_t)PD_ACTOR_PARAMS_LANDING_BURN * (size_t)N * sizeof(float)));
        e->allocs.push_back(e->pol_wc);
    }
    a.policy_wc = e->pol_wc;
    int64_t n_launch = N;
    int checks = 0;
    // F policy steps per launch (an episode that ends inside a launch is stored at its last step
    // and its lanes freeze); the live list is compacted once per launch
    const int F = e->tune.policy_fuse;
    const int check_launches = check_every > 0 ? std::max(1, check_every / F) : 0;
    int32_t t = 0;
    for (int l = 0; t < max_steps; ++l) {
        a.n_fused = std::min<int32_t>(F, max_steps - t);
        t += a.n_fused;
        a.list_in = e->live[l & 1]; a.list_out = e->live[(l + 1) & 1];
        a.cnt_in = e->live_cnt + l % 3; a.cnt_out = e->live_cnt + (l + 1) % 3; a.cnt_zero = e->live_cnt + (l + 2) % 3;
        if (e->cfg.phase == PD_PHASE_PURE_THROTTLE) { if (wind) launch_policy<R, 0, true>(plpe, a, n_launch, s); else launch_policy<R, 0, false>(plpe, a, n_launch, s); }
        else { if (wind) launch_policy<R, 1, true>(plpe, a, n_launch, s); else launch_policy<R, 1, false>(plpe, a, n_launch, s); }
        PD_HIP(hipGetLastError());
        if (F >= 16 || (l & (16 / F - 1)) == 16 / F - 1) launch_insert<R>(e, s);
        if (check_launches > 0 && (l + 1) % check_launches == 0 && t < max_steps) {
            const int k = checks & 1;
            PD_HIP(hipMemcpyAsync(e->host_cnt + k, e->live_cnt + (l + 1) % 3, 4, hipMemcpyDeviceToHost, s));
            PD_HIP(hipEventRecord(e->cnt_ev[k], s));
            if (checks > 0) {
                PD_HIP(hipEventSynchronize(e->cnt_ev[k ^ 1]));
                const uint32_t live = ((volatile uint32_t*)e->host_cnt)[k ^ 1];
                if (live == 0) break;
                if (!a.use_list && compact_at > 0.0 && (double)live <= compact_at * (double)N) a.use_list = 1;
                if (a.use_list) n_launch = live;
            }
            ++checks;
        }
    }
    launch_policy_finish<R>(e, steps, s);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

// Launch tuning defaults (pd_tuning).  policy_fuse 64: a wave whose episodes have all ended leaves
// its launch, so a longer launch costs no frozen steps at the swarm's tail; it saves launches,
// their table staging and the count checks between them (c4: 8 -> 1.66, 16 -> 1.57, 32 ->
// 1.53-1.57, 64 -> 1.49-1.50 ms per generation, profiles/r04_exp_s16_pol_exit.jsonl,
// r04_exp_s17_pfuse.jsonl).  step_fuse 128: the miss flush runs between launches, so a
// neighbourhood solved on device is re-solved at most this many steps before it is in the tables
// (c3 ms per env-step, payload sums: 16 -> 0.0450, 32 -> 0.0442, 64 -> 0.0421; cell pieces: 64 ->
// 0.0341, 128 -> 0.0335, 256 -> 0.0337).

// n_steps env-steps in launches of pd_tuning.step_fuse fused steps (each inserts its own misses).
// Row t of every [n_steps][N...] array belongs to step t; NULL outputs are not written.
pd_status step_n_impl(pd_env* e, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                      uint8_t* trunc, int8_t* tid, void* reward_sum, hipStream_t s, void* info = nullptr,
                      uint64_t info_mask = 0) {
    const size_t N = (size_t)e->cfg.n_envs;
    const size_t sa = N * e->act_dim * (e->cfg.action_f64 ? 8 : 4), so = N * e->obs_dim * e->rsize;
    const size_t sr = N * e->rsize;
    const size_t si = N * e->rsize * (size_t)__builtin_popcountll(info_mask);   // one step's info rows
    const int K = e->tune.step_fuse;
    for (int32_t t = 0; t < n_steps; t += K) {
        const int k = n_steps - t < K ? n_steps - t : K;
        auto at = [&](void* p, size_t stride) { return p ? (void*)((char*)p + stride * t) : nullptr; };
        const void* act = (const char*)actions + sa * t;
        pd_status st = e->rsize == 8
            ? step_impl<double>(e, act, at(obs, so), at(reward, sr), (uint8_t*)at(done, N), (uint8_t*)at(trunc, N),
                                (int8_t*)at(tid, N), nullptr, at(info, si), reward_sum, s, k, nullptr, info_mask)
            : step_impl<float>(e, act, at(obs, so), at(reward, sr), (uint8_t*)at(done, N), (uint8_t*)at(trunc, N),
                               (int8_t*)at(tid, N), nullptr, at(info, si), reward_sum, s, k, nullptr, info_mask);
        if (st != PD_OK) return st;
        // (no miss flush between the launches: each step launch's last workgroup inserts the
        // neighbourhoods its launch solved, k_step's tail)
    }
    return PD_OK;
}

}  // namespace

// ================================================================ C ABI
extern "C" {

int pd_abi_version(void) { return PD_ABI_VERSION; }

extern "C++" {
namespace {
// the device's table evaluation (atmosphere<R, true>, pd_physics.h) on the host, in R
template <typename R>
void eval_atm_table(const pd_params* p, const double* alt, int64_t n_alt, double* atm_out, double* max_rel) {
    std::vector<R> atm;
    int n_atm = 0;
    build_atm_table<R>(p, atm, n_atm, *max_rel);
    for (int64_t i = 0; i < n_alt; ++i) {
        R y = (R)alt[i], al = y < R(0) ? R(0) : y, out[3] = {R(0), R(0), R(0)};
        if (al < (R)p->isa_alt_max) {
            int k = (int)(al * (R)(1.0 / kAtmW));
            k = k > n_atm - 1 ? n_atm - 1 : k;
            const R* rec = atm.data() + (size_t)k * kAtmStride;
            if (rec[1] < R(1e29) && (R)p->isa_r * al / ((R)p->isa_r + al) >= rec[1]) rec += kAtmRec;
            const R t = al - rec[0];
            for (int fn = 0; fn < 3; ++fn) out[fn] = horner_host<R>(rec + 2 + fn * (kAtmDeg + 1), kAtmDeg, t);
        }
        atm_out[3 * i] = (double)out[1]; atm_out[3 * i + 1] = (double)out[0]; atm_out[3 * i + 2] = (double)out[2];
    }
}
}  // namespace
}  // extern "C++"

pd_status pd_atm_table(const pd_params* p, int32_t precision, const double* alt, int64_t n_alt, double* atm_out,
                       double* max_rel) {
    if (!p || !max_rel || n_alt < 0 || (n_alt && (!alt || !atm_out))) return fail(PD_ERR_INVALID, "pd_atm_table: bad arguments");
    if (precision == PD_F32) eval_atm_table<float>(p, alt, n_alt, atm_out, max_rel);
    else eval_atm_table<double>(p, alt, n_alt, atm_out, max_rel);
    return PD_OK;
}
pd_status pd_cell_piece_info(const pd_params* p, int32_t table, int64_t piece, double* out, int32_t n_out) {
    if (!p || !out || n_out < 16 || (table != 0 && table != 1)) return fail(PD_ERR_INVALID, "pd_cell_piece_info: bad arguments");
    const pd_aero_table& t = table ? p->cl : p->cd;
    if (t.n_pts < kNbr || t.n_pts > PD_MAX_PTS || t.n_cols != kCols) return fail(PD_ERR_INVALID, "pd_cell_piece_info: bad table");
    int nm, na;
    double a0, a1;
    grid_geometry(table, nm, na, a0, a1);
    CellPieces& cp = const_cast<CellPieces&>(cell_pieces(t, a0, a1, nm, na));
    ensure_f32(cp);
    int64_t ok32 = 0;
    for (uint8_t c : cp.cell_ok32) ok32 += c;
    int64_t ok64 = 0;
    for (uint8_t c : cp.cell_ok) ok64 += c;
    const double v[16] = {(double)cp.pieces, (double)cp.rejected, cp.max_rel, cp.build_s, (double)(cp.rec.size() / kCellStride),
                          (double)nm, (double)na, a0, a1, (double)kCellDeg, (double)kCellExact, (double)kCellStride,
                          (double)cp.rejected32, cp.max_rel32, (double)ok64, (double)ok32};
    for (int k = 0; k < 16; ++k) out[k] = v[k];
    if (piece >= 0) {
        if ((size_t)(piece + 1) * kCellStride > cp.rec.size() || n_out < 16 + kCellStride)
            return fail(PD_ERR_INVALID, "pd_cell_piece_info: piece out of range or out too short");
        std::memcpy(out + 16, cp.rec.data() + (size_t)piece * kCellStride, kCellStride * sizeof(double));
    }
    return PD_OK;
}

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
    // default lanes per env.  Below ~64k envs the step is bound by one wave's latency: splitting
    // each table's sum over LPE / 2 lanes shortens it, while LPE 2 alone has the Taylor lines,
    // cell pieces and fine index.  Measured on the round-3 kernels (f64 ms per
    // env-step, 128 steps per launch, wind / no wind; profiles/r03_exp_lpe_sweep.jsonl):
    //   4 096: LPE 16 0.0221 / 0.0186, 8 0.0242, 2 0.0261 / 0.0237
    //   8 192: LPE 8 0.0249 / 0.0210, 2 0.0260 / 0.0235, 4 0.0277 / 0.0241, 16 0.0274 / 0.0235
    //  16 384: LPE 2 0.0261 / 0.0234, 4 0.0277 / 0.0240, 8 0.0306
    //  32 768: LPE 2 0.0263, 4 0.0352; 65 536: LPE 2
    e->lpe = cfg->lanes_per_env != 0 ? cfg->lanes_per_env
                                     : (cfg->n_envs <= 4096 ? 16 : (cfg->n_envs <= 8192 ? 8 : 2));
    if (e->lpe != 1 && e->lpe != 2 && e->lpe != 4 && e->lpe != 8 && e->lpe != 16) { delete e; return fail(PD_ERR_INVALID, "lanes_per_env must be 0, 1, 2, 4, 8 or 16"); }
    if (cfg->integrator == PD_INTEG_RK4) e->lpe = e->lpe <= 2 ? 2 : 16;   // the RK4 instantiations
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

pd_status pd_set_tuning(pd_env* e, const pd_tuning* t) {
    if (!e || !t) return fail(PD_ERR_INVALID, "pd_set_tuning: null env/tuning");
    const int pf = t->policy_fuse;
    if (t->step_fuse < 1 || t->step_fuse > 256) return fail(PD_ERR_INVALID, "pd_set_tuning: step_fuse must be 1..256");
    if (pf < 1 || pf > 64 || (pf & (pf - 1))) return fail(PD_ERR_INVALID, "pd_set_tuning: policy_fuse must be a power of two 1..64");
    if (t->policy_lanes != 2 && t->policy_lanes != 4 && t->policy_lanes != 8)
        return fail(PD_ERR_INVALID, "pd_set_tuning: policy_lanes must be 2, 4 or 8");
    if (t->policy_list < -1 || t->policy_list > 1) return fail(PD_ERR_INVALID, "pd_set_tuning: policy_list must be -1, 0 or 1");
    if (!(t->policy_list_at >= 0.0 && t->policy_list_at <= 1.0))
        return fail(PD_ERR_INVALID, "pd_set_tuning: policy_list_at must be in [0, 1]");
    if (t->policy_refill < -1 || t->policy_refill > 64)
        return fail(PD_ERR_INVALID, "pd_set_tuning: policy_refill must be -1 (auto), 0 (off) or a batch of 1..64 slots");
    if (t->policy_slots < 0) return fail(PD_ERR_INVALID, "pd_set_tuning: policy_slots must be >= 0");
    if (t->policy_refill_own < -1 || t->policy_refill_own > 100)
        return fail(PD_ERR_INVALID, "pd_set_tuning: policy_refill_own must be -1 (auto) or a percentage 0..100");
    e->tune = *t;
    return PD_OK;
}

pd_status pd_get_tuning(const pd_env* e, pd_tuning* t) {
    if (!e || !t) return fail(PD_ERR_INVALID, "pd_get_tuning: null env/tuning");
    *t = e->tune;
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

pd_status pd_step_sac(pd_env* e, const float* mean, const float* log_std, int32_t head_stride, const float* eps,
                      float log_std_min, float log_std_max, float max_action, float* action, float* slab, float* obs32,
                      void* stream) {
    if (!e || !mean) return fail(PD_ERR_INVALID, "null env/mean");
    if (head_stride != 0 && head_stride < e->act_dim) return fail(PD_ERR_INVALID, "pd_step_sac: head_stride < action dim");
    if (eps && !log_std) return fail(PD_ERR_INVALID, "pd_step_sac: eps given without log_std");
    if (e->cfg.action_f64) return fail(PD_ERR_UNSUPPORTED, "pd_step_sac: float32 actions only (action_f64 = 0)");
    if (e->cfg.rtd == PD_RTD_PSO || e->cfg.integrator != PD_INTEG_REFERENCE ||
        (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN))
        return fail(PD_ERR_UNSUPPORTED, "pd_step_sac: the RL landing burns (reference integrator) only");
    PD_HIP(hipSetDevice(e->device));
    const SacIO io{mean, log_std, eps, log_std_min, log_std_max, max_action, action, slab, obs32,
                   (uint32_t)(head_stride ? head_stride : e->act_dim)};
    if (e->rsize == 8)
        return step_impl<double>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 (hipStream_t)stream, 1, &io);
    return step_impl<float>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                            (hipStream_t)stream, 1, &io);
}

pd_status pd_step_sac_ring(pd_env* e, const float* heads, int32_t deterministic, float log_std_min, float log_std_max,
                           float max_action, float* eps_out, float* action, float* ring, int64_t capacity,
                           long long* ring_state, float* priorities, const float* max_priority, float* obs32,
                           void* stream) {
    if (!e || !heads) return fail(PD_ERR_INVALID, "null env/heads");
    if (e->cfg.action_f64) return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_ring: float32 actions only (action_f64 = 0)");
    if (e->cfg.rtd == PD_RTD_PSO || e->cfg.integrator != PD_INTEG_REFERENCE ||
        (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN))
        return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_ring: the RL landing burns (reference integrator) only");
    const int64_t N = e->cfg.n_envs;
    const int64_t W = 2 * (int64_t)e->obs_dim + e->act_dim + 2;
    if (ring_state) {
        if (!ring || capacity < N) return fail(PD_ERR_INVALID, "pd_step_sac_ring: ring mode needs ring and capacity >= n_envs");
        if (capacity * W >= (1ll << 32)) return fail(PD_ERR_INVALID, "pd_step_sac_ring: capacity x row width must be below 2^32");
        if (priorities && !max_priority) return fail(PD_ERR_INVALID, "pd_step_sac_ring: priorities without max_priority");
    }
    PD_HIP(hipSetDevice(e->device));
    const int A = e->act_dim;
    SacIO io{heads, heads + A, nullptr, log_std_min, log_std_max, max_action, action, ring, obs32, (uint32_t)(2 * A)};
    io.draw = deterministic ? 0 : 1;
    io.eps_out = deterministic ? nullptr : eps_out;
    io.ring_cap = ring_state ? capacity : 0;
    io.ring_state = ring_state;
    io.prio = ring_state ? priorities : nullptr;
    io.max_prio = max_priority;
    if (e->rsize == 8)
        return step_impl<double>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 (hipStream_t)stream, 1, &io);
    return step_impl<float>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                            (hipStream_t)stream, 1, &io);
}

pd_status pd_step_sac_fused(pd_env* e, int32_t state_dim, int32_t action_dim, int32_t hidden, int32_t n_hidden_layers,
                            const float* const* params, float* heads, int32_t deterministic, float log_std_min,
                            float log_std_max, float max_action, float* eps_out, float* action, float* ring,
                            int64_t capacity, long long* ring_state, float* priorities, const float* max_priority,
                            float* obs32, void* stream) {
    if (!e || !params || !obs32) return fail(PD_ERR_INVALID, "pd_step_sac_fused: null env/params/obs32");
    const int S = e->obs_dim, A = e->act_dim;
    // the actor's widths must be the handle's: its weights are read with the handle's row strides
    if (state_dim != S || action_dim != A)
        return fail(PD_ERR_INVALID, "pd_step_sac_fused: the actor's state_dim / action_dim differ from the handle's");
    if (n_hidden_layers < 1 || n_hidden_layers > kSacMaxLayers || A > 8 || S > 16)
        return fail(PD_ERR_INVALID, "pd_step_sac_fused: 1..8 hidden layers, state_dim <= 16, action_dim <= 8");
    if (hidden != 128 && hidden != 256 && hidden != 512)
        return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_fused: hidden width 128, 256 or 512 only");
    for (int k = 0; k < 2 * (n_hidden_layers + 2); ++k) {
        if (!params[k]) return fail(PD_ERR_INVALID, "pd_step_sac_fused: null parameter");
        if ((uintptr_t)params[k] % 16 != 0) return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_fused: parameter not 16-byte aligned");
    }
    // one launch where the workgroup's envs are one MLP tile (16 lanes per env) and the tile's
    // activations fit the kernel's LDS (hidden <= 256); else pd_sac_actor into `heads` (or the
    // handle's scratch rows) and pd_step_sac_ring: two launches, the same heads bit for bit
    if (e->lpe != 16 || hidden > 256) {
        const int64_t N = e->cfg.n_envs;
        float* h = heads;
        if (!h) {
            if (!e->sac_heads) {
                PD_HIP(hipSetDevice(e->device));
                PD_HIP(hipMalloc((void**)&e->sac_heads, (size_t)N * 2 * A * sizeof(float)));
                e->allocs.push_back(e->sac_heads);
            }
            h = e->sac_heads;
        }
        PD_HIP(hipSetDevice(e->device));
        const pd_status st = pd_sac_actor(N, S, hidden, n_hidden_layers, A, obs32, params, h, stream);
        if (st != PD_OK) return st;
        return pd_step_sac_ring(e, h, deterministic, log_std_min, log_std_max, max_action, eps_out, action, ring,
                                capacity, ring_state, priorities, max_priority, obs32, stream);
    }
    if (e->cfg.action_f64) return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_fused: float32 actions only (action_f64 = 0)");
    if (e->cfg.rtd == PD_RTD_PSO || e->cfg.integrator != PD_INTEG_REFERENCE ||
        (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN))
        return fail(PD_ERR_UNSUPPORTED, "pd_step_sac_fused: the RL landing burns (reference integrator) only");
    const int64_t N = e->cfg.n_envs;
    const int64_t W = 2 * (int64_t)S + A + 2;
    if (ring_state) {
        if (!ring || capacity < N) return fail(PD_ERR_INVALID, "pd_step_sac_fused: ring mode needs ring and capacity >= n_envs");
        if (capacity * W >= (1ll << 32)) return fail(PD_ERR_INVALID, "pd_step_sac_fused: capacity x row width must be below 2^32");
        if (priorities && !max_priority) return fail(PD_ERR_INVALID, "pd_step_sac_fused: priorities without max_priority");
    }
    PD_HIP(hipSetDevice(e->device));
    SacIO io{nullptr, nullptr, nullptr, log_std_min, log_std_max, max_action, action, ring, obs32, (uint32_t)(2 * A)};
    io.draw = deterministic ? 0 : 1;
    io.eps_out = deterministic ? nullptr : eps_out;
    io.ring_cap = ring_state ? capacity : 0;
    io.ring_state = ring_state;
    io.prio = ring_state ? priorities : nullptr;
    io.max_prio = max_priority;
    io.mlp.S = S; io.mlp.L = n_hidden_layers; io.mlp.A = A; io.mlp.H = hidden; io.mlp.obs = obs32;
    for (int l = 0; l < n_hidden_layers; ++l) { io.mlp.w[l] = params[2 * l]; io.mlp.b[l] = params[2 * l + 1]; }
    io.mlp.wm = params[2 * n_hidden_layers]; io.mlp.bm = params[2 * n_hidden_layers + 1];
    io.mlp.ws = params[2 * n_hidden_layers + 2]; io.mlp.bs = params[2 * n_hidden_layers + 3];
    io.heads_out = heads;
    if (e->rsize == 8)
        return step_impl<double>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 (hipStream_t)stream, 1, &io);
    return step_impl<float>(e, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                            (hipStream_t)stream, 1, &io);
}

pd_status pd_step_n(pd_env* e, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                    uint8_t* truncated, int8_t* trunc_id, void* stream) {
    if (!e || !actions || n_steps < 0) return fail(PD_ERR_INVALID, "bad step_n args");
    if (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN)
        return fail(PD_ERR_UNSUPPORTED, "pd_step_n: landing-burn phases only (use pd_step)");
    PD_HIP(hipSetDevice(e->device));
    return step_n_impl(e, actions, n_steps, obs, reward, done, truncated, trunc_id, nullptr, (hipStream_t)stream);
}

pd_status pd_step_n_info(pd_env* e, const void* actions, int32_t n_steps, void* obs, void* reward, uint8_t* done,
                         uint8_t* truncated, int8_t* trunc_id, void* info, uint64_t info_mask, void* stream) {
    if (!e || !actions || n_steps < 0) return fail(PD_ERR_INVALID, "bad step_n_info args");
    if (e->cfg.phase != PD_PHASE_PURE_THROTTLE && e->cfg.phase != PD_PHASE_LANDING_BURN)
        return fail(PD_ERR_UNSUPPORTED, "pd_step_n_info: landing-burn phases only (use pd_step)");
    if (info && (info_mask == 0 || (info_mask >> PD_N_INFO) != 0))
        return fail(PD_ERR_INVALID, "pd_step_n_info: info_mask must select 1..PD_N_INFO fields of pd_info_field");
    PD_HIP(hipSetDevice(e->device));
    return step_n_impl(e, actions, n_steps, obs, reward, done, truncated, trunc_id, nullptr, (hipStream_t)stream,
                       info, info ? info_mask : 0);
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
    }
    return PD_OK;
}

extern "C++" {
namespace {
pd_status rollout_policy_entry(pd_env* e, const float* weights, int32_t n_params, int32_t max_steps, void* fitness,
                               int32_t* steps, int32_t check_every, void* stream, bool chunked) {
    if (!e || !weights || !fitness || max_steps < 0) return fail(PD_ERR_INVALID, "bad policy rollout args");
    if (e->cfg.rtd != PD_RTD_PSO) return fail(PD_ERR_UNSUPPORTED, "policy rollouts need rtd = PD_RTD_PSO");
    if (e->cfg.integrator != PD_INTEG_REFERENCE) return fail(PD_ERR_UNSUPPORTED, "policy rollouts use the reference integrator");
    int want = e->cfg.phase == PD_PHASE_PURE_THROTTLE ? PD_ACTOR_PARAMS_PURE_THROTTLE : PD_ACTOR_PARAMS_LANDING_BURN;
    if (n_params != want) return fail(PD_ERR_INVALID, "n_params does not match the phase's actor");
    if (chunked && (uintptr_t)weights % 16 != 0) return fail(PD_ERR_INVALID, "chunked policy weights must be 16-byte aligned");
    // the kernel addresses the chunked weights [ceil(P/4)][N][4] with 32-bit per-lane byte offsets
    if ((uint64_t)e->cfg.n_envs * (uint64_t)((n_params + 3) / 4) * 16ull >= (1ull << 32))
        return fail(PD_ERR_INVALID, "policy rollouts: n_envs x ceil(n_params / 4) x 16 must be below 2^32 bytes");
    PD_HIP(hipSetDevice(e->device));
    return e->rsize == 8 ? rollout_policy_impl<double>(e, weights, max_steps, fitness, steps, check_every, (hipStream_t)stream, chunked)
                         : rollout_policy_impl<float>(e, weights, max_steps, fitness, steps, check_every, (hipStream_t)stream, chunked);
}
}  // namespace
}  // extern "C++"

pd_status pd_rollout_policy(pd_env* e, const float* weights, int32_t n_params, int32_t max_steps, void* fitness,
                            int32_t* steps, int32_t check_every, void* stream) {
    return rollout_policy_entry(e, weights, n_params, max_steps, fitness, steps, check_every, stream, false);
}

pd_status pd_rollout_policy_chunked(pd_env* e, const float* weights4, int32_t n_params, int32_t max_steps,
                                    void* fitness, int32_t* steps, int32_t check_every, void* stream) {
    return rollout_policy_entry(e, weights4, n_params, max_steps, fitness, steps, check_every, stream, true);
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
    unsigned long long st[kStats];
    PD_HIP(hipMemcpy(st, e->pend.stats, sizeof(st), hipMemcpyDeviceToHost));
    if (misses) *misses = (int64_t)st[0];
    if (nans) *nans = (int64_t)st[1];
    if (ecd) *ecd = (int64_t)st[2];
    if (ecl) *ecl = (int64_t)st[3];
    return PD_OK;
}

pd_status pd_atmosphere(pd_env* e, const void* altitude, void* out, int64_t n, void* stream) {
    if (!e || !altitude || !out || n < 0) return fail(PD_ERR_INVALID, "bad pd_atmosphere args");
    if (n == 0) return PD_OK;
    PD_HIP(hipSetDevice(e->device));
    unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
    hipStream_t s = (hipStream_t)stream;
    if (e->rsize == 8) hipLaunchKernelGGL(k_atmosphere<double>, dim3(grid), dim3(kBlock), 0, s, make_args<double>(e), (const double*)altitude, (double*)out, n);
    else hipLaunchKernelGGL(k_atmosphere<float>, dim3(grid), dim3(kBlock), 0, s, make_args<float>(e), (const float*)altitude, (float*)out, n);
    PD_HIP(hipGetLastError());
    return PD_OK;
}

pd_status pd_stats(pd_env* e, int64_t* out, int32_t n) {
    if (!e || !out || n < 0) return fail(PD_ERR_INVALID, "bad pd_stats args");
    PD_HIP(hipSetDevice(e->device));
    unsigned long long st[kStats];
    PD_HIP(hipMemcpy(st, e->pend.stats, sizeof(st), hipMemcpyDeviceToHost));
    for (int32_t k = 0; k < n && k < kStats; ++k) out[k] = (int64_t)st[k];
    return PD_OK;
}

pd_status pd_count_work(pd_env* e, int32_t enable) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    e->count_work = enable != 0;
    return PD_OK;
}

pd_status pd_get_gload_window(pd_env* e, void* vprev, void* window, uint8_t* len, uint8_t* head, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    if (vprev) PD_HIP(hipMemcpyAsync(vprev, e->vprev, N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (window) PD_HIP(hipMemcpyAsync(window, e->gwin, 10 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (len) PD_HIP(hipMemcpyAsync(len, e->glen, N, hipMemcpyDeviceToDevice, s));
    if (head) PD_HIP(hipMemcpyAsync(head, e->ghead, N, hipMemcpyDeviceToDevice, s));
    return PD_OK;
}

pd_status pd_get_wind_state(pd_env* e, void* filters, void* sigmas, uint8_t* profile, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    if (filters) PD_HIP(hipMemcpyAsync(filters, e->wind, 4 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (sigmas) PD_HIP(hipMemcpyAsync(sigmas, (char*)e->wind + 4 * N * e->rsize, 2 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (profile) PD_HIP(hipMemcpyAsync(profile, e->wprof, N, hipMemcpyDeviceToDevice, s));
    return PD_OK;
}

// The wind profile bytes of n envs (device memory) are all valid ids (percentile - 50 in 0..49):
// k_step indexes the LDS profiles and wind_n[] with them.  Stream-ordered read-back (setters only).
static pd_status check_profiles(const uint8_t* dev, size_t n, hipStream_t s) {
    std::vector<uint8_t> h(n);
    PD_HIP(hipMemcpyAsync(h.data(), dev, n, hipMemcpyDeviceToHost, s));
    PD_HIP(hipStreamSynchronize(s));
    for (size_t i = 0; i < n; ++i)
        if (h[i] >= PD_N_WIND_PROFILES)
            return fail(PD_ERR_INVALID, "wind profile id " + std::to_string(h[i]) + " of env " + std::to_string(i) +
                                            " out of range (percentile must be 50..99)");
    return PD_OK;
}

pd_status pd_set_wind_state(pd_env* e, const void* filters, const void* sigmas, const uint8_t* profile, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    if (profile) {   // refused before anything is written
        pd_status st = check_profiles(profile, N, s);
        if (st != PD_OK) return st;
    }
    if (filters) PD_HIP(hipMemcpyAsync(e->wind, filters, 4 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (sigmas) PD_HIP(hipMemcpyAsync((char*)e->wind + 4 * N * e->rsize, sigmas, 2 * N * e->rsize, hipMemcpyDeviceToDevice, s));
    if (profile) PD_HIP(hipMemcpyAsync(e->wprof, profile, N, hipMemcpyDeviceToDevice, s));
    return PD_OK;
}

pd_status pd_get_counters(pd_env* e, uint32_t* episode, uint32_t* step, int8_t* trunc_id, void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    if (episode) PD_HIP(hipMemcpyAsync(episode, e->epi, N * 4, hipMemcpyDeviceToDevice, s));
    if (step) PD_HIP(hipMemcpyAsync(step, e->tstep, N * 4, hipMemcpyDeviceToDevice, s));
    if (trunc_id) PD_HIP(hipMemcpyAsync(trunc_id, e->tid, N, hipMemcpyDeviceToDevice, s));
    return PD_OK;
}

pd_status pd_set_counters(pd_env* e, const uint32_t* episode, const uint32_t* step, const int8_t* trunc_id,
                          void* stream) {
    if (!e) return fail(PD_ERR_INVALID, "null env");
    PD_HIP(hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t N = (size_t)e->cfg.n_envs;
    if (episode) PD_HIP(hipMemcpyAsync(e->epi, episode, N * 4, hipMemcpyDeviceToDevice, s));
    if (step) PD_HIP(hipMemcpyAsync(e->tstep, step, N * 4, hipMemcpyDeviceToDevice, s));
    if (trunc_id) PD_HIP(hipMemcpyAsync(e->tid, trunc_id, N, hipMemcpyDeviceToDevice, s));
    return PD_OK;
}

// The per-env buffers of a handle in checkpoint-blob order, each 16-byte aligned in the blob.
static int checkpoint_fields(const pd_env* e, void** ptr, size_t* bytes) {
    const size_t N = (size_t)e->cfg.n_envs, R = e->rsize;
    void* p[] = {e->st, e->vprev, e->gwin, e->act, e->wind, e->ghead, e->glen, e->wprof, e->key, e->slot,
                 e->tid, e->epi, e->tstep, e->fin};
    size_t b[] = {11 * N * R, N * R, 10 * N * R, 3 * N * R, 6 * N * R, N, N, N, 2 * N * 8, 2 * N * 4, N, N * 4, N * 4, N};
    const int n = (int)(sizeof(b) / sizeof(b[0]));
    for (int k = 0; k < n; ++k) { ptr[k] = p[k]; bytes[k] = b[k]; }
    return n;
}
static size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

size_t pd_checkpoint_size(const pd_env* e) {
    if (!e) return 0;
    void* p[16]; size_t b[16];
    int n = checkpoint_fields(e, p, b);
    size_t t = 0;
    for (int k = 0; k < n; ++k) t += align16(b[k]);
    return t;
}

pd_status pd_checkpoint_save(pd_env* e, void* blob, void* stream) {
    if (!e || !blob) return fail(PD_ERR_INVALID, "null env/blob");
    PD_HIP(hipSetDevice(e->device));
    void* p[16]; size_t b[16];
    int n = checkpoint_fields(e, p, b);
    size_t off = 0;
    for (int k = 0; k < n; ++k) {
        PD_HIP(hipMemcpyAsync((char*)blob + off, p[k], b[k], hipMemcpyDeviceToDevice, (hipStream_t)stream));
        off += align16(b[k]);
    }
    return PD_OK;
}

pd_status pd_checkpoint_load(pd_env* e, const void* blob, void* stream) {
    if (!e || !blob) return fail(PD_ERR_INVALID, "null env/blob");
    PD_HIP(hipSetDevice(e->device));
    void* p[16]; size_t b[16];
    int n = checkpoint_fields(e, p, b);
    size_t off = 0;
    for (int k = 0; k < n; ++k) {   // a blob with invalid wind profile ids is refused before loading
        if (p[k] == e->wprof) {
            pd_status st = check_profiles((const uint8_t*)blob + off, b[k], (hipStream_t)stream);
            if (st != PD_OK) return st;
        }
        off += align16(b[k]);
    }
    off = 0;
    for (int k = 0; k < n; ++k) {
        PD_HIP(hipMemcpyAsync(p[k], (const char*)blob + off, b[k], hipMemcpyDeviceToDevice, (hipStream_t)stream));
        off += align16(b[k]);
    }
    return PD_OK;
}

int pd_obs_dim(const pd_env* e) { return e ? e->obs_dim : 0; }
int pd_action_dim(const pd_env* e) { return e ? e->act_dim : 0; }

}  // extern "C"
