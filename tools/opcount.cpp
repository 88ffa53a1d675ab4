// opcount.cpp -- the exact algorithmic operation count of one env-step of the step kernel
// (SURVEY 8(d) "ALGORITHMIC FLOPs").
//
// The device step (csrc/pd_step_impl.h k_step, pure throttle, rtd_rl, wind, binary64) is restated
// here operation by operation as templates over the scalar type T, and instantiated twice:
//   T = double : a CHECK that the restatement computes the env step -- one env-step from any state
//                equals the oracle's (oracle/pd_oracle.c orc_step, C_D / C_L from its exact RBF)
//                to the per-step parity tolerances (tests/test_opcount.py);
//   T = Cnt    : every +, -, *, /, fma, sqrt and comparison executed is counted, and every
//                transcendental (log, exp, sin, cos, atan2, hypot) counted apart.
// The aero tables are served, per query, by one of the kernel's paths -- a clamped-line query by
// its Taylor piece (pd_step_impl.h taylor_eval), an interior query by its cell piece (cell_eval,
// through the fine index; a bisector sub-cell adds the side test), a verified query by the
// payload sums (chunk_sum / rbf_finish) -- and each path's formulas are executed with T = Cnt on
// a record of the right shape, so the count is per path.  The counts cover what one env computes
// (algorithmic work): not the instructions a SIMD issues for it (both lanes of an env, masked
// lanes, address arithmetic, the v_div / sqrt / log expansions).  FLOPs: add, sub, mul, div and
// sqrt count 1, fma counts 2; transcendentals, comparisons and binary32 operations are listed
// apart.  Philox's integer rounds are not floating point and not counted.
//
// Build (test infrastructure; links the oracle for the check only):
//   g++ -O1 -std=c++17 -ffp-contract=off -shared -fPIC tools/opcount.cpp -I oracle -o <lib> oracle/build/liborc.so
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "pd_oracle.h"

namespace {

// ---------------------------------------------------------------- the counting scalar types
struct Ops { double add, mul, div, fma, sqrt, cmp, log, exp, sin, cos, atan2, hypot, tanh, f32; };
Ops g;

struct Cnt {
    double v;
    Cnt() : v(0) {}
    Cnt(double x) : v(x) {}   // literals and parameters enter uncounted
};
inline Cnt operator+(Cnt a, Cnt b) { ++g.add; return Cnt(a.v + b.v); }
inline Cnt operator-(Cnt a, Cnt b) { ++g.add; return Cnt(a.v - b.v); }
inline Cnt operator*(Cnt a, Cnt b) { ++g.mul; return Cnt(a.v * b.v); }
inline Cnt operator/(Cnt a, Cnt b) { ++g.div; return Cnt(a.v / b.v); }
inline Cnt operator-(Cnt a) { return Cnt(-a.v); }                      // sign flip: free
inline Cnt& operator+=(Cnt& a, Cnt b) { a = a + b; return a; }
inline Cnt& operator-=(Cnt& a, Cnt b) { a = a - b; return a; }
inline bool operator<(Cnt a, Cnt b) { ++g.cmp; return a.v < b.v; }
inline bool operator>(Cnt a, Cnt b) { ++g.cmp; return a.v > b.v; }
inline bool operator<=(Cnt a, Cnt b) { ++g.cmp; return a.v <= b.v; }
inline bool operator>=(Cnt a, Cnt b) { ++g.cmp; return a.v >= b.v; }
inline bool operator==(Cnt a, Cnt b) { ++g.cmp; return a.v == b.v; }
inline bool operator!=(Cnt a, Cnt b) { ++g.cmp; return a.v != b.v; }
inline Cnt fma(Cnt a, Cnt b, Cnt c) { ++g.fma; return Cnt(std::fma(a.v, b.v, c.v)); }
inline Cnt sqrt(Cnt a) { ++g.sqrt; return Cnt(std::sqrt(a.v)); }
inline Cnt fabs(Cnt a) { return Cnt(std::fabs(a.v)); }
inline Cnt log(Cnt a) { ++g.log; return Cnt(std::log(a.v)); }
inline Cnt exp(Cnt a) { ++g.exp; return Cnt(std::exp(a.v)); }
inline Cnt atan2(Cnt a, Cnt b) { ++g.atan2; return Cnt(std::atan2(a.v, b.v)); }
inline Cnt hypot(Cnt a, Cnt b) { ++g.hypot; return Cnt(std::hypot(a.v, b.v)); }
inline void sincos_t(Cnt x, Cnt& s, Cnt& c) { ++g.sin; ++g.cos; s = Cnt(std::sin(x.v)); c = Cnt(std::cos(x.v)); }
inline void sincos_t(double x, double& s, double& c) { s = std::sin(x); c = std::cos(x); }
inline double val(Cnt a) { return a.v; }
inline double val(double a) { return a; }

// binary32 island operations (counted apart)
struct CntF {
    float v;
    CntF() : v(0) {}
    CntF(float x) : v(x) {}
};
inline CntF operator+(CntF a, CntF b) { ++g.f32; return CntF(a.v + b.v); }
inline CntF operator-(CntF a, CntF b) { ++g.f32; return CntF(a.v - b.v); }
inline CntF operator*(CntF a, CntF b) { ++g.f32; return CntF(a.v * b.v); }
inline CntF operator/(CntF a, CntF b) { ++g.f32; return CntF(a.v / b.v); }
template <typename T> struct F32 { using type = float; };
template <> struct F32<Cnt> { using type = CntF; };
inline float fval(float a) { return a; }
inline float fval(CntF a) { return a.v; }

using std::fabs;
using std::fma;
using std::sqrt;
using std::log;
using std::exp;
using std::atan2;
using std::hypot;

constexpr double kPi = 3.141592653589793, kDeg = kPi / 180.0, kRad = 180.0 / kPi;

// ---------------------------------------------------------------- the step, restated
// pd_physics.h atmosphere (per-layer terms precomputed on the host, as D.isa_bt / ex / iso)
template <typename T>
void atmosphere(const orc_params* P, T y, T& rho, T& p, T& a) {
    T alt = y < T(0) ? T(0) : y;
    if (alt < T(P->isa_alt_max)) {
        T H = T(P->isa_r) * alt / (T(P->isa_r) + alt);
        int i = 0;
        for (int k = 1; k < 9; ++k) i = (T(P->isa_Hb[k]) <= H) ? k : i;
        const double b = P->isa_beta[i], Tb = P->isa_Tb[i];
        T dH = H - T(P->isa_Hb[i]);
        T Tk = T(Tb) + T(b) * dH;
        T pp;
        if (b != 0.0) pp = T(P->isa_pb[i]) * exp(T(-P->isa_g0 / (b * P->isa_R)) * log(T(1) + T(b / Tb) * dH));
        else pp = T(P->isa_pb[i]) * exp(T(-P->isa_g0 / (P->isa_R * Tb)) * dH);
        p = pp;
        rho = pp / (T(P->isa_R) * Tk);
        a = sqrt(T(P->isa_kappa * P->isa_R) * Tk);
    } else {
        rho = T(0); p = T(0); a = T(0);
    }
}

// pd_physics.h inertia (stage_inertia closure)
template <typename T>
void inertia(const orc_params* P, T fill, T& x_cog, T& I) {
    T h_ox_t = T(P->h_ox) * fill, h_f_t = T(P->h_f) * fill, m_ox_t = T(P->m_ox) * fill, m_f_t = T(P->m_f) * fill;
    T x_prop = (m_ox_t * (T(P->h_lower) + h_ox_t / T(2)) + m_f_t * (T(P->h_lower) + T(P->h_ox) + h_f_t / T(2))) / (m_ox_t + m_f_t);
    T t1 = T(P->h_lower) + h_ox_t / T(2) - x_prop;
    T I_ox = T(1.0 / 12) * m_ox_t * (h_ox_t * h_ox_t) + m_ox_t * (t1 * t1);
    T t2 = T(P->h_lower) + T(P->h_ox) + h_f_t / T(2) - x_prop;
    T I_f = T(1.0 / 12) * m_f_t * (h_f_t * h_f_t) + m_f_t * (t2 * t2);
    T mp_t = m_ox_t + m_f_t;
    T x_wet = (T(P->m_dry) * T(P->x_dry) + mp_t * x_prop) / (T(P->m_dry) + mp_t);
    T t3 = T(P->x_dry) - x_wet, t4 = x_prop - x_wet;
    x_cog = x_wet;
    I = (T(P->I_dry) + T(P->m_dry) * (t3 * t3)) + ((I_ox + I_f) + mp_t * (t4 * t4));
}

// pd_physics.h grid_fin_ca with the interval slopes tabulated (one subtraction, one product, one
// sum per query; the binary search and the bucket are comparisons)
template <typename T>
T grid_fin_ca(const orc_params* P, T mach) {
    if (mach < T(P->ca_min_mach)) return T(P->ca_min_val);
    const int n = P->ca_n;
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (T(P->ca_x[mid]) < mach) lo = mid + 1; else hi = mid; }
    const int idx = lo < 1 ? 1 : (lo > n - 1 ? n - 1 : lo);
    const double sl = (P->ca_y[idx] - P->ca_y[idx - 1]) / (P->ca_x[idx] - P->ca_x[idx - 1]);   // (tabulated)
    return T(sl) * (mach - T(P->ca_x[idx - 1])) + T(P->ca_y[idx - 1]);
}

// np.interp of the wind profile (slope computed per query, as the kernel does)
template <typename T>
T np_interp(const double* x, const double* y, int n, T v) {
    if (v < T(x[0])) return T(y[0]);
    if (v >= T(x[n - 1])) return T(y[n - 1]);
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (T(x[mid]) <= v) lo = mid + 1; else hi = mid; }
    const int j = lo - 1;
    if (T(x[j]) == v) return T(y[j]);
    const T sl = (T(y[j + 1]) - T(y[j])) / (T(x[j + 1]) - T(x[j]));
    return sl * (v - T(x[j])) + T(y[j]);
}

// ---- the aero query paths (pd_step_impl.h), executed on a record of the right shape
constexpr int kTayDeg = 10, kTayExact = 2, kCellDeg = 8, kCellExact = 4;

// a clamped-line query: the Mach bucket, the interval test against the breakpoints, the Taylor
// cell, then taylor_eval
template <typename T>
T line_query(T M, const double* rec, double blo, double bhi) {
    T bk = M * T(128 / 10.0);
    (void)bk;
    const bool trusted = (M - T(blo) > T(1e-9)) && (T(bhi) - M > T(1e-9));
    (void)trusted;
    T cellf = M * T(2048 / 10.0);
    const int cell = (int)val(cellf);
    const double w = 10.0 / 2048;
    T t = M - fma(T((double)cell), T(w), T(0.5 * w));
    T f = T(rec[kTayDeg]);
    for (int n = kTayDeg - 1; n >= 0; --n) f = fma(f, t, T(rec[n]));
    for (int e = 0; e < kTayExact; ++e) {
        const double* x = rec + kTayDeg + 1 + 3 * e;
        T dm = M - T(x[0]);
        T d2 = fma(dm, dm, T(x[2]));
        f = fma(T(x[1]) * d2, T(4) * log(d2), f);   // (the kernel's log4: one log, scaled by 4)
    }
    return f;
}

// an interior query: the grid and sub-cell position, the margins, the bisector side test
// (bisect), then cell_eval
template <typename T>
T piece_query(T M, T aq, const double* rec, double inv_dm, double a0, double inv_da, bool bisect) {
    T fm = M * T(inv_dm), fa = (aq - T(a0)) * T(inv_da);
    const double im = std::floor(val(fm)), ia = std::floor(val(fa));
    T um = fm - T(im), ua = fa - T(ia);
    T sm = um * T(8), sa = ua * T(8);
    T fsm = sm - T(std::floor(val(sm))), fsa = sa - T(std::floor(val(sa)));
    const bool inside = fsm > T(1e-9) && T(1) - fsm > T(1e-9) && fsa > T(1e-9) && T(1) - fsa > T(1e-9);
    (void)inside;
    if (bisect) {
        T sv = fma(T(0.7), M, fma(T(0.3), aq, T(-0.5)));
        const bool trusted = fabs(sv) > T(3.0) * T(1e-12);
        (void)trusted;
    }
    T u = T(2) * um - T(1), v = T(2) * ua - T(1);
    T f = T(0);
    int q = 0;
    for (int i = kCellDeg; i >= 0; --i) {
        T qi = T(rec[q++]);
        for (int j = kCellDeg - i - 1; j >= 0; --j) qi = fma(qi, v, T(rec[q++]));
        f = i == kCellDeg ? qi : fma(f, u, qi);
    }
    for (int e = 0; e < kCellExact; ++e) {
        const double* x = rec + (kCellDeg + 1) * (kCellDeg + 2) / 2 + 3 * e;
        T dm = M - T(x[0]), da = aq - T(x[2]);
        T d2 = fma(dm, dm, da * da);
        f = fma(T(x[1]) * d2, T(4) * log(d2), f);
    }
    return f;
}

// a verified query's payload sums: five chunks of five pair slots (ten terms; the general slot's
// second point has its own AoA), summed in order, then rbf_finish
template <typename T>
T payload_query(T M, T a, const double* pay) {
    T tot = T(0);
    for (int c = 0; c < 5; ++c) {
        T s0 = T(0), s1 = T(0);
        T da2[6];
        for (int u = 0; u < 6; ++u) { T da = a - T(2.0 * u); da2[u] = da * da; }
        for (int u = 0; u < 5; ++u)
            for (int i = 0; i < 2; ++i) {
                T dm = M - T(0.1 * (2 * u + i + 1));
                T d2 = fma(dm, dm, da2[u == 4 && i ? 5 : u]);
                T wk = d2 * T(pay[10 * c + 2 * u + i]);
                if (i) s1 = fma(wk, T(4) * log(d2), s1); else s0 = fma(wk, T(4) * log(d2), s0);
            }
        T cs = s0 + s1;
        tot = c == 0 ? cs : tot + cs;
    }
    T s = T(0.125) * tot;
    s += T(1) * T(pay[50]);
    s += (M - T(pay[53])) / T(pay[55]) * T(pay[51]);
    s += (a - T(pay[54])) / T(pay[56]) * T(pay[52]);
    return s;
}

// the queries' abscissae (cd_query / cl_query)
template <typename T>
void queries(T ae, T& aq_cd, T& aq_cl, T& sgn, bool& zero) {
    aq_cd = ae * T(kRad);
    if (aq_cd > T(10 * kDeg)) aq_cd = T(10 * kDeg); else if (aq_cd < T(-10 * kDeg)) aq_cd = T(-10 * kDeg);
    aq_cl = (ae * T(kRad)) * T(kRad);
    sgn = T(1); zero = false;
    if (aq_cl > T(10)) aq_cl = T(10);
    else if (aq_cl < T(-10)) aq_cl = T(-10);
    else if (fabs(aq_cl) < T(1e-6)) zero = true;
    else if (aq_cl < T(0)) { aq_cl = fabs(aq_cl); sgn = T(-1); }
}

// the wind block: the profile, and in the gust band the Box-Muller pair and both filters
template <typename T>
void wind_block(const orc_params* P, T y, bool gust, double w0, double w1, T* fu, T* fv, double sgu, double sgv,
                T& ug, T& vg) {
    T km = y / T(1000);
    ug = np_interp<T>(P->wind_alt_km, P->wind_speed, P->wind_n, km);
    vg = T(0);
    if (gust) {
        // gauss_pair (one pair per sub-step): u1 = 1 - u01, rho = sqrt(-2 log u1), (rho cos, rho sin)(2 pi u2)
        T u1 = T(1) - T(0.37), u2 = T(0.61);
        T rho = sqrt(T(-2) * log(u1));
        T s, c;
        sincos_t(T(2 * kPi) * u2, s, c);
        T z0 = rho * c, z1 = rho * s;
        (void)z0; (void)z1;
        T n0 = (T(P->vk_Ad_u[0]) * fu[0] + T(P->vk_Ad_u[1]) * fu[1]) + (T(sgu) * T(P->vk_Bd_u[0])) * T(w0);
        T n1 = (T(P->vk_Ad_u[2]) * fu[0] + T(P->vk_Ad_u[3]) * fu[1]) + (T(sgu) * T(P->vk_Bd_u[1])) * T(w0);
        fu[0] = n0; fu[1] = n1;
        n0 = (T(P->vk_Ad_v[0]) * fv[0] + T(P->vk_Ad_v[1]) * fv[1]) + (T(sgv) * T(P->vk_Bd_v[0])) * T(w1);
        n1 = (T(P->vk_Ad_v[2]) * fv[0] + T(P->vk_Ad_v[3]) * fv[1]) + (T(sgv) * T(P->vk_Bd_v[1])) * T(w1);
        fv[0] = n0; fv[1] = n1;
        ug = ug + fu[1];
        vg = fv[1];
    }
}

// Aero values: the double instantiation takes the oracle's exact RBF (what every path of the
// kernel reproduces to 1e-13); the counting one runs the chosen path's formulas.
enum Path { LINE = 0, PIECE = 1, BISECT = 2, PAYLOAD = 3 };
double g_rec[128];

template <typename T>
T aero_value(const orc_params* P, int table, T M, T aq, int path);
template <>
double aero_value<double>(const orc_params* P, int table, double M, double aq, int) {
    return orc_rbf(P, table, M, aq);
}
template <>
Cnt aero_value<Cnt>(const orc_params*, int, Cnt M, Cnt aq, int path) {
    if (path == LINE) return line_query<Cnt>(M, g_rec, 0.0, 10.0);
    if (path == PAYLOAD) return payload_query<Cnt>(M, aq, g_rec);
    return piece_query<Cnt>(M, aq, g_rec, 80.0, 0.0, 40.0, path == BISECT);
}

// One physics sub-step (pd_step_impl.h k_step's loop body, PHASE 0 with float32 actions).
// atm_fresh: false on a step's first sub-step (the previous step's rtd atmosphere is reused).
template <typename T>
void substep(const orc_params* P, T* s, float u0, bool atm_fresh, T* atm, bool wind, bool gust, T* fu, T* fv,
             int path_cd, int path_cl) {
    using F = typename F32<T>::type;
    T x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], thd = s[5], ga = s[6], al = s[7], m = s[8], mp = s[9];
    T rho, patm, asnd, speed;
    if (!atm_fresh) { rho = atm[0]; patm = atm[1]; asnd = atm[2]; speed = atm[3]; }
    else { atmosphere<T>(P, y, rho, patm, asnd); speed = sqrt(vx * vx + vy * vy); }
    T mach = T(0);
    if (asnd != T(0)) { T mr = speed / asnd; mach = (T(10) < mr) ? T(10) : mr; }
    T ae = (vy < T(0)) ? ga - th - T(kPi) : al;
    T ug = T(0), vg = T(0);
    if (wind) wind_block<T>(P, y, gust, 0.3, -0.7, fu, fv, 1.0, 1.5, ug, vg);
    T aq_cd, aq_cl, sgn;
    bool zero;
    queries<T>(ae, aq_cd, aq_cl, sgn, zero);
    const bool have = asnd != T(0);
    T vcd = aero_value<T>(P, 0, mach, aq_cd, path_cd);
    T vcl = aero_value<T>(P, 1, mach, aq_cl, path_cl);
    T CD = have ? vcd : T(0);
    T CL = (!have || zero) ? T(0) : (sgn < T(0) ? -vcl : vcl);
    T q = T(0.5) * rho * (speed * speed);
    T fpc = (T(P->m_prop0) - mp) / T(P->m_prop0);
    if (fpc == T(0)) fpc = T(1e-6);
    T x_cog, I;
    inertia<T>(P, T(1) - fpc, x_cog, I);
    T d_cp_cg = x_cog - T(P->cop);
    T Fwx = T(0.5) * rho * (ug * ug) * T(P->A_front) * T(P->C_gust_x);
    T Fwy = T(0.5) * rho * (vg * vg) * T(P->A_front) * T(P->C_gust_y);
    T Mw = -d_cp_cg * Fwy;
    T drag = T(0.5) * rho * (speed * speed) * CD * T(P->A_front);
    T lift = T(0.5) * rho * (speed * speed) * CL * T(P->A_front);
    T sae, cae, sth, cth;
    sincos_t(ae, sae, cae);
    sincos_t(th, sth, cth);
    T apar, aperp;
    if (vy >= T(0)) { apar = lift * sae - drag * cae; aperp = -lift * cae - drag * sae; }
    else { apar = drag * cae - lift * sae; aperp = -drag * sae - lift * cae; }
    T aero_x = apar * cth + aperp * sth;
    T aero_y = apar * sth - aperp * cth;
    T aero_m = aperp * d_cp_cg;
    T T_full = T(P->T_e) + (T(P->p_e) - patm) * T(P->A_e);
    T qS = q * T(P->S_gf);
    T Ca = grid_fin_ca<T>(P, mach);
    T acs_par = qS * (Ca * T(4));
    // the float32 island (rockets_physics.py:372-379 under NEP 50)
    const float tau_nom = (float)(0.0 * 0.4 / 16);
    F nnt = (F(u0) + F(1.0f)) / F(2.0f);
    F thr = nnt * F((float)(1.0 - tau_nom)) + F(tau_nom);
    F tg = F((float)val(T_full * T((double)P->n_eng))) * thr;
    F md = F((float)(P->T_e / P->v_ex)) * (tg / F((float)val(T_full)));
    T cfp = T((double)fval(tg)) + acs_par;
    T mdot_dt = T((double)fval(md * F(0.025f)));
    T cfperp = T(0), cm = T(0);
    T cfx = cfp * cth + cfperp * sth;
    T cfy = cfp * sth - cfperp * cth;
    T fx = aero_x + cfx + Fwx, fy = aero_y + cfy + Fwy;
    T mz = cm + aero_m + Mw;
    T vxd = fx / m, vyq = fy / m, thdd = mz / I, grq = T(P->grav_R) / (T(P->grav_R) + y);
    T gr = T(P->grav_g0) * (grq * grq);
    T vyd = vyq - gr;
    const T dt = T(0.025);
    vx += vxd * dt; vy += vyd * dt; x += vx * dt; y += vy * dt;
    thd += thdd * dt; th += thd * dt;
    ga = atan2(vy, vx);
    if (th > T(2 * kPi)) th -= T(2 * kPi);
    if (ga < T(0)) ga = T(2 * kPi) + ga;
    al = th - ga;
    mp -= mdot_dt; m -= mdot_dt;
    s[0] = x; s[1] = y; s[2] = vx; s[3] = vy; s[4] = th; s[5] = thd; s[6] = ga; s[7] = al; s[8] = m; s[9] = mp;
    s[10] = s[10] + dt;
}

// The step's tail (pd_step_impl.h: g-load window, rtd_rl pure-throttle truncation / done /
// reward, the observation); ring/len: the window; atm receives the rtd's atmosphere and speed
template <typename T>
T step_tail(const orc_params* P, const T* s, T vprev, T* ring, int& len, T* atm, int& done, int& trunc,
            T* obs) {
    T v = sqrt(s[2] * s[2] + s[3] * s[3]);
    T gl_new = fabs(v - vprev) / T(0.1) * T(1) / T(9.81);
    if (len < 10) ring[len++] = gl_new;
    else { for (int k = 0; k < 9; ++k) ring[k] = ring[k + 1]; ring[9] = gl_new; }
    T gsum = T(0);
    for (int k = 0; k < len; ++k) gsum += ring[k];
    T gl = gsum / T(10);
    T x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], mp = s[9];
    (void)x;
    T rho, pa, as;
    atmosphere<T>(P, y, rho, pa, as);
    atm[0] = rho; atm[1] = pa; atm[2] = as; atm[3] = v;
    T speed = v;
    T q = T(0.5) * rho * (speed * speed);
    int tr = 0, dn;
    const T r2 = T(2 * kDeg);
    if (y < T(-10)) tr = 1;
    else if (mp <= T(0)) tr = 1;
    else if (th > T(kPi) + r2) tr = 1;
    else if (q > T(65000)) tr = 1;
    else if (gl > T(6)) tr = 1;
    else if (vy > T(0)) tr = 1;
    else if (vx > T(0.01)) tr = 1;
    dn = (y > T(0) && y < T(1) && speed < T(5));
    T rew = T(0);
    T sp = hypot(vx, vy);
    T qr = T(0.5) * rho * (sp * sp);
    if (qr > T(60000)) { T e_ = (qr - T(60000)) / T(5000); T e2 = e_ * e_; rew -= T(1) * (e2 > T(1) ? T(1) : e2); }
    if (gl > T(5.5)) { T e_ = (gl - T(5.5)) / (T(6) - T(5.5)); T e2 = e_ * e_; rew -= T(1) * (e2 > T(1) ? T(1) : e2); }
    T prog = (T(P->state0[1]) - y) / T(P->state0[1]);
    T wp = (qr <= T(60000) && gl <= T(5.5)) ? T(0.5) : T(0.5) * T(0.1);
    rew += wp * prog;
    if (y < T(100)) rew += T(5.5) * (T(1) - fabs(vy) / T(50));
    if (dn && !tr) rew += T(400) * mp / T(P->state0[8]);
    else if (tr && y > T(0)) rew -= T(50) * (fabs(y) / T(P->state0[1]));
    else if (tr && y < T(0)) rew -= T(50) * (fabs(vy) / T(10));
    if (!dn || !(tr && y < T(0))) rew = rew < T(-10) ? T(-10) : (rew > T(10) ? T(10) : rew);
    obs[0] = (T(1) - T((double)(float)val(s[1])) / T(P->norm_y)) * T(2) - T(1);
    obs[1] = (T(1) - T((double)(float)val(s[3])) / T(P->norm_vy)) * T(2) - T(1);
    done = dn; trunc = tr;
    return rew;
}

}  // namespace

extern "C" {

// One env-step of the restatement in binary64 from state s (pure throttle, rtd_rl, no wind, a
// fresh window [vprev, ring of len]): the check against orc_step.  Returns the reward.
double oc_step(const orc_params* P, double* s, float u0, double vprev, double* ring, int len, int* done, int* trunc,
               double* obs) {
    double atm[4] = {0, 0, 0, 0}, fu[2] = {0, 0}, fv[2] = {0, 0};
    for (int k = 0; k < 4; ++k) substep<double>(P, s, u0, true, atm, false, false, fu, fv, 0, 0);
    return step_tail<double>(P, s, vprev, ring, len, atm, *done, *trunc, obs);
}

// The counts, per unit (rows) x operation (columns: add mul div fma sqrt cmp log exp sin cos
// atan2 hypot tanh f32):
//  0 physics sub-step with a fresh atmosphere, no wind, the aero queries excluded
//  1 the same on a step's first sub-step (the rtd atmosphere reused)
//  2 the wind profile (every sub-step, wind on)   3 the gust block (a sub-step in the gust band)
//  4 a clamped-line query (Taylor piece)   5 an interior query (cell piece)
//  6 an interior query split by a bisector (cell piece + side test)   7 a verified query (payload sums)
//  8 the step tail (g-load window, rtd_rl, observation)
//  9 the atmosphere alone (a layer with a temperature gradient: the power law's log and exp)
void oc_counts(const orc_params* P, double* out /* [10][14] */) {
    for (int i = 0; i < 128; ++i) g_rec[i] = 1e-3 * (i + 1);
    g_rec[55] = 1.0; g_rec[56] = 1.0;
    auto take = [&](int row) {
        const double v[14] = {g.add, g.mul, g.div, g.fma, g.sqrt, g.cmp, g.log, g.exp, g.sin, g.cos, g.atan2, g.hypot,
                              g.tanh, g.f32};
        for (int k = 0; k < 14; ++k) out[row * 14 + k] = v[k];
        std::memset(&g, 0, sizeof g);
    };
    Cnt s0[11];
    for (int k = 0; k < 11; ++k) s0[k] = Cnt(P->state0[k]);
    Cnt atm[4] = {Cnt(0.4), Cnt(2e4), Cnt(300.0), Cnt(1000.0)}, fu[2] = {}, fv[2] = {};
    // rows 0 / 1: the sub-step with both queries counted separately (subtract them below)
    auto sub = [&](bool fresh) {
        Cnt s[11];
        for (int k = 0; k < 11; ++k) s[k] = s0[k];
        std::memset(&g, 0, sizeof g);
        substep<Cnt>(P, s, 0.3f, fresh, atm, false, false, fu, fv, LINE, LINE);
    };
    Ops q;
    {   // one line query alone (to subtract the sub-step's two)
        std::memset(&g, 0, sizeof g);
        (void)line_query<Cnt>(Cnt(3.0031), g_rec, 0.0, 10.0);
        q = g;
    }
    auto minus2 = [&](int row) {
        double* r = out + row * 14;
        const double v[14] = {q.add, q.mul, q.div, q.fma, q.sqrt, q.cmp, q.log, q.exp, q.sin, q.cos, q.atan2, q.hypot,
                              q.tanh, q.f32};
        for (int k = 0; k < 14; ++k) r[k] -= 2 * v[k];
    };
    sub(true); take(0); minus2(0);
    sub(false); take(1); minus2(1);
    { Cnt ug, vg; std::memset(&g, 0, sizeof g); wind_block<Cnt>(P, Cnt(20000.0), false, 0, 0, fu, fv, 1, 1.5, ug, vg); take(2); }
    {
        Cnt ug, vg, ug0, vg0;
        std::memset(&g, 0, sizeof g); wind_block<Cnt>(P, Cnt(9000.0), false, 0, 0, fu, fv, 1, 1.5, ug0, vg0);
        const Ops base = g;
        std::memset(&g, 0, sizeof g); wind_block<Cnt>(P, Cnt(9000.0), true, 0.3, -0.7, fu, fv, 1, 1.5, ug, vg);
        take(3);
        double* r = out + 3 * 14;
        const double v[14] = {base.add, base.mul, base.div, base.fma, base.sqrt, base.cmp, base.log, base.exp, base.sin,
                              base.cos, base.atan2, base.hypot, base.tanh, base.f32};
        for (int k = 0; k < 14; ++k) r[k] -= v[k];
    }
    // (query points inside their interval / sub-cell, so that every margin test runs)
    std::memset(&g, 0, sizeof g); (void)line_query<Cnt>(Cnt(3.0031), g_rec, 0.0, 10.0); take(4);
    std::memset(&g, 0, sizeof g); (void)piece_query<Cnt>(Cnt(3.0031), Cnt(2.5117), g_rec, 80.0, 0.0, 40.0, false); take(5);
    std::memset(&g, 0, sizeof g); (void)piece_query<Cnt>(Cnt(3.0031), Cnt(2.5117), g_rec, 80.0, 0.0, 40.0, true); take(6);
    std::memset(&g, 0, sizeof g); (void)payload_query<Cnt>(Cnt(3.0), Cnt(2.5), g_rec); take(7);
    {
        Cnt s[11], ring[10], obs[2];
        for (int k = 0; k < 11; ++k) s[k] = s0[k];
        for (int k = 0; k < 10; ++k) ring[k] = Cnt(0.1 * k);
        int len = 10, dn, tr;
        std::memset(&g, 0, sizeof g);
        (void)step_tail<Cnt>(P, s, Cnt(1000.0), ring, len, atm, dn, tr, obs);
        take(8);
    }
    { Cnt r, p, a; std::memset(&g, 0, sizeof g); atmosphere<Cnt>(P, Cnt(30000.0), r, p, a); take(9); }
}

}  // extern "C"
