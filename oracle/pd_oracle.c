/* pd_oracle.c -- scalar CPU restatement of the reference env (TEST INFRASTRUCTURE, see pd_oracle.h).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA contraction, like CPython).
 * Every function names the reference file:line it restates. */
#include "pd_oracle.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#define N_NB 50
#define N_SYS (N_NB + 3)

/* CPython math.radians / math.degrees (mathmodule.c: x * (pi/180), x * (180/pi)) */
static const double DEG2RAD = 3.141592653589793 / 180.0;
static const double RAD2DEG = 180.0 / 3.141592653589793;
static double radians(double x) { return x * DEG2RAD; }
static double degrees(double x) { return x * RAD2DEG; }
static const double PI = 3.141592653589793;

/* ---------------------------------------------------------------- atmosphere
 * atmosphere_dynamics.py:5-27 -> ambiance.Atmosphere (third-party, absent here; its
 * published ISA/US-1976 layer model restated: geopotential H = r h/(r+h), layer base
 * table, T = Tb + beta (H-Hb), p = pb (1+beta/Tb (H-Hb))^(-g0/(beta R)) or
 * pb exp(-g0/(R T) (H-Hb)), rho = p/(R T), a = sqrt(kappa R T)). */
void orc_atmosphere(const orc_params* P, double alt, double* rho, double* p, double* a) {
    if (alt < 0) alt = 0.0;
    if (alt < P->isa_alt_max) {
        double H = P->isa_r * alt / (P->isa_r + alt);
        int i = 0;
        for (int k = 0; k < 9; ++k) if (P->isa_Hb[k] <= H) i = k;  /* searchsorted(side=right)-1 */
        double Hb = P->isa_Hb[i], Tb = P->isa_Tb[i], b = P->isa_beta[i], pb = P->isa_pb[i];
        double T = Tb + b * (H - Hb);
        double pp;
        if (b != 0.0) pp = pb * pow(1.0 + b / Tb * (H - Hb), -P->isa_g0 / (b * P->isa_R));
        else pp = pb * exp(-P->isa_g0 / (P->isa_R * T) * (H - Hb));
        *p = pp;
        *rho = pp / (P->isa_R * T);
        *a = sqrt(P->isa_kappa * P->isa_R * T);
    } else {
        *rho = 0.0; *p = 0.0; *a = 0.0;
    }
}

/* atmosphere_dynamics.py:29-33 */
double orc_gravity(const orc_params* P, double alt) {
    double q = P->grav_R / (P->grav_R + alt);
    return P->grav_g0 * (q * q);
}

/* ---------------------------------------------------------------- RBF
 * scipy.interpolate.RBFInterpolator(points, coef, kernel='thin_plate_spline',
 * neighbors=50) as called by aerodynamic_coefficients.py:57-66: per query a 50-NN
 * search (euclidean, raw (Mach, AoA-deg) space), neighbourhood sorted by index,
 * 53x53 system [[K, P],[P^T, 0]] with K_ij = r^2 log r, P = [1, (y-shift)/scale],
 * shift = (min+max)/2, scale = (max-min)/2 (0 -> 1); solved by LU with partial pivoting
 * (LAPACK dgesv); value = sum phi(|x-y_j|) c_j + [1, xhat] . c_poly. */
static double tps(double r) { return r == 0.0 ? 0.0 : r * r * log(r); }

static int lu_solve(double* A, double* b, int n) {
    int piv[N_SYS];
    for (int k = 0; k < n; ++k) {
        int p = k; double best = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; ++i) { double v = fabs(A[i * n + k]); if (v > best) { best = v; p = i; } }
        if (best == 0.0) return -1;
        piv[k] = p;
        if (p != k) {
            for (int j = 0; j < n; ++j) { double t = A[k * n + j]; A[k * n + j] = A[p * n + j]; A[p * n + j] = t; }
            double t = b[k]; b[k] = b[p]; b[p] = t;
        }
        double r = 1.0 / A[k * n + k];
        for (int i = k + 1; i < n; ++i) {
            double l = A[i * n + k] * r;
            A[i * n + k] = l;
            if (l != 0.0) for (int j = k + 1; j < n; ++j) A[i * n + j] -= l * A[k * n + j];
            b[i] -= l * b[k];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int j = i + 1; j < n; ++j) s -= A[i * n + j] * b[j];
        b[i] = s / A[i * n + i];
    }
    (void)piv;
    return 0;
}

double orc_rbf(const orc_params* P, int which, double mach, double aoa) {
    const double *pm = which ? P->cl_m : P->cd_m, *pa = which ? P->cl_a : P->cd_a,
                 *pc = which ? P->cl_c : P->cd_c;
    int n = which ? P->cl_n : P->cd_n;
    /* 50 nearest: selection by (d2, index) */
    double bd[N_NB]; int bi[N_NB]; int cnt = 0;
    for (int i = 0; i < n; ++i) {
        double dm = mach - pm[i], da = aoa - pa[i];
        double d2 = dm * dm + da * da;
        if (cnt < N_NB || d2 < bd[cnt - 1]) {
            int pos = cnt < N_NB ? cnt : N_NB - 1;
            while (pos > 0 && bd[pos - 1] > d2) { if (pos < N_NB) { bd[pos] = bd[pos - 1]; bi[pos] = bi[pos - 1]; } --pos; }
            bd[pos] = d2; bi[pos] = i;
            if (cnt < N_NB) ++cnt;
        }
    }
    /* sort neighbour indices ascending (np.sort(yindices)) */
    for (int i = 1; i < N_NB; ++i) { int v = bi[i], j = i; while (j > 0 && bi[j - 1] > v) { bi[j] = bi[j - 1]; --j; } bi[j] = v; }
    double ym[N_NB], ya[N_NB], yd[N_NB];
    double mn0 = 1e300, mx0 = -1e300, mn1 = 1e300, mx1 = -1e300;
    for (int j = 0; j < N_NB; ++j) {
        ym[j] = pm[bi[j]]; ya[j] = pa[bi[j]]; yd[j] = pc[bi[j]];
        if (ym[j] < mn0) mn0 = ym[j]; if (ym[j] > mx0) mx0 = ym[j];
        if (ya[j] < mn1) mn1 = ya[j]; if (ya[j] > mx1) mx1 = ya[j];
    }
    double sh0 = (mx0 + mn0) / 2, sc0 = (mx0 - mn0) / 2, sh1 = (mx1 + mn1) / 2, sc1 = (mx1 - mn1) / 2;
    if (sc0 == 0.0) sc0 = 1.0;
    if (sc1 == 0.0) sc1 = 1.0;
    double A[N_SYS * N_SYS];
    double b[N_SYS];
    for (int i = 0; i < N_NB; ++i) {
        for (int j = 0; j < N_NB; ++j) {
            double d0 = ym[i] - ym[j], d1 = ya[i] - ya[j];
            A[i * N_SYS + j] = tps(sqrt(d0 * d0 + d1 * d1));
        }
        double h0 = (ym[i] - sh0) / sc0, h1 = (ya[i] - sh1) / sc1;
        A[i * N_SYS + N_NB] = 1.0; A[i * N_SYS + N_NB + 1] = h0; A[i * N_SYS + N_NB + 2] = h1;
        A[N_NB * N_SYS + i] = 1.0; A[(N_NB + 1) * N_SYS + i] = h0; A[(N_NB + 2) * N_SYS + i] = h1;
        b[i] = yd[i];
    }
    for (int i = N_NB; i < N_SYS; ++i) { for (int j = N_NB; j < N_SYS; ++j) A[i * N_SYS + j] = 0.0; b[i] = 0.0; }
    if (lu_solve(A, b, N_SYS) != 0) return NAN;
    double v = 0.0;
    for (int j = 0; j < N_NB; ++j) {
        double d0 = mach - ym[j], d1 = aoa - ya[j];
        v += tps(sqrt(d0 * d0 + d1 * d1)) * b[j];
    }
    v += 1.0 * b[N_NB];
    v += (mach - sh0) / sc0 * b[N_NB + 1];
    v += (aoa - sh1) / sc1 * b[N_NB + 2];
    return v;
}

/* rockets_physics.py:712 CD_func = rocket_CD(M, degrees(alpha)); aerodynamic_coefficients.py:105-115
 * (the clamp compares the DEGREE value against radians(10): bug kept) */
double orc_CD(const orc_params* P, double mach, double alpha_rad) {
    double aoa = degrees(alpha_rad);
    double r10 = radians(10.0);
    if (aoa > r10) return orc_rbf(P, 0, mach, r10);
    else if (aoa < radians(-10.0)) return orc_rbf(P, 0, mach, radians(-10.0));
    return orc_rbf(P, 0, mach, aoa);
}

/* rockets_physics.py:711 CL_func = rocket_CL(M, degrees(alpha)) and rocket_CL converts to
 * degrees AGAIN (aerodynamic_coefficients.py:117-132): a = deg(deg(alpha)) */
double orc_CL(const orc_params* P, double mach, double alpha_rad) {
    double a = degrees(degrees(alpha_rad));
    if (a > 10) return orc_rbf(P, 1, mach, 10.0);
    else if (a < -10) return orc_rbf(P, 1, mach, -10.0);
    else if (fabs(a) < 1e-6) return 0.0;
    else if (a < 0) return -orc_rbf(P, 1, mach, fabs(a));
    return orc_rbf(P, 1, mach, a);
}

/* ---------------------------------------------------------------- grid fins
 * grid_fin_aerodynamics.py:7-18: interp1d(kind='linear', fill_value='extrapolate')
 * -> scipy _call_linear: idx = searchsorted(x, M).clip(1, n-1) */
double orc_Ca(const orc_params* P, double mach) {
    if (mach < P->ca_min_mach) return P->ca_min_val;
    int n = P->ca_n, idx = 0;
    while (idx < n && P->ca_x[idx] < mach) ++idx;   /* searchsorted side='left' */
    if (idx < 1) idx = 1;
    if (idx > n - 1) idx = n - 1;
    double xl = P->ca_x[idx - 1], xh = P->ca_x[idx], yl = P->ca_y[idx - 1], yh = P->ca_y[idx];
    double slope = (yh - yl) / (xh - xl);
    return slope * (mach - xl) + yl;
}

/* np.interp (numpy compiled_base.c arr_interp) for one in-range query */
static double np_interp(const double* x, const double* y, int n, double v) {
    if (v < x[0]) return y[0];
    if (v > x[n - 1]) return y[n - 1];
    if (v == x[n - 1]) return y[n - 1];
    int j = 0;
    while (j + 1 < n && x[j + 1] <= v) ++j;
    if (x[j] == v) return y[j];
    double slope = (y[j + 1] - y[j]) / (x[j + 1] - x[j]);
    return slope * (v - x[j]) + y[j];
}

/* grid_fin_aerodynamics.py:21-46 */
double orc_Cn(const orc_params* P, double mach, double alpha_rad) {
    double ad = degrees(alpha_rad);
    double cna;
    if (mach < P->cn_min_mach) cna = P->cn_min_val;
    else if (mach <= P->cn_max_mach) cna = np_interp(P->cn_x, P->cn_y, P->cn_n, mach);
    else cna = P->cn_max_val + P->cn_slope * (mach - P->cn_max_mach);
    return cna * ad;
}

/* ---------------------------------------------------------------- mass properties
 * stage_inertia closure (rocket_dimensions.py:167-196), stage-2 constants */
void orc_inertia(const orc_params* P, double fill, double* x_cog, double* inertia) {
    double h_ox_t = P->h_ox * fill, h_f_t = P->h_f * fill, m_ox_t = P->m_ox * fill, m_f_t = P->m_f * fill;
    double x_prop = (m_ox_t * (P->h_lower + h_ox_t / 2) + m_f_t * (P->h_lower + P->h_ox + h_f_t / 2)) / (m_ox_t + m_f_t);
    double t1 = P->h_lower + h_ox_t / 2 - x_prop;
    double I_ox = 1.0 / 12 * m_ox_t * (h_ox_t * h_ox_t) + m_ox_t * (t1 * t1);
    double t2 = P->h_lower + P->h_ox + h_f_t / 2 - x_prop;
    double I_f = 1.0 / 12 * m_f_t * (h_f_t * h_f_t) + m_f_t * (t2 * t2);
    double I_prop = I_ox + I_f;
    double x_wet = (P->m_dry * P->x_dry + (m_ox_t + m_f_t) * x_prop) / (P->m_dry + m_ox_t + m_f_t);
    double t3 = P->x_dry - x_wet, t4 = x_prop - x_wet;
    double I_dry_hat = P->I_dry + P->m_dry * (t3 * t3);
    double I_prop_hat = I_prop + (m_ox_t + m_f_t) * (t4 * t4);
    *x_cog = x_wet;
    *inertia = I_dry_hat + I_prop_hat;
}

/* full_rocket_inertia closure (rocket_dimensions.py:198-241), the ascent phases'
 * x_cog_inertia_subrocket_0_lambda; restated with its own expression order (x_prop_1 uses the
 * untilded m_1_f and h_ox_1_tilde as written). */
static void orc_inertia_full(const orc_params* P, double fill, double* x_cog, double* inertia) {
    const double* c = P->fr;
    double x_wet2 = c[0], x_dry1 = c[1], m_s1 = c[2], m_pay = c[3], m_2 = c[4], m1_ox = c[5], m1_f = c[6];
    double h_lower1 = c[7], h1_ox = c[8], h1_f = c[9], h1 = c[10], I_wet2 = c[11], I_dry1 = c[12];
    double h_ox_t = h1_ox * fill, h_f_t = h1_f * fill, m_ox_t = m1_ox * fill, m_f_t = m1_f * fill;
    double m_prop_t = m_ox_t + m_f_t;
    double x_prop = (m_ox_t * (h_lower1 + h_ox_t / 2) + m1_f * (h_lower1 + h_ox_t + h_f_t / 2)) / (m_ox_t + m_f_t);
    double t1 = h_lower1 + h_ox_t / 2 - x_prop;
    double I_ox = 1.0 / 12 * m_ox_t * (h_ox_t * h_ox_t) + m_ox_t * (t1 * t1);
    double t2 = h_lower1 + h_ox_t + h_f_t / 2 - x_prop;
    double I_f = 1.0 / 12 * m_f_t * (h_f_t * h_f_t) + m_f_t * (t2 * t2);
    double I_prop = I_ox + I_f;
    double xr = (m_s1 * x_dry1 + (m_2 + m_pay) * (x_wet2 + h1) + m_prop_t * x_prop) / (m_s1 + m_2 + m_pay + m_prop_t);
    double a = x_dry1 - xr, b = x_wet2 - xr, d = x_prop - xr;
    *x_cog = xr;
    *inertia = I_dry1 + m_s1 * (a * a) + I_wet2 + m_2 * (b * b) + I_prop + m_prop_t * (d * d);
}

/* scipy interp1d(kind='linear', fill_value='extrapolate') -> _call_linear: lo/hi from
 * searchsorted(x, v) (side='left') clipped to [1, n-1] */
static double interp1d_ext(const double* x, const double* y, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) / 2; if (x[mid] < v) lo = mid + 1; else hi = mid; }
    int i = lo < 1 ? 1 : (lo > n - 1 ? n - 1 : lo);
    double slope = (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
    return slope * (v - x[i - 1]) + y[i - 1];
}

/* ---------------------------------------------------------------- ACS (acs_model.py:13-87) */
typedef struct { double f_perp, f_par, m_z, dcmd_l, dcmd_r, ca, cn_l; } acs_res;
static acs_res acs(const orc_params* P, double alpha_eff, double q, double mach, double x_cog,
                   double cmd_l_deg, double cmd_r_deg, double prev_l, double prev_r, double dt) {
    acs_res r;
    r.dcmd_l = radians(cmd_l_deg);   /* caller already multiplied by 60 (f32 or f64 path) */
    r.dcmd_r = radians(cmd_r_deg);
    double dl = prev_l + dt * ((-prev_l + r.dcmd_l) / 0.5);
    double dr = prev_r + dt * ((-prev_r + r.dcmd_r) / 0.5);
    double all = alpha_eff - dl, alr = alpha_eff - dr;
    double qS = q * P->S_gf;
    double Ca = orc_Ca(P, mach), CnL = orc_Cn(P, mach, all), CnR = orc_Cn(P, mach, alr);
    double cl = cos(dl), cr = cos(dr), sl = sin(dl), sr = sin(dr);
    r.f_perp = qS * (CnR * cr - CnL * cl - Ca * (sl - sr));
    r.f_par = qS * (Ca * (2 + cl + cr) - CnL * sl + CnR * sr);
    r.m_z = -(P->d_base_gf - x_cog) * r.f_perp + P->R_rocket * qS * (Ca * (sr - sl) - CnL * cl + CnR * cr);
    r.ca = Ca; r.cn_l = CnL;
    return r;
}

/* ---------------------------------------------------------------- wind (full_wind_model.py:35-43) */
static double wind_profile(const orc_params* P, const orc_env* E, double y) {
    /* HorizontalWindSpeed.py:58-68: interp1d(alt_km, speed, fill_value=(first,last)) of the
     * env's percentile (E->wind_prof) or of P's single profile */
    double km = y / 1000.0;
    const int w = E->wind_prof;
    const int n = w >= 0 ? P->wind_n_all[w] : P->wind_n;
    const double* xa = w >= 0 ? P->wind_alt_all[w] : P->wind_alt_km;
    const double* ya = w >= 0 ? P->wind_sp_all[w] : P->wind_speed;
    if (km < xa[0]) return ya[0];
    if (km > xa[n - 1]) return ya[n - 1];
    return np_interp(xa, ya, n, km);
}

/* The profile of percentile 50 + prof at altitude y (m): the interpolation wind_profile uses
 * (tests against HorizontalWindSpeed.compile_horizontal_fixed_wind) */
double orc_wind_at(const orc_params* P, int prof, double y) {
    orc_env E;
    memset(&E, 0, sizeof(E));
    E.wind_prof = prof;
    return wind_profile(P, &E, y);
}

/* ---------------------------------------------------------------- the device's random draws
 * Restatement of libpdenv's scheme (test infrastructure, so that a stochastic env can be
 * followed env for env): Philox4x32-10 (Salmon et al., SC'11; constants of the Random123
 * reference), 53-bit uniforms, Box-Muller with a cell-table log (512 cells, degree-5 log1p)
 * and fdlibm's sin/cos kernels -- IEEE +, *, fma, sqrt and rint only, so the draws are the
 * device's bit for bit. */
orc_u32x4 orc_philox(orc_u32x4 c, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        orc_u32x4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c;
}
double orc_u01(uint32_t hi, uint32_t lo) {
    return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6)) * (1.0 / 9007199254740992.0);
}
#define ORC_LOG_CELLS 512
static double g_invc[ORC_LOG_CELLS], g_logc[ORC_LOG_CELLS];
static pthread_once_t g_log_once = PTHREAD_ONCE_INIT;
static void log_cells_fill(void) {
    for (int i = 0; i < ORC_LOG_CELLS; ++i) {
        long double c = 1.0L + (i + 0.5L) / ORC_LOG_CELLS;
        double invc = (double)(1.0L / c);
        g_invc[i] = invc;
        g_logc[i] = (double)(-logl((long double)invc));
    }
}
static double log_cells(double x) {
    uint64_t b;
    memcpy(&b, &x, 8);
    uint32_t hi = (uint32_t)(b >> 32);
    double e = (double)((int)(hi >> 20) - 1023);
    uint32_t i = (hi >> (20 - 9)) & (ORC_LOG_CELLS - 1);
    uint64_t mb = (b & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m;
    memcpy(&m, &mb, 8);
    double r = fma(m, g_invc[i], -1.0);
    double t = fma(r, 0.2, -0.25);
    t = fma(r, t, 1.0 / 3.0);
    t = fma(r, t, -0.5);
    double p = fma(r * r, t, r);
    return fma(e, 6.93147180559945286227e-01, g_logc[i] + p);
}
static void sincos_fd(double x, double* s, double* c) {
    if (!(fabs(x) < 1.0e6)) { *s = sin(x); *c = cos(x); return; }
    const double k = rint(x * 6.36619772367581382433e-01);
    const double r1 = fma(-k, 1.57079632679489655800e+00, x);
    const double ph = k * 6.12323399573676603587e-17;
    const double pl = fma(k, 6.12323399573676603587e-17, -ph) + k * -1.4973849048591698e-33;
    const double r = r1 - ph;
    const double y = ((r1 - r) - ph) - pl;
    const double z = r * r, v = z * r, w = z * z;
    const double ps = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * (2.75573137070700676789e-06 +
                      z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    const double sn = r - ((z * (0.5 * y - v * ps) - y) - v * -1.66666666666666324348e-01);
    const double pc = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * 2.48015872894767294178e-05)) +
                      w * w * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11));
    const double hz = 0.5 * z, ww = 1.0 - hz;
    const double cs = ww + (((1.0 - ww) - hz) + (z * pc - r * y));
    const int q = (int)(long long)k & 3;
    *s = q == 0 ? sn : (q == 1 ? cs : (q == 2 ? -sn : -cs));
    *c = q == 0 ? cs : (q == 1 ? -sn : (q == 2 ? -cs : sn));
}
void orc_gauss_pair(orc_u32x4 r, double* z0, double* z1) {
    pthread_once(&g_log_once, log_cells_fill);
    const double u1 = 1.0 - orc_u01(r.x, r.y), u2 = orc_u01(r.z, r.w);
    const double rho = sqrt(-2.0 * log_cells(u1));
    double s, c;
    sincos_fd(6.283185307179586 * u2, &s, &c);
    *z0 = rho * c;
    *z1 = rho * s;
}
enum { ORC_TAG_WIND_SUB = 0, ORC_TAG_RESET = 16, ORC_TAG_TILT = 17, ORC_TAG_PROF = 18 };

static void vk_step(const double* Ad, const double* Bd, double sigma, double* s, double w) {
    /* vonkarman.py:33-36: state = Ad @ state + Bd * w, Bd = sigma * Bd(sigma=1) */
    double n0 = (Ad[0] * s[0] + Ad[1] * s[1]) + (sigma * Bd[0]) * w;
    double n1 = (Ad[2] * s[0] + Ad[3] * s[1]) + (sigma * Bd[1]) * w;
    s[0] = n0; s[1] = n1;
}

/* ---------------------------------------------------------------- one physics sub-step
 * rocket_physics_fcn (rockets_physics.py:455-704) with the landing-burn control laws
 * force_moment_decomposer_landing_burn_throttle_only (:340-400) and
 * force_moment_decomposer_landing_burn_gimballed (:168-269). */
/* One rocket_physics_fcn call (rockets_physics.py:455-704).  kout == NULL: the reference's
 * semi-implicit Euler update of E->s at dt.  kout != NULL (the non-parity RK4 mode): E->s is left
 * alone and kout receives d/dt of (x, y, vx, vy, theta, theta_dot, mass, mass_propellant). */
/* Analysis hook (tools/regime_persistence.py; nothing on the parity path reads it): when a log
 * is set, each Euler sub-step of orc_rollout_philox records which table path its two queries
 * take: 1 = the clamped lines (|degrees(alpha_eff)| > radians(10), both tables clamp), 2 = the
 * interior grids, 0 = no query (a == 0). */
static uint8_t* g_qlog;
static __thread uint8_t* g_qlog_step;
void orc_set_qlog(uint8_t* buf) { g_qlog = buf; }

static void substep(const orc_params* P, orc_env* E, int phase, const double* u, int f32,
                    double dt, double dt_act, const double* noise2, double* info, double* kout) {
    double* s = E->s;
    double x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], thd = s[5], ga = s[6], al = s[7];
    double m = s[8], mp = s[9], t = s[10];
    double rho, patm, a;
    orc_atmosphere(P, y, &rho, &patm, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double mach = 0.0;
    if (a != 0.0) { double mr = speed / a; mach = (10.0 < mr) ? 10.0 : mr; }   /* min(speed/a, 10.0) */
    double q = 0.5 * rho * (speed * speed);
    double fpc = (P->m_prop0 - mp) / P->m_prop0;
    if (fpc == 0.0) fpc = 1e-6;
    double x_cog, inertia;
    const int ascent = phase == ORC_PHASE_SUBSONIC || phase == ORC_PHASE_SUPERSONIC;
    /* subrocket_0 closures for the ascent, subrocket_2 for everything after (:748-750, :772-774) */
    if (ascent) orc_inertia_full(P, 1 - fpc, &x_cog, &inertia);
    else orc_inertia(P, 1 - fpc, &x_cog, &inertia);
    double d_thrust = x_cog + P->engine_height;
    double ae = (vy < 0) ? ga - th - PI : al;
    double d_cp_cg = x_cog - (ascent ? P->cop_ascent : P->cop);
    if (g_qlog_step && !kout && E->cur_sub >= 0 && E->cur_sub < 4)
        g_qlog_step[E->cur_sub] = a == 0.0 ? 0 : (fabs(degrees(ae)) > radians(10.0) ? 1 : 2);
    double ug = 0.0, vg = 0.0;
    if (E->wind_on) {
        ug = wind_profile(P, E, y);
        if (y < P->vk_y_threshold && E->wind_stoch) {
            /* vonkarman.py:34: one np.random.randn() per filter step, u first then v */
            double w0 = 0.0, w1 = 0.0;
            if (noise2) {
                int off = E->noise_slotted ? 0 : E->noise_used;
                w0 = noise2[off]; w1 = noise2[off + 1];
            } else if (E->rng_philox) {
                orc_u32x4 c = {(uint32_t)E->rng_g, (uint32_t)(E->rng_g >> 32) ^ E->rng_ep, E->rng_ts,
                               ORC_TAG_WIND_SUB + (uint32_t)E->cur_sub};
                orc_gauss_pair(orc_philox(c, E->seed_lo, E->seed_hi), &w0, &w1);
            }
            E->noise_used += 2;
            vk_step(P->vk_Ad_u, P->vk_Bd_u, E->sigma_u, E->fu, w0);
            vk_step(P->vk_Ad_v, P->vk_Bd_v, E->sigma_v, E->fv, w1);
            ug = ug + E->fu[1];
            vg = E->fv[1];
        }
    }
    double Fwx = 0.5 * rho * (ug * ug) * P->A_front * P->C_gust_x;
    double Fwy = 0.5 * rho * (vg * vg) * P->A_front * P->C_gust_y;
    double Mw = -d_cp_cg * Fwy;
    double CL = 0.0, CD = 0.0;
    if (a != 0.0) { CL = orc_CL(P, mach, ae); CD = orc_CD(P, mach, ae); }
    double drag = 0.5 * rho * (speed * speed) * CD * P->A_front;
    double lift = 0.5 * rho * (speed * speed) * CL * P->A_front;
    double apar, aperp;
    if (vy >= 0.0) { apar = lift * sin(ae) - drag * cos(ae); aperp = -lift * cos(ae) - drag * sin(ae); }
    else { apar = drag * cos(ae) - lift * sin(ae); aperp = -drag * sin(ae) - lift * cos(ae); }
    double aero_x = apar * cos(th) + aperp * sin(th);
    double aero_y = apar * sin(th) - aperp * cos(th);
    double aero_m = aperp * d_cp_cg;

    double T_full = P->T_e + (P->p_e - patm) * P->A_e;
    double cfp, cfperp, cm, mdot_dt, mdot_info, throttle_info, gimbal_deg_out = 0.0;
    /* binary32 control forces (ascent with float32 actions): the force sums below then run in
     * binary32 too, because the aerodynamic terms are Python floats (weak under NEP 50) */
    int f32_forces = 0;
    float cfp_f = 0.0f, cfperp_f = 0.0f;
    acs_res ac;
    memset(&ac, 0, sizeof(ac));
    if (phase == ORC_PHASE_FLIP) {
        /* flip-over aero is zeroed after the coefficients are computed (:548-551) */
        aero_x = 0.0; aero_y = 0.0; aero_m = 0.0;
    }
    if (phase == ORC_PHASE_PCONTROL) {
        /* force_moment_decomposer_landing_burn_throttle_PID (:402-451): Kp -0.08 on v_ref - speed,
         * clip to [0, 1], handed to throttle_only as a list -> u0 = float(...) (binary64 onward) */
        double u0;
        if (f32) {
            float err = (float)u[0] - (float)speed;
            float nt = err * (float)(-0.08);
            nt = nt < 0.0f ? 0.0f : (nt > 1.0f ? 1.0f : nt);
            u0 = (double)(2.0f * (nt - 0.5f));
        } else {
            double nt = (u[0] - speed) * -0.08;
            nt = nt < 0.0 ? 0.0 : (nt > 1.0 ? 1.0 : nt);
            u0 = 2 * (nt - 0.5);
        }
        const double nominal = (0 * 0.4) / (double)P->n_eng;
        double thr = (u0 + 1) / 2 * (1 - nominal) + nominal;
        double tg = T_full * P->n_eng * thr;
        double md = (P->T_e / P->v_ex) * (tg / T_full);
        ac = acs(P, ae, q, mach, x_cog, 0.0, 0.0, 0.0, 0.0, dt_act);
        cfp = tg + ac.f_par; cfperp = ac.f_perp; cm = ac.m_z;
        mdot_dt = md * dt; mdot_info = md; throttle_info = thr;
    } else if (phase == ORC_PHASE_BALLISTIC) {
        /* RCS (:149-166): thruster force = max * action (array), moment promoted to binary64 by
         * the float64 x_cog; no forces, no mass flow */
        double tf = f32 ? (double)((float)P->rcs_force * (float)u[0]) : P->rcs_force * u[0];
        cfp = 0.0; cfperp = 0.0;
        cm = -tf * (x_cog - P->rcs_d_bottom) + tf * (P->rcs_d_top - x_cog);
        mdot_dt = 0.0; mdot_info = 0.0; throttle_info = 0.0;
    } else if (phase == ORC_PHASE_FLIP) {
        /* force_moment_decomposer_flipoverboostbackburn (:63-92): low-pass of the gimbal command
         * (tau 1, dt = physics dt), all 16 gimballed engines at full throttle.  The filtered
         * angle is the action's dtype (float32 array with float32 actions). */
        double gd;
        if (f32) {
            float cmd = (float)u[0] * 10.0f, x0 = (float)E->gimbal_prev;
            gd = (double)(x0 + (float)dt * ((-x0 + cmd) / 1.0f));
        } else {
            double cmd = u[0] * 10;
            gd = E->gimbal_prev + dt * ((-E->gimbal_prev + cmd) / 1.0);
        }
        double grad = radians(gd);
        double tg = T_full * P->n_eng * 1;
        double tpar = tg * cos(grad), tperp = -tg * sin(grad);
        cfp = tpar; cfperp = tperp; cm = -tg * sin(grad) * d_thrust;
        double md = (P->T_e / P->v_ex) * (sqrt(tpar * tpar + tperp * tperp) / T_full);
        mdot_dt = md * dt; mdot_info = md; throttle_info = 1.0;
        gimbal_deg_out = gd;
        E->gimbal_prev = gd;   /* base_environment.py:110 */
    } else if (ascent) {
        /* force_moment_decomposer_ascent (:17-56): 16 gimballed + 26 fixed engines, nominal 0.5,
         * gimbal radians(7) */
        const int ng = P->n_eng, nng = P->n_eng_stage1 - P->n_eng;
        const double mg = radians(7.0);
        if (f32) {
            float grad = (float)u[0] * (float)mg;
            float nnt = ((float)u[1] + 1.0f) / 2.0f;
            float thr = nnt * (float)(1 - 0.5) + (float)0.5;
            float tg = (float)(T_full * ng) * thr, tng = (float)(T_full * nng) * thr;
            float cg = (float)cos((double)grad), sg = (float)sin((double)grad);
            float tpar = tng + tg * cg;
            float tperp = (-tg) * sg;
            float tot = sqrtf(tpar * tpar + tperp * tperp);
            float md = (float)(P->T_e / P->v_ex) * (tot / (float)T_full);
            cfp_f = tpar; cfperp_f = tperp; f32_forces = 1;
            cfp = tpar; cfperp = tperp; cm = (double)((-tg) * sg) * d_thrust;
            mdot_dt = (double)(md * (float)dt); mdot_info = md; throttle_info = thr;
            gimbal_deg_out = degrees((double)grad);
        } else {
            double grad = u[0] * mg;
            double thr = (u[1] + 1) / 2 * (1 - 0.5) + 0.5;
            double tg = T_full * ng * thr, tng = T_full * nng * thr;
            double tpar = tng + tg * cos(grad), tperp = -tg * sin(grad);
            cfp = tpar; cfperp = tperp; cm = -tg * sin(grad) * d_thrust;
            double md = (P->T_e / P->v_ex) * (sqrt(tpar * tpar + tperp * tperp) / T_full);
            mdot_dt = md * dt; mdot_info = md; throttle_info = thr;
            gimbal_deg_out = degrees(grad);
        }
    } else if (phase == ORC_PHASE_PURE_THROTTLE) {
        const double nominal = (0 * 0.4) / (double)P->n_eng;
        if (f32) {
            float u0 = (float)u[0];
            float nnt = (u0 + 1.0f) / 2.0f;
            float thr = nnt * (float)(1 - nominal) + (float)nominal;
            float tg = (float)(T_full * P->n_eng) * thr;
            float ntot = tg / (float)T_full;
            float md = (float)(P->T_e / P->v_ex) * ntot;
            ac = acs(P, ae, q, mach, x_cog, 0.0, 0.0, 0.0, 0.0, dt_act);
            cfp = (double)tg + ac.f_par;
            cfperp = ac.f_perp; cm = ac.m_z;
            mdot_dt = (double)(md * (float)dt);
            mdot_info = md; throttle_info = thr;
        } else {
            double u0 = u[0];
            double nnt = (u0 + 1) / 2;
            double thr = nnt * (1 - nominal) + nominal;
            double tg = T_full * P->n_eng * thr;
            double ntot = tg / T_full;
            double md = (P->T_e / P->v_ex) * ntot;
            ac = acs(P, ae, q, mach, x_cog, 0.0, 0.0, 0.0, 0.0, dt_act);
            cfp = tg + ac.f_par; cfperp = ac.f_perp; cm = ac.m_z;
            mdot_dt = md * dt; mdot_info = md; throttle_info = thr;
        }
    } else {
        /* landing_burn: 18 gimballed engines, nominal 3*0.4/16, gimbal 5 deg, fins radians(20) */
        const int n_eng = P->n_eng + 2;
        const double nominal = (3 * 0.4) / (double)P->n_eng;
        const double max_gimbal_rad = radians(5.0), max_defl = radians(20.0);
        const double max_gimbal_deg = degrees(max_gimbal_rad);
        double gdeg_cmd, thr_d, tg_d, tpar, tperp, mz, md_d, cmd_l, cmd_r;
        float thr_f = 0.0f, md_f = 0.0f;
        if (f32) {
            float u0 = (float)u[0], u1 = (float)u[1], u2 = (float)u[2], u3 = (float)u[3];
            float grad = u0 * (float)max_gimbal_rad;
            gdeg_cmd = degrees((double)grad);
            double gd = E->gimbal_prev + dt_act * ((-E->gimbal_prev + gdeg_cmd) / 1.0);
            if (gd < -max_gimbal_deg) gd = -max_gimbal_deg;
            if (gd > max_gimbal_deg) gd = max_gimbal_deg;
            double grad2 = radians(gd);
            float nnt = (u1 + 1.0f) / 2.0f;
            thr_f = nnt * (float)(1 - nominal) + (float)nominal;
            float tg = (float)(T_full * n_eng) * thr_f;
            float fpar = tg * (float)cos(grad2);
            float fperp = (-tg) * (float)sin(grad2);
            /* (-T sin d) * d_thrust_cg: d_thrust_cg is np.float64 (x_cog derives from the
             * np.float64 state), so this last product promotes to binary64 */
            float fm = (-tg) * (float)sin(grad2);
            float tot = sqrtf(fpar * fpar + fperp * fperp);
            float ntot = tot / (float)T_full;
            md_f = (float)(P->T_e / P->v_ex) * ntot;
            gimbal_deg_out = degrees(grad2);
            float dl = u2 * (float)max_defl, dr = u3 * (float)max_defl;
            cmd_l = (double)(dl * (float)60); cmd_r = (double)(dr * (float)60);
            tpar = fpar; tperp = fperp; mz = (double)fm * d_thrust;
            thr_d = thr_f; md_d = md_f; (void)tg_d;
        } else {
            double grad = u[0] * max_gimbal_rad;
            gdeg_cmd = degrees(grad);
            double gd = E->gimbal_prev + dt_act * ((-E->gimbal_prev + gdeg_cmd) / 1.0);
            if (gd < -max_gimbal_deg) gd = -max_gimbal_deg;
            if (gd > max_gimbal_deg) gd = max_gimbal_deg;
            double grad2 = radians(gd);
            double nnt = (u[1] + 1) / 2;
            thr_d = nnt * (1 - nominal) + nominal;
            tg_d = T_full * n_eng * thr_d;
            tpar = tg_d * cos(grad2);
            tperp = -tg_d * sin(grad2);
            mz = -tg_d * sin(grad2) * d_thrust;
            double tot = sqrt(tpar * tpar + tperp * tperp);
            md_d = (P->T_e / P->v_ex) * (tot / T_full);
            gimbal_deg_out = degrees(grad2);
            cmd_l = u[2] * max_defl * 60; cmd_r = u[3] * max_defl * 60;
        }
        ac = acs(P, ae, q, mach, x_cog, cmd_l, cmd_r, E->dl_prev, E->dr_prev, dt_act);
        cfp = tpar + ac.f_par; cfperp = tperp + ac.f_perp; cm = mz + ac.m_z;
        if (f32) mdot_dt = (double)(md_f * (float)dt); else mdot_dt = md_d * dt;
        mdot_info = md_d; throttle_info = thr_d;
    }
    /* NaN guard (rockets_physics.py:599-607): an elif chain */
    if (isnan(cfp)) cfp = 0.0;
    else if (isnan(cfperp)) cfperp = 0.0;
    else if (isnan(cm)) cm = 0.0;
    double cfx, cfy, fx, fy;
    double g = orc_gravity(P, y);
    if (f32_forces) {
        /* rockets_physics.py:608-616 with float32 control forces: cfx, cfy in binary32; the
         * Python-float aero terms and F_wind_y join in binary32; with wind on F_wind_x is a numpy
         * float64 (interp1d output) and promotes the last sum */
        if (isnan(cfp_f)) cfp_f = 0.0f;
        else if (isnan(cfperp_f)) cfperp_f = 0.0f;
        float c = (float)cos(th), sn = (float)sin(th);
        float cx = cfp_f * c + cfperp_f * sn;
        float cy = cfp_f * sn - cfperp_f * c;
        float sx = (float)aero_x + cx, sy = (float)aero_y + cy;
        fx = E->wind_on ? (double)sx + Fwx : (double)(sx + (float)Fwx);
        fy = (double)(sy + (float)Fwy);
        cfx = cx; cfy = cy;
    } else {
        cfx = cfp * cos(th) + cfperp * sin(th);
        cfy = cfp * sin(th) - cfperp * cos(th);
        fx = aero_x + cfx + Fwx; fy = aero_y + cfy + Fwy;
    }
    double vxd = fx / m, vyd = fy / m - g;
    double mz_tot = cm + aero_m + Mw;
    double thdd = mz_tot / inertia;
    if (kout) {
        kout[0] = vx; kout[1] = vy; kout[2] = vxd; kout[3] = vyd; kout[4] = thd; kout[5] = thdd;
        kout[6] = -mdot_info; kout[7] = -mdot_info;
    }
    if (info) {
        info[ORC_I_RHO] = rho; info[ORC_I_P] = patm; info[ORC_I_A] = a; info[ORC_I_MACH] = mach;
        info[ORC_I_Q] = q; info[ORC_I_CL] = CL; info[ORC_I_CD] = CD; info[ORC_I_MDOT] = mdot_info;
        info[ORC_I_XCOG] = x_cog; info[ORC_I_INERTIA] = inertia; info[ORC_I_DTHRUST] = d_thrust;
        info[ORC_I_ALPHA_EFF] = ae; info[ORC_I_THROTTLE] = throttle_info; info[ORC_I_CFPAR] = cfp;
        info[ORC_I_CFPERP] = cfperp; info[ORC_I_CM] = cm; info[ORC_I_AERO_X] = aero_x; info[ORC_I_AERO_Y] = aero_y;
        info[ORC_I_UG] = ug; info[ORC_I_VG] = vg; info[ORC_I_CA] = ac.ca; info[ORC_I_CNL] = ac.cn_l;
        info[ORC_I_GIMBAL_DEG] = gimbal_deg_out; info[ORC_I_DCMD_L] = ac.dcmd_l; info[ORC_I_DCMD_R] = ac.dcmd_r;
        info[ORC_I_DRAG] = drag; info[ORC_I_LIFT] = lift;
    }
    if (kout) return;
    vx += vxd * dt; vy += vyd * dt; x += vx * dt; y += vy * dt;
    thd += thdd * dt; th += thd * dt;
    ga = atan2(vy, vx);
    if (th > 2 * PI) th -= 2 * PI;
    if (ga < 0) ga = 2 * PI + ga;
    al = th - ga;
    mp -= mdot_dt; m -= mdot_dt; t += dt;
    s[0] = x; s[1] = y; s[2] = vx; s[3] = vy; s[4] = th; s[5] = thd; s[6] = ga; s[7] = al;
    s[8] = m; s[9] = mp; s[10] = t;
}

int orc_physics(const orc_params* P, orc_env* E, int phase, const double* u, int f32,
                const double* noise, double* info) {
    /* compile_physics: pure throttle dt_temp = 0.025 x4 (rockets_physics.py:909-957);
     * landing_burn physics dt = 0.1 x4 with actuator dt 0.025 (:803-861) */
    double dt = phase == ORC_PHASE_PURE_THROTTLE ? 0.025 : 0.1;
    E->noise_used = 0;
    if (E->integrator == ORC_INTEG_RK4) {
        /* NOT the reference's integrator: BASELINE config c2's "RK4 dt=0.01 s" (SURVEY 8(d) c2),
         * classical RK4 over (x, y, vx, vy, theta, theta_dot, mass, mass_propellant) with the
         * forces of rocket_physics_fcn at each stage, 10 x 0.01 s per 0.1 s env step; gamma and
         * alpha follow the stage velocity (gamma = atan2(vy, vx) in [0, 2 pi), alpha = theta -
         * gamma), theta wrapped once per 0.01 s.  Pure throttle without wind only.  libpdenv's
         * k_step<..., RK4> runs the same operations in the same order. */
        if (phase != ORC_PHASE_PURE_THROTTLE || E->wind_on) return -1;
        static const int idx[8] = {0, 1, 2, 3, 4, 5, 8, 9};
        /* h: 0.01 s; E->dt > 0 overrides it (convergence tests), 0.1 / h steps */
        const double h = E->dt > 0 ? E->dt : 0.01;
        const int n_rk = (int)llround(0.1 / h);
        double* s = E->s;
        for (int n = 0; n < n_rk; ++n) {
            double b[8], acc[8], k[8];
            for (int i = 0; i < 8; ++i) b[i] = s[idx[i]];
            for (int st = 0; st < 4; ++st) {
                E->cur_sub = 4 * n + st;
                substep(P, E, phase, u, f32, h, 0.025, NULL, info, k);
                for (int i = 0; i < 8; ++i)
                    acc[i] = st == 0 ? k[i] : (st == 3 ? acc[i] + k[i] : acc[i] + 2.0 * k[i]);
                if (st < 3) {
                    const double c = st == 2 ? h : 0.5 * h;
                    for (int i = 0; i < 8; ++i) s[idx[i]] = b[i] + c * k[i];
                } else {
                    for (int i = 0; i < 8; ++i) s[idx[i]] = b[i] + (h / 6.0) * acc[i];
                    if (s[4] > 2 * PI) s[4] -= 2 * PI;
                    s[10] += h;
                }
                double ga = atan2(s[3], s[2]);
                if (ga < 0) ga = 2 * PI + ga;
                s[6] = ga; s[7] = s[4] - ga;
            }
        }
        return 0;
    }
    if (phase >= ORC_PHASE_PCONTROL) {
        /* the other phases: one call of rocket_physics_fcn at the env dt (:728-802, :959-997);
         * actuator filters at the same dt */
        double d = E->dt > 0 ? E->dt : 0.1;
        E->cur_sub = 0;
        substep(P, E, phase, u, f32, d, d, noise, info, NULL);
        return 0;
    }
    for (int k = 0; k < 4; ++k) {
        E->cur_sub = k;
        substep(P, E, phase, u, f32, dt, 0.025, noise ? (E->noise_slotted ? noise + 2 * k : noise) : NULL, info, NULL);
    }
    if (phase == ORC_PHASE_LANDING_BURN && info) {
        /* base_environment.py:122-124: prevs <- filtered gimbal, fin COMMANDS */
        E->gimbal_prev = info[ORC_I_GIMBAL_DEG];
        E->dl_prev = info[ORC_I_DCMD_L];
        E->dr_prev = info[ORC_I_DCMD_R];
    }
    return 0;
}

void orc_reset(const orc_params* P, orc_env* E, const double* s0, int wind_on, int wind_stoch,
               double sigma_u, double sigma_v) {
    memset(E, 0, sizeof(*E));
    memcpy(E->s, s0 ? s0 : P->state0, sizeof(E->s));
    memcpy(E->prev_s, E->s, sizeof(E->s));
    E->wind_on = wind_on; E->wind_stoch = wind_stoch; E->sigma_u = sigma_u; E->sigma_v = sigma_v;
    E->wind_prof = -1;
}

/* base_environment.py:80-97 with the device's draws (libpdenv reset_values): the phase's initial
 * state, pitch tilt N(0, tilt) (theta += tilt z, alpha = theta - gamma; tag ORC_TAG_TILT),
 * sigma_u ~ U(0.5, 2.25) and sigma_v ~ U(1.25, 2.0) (vonkarman.py:60-66; tag ORC_TAG_RESET) and
 * the percentile randint(50, 99) (full_wind_model.py:27-33; tag ORC_TAG_PROF) unless fixed --
 * three independent draws, as the reference's three np.random calls are. */
void orc_reset_philox(const orc_params* P, orc_env* E, int phase, uint64_t seed, uint64_t g,
                      uint32_t episode, int wind_on, int wind_stoch, int fixed_prof, double tilt) {
    double s0[11];
    memcpy(s0, P->state0_ph[phase], sizeof(s0));
    const uint32_t klo = (uint32_t)seed, khi = (uint32_t)(seed >> 32);
    if (tilt > 0) {
        orc_u32x4 c = {(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, ORC_TAG_TILT};
        double z0, z1;
        orc_gauss_pair(orc_philox(c, klo, khi), &z0, &z1);
        s0[4] = s0[4] + tilt * z0;
        s0[7] = s0[4] - s0[6];
    }
    orc_u32x4 c = {(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, ORC_TAG_RESET};
    orc_u32x4 r = orc_philox(c, klo, khi);
    const double su = 0.5 + (2.25 - 0.5) * orc_u01(r.x, r.y);
    const double sv = 1.25 + (2.0 - 1.25) * orc_u01(r.z, r.w);
    orc_reset(P, E, s0, wind_on, wind_stoch, su, sv);
    E->wind_prof = -1;
    if (wind_on && fixed_prof >= 0) E->wind_prof = fixed_prof;
    else if (wind_on) {
        /* the percentile's own draw (tag ORC_TAG_PROF): floor(49 u / 2^32), u one Philox word */
        orc_u32x4 cp = {(uint32_t)g, (uint32_t)(g >> 32) ^ episode, 0u, ORC_TAG_PROF};
        E->wind_prof = (int)(((uint64_t)orc_philox(cp, klo, khi).x * 49u) >> 32);
    }
    E->rng_philox = 1;
    E->rng_g = g; E->rng_ep = episode; E->rng_ts = 0;
    E->seed_lo = klo; E->seed_hi = khi;
}

/* ---------------------------------------------------------------- rtd */
static void rtd_rl_pure_throttle(const orc_params* P, const orc_env* E, double gl, orc_out* o) {
    /* rtd_rl.py:190-336 */
    const double* s = E->s;
    double x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], mp = s[9];
    (void)x;
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double q = 0.5 * rho * (speed * speed);
    int tr = 0, id = 0;
    if (y < -10) { tr = 1; id = 1; }
    else if (mp <= 0) { tr = 1; id = 2; }
    else if (th > PI + radians(2)) { tr = 1; id = 3; }
    else if (q > 65000) { tr = 1; id = 4; }
    else if (gl > 6.0) { tr = 1; id = 5; }
    else if (vy > 0.0) { tr = 1; id = 6; }
    else if (vx > 0.01) { tr = 1; id = 7; }
    int done = (y > 0 && y < 1 && speed < 5.0);
    double y0 = P->state0[1], m0 = P->state0[8];
    double sp = hypot(vx, vy);          /* reward_func uses math.hypot (rtd_rl.py:292) */
    double qr = 0.5 * rho * (sp * sp);
    double r = 0.0;
    if (qr > 60000.0) { double e = (qr - 60000.0) / (65000.0 - 60000.0); r -= 1.0 * fmin(e * e, 1.0); }
    if (gl > 5.5) { double e = (gl - 5.5) / (6.0 - 5.5); r -= 1.0 * fmin(e * e, 1.0); }
    double prog = (y0 - y) / y0;
    double wp = (qr <= 60000.0 && gl <= 5.5) ? 0.5 : 0.5 * 0.1;
    r += wp * prog;
    if (y < 100.0) r += 5.5 * (1.0 - fabs(vy) / 50.0);
    if (done && !tr) r += 400.0 * mp / m0;
    else if (tr && y > 0) r -= 50.0 * (fabs(y) / y0);
    else if (tr && y < 0) r -= 50.0 * (fabs(vy) / 10);
    if (!done || !(tr && y < 0)) { if (r < -10.0) r = -10.0; if (r > 10.0) r = 10.0; }
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}

static void rtd_pso(const orc_params* P, const orc_env* E, int phase, double gl, orc_out* o) {
    const double* s = E->s;
    double x = s[0], y = s[1], vx = s[2], vy = s[3], th = s[4], ga = s[6], mp = s[9];
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double q = 0.5 * rho * (speed * speed);
    int tr = 0, id = 0, done = 0;
    double r = 0.0;
    if (phase == ORC_PHASE_PURE_THROTTLE) {   /* rtd_pso.py:172-230 */
        if (y < 0.0) { tr = 1; id = 1; }
        else if (mp <= 0) { tr = 1; id = 2; }
        else if (th > PI + radians(2)) { tr = 1; id = 3; }
        else if (q > 65000) { tr = 1; id = 4; }
        else if (vy > 0.0) { tr = 1; id = 6; }
        else if (gl > 6.0) { tr = 1; id = 7; }
        done = (y > 0 && y < 1 && speed < 5.5);
        if (tr && y > 0) r = -fabs(y);
        else if (tr && y < 0) r = 200 - fabs(speed);
        else if (done) r = mp;
    } else {                                   /* rtd_pso.py:234-317 */
        double dist = sqrt(x * x + y * y);
        double over;
        if (x < 0 && y < 0) over = sqrt(x * x + y * y);
        else if (x < 0) over = -x;
        else if (y < 0) over = -y;
        else over = 0;
        double aeff = (vy < 0) ? fabs(ga - th - PI) : fabs(th - ga);
        if (over > 0.5) { tr = 1; id = 1; }
        else if (mp <= 0) { tr = 1; id = 2; }
        else if (aeff > radians(10)) { tr = 1; id = 3; }
        else if (q > 65000) { tr = 1; id = 4; }
        else if (vy > 0.0) { tr = 1; id = 6; }
        else if (gl > 6.0) { tr = 1; id = 7; }
        else if (y > 1000 && vx > 0.0) { tr = 1; id = 8; }
        done = (dist > 0 && dist < 1 && speed < 2.5);
        if (tr && over < 0.5) r = -fabs(dist);
        else if (tr) r = 200 - fabs(speed);
        else if (done) r = mp;
    }
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}


/* rtd_rl.py:190-240 (truncated/done shared by both landing-burn RL flavours) + :243-269 (the
 * reward of landing_burn / landing_burn_ACS).  u0 = actions[0] as the env receives it. */
static void rtd_rl_landing_burn(const orc_params* P, const orc_env* E, double gl, const double* u, int f32,
                                orc_out* o) {
    const double* s = E->s;
    double y = s[1], vx = s[2], vy = s[3], th = s[4], ga = s[6], mp = s[9];
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double q = 0.5 * rho * (speed * speed);
    int tr = 0, id = 0;
    if (y < -10) { tr = 1; id = 1; }
    else if (mp <= 0) { tr = 1; id = 2; }
    else if (th > PI + radians(2)) { tr = 1; id = 3; }
    else if (q > 65000) { tr = 1; id = 4; }
    else if (gl > 6.0) { tr = 1; id = 5; }
    else if (vy > 0.0) { tr = 1; id = 6; }
    else if (vx > 0.01) { tr = 1; id = 7; }
    int done = (y > 0 && y < 1 && speed < 5.0);
    double y0 = P->state0[1];
    double ae = fabs(ga - th - PI);
    double lead = 1.5 - log(1 + ae) / log(1 + radians(20));
    double X;
    if (f32) {   /* tau = (u0 + 1)/2 in binary32; Python float - float32 -> float32 */
        float tau = ((float)u[0] + 1.0f) / 2.0f;
        X = (double)((float)lead - tau * 0.5f);
    } else {
        double tau = (u[0] + 1) / 2;
        X = lead - tau * 0.5;
    }
    double r = 0.0;
    r += X * (1 - y / y0) * 2 / 3;
    if (y < 100) r += 1 - tanh((speed - 15) / 15);
    if (tr && y < 5) r += 1 - tanh((speed - 5) / 5);
    if (done) r += 5;
    r *= (1 - P->rl_discount) / (1 - pow(P->rl_discount, (double)P->rl_traj_len));
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}

/* compile_rtd_rl_landing_burn_PDcontrol (rtd_rl.py:353-534); the reward is the SECOND
 * reward_func_lambda (:479-531), which rebinds the first.  v_ref = actions[0]. */
static void rtd_rl_pcontrol(const orc_params* P, const orc_env* E, double gl, const double* u, int f32,
                            orc_out* o) {
    const double* s = E->s;
    double y = s[1], vx = s[2], vy = s[3], th = s[4], m = s[8], mp = s[9];
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double q = 0.5 * rho * (speed * speed);
    int tr = 0, id = 0;
    if (y < -10) { tr = 1; id = 1; }
    else if (mp <= 0) { tr = 1; id = 2; }
    else if (th > PI + radians(2)) { tr = 1; id = 3; }
    else if (q > 65000) { tr = 1; id = 4; }
    else if (gl > 6.0) { tr = 1; id = 5; }
    else if (vy > 0.0) { tr = 1; id = 6; }
    int done = (y > 0 && y < 5 && speed < 1);
    double y0 = P->state0[1], m0 = P->state0[8];
    double sp = hypot(vx, vy);
    double qr = 0.5 * rho * (sp * sp);
    double r = 0.0;
    if (qr > 60000.0) { double e = (qr - 60000.0) / (65000.0 - 60000.0); r -= 1.0 * fmin(e * e, 1.0); }
    if (gl > 5.5) { double e = (gl - 5.5) / (6.0 - 5.5); r -= 1.0 * fmin(e * e, 1.0); }
    double prog = (y0 - y) / y0;
    double vt;
    if (f32) {   /* speed - v_ref: Python float - float32 -> float32 */
        float d = fabsf((float)sp - (float)u[0]) / 10.0f;
        float t = 1.0f - d;
        vt = t > 0.0f ? (double)t : 0.0;
    } else {
        double t = 1.0 - fabs(sp - u[0]) / 10.0;
        vt = t > 0.0 ? t : 0.0;
    }
    double wp = (qr <= 60000.0 && gl <= 5.5) ? 0.5 : 0.5 * 0.1;
    r += wp * prog * vt;
    if (y < 100.0) { double t = 1.0 - fabs(vy - 0.0) / 50.0; r += 0.5 * (t > 0.0 ? t : 0.0); }
    r += 0.01 * (1 - P->rl_discount);
    if (done && !tr) { r += 5.0; double used = y0 * 0.0 + (m0 - m); r -= fmin(0.1 * used, 1.0); }
    else if (tr) { double imp = fabs(vy), af = y / y0; r -= fmin(4.0 * af * (imp / 100.0), 5.0); }
    if (r < -10.0) r = -10.0;
    if (r > 10.0) r = 10.0;
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}

/* compile_rtd_rl_ballistic_arc_descent (rtd_rl.py:153-188) */
static void rtd_rl_ballistic(const orc_params* P, const orc_env* E, orc_out* o) {
    const double* s = E->s;
    double y = s[1], vx = s[2], vy = s[3], th = s[4], ga = s[6];
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double q = 0.5 * rho * (speed * speed);
    double ae = fabs(ga - th - PI);
    int done = (q > 10000 && ae < radians(3));
    int tr = 0, id = 0;
    if (q > 10000 - 2000 && ae > radians(5)) { tr = 1; id = 1; }
    double r = (PI - ae) / PI;
    if (done) r += 3.5;
    r /= 100;
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}

/* compile_rtd_rl_ascent (rtd_rl.py:11-114) with the subsonic / supersonic hyper-parameter
 * tables (:543-574) and the ascent reference trajectory (reference_trajectory_interpolation.py) */
static void rtd_rl_ascent(const orc_params* P, const orc_env* E, int which, orc_out* o) {
    const double* s = E->s;
    double x = s[0], y = s[1], vx = s[2], vy = s[3], al = s[7], mp = s[9];
    int nan = 0;
    for (int k = 0; k < 11; ++k) nan |= isnan(s[k]);
    if (nan) { o->reward = 0; o->done = 0; o->trunc = 1; o->trunc_id = 0; return; }
    double rho, pa, a;
    orc_atmosphere(P, y, &rho, &pa, &a);
    double speed = sqrt(vx * vx + vy * vy);
    double mach = (speed != 0 && a != 0) ? speed / a : 0;
    double tm = P->terminal_mach[which];
    double h[9][12];
    for (int k = 0; k < 12; ++k) for (int f = 0; f < 9; ++f) h[f][k] = P->hyper[which][k][f];
    double mx = interp1d_ext(h[0], h[1], 12, mach), mvy = interp1d_ext(h[0], h[2], 12, mach);
    double mvx = interp1d_ext(h[0], h[3], 12, mach), mal = interp1d_ext(h[0], h[4], 12, mach);
    double wal = interp1d_ext(h[0], h[5], 12, mach), wx = interp1d_ext(h[0], h[6], 12, mach);
    double wvy = interp1d_ext(h[0], h[7], 12, mach), wvx = interp1d_ext(h[0], h[8], 12, mach);
    int n = P->n_ref;
    double xr = interp1d_ext(P->ref_y, P->ref_x, n, y), vxr = interp1d_ext(P->ref_y, P->ref_vx, n, y);
    double vyr = interp1d_ext(P->ref_y, P->ref_vy, n, y);
    int done = (mp >= 0 && mach > tm);
    int tr = 0, id = 0;
    if (mp <= 0) { tr = 1; id = 1; }
    else if (mach > tm + 0.09) { tr = 1; id = 2; }
    else if (fabs(x - xr) > mx) { tr = 1; id = 3; }
    else if (y < 0) { tr = 1; id = 4; }
    else if (fabs(al) > radians(mal)) { tr = 1; id = 5; }
    else if (fabs(vx - vxr) > mvx) { tr = 1; id = 6; }
    else if (fabs(vy - vyr) > mvy) { tr = 1; id = 7; }
    double r = 0.0;
    if (!(y < 0)) {
        double d;
        d = vx - vxr; r += exp(-4 * (d * d) / (mvx * mvx)) * wvx;
        d = vy - vyr; r += exp(-4 * (d * d) / (mvy * mvy)) * wvy;
        d = x - xr; r += exp(-4 * (d * d) / (mx * mx)) * wx;
        d = degrees(al); r += exp(-4 * (d * d) / (mal * mal)) * wal;
        if (done) r += 2.5;
        r /= 10000;
    }
    o->reward = r; o->done = done; o->trunc = tr; o->trunc_id = id;
}

/* RL wrapper observation (env_wrapped_rl_pytorch.py:41-47 float32 cast, then augment_state
 * :167-202) for every phase */
static void obs_rl(const orc_params* P, int phase, const double* s, double* ob) {
    float f[11];
    for (int k = 0; k < 11; ++k) f[k] = (float)s[k];
    const double* nm = P->norm_ph[phase];
    switch (phase) {
        case ORC_PHASE_PURE_THROTTLE:
            ob[0] = (1 - (double)f[1] / P->norm_y) * 2 - 1;
            ob[1] = (1 - (double)f[3] / P->norm_vy) * 2 - 1;
            break;
        case ORC_PHASE_PCONTROL:
            ob[0] = (1 - (double)f[1] / P->norm_y) * 2 - 1;
            break;
        case ORC_PHASE_LANDING_BURN: {
            /* y, vy / norms (binary64); theta, theta_dot, gamma through float32 islands */
            double kt = atanh(0.75) / radians(5), ktd = atanh(0.75) / 0.01, kg = atanh(0.75) / radians(5);
            ob[0] = (double)f[1] / P->norm_y;
            ob[1] = (double)f[3] / P->norm_vy;
            ob[2] = tanh((double)((float)kt * (f[4] - (float)(PI / 2))));
            ob[3] = tanh((double)((float)ktd * f[5]));
            ob[4] = tanh((double)((float)kg * (f[6] - (float)(3.0 / 2 * PI))));
            break;
        }
        case ORC_PHASE_BALLISTIC: {   /* [theta, theta_dot, gamma, alpha] /= norms, in float32 */
            const int idx[4] = {4, 5, 6, 7};
            for (int k = 0; k < 4; ++k) ob[k] = (double)(float)((double)f[idx[k]] / nm[k]);
            break;
        }
        case ORC_PHASE_FLIP:
            ob[0] = (double)(float)((double)f[4] / nm[0]);
            ob[1] = (double)(float)((double)f[5] / nm[1]);
            break;
        default: {   /* ascent: [x, y, vx, vy, theta, theta_dot, alpha, mass] */
            const int idx[8] = {0, 1, 2, 3, 4, 5, 7, 8};
            for (int k = 0; k < 8; ++k) ob[k] = (double)(float)((double)f[idx[k]] / nm[k]);
        }
    }
}

/* ---------------------------------------------------------------- env step
 * rocket_environment_pre_wrap.step (base_environment.py:99-154) */
int orc_step(const orc_params* P, orc_env* E, int phase, int rtd, const double* u, int f32,
             const double* noise, orc_out* o) {
    memset(o, 0, sizeof(*o));
    orc_physics(P, E, phase, u, f32, noise, o->info);
    const double *s = E->s, *ps = E->prev_s;
    double v = sqrt(s[2] * s[2] + s[3] * s[3]);
    double vp = sqrt(ps[2] * ps[2] + ps[3] * ps[3]);
    double gload = fabs(v - vp) / 0.1 * 1 / 9.81;
    if (E->gwin_len < 10) E->gwin[E->gwin_len++] = gload;
    else { memmove(E->gwin, E->gwin + 1, 9 * sizeof(double)); E->gwin[9] = gload; }
    double sum = 0.0;
    for (int i = 0; i < E->gwin_len; ++i) sum += E->gwin[i];
    double gl = sum / 10;
    o->info[ORC_I_GLOAD] = gl;
    if (rtd == ORC_RTD_NONE) { o->reward = 0; o->done = 0; o->trunc = 0; o->trunc_id = 0; }
    else if (rtd == ORC_RTD_PSO) rtd_pso(P, E, phase, gl, o);
    else if (phase == ORC_PHASE_PURE_THROTTLE) rtd_rl_pure_throttle(P, E, gl, o);
    else if (phase == ORC_PHASE_LANDING_BURN) rtd_rl_landing_burn(P, E, gl, u, f32, o);
    else if (phase == ORC_PHASE_PCONTROL) rtd_rl_pcontrol(P, E, gl, u, f32, o);
    else if (phase == ORC_PHASE_BALLISTIC) rtd_rl_ballistic(P, E, o);
    else if (phase == ORC_PHASE_SUBSONIC || phase == ORC_PHASE_SUPERSONIC)
        rtd_rl_ascent(P, E, phase == ORC_PHASE_SUPERSONIC, o);
    E->trunc_id = o->trunc_id;
    E->rng_ts += 1;   /* the device's step-within-episode counter (Philox counter word) */
    memcpy(E->prev_s, E->s, sizeof(E->s));
    /* observations: RL pure throttle (env_wrapped_rl_pytorch.py:195-198), PSO (env_wrapped_ea.py:108-122) */
    if (rtd != ORC_RTD_PSO) {   /* the RL wrapper casts the state to float32 first */
        obs_rl(P, phase, s, o->obs);
    } else if (phase == ORC_PHASE_PURE_THROTTLE) {
        o->obs[0] = s[1] / P->norm_y; o->obs[1] = s[3] / P->norm_vy;
    } else {
        double k = atanh(0.75) / radians(25);
        o->obs[0] = s[0] / P->norm_x; o->obs[1] = s[1] / P->norm_y;
        o->obs[2] = s[2] / P->norm_vx; o->obs[3] = s[3] / P->norm_vy;
        o->obs[4] = tanh(k * (s[4] - PI / 2));
    }
    return 0;
}

/* Batched rollout with the device's draws: envs [i0, i1) of n (global indices g[i], first
 * episode ep0[i]), actions [T][n][A] float32, auto-reset into episode + 1. */
typedef struct {
    const orc_params* P; int phase, rtd, n, i0, i1, n_steps; const uint64_t* g; const uint32_t* ep0;
    const float* actions; int auto_reset, wind, stoch, fixed_prof; double tilt; uint64_t seed;
    double* reward; uint8_t* done; uint8_t* trunc; int8_t* tid; double* obs; int obs_dim; double* state_final;
    double acc; int64_t steps;
} philox_job;

static void philox_range(philox_job* j) {
    const orc_params* P = j->P;
    const int A = j->phase == ORC_PHASE_LANDING_BURN ? 4 : ((j->phase == ORC_PHASE_SUBSONIC || j->phase == ORC_PHASE_SUPERSONIC) ? 2 : 1);
    double acc = 0.0; int64_t steps = 0;
    orc_env E;
    orc_out o;
    for (int i = j->i0; i < j->i1; ++i) {
        uint32_t ep = j->ep0 ? j->ep0[i] : 0u;
        const uint64_t g = j->g ? j->g[i] : (uint64_t)i;
        orc_reset_philox(P, &E, j->phase, j->seed, g, ep, j->wind, j->stoch, j->fixed_prof, j->tilt);
        for (int t = 0; t < j->n_steps; ++t) {
            double u[4] = {0, 0, 0, 0};
            for (int k = 0; k < A; ++k) u[k] = j->actions[((size_t)t * j->n + i) * A + k];
            g_qlog_step = g_qlog ? g_qlog + ((size_t)t * j->n + i) * 4 : NULL;
            orc_step(P, &E, j->phase, j->rtd, u, 1, NULL, &o);
            g_qlog_step = NULL;
            acc += o.reward; ++steps;
            const size_t at = (size_t)t * j->n + i;
            if (j->reward) j->reward[at] = o.reward;
            if (j->done) j->done[at] = (uint8_t)o.done;
            if (j->trunc) j->trunc[at] = (uint8_t)o.trunc;
            if (j->tid) j->tid[at] = (int8_t)o.trunc_id;
            if (j->obs) for (int k = 0; k < j->obs_dim; ++k) j->obs[at * j->obs_dim + k] = o.obs[k];
            if (j->auto_reset && (o.done || o.trunc)) {
                ++ep;
                orc_reset_philox(P, &E, j->phase, j->seed, g, ep, j->wind, j->stoch, j->fixed_prof, j->tilt);
            }
        }
        if (j->state_final) memcpy(j->state_final + (size_t)i * 11, E.s, sizeof(E.s));
    }
    j->acc = acc; j->steps = steps;
}
static void* philox_worker(void* p) { philox_range((philox_job*)p); return NULL; }

double orc_rollout_philox(const orc_params* P, int phase, int rtd, int n, const uint64_t* g, const uint32_t* ep0,
                          int n_steps, const float* actions, int auto_reset, int wind, int stoch, int fixed_prof,
                          double tilt, uint64_t seed, double* reward, uint8_t* done, uint8_t* trunc, int8_t* tid,
                          double* obs, int obs_dim, double* state_final, int n_threads, int64_t* env_steps_out) {
    pthread_once(&g_log_once, log_cells_fill);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n > 0 ? n : 1;
    philox_job* jobs = (philox_job*)calloc((size_t)n_threads, sizeof(philox_job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int k = 0; k < n_threads; ++k) {
        philox_job* j = &jobs[k];
        j->P = P; j->phase = phase; j->rtd = rtd; j->n = n; j->n_steps = n_steps; j->g = g; j->ep0 = ep0;
        j->i0 = (int)((int64_t)n * k / n_threads); j->i1 = (int)((int64_t)n * (k + 1) / n_threads);
        j->actions = actions; j->auto_reset = auto_reset; j->wind = wind; j->stoch = stoch;
        j->fixed_prof = fixed_prof; j->tilt = tilt; j->seed = seed;
        j->reward = reward; j->done = done; j->trunc = trunc; j->tid = tid; j->obs = obs; j->obs_dim = obs_dim;
        j->state_final = state_final;
        if (n_threads > 1) pthread_create(&th[k], NULL, philox_worker, j);
        else philox_range(j);
    }
    double acc = 0.0; int64_t steps = 0;
    for (int k = 0; k < n_threads; ++k) {
        if (n_threads > 1) pthread_join(th[k], NULL);
        acc += jobs[k].acc; steps += jobs[k].steps;
    }
    free(jobs); free(th);
    if (env_steps_out) *env_steps_out = steps;
    return acc;
}

/* CPU baseline driver: n_env independent envs (the reference runs one env per process; this is
 * its scalar port), the device's draws for wind and tilt (seed, env i, episodes from 0). */
double orc_rollout(const orc_params* P, int phase, int rtd, int n_env, int n_steps,
                   const float* actions, int auto_reset, int64_t* env_steps_out) {
    return orc_rollout_ex(P, phase, rtd, n_env, n_steps, actions, auto_reset, 0, 0.0, 1, env_steps_out);
}
double orc_rollout_ex(const orc_params* P, int phase, int rtd, int n_env, int n_steps,
                      const float* actions, int auto_reset, int wind, double tilt, uint64_t seed,
                      int64_t* env_steps_out) {
    return orc_rollout_philox(P, phase, rtd, n_env, NULL, NULL, n_steps, actions, auto_reset, wind, wind, -1, tilt,
                              seed, NULL, NULL, NULL, NULL, NULL, 0, NULL, 1, env_steps_out);
}
/* The same on n_threads host threads over a static contiguous env partition (the multi-core
 * CPU baseline). */
double orc_rollout_mt(const orc_params* P, int phase, int rtd, int n_env, int n_steps,
                      const float* actions, int auto_reset, int wind, double tilt, uint64_t seed,
                      int n_threads, int64_t* env_steps_out) {
    return orc_rollout_philox(P, phase, rtd, n_env, NULL, NULL, n_steps, actions, auto_reset, wind, wind, -1, tilt,
                              seed, NULL, NULL, NULL, NULL, NULL, 0, NULL, n_threads, env_steps_out);
}

/* ---------------------------------------------------------------- PSO actor (test oracle)
 * simple_actor.forward (env_wrapped_ea.py:18-44) on pso_wrapper.augment_state
 * (env_wrapped_ea.py:97-123): Linear(IN,8)-ReLU-[Linear(8,8)-ReLU]xNL-Linear(8,OUT)-Tanh in
 * binary32, parameters in named_parameters() order.  Summation order: sequential over the
 * inputs, then + bias; tanh in binary64 rounded to binary32 (the order the GPU kernel uses;
 * torch's CPU sgemv may round differently in the last ulp). */
static void actor_layer(const float* w, const float* b, int in, int out, const float* x, float* y, int act) {
    for (int j = 0; j < out; ++j) {
        float acc = 0.f;
        for (int k = 0; k < in; ++k) acc = acc + w[j * in + k] * x[k];
        acc = acc + b[j];
        if (act == 0) y[j] = acc < 0.f ? 0.f : acc;
        else y[j] = (float)tanh((double)acc);
    }
}

void orc_actor(const orc_params* P, int phase, const float* w, const double* s, float* out) {
    float x[5], h[8], g[8];
    int in, nl, nout;
    if (phase == ORC_PHASE_PURE_THROTTLE) {
        in = 2; nl = 3; nout = 1;
        x[0] = (float)(s[1] / P->norm_y); x[1] = (float)(s[3] / P->norm_vy);
    } else {
        double k = atanh(0.75) / radians(25);
        in = 5; nl = 4; nout = 4;
        x[0] = (float)(s[0] / P->norm_x); x[1] = (float)(s[1] / P->norm_y);
        x[2] = (float)(s[2] / P->norm_vx); x[3] = (float)(s[3] / P->norm_vy);
        x[4] = (float)tanh(k * (s[4] - PI / 2));
    }
    const float* p = w;
    actor_layer(p, p + 8 * in, in, 8, x, h, 0); p += 8 * in + 8;
    for (int l = 0; l < nl; ++l) {
        actor_layer(p, p + 64, 8, 8, h, g, 0); p += 72;
        memcpy(h, g, sizeof(h));
    }
    actor_layer(p, p + 8 * nout, 8, nout, h, out, 1);
}

int orc_actor_params(int phase) { return phase == ORC_PHASE_PURE_THROTTLE ? 249 : 372; }

/* pso_wrapped_env.objective_function (env_wrapped_ea.py:200-222) for n particles (weights
 * [n][orc_actor_params(phase)]), each from the nominal initial state, no wind, until done or
 * truncated or max_steps: fitness[i] = -sum(reward), steps[i] = episode length. */
void orc_rollout_policy(const orc_params* P, int phase, int n, const float* w, int max_steps,
                        double* fitness, int32_t* steps) {
    int np_ = orc_actor_params(phase);
    for (int i = 0; i < n; ++i) {
        orc_env E;
        orc_out o;
        orc_reset(P, &E, NULL, 0, 0, 1.0, 1.0);
        double fit = 0.0;
        int t = 0;
        while (t < max_steps) {
            float a[4];
            double u[4];
            orc_actor(P, phase, w + (size_t)i * np_, E.s, a);
            for (int k = 0; k < 4; ++k) u[k] = a[k];
            orc_step(P, &E, phase, ORC_RTD_PSO, u, 1, NULL, &o);
            fit -= o.reward;
            ++t;
            if (o.done || o.trunc) break;
        }
        fitness[i] = fit;
        steps[i] = t;
    }
}

/* ---------------------------------------------------------------- CPU baselines (bench.py)
 * The oracle is test infrastructure; these two drivers exist only as bench.py's cpu_baseline legs
 * for BASELINE configs c4 and c5, timed on the host's cores over a static partition. */
typedef struct { const orc_params* P; int phase, n, max_steps; const float* w; double* fit; int32_t* steps; } pol_job;
static void* pol_worker(void* p) {
    pol_job* j = (pol_job*)p;
    orc_rollout_policy(j->P, j->phase, j->n, j->w, j->max_steps, j->fit, j->steps);
    return NULL;
}

/* orc_rollout_policy on n_threads host threads, particles split in contiguous blocks */
void orc_rollout_policy_mt(const orc_params* P, int phase, int n, const float* w, int max_steps, double* fitness,
                           int32_t* steps, int n_threads) {
    pthread_once(&g_log_once, log_cells_fill);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n > 0 ? n : 1;
    const int np_ = orc_actor_params(phase);
    pol_job* jobs = (pol_job*)calloc((size_t)n_threads, sizeof(pol_job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int k = 0; k < n_threads; ++k) {
        const int i0 = (int)((int64_t)n * k / n_threads), i1 = (int)((int64_t)n * (k + 1) / n_threads);
        pol_job* j = &jobs[k];
        j->P = P; j->phase = phase; j->n = i1 - i0; j->max_steps = max_steps; j->w = w + (size_t)i0 * np_;
        j->fit = fitness + i0; j->steps = steps + i0;
        if (n_threads > 1) pthread_create(&th[k], NULL, pol_worker, j);
        else pol_worker(j);
    }
    if (n_threads > 1)
        for (int k = 0; k < n_threads; ++k) pthread_join(th[k], NULL);
    free(jobs); free(th);
}

/* c5's collection step per env (sac_pytorch_powered_descent.py:160-183), pure throttle, rtd RL,
 * no wind, auto-reset: the Actor's forward pass (sac_pytorch.py:129-159: Linear(S, H) ReLU,
 * (L - 1) x [Linear(H, H) ReLU], the mean and log_std heads; torch's named_parameters() order and
 * [out][in] weights) in binary32 with sequential sums, Actor.sample (sac_pytorch.py:161-179: log_std
 * clamped to [-20, 2], std = exp, tanh(mean + std eps), max_action 1) with eps drawn as the device
 * draws it (Philox tag 19: (env, episode, step)), the env step, and the transition row
 * state | action | reward | next_state | done into the thread's ring of `ring_rows` rows. */
#define ORC_SAC_MAXH 512
typedef struct {
    const orc_params* P; int i0, i1, n_steps, S, H, L, A, ring_rows; const float* const* prm; uint64_t seed;
    int64_t steps; double acc;
} sac_job;
static void sac_dense(const float* w, const float* b, int in, int out, const float* x, float* y, int relu) {
    for (int j = 0; j < out; ++j) {
        float acc = 0.f;
        const float* wr = w + (size_t)j * in;
        for (int k = 0; k < in; ++k) acc = acc + wr[k] * x[k];
        acc = acc + b[j];
        y[j] = relu && acc < 0.f ? 0.f : acc;
    }
}
static void sac_range(sac_job* j) {
    const orc_params* P = j->P;
    const int S = j->S, H = j->H, L = j->L, A = j->A, W = 2 * S + A + 2;
    float* ring = (float*)calloc((size_t)j->ring_rows * W, sizeof(float));
    float h0[ORC_SAC_MAXH], h1[ORC_SAC_MAXH];
    int64_t steps = 0, row = 0;
    double acc = 0.0;
    orc_env E;
    orc_out o;
    for (int i = j->i0; i < j->i1; ++i) {
        uint32_t ep = 0;
        orc_reset_philox(P, &E, ORC_PHASE_PURE_THROTTLE, j->seed, (uint64_t)i, ep, 0, 0, -1, 0.0);
        double ob[8];
        obs_rl(P, ORC_PHASE_PURE_THROTTLE, E.s, ob);
        for (int t = 0; t < j->n_steps; ++t) {
            float x[16], mean[8], lstd[8], a[8];
            for (int k = 0; k < S; ++k) x[k] = (float)ob[k];
            sac_dense(j->prm[0], j->prm[1], S, H, x, h0, 1);
            for (int l = 1; l < L; ++l) {
                sac_dense(j->prm[2 * l], j->prm[2 * l + 1], H, H, h0, h1, 1);
                memcpy(h0, h1, (size_t)H * sizeof(float));
            }
            sac_dense(j->prm[2 * L], j->prm[2 * L + 1], H, A, h0, mean, 0);
            sac_dense(j->prm[2 * L + 2], j->prm[2 * L + 3], H, A, h0, lstd, 0);
            double u[4] = {0, 0, 0, 0};
            for (int k = 0; k < A; k += 2) {
                orc_u32x4 c = {(uint32_t)i, ep, (uint32_t)E.rng_ts, 19u + (uint32_t)(k >> 1)};
                double z0, z1;
                orc_gauss_pair(orc_philox(c, (uint32_t)j->seed, (uint32_t)(j->seed >> 32)), &z0, &z1);
                for (int q = k; q < k + 2 && q < A; ++q) {
                    float ls = lstd[q] < -20.f ? -20.f : (lstd[q] > 2.f ? 2.f : lstd[q]);
                    a[q] = tanhf(mean[q] + expf(ls) * (float)(q == k ? z0 : z1));
                    u[q] = a[q];
                }
            }
            orc_step(P, &E, ORC_PHASE_PURE_THROTTLE, ORC_RTD_RL, u, 1, NULL, &o);
            float* r = ring + (size_t)(row % j->ring_rows) * W;
            for (int k = 0; k < S; ++k) r[k] = (float)ob[k];
            for (int k = 0; k < A; ++k) r[S + k] = a[k];
            r[S + A] = (float)o.reward;
            for (int k = 0; k < S; ++k) r[S + A + 1 + k] = (float)o.obs[k];
            r[2 * S + A + 1] = (float)o.done;
            ++row; ++steps; acc += o.reward;
            if (o.done || o.trunc) {
                ++ep;
                orc_reset_philox(P, &E, ORC_PHASE_PURE_THROTTLE, j->seed, (uint64_t)i, ep, 0, 0, -1, 0.0);
                obs_rl(P, ORC_PHASE_PURE_THROTTLE, E.s, ob);
            } else {
                for (int k = 0; k < S; ++k) ob[k] = o.obs[k];
            }
        }
    }
    free(ring);
    j->steps = steps; j->acc = acc;
}
static void* sac_worker(void* p) { sac_range((sac_job*)p); return NULL; }

double orc_sac_collect_mt(const orc_params* P, int n_env, int n_steps, int S, int H, int L, int A,
                          const float* const* prm, uint64_t seed, int n_threads, int64_t* env_steps_out) {
    pthread_once(&g_log_once, log_cells_fill);
    /* the pure-throttle SAC task only (sac_range hard-codes that phase: S = 2 observations, A = 1
     * action); anything else is refused rather than run on fixed-size buffers */
    if (S != 2 || A != 1 || H > ORC_SAC_MAXH || H < 1 || L < 1) return 0.0;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n_env) n_threads = n_env > 0 ? n_env : 1;
    sac_job* jobs = (sac_job*)calloc((size_t)n_threads, sizeof(sac_job));
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int k = 0; k < n_threads; ++k) {
        sac_job* j = &jobs[k];
        j->P = P; j->i0 = (int)((int64_t)n_env * k / n_threads); j->i1 = (int)((int64_t)n_env * (k + 1) / n_threads);
        j->n_steps = n_steps; j->S = S; j->H = H; j->L = L; j->A = A; j->prm = prm; j->seed = seed;
        j->ring_rows = 4096;
        if (n_threads > 1) pthread_create(&th[k], NULL, sac_worker, j);
        else sac_range(j);
    }
    double acc = 0.0; int64_t steps = 0;
    for (int k = 0; k < n_threads; ++k) {
        if (n_threads > 1) pthread_join(th[k], NULL);
        acc += jobs[k].acc; steps += jobs[k].steps;
    }
    free(jobs); free(th);
    if (env_steps_out) *env_steps_out = steps;
    return acc;
}
