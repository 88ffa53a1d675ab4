// pd_physics.h -- device physics of the landing burn, templated on the state precision.
//
// One lane = one environment.  Every function restates a reference function (file:line)
// with the same operation order, so that the binary64 instantiation reproduces the
// reference's IEEE results (up to libm ulps); the float instantiation is the throughput mode.
#pragma once
#include "pd_common.h"

namespace pd {

template <typename R> struct Cst;
template <> struct Cst<double> {
    static constexpr double deg2rad = kDeg2Rad, rad2deg = kRad2Deg, pi = kPi, two_pi = 2 * kPi;
    static constexpr double inf = __builtin_huge_val();
};
template <> struct Cst<float> {
    static constexpr float deg2rad = (float)kDeg2Rad, rad2deg = (float)kRad2Deg, pi = (float)kPi,
                           two_pi = (float)(2 * kPi);
    static constexpr float inf = __builtin_huge_valf();
};

// a / b for a divisor known ahead of the call -- a literal or a per-handle parameter -- given
// rb = RN(1/b), its correctly rounded reciprocal (a compile-time or host division), as the IEEE
// quotient RN(a / b) (finite a, b > 0, a / b away from underflow and overflow, as every quotient
// here is).  Markstein's theorem: if rb is within half an ulp of 1/b and q is within one ulp of
// a/b (faithful), then r = a - b q is exact (one FMA) and RN(q + r rb) = RN(a/b).  Whether
// q = RN(a rb) is faithful depends on the divisor: with eps = b rb - 1 (exact), |a rb - a/b| =
// |a/b| |eps| < 2^(e+1) |eps| for a/b in [2^e, 2^(e+1)), below half an ulp of a/b when
// |eps| <= 2^-(p+1) (p = 53 / 24), and q is then faithful for every a (one_step_ok).  Other
// divisors take one more correction first: q1 = RN(q + r rb) is within half an ulp plus
// |a/b - q| 2^(1-p) of a/b, so faithful, and the final step is Markstein's.  Each step is
// computed negated, -RN(-r rb - q), so that a zero numerator keeps its sign.  Three (five) VALU
// operations where a general division is the ten-deep v_div_scale / v_rcp / Newton / v_div_fmas
// / v_div_fixup sequence.  tests/test_markstein.py checks the classification in exact rational
// arithmetic, every binary32 numerator of every divisor the kernel replaces, and sampled
// binary64 numerators, bit for bit against IEEE division.
template <typename R> constexpr R veltkamp_c() { return sizeof(R) == 8 ? R(134217729.0) : R(4097.0f); }
// eps = b rb - 1 as (hi - 1) + lo, hi + lo = b rb exactly (Dekker's product; no FMA contraction
// in this build), so both the compiler (literals) and the host (handle divisors) classify
template <typename R> constexpr bool one_step_ok(R b, R rb) {
    const R p = b * rb;
    const R C = veltkamp_c<R>();
    const R tb = C * b, bh = tb - (tb - b), bl = b - bh;
    const R tr = C * rb, rh = tr - (tr - rb), rl = rb - rh;
    const R lo = ((bh * rh - p) + bh * rl + bl * rh) + bl * rl;
    const R eps = (p - R(1)) + lo;
    // |eps| <= 2^-(p+1), with a 1 % margin for the rounding of the sum (conservative: a divisor
    // at the bound takes the second correction)
    const R lim = sizeof(R) == 8 ? R(0.99 * 0x1p-54) : R(0.99f * 0x1p-25f);
    return eps <= lim && -eps <= lim;
}
template <typename R> __device__ __forceinline__ R div_known(R a, R b, R rb, bool two) {
    R q = a * rb;
    R r = fma(-b, q, a);
    if (two) {
        q = -fma(-r, rb, -q);
        r = fma(-b, q, a);
    }
    return -fma(-r, rb, -q);
}
// the reciprocal of a literal divisor, folded at compile time in R's precision
template <typename R> constexpr R rcp_c(R b) { return R(1) / b; }
// DevParams::div2 bits (the handle's divisors)
constexpr uint32_t kDiv2MProp0 = 1, kDiv2Y0 = 2, kDiv2M0 = 4, kDiv2NormY = 8, kDiv2NormVy = 16, kDiv2NormX = 32,
                   kDiv2NormVx = 64;
#define PD_DIVC(R_, a, b) div_known<R_>((a), R_(b), rcp_c<R_>(R_(b)), !one_step_ok<R_>(R_(b), rcp_c<R_>(R_(b))))

constexpr int kLineMax = 96;   // breakpoints per clamped query line
// line search buckets: Mach [0, 10) in kLineBuckets; bucket b's breakpoint index range (lo, hi),
// lo = #{bp < b w - 1e-4}, hi = #{bp < (b + 1) w + 1e-4}, packed lo | hi << 8
constexpr int kLineBuckets = 128;
// Taylor pieces of the clamped query lines (pdenv.hip build_taylor): Mach [0, 10] in kTayCells
// uniform cells; a cell's piece for neighbourhood interval l is at line offset + cell + l.  A
// piece: kTayDeg + 1 coefficients of the expansion at the cell centre, then kTayExact exact
// terms (Mach, coefficient / 8, d_a^2) for the singularities nearest to the cell.
constexpr int kTayCells = 2048, kTayDeg = 10, kTayExact = 2;
constexpr int kTayStride = kTayDeg + 1 + 3 * kTayExact + 1;

// The tabulated atmosphere (pdenv.hip build_atm_table): the ISA rho, p, a by geometric altitude
// in cells of kAtmW m (degree kAtmDeg in t = y - centre; a record is the cell's piece -- centre,
// the base H of a layer boundary inside the cell or 1e30, coefficients -- and then the upper
// layer's piece)
constexpr int kAtmDeg = 5, kAtmRec = 2 + 3 * (kAtmDeg + 1), kAtmStride = 2 * kAtmRec;
constexpr double kAtmW = 100.0;

// Address spaces of the step kernel's memory: the per-handle parameter block is read through a
// constant-address-space view (uniform fields become scalar loads into SGPRs), the tables behind
// its pointers through global-address-space pointers (global_load, not flat: a flat load waits
// on both the LDS and the vector-memory counters).
#define PD_AS1 __attribute__((address_space(1)))
#define PD_AS4 __attribute__((address_space(4)))

// Device parameter block (one per handle, in HBM, read with uniform scalar loads).
template <typename R> struct DevParams {
    // sizing
    R T_e, p_e, A_e, v_ex, S_gf, d_base_gf, R_rocket, A_front, m_prop0, C_gust_x, C_gust_y;
    int n_eng, pad0;
    // float32 islands: constants as NumPy casts them (weak Python scalars -> float32)
    float f_Te_over_vex, f_one_minus_nom_pt, f_nom_pt, f_one_minus_nom_lb, f_nom_lb, f_dt_pt, f_dt_lb,
        f_max_gimbal_rad, f_max_defl_rad, pad1;
    R Te_over_vex, one_minus_nom_pt, nom_pt, one_minus_nom_lb, nom_lb, max_gimbal_rad, max_gimbal_deg,
        max_defl_rad;
    // mass properties
    R h_ox, h_f, m_ox, m_f, h_lower, m_dry, x_dry, I_dry, engine_height, cop;
    // ISA: per layer base, T, p, beta, beta/Tb, exponent -g0/(beta R), isothermal -g0/(R Tb)
    R isa_Hb[9], isa_Tb[9], isa_beta[9], isa_pb[9], isa_bt[9], isa_ex[9], isa_iso[9];
    R isa_r, isa_R, isa_kappaR, isa_alt_max, grav_R, grav_g0;
    // aero tables: geometry (the Mach arrays are staged into LDS)
    int cd_start[kCols], cd_len[kCols], cl_start[kCols], cl_len[kCols];
    R cd_aoa[kCols], cl_aoa[kCols];
    int cd_n, cl_n;
    R cd_mach[256], cl_mach[256];
    R cd_pt_aoa[256], cl_pt_aoa[256];   // AoA of every table point (its column's)
    // binary64 copies for on-device neighbourhood solves
    double cd_mach_d[256], cd_coef_d[256], cl_mach_d[256], cl_coef_d[256], cd_aoa_d[kCols], cl_aoa_d[kCols];
    // grid fins
    int ca_n, cn_n;
    R ca_x[64], ca_y[64], ca_min_mach, ca_min_val;
    uint16_t ca_lb[64];              // C_a search buckets over Mach [0, 10) (as line_lb)
    R cn_x[64], cn_y[64], cn_min_mach, cn_max_mach, cn_min_val, cn_max_val, cn_slope;
    // wind
    int wind_n[50];
    R wind_alt_km[50][16], wind_speed[50][16];
    R vk_Ad_u[4], vk_Bd_u[2], vk_Ad_v[4], vk_Bd_v[2], vk_y_threshold;
    double sigma_u_lo, sigma_u_hi, sigma_v_lo, sigma_v_hi;
    // initial state, observation normalisers
    R state0[11];
    double state0_d[11];
    R norm_y, norm_vy, norm_x, norm_vx, k_theta_pso;
    LogTable logtab;   // log_tab cells (pd_common.h): the Box-Muller draws (oracle-restated)
    LogTableD logtab_d;   // eval_log cells, staged into LDS by the step kernel
    R y0_rl, m0_rl;
    // correctly rounded reciprocals of the divisors above (div_known): 1 / m_prop0, y0_rl, m0_rl,
    // norm_y, norm_vy, norm_x, norm_vx
    R inv_m_prop0, inv_y0_rl, inv_m0_rl, inv_norm_y, inv_norm_vy, inv_norm_x, inv_norm_vx;
    // bit k set: divisor k of that list needs div_known's second correction (!one_step_ok)
    uint32_t div2, pad_div2;
    // neighbourhood hash tables
    const unsigned long long* keys_cd;
    const unsigned long long* keys_cl;
    const R* pay_cd;
    const R* pay_cl;
    int logcap_cd, logcap_cl;
    unsigned long long init_key_cd, init_key_cl;
    // neighbourhood intervals along the four clamped query lines (C_D at +-radians(10) "deg",
    // C_L at +-10): breakpoints in Mach, and the key/slot of each interval
    R line_a[4];
    int line_nbp[4];
    uint16_t line_lb[4][kLineBuckets];
    // Taylor pieces of the four lines in one array; tay_off[li]: the line's first piece, -1 none
    const R* tay;
    const void* stage_img;   // StepStatic<R, wind> of the handle (pd_step.h): the LDS tables' image
    int tay_off[4];
    // 2-D candidate grids over the interior query domain (Mach x AoA-abscissa), one per table:
    // the key/slot of the 50-NN set at each cell centre
    int grid_nm[2], grid_na[2];
    R grid_a0[2], grid_inv_da[2], grid_inv_dm[2];
    const unsigned long long* grid_key[2];
    const int* grid_slot[2];
    // refined cells (kGridRefine): kGridSub x kGridSub sub-cells each, Mach-major
    const unsigned long long* sub_key[2];
    const int* sub_slot[2];
    const void* sub_bis[2];          // GridBisect records (pd_step.h) of the kGridBisect sub-cells
    // cell pieces (pd_step.h cell_stride<R>() words each, in R; nullptr: none): an exact
    // cell's piece at its cell index, a refined cell's at sub_piece[sub-cell] (-1: none)
    const R* cell_pc[2];
    const int* sub_piece[2];
    const uint32_t* fine[2];           // fine index (pd_step.h kFinePiece; nullptr: none)
    R line_bp[4][kLineMax];
    int line_slot[4][kLineMax + 1];
    unsigned long long line_key[4][kLineMax + 1];
    // ---- the other flight phases (rockets_physics.py:17-166,402-451,728-802,959-997)
    int phase, obs_kind;           // pd_phase of the handle; observation layout (obs_write)
    R fr[13];                      // full_rocket_inertia cells (ascent), see inertia_full
    R cop_ascent, mg_ascent, kp_pc, rcs_force, rcs_d_bottom, rcs_d_top;
    int n_eng_stage1, n_ref;
    float f_mg_ascent, f_kp_pc, f_rcs_force, f_k_theta_rl, f_k_thetad_rl, f_k_gamma_rl, f_pi_2, f_pi_3_2;
    R norm_ph[8];                  // RL observation normalisers of the phase
    const R* ref_y;                // ascent reference trajectory, sorted by y (n_ref rows)
    const R* ref_x;
    const R* ref_vx;
    const R* ref_vy;
    R hyper[12][9];                // ascent rtd hyper-parameters by Mach (rtd_rl.py:543-574)
    R terminal_mach;
    R rl_scale, alive_bonus, log_1p_max_ae;   // (1-g)/(1-g^L), 0.01 (1-g), log(1 + radians(20))
    // the tabulated atmosphere (atmosphere<R, true> below; nullptr: the exact formulas)
    const R* atm_tab;
    R atm_inv_w;
    int atm_n;
};
template <typename R> using DP = const PD_AS4 DevParams<R>;
template <typename T> __device__ __forceinline__ const PD_AS1 T* gbl(const T* p) { return (const PD_AS1 T*)(uint64_t)p; }
template <typename T> __device__ __forceinline__ PD_AS1 T* gblw(T* p) { return (PD_AS1 T*)(uint64_t)p; }

// ISA layer constants staged in LDS per workgroup (the layer is a per-lane index):
// Hb, Tb, beta, pb, beta/Tb, exponent -g0/(beta R), isothermal -g0/(R Tb), pad
constexpr int kIsaCols = 8;

// ---------------------------------------------------------------- logarithms
// Hot-path log(): binary64 through the LDS-staged cell table (log_tab, pd_common.h; the step
// kernel stages it before its barrier), binary32 through the hardware log2.
// eval_log's cells (LogTableD): (2 invc, logc - ln 2) of cell i at [2i], [2i + 1], one 16-byte
// ds_read_b128 per log
__shared__ __attribute__((aligned(16))) double s_logtab[2 * kLogCellsD];
template <typename R> __device__ __forceinline__ R eval_log(R x);
// 4 ((logc - ln2) + log1p(r)), r = m1 (2 invc) - 1, |r| <= 2^-11, c.y = 4 (logc - ln2): the
// degree-4 series in Horner form scaled by 4 (exact), 4 log1p(r) = r (4 + r (-2 + r (4/3 - r))),
// so that each step has one SGPR constant at most (4, -2 and -1 are inline operands): five
// VALU operations, no constant moves
__device__ __forceinline__ double log_cell_poly4(double m1, double2 c) {
    const double r = fma(m1, c.x, -1.0);
    const double t = fma(r, fma(r, 4.0 / 3.0 - r, -2.0), 4.0);
    return fma(r, t, c.y);
}
// 4 log x (the RBF sums accumulate 4 d2 log d2 and scale once at the end)
__device__ __forceinline__ double log4_from(int e1, double m1, double2 c) {
    return fma((double)e1, 4.0 * 6.93147180559945286227e-01, log_cell_poly4(m1, c));
}
template <> __device__ __forceinline__ double eval_log<double>(double x) {
    // x = 2^e1 m1, m1 in [0.5, 1) (v_frexp_*); cell from the top 10 mantissa bits;
    // r = m1 (2 invc) - 1 = m invc - 1; log x = e1 ln2 + (logc - ln2) + log1p(r)
    // (v_frexp_*: extracting exponent and mantissa by bit operations measured 2.6 % slower)
    const int e1 = __builtin_amdgcn_frexp_exp(x);
    const double m1 = __builtin_amdgcn_frexp_mant(x);
    const uint32_t hi = (uint32_t)(__double_as_longlong(x) >> 32);
    const uint32_t off = (hi >> (16 - kLogBitsD)) & ((kLogCellsD - 1) << 4);   // cell * 16 bytes
    const double2 c = *(const double2*)((const char*)s_logtab + off);
    return 0.25 * log4_from(e1, m1, c);
}
// eval_log<double> in two stages, so that a caller can issue the cell reads of several
// arguments before finishing any of them (same arithmetic, same bits)
struct LogPart { double m1; int e1; double2 c; };
__device__ __forceinline__ LogPart log_start(double x) {
    LogPart q;
    q.e1 = __builtin_amdgcn_frexp_exp(x);
    q.m1 = __builtin_amdgcn_frexp_mant(x);
    const uint32_t hi = (uint32_t)(__double_as_longlong(x) >> 32);
    q.c = *(const double2*)((const char*)s_logtab + ((hi >> (16 - kLogBitsD)) & ((kLogCellsD - 1) << 4)));
    return q;
}
// 4 log x
__device__ __forceinline__ double log4_finish(const LogPart& q) { return log4_from(q.e1, q.m1, q.c); }
template <> __device__ __forceinline__ float eval_log<float>(float x) {
    return __builtin_amdgcn_logf(x) * 0.693147180559945309f;
}
// 4 log x (the RBF term sums)
template <typename R> __device__ __forceinline__ R eval_log4(R x);
template <> __device__ __forceinline__ double eval_log4<double>(double x) {
    const int e1 = __builtin_amdgcn_frexp_exp(x);
    const double m1 = __builtin_amdgcn_frexp_mant(x);
    const uint32_t hi = (uint32_t)(__double_as_longlong(x) >> 32);
    const double2 c = *(const double2*)((const char*)s_logtab + ((hi >> (16 - kLogBitsD)) & ((kLogCellsD - 1) << 4)));
    return log4_from(e1, m1, c);
}
template <> __device__ __forceinline__ float eval_log4<float>(float x) {
    return __builtin_amdgcn_logf(x) * (4.0f * 0.693147180559945309f);
}

// ---------------------------------------------------------------- sine and cosine together
// Binary64: sincos_fd (pd_common.h, fdlibm kernels, <= 1 ulp); binary32: the device library.
template <typename R> __device__ __forceinline__ void pd_sincos(R x, R& s, R& c) {
    s = sin(x); c = cos(x);
}
template <> __device__ __forceinline__ void pd_sincos<double>(double x, double& s, double& c) {
    sincos_fd(x, s, c);
}

// ---------------------------------------------------------------- flight-path angle
// gamma = atan2(vy, vx) (rockets_physics.py:631): the device library's atan2 (fdlibm's reduction
// with one division, tools/experiments/atan2_fd.patch, measured 3 % slower on c3 and c3-descent,
// 5 % on c2: profiles/r04_exp_s2_variants.jsonl)
template <typename R> __device__ __forceinline__ R pd_atan2(R y, R x) { return atan2(y, x); }

// ---------------------------------------------------------------- atmosphere
// atmosphere_dynamics.py:5-27 (ambiance ISA restated)
// TAB: from the table (build_atm_table: every piece within 2e-15 of the long double ISA in
// binary64, 2e-16 typical; the exact path's own rounding reaches 5e-15 where pow's exponent is
// large): one cell record, the upper layer's piece past a layer boundary inside the cell, three
// Horner chains -- about a fifth of the exact path's instructions (two divisions, exp, log, sqrt,
// the layer search), but an L2 load at the head of the sub-step's chain.  Measured
// (profiles/r04_exp_s10_tables.jsonl): c2 -2 %, binary32 c3 -5 %, binary64 c3 with wind +1.5 %;
// the step kernel takes it where it pays (k_step kAtmTab).  No table uploaded: the exact path.
template <typename R, bool TAB = true>
__device__ __forceinline__ void atmosphere(DP<R>& P, const R* isa, R y, R& rho, R& p, R& a) {
    R alt = y < R(0) ? R(0) : y;
    if (TAB && P.atm_tab != nullptr) {
        if (alt < P.isa_alt_max) {
            int k = (int)(alt * P.atm_inv_w);
            k = k > P.atm_n - 1 ? P.atm_n - 1 : k;
            const PD_AS1 R* rec = gbl(P.atm_tab) + (uint32_t)k * (uint32_t)kAtmStride;
            R c[kAtmRec];
#pragma unroll
            for (int u = 0; u < kAtmRec; ++u) c[u] = rec[u];
            // a layer boundary inside this cell (c[1] its base H): the exact path's layer test,
            // so that both take the same side of the pb jump (lanes of ~0.7 % of the altitudes)
            if (c[1] < R(1e29) && P.isa_r * alt / (P.isa_r + alt) >= c[1]) {
#pragma unroll
                for (int u = 0; u < kAtmRec; ++u) c[u] = rec[kAtmRec + u];
            }
            const R t = alt - c[0];
            R fp = c[2 + kAtmDeg], fr = c[2 + 2 * kAtmDeg + 1], fa = c[2 + 3 * kAtmDeg + 2];
#pragma unroll
            for (int j = kAtmDeg - 1; j >= 0; --j) {
                fp = fma(fp, t, c[2 + j]);
                fr = fma(fr, t, c[2 + kAtmDeg + 1 + j]);
                fa = fma(fa, t, c[2 + 2 * (kAtmDeg + 1) + j]);
            }
            p = fp; rho = fr; a = fa;
        } else {
            rho = R(0); p = R(0); a = R(0);
        }
        return;
    }
    if (alt < P.isa_alt_max) {
        R H = P.isa_r * alt / (P.isa_r + alt);
        int i = 0;
#pragma unroll
        for (int k = 1; k < 9; ++k) i = (P.isa_Hb[k] <= H) ? k : i;   // uniform bases (SGPRs)
        const R* L = isa + i * kIsaCols;                                  // the lane's layer (LDS)
        R Hb = L[0], Tb = L[1], b = L[2], pb = L[3];
        R dH = H - Hb;
        R T = Tb + b * dH;
        R pp;
        // (1 + beta/Tb dH)^ex; binary64 as exp(ex log(.)) with the table log (|err| < 1e-15 rel)
        if (b != R(0)) {
            if constexpr (sizeof(R) == 8) pp = pb * exp(L[5] * eval_log<R>(R(1) + L[4] * dH));
            else pp = pb * pow(R(1) + L[4] * dH, L[5]);
        }
        else pp = pb * exp(L[6] * dH);
        p = pp;
        rho = pp / (P.isa_R * T);
        a = sqrt(P.isa_kappaR * T);
    } else {
        rho = R(0); p = R(0); a = R(0);
    }
}

template <typename R> __device__ __forceinline__ R gravity(DP<R>& P, R y) {
    R q = P.grav_R / (P.grav_R + y);      // atmosphere_dynamics.py:29-33
    return P.grav_g0 * (q * q);
}

// stage_inertia closure (rocket_dimensions.py:167-196)
template <typename R>
__device__ __forceinline__ void inertia(DP<R>& P, R fill, R& x_cog, R& I) {
    R h_ox_t = P.h_ox * fill, h_f_t = P.h_f * fill, m_ox_t = P.m_ox * fill, m_f_t = P.m_f * fill;
    R x_prop = (m_ox_t * (P.h_lower + h_ox_t / R(2)) + m_f_t * (P.h_lower + P.h_ox + h_f_t / R(2))) / (m_ox_t + m_f_t);
    R t1 = P.h_lower + h_ox_t / R(2) - x_prop;
    R I_ox = R(1.0 / 12) * m_ox_t * (h_ox_t * h_ox_t) + m_ox_t * (t1 * t1);
    R t2 = P.h_lower + P.h_ox + h_f_t / R(2) - x_prop;
    R I_f = R(1.0 / 12) * m_f_t * (h_f_t * h_f_t) + m_f_t * (t2 * t2);
    R mp_t = m_ox_t + m_f_t;
    R x_wet = (P.m_dry * P.x_dry + mp_t * x_prop) / (P.m_dry + mp_t);
    R t3 = P.x_dry - x_wet, t4 = x_prop - x_wet;
    x_cog = x_wet;
    I = (P.I_dry + P.m_dry * (t3 * t3)) + ((I_ox + I_f) + mp_t * (t4 * t4));
}

// full_rocket_inertia closure (rocket_dimensions.py:198-241), x_cog_inertia_subrocket_0_lambda of
// the ascent phases, with its own expression order (x_prop_1 uses the untilded m_1_f and
// h_ox_1_tilde as written)
template <typename R>
__device__ __forceinline__ void inertia_full(DP<R>& P, R fill, R& x_cog, R& I) {
    const PD_AS4 R* c = P.fr;
    const R x_wet2 = c[0], x_dry1 = c[1], m_s1 = c[2], m_pay = c[3], m_2 = c[4], m1_ox = c[5], m1_f = c[6];
    const R h_lower1 = c[7], h1_ox = c[8], h1_f = c[9], h1 = c[10], I_wet2 = c[11], I_dry1 = c[12];
    R h_ox_t = h1_ox * fill, h_f_t = h1_f * fill, m_ox_t = m1_ox * fill, m_f_t = m1_f * fill;
    R m_prop_t = m_ox_t + m_f_t;
    R x_prop = (m_ox_t * (h_lower1 + h_ox_t / R(2)) + m1_f * (h_lower1 + h_ox_t + h_f_t / R(2))) / (m_ox_t + m_f_t);
    R t1 = h_lower1 + h_ox_t / R(2) - x_prop;
    R I_ox = R(1.0 / 12) * m_ox_t * (h_ox_t * h_ox_t) + m_ox_t * (t1 * t1);
    R t2 = h_lower1 + h_ox_t + h_f_t / R(2) - x_prop;
    R I_f = R(1.0 / 12) * m_f_t * (h_f_t * h_f_t) + m_f_t * (t2 * t2);
    R xr = (m_s1 * x_dry1 + (m_2 + m_pay) * (x_wet2 + h1) + m_prop_t * x_prop) / (m_s1 + m_2 + m_pay + m_prop_t);
    R d1 = x_dry1 - xr, d2 = x_wet2 - xr, d3 = x_prop - xr;
    x_cog = xr;
    I = I_dry1 + m_s1 * (d1 * d1) + I_wet2 + m_2 * (d2 * d2) + (I_ox + I_f) + m_prop_t * (d3 * d3);
}

// scipy interp1d(kind='linear', fill_value='extrapolate') on a sorted table in global memory:
// _call_linear (searchsorted side='left', index clipped to [1, n-1])
template <typename R>
__device__ __forceinline__ R interp1d_ext(const PD_AS1 R* x, const PD_AS1 R* y, int n, R v) {
    int lo = 0, hi = n;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (x[mid] < v) lo = mid + 1; else hi = mid; }
    int i = lo < 1 ? 1 : (lo > n - 1 ? n - 1 : lo);
    R slope = (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
    return slope * (v - x[i - 1]) + y[i - 1];
}

// The same on one column of the ascent hyper-parameter table (Mach in column 0, 12 rows).
template <typename R>
__device__ __forceinline__ R hyper_interp(DP<R>& P, int col, R mach) {
    int lo = 0, hi = 12;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (P.hyper[mid][0] < mach) lo = mid + 1; else hi = mid; }
    int i = lo < 1 ? 1 : (lo > 11 ? 11 : lo);
    R slope = (P.hyper[i][col] - P.hyper[i - 1][col]) / (P.hyper[i][0] - P.hyper[i - 1][0]);
    return slope * (mach - P.hyper[i - 1][0]) + P.hyper[i - 1][col];
}

// Observation of state s, written to out[0..dim) (dim = obs_dim(kind)):
//  0 RL pure throttle  (env_wrapped_rl_pytorch.py:195-198)   1 PSO pure throttle (env_wrapped_ea.py:108-111)
//  2 PSO landing_burn  (env_wrapped_ea.py:112-122)           3 RL landing_burn / ACS (env_wrapped_rl_pytorch.py:178-194)
//  4 RL Pcontrol (:199-201)  5 RL ballistic arc (:175-177)  6 RL flip-over (:172-174)  7 RL ascent (:169-171)
// The RL wrapper casts the state to float32 before augment_state (:41-47); the divisions by the
// float64 normalisers of kinds 5-7 happen in place on a float32 array (so round back to float32).
__host__ __device__ constexpr int obs_dim(int kind) {
    return kind == 2 || kind == 3 ? 5 : (kind == 4 ? 1 : (kind == 5 ? 4 : (kind == 7 ? 8 : 2)));
}
// obs_eval: the observation's components to put(k, value); obs_write: to row idx of out [N][dim]
template <typename R, typename Put>
__device__ __forceinline__ void obs_eval(DP<R>& P, int kind, const R* s, Put&& put) {
    // (divisions by the normalisers through their reciprocals: div_known, the same quotients)
    auto ny = [&](R v) { return div_known<R>(v, P.norm_y, P.inv_norm_y, P.div2 & kDiv2NormY); };
    auto nvy = [&](R v) { return div_known<R>(v, P.norm_vy, P.inv_norm_vy, P.div2 & kDiv2NormVy); };
    if (kind == 0) {
        put(0, (R(1) - ny((R)(float)s[1])) * R(2) - R(1));
        put(1, (R(1) - nvy((R)(float)s[3])) * R(2) - R(1));
    } else if (kind == 1) {
        put(0, ny(s[1])); put(1, nvy(s[3]));
    } else if (kind == 2) {
        put(0, div_known<R>(s[0], P.norm_x, P.inv_norm_x, P.div2 & kDiv2NormX)); put(1, ny(s[1]));
        put(2, div_known<R>(s[2], P.norm_vx, P.inv_norm_vx, P.div2 & kDiv2NormVx)); put(3, nvy(s[3]));
        put(4, tanh(P.k_theta_pso * (s[4] - Cst<R>::pi / R(2))));
    } else if (kind == 3) {
        put(0, ny((R)(float)s[1])); put(1, nvy((R)(float)s[3]));
        put(2, tanh((R)(P.f_k_theta_rl * ((float)s[4] - P.f_pi_2))));
        put(3, tanh((R)(P.f_k_thetad_rl * (float)s[5])));
        put(4, tanh((R)(P.f_k_gamma_rl * ((float)s[6] - P.f_pi_3_2))));
    } else if (kind == 4) {
        put(0, (R(1) - ny((R)(float)s[1])) * R(2) - R(1));
    } else {
        const int n = kind == 5 ? 4 : (kind == 6 ? 2 : 8);
        for (int k = 0; k < n; ++k) {
            int j = kind == 5 ? 4 + k : (kind == 6 ? 4 + k : (k < 6 ? k : k + 1));   // ascent skips gamma
            put(k, (R)(float)((R)(float)s[j] / P.norm_ph[k]));
        }
    }
}
template <typename R>
__device__ __forceinline__ void obs_write(DP<R>& P, int kind, const R* s, R* out, uint32_t idx) {
    const int d = obs_dim(kind);
    PD_AS1 char* o = (PD_AS1 char*)(uint64_t)out;
    obs_eval<R>(P, kind, s, [&](int k, R v) {
        *(PD_AS1 R*)(o + (uint32_t)(idx * (uint32_t)(d * sizeof(R)) + k * (uint32_t)sizeof(R))) = v;
    });
}

// ---------------------------------------------------------------- tables in LDS
// scipy interp1d._call_linear with fill_value='extrapolate' (grid_fin_aerodynamics.py:7-18)
// (slope: the intervals' slopes (y[i] - y[i-1]) / (x[i] - x[i-1]) at index i, tabulated with the
// same operation, or nullptr: computed here)
template <typename R>
__device__ __forceinline__ R grid_fin_ca(DP<R>& P, const R* sx, const R* sy, R mach, const uint16_t* lb = nullptr,
                                         const R* slope = nullptr) {
    if (mach < P.ca_min_mach) return P.ca_min_val;
    int n = P.ca_n;
    int lo = 0, hi = n;                       // lower_bound: first x >= mach
    if (lb != nullptr && mach >= R(0) && mach < R(10)) {   // within the Mach bucket's index range
        int b = (int)(mach * R(6.4));
        b = b > 63 ? 63 : b;
        const uint32_t rg = lb[b];
        lo = (int)(rg & 0xffu); hi = (int)(rg >> 8);
    }
    while (lo < hi) { int mid = (lo + hi) >> 1; if (sx[mid] < mach) lo = mid + 1; else hi = mid; }
    int idx = lo < 1 ? 1 : (lo > n - 1 ? n - 1 : lo);
    R xl = sx[idx - 1], yl = sy[idx - 1];
    const R sl = slope ? slope[idx] : (sy[idx] - yl) / (sx[idx] - xl);
    return sl * (mach - xl) + yl;
}

// np.interp for an in-range query (numpy compiled_base.c arr_interp)
// (slope: (y[j + 1] - y[j]) / (x[j + 1] - x[j]) tabulated at index j, or nullptr: computed here)
template <typename R>
__device__ __forceinline__ R np_interp(const R* x, const R* y, int n, R v, const R* slope = nullptr) {
    if (v < x[0]) return y[0];
    if (v >= x[n - 1]) return y[n - 1];
    int lo = 0, hi = n;                       // upper_bound: first x > v
    while (lo < hi) { int mid = (lo + hi) >> 1; if (x[mid] <= v) lo = mid + 1; else hi = mid; }
    int j = lo - 1;
    if (x[j] == v) return y[j];
    const R sl = slope ? slope[j] : (y[j + 1] - y[j]) / (x[j + 1] - x[j]);
    return sl * (v - x[j]) + y[j];
}

// grid_fin_aerodynamics.py:21-46: cn_alpha(M) * degrees(alpha)
template <typename R>
__device__ __forceinline__ R grid_fin_cn_alpha(DP<R>& P, const R* sx, const R* sy, R mach, const R* slope = nullptr) {
    if (mach < P.cn_min_mach) return P.cn_min_val;
    if (mach <= P.cn_max_mach) return np_interp(sx, sy, P.cn_n, mach, slope);
    return P.cn_max_val + P.cn_slope * (mach - P.cn_max_mach);
}

// ---------------------------------------------------------------- exact local-RBF aero
// Incremental 50-NN maintenance on the per-column Mach windows.  Within one AoA column the
// squared distance is convex in the Mach-sorted index, so a neighbourhood is one contiguous
// window per column; the 50-NN set is the unique window set with
//      max(included endpoint distance) <= min(adjacent excluded distance).
// Starting from the env's cached window set we swap (worst included) <-> (best adjacent
// excluded) until that holds; each swap strictly lowers the sum of included distances.
template <typename R> struct RbfCache {
    unsigned long long key;
    int slot;
};

template <typename R>
__device__ __forceinline__ R d2_at(const R* mach, int start, int i, R M, R dz) {
    R dm = M - mach[2 * (start + i)];   // (Mach, AoA) pairs in LDS
    return dm * dm + dz;
}

template <typename R>
__device__ __forceinline__ int knn_windows(const R* smach, const PD_AS4 int* start, const PD_AS4 int* n,
                                           const PD_AS4 R* aoa, R M, R a, int lo[kCols], int len[kCols]) {
    R dz[kCols];
#pragma unroll
    for (int c = 0; c < kCols; ++c) { R da = a - aoa[c]; dz[c] = da * da; }
    // each column's insertion point of M (lower_bound), searched the first time the column is
    // needed empty (its nearest candidates are then points ins - 1 and ins); -1: not yet
    int ins[kCols];
#pragma unroll
    for (int c = 0; c < kCols; ++c) ins[c] = -1;
    int it = 0;
    for (; it < 256; ++it) {
        R maxin = R(-1); int maxc = -1, maxi = 0;
        R minex = Cst<R>::inf; int minc = -1, mini = 0;
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
            if (len[c] > 0) {
                int l0 = lo[c], l1 = lo[c] + len[c] - 1;
                R da0 = d2_at(smach, start[c], l0, M, dz[c]);
                R da1 = d2_at(smach, start[c], l1, M, dz[c]);
                if (da0 > maxin) { maxin = da0; maxc = c; maxi = l0; }
                if (da1 > maxin) { maxin = da1; maxc = c; maxi = l1; }
                if (l0 > 0) { R d = d2_at(smach, start[c], l0 - 1, M, dz[c]); if (d < minex) { minex = d; minc = c; mini = l0 - 1; } }
                if (l1 + 1 < n[c]) { R d = d2_at(smach, start[c], l1 + 1, M, dz[c]); if (d < minex) { minex = d; minc = c; mini = l1 + 1; } }
            }
        }
        // empty columns: every point is at distance >= dz[c]; only columns that could hold a
        // point closer than the worst included one need their nearest point (binary search)
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
            if (len[c] == 0 && dz[c] < maxin) {
                if (ins[c] < 0) {
                    int l = 0, h = n[c];
                    while (l < h) { int mid = (l + h) >> 1; if (smach[2 * (start[c] + mid)] < M) l = mid + 1; else h = mid; }
                    ins[c] = l;
                }
                const int l = ins[c];
                if (l > 0) { R d = d2_at(smach, start[c], l - 1, M, dz[c]); if (d < minex) { minex = d; minc = c; mini = l - 1; } }
                if (l < n[c]) { R d = d2_at(smach, start[c], l, M, dz[c]); if (d < minex) { minex = d; minc = c; mini = l; } }
            }
        }
        if (!(maxin > minex)) break;          // also exits on NaN queries
        // add the best excluded point, then drop the worst included one
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
            if (c == minc) {
                if (len[c] == 0) { lo[c] = mini; len[c] = 1; }
                else if (mini < lo[c]) { lo[c] = mini; len[c] += 1; }
                else { len[c] += 1; }
            }
        }
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
            if (c == maxc) {
                if (maxi == lo[c]) { lo[c] += 1; len[c] -= 1; }
                else { len[c] -= 1; }
            }
        }
    }
    return it;
}

}  // namespace pd
