// pd_common.h -- host+device helpers of libpdenv (product code; independent of oracle/).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PD_HD __host__ __device__ __forceinline__

namespace pd {

constexpr int kNbr = 50;            // RBFInterpolator(neighbors=50), aerodynamic_coefficients.py:59
constexpr int kSys = kNbr + 3;      // + degree-1 polynomial tail (TPS default degree)
constexpr int kCols = 5;            // AoA columns of each V2 table
// Payload of one neighbourhood (binary64 words).  The 50 terms are stored as 25 pair slots:
// a window of consecutive table points (one column's Mach run) is cut into pairs (p, p + 1), so
// that one 16-byte LDS read (the point table holds (Mach_p, Mach_p+1) per entry) serves two
// terms that share the column's AoA.  50 points in <= 5 windows leave an even number (<= 4) of
// odd windows; their last points are paired across columns ("cross" slots, two points with their
// own entries and AoAs).  Slot 5c + 4 (the last of each chunk of five) is a general slot whose
// second point has its own index bytes: cross slot x sits at 5x + 4, the window pairs fill the
// other positions in order (see slot_of_pair).  Five chunks of five slots, no padding.
//   [0, 50)   coefficients, slot k at 2k, 2k + 1
//   [50, 53)  degree-1 polynomial coefficients
//   [53, 57)  shift0, shift1, scale0, scale1
//   [57, 65)  60 index bytes, 12 per chunk: per slot its first point's entry and the column's
//             integer AoA (pair_entry_pos / pair_aoa_pos), then the general slot's second point
//             (entry, AoA) at second_entry_pos / second_aoa_pos
//   [65]      padding (16-byte stride)
constexpr int kChunks = 5;       // chunks of five slots (ten terms) per payload
constexpr int kPairs = 5 * kChunks;
constexpr int kPairsUsed = kPairs;
constexpr int kPayPoly = 2 * kPairs;
constexpr int kPaySS = kPayPoly + 3;
constexpr int kPayIdx = kPaySS + 4;
constexpr int kPayIdxBytes = 12 * kChunks;
constexpr int kPay = (kPayIdx + (kPayIdxBytes + 7) / 8 + 1) & ~1;
// Byte positions in the index area: slot 5c + u (chunk c of five) at 12c + 2u (entry) and
// 12c + 2u + 1 (AoA); the chunk's general slot (u = 4) has its second point at 12c + 10 / 11, so
// that a chunk's twelve bytes are one 3-dword load issued with its ten coefficients.
PD_HD constexpr int pair_entry_pos(int k) { return 12 * (k / 5) + 2 * (k % 5); }
PD_HD constexpr int pair_aoa_pos(int k) { return pair_entry_pos(k) + 1; }
PD_HD constexpr bool slot_general(int k) { return k % 5 == 4; }
PD_HD constexpr int second_entry_pos(int k) { return 12 * (k / 5) + 10; }
PD_HD constexpr int second_aoa_pos(int k) { return 12 * (k / 5) + 11; }
// Slot of the np-th window pair when nx cross slots take the general positions 4, 9, ... first.
PD_HD int slot_of_pair(int np, int nx) {
    int cnt = -1;
    for (int k = 0; k < kPairs; ++k) {
        if (slot_general(k) && k / 5 < nx) continue;
        if (++cnt == np) return k;
    }
    return -1;
}
// Where term t of a neighbourhood's window order (columns in order, Mach-sorted within) goes:
// slot k and position i (coefficient 2k + i).  len: the five window lengths.
PD_HD void term_slot(const int len[kCols], int t, int& k, int& i) {
    int acc = 0, np = 0, nodd = 0, nx = 0;
    for (int c = 0; c < kCols; ++c) nodd += len[c] & 1;
    nx = nodd / 2;
    int odd_before = 0;
    for (int c = 0; c < kCols; ++c) {
        if (t < acc + len[c]) {
            const int off = t - acc;
            if (off < (len[c] & ~1)) { k = slot_of_pair(np + off / 2, nx); i = off & 1; }
            else { k = 5 * (odd_before / 2) + 4; i = odd_before & 1; }
            return;
        }
        acc += len[c];
        np += len[c] / 2;
        odd_before += len[c] & 1;
    }
    k = -1; i = 0;
}
constexpr int kKeyLoBits = 6, kKeyLenBits = 6, kKeyField = kKeyLoBits + kKeyLenBits;
constexpr uint64_t kEmptyKey = ~0ull;

// CPython math.radians / math.degrees: x * (pi/180), x * (180/pi)
constexpr double kPi = 3.141592653589793;
constexpr double kDeg2Rad = kPi / 180.0;
constexpr double kRad2Deg = 180.0 / kPi;

PD_HD uint64_t key_pack(const int lo[kCols], const int len[kCols]) {
    uint64_t k = 0;
    for (int c = 0; c < kCols; ++c) {
        uint64_t f = (uint64_t)(len[c] > 0 ? lo[c] : 0) | ((uint64_t)len[c] << kKeyLoBits);
        k |= f << (kKeyField * c);
    }
    return k;
}
PD_HD void key_unpack(uint64_t k, int lo[kCols], int len[kCols]) {
    for (int c = 0; c < kCols; ++c) {
        uint64_t f = (k >> (kKeyField * c)) & ((1ull << kKeyField) - 1);
        lo[c] = (int)(f & ((1u << kKeyLoBits) - 1));
        len[c] = (int)(f >> kKeyLoBits);
    }
}
PD_HD uint32_t key_hash(uint64_t k, int log2cap) {
    return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - log2cap));
}

// Natural log for the neighbourhood solves, evaluated with plain IEEE arithmetic only so that
// the host-built and the device-built (wave-cooperative) payloads are bit-identical; libm's and
// the device library's log differ in the last ulp.  Classic argument reduction
// x = 2^k (1 + f), sqrt(2)/2 <= 1+f < sqrt(2); s = f / (2 + f); log(1+f) = f - hfsq + s (hfsq + R(s^2))
// with the degree-14 minimax R of the public-domain fdlibm e_log.c; error < 1 ulp.
// Valid for positive normal finite x (distances between distinct table points).
PD_HD double pd_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t bits;
    __builtin_memcpy(&bits, &x, 8);
    int32_t hx = (int32_t)(bits >> 32);
    int k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    bits = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (bits & 0xffffffffull);
    double xn;
    __builtin_memcpy(&xn, &bits, 8);
    k += i >> 20;
    double f = xn - 1.0;
    double dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    double s = f / (2.0 + f);
    double z = s * s;
    int32_t i2 = hx - 0x6147a;
    double w = z * z;
    int32_t j = 0x6b851 - hx;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i2 |= j;
    double R = t2 + t1;
    if (i2 > 0) {
        double hfsq = 0.5 * f * f;
        return k == 0 ? f - (hfsq - s * (hfsq + R)) : dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    return k == 0 ? f - s * (f - R) : dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

PD_HD double tps(double r) { return r == 0.0 ? 0.0 : r * r * pd_log(r); }

// Table-driven natural log for the RBF evaluation (the hot transcendental: 200 per lane per
// env-step).  x = 2^e m, m in [1, 2); the top 9 mantissa bits pick a cell with rounded inverse
// centre invc and logc = -log(invc); r = m * invc - 1 (one fma, |r| < 2^-9.9) and
// log x = e ln2 + logc + log1p(r), log1p to degree 5 (truncation < 2e-19).  Absolute error
// below 5e-16 over the RBF's argument range (host-checked against long double); a third of
// the device library's double log.  Positive normal finite x; x = 0 gives a finite value.
constexpr int kLogBits = 9, kLogCells = 1 << kLogBits;
struct LogTable { double invc[kLogCells], logc[kLogCells]; };
// The step kernel's hot-path log (eval_log, pd_physics.h): 1024 cells of (2 invc, 4 (-log(invc) -
// ln 2)), interleaved for one 16-byte LDS read, used with frexp's mantissa in [0.5, 1) and a
// degree-4 log1p (|r| < 2^-11, truncation < 6e-18); same accuracy as log_tab (max 1.4e-15
// absolute over [1e-6, 300] against long double, 2e7 arguments), fewer instructions.  The
// second entry is scaled by 4 (exactly) so that the Horner steps run on 4 log1p and every FMA
// has at most one non-inline constant (pd_physics.h log_cell_poly4).
constexpr int kLogBitsD = 10, kLogCellsD = 1 << kLogBitsD;
struct alignas(16) LogTableD { double cell[2 * kLogCellsD]; };   // (16-byte aligned: the step kernel copies it with 16-byte loads)
inline void log_table_fill(LogTableD& t) {
    for (int i = 0; i < kLogCellsD; ++i) {
        long double c = 1.0L + (i + 0.5L) / kLogCellsD;
        double invc = (double)(1.0L / c);
        t.cell[2 * i] = 2.0 * invc;
        t.cell[2 * i + 1] = 4.0 * (double)(-logl((long double)invc) - logl(2.0L));
    }
}
inline void log_table_fill(LogTable& t) {
    for (int i = 0; i < kLogCells; ++i) {
        long double c = 1.0L + (i + 0.5L) / kLogCells;
        double invc = (double)(1.0L / c);
        t.invc[i] = invc;
        t.logc[i] = (double)(-logl((long double)invc));
    }
}
// S: element stride of the cell arrays (the device keeps (invc, logc) interleaved, S = 2)
// log x from x = 2^e m and the cell's (invc, logc)
PD_HD double log_tab_finish(double m, double e, double invc, double logc) {
    const double ln2 = 6.93147180559945286227e-01;
    double r = fma(m, invc, -1.0);
    double t = fma(r, 0.2, -0.25);
    t = fma(r, t, 1.0 / 3.0);
    t = fma(r, t, -0.5);
    double p = fma(r * r, t, r);
    return fma(e, ln2, logc + p);
}
template <int S = 1>
PD_HD double log_tab(double x, const double* invc, const double* logc) {
    uint64_t b;
    __builtin_memcpy(&b, &x, 8);
    uint32_t hi = (uint32_t)(b >> 32);
    double e = (double)((int)(hi >> 20) - 1023);
    uint32_t i = (hi >> (20 - kLogBits)) & (kLogCells - 1);
    uint64_t mb = (b & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m;
    __builtin_memcpy(&m, &mb, 8);
    return log_tab_finish(m, e, invc[S * i], logc[S * i]);
}

// Build and solve the thin-plate-spline system of ONE 50-point neighbourhood, exactly the
// system scipy's RBFInterpolator builds (scipy/interpolate/_rbfinterp.py _build_system:
// shift=(min+max)/2, scale=(max-min)/2 (0->1), K_ij = r^2 log r, P = [1, (y-shift)/scale],
// [[K, P], [P^T, 0]] c = [d, 0]) and solve it by LU with partial pivoting (LAPACK dgesv's
// algorithm).  Points are taken in window order (column by column, Mach-ascending).
//   mach/coef: table arrays (column-grouped); col_start/col_aoa: column geometry
//   work: >= kSys*kSys + kSys + 3*kNbr doubles of scratch;  payload: kPay doubles out in the
//   pair-slot layout above (column AoAs must be integers in [0, 255], checked by pd_create).
// Returns 0 on success, -1 on a singular system.
PD_HD int solve_neighbourhood(const double* mach, const double* coef, const int* col_start,
                              const double* col_aoa, uint64_t key, double* work, double* payload) {
    int lo[kCols], len[kCols];
    key_unpack(key, lo, len);
    double* A = work;
    double* b = A + kSys * kSys;
    double* ym = b + kSys;
    double* ya = ym + kNbr;
    double* yd = ya + kNbr;
    int n = 0;
    uint8_t idx[kNbr];
    for (int c = 0; c < kCols; ++c)
        for (int i = 0; i < len[c]; ++i) {
            if (n >= kNbr) return -1;
            idx[n] = (uint8_t)(col_start[c] + lo[c] + i);
            ym[n] = mach[col_start[c] + lo[c] + i];
            ya[n] = col_aoa[c];
            yd[n] = coef[col_start[c] + lo[c] + i];
            ++n;
        }
    if (n != kNbr) return -1;
    double mn0 = ym[0], mx0 = ym[0], mn1 = ya[0], mx1 = ya[0];
    for (int j = 1; j < kNbr; ++j) {
        mn0 = ym[j] < mn0 ? ym[j] : mn0; mx0 = ym[j] > mx0 ? ym[j] : mx0;
        mn1 = ya[j] < mn1 ? ya[j] : mn1; mx1 = ya[j] > mx1 ? ya[j] : mx1;
    }
    double sh0 = (mx0 + mn0) / 2, sc0 = (mx0 - mn0) / 2, sh1 = (mx1 + mn1) / 2, sc1 = (mx1 - mn1) / 2;
    if (sc0 == 0.0) sc0 = 1.0;
    if (sc1 == 0.0) sc1 = 1.0;
    for (int i = 0; i < kNbr; ++i) {
        for (int j = 0; j < kNbr; ++j) {
            double d0 = ym[i] - ym[j], d1 = ya[i] - ya[j];
            A[i * kSys + j] = tps(sqrt(d0 * d0 + d1 * d1));
        }
        double h0 = (ym[i] - sh0) / sc0, h1 = (ya[i] - sh1) / sc1;
        A[i * kSys + kNbr] = 1.0; A[i * kSys + kNbr + 1] = h0; A[i * kSys + kNbr + 2] = h1;
        A[kNbr * kSys + i] = 1.0; A[(kNbr + 1) * kSys + i] = h0; A[(kNbr + 2) * kSys + i] = h1;
        b[i] = yd[i];
    }
    for (int i = kNbr; i < kSys; ++i) {
        for (int j = kNbr; j < kSys; ++j) A[i * kSys + j] = 0.0;
        b[i] = 0.0;
    }
    for (int k = 0; k < kSys; ++k) {
        int p = k;
        double best = fabs(A[k * kSys + k]);
        for (int i = k + 1; i < kSys; ++i) {
            double v = fabs(A[i * kSys + k]);
            if (v > best) { best = v; p = i; }
        }
        if (best == 0.0) return -1;
        if (p != k) {
            for (int j = 0; j < kSys; ++j) { double t = A[k * kSys + j]; A[k * kSys + j] = A[p * kSys + j]; A[p * kSys + j] = t; }
            double t = b[k]; b[k] = b[p]; b[p] = t;
        }
        double r = 1.0 / A[k * kSys + k];
        for (int i = k + 1; i < kSys; ++i) {
            double l = A[i * kSys + k] * r;
            if (l != 0.0)
                for (int j = k + 1; j < kSys; ++j) A[i * kSys + j] -= l * A[k * kSys + j];
            b[i] -= l * b[k];
        }
    }
    // column-oriented back substitution (the device's wave-cooperative solve does the same
    // operations in the same order, so host-built and device-built payloads agree bit-for-bit)
    for (int i = kSys - 1; i >= 0; --i) {
        double xi = b[i] / A[i * kSys + i];
        b[i] = xi;
        for (int r = 0; r < i; ++r) b[r] -= A[r * kSys + i] * xi;
    }
    for (int j = 0; j < kPay; ++j) payload[j] = 0.0;
    uint8_t* ib = (uint8_t*)(payload + kPayIdx);
    int t = 0;
    for (int c = 0; c < kCols; ++c)
        for (int i = 0; i < len[c]; ++i, ++t) {
            int k, pos;
            term_slot(len, t, k, pos);
            if (k < 0) return -1;
            payload[2 * k + pos] = b[t];
            if (pos == 0) { ib[pair_entry_pos(k)] = idx[t]; ib[pair_aoa_pos(k)] = (uint8_t)col_aoa[c]; }
            else if (slot_general(k)) { ib[second_entry_pos(k)] = idx[t]; ib[second_aoa_pos(k)] = (uint8_t)col_aoa[c]; }
        }
    for (int j = 0; j < 3; ++j) payload[kPayPoly + j] = b[kNbr + j];
    payload[kPaySS + 0] = sh0; payload[kPaySS + 1] = sh1;
    payload[kPaySS + 2] = sc0; payload[kPaySS + 3] = sc1;
    return 0;
}

// Payload in a handle's precision: coefficients converted, index bytes copied.  Stride in R
// units: kPay = 66 (binary64) or 72 (binary32: 57 values + 60 bytes = 15 floats, 16-byte stride).
template <typename R> constexpr int pay_stride() { return sizeof(R) == 8 ? kPay : 72; }
template <typename R> PD_HD void pay_store(const double* src, R* dst) {
    for (int j = 0; j < kPayIdx; ++j) dst[j] = (R)src[j];
    for (int j = kPayIdx; j < pay_stride<R>(); ++j) dst[j] = R(0);
    __builtin_memcpy((uint8_t*)(dst + kPayIdx), (const uint8_t*)(src + kPayIdx), kPayIdxBytes);
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };
PD_HD u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        u32x4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c;
}
// 53-bit uniform in [0, 1)
PD_HD double u01(uint32_t hi, uint32_t lo) {
    return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6)) * (1.0 / 9007199254740992.0);
}
// Philox purpose tags (4th counter word)
constexpr uint32_t kTagWindSub = 0;   // +substep 0..3
constexpr uint32_t kTagReset = 16;
constexpr uint32_t kTagTilt = 17;
constexpr uint32_t kTagProf = 18;      // the wind percentile (its own draw: independent of the sigmas)
constexpr uint32_t kTagSacEps = 19;    // +a/2: pd_step_sac_ring's rsample noise of action components a, a+1
// randint(50, 99) - 50 from one Philox word: floor(49 u / 2^32) (multiply-shift; bias < 1.2e-8)
PD_HD int prof_draw(uint32_t u) { return (int)(((uint64_t)u * 49u) >> 32); }

// ---------------------------------------------------------------- sine and cosine together
// Binary64 sin and cos of one angle in one pass: reduction by pi/2 to a double-double r + y
// (the first fma term is exact for |k| < 2^20; beyond 1e6 rad, the library), then the
// public-domain fdlibm kernels k_sin.c / k_cos.c with their tail argument, and a quadrant swap.
// <= 1 ulp against long double over 2e7 arguments.  Only IEEE +, *, fma and rint: the host and
// the device give the same bits (the wind normals below rely on that).
PD_HD void sincos_fd(double x, double& s, double& c) {
    if (!(fabs(x) < 1.0e6)) { s = sin(x); c = cos(x); return; }   // huge or NaN
    const double k = rint(x * 6.36619772367581382433e-01);
    const double r1 = fma(-k, 1.57079632679489655800e+00, x);      // exact for |k| < 2^20
    const double ph = k * 6.12323399573676603587e-17;               // k (pi/2 - high), two terms
    const double pl = fma(k, 6.12323399573676603587e-17, -ph) + k * -1.4973849048591698e-33;
    const double r = r1 - ph;                                       // reduced angle r + y
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
    s = q == 0 ? sn : (q == 1 ? cs : (q == 2 ? -sn : -cs));
    c = q == 0 ? cs : (q == 1 ? -sn : (q == 2 ? -cs : sn));
}

// atan2(y, x) in binary64: fdlibm's e_atan2.c / s_atan.c (public domain; the same reduction
// intervals, polynomial and atan(c) hi/lo pairs) with the ratio and its reduction fused into ONE
// division: for t = |y/x| in interval id, atan(t) = atan(c_id) + atan(N/D) with
//   id -1 (t < 7/16)        N = |y|,               D = |x|
//   id 0  (t < 11/16)       N = 2|y| - |x|,        D = 2|x| + |y|          (c = 1/2)
//   id 1  (t < 19/16)       N = |y| - |x|,         D = |y| + |x|           (c = 1)
//   id 2  (t < 39/16)       N = fma(-1.5, |x|, |y|), D = fma(1.5, |y|, |x|) (c = 3/2)
//   id 3                    N = -|x|,              D = |y|                 (c = inf)
// (fdlibm divides y/x first and then reduces the rounded ratio: a second division and one more
// rounding; the numerators above are exact by Sterbenz's lemma or one fused rounding).  Then
// fdlibm's quadrant rule.  <= 1 ulp against glibc's atan2 (tests/test_atan2.py, 4e6 arguments
// over the descent's range and beyond); about half the device library's instructions.  Zeros,
// infinities and NaNs take the library atan2.
PD_HD double atan2_fd(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    if (!(ax > 0.0 && ay > 0.0 && ax < __builtin_huge_val() && ay < __builtin_huge_val())) return atan2(y, x);
    const int id = ay < 0.4375 * ax ? -1 : (ay < 0.6875 * ax ? 0 : (ay < 1.1875 * ax ? 1 : (ay < 2.4375 * ax ? 2 : 3)));
    double n, d, hi, lo;
    if (id < 0) { n = ay; d = ax; hi = 0.0; lo = 0.0; }
    else if (id == 0) { n = 2.0 * ay - ax; d = 2.0 * ax + ay; hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
    else if (id == 1) { n = ay - ax; d = ay + ax; hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
    else if (id == 2) { n = fma(-1.5, ax, ay); d = fma(1.5, ay, ax); hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
    else { n = -ax; d = ay; hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
    const double t = n / d;
    // the quotient's rounding error, (n - t d) / d (exact remainder by one FMA; the reciprocal
    // only needs a few bits: the term is below half an ulp of t)
    const double et = fma(-t, d, n) * (1.0 / d);
    const double z = t * t, w = z * z;
    const double s1 = z * (3.33333333333329318027e-01 + w * (1.42857142725034663711e-01 + w * (9.09088713343650656196e-02 +
                      w * (6.66107313738753120669e-02 + w * (4.97687799461593236017e-02 + w * 1.62858201153657823623e-02)))));
    const double s2 = w * (-1.99999999998764832476e-01 + w * (-1.11111104054623557880e-01 + w * (-7.69187620504482999495e-02 +
                      w * (-5.83357013379057348645e-02 + w * -3.65315727442169155270e-02))));
    // atan(|y / x|) = hi + t + (lo + et - t (s1 + s2)) as a double-double (ah, al): hi + t by
    // TwoSum, the small terms added to its error
    const double sh = hi + t, sb = sh - hi;
    const double se = (hi - (sh - sb)) + (t - sb);
    const double small = se + ((lo + et) - t * (s1 + s2));
    const double ah = sh + small, al = small - (ah - sh);
    const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
    if (x > 0.0) return y > 0.0 ? ah + al : -(ah + al);
    // x < 0: pi - atan (y > 0) or atan - pi (y < 0), again as TwoSum + the low parts
    const double ph = pi - ah, pb = ph - pi;
    const double pe = (pi - (ph - pb)) + (-ah - pb);
    const double r = ph + (pe + (pi_lo - al));
    return y > 0.0 ? r : -r;
}

// Two standard normals from one Philox4x32-10 block by Box-Muller in binary64:
// u1 = 1 - u01(x, y) in (0, 1], u2 = u01(z, w); rho = sqrt(-2 log u1); (rho cos 2 pi u2,
// rho sin 2 pi u2).  The log is log_tab (cell table from log_table_fill), sqrt is correctly
// rounded, sincos_fd is IEEE-only: the oracle restates this and draws the same bits.  The
// wind gusts (vonkarman.py:34, one np.random.randn() per filter step) and the tilt use it.
template <int S = 1>
PD_HD void gauss_pair(u32x4 r, const double* invc, const double* logc, double& z0, double& z1) {
    const double u1 = 1.0 - u01(r.x, r.y), u2 = u01(r.z, r.w);
    const double rho = sqrt(-2.0 * log_tab<S>(u1, invc, logc));
    double s, c;
    sincos_fd(6.283185307179586 * u2, s, c);
    z0 = rho * c;
    z1 = rho * s;
}

}  // namespace pd
