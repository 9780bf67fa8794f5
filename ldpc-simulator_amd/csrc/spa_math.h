// spa_math.h -- fp64 tanh / atanh of the check-node update, host+device.
//
// np_tanh  numpy 2.2.6's float64 tanh (the reference's np.tanh,
//          spa_decoder.py:145): 16 intervals selected from the exponent and
//          top mantissa bit of |x|, y = |x| - b[i], degree-16 Horner with
//          fused multiply-adds (c16 .. c0), |x| >= 24 -> 1, sign OR-ed back.
//          Bit-identical to np.tanh (tests/test_math.py), so the parked
//          t = tanh(M/2) values -- and with them P, q = P/t and the clip
//          decisions -- are the reference's own bits.  On the GPU the
//          coefficients sit in LDS as {b,c0},{c1,c2},...,{c15,c16} pairs:
//          9 ds_read_b128 + 16 v_fma_f64 per call.
// atanh_f  atanh for |q| <= CL (spa_decoder.py:167-168), our design:
//          |q| < 2^-5: odd Taylor polynomial; else the log form below.
//          (A table form, atanh(c) + atanh((a-c)/(1-ac)) at the centre c of
//          a's interval, had 25 % fewer VALU per call and was no faster in the
//          kernels -- latency-bound, more spills: profiles/r4n_ab; git history.)
//          The log form: atanh(a) = log(y)/2 with
//          y = (1+a)/(1-a) carried as a double-double (faithful quotient +
//          exact fma residual + the exact rounding errors of 1+a and 1-a), the
//          log from a 128-entry {1/c, -log(1/c)} table and a degree-8
//          polynomial (glibc-style reduction r = z/c - 1 by one fma).  About
//          0.51 ulp; it agrees with numpy's own arctanh on > 98% of inputs and
//          is faithful on all.
//          (numpy's arctanh is Intel SVML, which relies on x86-only
//          reciprocal approximations and cannot be restated portably.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "spa_math_tables.h"

namespace ldpc {

__host__ __device__ __forceinline__ uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double dfrom(uint64_t u) { return __builtin_bit_cast(double, u); }

struct alignas(16) Pair {
    double a, b;
};

// ----------------------------------------------------------------- tanh
// tab(p, i) returns {b, c0} for p = 0 and {c(2p-1), c(2p)} for p = 1..8.
template <class Tab>
__host__ __device__ __forceinline__ double np_tanh(double x, const Tab &tab) {
    const uint64_t ux = dbits(x);
    const uint64_t nd = ux & 0x7ff8000000000000ull;
    int hi = (int)(nd >> 32) - 0x3fc00000;
    hi = hi < 0 ? 0 : (hi > 0x780000 ? 0x780000 : hi);
    const int i = hi >> 19;
    const Pair p0 = tab(0, i);
    const double y = __builtin_fabs(x) - p0.a;
    Pair c = tab(8, i);
    double r = __builtin_fma(c.b, y, c.a);  // c16*y + c15
#pragma unroll
    for (int p = 7; p >= 1; --p) {
        c = tab(p, i);
        r = __builtin_fma(r, y, c.b);
        r = __builtin_fma(r, y, c.a);
    }
    r = __builtin_fma(r, y, p0.b);
    if (nd > 0x7fe0000000000000ull) r = 1.0;  // huge, inf (NaN -> 1 too; never reached here)
    return dfrom(dbits(r) | (ux & 0x8000000000000000ull));
}

// The check node's t = tanh(M/2) with the reference's clip (spa_decoder.py:
// 138-146: d = M/2; d > 17.5 -> CL, d < -17.5 -> -CL, else np.tanh(d)), as
// np_tanh of d clamped to +-17.5: np.tanh(17.5) == CL exactly and np_tanh is
// monotone across 17.5 (tests/test_math.py), so this equals the reference for
// every non-NaN M, and |x| <= 17.5 lets np_tanh skip its huge-argument select
// and the output clip.
template <class Tab>
__host__ __device__ __forceinline__ double tanh_half_clipped(double M, const Tab &tab);

// np_tanh of G independent arguments, Horner steps in lockstep across them:
// each argument gets exactly np_tanh's operations in np_tanh's order (so the
// results are bit-identical), but the G coefficient-table reads of a step are
// independent and can be in flight together instead of one dependent read per
// step of one chain.
// kSmall: every |x| <= 17.5 (tanh_half_clipped): the interval index needs no
// upper clamp and the huge-argument select never fires, so both are left out.
template <int G, class Tab, bool kSmall = false>
__host__ __device__ __forceinline__ void np_tanh_n(double (&x)[G], const Tab &tab) {
    int idx[G];
    double y[G], r[G], b0[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint64_t nd = dbits(x[g]) & 0x7ff8000000000000ull;
        int hi = (int)(nd >> 32) - 0x3fc00000;
        hi = hi < 0 ? 0 : (kSmall ? hi : (hi > 0x780000 ? 0x780000 : hi));
        idx[g] = hi >> 19;
        const Pair p0 = tab(0, idx[g]);
        y[g] = __builtin_fabs(x[g]) - p0.a;
        b0[g] = p0.b;
        const Pair c = tab(8, idx[g]);
        r[g] = __builtin_fma(c.b, y[g], c.a);  // c16*y + c15
    }
#pragma unroll
    for (int p = 7; p >= 1; --p) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const Pair c = tab(p, idx[g]);
            r[g] = __builtin_fma(r[g], y[g], c.b);
            r[g] = __builtin_fma(r[g], y[g], c.a);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint64_t ux = dbits(x[g]);
        double v = __builtin_fma(r[g], y[g], b0[g]);
        if (!kSmall && (ux & 0x7ff8000000000000ull) > 0x7fe0000000000000ull) v = 1.0;
        x[g] = dfrom(dbits(v) | (ux & 0x8000000000000000ull));
    }
}

// Evaluated on a = min(|M|, 35) = 2|d| clamped (exact): np_tanh's interval of
// a/2 is the exponent-and-top-mantissa field of a minus 2 (halving is exact
// for the normal a of intervals >= 1; below 2^-3 both give interval 0),
// y = |d| - b as fma(a, 0.5, -b) (one rounding either way: a*0.5 is exact
// wherever b != 0, and b = 0 in interval 0), and the sign of M OR-ed back.
// Same operations on the same values as np_tanh(clamped d) from the first
// fma on, so bit-identical (tests/test_math.py), in 6 fewer VALU.  (tile8.hip
// runs this form; tile_sub.hip keeps np_tanh_n<.., kSmall> of the clamped
// d, which spills less there: 0.453 vs 0.437 at 1 dB.)
template <class Tab>
__host__ __device__ __forceinline__ double tanh_half_clipped(double M, const Tab &tab) {
    const double a = __builtin_fmin(__builtin_fabs(M), 35.0);
    const uint32_t e = (uint32_t)(dbits(a) >> 32) >> 19;  // 12 bits: a >= 0
    const int i = (int)__builtin_elementwise_sub_sat(e, 0x7fau);  // 0 .. 14
    const Pair p0 = tab(0, i);
    const double y = __builtin_fma(a, 0.5, -p0.a);
    Pair c = tab(8, i);
    double r = __builtin_fma(c.b, y, c.a);  // c16*y + c15
#pragma unroll
    for (int p = 7; p >= 1; --p) {
        c = tab(p, i);
        r = __builtin_fma(r, y, c.b);
        r = __builtin_fma(r, y, c.a);
    }
    r = __builtin_fma(r, y, p0.b);
    return dfrom(dbits(r) | (dbits(M) & 0x8000000000000000ull));
}

// ----------------------------------------------------------------- log
constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;  // 11 trailing zero bits: k*kLn2Hi exact
constexpr double kLn2Lo = 0x1.ef35793c76730p-45;

struct LogEntry {
    double invc, hi, lo;
};

// Polynomial coefficients of log_hilo / atanh_f.  Kernels take a copy as a
// kernel argument: the values then live in SGPRs and feed v_fma_f64 directly
// (gfx950 VOP3 has no 64-bit literals, so literal coefficients are copied into
// VGPRs before every use -- two v_mov each, per edge).  Same values either way.
struct AtanhCoef {
    double t15, t13, t11, t9, t7, t5, t3;  // atanh Taylor: 1/15 .. 1/3
    double l8, l7, l6, l5, l4, l3, l2;    // log1p(r) - r: -1/8, 1/7, -1/6, 1/5, -1/4, 1/3, -1/2
    double ln2hi, ln2lo;
};
constexpr AtanhCoef kAtanhCoef{1.0 / 15.0, 1.0 / 13.0, 1.0 / 11.0, 1.0 / 9.0, 1.0 / 7.0, 0.2, 1.0 / 3.0,
                               -0.125, 0x1.2492492492492p-3, -0x1.5555555555555p-3, 0x1.999999999999ap-3,
                               -0.25, 0x1.5555555555555p-2, -0.5,
                               kLn2Hi, kLn2Lo};

// log(x) = hi + lo for a positive normal x.  Accurate away from x ~ 1 (the
// interval holding 1.0 itself is exact: invc = 1), which is all atanh needs.
template <class LogTab>
__host__ __device__ __forceinline__ void log_hilo(double x, const LogTab &lt, double &hi, double &lo,
                                                  const AtanhCoef &c = kAtanhCoef) {
    // glibc-style reduction on the high word only (the offset's low word is 0,
    // so no borrow): tmp = hi(x) - hi(OFF); 32-bit integer ops throughout.
    const uint64_t ix = dbits(x);
    const int tmp = (int)(uint32_t)(ix >> 32) - 0x3fe60000;
    const int i = (tmp >> 13) & 127;
    const int k = tmp >> 20;  // arithmetic shift
    const double z = dfrom(ix - ((uint64_t)(uint32_t)(tmp & 0xfff00000) << 32));
    const LogEntry t = lt(i);
    const double r = __builtin_fma(z, t.invc, -1.0);  // |r| < 2^-7
    const double kd = (double)k;
    const double w = __builtin_fma(kd, c.ln2hi, t.hi);  // exact
    hi = w + r;
    const double r2 = r * r;
    // log1p(r) - r, Taylor to r^8
    double p = __builtin_fma(r, c.l8, c.l7);  // -1/8, 1/7
    p = __builtin_fma(p, r, c.l6);            // -1/6
    p = __builtin_fma(p, r, c.l5);            // 1/5
    p = __builtin_fma(p, r, c.l4);            // -1/4
    p = __builtin_fma(p, r, c.l3);            // 1/3
    p = __builtin_fma(p, r, c.l2);            // -1/2
    lo = ((w - hi) + r) + (__builtin_fma(kd, c.ln2lo, t.lo) + r2 * p);
}

// ~1-ulp reciprocal (v_rcp_f64); only used where the result is corrected or
// multiplies a tiny correction term.
__host__ __device__ __forceinline__ double fast_rcp(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(d);
#else
    return 1.0 / d;
#endif
}

// atanh(a) for 0 <= a < 2^-5: odd Taylor polynomial (the small branch of atanh_f)
__host__ __device__ __forceinline__ double atanh_small_abs(double a, const AtanhCoef &c = kAtanhCoef) {
    const double a2 = a * a;
    double p = __builtin_fma(a2, c.t13, c.t11);
    p = __builtin_fma(p, a2, c.t9);
    p = __builtin_fma(p, a2, c.t7);
    p = __builtin_fma(p, a2, c.t5);
    p = __builtin_fma(p, a2, c.t3);
    return __builtin_fma(a * a2, p, a);
}
constexpr double kAtanhSmall = 0x1p-5;  // atanh_f's Taylor / log switch
// Below 2^-27 the Taylor branch returns its argument: fma(a*a2, p, a) adds
// a^3/3 < ulp(a)/6 to a, which rounds back to a.  So atanh_f(q) == q bit for
// bit for |q| < kAtanhIdent (tests/test_math.py), and a check node whose
// quotients are all that small (long rows at low SNR: the product of ~576
// values of |t| < 1) forms E_new = 2q with no atanh and no clip.
constexpr double kAtanhIdent = 0x1p-27;

// atanh(q) for |q| < 2^-5 only; equals atanh_f(q) bit for bit there
__host__ __device__ __forceinline__ double atanh_small(double q, const AtanhCoef &c = kAtanhCoef) {
    const double res = atanh_small_abs(__builtin_fabs(q), c);
    return dfrom(dbits(res) | (dbits(q) & 0x8000000000000000ull));
}

// atanh(q) for |q| <= CL.
template <class LogTab>
__host__ __device__ __forceinline__ double atanh_f(double q, const LogTab &lt, const AtanhCoef &c = kAtanhCoef) {
    const double a = __builtin_fabs(q);
    double res;
    if (a < kAtanhSmall) {
        res = atanh_small_abs(a, c);
    } else {
        // atanh(a) = log(y)/2, y = (1+a)/(1-a) carried as y_hi + y_lo:
        // u = 1+a and v = 1-a are rounded, their errors cu, cv exact (u-1, v-1
        // exact); y_hi = faithful u/v (rcp + one Newton step), its residual
        // u - y_hi*v exact by fma; y_lo/y_hi ~= (rem + cu - y_hi*cv)/u.
        const double u = 1.0 + a, v = 1.0 - a;
        const double cu = a - (u - 1.0);   // exact
        const double cv = -a - (v - 1.0);  // exact; 0 for a >= 0.5
        const double rv = fast_rcp(v);
        const double y0 = u * rv;
        const double yh = __builtin_fma(__builtin_fma(-y0, v, u), rv, y0);
        const double rem = __builtin_fma(-yh, v, u);
        const double corr = __builtin_fma(-yh, cv, rem + cu) * fast_rcp(u);
        double h, l;
        log_hilo(yh, lt, h, l, c);
        res = 0.5 * (h + (l + corr));
    }
    return dfrom(dbits(res) | (dbits(q) & 0x8000000000000000ull));
}

// Host-side table views (tests, host build of this header).
struct HostTanhTab {
    __host__ Pair operator()(int p, int i) const {
        if (p == 0) return {dfrom(tab::kTanhB[i]), dfrom(tab::kTanhC[0][i])};
        return {dfrom(tab::kTanhC[2 * p - 1][i]), dfrom(tab::kTanhC[2 * p][i])};
    }
};
struct HostLogTab {
    __host__ LogEntry operator()(int i) const {
        return {dfrom(tab::kLog[i][0]), dfrom(tab::kLog[i][1]), dfrom(tab::kLog[i][2])};
    }
};
using HostAtanhTab = HostLogTab;  // the table atanh_f reads

}  // namespace ldpc
