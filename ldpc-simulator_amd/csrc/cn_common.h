// cn_common.h -- device pieces shared by the parity-mode check-node kernels
// (spa_kernels.hip: cn_kernel / cn_row_kernel / cn_rare_kernel;
// tile_kernels.hip: the tile-resident decoder): the reference's clip constants,
// numpy's tanh with its coefficient table staged in LDS, and the atanh table.
#pragma once
#include <hip/hip_runtime.h>

#include "spa_math.h"

namespace ldpc {
namespace {

constexpr double kCL = 0.99999999999999878;  // spa_decoder.py:141,167
constexpr double kTiny = 1e-10;              // spa_decoder.py:159
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// np.clip(q, -CL, CL) as v_max_f64 + v_min_f64 (2 VALU instead of 2 compares
// and 4 selects).  Differs from np.clip only for NaN, which a message cannot
// be for finite or infinite channel LLRs (|t| <= 1, |E| <= 35.04).
__device__ __forceinline__ double clip_cl(double q) { return fmin(fmax(q, -kCL), kCL); }

// P / t as the compiler's own f64 division sequence (reciprocal, two Newton
// steps, quotient, one fma correction -- the operations v_div_fmas_f64 and
// v_div_fixup_f64 wrap) without v_div_scale_f64 / v_div_fmas / v_div_fixup.
// Those only act on operands that need scaling or on special values, so the
// result is the IEEE quotient, bit for bit, whenever t is normal with
// |t| < 1 (every t of a non-rare row: 1e-10 < |t| <= CL) and |P| >= 2^-900
// (callers check the latter per wavefront and divide normally otherwise).
constexpr double kDivNrMin = 0x1p-900;
__device__ __forceinline__ double div_nr(double P, double t) {
    const double r0 = __builtin_amdgcn_rcp(t);
    const double r1 = __builtin_fma(r0, __builtin_fma(-t, r0, 1.0), r0);
    const double r2 = __builtin_fma(r1, __builtin_fma(-t, r1, 1.0), r1);
    const double q = P * r2;
    return __builtin_fma(__builtin_fma(-t, q, P), r2, q);
}
// whether every lane of the wavefront may take div_nr for numerator P
__device__ __forceinline__ bool div_nr_ok(double P) {
    return __ballot(!(__builtin_fabs(P) >= kDivNrMin)) == 0ull;
}

// ---- math tables in LDS: 9 x 16 tanh pairs + atanh_f's log table (128
// entries padded to 32 B: 4 KB)
struct LdsTanh {
    const Pair *p;
    __device__ __forceinline__ Pair operator()(int pp, int i) const { return p[pp * 16 + i]; }
};
struct alignas(16) LogEntry4 {
    double invc, hi, lo, pad;
};
struct LdsAtanh {
    const LogEntry4 *e;
    __device__ __forceinline__ LogEntry operator()(int i) const {
        const LogEntry4 v = e[i];
        return {v.invc, v.hi, v.lo};
    }
};
struct MathLds {
    Pair tanh[9 * 16];
    LogEntry4 atanh[128];
};

__device__ __forceinline__ void fill_math_lds(MathLds &m) {
    for (int k = threadIdx.x; k < 9 * 16; k += blockDim.x) {
        const int pp = k >> 4, i = k & 15;
        m.tanh[k] = pp == 0 ? Pair{dfrom(tab::kTanhB[i]), dfrom(tab::kTanhC[0][i])}
                            : Pair{dfrom(tab::kTanhC[2 * pp - 1][i]), dfrom(tab::kTanhC[2 * pp][i])};
    }
    for (int i = threadIdx.x; i < 128; i += blockDim.x)
        m.atanh[i] = {dfrom(tab::kLog[i][0]), dfrom(tab::kLog[i][1]), dfrom(tab::kLog[i][2]), 0.0};
}

// t = tanh(M/2) with the reference's clip (:138-146) applied to the output:
// np.tanh(17.5) == CL and np.tanh is monotone across +-17.5, so
// clip(np_tanh(d), -CL, CL) is the input clip bit for bit (tests/test_math.py).
// (The clamped-input form, spa_math.h tanh_half_clipped, has fewer VALU but
// makes cn_row_kernel and tile_kernel spill; tile_sub.hip and tile8.hip use it.)
__device__ __forceinline__ double cn_tanh(double M, const LdsTanh &t) { return clip_cl(np_tanh(M * 0.5, t)); }

// atanh_f's 16 polynomial / log2 coefficients in constant memory, loaded with
// two s_load_dwordx16 right where a kernel runs atanh_f.  The asm makes the
// address opaque so the loads are not hoisted out of the row loop: passed as a
// kernel argument (or hoisted) they would hold 32 SGPRs for the whole kernel,
// which in the row-pipeline decoders spills other uniforms into VGPR lanes and
// reloads them with v_readlane in the loop.
// The streaming tile kernels run atanh_f on most rows at 2-3 dB, where the
// loads (and their lgkmcnt waits, shared with LDS) cost more than the held
// SGPRs: they take the coefficients as a kernel argument (kStreamCoefArg).
#ifndef LDPC_STREAM_COEF_ARG
#define LDPC_STREAM_COEF_ARG 1
#endif
constexpr bool kStreamCoefArg = LDPC_STREAM_COEF_ARG != 0;
static __constant__ AtanhCoef kAtanhCoefK = kAtanhCoef;
typedef __attribute__((address_space(4))) const AtanhCoef ConstCoef;
__device__ __forceinline__ AtanhCoef coef_load() {
    ConstCoef *p = (ConstCoef *)&kAtanhCoefK;
    asm volatile("" : "+s"(p));
    return {p->t15, p->t13, p->t11, p->t9, p->t7, p->t5, p->t3, p->l8,
            p->l7,  p->l6,  p->l5,  p->l4, p->l3, p->l2, p->ln2hi, p->ln2lo};
}


}  // namespace
}  // namespace ldpc
