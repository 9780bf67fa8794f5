// phys_math.h -- fp32 phi(x) = -log tanh(x/2) of the physical-mode decoders
// (phys_kernels.hip: LDS-resident; phys_tile.hip: HBM-resident tiles).  Both
// use this one definition, so the two paths are bit-identical.
// CPU restatement: oracle/phys_oracle.c:phi.
#pragma once
#include <hip/hip_runtime.h>

namespace ldpc {

constexpr float kPhiMin = 1.0e-7f;  // phi(1e-7) ~ 16.8: caps the magnitude
constexpr float kPhiMax = 30.0f;    // phi(30) ~ 1.9e-13

// phi(x) = log((e^x + 1)/(e^x - 1)) straight on the hardware transcendentals
// v_exp_f32 (2^x), v_rcp_f32 and v_log_f32 (log2), one instruction each: the
// clamped x keeps every operand normal (t = e^x in [1.03, 1.1e13], the
// quotient in [1, 65]), so none of the denormal / correct-rounding wrappers
// of __expf, __frcp_rn and __logf is needed (they made phi ~30 VALU; the
// physical mode is our fp32 design, checked against its CPU restatement by
// decisions, tests/test_phys.py).  Below x = 2^-5 the quotient loses bits to
// e^x - 1, so there phi ~ log(2/x) + x^2/12 = ln2 (1 - log2 x) + x^2/12.
__device__ __forceinline__ float phi(float x) {
    constexpr float kLn2 = 0.693147180559945309f, kLog2e = 1.442695040888963407f;
    x = fminf(fmaxf(x, kPhiMin), kPhiMax);
    const float t = __builtin_amdgcn_exp2f(x * kLog2e);
    const float big = __builtin_amdgcn_logf((t + 1.0f) * __builtin_amdgcn_rcpf(t - 1.0f)) * kLn2;
    const float small = (1.0f - __builtin_amdgcn_logf(x)) * kLn2 + x * x * (1.0f / 12.0f);
    return x < 0.03125f ? small : big;
}

}  // namespace ldpc
