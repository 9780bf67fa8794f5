// phys_math.h -- fp32 phi(x) = -log tanh(x/2) of the physical-mode decoders
// (phys_kernels.hip: LDS-resident; phys_tile.hip: HBM-resident tiles).  Both
// use this one definition, so the two paths are bit-identical.
// CPU restatement: oracle/phys_oracle.c:phi.
#pragma once
#include <hip/hip_runtime.h>

namespace ldpc {

constexpr float kPhiMin = 1.0e-7f;  // phi(1e-7) ~ 16.8: caps the magnitude
constexpr float kPhiMax = 30.0f;    // phi(30) ~ 1.9e-13

// phi(x) = log((e^x + 1)/(e^x - 1)) with the hardware v_exp_f32 / v_log_f32 /
// v_rcp_f32 (one instruction each).  Below x = 2^-5 the quotient loses bits to
// e^x - 1, so use the series phi(x) ~ log(2/x) + x^2/12 there.
__device__ __forceinline__ float phi(float x) {
    x = fminf(fmaxf(x, kPhiMin), kPhiMax);
    if (x < 0.03125f) return __logf(2.0f * __frcp_rn(x)) + x * x * (1.0f / 12.0f);
    const float t = __expf(x);
    return __logf((t + 1.0f) * __frcp_rn(t - 1.0f));
}

}  // namespace ldpc
