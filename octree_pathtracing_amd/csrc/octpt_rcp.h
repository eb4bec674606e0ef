// Correctly rounded f32 reciprocal from the hardware estimate (v_rcp_f32, 1 ulp) and one Newton step
// in fused multiply-adds (Markstein): e = 1 - a*r exactly-rounded once, r' = r + e*r.  Used where the
// kernels need 1/x bit-identical to the oracle's correctly rounded division, on the domain where
// tools/rcp_check.hip has compared it with the division for every float: |a| in [2^-23, 2^126]
// (ESVO's t_coef = 1 / -|d|: |d| is clamped to OCTREE_EPSILON = 2^-23 and is a unit vector's).
#pragma once
#include <hip/hip_runtime.h>

namespace octpt {
__device__ __forceinline__ float rcp_rn(float a) {
    const float r = __builtin_amdgcn_rcpf(a);
    const float e = __builtin_fmaf(-a, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
}  // namespace octpt
