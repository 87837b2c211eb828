// ptmi_fp64core.h -- the core sequences of the compiler's double divide, sqrt and
// rsqrt for gfx950, without their range steps (used by ptmi_kernels.hip's affine
// instantiations; checked against the operators by tests/test_gpu_rng.py).
#pragma once

namespace ptmi {

// ---- Double divide / sqrt / rsqrt: the compiler's core sequences ------------------
// LLVM's gfx950 expansions of x / y, sqrt(x) and rsqrt(x) for double wrap a fixed
// core -- Newton-refined v_rcp_f64 / v_rsq_f64 plus FMA corrections -- in range
// steps: v_div_scale / v_div_fixup, ldexp by 2^+-256 for tiny inputs, and class
// fix-ups for 0, inf and NaN.  Where those steps are identities the core alone
// returns the same bits; below, each core is written out operation for operation
// (same operands, same order) without the range steps.  The affine instantiations
// use a core only where that holds whenever the result is used (each call site
// says why).  tests/test_gpu_rng.py checks the cores against
// the compiler's operators, and tests/test_gpu_parity.py the affine images against
// the generic instantiation, which keeps the full expansions.
__device__ __forceinline__ double div_core(double x, double y) {  // x / y: v_div_fmas with vcc = 0, no fix-up
    double r = __builtin_amdgcn_rcp(y);
    double e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    const double q = x * r;
    const double rem = fma(-y, q, x);
    return fma(rem, r, q);
}
__device__ __forceinline__ double sqrt_core(double x) {  // sqrt(x) for x in [2^-767, 2^1023]
    const double r = __builtin_amdgcn_rsq(x);
    double g = x * r;
    double h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
__device__ __forceinline__ double rsqrt_core(double x) {  // ocml rsqrt_f64 for positive normal x
    const double r = __builtin_amdgcn_rsq(x);
    double e = r * -x;
    e = fma(e, r, 1.0);
    const double t = r * e;
    e = fma(e, 0.375, 0.5);
    return fma(t, e, r);
}

}  // namespace ptmi
