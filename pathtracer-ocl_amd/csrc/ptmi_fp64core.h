// ptmi_fp64core.h -- the core sequences of the compiler's double divide, sqrt and
// rsqrt for gfx950, without their range steps (used by ptmi_kernels.hip's affine
// instantiations; checked against the operators by tests/test_gpu_rng.py).
#pragma once
#include <stdint.h>

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
// The divide core in two steps: the Newton-refined reciprocal depends on y alone, so
// quotients with one denominator can share it (sphere roots) and stay bit-identical.
__device__ __forceinline__ double rcp_core(double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    e = fma(-y, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double div_core_r(double x, double y, double r) {  // r = rcp_core(y)
    const double q = x * r;
    const double rem = fma(-y, q, x);
    return fma(rem, r, q);
}
__device__ __forceinline__ double div_core(double x, double y) {  // x / y: v_div_fmas with vcc = 0, no fix-up
    return div_core_r(x, y, rcp_core(y));
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

// The constants of sincos_core (ocml's __ocml_sincos_f64), in order of first use.
static constexpr uint64_t kSincosBits[17] = {0x3FE45F306DC9C883ull, 0xBFF921FB54442D18ull, 0xBC91A62633145C00ull, 0x3C91A62633145C00ull, 0xB97B839A252049C0ull, 0xBDA907DB46CC5E42ull, 0x3E21EEB69037AB78ull, 0xBE927E4FA17F65F6ull, 0x3EFA01A019F4EC90ull, 0xBF56C16C16C16967ull, 0x3FA5555555555555ull, 0x3DE5E0B2F9A43BB8ull, 0xBE5AE600B42FDFA7ull, 0x3EC71DE3796CDE01ull, 0xBF2A01A019E83E5Cull, 0x3F81111111110BB3ull, 0xBFC5555555555555ull};
static __constant__ double kSincosK[17] = {__builtin_bit_cast(double, 0x3FE45F306DC9C883ull), __builtin_bit_cast(double, 0xBFF921FB54442D18ull), __builtin_bit_cast(double, 0xBC91A62633145C00ull), __builtin_bit_cast(double, 0x3C91A62633145C00ull), __builtin_bit_cast(double, 0xB97B839A252049C0ull), __builtin_bit_cast(double, 0xBDA907DB46CC5E42ull), __builtin_bit_cast(double, 0x3E21EEB69037AB78ull), __builtin_bit_cast(double, 0xBE927E4FA17F65F6ull), __builtin_bit_cast(double, 0x3EFA01A019F4EC90ull), __builtin_bit_cast(double, 0xBF56C16C16C16967ull), __builtin_bit_cast(double, 0x3FA5555555555555ull), __builtin_bit_cast(double, 0x3DE5E0B2F9A43BB8ull), __builtin_bit_cast(double, 0xBE5AE600B42FDFA7ull), __builtin_bit_cast(double, 0x3EC71DE3796CDE01ull), __builtin_bit_cast(double, 0xBF2A01A019E83E5Cull), __builtin_bit_cast(double, 0x3F81111111110BB3ull), __builtin_bit_cast(double, 0xBFC5555555555555ull)};

// ocml's __ocml_sincos_f64 for 0 <= x < 1024 (ROCm 7.2 ocml.bc, read off the IR):
// __ocmlpriv_trigredsmall_f64 (Cody-Waite with a double-double remainder), then
// __ocmlpriv_sincosred2_f64 and the quadrant swap.  Left out, being identities on
// this domain: the large-argument branch (x >= 2^30), the sign of x (+0), the
// non-finite fix-up, and the error term fma(k, pio2_m, -k * pio2_m), which is +0
// because pio2_m has 43 significant bits and k = rint(x * 2/pi) < 2^10.
template <bool kMem = false>
__device__ __forceinline__ void sincos_core(double x, double* sp, double* cp) {
    // kMem: the constants are read from a __constant__ table (scalar loads into SGPRs)
    // instead of being materialised as literals, which the allocator hoists out of the
    // bounce loop into ~20 VGPRs (same values, same bits).  The product kernels use the
    // table: the group kernels then stop spilling, and C2/C3 fit 5 waves per SIMD.
    auto K = [](int i) -> double {
        if constexpr (kMem) return kSincosK[i];
        else return __builtin_bit_cast(double, kSincosBits[i]);
    };
    const double dn = __builtin_rint(x * K(0));
    const double t4 = fma(dn, K(1), x);
    const double t5 = fma(dn, K(2), t4);
    const double t6 = dn * K(3);
    const double t9 = t4 - t6;
    const double t10 = t4 - t9;
    const double t11 = t10 - t6;
    const double t12 = t9 - t5;
    const double t13 = t12 + t11;
    const double t15 = fma(dn, K(4), t13);
    const double rh = t5 + t15;
    const double rl = t15 - (rh - t5);
    const int q = ((int)dn) & 3;
    // __ocmlpriv_sincosred2_f64(rh, rl)
    const double x2 = rh * rh;
    const double hx = x2 * 0.5;
    const double c0 = 1.0 - hx;
    const double c1 = (1.0 - c0) - hx;
    const double x4 = x2 * x2;
    double pc = fma(x2, K(5), K(6));
    pc = fma(x2, pc, K(7));
    pc = fma(x2, pc, K(8));
    pc = fma(x2, pc, K(9));
    pc = fma(x2, pc, K(10));
    const double cc = c0 + fma(x4, pc, fma(rh, -rl, c1));
    double ps = fma(x2, K(11), K(12));
    ps = fma(x2, ps, K(13));
    ps = fma(x2, ps, K(14));
    ps = fma(x2, ps, K(15));
    const double x3 = rh * -x2;
    const double s1 = fma(x3, ps, rl * 0.5);
    const double s2 = fma(x2, s1, -rl);
    const double ss = rh - fma(x3, K(16), s2);
    // __ocml_sincos_f64: quadrant swap and sign flips (x >= 0)
    const uint64_t flip = (q > 1) ? 0x8000000000000000ull : 0ull;
    const double sv = (q & 1) ? cc : ss;
    const double cv = (q & 1) ? -ss : cc;
    *sp = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, sv) ^ flip);
    *cp = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, cv) ^ flip);
}

}  // namespace ptmi
