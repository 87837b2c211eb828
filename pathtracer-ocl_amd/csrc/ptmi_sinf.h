// ptmi_sinf.h -- the reference RNG's float sin (noise3D, tracer.cl:314-317, whose
// sin(float) is ROCm device-libs' __ocml_sin_f32) with the same result bits for
// every finite |x| < 2^19 and a cheaper argument reduction for 2^17 <= |x| < 2^19.
//
// ocml reduces |x| >= 2^17 with a general Payne-Hanek step: seven chained 32x32->64
// multiplies of the mantissa by 224 bits of 2/pi, then ~20 selects that pick a
// 96-bit window of the product by the exponent, then the normalisation of that
// window into a float hi/lo pair.  The noise arguments of the bench scenes lie
// below 2^19 (sample index <= 2047: 237.212 n + ... < 5.3e5), where the exponent
// is 144 or 145: the window is fixed (product words p4..p7, shift 152 - e) and
// every select folds away.  The four least significant table words only reach
// the window through the carry into p4, whose bits end ~90 places below the
// binary point of x * 2/pi: leaving them out (3 multiplies instead of 7) changes no
// result bit in the domain -- checked for every float |x| < 2^19 against the
// oracle's restatement (tools/sinf_check.cpp) and against the device library
// itself (tests/test_gpu_rng.py).  Without p4 as well, 38 floats would differ.
// The reduced argument itself is then F' * pi/2 in FP64 rounded once to float,
// except within a guard band around float rounding midpoints, where ocml's own
// truncated hi/lo sequence runs (PTMI_SIN_FP64R; same checks).
// Ahead of all that, an FP64 Cody-Waite step (PTMI_SIN_CW64) computes the same r and
// q for all but 28 of the 2^24 floats in [2^17, 2^19); those lanes take the product.
// The small-argument path, the polynomials and the sign logic are ocml's,
// operation for operation (cf. oracle/ocml_sinf.h, verified against ocml over
// all 2^32 floats).
//
// Plain C++ on bit patterns (fshr / clz / fmaf), so the same source compiles for
// gfx950 (v_alignbit_b32, v_ffbh_u32, v_fma_f32) and for a host-side check.
#pragma once
#include <math.h>
#include <stdint.h>

#ifndef PTMI_SINF_FN
#define PTMI_SINF_FN __device__ __forceinline__
#endif
#ifndef PTMI_SIN_FP64R
#define PTMI_SIN_FP64R 1  // large-argument r from one FP64 product (ocml's hi/lo sequence near midpoints only)
#endif
#ifndef PTMI_SIN_CW64
#define PTMI_SIN_CW64 1  // large-argument reduction by FP64 Cody-Waite (Payne-Hanek only near ties)
#endif

namespace ptmi {

PTMI_SINF_FN uint32_t sf_bits(float f) { return __builtin_bit_cast(uint32_t, f); }
PTMI_SINF_FN float sf_float(uint32_t u) { return __builtin_bit_cast(float, u); }
// llvm.fshr.i32 (s taken mod 32) -- one v_alignbit_b32 on the GPU -- and fshl for a
// constant 0 < s < 32; clz with clz(0) = 32, as ocml uses them.
PTMI_SINF_FN uint32_t sf_fshr(uint32_t a, uint32_t b, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(a, b, s);
#else
    return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31u));  // host build of tools/sinf_check.cpp
#endif
}
PTMI_SINF_FN uint32_t sf_fshl(uint32_t a, uint32_t b, uint32_t s) { return sf_fshr(a, b, 32u - s); }
PTMI_SINF_FN uint32_t sf_clz(uint32_t v) { return v ? (uint32_t)__builtin_clz(v) : 32u; }

// __ocmlpriv_trigredsmall_f32 (ISA >= 9.0): 3-constant Cody-Waite, |x| < 2^17.
PTMI_SINF_FN float sf_redux_small(float x, int& q) {
    const float t = x * sf_float(0x3F22F983u);  // 2/pi
    const float r = rintf(t);
    float a = fmaf(r, sf_float(0xBFC90FDAu), x);
    a = fmaf(r, sf_float(0xB3A22168u), a);
    a = fmaf(r, sf_float(0xA7C234C4u), a);
    q = ((int)r) & 3;
    return a;
}

// __ocmlpriv_trigredlarge_f32 specialised to 2^17 <= x < 2^19 (exponent 144, 145).
PTMI_SINF_FN float sf_redux_large_17_19(float x, int& q) {
#if PTMI_SIN_CW64
    // ocml's large reduction returns k = the nearest integer to x 2/pi (as q = k mod 4)
    // and r = RN((x - k pi/2) (1 + d)), |d| < 2^-46.  For x < 2^19 a three-part FP64
    // Cody-Waite step gives x - k pi/2 to ~2^-51 relative: pi/2 = P1 + P2 + P3 with a
    // 33-bit P1, so k P1 (k < 2^19) and x - k P1 are exact and the two remaining fmas
    // round once each.  That r rounded once to float is ocml's r except (a) when x 2/pi
    // lies so close to a half-integer that the FP64 product may round k the other way
    // (then |r| is within 2^-25 of pi/4), or (b) within the midpoint guard band of the
    // FP64R block below; both take the Payne-Hanek path.  Same exhaustive checks.
    {
        const double xd = (double)x;
        const double kd = __builtin_rint(xd * 0x1.45f306dc9c883p-1);
        double r = fma(-kd, 0x1.921fb54400000p+0, xd);
        r = fma(-kd, 0x1.0b4611a600000p-34, r);
        r = fma(-kd, 0x1.3198a2e037073p-69, r);
        const uint64_t rb = __builtin_bit_cast(uint64_t, r);
        const uint32_t tail = ((uint32_t)rb + 0x200u) & 0x1FFFFFFFu;
        if (((uint32_t)(rb >> 32) & 0x7FFFFFFFu) < 0x3FE921FBu && tail - 0x10000000u >= 0x400u) {
            q = ((int)kd) & 3;
            return (float)r;
        }
    }
#endif
    const uint32_t bits = sf_bits(x);
    const uint32_t e = bits >> 23;
    const uint64_t m = (uint64_t)((bits & 0x7FFFFFu) | 0x800000u);
    // mantissa * 2/pi words w4..w6: the carry of w0..w3 into p4 is dropped (see header)
    uint64_t t = m * 4230436817ull;
    const uint32_t p4 = (uint32_t)t;
    t = (t >> 32) + m * 1313084713ull;
    const uint32_t p5 = (uint32_t)t;
    t = (t >> 32) + m * 2734261102ull;
    const uint32_t p6 = (uint32_t)t;
    const uint32_t p7 = (uint32_t)(t >> 32);
    // ocml's window for e - 120 in [0, 31]: (p7, p6, p5, p4) shifted by 32 - (e - 120)
    const uint32_t s61 = 152u - e;
    const uint32_t a65 = sf_fshr(p7, p6, s61);
    const uint32_t a66 = sf_fshr(p6, p5, s61);
    const uint32_t a67 = sf_fshr(p5, p4, s61);
    // from here on ocml's normalisation, unchanged
    const uint32_t a68 = a65 >> 29;
    const uint32_t a69 = sf_fshl(a65, a66, 2), a70 = sf_fshl(a66, a67, 2), a71 = sf_fshl(a67, p4, 2);
    const uint32_t a72 = a68 & 1u;
    const uint32_t a73 = 0u - a72;
    const uint32_t a74 = a68 << 31;
    const uint32_t a75 = a69 ^ a73, a76 = a70 ^ a73, a77 = a71 ^ a73;
    q = (int)((a72 + (a65 >> 30)) & 3u);
#if PTMI_SIN_FP64R
    // ocml turns F' = a75:a76:a77 * 2^-96 (< 1/2) into a truncated float pair hi + lo and
    // returns r = RN(p + e1) = RN(F' pi/2 (1 + d)), |d| < 2^-46.  F' pi/2 in FP64 (relative
    // error < 2^-51), rounded once to float, is the same r unless it lies within 2^9 double
    // ulps of a float rounding midpoint (low 29 mantissa bits near 0x10000000): those rare
    // lanes (24 of the 2^24 floats in [2^18, 2^19)) take ocml's sequence below.
    {
        const double fd = fma((double)a76, 0x1p-32, (double)a75) + (double)a77 * 0x1p-64;
        const double rd = fd * (0x1p-32 * 1.5707963267948966);
        const uint32_t tail = ((uint32_t)__builtin_bit_cast(uint64_t, rd) + 0x200u) & 0x1FFFFFFFu;
        if (a75 != 0u && tail - 0x10000000u >= 0x400u) return sf_float(sf_bits((float)rd) ^ a74);
    }
#endif
    const uint32_t a78 = sf_clz(a75);
    const uint32_t a79 = 31u - a78;
    const uint32_t a80 = sf_fshr(a75, a76, a79);
    const uint32_t a81 = sf_fshr(a76, a77, a79);
    const float hi = sf_float(((a80 >> 9) - (a78 << 23)) + 1056964608u + a74);
    const uint32_t a88 = sf_fshl(a80, a81, 23);
    const uint32_t a89 = sf_clz(a88);
    const uint32_t a91 = sf_fshr(a88, a81, ~a89);
    const float lo = sf_float(((a91 >> 9) - ((a89 + a78) << 23)) + 855638016u + a74);
    const float pio2_hi = sf_float(0x3FC90FDAu), pio2_mid = sf_float(0x33A22168u);
    const float p = hi * pio2_hi;
    float e1 = fmaf(hi, pio2_hi, -p);
    e1 = fmaf(hi, pio2_mid, e1);
    e1 = fmaf(lo, pio2_hi, e1);
    return e1 + p;
}

// __ocmlpriv_sincosred_f32 on the reduced argument r (quadrant q) and the quadrant / sign
// fix-ups of __ocml_sin_f32 for x (ax = |x|).
PTMI_SINF_FN float sf_sin_poly(float x, float ax, float r, int q) {
    const float x2 = r * r;
    float s = fmaf(x2, sf_float(0xB94C1982u), sf_float(0x3C0881C4u));
    s = fmaf(x2, s, sf_float(0xBE2AAA9Du));
    s = x2 * s;
    s = fmaf(r, s, r);
    float c = fmaf(x2, sf_float(0x37D75334u), sf_float(0xBAB64F3Bu));
    c = fmaf(x2, c, sf_float(0x3D2AABF7u));
    c = fmaf(x2, c, sf_float(0xBF000004u));
    c = fmaf(x2, c, 1.0f);
    const uint32_t v = (q & 1) ? sf_bits(c) : sf_bits(s);
    const uint32_t neg = (q > 1) ? 0x80000000u : 0u;
    return sf_float((sf_bits(ax) ^ sf_bits(x)) ^ neg ^ v);
}

// __ocml_sin_f32 for finite |x| < 2^19 (callers route everything else to ocml).
PTMI_SINF_FN float sinf_lt19(float x) {
    const float ax = fabsf(x);
    int q;
    float r;
    if (ax < 131072.0f) {
        r = sf_redux_small(ax, q);
    } else {
        r = sf_redux_large_17_19(ax, q);
    }
    // __ocmlpriv_sincosred_f32 and the quadrant / sign fix-ups
    const float x2 = r * r;
    float s = fmaf(x2, sf_float(0xB94C1982u), sf_float(0x3C0881C4u));
    s = fmaf(x2, s, sf_float(0xBE2AAA9Du));
    s = x2 * s;
    s = fmaf(r, s, r);
    float c = fmaf(x2, sf_float(0x37D75334u), sf_float(0xBAB64F3Bu));
    c = fmaf(x2, c, sf_float(0x3D2AABF7u));
    c = fmaf(x2, c, sf_float(0xBF000004u));
    c = fmaf(x2, c, 1.0f);
    const uint32_t v = (q & 1) ? sf_bits(c) : sf_bits(s);
    const uint32_t neg = (q > 1) ? 0x80000000u : 0u;
    return sf_float((sf_bits(ax) ^ sf_bits(x)) ^ neg ^ v);
}

// __ocml_sin_f32 for 2^19 <= |x| < 2^30 (the glass noise, noise3D(fgi, n*n, b)) by a
// four-part FP64 Cody-Waite reduction: 23-bit P1, P2, P3, so k P1, k P2, k P3 are
// exact for k < 2^30 and x - k P1, (x - k P1) - k P2 too; the last two fmas round
// once each (~2^-51 relative).  Returns false, and the caller runs ocml's own sin,
// where that r may differ from ocml's: k possibly rounded the other way (|r| within
// 2^-20 of pi/4) or r in the float-midpoint guard band.  Exhaustive host check in
// tools/sinf_check.cpp.
PTMI_SINF_FN bool sinf_cw30(float x, float& out) {
    const float ax = fabsf(x);
    const double xd = (double)ax;
    const double kd = __builtin_rint(xd * 0x1.45f306dc9c883p-1);
    double r = fma(-kd, 0x1.921fb4p+0, xd);
    r = fma(-kd, 0x1.4442d0p-24, r);
    r = fma(-kd, 0x1.846988p-48, r);
    r = fma(-kd, 0x1.8cc51701b839ap-72, r);
    const uint64_t rb = __builtin_bit_cast(uint64_t, r);
    const uint32_t tail = ((uint32_t)rb + 0x200u) & 0x1FFFFFFFu;
    if (!(((uint32_t)(rb >> 32) & 0x7FFFFFFFu) < 0x3FE921F5u && tail - 0x10000000u >= 0x400u)) return false;
    const int q = ((int)(int64_t)kd) & 3;
    const float rf = (float)r;
    const float x2 = rf * rf;
    float s = fmaf(x2, sf_float(0xB94C1982u), sf_float(0x3C0881C4u));
    s = fmaf(x2, s, sf_float(0xBE2AAA9Du));
    s = x2 * s;
    s = fmaf(rf, s, rf);
    float c = fmaf(x2, sf_float(0x37D75334u), sf_float(0xBAB64F3Bu));
    c = fmaf(x2, c, sf_float(0x3D2AABF7u));
    c = fmaf(x2, c, sf_float(0xBF000004u));
    c = fmaf(x2, c, 1.0f);
    const uint32_t v = (q & 1) ? sf_bits(c) : sf_bits(s);
    const uint32_t neg = (q > 1) ? 0x80000000u : 0u;
    out = sf_float((sf_bits(ax) ^ sf_bits(x)) ^ neg ^ v);
    return true;
}

// The kernel's noise sin (noise3d in ptmi_kernels.hip), composed in one place so the
// GPU probe (tests/gpu_probe/sinf_probe.hip) checks exactly what the kernel runs:
//   |x| < 2^19           sinf_lt19 (every argument of a <= 2210-spp frame but glass)
//   2^19 <= |x| < 2^30   sinf_cw30, or `fallback` (ocml's own sin) where it declines
//   otherwise            `fallback`
template <typename Fallback>
PTMI_SINF_FN float noise_sinf(float x, Fallback fallback) {
    float sn;
    if (fabsf(x) < 0x1p19f) {
        sn = sinf_lt19(x);
    } else if (!(fabsf(x) < 0x1p30f) || !sinf_cw30(x, sn)) {
        sn = fallback(x);
    }
    return sn;
}

// The FP64 Cody-Waite step of sf_redux_large_17_19 alone (2^17 <= ax < 2^19): true, with ocml's
// r and q, on every argument but the ~28 per 2^24 that sf_redux_large_17_19 hands to its
// Payne-Hanek product.
PTMI_SINF_FN bool sf_cw64(float ax, float& rf, int& q) {
    const double xd = (double)ax;
    const double kd = __builtin_rint(xd * 0x1.45f306dc9c883p-1);
    double r = fma(-kd, 0x1.921fb54400000p+0, xd);
    r = fma(-kd, 0x1.0b4611a600000p-34, r);
    r = fma(-kd, 0x1.3198a2e037073p-69, r);
    const uint64_t rb = __builtin_bit_cast(uint64_t, r);
    const uint32_t tail = ((uint32_t)rb + 0x200u) & 0x1FFFFFFFu;
    q = ((int)kd) & 3;
    rf = (float)r;
    return ((uint32_t)(rb >> 32) & 0x7FFFFFFFu) < 0x3FE921FBu && tail - 0x10000000u >= 0x400u;
}

// Two noise sins at once (round 6): noise_sinf(x1) and noise_sinf(x2), bit for bit.  The two
// draws of a noise3D pair (the camera's anti-aliasing offsets, the hemisphere's uniforms) are
// independent; evaluated one after the other their branchy reductions run as separate blocks and
// each dependent chain is exposed in turn.  Here each reduction block serves both draws (a block
// runs when either draw needs it), so the two chains interleave.  Lanes with an argument the
// common blocks do not finish -- the Payne-Hanek band of [2^17, 2^19) and |x| >= 2^19 -- take
// noise_sinf itself afterwards.
template <typename Fallback>
PTMI_SINF_FN void noise_sinf2(float x1, float x2, Fallback fallback, float& o1, float& o2) {
    const float a1 = fabsf(x1), a2 = fabsf(x2);
    const bool sm1 = a1 < 131072.0f, sm2 = a2 < 131072.0f;
    bool ok1 = a1 < 0x1p19f, ok2 = a2 < 0x1p19f;  // (NaN: false)
    float r1 = 0.0f, r2 = 0.0f;
    int q1 = 0, q2 = 0;
    if (sm1 || sm2) {
        int qa, qb;
        const float ra = sf_redux_small(a1, qa), rb = sf_redux_small(a2, qb);
        r1 = sm1 ? ra : r1;
        q1 = sm1 ? qa : q1;
        r2 = sm2 ? rb : r2;
        q2 = sm2 ? qb : q2;
    }
    const bool lg1 = ok1 && !sm1, lg2 = ok2 && !sm2;
    if (lg1 || lg2) {
        float ra, rb;
        int qa, qb;
        const bool ca = sf_cw64(a1, ra, qa), cb = sf_cw64(a2, rb, qb);
        r1 = lg1 ? ra : r1;
        q1 = lg1 ? qa : q1;
        r2 = lg2 ? rb : r2;
        q2 = lg2 ? qb : q2;
        ok1 = ok1 && (sm1 || ca);
        ok2 = ok2 && (sm2 || cb);
    }
    o1 = sf_sin_poly(x1, a1, r1, q1);
    o2 = sf_sin_poly(x2, a2, r2, q2);
    if (!ok1) o1 = noise_sinf(x1, fallback);
    if (!ok2) o2 = noise_sinf(x2, fallback);
}

}  // namespace ptmi
