/*
 * ocml_sinf.h -- portable C restatement of ROCm device-libs' __ocml_sin_f32 and
 * __ocml_fract_f32 as built for gfx950 (ROCm 7.2 ocml.bc; ISA >= 9.0 paths).
 * TEST INFRASTRUCTURE (oracle).
 *
 * Why: the reference RNG (tracer.cl:314-317)
 *     noise3D(x,y,z) = fract(sin(x*112.9898f + y*179.233f + z*237.212f) * 43758.5453f)
 * multiplies one float ULP of sin() by ~4e4, so the CPU restatement must produce
 * the SAME float sin the reference kernel gets from the AMD OpenCL builtin
 * library (opencl.bc `_Z3sinf` -> __ocml_sin_f32), not glibc's sinf.
 *
 * The algorithm is read off the device-library IR:
 *   __ocmlpriv_trigred_f32   |x| < 131072 -> trigredsmall (3-constant FMA
 *                            Cody-Waite), else trigredlarge (integer Payne-Hanek
 *                            with a 224-bit 2/pi table, then FMA recombination)
 *   __ocmlpriv_sincosred_f32 degree-7/8 float polynomials (fmuladd == fma on gfx950)
 *   __ocml_sin_f32           quadrant select + sign fix-ups
 * Every step is an exact integer op or a single IEEE float op / fmaf, so the
 * result is bit-identical on any IEEE-754 host with a correct fmaf.  Verified
 * exhaustively against the GPU's ocml (tests/test_gpu_rng.py).
 */
#ifndef PT_OCML_SINF_H
#define PT_OCML_SINF_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef PT_FN
#define PT_FN static inline
#endif

PT_FN float pto_bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
PT_FN uint32_t pto_f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* llvm.fshr.i32(a, b, s): low 32 bits of (a:b) >> (s mod 32). */
PT_FN uint32_t pto_fshr(uint32_t a, uint32_t b, uint32_t s) {
    s &= 31u;
    return s ? (uint32_t)((((uint64_t)a << 32) | b) >> s) : b;
}
/* llvm.fshl.i32(a, b, s): high 32 bits of (a:b) << (s mod 32). */
PT_FN uint32_t pto_fshl(uint32_t a, uint32_t b, uint32_t s) {
    s &= 31u;
    return s ? (uint32_t)(((((uint64_t)a << 32) | b) << s) >> 32) : a;
}
PT_FN uint32_t pto_clz32(uint32_t v) { return v ? (uint32_t)__builtin_clz(v) : 32u; }

/* __ocmlpriv_trigredsmall_f32, ISA >= 9000 branch. x = |x| < 131072. */
PT_FN float pto_trigred_small(float x, int* q) {
    float t = x * pto_bits2f(0x3F22F983u);                 /* 2/pi */
    float r = rintf(t);
    float a = fmaf(r, pto_bits2f(0xBFC90FDAu), x);         /* -pi/2 hi  */
    a = fmaf(r, pto_bits2f(0xB3A22168u), a);               /* -pi/2 mid */
    a = fmaf(r, pto_bits2f(0xA7C234C4u), a);               /* -pi/2 lo  */
    *q = ((int)r) & 3;
    return a;
}

/* __ocmlpriv_trigredlarge_f32, ISA >= 9000 branch. x = |x| >= 131072 (finite). */
PT_FN float pto_trigred_large(float x, int* q) {
    uint32_t bits = pto_f2bits(x);
    uint32_t e = bits >> 23;
    uint64_t m = (uint64_t)((bits & 0x7FFFFFu) | 0x800000u);
    uint64_t t;
    uint32_t p0, p1, p2, p3, p4, p5, p6, p7;
    t = m * 4266746795ull;            p0 = (uint32_t)t;
    t = (t >> 32) + m * 1011060801ull; p1 = (uint32_t)t;
    t = (t >> 32) + m * 3680671129ull; p2 = (uint32_t)t;
    t = (t >> 32) + m * 4113882560ull; p3 = (uint32_t)t;
    t = (t >> 32) + m * 4230436817ull; p4 = (uint32_t)t;
    t = (t >> 32) + m * 1313084713ull; p5 = (uint32_t)t;
    t = (t >> 32) + m * 2734261102ull; p6 = (uint32_t)t;
    p7 = (uint32_t)(t >> 32);
    uint32_t sh = e - 120u;
    int big = sh > 63u;
    uint32_t a37 = big ? p5 : p7, a38 = big ? p4 : p6, a39 = big ? p3 : p5;
    uint32_t a40 = big ? p2 : p4, a41 = big ? p1 : p3, a42 = big ? p0 : p2;
    uint32_t s44 = (big ? (uint32_t)-64 : 0u) + sh;
    int g45 = s44 > 31u;
    uint32_t a46 = g45 ? a38 : a37, a47 = g45 ? a39 : a38, a48 = g45 ? a40 : a39;
    uint32_t a49 = g45 ? a41 : a40, a50 = g45 ? a42 : a41;
    uint32_t s52 = (g45 ? (uint32_t)-32 : 0u) + s44;
    int g53 = s52 > 31u;
    uint32_t a54 = g53 ? a47 : a46, a55 = g53 ? a48 : a47, a56 = g53 ? a49 : a48;
    uint32_t a57 = g53 ? a50 : a49;
    uint32_t s59 = (g53 ? (uint32_t)-32 : 0u) + s52;
    int z60 = s59 == 0u;
    uint32_t s61 = 32u - s59;
    uint32_t a65 = z60 ? a54 : pto_fshr(a54, a55, s61);
    uint32_t a66 = z60 ? a55 : pto_fshr(a55, a56, s61);
    uint32_t a67 = z60 ? a56 : pto_fshr(a56, a57, s61);
    uint32_t a68 = a65 >> 29;
    uint32_t a69 = pto_fshl(a65, a66, 2), a70 = pto_fshl(a66, a67, 2), a71 = pto_fshl(a67, a57, 2);
    uint32_t a72 = a68 & 1u;
    uint32_t a73 = 0u - a72;
    uint32_t a74 = a68 << 31;
    uint32_t a75 = a69 ^ a73, a76 = a70 ^ a73, a77 = a71 ^ a73;
    uint32_t a78 = pto_clz32(a75);
    uint32_t a79 = 31u - a78;
    uint32_t a80 = pto_fshr(a75, a76, a79);
    uint32_t a81 = pto_fshr(a76, a77, a79);
    uint32_t a86 = ((a80 >> 9) - (a78 << 23)) + 1056964608u + a74;
    float hi = pto_bits2f(a86);
    uint32_t a88 = pto_fshl(a80, a81, 23);
    uint32_t a89 = pto_clz32(a88);
    uint32_t a91 = pto_fshr(a88, a81, ~a89);
    uint32_t a97 = ((a91 >> 9) - ((a89 + a78) << 23)) + 855638016u + a74;
    float lo = pto_bits2f(a97);
    const float PIO2_HI = pto_bits2f(0x3FC90FDAu), PIO2_MID = pto_bits2f(0x33A22168u);
    float p = hi * PIO2_HI;
    float e1 = fmaf(hi, PIO2_HI, -p);
    e1 = fmaf(hi, PIO2_MID, e1);
    e1 = fmaf(lo, PIO2_HI, e1);
    *q = (int)((a72 + (a65 >> 30)) & 3u);
    return e1 + p;
}

/* __ocml_sin_f32 (finite_only off). */
PT_FN float pto_sinf(float x) {
    float ax = fabsf(x);
    int q;
    float r = (ax < 131072.0f) ? pto_trigred_small(ax, &q) : pto_trigred_large(ax, &q);
    /* __ocmlpriv_sincosred_f32 */
    float x2 = r * r;
    float s = fmaf(x2, pto_bits2f(0xB94C1982u), pto_bits2f(0x3C0881C4u));
    s = fmaf(x2, s, pto_bits2f(0xBE2AAA9Du));
    s = x2 * s;
    s = fmaf(r, s, r);
    float c = fmaf(x2, pto_bits2f(0x37D75334u), pto_bits2f(0xBAB64F3Bu));
    c = fmaf(x2, c, pto_bits2f(0x3D2AABF7u));
    c = fmaf(x2, c, pto_bits2f(0xBF000004u));
    c = fmaf(x2, c, 1.0f);
    uint32_t v = (q & 1) ? pto_f2bits(c) : pto_f2bits(s);
    uint32_t neg = (q > 1) ? 0x80000000u : 0u;
    uint32_t res = (pto_f2bits(ax) ^ pto_f2bits(x)) ^ neg ^ v;
    /* fcmp one |x|, inf  is false for NaN and for inf -> quiet NaN */
    return (isinf(ax) || isnan(ax)) ? pto_bits2f(0x7FC00000u) : pto_bits2f(res);
}

/* __ocml_fract_f32 (finite_only off): min(x - floor(x), 0x1.fffffep-1f). */
PT_FN float pto_fractf(float x) {
    float r = fminf(x - floorf(x), pto_bits2f(0x3F7FFFFFu));
    if (isnan(x)) return x;
    if (isinf(x)) return 0.0f;
    return r;
}

#endif
