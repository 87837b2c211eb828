// ptmi_kernels.hip -- gfx950 (MI355X / CDNA4) path-tracing kernels.
//
// One lane = one pixel of an 8x8 tile (one wave64 per tile), looping over a
// chunk of that pixel's samples; FP64 throughout, float RNG exactly as the
// reference (tracer.cl:314-317).  The integrator restates `trace`
// (tracer.cl:831-1188); every helper cites the reference lines it follows.
//
// Compiled with -ffp-contract=off (separately rounded user arithmetic, as the
// pinned reference build) and calls the same ROCm device-library functions the
// reference's OpenCL builtins resolve to (ocml sin_f32 / sin/cos/pow/sqrt/rsqrt
// f64, maxnum/minnum), so on the same inputs the image matches the reference
// kernel bit-for-bit in practice (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ptmi_device.h"
#include "ptmi_sinf.h"
#include "ptmi_fp64core.h"

// PTMI_ABLATE: DIAGNOSTIC builds only (make ablate) -- removes a component to
// measure its share of the run time.  Images from such builds are wrong by
// design; the product is always built with PTMI_ABLATE == 0.
#ifndef PTMI_ABLATE
#define PTMI_ABLATE 0
#endif
// PTMI_STATS: DIAGNOSTIC builds -- 1 (make stats): tallies traversal events into
// ptmi_stats[] (read with ptmi_stats_read); 2 (make timers): per-wave phase clocks
// and per-wave counters only (the per-lane event atomics of 1 distort timing).
// The product has PTMI_STATS == 0.
#ifndef PTMI_STATS
#define PTMI_STATS 0
#endif
#if PTMI_STATS
// Counters (tools/bvh_stats.py names them): [0] walks [1] node4 visits [2] leaves
// [3] triangle tests [4] certified winners [5] gate rejections [6] (unused) [7] group
// object tests [8] walk phases [9] lanes in phases [10] wave loop iterations [11] eager
// re-walks [12..16] shader-clock cycles in refill / closest-prims+gate / walk phases /
// shade / whole loop [17] exact chain verifications [18] cycles in walk loops
// [19] wave-level walk loop iterations [27] / [28] (mesh kernels, timers build) lane-cycles
// of lanes whose work item is finished / all lane-cycles of the loop.
// Round 6 (kernels without meshes, wave-level executions of each block, for the dynamic
// instruction budget tools/dyn_budget.py): [32] camera refills [33] deferred sphere roots
// [34] in-place sphere roots (a lane's second sphere) [35] hemisphere sincos fallback
// [36] hemisphere sqrt fallback [37] / [38] / [39] noise draws with a lane below 2^17 / in
// [2^17, 2^19) / at or above 2^19 [40] noise draws (any path) [41] plane normal block
// [42] other-normal block [43] emission block [44] shading past the miss test [45] prims
// [46] active lanes summed over the iterations that run prims; [47] / [48] / [49] floor-ceiling plane
// pairs / other plane pairs / single planes [50] / [51] / [52] first sphere pair / later pairs / single
// [53] iterations of the loop over spheres with other matrices.
__device__ unsigned long long ptmi_stats[80];
// Per-wave accumulators (one writer per wave: the first active lane), flushed to
// ptmi_stats with one atomic per counter when the wave leaves its loop, so clock
// and per-wave counts do not serialise on global atomics.
__shared__ unsigned long long ptmi_wstat[1][64];
#define PTMI_FIRST_ACTIVE() ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1)
#define PTMI_WADD(i, v)                                                \
    do {                                                               \
        const unsigned long long v_ = (v);                             \
        if (PTMI_FIRST_ACTIVE()) ptmi_wstat[0][i] += v_;                   \
    } while (0)
#if PTMI_STATS == 2
#define PTMI_COUNT(i) ((void)0)
#else
#define PTMI_COUNT(i) atomicAdd(&ptmi_stats[i], 1ull)
#endif
#define PTMI_TSTAMP(v) const unsigned long long v = clock64()
#define PTMI_TADD(i, t0) PTMI_WADD(i, clock64() - (t0))
#define PTMI_TADD_ACTIVE(i, t0) PTMI_WADD(i, clock64() - (t0))
#define PTMI_COUNT_ACTIVE(i) PTMI_WADD(i, 1ull)
#else
#define PTMI_COUNT(i) ((void)0)
#define PTMI_TSTAMP(v) ((void)0)
#define PTMI_TADD(i, t0) ((void)0)
#define PTMI_TADD_ACTIVE(i, t0) ((void)0)
#define PTMI_COUNT_ACTIVE(i) ((void)0)
#define PTMI_WADD(i, v) ((void)0)
#endif

// PTMI_CAPTURE: DIAGNOSTIC build (make capture) -- the mesh kernels record each BVH walk
// of their walk phases (the ray, the primitive best it starts from, and the result)
// into device buffers set by ptmi_diag_capture_setup, for the standalone walk kernels'
// measurement (tools/walk_bench.py).  Same images; the product has PTMI_CAPTURE == 0.
#ifndef PTMI_CAPTURE
#define PTMI_CAPTURE 0
#endif
// PTMI_TIMELINE: DIAGNOSTIC build (make timeline) -- trace_kernel records each work
// item's start and end (wall_clock64, lane 0, vector stores) into a device buffer set by
// ptmi_diag_timeline_setup, for the launch's ramp / tail analysis (tools/timeline.py).
// Same images; the product has PTMI_TIMELINE == 0.
#ifndef PTMI_TIMELINE
#define PTMI_TIMELINE 0
#endif
// DIAGNOSTIC study build (make study): the standalone walk kernels, the split execution
// form and the measured tile order -- measured alternatives, compiled
// out of the product library.
#ifndef PTMI_STUDY
#define PTMI_STUDY 0
#endif

// Round-6 instruction cuts of the bounce loop (each a switch, measured one by one on the GPU;
// profiles/r6/SUMMARY.md).  Every one leaves the images bit-identical.
#ifndef PTMI_R6_LOOP
#define PTMI_R6_LOOP 1  // the hit scoped to the active block (no loop-carried copies)
#endif
#ifndef PTMI_R6_SPH
#define PTMI_R6_SPH 1  // deferred sphere roots: first sphere taken without selects, (slot, key) packed
#endif
#ifndef PTMI_R6_SLOT
#define PTMI_R6_SLOT 1  // hemisphere-table slot test: one conversion pair, no range test
#endif
#ifndef PTMI_R6_PLNZ
#define PTMI_R6_PLNZ 0  // affine planes past the floor / ceiling run: +-0 row entries skipped by pattern
                        // (measured slower: C2 +0.8 %, C3 +2.3 %, profiles/r6/SUMMARY.md)
#endif
#ifndef PTMI_R6_VACC
#define PTMI_R6_VACC 1  // the per-pixel colour sums really in LDS (volatile slots), not promoted to VGPRs
#endif
#ifndef PTMI_R6_FRACT
#define PTMI_R6_FRACT 1  // noise fract as v_fract_f32 (exhaustively checked equal to ocml's fract)
#endif
#ifndef PTMI_R6_NPAIR
#define PTMI_R6_NPAIR 0  // the two draws of a noise3D pair evaluated together (ptmi_sinf.h noise_sinf2):
                         // 1 both sites, 2 camera only, 3 hemisphere only.  Measured slower, C2 +0.6 / +0.3 /
                         // +0.5 % (its two interleaved chains hold more registers at the peak)
#endif

namespace ptmi {

#if PTMI_TIMELINE
__device__ unsigned long long* ptmi_tl;
__device__ unsigned ptmi_tl_max;
#endif

#if PTMI_CAPTURE
__device__ WalkReq* ptmi_cap_req;
__device__ WalkRes* ptmi_cap_res;
__device__ unsigned ptmi_cap_n, ptmi_cap_max;
#endif

static constexpr unsigned kMaxEffectiveBounces = 4;  // tracer.cl:2
static constexpr unsigned kMaxBounces = 10;          // tracer.cl:3
static constexpr double kEps = 0.0001;               // tracer.cl:4
static constexpr double kPi = (double)3.14159265359f;  // tracer.cl:1 (a float literal)
// Camera-ray refill of a wave (trace_kernel): when kRefillNeed lanes have an empty
// buffer (64: all of them), or kRefillStarve lanes sit idle without a path.  Full
// batches amortise the camera block; measured on C2 (512 spp): 24/6 61.9 ms,
// 40/10 61.1, 60/24 60.3, 64/24 59.7; the group scenes prefer 64/12.
#ifndef PTMI_REFILL_NEED
#define PTMI_REFILL_NEED 64
#endif
#ifndef PTMI_REFILL_STARVE
#define PTMI_REFILL_STARVE 24
#endif
#ifndef PTMI_REFILL_STARVE_GROUPS
#define PTMI_REFILL_STARVE_GROUPS 12
#endif
static constexpr int kRefillNeed = PTMI_REFILL_NEED;
// The walk batch -- parked lanes that start a wave's BVH walk phase -- is a scene value since round 6
// (DevScene::walk_batch, chosen in ptmi_api.cpp).

struct d4 {
    double x, y, z, w;
};
__device__ __forceinline__ d4 mk(double x, double y, double z, double w) { return d4{x, y, z, w}; }
__device__ __forceinline__ d4 add4(d4 a, d4 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ d4 sub4(d4 a, d4 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ d4 scl4(d4 a, double s) { return mk(a.x * s, a.y * s, a.z * s, a.w * s); }
__device__ __forceinline__ d4 ld4(const double* p) { return mk(p[0], p[1], p[2], p[3]); }

// OpenCL dot/cross(double4) as ROCm device-libs implement them (fmuladd == fma).
__device__ __forceinline__ double dot4(d4 a, d4 b) {
    double d = a.x * b.x;
    d = fma(a.y, b.y, d);
    d = fma(a.z, b.z, d);
    return fma(a.w, b.w, d);
}
__device__ __forceinline__ d4 cross4(d4 a, d4 b) {
    return mk(fma(a.y, b.z, b.y * -a.z), fma(a.z, b.x, b.z * -a.x), fma(a.x, b.y, b.x * -a.y), 0.0);
}
// OpenCL normalize(double4) (opencl.bc): zero passthrough, range scaling, rsqrt.
__device__ __noinline__ d4 normalize4(d4 v) {
    if (v.x == 0.0 && v.y == 0.0 && v.z == 0.0 && v.w == 0.0) return v;
    double d = dot4(v, v);
    d4 p = v;
    if (d < 0x1p-1022) {
        p = scl4(v, 0x1p563);
        d = dot4(p, p);
    } else if (d == __builtin_inf()) {
        p = scl4(v, 0x1p-514);
        d = dot4(p, p);
        if (d == __builtin_inf()) {
            p = mk(copysign(isinf(p.x) ? 1.0 : 0.0, p.x), copysign(isinf(p.y) ? 1.0 : 0.0, p.y),
                   copysign(isinf(p.z) ? 1.0 : 0.0, p.z), copysign(isinf(p.w) ? 1.0 : 0.0, p.w));
            d = dot4(p, p);
        }
    }
    return scl4(p, rsqrt(d));
}
// Affine scenes (F_PROJ clear; ptmi_api.cpp checks at upload that the camera's
// and every object's inverse end in the row (+-0, +-0, +-0, 1), that the inverse
// transposes' column 3 is +-0 in rows 0-2 and that triangle normals are finite):
// points then carry w == 1 and directions w == 0 along every path, so every
// w-lane term of the reference's double4 arithmetic is an exact no-op (a +-0
// product or m * 1), up to the sign of an exact-zero result, which nothing
// observes.  With A = true the helpers below skip the w lane (and all w values
// become dead code); with A = false they are the literal double4 arithmetic.
template <bool A>
__device__ __forceinline__ double dotv(d4 a, d4 b) {  // dot of two directions (w == 0 when A)
    double d = a.x * b.x;
    d = fma(a.y, b.y, d);
    d = fma(a.z, b.z, d);
    return A ? d : fma(a.w, b.w, d);
}
// normalize of a direction, affine case: the w lane is 0 in and out.
__device__ __noinline__ d4 normalize3(double x, double y, double z) {
    if (x == 0.0 && y == 0.0 && z == 0.0) return mk(x, y, z, 0.0);
    double d = x * x;
    d = fma(y, y, d);
    d = fma(z, z, d);
    double px = x, py = y, pz = z;
    if (d < 0x1p-1022) {
        px = x * 0x1p563, py = y * 0x1p563, pz = z * 0x1p563;
        d = fma(pz, pz, fma(py, py, px * px));
    } else if (d == __builtin_inf()) {
        px = x * 0x1p-514, py = y * 0x1p-514, pz = z * 0x1p-514;
        d = fma(pz, pz, fma(py, py, px * px));
        if (d == __builtin_inf()) {
            px = copysign(isinf(px) ? 1.0 : 0.0, px);
            py = copysign(isinf(py) ? 1.0 : 0.0, py);
            pz = copysign(isinf(pz) ? 1.0 : 0.0, pz);
            d = fma(pz, pz, fma(py, py, px * px));
        }
    }
    // d is a positive normal here (zero returned above, tiny / huge rescaled): rsqrt's core
    const double s = (PTMI_ABLATE & 256) ? __builtin_amdgcn_rsq(d) : rsqrt_core(d);  // DIAGNOSTIC 256
    return mk(px * s, py * s, pz * s, 0.0);
}
// normalize3's main path alone -- for vectors whose squared length is known to be a
// positive normal double, where the zero test and the rescaling branches are identities.
__device__ __forceinline__ d4 norm3_core(d4 v) {
    double d = v.x * v.x;
    d = fma(v.y, v.y, d);
    d = fma(v.z, v.z, d);
    const double s = rsqrt_core(d);
    return mk(v.x * s, v.y * s, v.z * s, 0.0);
}
template <bool A>
__device__ __forceinline__ d4 normv(d4 v) {
    if constexpr (A) return normalize3(v.x, v.y, v.z);
    else return normalize4(v);
}

// maxX / minX (tracer.cl:110-111): OpenCL max/min -> maxnum/minnum.
__device__ __forceinline__ double max3(double a, double b, double c) { return fmax(fmax(a, b), c); }
__device__ __forceinline__ double min3(double a, double b, double c) { return fmin(fmin(a, b), c); }

// Uniform scene records (planes, spheres, group objects, traversal roots) are read through
// the constant address space: read-only for the kernel's lifetime, they stay scalar loads
// whatever the kernel writes before them (the mesh kernels' work-item atomic, take_item).
template <typename T>
using CPtr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ CPtr<T> cmem(const T* p) { return (CPtr<T>)p; }

// mul (tracer.cl:369-376): row-major mat4 x vec4, rows summed x+y+z+w.
template <typename M>
__device__ __forceinline__ d4 mat_mul(M m, d4 v) {
    return mk(((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * v.w,
              ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w,
              ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * v.w,
              ((m[12] * v.x + m[13] * v.y) + m[14] * v.z) + m[15] * v.w);
}

// mul() for a matrix with the scale+translate zero pattern
//   [a 0 0 d; 0 b 0 e; 0 0 c f; 0 0 0 g]   (DevObject::st, checked on the host).
// The reference's ((m0 x + m1 y) + m2 z) + m3 w with m1 = m2 = +-0 equals
// m0 x + m3 w bit-for-bit for a finite ray, up to the sign of an exact-zero
// result, which no branch or output of the path depends on (rays are finite
// here: see PathState::dead).
template <typename M>
__device__ __forceinline__ d4 xform_st(M m, d4 v) {
    return mk(m[0] * v.x + m[3] * v.w, m[5] * v.y + m[7] * v.w, m[10] * v.z + m[11] * v.w, m[15] * v.w);
}
template <typename M>
__device__ __forceinline__ d4 xform(M m, bool st, d4 v) {
    return st ? xform_st(m, v) : mat_mul(m, v);
}
// mul(m, point) / mul(m, direction): in the affine case m * 1 == m and
// m * 0 == +-0 make the w column an exact add of m[3] / a no-op, and row 3 is dead.
template <bool A, typename M>
__device__ __forceinline__ d4 xpt(M m, bool st, d4 v) {
    if constexpr (!A) return xform(m, st, v);
    if (st) return mk(m[0] * v.x + m[3], m[5] * v.y + m[7], m[10] * v.z + m[11], 1.0);
    return mk(((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3], ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7],
              ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11], 1.0);
}
template <bool A, typename M>
__device__ __forceinline__ d4 xdir(M m, bool st, d4 v) {
    if constexpr (!A) return xform(m, st, v);
    if (st) return mk(m[0] * v.x, m[5] * v.y, m[10] * v.z, 0.0);
    return mk((m[0] * v.x + m[1] * v.y) + m[2] * v.z, (m[4] * v.x + m[5] * v.y) + m[6] * v.z,
              (m[8] * v.x + m[9] * v.y) + m[10] * v.z, 0.0);
}

// Row 1 of mul() only (intersectPlane reads nothing else, tracer.cl:478-483).
__device__ __forceinline__ double row1(const double* __restrict__ m, bool st, d4 v) {
    return st ? m[5] * v.y + m[7] * v.w : ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w;
}

// ocml's sin_f32 out of line: only noise arguments >= 2^30, and the few lanes of
// [2^19, 2^30) near a tie or float midpoint that sinf_cw30 declines, reach it
// (2^19 is passed at sample indices above ~2210, or by the n*n of refractive
// materials), so its general reduction is not inlined into every noise call.
#ifndef PTMI_SIN_FALLBACK_INLINE
#define PTMI_SIN_FALLBACK_INLINE __noinline__
#endif
__device__ PTMI_SIN_FALLBACK_INLINE float sinf_ocml(float x) { return sinf(x); }

// noise3D (tracer.cl:314-317): float math, ocml sin_f32, ocml fract_f32.
__device__ __forceinline__ float noise3d(float x, float y, float z) {
    if (PTMI_ABLATE & 1) {
        float v = x * 0.6180339f + y * 0.3473f + z * 0.1234f;
        return v - floorf(v);
    }
    float a = x * 112.9898f;
    float b = y * 179.233f;
    float c = z * 237.212f;
    float s = (a + b) + c;
    if (PTMI_ABLATE & 32) s = s * 1e-6f;  // DIAGNOSTIC: small-argument sin path only
    // Every call site passes finite floats below 2^33 (fgi, fgi2 in [0, 1], sample and
    // bounce indices and n*n as u32), so s, sin(s) and v are finite and ocml fract's
    // NaN / inf cases (fract(NaN) = NaN, fract(inf) = 0) are unreachable.
    // ocml's sin_f32, bit for bit (ptmi_sinf.h noise_sinf): below 2^19 (every bench
    // argument) the specialised reduction, up to 2^30 (glass noise) an FP64 Cody-Waite
    // step, else and near ties ocml itself (out of line).
#if PTMI_STATS
    PTMI_WADD(40, 1ull);
    if (__ballot(fabsf(s) < 0x1p17f)) PTMI_WADD(37, 1ull);
    if (__ballot(fabsf(s) >= 0x1p17f && fabsf(s) < 0x1p19f)) PTMI_WADD(38, 1ull);
    if (__ballot(!(fabsf(s) < 0x1p19f))) PTMI_WADD(39, 1ull);
#endif
    const float sn = noise_sinf(s, [](float v) { return sinf_ocml(v); });
    float v = sn * 43758.5453f;
    // ocml's fract: min(v - floor(v), 0x1.fffffep-1).  v_fract_f32 returns the same bits for every
    // finite float (tests/test_gpu_rng.py, exhaustive on the GPU), in one instruction instead of three.
    if (PTMI_R6_FRACT) return __builtin_amdgcn_fractf(v);
    return fminf(v - floorf(v), 0x1.fffffep-1f);
}

// Two noise3D draws at once (the camera's offsets, the hemisphere's uniforms): each draw's
// arithmetic as in noise3d, the two sins through noise_sinf2, so the two dependent chains
// interleave (round 6).  Bit-identical to two noise3d calls (tests/test_gpu_rng.py).
__device__ __forceinline__ void noise3d_pair(float x1, float y1, float z1, float x2, float y2, float z2, float& u1,
                                             float& u2) {
    if (PTMI_ABLATE & 33) {  // (DIAGNOSTIC ablations of noise3d)
        u1 = noise3d(x1, y1, z1);
        u2 = noise3d(x2, y2, z2);
        return;
    }
    const float s1 = (x1 * 112.9898f + y1 * 179.233f) + z1 * 237.212f;
    const float s2 = (x2 * 112.9898f + y2 * 179.233f) + z2 * 237.212f;
#if PTMI_STATS
    PTMI_WADD(40, 2ull);
    if (__ballot(fabsf(s1) < 0x1p17f || fabsf(s2) < 0x1p17f)) PTMI_WADD(37, 2ull);
    if (__ballot((fabsf(s1) >= 0x1p17f && fabsf(s1) < 0x1p19f) || (fabsf(s2) >= 0x1p17f && fabsf(s2) < 0x1p19f)))
        PTMI_WADD(38, 2ull);
    if (__ballot(!(fabsf(s1) < 0x1p19f) || !(fabsf(s2) < 0x1p19f))) PTMI_WADD(39, 2ull);
#endif
    float sn1, sn2;
    noise_sinf2(s1, s2, [](float v) { return sinf_ocml(v); }, sn1, sn2);
    const float v1 = sn1 * 43758.5453f, v2 = sn2 * 43758.5453f;
    u1 = PTMI_R6_FRACT ? __builtin_amdgcn_fractf(v1) : fminf(v1 - floorf(v1), 0x1.fffffep-1f);
    u2 = PTMI_R6_FRACT ? __builtin_amdgcn_fractf(v2) : fminf(v2 - floorf(v2), 0x1.fffffep-1f);
}

// ---- Opt-in statistical RNG (F_XRNG, ptmi_scene_set_rng) ---------------------------
// The reference's noise3D (above) is a hash of (seed, sample, bounce) through a float
// sin with large-argument reductions -- the parity path keeps it bit for bit.  The
// statistical mode draws the same uniforms from xoshiro128** (Blackman & Vigna): one
// stream per path, seeded from the pixel's seed bits and the sample index through a
// 32-bit hash (xseed), so the image does not depend on which lane, chunk or GPU traces
// a sample; the camera's two anti-aliasing offsets come from two more hashes of the
// same pair.  Uniform floats are the top 24 bits x 2^-24, in [0, 1) like fract.
struct Xrng {
    uint32_t s0, s1, s2, s3;
};
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
__device__ __forceinline__ float xnext(Xrng& r) {
    const uint32_t res = rotl32(r.s1 * 5u, 7) * 9u;
    const uint32_t t = r.s1 << 9;
    r.s2 ^= r.s0;
    r.s3 ^= r.s1;
    r.s1 ^= r.s2;
    r.s0 ^= r.s3;
    r.s2 ^= t;
    r.s3 = rotl32(r.s3, 11);
    return (float)(res >> 8) * 0x1p-24f;
}
// The hemisphere's two draws at 16 bits (k 2^-16): on the grid of the hemisphere table
// (random_hemisphere), so the statistical mode never evaluates the sincos / sqrt chain
// there.  A 2^-16 step in u is ~1e-4 rad of direction, far below the Monte-Carlo noise.
__device__ __forceinline__ float xnext16(Xrng& r) {
    const uint32_t res = rotl32(r.s1 * 5u, 7) * 9u;
    const uint32_t t = r.s1 << 9;
    r.s2 ^= r.s0;
    r.s3 ^= r.s1;
    r.s1 ^= r.s2;
    r.s0 ^= r.s3;
    r.s2 ^= t;
    r.s3 = rotl32(r.s3, 11);
    return (float)(res >> 16) * 0x1p-16f;
}
#ifndef PTMI_XSEED32
#define PTMI_XSEED32 1
#endif
// 32-bit integer finaliser (lowbias32 form: two 32-bit multiplies, three xor-shifts).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
#if PTMI_XSEED32
// The pixel's stream key: its seed's 64 bits folded once per work item into two 32-bit
// words (xseed_of), so a path seeds from (key, n) with 32-bit multiplies only.  xoshiro128**'s
// state words s0 / s1 finalise (key.lo ^ nG) / (key.hi ^ nG), s2 / s3 finalise those mixed
// with the other key word: eight 32-bit multiplies per path (round 3 took two SplitMix64
// draws, four 64-bit multiplies, and a third for the camera).  Both key words enter the
// state (a key of 32 bits alone gave 2^32 streams, so a 1080p x 2048-spp frame,
// ~4.2e9 paths, reused streams across pixels).
struct XSeed {
    uint32_t lo, hi;
};
__device__ __forceinline__ XSeed xseed_of(uint64_t seed_bits) {
    const uint32_t a = (uint32_t)seed_bits, b = (uint32_t)(seed_bits >> 32);
    return XSeed{mix32(a ^ mix32(b + 0x9E3779B9u)), mix32(b ^ mix32(a + 0x85EBCA6Bu))};
}
__device__ __forceinline__ Xrng xseed(XSeed key, uint32_t n) {
    const uint32_t g = n * 0x9E3779B9u;
    const uint32_t s0 = mix32((key.lo ^ g) + 0x632BE5ABu), s1 = mix32((key.hi ^ g) + 0x85157AF5u);
    Xrng r{s0, s1, mix32((s0 ^ key.hi) + 0x2545F491u), mix32((s1 ^ key.lo) + 0xB5297A4Du)};
    if ((r.s0 | r.s1 | r.s2 | r.s3) == 0) r.s0 = 1;  // the all-zero state is the one fixed point
    return r;
}
__device__ __forceinline__ void xcamera(XSeed key, uint32_t n, float& rx, float& ry) {
    const uint32_t g = n * 0x9E3779B9u;
    rx = (float)(mix32(((key.lo ^ g) + key.hi) ^ 0x68E31DA4u) >> 8) * 0x1p-24f;
    ry = (float)(mix32(((key.hi ^ g) + key.lo) ^ 0x1B56C4E9u) >> 8) * 0x1p-24f;
}
#else
typedef uint64_t XSeed;
__device__ __forceinline__ XSeed xseed_of(uint64_t seed_bits) { return seed_bits; }
__device__ __forceinline__ Xrng xseed(XSeed seed_bits, uint32_t n) {
    const uint64_t base = seed_bits ^ (0x9E3779B97F4A7C15ull * ((uint64_t)n + 1));
    const uint64_t a = splitmix64(base + 0x9E3779B97F4A7C15ull), b = splitmix64(base + 0x3C6EF372FE94F82Aull);
    Xrng r{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
    if ((r.s0 | r.s1 | r.s2 | r.s3) == 0) r.s0 = 1;  // the all-zero state is the one fixed point
    return r;
}
__device__ __forceinline__ void xcamera(XSeed seed_bits, uint32_t n, float& rx, float& ry) {
    const uint64_t v = splitmix64(seed_bits + 0xD1B54A32D192ED03ull * ((uint64_t)n + 1));
    rx = (float)(uint32_t)(v >> 40) * 0x1p-24f;
    ry = (float)(uint32_t)((v >> 16) & 0xFFFFFFu) * 0x1p-24f;
}
#endif
// checkAxis (tracer.cl:250-268)
__device__ __forceinline__ void check_axis(double o, double d, double mn, double mx, double& t0, double& t1) {
    double a0 = mn - o, a1 = mx - o;
    double a, b;
    if (fabs(d) >= kEps) {
        a = a0 / d;
        b = a1 / d;
    } else {
        a = a0 * __builtin_huge_val();
        b = a1 * __builtin_huge_val();
    }
    t0 = a > b ? b : a;
    t1 = a > b ? a : b;
}

// intersectRayWithBox (tracer.cl:270-280): a line test (no t range).
__device__ __forceinline__ bool ray_box(d4 o, d4 d, const double* mn, const double* mx) {
    double x0, x1, y0, y1, z0, z1;
    check_axis(o.x, d.x, mn[0], mx[0], x0, x1);
    check_axis(o.y, d.y, mn[1], mx[1], y0, y1);
    check_axis(o.z, d.z, mn[2], mx[2], z0, z1);
    return max3(x0, y0, z0) < min3(x1, y1, z1);
}

struct Hit {
    double t;
    int pk;     // (key << 16) | slot: the object's index in the reference's list and its
                // slot in DevScene::objs (type-run order); -1 = no hit.  One select per
                // candidate instead of two, and key order is pk order (keys are distinct).
    int tri;    // reference triangle index, -1 for other shapes
    int ti;     // a winning triangle's leaf-order index (DevScene::tris): its gate chain and
                // barycentrics are re-derived from it after the walks, so they are not
                // carried through the traversal loop (registers)
    double u, v;
};

// The reference records every candidate, then picks the FIRST (in recording
// order) t > EPSILON that is strictly below the running best, which starts at
// 1024 (tracer.cl:728-739).  Objects are visited here in type runs, not in
// list order, so a tie in t is broken by the object's list index: the winner is
// the lexicographic minimum (t, key) -- the same candidate.  Candidates of one
// object are still produced in the reference's order (strict < keeps the first).
// Evaluated without short-circuits: compares and mask ops, no exec-mask branches.
__device__ __forceinline__ int pack_hit(int slot, int key) { return (key << 16) | slot; }
__device__ __forceinline__ int hit_obj(const Hit& h) { return h.pk < 0 ? -1 : (h.pk & 0xFFFF); }
__device__ __forceinline__ bool better(const Hit& h, double t, int pk) {
    return (t > kEps) & ((t < h.t) | ((t == h.t) & (pk < h.pk)));
}
// Triangles of one group object are recorded by the reference in increasing
// triangle index (nodes are numbered, and their triangles appended, in the same
// preorder the walk follows: scene.go:96-155, tracer.cl:621-719), so a tie in
// (t, object) is broken by the triangle index.
__device__ __forceinline__ bool better_tri(const Hit& h, double t, int pk, int tri) {
    return t > kEps && (t < h.t || (t == h.t && (pk < h.pk || (pk == h.pk && tri < h.tri))));
}
__device__ __forceinline__ void consider(Hit& h, double t, int obj, int key) {
    const int pk = pack_hit(obj, key);
    if (better(h, t, pk)) {
        h.t = t;
        h.pk = pk;
        h.tri = -1;
    }
}

// Scene-feature flags: the host inspects the records once and launches the
// instantiation that compiles out absent object types / materials / DoF.  Every
// type or material present in the scene keeps its flag, so the result is the
// same as the generic path.
enum : int {
    F_GROUPS = 1,     // a type-4 object with BVH roots
    F_CYLCUBE = 2,    // cylinders or cubes present
    F_MATERIALS = 4,  // reflectivity != 0 or refractive index != 1 somewhere
    F_DOF = 8,        // camera aperture != 0
    F_ALL = 15,
    F_PROJ = 16,      // not affine (see dotv): the literal double4 arithmetic, generic path only
    F_TEX = 32,       // textured objects: with F_ALL | F_PROJ, the one textured instantiation
    F_TLIST = 128,    // tile-split launch with an owned-tile list (WorkPlan::tiles): affine mesh kernels only
    F_XRNG = 64,      // opt-in statistical mode (ptmi_scene_set_rng): xoshiro128** instead of noise3D,
                      // affine instantiations only; never the parity path
    F_WIDE = 256      // affine mesh scene whose child codes need 31 bits (>= 2^15 Node4s or triangles):
                      // the affine kernel with a 32-bit LDS traversal stack (one F_ALL | F_WIDE
                      // instantiation, +- F_XRNG; ADVICE r5: such scenes had been sent to F_PROJ)
};

// The camera ray's two anti-aliasing offsets of sample n (tracer.cl:869).
template <int FL>
__device__ __forceinline__ void camera_offsets(float fgi, float fgi2, XSeed seed_bits, uint32_t n, float& rx,
                                               float& ry) {
    if constexpr ((FL & F_XRNG) != 0) {
        xcamera(seed_bits, n, rx, ry);
    } else {
        if (PTMI_R6_NPAIR == 1 || PTMI_R6_NPAIR == 2) {
            noise3d_pair(fgi, (float)n, fgi2, fgi, fgi2, (float)n, rx, ry);
        } else {
            rx = noise3d(fgi, (float)n, fgi2);
            ry = noise3d(fgi, fgi2, (float)n);
        }
    }
}

// Threads per workgroup of trace_kernel: one wave.  A wave that finishes its work
// item frees its slot (LDS included) at once; with 4-wave groups the slot waited for
// the slowest of the four (measured, 256 spp: teapot 118.9 -> 116.7 ms, gopher
// 189.0 -> 177.1 ms, C2 236.0 -> 235.3 ms per 2048 spp).  BVH scenes then stage
// only the top 3 levels of the traversal index per group (kLdsNodes).
static constexpr int kBlock = 64;
// Per-lane traversal stacks are lane-interleaved: entry k of lane t at [k * kStkStride + t].
static constexpr int kStkStride = kBlock;


// intersectRayWithBox (tracer.cl:270-280) returning the line's slab interval.
// The hit decision tmin < tmax is the reference's, bit for bit.
__device__ __forceinline__ bool ray_box_t(d4 o, d4 d, const double* mn, const double* mx, double& tmin,
                                          double& tmax) {
    double x0, x1, y0, y1, z0, z1;
    check_axis(o.x, d.x, mn[0], mx[0], x0, x1);
    check_axis(o.y, d.y, mn[1], mx[1], y0, y1);
    check_axis(o.z, d.z, mn[2], mx[2], z0, z1);
    tmin = max3(x0, y0, z0);
    tmax = min3(x1, y1, z1);
    return tmin < tmax;
}

// Conservative slack for pruning by t: computed Moller-Trumbore t values and
// slab bounds each carry ~1e-16 relative rounding error (~1e-12 absolute at the
// reference's det >= 1e-4); 1e-9 (1 + t) is orders of magnitude larger.
__device__ __forceinline__ double prune_margin(double t) { return 1e-9 * (1.0 + fabs(t)); }

// 1/d for the conservative (margin-widened) traversal tests only -- never for a
// value the reference computes: v_rcp_f64 plus one Newton step (relative error
// <= ~2^-40 from the hardware estimate's ~2^-23; every consumer widens by >= 2^-30);
// zero / denormal / non-finite d takes the exact quotient.
__device__ __forceinline__ double rcp_walk(double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    double r = fma(r0, fma(-d, r0, 1.0), r0);
    if (!isfinite(r) || !(fabs(d) > 0x1p-1000)) r = 1.0 / d;
    return r;
}

// One slab of intersectRayWithBox evaluated with the ray's reciprocal instead of
// the reference's division: |a*r - RN(a/d)| <= 3u|a/d| (u = 2^-53), bounded here
// by e = 2^-50 |a*r| + tiny.  Axes with |d| < EPSILON are computed exactly as the
// reference does (a * +inf, possibly NaN) with e = 0.
__device__ __forceinline__ void slab_fast(double o, double d, double r, double mn, double mx, double& lo,
                                          double& hi, double& e) {
    const double a0 = mn - o, a1 = mx - o;
    const bool big = fabs(d) >= kEps;
    const double a = big ? a0 * r : a0 * __builtin_huge_val();
    const double b = big ? a1 * r : a1 * __builtin_huge_val();
    lo = a > b ? b : a;  // the reference's swap (tracer.cl:263-266)
    hi = a > b ? a : b;
    e = big ? fmax(fabs(a), fabs(b)) * 0x1p-50 + 0x1p-1000 : 0.0;
}

// intersectRayWithBox (tracer.cl:270-280), decision bit-identical to ray_box_t:
// interval bounds on the reference's tmin = max(x0,y0,z0), tmax = min(x1,y1,z1)
// decide almost every box; only boxes within rounding distance of the decision
// boundary (or with non-finite bounds) are recomputed with the exact divisions.
// [tlo, thi] bound the reference's (tmin, tmax) for pruning.
__device__ __forceinline__ bool ray_box_ref(d4 o, d4 d, d4 r, const double* mn, const double* mx, double& tlo,
                                            double& thi) {
    double xl, xh, xe, yl, yh, ye, zl, zh, ze;
    slab_fast(o.x, d.x, r.x, mn[0], mx[0], xl, xh, xe);
    slab_fast(o.y, d.y, r.y, mn[1], mx[1], yl, yh, ye);
    slab_fast(o.z, d.z, r.z, mn[2], mx[2], zl, zh, ze);
    const double t0lo = max3(xl - xe, yl - ye, zl - ze), t0hi = max3(xl + xe, yl + ye, zl + ze);
    const double t1lo = min3(xh - xe, yh - ye, zh - ze), t1hi = min3(xh + xe, yh + ye, zh + ze);
    tlo = t0lo;
    thi = t1hi;
    if (t0hi < t1lo) return true;    // every tmin <= t0hi < t1lo <= every tmax
    if (t0lo >= t1hi) return false;  // every tmin >= t0lo >= t1hi >= every tmax
    double a, b;                     // undecided (or NaN bounds): the reference's arithmetic
    const bool hit = ray_box_t(o, d, mn, mx, a, b);
    tlo = a;
    thi = b;
    return hit;
}

// Moller-Trumbore (tracer.cl:640-675) on the 3 live components: the w terms of
// the reference's dot() products multiply a cross() result whose w is exactly 0.
__device__ __forceinline__ bool verify_chain(const DevScene& S, int chain, d4 o, d4 d);
__device__ __forceinline__ bool chain_certified(const DevScene& S, int chain, d4 o, d4 d, double t);

template <bool kVerify>
__device__ __forceinline__ void tri_test(const DevScene& S, const DevTri& T, int ti, d4 o, d4 d, int slot, int key,
                                         Hit& h, int& vchain) {
    const double e1x = T.e1[0], e1y = T.e1[1], e1z = T.e1[2];
    const double e2x = T.e2[0], e2y = T.e2[1], e2z = T.e2[2];
    // dirCrossE2 = cross(d, e2)
    const double cx = fma(d.y, e2z, e2y * -d.z), cy = fma(d.z, e2x, e2z * -d.x), cz = fma(d.x, e2y, e2x * -d.y);
    double det = e1x * cx;
    det = fma(e1y, cy, det);
    det = fma(e1z, cz, det);
    if (fabs(det) < kEps) return;
    const double px = o.x - T.p1[0], py = o.y - T.p1[1], pz = o.z - T.p1[2];
    double du = px * cx;
    du = fma(py, cy, du);
    du = fma(pz, cz, du);
    // u = (1/det) * du.  Reject before the reciprocal when the sign alone (u < 0)
    // or |du| >= 2|det| (u > 1 after rounding) decides it.
    if ((du < 0.0) != (det < 0.0) && du != 0.0) return;
    if (fabs(du) >= 2.0 * fabs(det)) return;
    const double f = 1.0 / det;
    const double u = f * du;
    if (u < 0 || u > 1) return;
    // originCrossE1 = cross(p1ToOrigin, e1)
    const double qx = fma(py, e1z, e1y * -pz), qy = fma(pz, e1x, e1z * -px), qz = fma(px, e1y, e1x * -py);
    double dv = d.x * qx;
    dv = fma(d.y, qy, dv);
    dv = fma(d.z, qz, dv);
    const double v = f * dv;
    if (v < 0 || (u + v) > 1) return;
    double dt = e2x * qx;
    dt = fma(e2y, qy, dt);
    dt = fma(e2z, qz, dt);
    const double t = f * dt;
    const int n = T.n;
    if (better_tri(h, t, pack_hit(slot, key), n)) {
        const int c = T.chain & kChainMask;
        // Eager mode admits the hit only if the reference would have tested this
        // triangle: its gate chain (root -> its node) passes the exact line-box
        // tests.  The fast mode takes it tentatively; group_walks verifies the
        // final winner.
        if (kVerify && c != vchain) {
            if (!chain_certified(S, c, o, d, t) && !verify_chain(S, c, o, d)) {
                PTMI_COUNT(5);  // (stats build: gate rejections)
                return;
            }
            vchain = c;
        }
        h.ti = ti;
        h.t = t;
        h.pk = pack_hit(slot, key);
        h.tri = n;
    }
}

// The barycentrics of tri_test's hit, re-derived with its operations (bit-identical).
__device__ __forceinline__ void tri_uv(const DevTri& T, d4 o, d4 d, double& u, double& v) {
    const double e1x = T.e1[0], e1y = T.e1[1], e1z = T.e1[2];
    const double e2x = T.e2[0], e2y = T.e2[1], e2z = T.e2[2];
    const double cx = fma(d.y, e2z, e2y * -d.z), cy = fma(d.z, e2x, e2z * -d.x), cz = fma(d.x, e2y, e2x * -d.y);
    double det = e1x * cx;
    det = fma(e1y, cy, det);
    det = fma(e1z, cz, det);
    const double px = o.x - T.p1[0], py = o.y - T.p1[1], pz = o.z - T.p1[2];
    double du = px * cx;
    du = fma(py, cy, du);
    du = fma(pz, cz, du);
    const double f = 1.0 / det;
    u = f * du;
    const double qx = fma(py, e1z, e1y * -pz), qy = fma(pz, e1x, e1z * -px), qz = fma(px, e1y, e1x * -py);
    double dv = d.x * qx;
    dv = fma(d.y, qy, dv);
    dv = fma(d.z, qz, dv);
    v = f * dv;
}

#ifndef PTMI_STACK
#define PTMI_STACK 24
#endif
#ifndef PTMI_GROUP_ACM
#define PTMI_GROUP_ACM 1
#endif
#ifndef PTMI_GROUP_MASK
#define PTMI_GROUP_MASK 1
#endif
#ifndef PTMI_NCUR_LDS
#define PTMI_NCUR_LDS 1
#endif
// Per-lane LDS traversal stack: a Node4 visit pushes <= 3 entries and BVH4 chains are <= 7
// nodes long (ptmi_bvh.cpp checks it), so a walk holds <= 21 entries.
static constexpr int kStack = PTMI_STACK;
static_assert(kStack >= 21, "the BVH4 depth bound of ptmi_bvh.cpp needs 21 stack entries");
// The traversal stack's pointer types: LDS (address space 3), so every push and pop is a
// ds_write / ds_read whatever the optimiser makes of the pointer (a loop-carried generic
// pointer had turned the pop into a flat load).  Entries are child codes (ptmi_device.h
// Node4): 16 bits in the affine instantiations, whose scenes the host keeps to 16-bit
// codes (ptmi_bvh.cpp finalize_index_codes; 3 KB of stack per wave instead of 6 KB), 32
// bits in the generic ones.
typedef __attribute__((address_space(3))) int LdsInt;
typedef __attribute__((address_space(3))) uint16_t LdsU16;
__device__ __forceinline__ LdsInt* lds_ptr(int* p) { return (LdsInt*)p; }
__device__ __forceinline__ LdsU16* lds_ptr(uint16_t* p) { return (LdsU16*)p; }
template <bool A>
using StackEntry = typename std::conditional<A, uint16_t, int>::type;
// The leaf bit of the codes a stack of entry type E walks: 16-bit entries hold only narrow
// codes (a literal); 32-bit stacks take the scene's (a scalar).
template <typename E>
__device__ __forceinline__ int leaf_bit_of(const DevScene& S) {
    if constexpr (sizeof(E) == 2) return kLeafNarrow;
    else return S.leaf_bit;
}

// The reference's gate for one triangle: every reference node on the path from
// the walked root to the triangle's node passes intersectRayWithBox
// (tracer.cl:617-719).  Boxes are contiguous, so their loads are independent.
__device__ __forceinline__ bool verify_chain(const DevScene& S, int chain, d4 o, d4 d) {
    chain &= kChainMask;  // (bit 31: the leaf's last triangle)
    const d4 r = mk(1.0 / d.x, 1.0 / d.y, 1.0 / d.z, 0.0);  // recomputed: rare, and keeps r out of the walk
    const ChainBox* B = S.chains + (chain >> 5);
    const int len = chain & 31;
    PTMI_COUNT(17);  // (stats build: exact chain verifications, i.e. certificate failures)
    for (int i = 0; i < len; i++) {
        double a, b;
        if (!ray_box_ref(o, d, r, B[i].mn, B[i].mx, a, b)) return false;
    }
    return true;
}

// Certificate for the reference's gate chain of a hit at parameter t: the point
// o + t d lies strictly inside the chain's core box (the intersection of all its
// boxes) by a margin above the rounding of both this test and the reference's slab
// arithmetic, on every axis the reference divides by (|d| >= EPSILON); on the
// axes it treats as parallel (+-HUGE_VAL slabs) the origin itself lies strictly
// inside.  Then every box's computed slab interval contains t, so
// intersectRayWithBox passes for each of them (tmin <= t... < ...tmax) and
// verify_chain would return true.  Margin per axis: 2^-46 (|t d| + |o| + |mn| + |mx|),
// about 100x the 5 ulps the argument needs (error of o + t*d, plus the division's
// 2 roundings relative to |mn - o|).  NaN anywhere fails every test: no certificate.
__device__ __forceinline__ bool chain_certified(const DevScene& S, int chain, d4 o, d4 d, double t) {
    chain &= kChainMask;
    const ChainBox& C = S.chains[(chain >> 5) + (chain & 31)];
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const double td = t * dd[a];
        const double p = oo[a] + td;
        const double m = 0x1p-46 * (((fabs(td) + fabs(oo[a])) + fabs(C.mn[a])) + fabs(C.mx[a])) + 0x1p-1000;
        const bool in_div = (p > C.mn[a] + m) & (p < C.mx[a] - m);
        const bool in_par = (oo[a] > C.mn[a]) & (oo[a] < C.mx[a]);
        ok = ok & (fabs(dd[a]) >= kEps ? in_div : in_par);
    }
    return ok;
}

// Conservative slab test against a widened traversal box: false only when no
// t in [kEps, h.t] (with margins) can lie in the box.  A NaN bound (NaN ray)
// fails every comparison, so the box is entered.
__device__ __forceinline__ bool cull_box(d4 o, d4 r, double mnx, double mny, double mnz, double mxx, double mxy,
                                         double mxz, double lim, double& tn) {
    const double ax = (mnx - o.x) * r.x, bx = (mxx - o.x) * r.x;
    const double ay = (mny - o.y) * r.y, by = (mxy - o.y) * r.y;
    const double az = (mnz - o.z) * r.z, bz = (mxz - o.z) * r.z;
    tn = max3(fmin(ax, bx), fmin(ay, by), fmin(az, bz));
    const double tf = min3(fmax(ax, bx), fmax(ay, by), fmax(az, bz));
    return tn > tf || tn > lim || tf + prune_margin(tf) < kEps;
}

// A walk's FP32 ray, in the root's frame (RootRec: bounds b' = b - ctr stored as
// b' / sc).  With of = (float)(o - ctr), r = (float)(1/d) (|r| clamped to 1e30) and
// t' = fma(b' / sc, r * sc, -RN(of * r)) = fma(b', r, -RN(of * r)) (sc a power of two:
// r * sc is exact), the computed slab bound differs from the exact (b - o)/d = (b' - o')/d
// by at most e = 2^-23 |r| (|b'| + 2|o'|) (FP32 roundings of o', r, the product and the
// fma; the double rounding of o - ctr adds 2^-53 |o'|); each axis interval is widened by
// dt = 4e, so the test only rejects boxes the exact line misses.  The widening is folded
// into the offsets: entry = fma(near, rf, -(of r + dt)), exit = fma(far, rf, -(of r - dt)),
// whose extra roundings (of the offset sum, <= 2^-24 |of r + dt|, and of the one fma
// instead of fma then add) stay below e, inside the 3e of slack.  `neg`: the direction's
// sign per axis, which picks the entry (near) and exit (far) planes: min and max of the
// node's bounds for r >= 0, max and min for r < 0.
struct WalkRay {
    float rf[3];   // r * sc
    float olo[3];  // of * r + dt
    float ohi[3];  // of * r - dt
    bool neg[3];   // r < 0
};
template <typename RR>  // RootRec, generic or constant address space
__device__ __forceinline__ WalkRay walk_setup(d4 o, d4 rw, const RR& R) {
    const double oo[3] = {o.x, o.y, o.z}, rr[3] = {rw.x, rw.y, rw.z};
    float omax = 0.0f;
    float r[3], ofr[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float of = (float)(oo[a] - R.ctr[a]);
        r[a] = fminf(fmaxf((float)rr[a], -1e30f), 1e30f);  // rcp_walk: within 2^-40 of 1/d; NaN stays NaN
        ofr[a] = of * r[a];
        omax = fmaxf(omax, fabsf(of));
    }
    const float E = 0x1p-21f * (R.bmax + 2.0f * omax) + 0x1p-120f;
    WalkRay W;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float dt = E * fabsf(r[a]);
        W.olo[a] = ofr[a] + dt;
        W.ohi[a] = ofr[a] - dt;
        W.rf[a] = r[a] * R.sc;  // <= 1e30 * 2^28 < FLT_MAX
        W.neg[a] = r[a] < 0.0f;  // NaN: false (every slab value is NaN anyway)
    }
    return W;
}

// The pruning limit of the FP32 child tests, >= h.t + prune_margin(h.t): it changes only
// when a leaf improves the best hit, so the walk keeps it in a register.
__device__ __forceinline__ float walk_limit(double ht) {
    const double limd = ht + prune_margin(ht);
    return (float)limd * (1.0f + 0x1p-22f) + 0x1p-100f;
}

// Child order keys: a child's entry distance tn >= 0 (or +inf when culled) in the high
// word and its code in the low word of a double.  Float bits of non-negative values are
// ordered like the values, and 2^20 is added to the high word so the double is always a
// normal number (no denormal or NaN pattern: the high word stays in [2^20, 0x7f900000]),
// so v_min_f64 / v_max_f64 order the children by entry distance with one instruction per
// side of a compare-exchange.  (A -0 from the clamp gives a negative key: it sorts first,
// and the signed compare below still counts it as entered.)
static constexpr int32_t kKeyBias = 0x00100000;
static constexpr int32_t kKeyCulled = 0x7f800000 + kKeyBias;
__device__ __forceinline__ double child_key(float tn, int code) {
    const uint32_t hi = (uint32_t)(__float_as_int(tn) + kKeyBias);
    return __hiloint2double((int)hi, code);
}
__device__ __forceinline__ bool key_entered(double k) { return __double2hiint(k) < kKeyCulled; }
__device__ __forceinline__ int key_code(double k) { return __double2loint(k); }

// The four child slab tests of Node4 `cur` (one walk step): keys of its children.
#ifndef PTMI_STACKLESS
#define PTMI_STACKLESS 0  // DIAGNOSTIC (study builds): the stackless walk (walk_index_stackless)
#endif
__device__ __forceinline__ void node_children(const DevScene& S, int cur, const WalkRay& W, float lim, double k[4],
                                              int* parent = nullptr) {
    // The node's 64 B as four 16-B global loads issued together (one wait).  Bounds are
    // binary16 (ptmi_device.h), converted exactly to float inside v_fma_mix_f32, so the
    // slab test is the float-box one; a bound past the binary16 range is +-inf, whose
    // slab value is +-inf, exact.  Row a holds the four minima (.x, .y) and the four
    // maxima (.z, .w) of axis a; the ray's sign picks entry and exit halves (2 selects
    // per half and axis), so each child needs one fma per plane and no min / max per axis.
    const uint4* src = reinterpret_cast<const uint4*>(S.nodes4) + 4 * cur;
    uint4 q[4];
#pragma unroll
    for (int u = 0; u < 4; u++) q[u] = src[u];
    uint32_t nr[3][2], fr[3][2];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        nr[a][0] = W.neg[a] ? q[a].z : q[a].x;
        nr[a][1] = W.neg[a] ? q[a].w : q[a].y;
        fr[a][0] = W.neg[a] ? q[a].x : q[a].z;
        fr[a][1] = W.neg[a] ? q[a].y : q[a].w;
    }
    auto h16 = [](uint32_t w, int i) {
        return (float)__builtin_bit_cast(_Float16, (uint16_t)((i & 1) ? (w >> 16) : (w & 0xffffu)));
    };
#if PTMI_STACKLESS
    // (stackless study: child[0]'s high half holds the node's parent -- finalize_index_codes packs
    // it for narrow-code scenes only, so wide codes keep all their bits)
    const bool packed = S.leaf_bit == kLeafNarrow;
    const int ch[4] = {(int)(packed ? (q[3].x & 0xFFFFu) : q[3].x), (int)q[3].y, (int)q[3].z, (int)q[3].w};
    if (parent) *parent = (int)(q[3].x >> 16);
#else
    const int ch[4] = {(int)q[3].x, (int)q[3].y, (int)q[3].z, (int)q[3].w};
#endif
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float tn = 0.0f, tf = lim;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            tn = fmaxf(tn, fmaf(h16(nr[a][i >> 1], i), W.rf[a], -W.olo[a]));
            tf = fminf(tf, fmaf(h16(fr[a][i >> 1], i), W.rf[a], -W.ohi[a]));
        }
        // Entry clamped at 0 and exit clamped at the pruning limit, so one compare culls
        // a box that is behind the origin (tf < 0), beyond the best hit (tn > lim) or
        // missed (tn > tf).  NaN slab values (a NaN ray) drop out of the fmaxf / fminf
        // chains: such a child is entered.  Empty slots hold a point box at +infinity
        // (ptmi_bvh.cpp): both planes +-inf, so tn > tf or tf < 0; entering one would be
        // harmless (its code is the sentinel leaf of one degenerate triangle).
        k[i] = child_key(tn > tf ? __builtin_huge_valf() : tn, ch[i]);
    }
}

template <typename Stk>
__device__ __forceinline__ bool node_visit(const DevScene& S, Stk* __restrict__ stk, int cur, int& sp,
                                           const WalkRay& W, float lim, int& next) {
    PTMI_COUNT(1);
    double k[4];
    node_children(S, cur, W, lim, k);
    // sort the keys ascending: 5 compare-exchanges of one v_min_f64 + one v_max_f64
#define PTMI_CX(a, b)                        \
    {                                        \
        const double lo_ = fmin(k[a], k[b]); \
        const double hi_ = fmax(k[a], k[b]); \
        k[a] = lo_;                          \
        k[b] = hi_;                          \
    }
    PTMI_CX(0, 1) PTMI_CX(2, 3) PTMI_CX(0, 2) PTMI_CX(1, 3) PTMI_CX(1, 2)
#undef PTMI_CX
    // Unconditional stores above the top, the top advanced by the hit flags (sp <= 21
    // before a node, so the stores stay inside the 24 entries): no exec-mask branches
    // per child (C4 798 -> 778, C5 1250 -> 1216 ms per 2048-spp frame).
    stk[sp * kStkStride] = key_code(k[3]);
    sp += key_entered(k[3]) ? 1 : 0;
    stk[sp * kStkStride] = key_code(k[2]);
    sp += key_entered(k[2]) ? 1 : 0;
    stk[sp * kStkStride] = key_code(k[1]);
    sp += key_entered(k[1]) ? 1 : 0;
    next = key_code(k[0]);
    return key_entered(k[0]);
}

// The triangles of one leaf: tris[first ..] through the one marked kLastTri.
template <bool kVerify>
__device__ __forceinline__ void leaf_visit(const DevScene& S, int first, int slot, int key, d4 o, d4 d, Hit& h,
                                           int& vchain) {
    PTMI_WADD(31, 1ull);
    PTMI_COUNT(2);
    for (int i = first;; i++) {
        PTMI_COUNT(3);
        const DevTri& T = S.tris[i];
        tri_test<kVerify>(S, T, i, o, d, slot, key, h, vchain);
        if (T.chain < 0) break;  // kLastTri
    }
}

// Closest-hit walk of one root's 4-wide traversal index (ptmi_bvh.cpp): nearest
// child first, the others pushed far-to-near.  Which triangles are FOUND does
// not depend on the visiting order or the widened boxes (every triangle that
// can produce a winning t is reached); ties resolve through better_tri.
template <bool kVerify, typename Stk, typename RR>
__device__ __forceinline__ void walk_index(const DevScene& S, Stk* __restrict__ stk, const RR& R, int slot,
                                           int key, d4 o, d4 d, d4 rw, Hit& h, int& vchain) {
    const int lb = leaf_bit_of<Stk>(S);
    const WalkRay W = walk_setup(o, rw, R);  // FP32 slab tests
    float lim = walk_limit(h.t);
    int sp = 0;
    int cur = R.entry;
    PTMI_COUNT(0);
#if PTMI_STATS == 1
    int n_steps = 0, n_leaves = 0;  // (stats: walks that end at the root / without a leaf)
#endif
    while (true) {
#if PTMI_STATS == 1
        n_steps++;
        n_leaves += cur >= lb ? 1 : 0;
#endif
        PTMI_COUNT_ACTIVE(19);  // (stats: wave-level walk loop iterations)
        PTMI_TSTAMP(t_nd);
        if (cur < lb) {
            int next;
            const bool down = node_visit(S, stk, cur, sp, W, lim, next);
            PTMI_TADD(29, t_nd);
            if (down) {
                cur = next;
                continue;
            }
        } else {  // a leaf (an empty slot's sentinel leaf included: only a NaN ray enters one)
            PTMI_TSTAMP(t_lf);
            leaf_visit<kVerify>(S, cur - lb, slot, key, o, d, h, vchain);
            lim = walk_limit(h.t);
            PTMI_TADD(30, t_lf);
        }
        if (sp == 0) break;
        cur = stk[(--sp) * kStkStride];
    }
#if PTMI_STATS == 1
    if (n_leaves == 0) PTMI_COUNT(20);
    if (n_steps == 1) PTMI_COUNT(21);
#endif
}

#if PTMI_STACKLESS
// DIAGNOSTIC (study): the stackless form of walk_index that north_star names -- no traversal
// stack: a walk keeps its node, the key of the child it last left (the next child is the
// nearest entered one beyond it: child keys order children by (entry distance, code), the
// order walk_index pushes them in) and, on the way up, the child it came from, whose key it
// re-derives from the parent's re-tested children.  Each Node4 carries its parent in the
// high half of child[0] (finalize_index_codes, PTMI_STACKLESS builds).  Every node is re-tested
// once per child walked into; leaves are visited in the stack walk's order, so the candidates
// and hence the winner are the same (the pruning limit only shrinks: a child culled on a
// re-test lies beyond the best hit, and so do its later siblings).
template <bool kVerify, typename RR>
__device__ __forceinline__ void walk_index_stackless(const DevScene& S, const RR& R, int slot, int key, d4 o,
                                                     d4 d, d4 rw, Hit& h, int& vchain) {
    const WalkRay W = walk_setup(o, rw, R);
    float lim = walk_limit(h.t);
    int cur = R.entry;
    if (cur >= kLeafNarrow) {  // a root that is a single leaf (or empty)
        leaf_visit<kVerify>(S, cur - kLeafNarrow, slot, key, o, d, h, vchain);
        return;
    }
    const int root = cur;
    double thr = -__builtin_huge_val();  // children with keys above thr are still to walk
    int from = -1;                        // the child node walked out of, or -1
    while (true) {
        double k[4];
        int parent;
        node_children(S, cur, W, lim, k, &parent);
        if (from >= 0) {  // coming up from child `from`: resume after its key
            thr = __builtin_huge_val();  // (from culled now: so is every later sibling)
#pragma unroll
            for (int i = 0; i < 4; i++) thr = key_code(k[i]) == from ? k[i] : thr;
        }
        double nk = __builtin_huge_val();
#pragma unroll
        for (int i = 0; i < 4; i++) nk = (key_entered(k[i]) && k[i] > thr) ? fmin(nk, k[i]) : nk;
        if (nk == __builtin_huge_val()) {  // node exhausted
            if (cur == root) break;
            from = cur;
            cur = parent;
            continue;
        }
        const int c = key_code(nk);
        if (c < kLeafNarrow) {
            cur = c;
            from = -1;
            thr = -__builtin_huge_val();
        } else {
            leaf_visit<kVerify>(S, c - kLeafNarrow, slot, key, o, d, h, vchain);
            lim = walk_limit(h.t);
            from = -1;
            thr = nk;
        }
    }
}
#endif

// Candidate update as selects (no exec-mask branching).  t > EPSILON implies
// the reference's `t != 0.0` recording test.
__device__ __forceinline__ void consider_pk(Hit& h, double t, int pk) {
    const bool c = better(h, t, pk);
    h.t = c ? t : h.t;
    h.pk = c ? pk : h.pk;
    h.tri = c ? -1 : h.tri;
}
__device__ __forceinline__ void consider_sel(Hit& h, double t, int obj, int key) {
    consider_pk(h, t, pack_hit(obj, key));
}

// intersectSphere (tracer.cl:448-476) on an object-space ray: the quadratic ...
template <bool A>
__device__ __forceinline__ void sphere_quad(d4 o, d4 d, double& a, double& b, double& disc) {
    d4 vtc = mk(o.x - 0.0, o.y - 0.0, o.z - 0.0, A ? 0.0 : o.w - 1.0);
    a = dotv<A>(d, d);
    b = 2.0 * dotv<A>(d, vtc);
    double c = dotv<A>(vtc, vtc) - 1.0;
    disc = (b * b) - 4 * a * c;
}
// ... and its roots.
// Affine (A): sqrt / divide cores.  In a tame scene (ptmi_api.cpp) 2a >= 2^-500 for
// every ray, so a root that can be a candidate (EPSILON < t <= 1024) has a quotient
// and operands inside the cores' range; a root outside it is below EPSILON, above
// 1024 or NaN under both arithmetics, so the candidate set and the t1 > EPSILON
// branch are the same.  disc > 0 is a difference of two doubles, so it is either
// >= 2^-767 or so small that b is too (then both roots are below EPSILON).
template <bool A>
__device__ __forceinline__ void sphere_roots(Hit& h, double a, double b, double disc, int pk) {
    if (A && !(PTMI_ABLATE & 128)) {
        // Both roots from one reciprocal of 2a (div_core_r: bit-identical to two div_core
        // calls), then one candidate: t1 if it is one, else t2 -- the reference records
        // both, and t2 >= t1 can only win when t1 <= EPSILON (see below).
        if (disc > 0.0) {
            const double sq = sqrt_core(disc);
            const double y = 2 * a;
            const double r = rcp_core(y);
            const double t1 = div_core_r(-b - sq, y, r);
            const double t2 = div_core_r(-b + sq, y, r);
            consider_pk(h, t1 > kEps ? t1 : t2, pk);
        }
        return;
    }
    if (disc > 0.0) {
        // a > 0 and sq >= 0 give t1 <= t2 after rounding (rounding is monotonic),
        // so t2 can only be recorded as the winner when t1 itself is not a
        // candidate (t1 <= EPSILON); a tie t2 == t1 never replaces t1.
        double sq = (PTMI_ABLATE & 128) ? __builtin_amdgcn_sqrt(disc) : A ? sqrt_core(disc) : sqrt(disc);  // DIAGNOSTIC 128
        double t1 = (PTMI_ABLATE & 128) ? (-b - sq) * __builtin_amdgcn_rcp(2 * a)
                    : A                 ? div_core(-b - sq, 2 * a)
                                        : (-b - sq) / (2 * a);
        consider_pk(h, t1, pk);
        if (!(t1 > kEps)) {
            double t2 = (PTMI_ABLATE & 128) ? (-b + sq) * __builtin_amdgcn_rcp(2 * a)
                        : A                 ? div_core(-b + sq, 2 * a)
                                            : (-b + sq) / (2 * a);
            consider_pk(h, t2, pk);
        }
    }
}
template <bool A>
__device__ __forceinline__ void sphere_test(Hit& h, d4 o, d4 d, int slot, int key) {
    double a, b, disc;
    sphere_quad<A>(o, d, a, b, disc);
    sphere_roots<A>(h, a, b, disc, pack_hit(slot, key));
}

// Row 1 of mul() for a plane's origin and direction (intersectPlane, tracer.cl:478-483),
// affine case, with the +-0 entries of row1[0..2] (bit i of NZ clear) skipped: for a
// finite ray such a term adds an exact +-0, so the remaining terms, summed in the
// reference's order, give oy and dy bit for bit up to the sign of an exact zero, which
// neither t = -oy / dy nor its tests observe (t is then +-0, or |dy| is below EPSILON).
// The walls of the reference scenes have one or two such zeros.
template <int NZ, typename M>
__device__ __forceinline__ void plane_rows_nz(M m, d4 ro, d4 rd, double& oy, double& dy) {
    static_assert(NZ >= 1 && NZ <= 7, "at least one live term");
    double o = 0.0, d = 0.0;
    bool any = false;
    auto term = [&](double mi, double x, double dx) {
        o = any ? o + mi * x : mi * x;
        d = any ? d + mi * dx : mi * dx;
        any = true;
    };
    if constexpr ((NZ & 1) != 0) term(m[0], ro.x, rd.x);
    if constexpr ((NZ & 2) != 0) term(m[1], ro.y, rd.y);
    if constexpr ((NZ & 4) != 0) term(m[2], ro.z, rd.z);
    oy = o + m[3];
    dy = d;
}

// findClosestIntersection (tracer.cl:537-742), one loop per object type.  Loop
// indices are wave-uniform, so object data arrives through scalar loads.
template <int FL>
__device__ __forceinline__ Hit find_closest_prims(const DevScene& S, d4 ro, d4 rd) {
    constexpr bool A = !(FL & F_PROJ);
    Hit h{1024.0, -1, -1, -1, 0.0, 0.0};
    // Plane and sphere records are scalar loads; the next object's record is loaded
    // while the current one is intersected (its latency is otherwise exposed on
    // every object).  Duplicate-free: the last iteration re-loads its own record.
    // Planes come first, in increasing list index, so inside the plane loop a tie in
    // t can never favour the later plane: strict t < h.t is better() there.
    const int np = (PTMI_ABLATE & 8) ? 0 : S.n_planes;
    // intersectPlane (478-483): row 1 only.  Planes are taken two at a time so the
    // two independent division chains overlap (then one odd plane).
    // Row 1 of mul() for the plane's origin and direction (intersectPlane, 478-483).
    auto plane_rows = [&](const auto& P, double& oy, double& dy) {
        const auto* m = P.row1;
        oy = ((m[0] * ro.x + m[1] * ro.y) + m[2] * ro.z) + (A ? m[3] : m[3] * ro.w);
        const double dy0 = (m[0] * rd.x + m[1] * rd.y) + m[2] * rd.z;
        dy = A ? dy0 : dy0 + m[3] * rd.w;
    };
    auto plane_q = [&](double oy, double dy, double& q, bool& ok) {
        // Affine: the divide core.  Its range steps act only when |dy| is denormal or
        // above 2^1022, -oy is below 2^-970, or the quotient is denormal or above 2^767;
        // then q <= EPSILON, |dy| <= EPSILON, or q >= 1024 under both arithmetics, and
        // the plane is not taken either way.
        q = (PTMI_ABLATE & 64) ? -oy * __builtin_amdgcn_rcp(dy) : A ? div_core(-oy, dy) : -oy / dy;  // DIAGNOSTIC 64
        ok = (fabs(dy) > kEps) & (q > kEps);
    };
    // Two parallel planes (identical row1[0..2], affine: P.par): the same dy, so the
    // divide core's reciprocal is shared (div_core_r; bit-identical to two div_cores).
    auto plane_q2 = [&](double oy0, double oy1, double dy, double& q0, bool& k0, double& q1, bool& k1) {
        const double r = rcp_core(dy);
        q0 = div_core_r(-oy0, dy, r);
        q1 = div_core_r(-oy1, dy, r);
        const bool big = fabs(dy) > kEps;
        k0 = big & (q0 > kEps);
        k1 = big & (q1 > kEps);
    };
    auto plane_t = [&](const auto& P, double& q, bool& ok) {
        double oy, dy;
        plane_rows(P, oy, dy);
        plane_q(oy, dy, q, ok);
    };
    auto plane_take = [&](const auto& P, double q, bool ok) {
        const bool c = ok & (q < h.t);
        h.t = c ? q : h.t;
        h.pk = c ? pack_hit(P.slot, P.key) : h.pk;
    };
    int p = 0;
    // Affine scenes: the leading planes whose row 1 is (+-0, m1, +-0, m3) -- floors and
    // ceilings, S.n_planes_y of them in list order -- skip the +-0 terms (plane_rows_nz).
    // (Dispatching every plane, or every run of planes, on its zero pattern measured
    // slower: C2 +4-6 %.)
    if constexpr (A) {
        const int npy = (PTMI_ABLATE & 512) ? 0 : S.n_planes_y;  // DIAGNOSTIC 512: full rows for all
        for (; p + 1 < npy; p += 2) {
            PTMI_WADD(47, 1ull);
            const auto &P0 = cmem(S.planes)[p], &P1 = cmem(S.planes)[p + 1];
            double oy0, dy0, oy1, dy1, q0, q1;
            bool k0, k1;
            if (P0.par) {  // parallel pair: one product m1 y, one direction term, one reciprocal
                const double a = P0.row1[1] * ro.y;
                oy0 = a + P0.row1[3];
                oy1 = a + P1.row1[3];
                dy0 = P0.row1[1] * rd.y;
                plane_q2(oy0, oy1, dy0, q0, k0, q1, k1);
            } else {
                plane_rows_nz<2>(P0.row1, ro, rd, oy0, dy0);
                plane_rows_nz<2>(P1.row1, ro, rd, oy1, dy1);
                plane_q(oy0, dy0, q0, k0);
                plane_q(oy1, dy1, q1, k1);
            }
            plane_take(P0, q0, k0);
            plane_take(P1, q1, k1);
        }
    }
    // Affine planes after the floor / ceiling run: the +-0 entries of row1[0..2] skipped by their
    // pattern (PlaneRec::nz, a uniform switch; round 6): walls rotated about one axis keep one exact
    // zero (the reference scene's side walls (x, y), its back wall (y, z)).  Same terms in the same
    // order, so the sums are bit-identical up to the sign of an exact zero (plane_rows_nz).
    auto sum_nz = [&](auto nzc, const auto* m, double x, double y, double z) {
        constexpr int NZ = decltype(nzc)::value;
        double o = 0.0;
        bool any = false;
        if constexpr ((NZ & 1) != 0) {
            o = m[0] * x;
            any = true;
        }
        if constexpr ((NZ & 2) != 0) {
            o = any ? o + m[1] * y : m[1] * y;
            any = true;
        }
        if constexpr ((NZ & 4) != 0) o = any ? o + m[2] * z : m[2] * z;
        return o;
    };
    auto par_pair = [&](auto nzc, const auto& P0, const auto& P1, double& q0, bool& k0, double& q1, bool& k1) {
        const auto* m = P0.row1;
        const double a = sum_nz(nzc, m, ro.x, ro.y, ro.z);
        const double dy = sum_nz(nzc, m, rd.x, rd.y, rd.z);
        plane_q2(a + m[3], a + P1.row1[3], dy, q0, k0, q1, k1);
    };
    for (; p + 1 < np; p += 2) {
        PTMI_WADD(48, 1ull);
        const auto &P0 = cmem(S.planes)[p], &P1 = cmem(S.planes)[p + 1];
        double oy0, dy0, oy1, dy1, q0, q1;
        bool k0, k1;
        if (A && P0.par && PTMI_R6_PLNZ) {
            switch (P0.nz) {
                case 3: par_pair(std::integral_constant<int, 3>(), P0, P1, q0, k0, q1, k1); break;
                case 5: par_pair(std::integral_constant<int, 5>(), P0, P1, q0, k0, q1, k1); break;
                case 6: par_pair(std::integral_constant<int, 6>(), P0, P1, q0, k0, q1, k1); break;
                default: par_pair(std::integral_constant<int, 7>(), P0, P1, q0, k0, q1, k1); break;
            }
        } else if (A && P0.par) {  // parallel pair: one sum of the origin's x, y, z terms, one direction term
            const auto* m = P0.row1;  // and one reciprocal (row1[0..2] of P1 are the same bits)
            const double a = (m[0] * ro.x + m[1] * ro.y) + m[2] * ro.z;
            oy0 = a + m[3];
            oy1 = a + P1.row1[3];
            dy0 = (m[0] * rd.x + m[1] * rd.y) + m[2] * rd.z;
            plane_q2(oy0, oy1, dy0, q0, k0, q1, k1);
        } else {
            plane_rows(P0, oy0, dy0);
            plane_rows(P1, oy1, dy1);
            plane_q(oy0, dy0, q0, k0);
            plane_q(oy1, dy1, q1, k1);
        }
        plane_take(P0, q0, k0);
        plane_take(P1, q1, k1);
    }
    if (p < np) {
        PTMI_WADD(49, 1ull);
        const auto& P0 = cmem(S.planes)[p];
        double q0;
        bool k0;
        if (A && PTMI_R6_PLNZ) {
            double oy, dy;
            switch (P0.nz) {
                case 3: plane_rows_nz<3>(P0.row1, ro, rd, oy, dy); break;
                case 5: plane_rows_nz<5>(P0.row1, ro, rd, oy, dy); break;
                case 6: plane_rows_nz<6>(P0.row1, ro, rd, oy, dy); break;
                default: plane_rows(P0, oy, dy); break;
            }
            plane_q(oy, dy, q0, k0);
        } else {
            plane_t(P0, q0, k0);
        }
        plane_take(P0, q0, k0);
    }
    const int nq = (PTMI_ABLATE & 16) ? 0 : S.n_spheres_st;
    auto sphere_ray = [&](const auto& Q, d4& o, d4& d) {
        if constexpr (A) {
            o = mk(Q.m0 * ro.x + Q.m3, Q.m5 * ro.y + Q.m7, Q.m10 * ro.z + Q.m11, 1.0);
            d = mk(Q.m0 * rd.x, Q.m5 * rd.y, Q.m10 * rd.z, 0.0);
        } else {
            o = mk(Q.m0 * ro.x + Q.m3 * ro.w, Q.m5 * ro.y + Q.m7 * ro.w, Q.m10 * ro.z + Q.m11 * ro.w, Q.m15 * ro.w);
            d = mk(Q.m0 * rd.x + Q.m3 * rd.w, Q.m5 * rd.y + Q.m7 * rd.w, Q.m10 * rd.z + Q.m11 * rd.w, Q.m15 * rd.w);
        }
    };
    // A ray's line meets few spheres (disc > 0 in ~5 % of the tests), yet a wave of 64
    // rays almost always has one lane that does: evaluated in place, the root code would
    // run for every sphere.  Each lane instead keeps its first sphere with disc > 0 and
    // evaluates the roots once after the loop (a second such sphere -- rare -- in place).
    // The candidates are the same and the winner is their lexicographic minimum
    // (better()), so the order of evaluation does not matter.
    bool pend = false;
    double pa = 0.0, pb = 0.0, pd = 0.0;
    int ppk = 0;
    auto defer = [&](double a, double b, double disc, int slot, int key) {
        const bool has = disc > 0.0;
        const int pk = pack_hit(slot, key);  // (uniform: scalar)
        if (has && pend) {
            PTMI_WADD(34, 1ull);
            sphere_roots<A>(h, a, b, disc, pk);
        }
        const bool take = has && !pend;
        pa = take ? a : pa;
        pb = take ? b : pb;
        pd = take ? disc : pd;
        ppk = take ? pk : ppk;
        pend = pend || has;
    };
    // The first sphere's quadratic is kept as it is (round 6): nothing is pending before it, so
    // its selects would only choose between it and the initial zeros, which are never read
    // unless pend is set.
    auto first = [&](double a, double b, double disc, int slot, int key) {
        pa = a;
        pb = b;
        pd = disc;
        ppk = pack_hit(slot, key);
        pend = disc > 0.0;
    };
    int q = 0;
    if (PTMI_R6_SPH && nq == 1) {
        const auto& Q0 = cmem(S.spheres)[0];
        d4 o0, d0;
        sphere_ray(Q0, o0, d0);
        double a0, b0, disc0;
        sphere_quad<A>(o0, d0, a0, b0, disc0);
        first(a0, b0, disc0, Q0.slot, Q0.key);
        q = 1;
    }
    if (PTMI_R6_SPH && nq >= 2) {
        PTMI_WADD(50, 1ull);
        const auto &Q0 = cmem(S.spheres)[0], &Q1 = cmem(S.spheres)[1];
        d4 o0, d0, o1, d1;
        sphere_ray(Q0, o0, d0);
        sphere_ray(Q1, o1, d1);
        double a0, b0, disc0, a1, b1, disc1;
        sphere_quad<A>(o0, d0, a0, b0, disc0);
        sphere_quad<A>(o1, d1, a1, b1, disc1);
        first(a0, b0, disc0, Q0.slot, Q0.key);
        defer(a1, b1, disc1, Q1.slot, Q1.key);
        q = 2;
    }
    for (; q + 1 < nq; q += 2) {  // two spheres at a time: overlapping quadratic setups
        PTMI_WADD(51, 1ull);
        const auto &Q0 = cmem(S.spheres)[q], &Q1 = cmem(S.spheres)[q + 1];
        d4 o0, d0, o1, d1;
        sphere_ray(Q0, o0, d0);
        sphere_ray(Q1, o1, d1);
        double a0, b0, disc0, a1, b1, disc1;
        sphere_quad<A>(o0, d0, a0, b0, disc0);
        sphere_quad<A>(o1, d1, a1, b1, disc1);
        defer(a0, b0, disc0, Q0.slot, Q0.key);
        defer(a1, b1, disc1, Q1.slot, Q1.key);
    }
    if (q < nq) {
        PTMI_WADD(52, 1ull);
        const auto& Q0 = cmem(S.spheres)[q];
        d4 o0, d0;
        sphere_ray(Q0, o0, d0);
        double a0, b0, disc0;
        sphere_quad<A>(o0, d0, a0, b0, disc0);
        defer(a0, b0, disc0, Q0.slot, Q0.key);  // (q >= 2 here when PTMI_R6_SPH: the first sphere is peeled)
    }
    if (pend) {
        PTMI_WADD(33, 1ull);
        sphere_roots<A>(h, pa, pb, pd, ppk);
    }
    int j = S.run_end[0];
    // spheres with other matrices (none when every sphere is in S.spheres: the loop's scalar
    // record loads and waits are skipped)
    if (PTMI_R6_SPH && S.run_end[1] - j == S.n_spheres_st) j = S.run_end[1];
    for (; j < S.run_end[1]; j++) {
        PTMI_WADD(53, 1ull);
        const auto& ob = cmem(S.objs)[j];
        if (ob.st) continue;  // in S.spheres
        sphere_test<A>(h, xpt<A>(ob.inv, false, ro), xdir<A>(ob.inv, false, rd), j, ob.key);
    }
    if (FL & F_CYLCUBE) {
        for (; j < S.run_end[2]; j++) {  // cylinders: intersectCylinder (396-446), caps disabled
            const auto& ob = cmem(S.objs)[j];
            d4 o = xpt<A>(ob.inv, ob.st, ro);
            d4 d = xdir<A>(ob.inv, ob.st, rd);
            double a = d.x * d.x + d.z * d.z;
            if (!(fabs(a) < kEps)) {
                double b = 2 * o.x * d.x + 2 * o.z * d.z;
                double c1 = o.x * o.x + o.z * o.z - 1;
                double disc = b * b - 4 * a * c1;
                if (!(disc < 0.0)) {
                    double sq = sqrt(disc);
                    double t0 = (-b - sq) / (2 * a);
                    double t1 = (-b + sq) / (2 * a);
                    double y0 = o.y + t0 * d.y;
                    double y1 = o.y + t1 * d.y;
                    double r0 = (y0 > ob.min_y && y0 < ob.max_y) ? t0 : 0.0;
                    double r1 = (y1 > ob.min_y && y1 < ob.max_y) ? t1 : 0.0;
                    consider_sel(h, r0, j, ob.key);
                    consider_sel(h, r1, j, ob.key);
                }
            }
        }
        for (; j < S.run_end[3]; j++) {  // cubes: intersectCube (378-394)
            const auto& ob = cmem(S.objs)[j];
            d4 o = xpt<A>(ob.inv, ob.st, ro);
            d4 d = xdir<A>(ob.inv, ob.st, rd);
            double x0, x1, y0, y1, z0, z1;
            check_axis(o.x, d.x, -1.0, 1.0, x0, x1);
            check_axis(o.y, d.y, -1.0, 1.0, y0, y1);
            check_axis(o.z, d.z, -1.0, 1.0, z0, z1);
            double tmin = max3(x0, y0, z0), tmax = min3(x1, y1, z1);
            if (!(tmin > tmax)) {
                consider_sel(h, tmin, j, ob.key);
                consider_sel(h, tmax, j, ob.key);
            }
        }
    }
    return h;
}

// Groups (tracer.cl:598-720), split in two so a wave can defer the walks
// (see trace_groups): group_needs_walk is the cheap part -- the conservative cull
// of each object's traversal hull against the current best -- and group_walks
// walks every index that survives, updating h.  The reference's exact box gates
// (the object's, tracer.cl:609, and its nodes', 617-719) are checked per winning
// triangle on its gate chain (chain_certified / verify_chain).
template <bool A>
__device__ __forceinline__ bool group_needs_walk(const DevScene& S, d4 ro, d4 rd, const Hit& h) {
    for (int j = S.run_end[3]; j < S.run_end[4]; j++) {
        const auto& ob = cmem(S.objs)[j];
        const d4 o = xpt<A>(ob.inv, ob.st, ro);
        const d4 d = xdir<A>(ob.inv, ob.st, rd);
        const d4 r = mk(rcp_walk(d.x), rcp_walk(d.y), rcp_walk(d.z), 0.0);
        for (int ci = 0; ci < ob.child_count; ci++) {
            const auto& R = cmem(S.root_rec)[ob.child_base + ci];
            double tn;
            if (!cull_box(o, r, R.hull_mn[0], R.hull_mn[1], R.hull_mn[2], R.hull_mx[0], R.hull_mx[1],
                          R.hull_mx[2], h.t + prune_margin(h.t), tn))
                return true;
        }
    }
    return false;
}

// The walks of every group object for one ray.  kVerify: eager gate checks on
// each improving candidate (exact by construction, slower: the check runs
// inside the divergent walk loop).
template <bool A, bool kVerify, typename Stk>
__device__ __forceinline__ void group_walks_impl(const DevScene& S, Stk* __restrict__ stk, d4 ro, d4 rd, Hit& h,
                                                 bool& cert) {
    for (int j = S.run_end[3]; j < S.run_end[4]; j++) {
        const auto& ob = cmem(S.objs)[j];
        const d4 o = xpt<A>(ob.inv, ob.st, ro);
        const d4 d = xdir<A>(ob.inv, ob.st, rd);
        const d4 r = mk(rcp_walk(d.x), rcp_walk(d.y), rcp_walk(d.z), 0.0);
        PTMI_COUNT(7);
        // The object's own gate (tracer.cl:609) is the first box of every triangle's
        // gate chain, so it is checked with the rest of the chain (chain_certified /
        // verify_chain), not here.
        int vchain = -1;
        for (int ci = 0; ci < ob.child_count; ci++) {
            const auto& R = cmem(S.root_rec)[ob.child_base + ci];
            double tn;
            if (cull_box(o, r, R.hull_mn[0], R.hull_mn[1], R.hull_mn[2], R.hull_mx[0], R.hull_mx[1],
                         R.hull_mx[2], h.t + prune_margin(h.t), tn))
                continue;
            PTMI_TSTAMP(t_w);
#if PTMI_STACKLESS
            if constexpr (A && sizeof(Stk) == 2) walk_index_stackless<kVerify>(S, R, j, ob.key, o, d, r, h, vchain);
            else
#endif
            walk_index<kVerify>(S, stk, R, j, ob.key, o, d, r, h, vchain);
            PTMI_TADD_ACTIVE(18, t_w);  // (stats: cycles in walk loops)
        }
        // Tentative walks: certify the gate chain of a winner from this object while
        // its object-space ray is at hand (a later object that takes over re-certifies).
        if (!kVerify && h.tri >= 0 && hit_obj(h) == j) cert = chain_certified(S, S.tris[h.ti].chain, o, d, h.t);
    }
}


// Deferred gate verification.  The walks first take every Moller-Trumbore hit
// tentatively; their winner is the minimum over a SUPERSET of the reference's
// candidates, so if it passes its own gate chain it is the reference's winner.
// Only then (a lane whose winner fails -- seen only with degenerate boxes, see
// tests/adversarial.py) are this ray's walks redone with eager checks.  All
// lanes verify together after the loop instead of one by one inside it.
template <bool A, typename Stk>
__device__ __forceinline__ void group_walks(const DevScene& S, Stk* __restrict__ stk, d4 ro, d4 rd, Hit& h) {
    const Hit h0 = h;
    bool cert = false;
    group_walks_impl<A, false>(S, stk, ro, rd, h, cert);
    if (h.tri >= 0) PTMI_COUNT(4);
    if (h.tri >= 0 && !cert) {  // the winner is a triangle (h0 holds primitives only) without certificate
        const DevObject& ob = S.objs[hit_obj(h)];
        const d4 o = xpt<A>(ob.inv, ob.st, ro);
        const d4 d = xdir<A>(ob.inv, ob.st, rd);
        if (!verify_chain(S, S.tris[h.ti].chain, o, d)) {
            PTMI_COUNT(11);  // (stats build: eager re-walks)
            h = h0;
            group_walks_impl<A, true>(S, stk, ro, rd, h, cert);
        }
    }
    if (h.tri >= 0) {  // the winner's barycentrics (for its interpolated normal)
        const DevObject& ob = S.objs[hit_obj(h)];
        tri_uv(S.tris[h.ti], xpt<A>(ob.inv, ob.st, ro), xdir<A>(ob.inv, ob.st, rd), h.u, h.v);
    }
}

// schlick (tracer.cl:485-505)
template <bool A>
__device__ __noinline__ double schlick(d4 eye, d4 nrm, double n1, double n2) {
    double c = dotv<A>(eye, nrm);
    if (n1 > n2) {
        double n = n1 / n2;
        double s2 = (n * n) * (1.0 - (c * c));
        if (s2 > 1.0) return 1.0;
        c = sqrt(1.0 - s2);
    }
    double tmp = (n1 - n2) / (n1 + n2);
    double r0 = tmp * tmp;
    return r0 + (1 - r0) * pow(1 - c, 5.0);
}

// computeRefractedRay (tracer.cl:507-533)
template <bool A>
__device__ __noinline__ d4 refracted(d4 eye, d4 nrm, double n1, double n2) {
    double nr = n1 / n2;
    double ci = dotv<A>(eye, nrm);
    double s2 = (nr * nr) * (1.0 - (ci * ci));
    if (s2 > 1.0) return mk(0, 0, 0, 0);
    double ct = sqrt(1.0 - s2);
    return sub4(scl4(nrm, (nr * ci) - ct), scl4(eye, nr));
}

template <bool A>
__device__ __forceinline__ d4 reflect(d4 rd, d4 nv) { return sub4(rd, scl4(scl4(nv, 2.0), dotv<A>(rd, nv))); }

// randomVectorInHemisphere (tracer.cl:348-366) from its two uniforms
// u1 = noise3D(x, y, z), u2 = noise3D(y, z, x) (or the statistical mode's draws).
// Its transcendental half depends on the uniforms alone: (sin, cos)(2 pi u1) and
// (sqrt(u2), sqrt(1 - u2)), computed here ...
template <bool A>
__device__ __forceinline__ void hemi_sincos(float u1, double& sr, double& cr) {
    const double rand1 = 2.0 * kPi * (double)u1;
    if (PTMI_ABLATE & 4) {
        cr = 1.0 - rand1 * 0.1;
        sr = rand1 * 0.15;
    } else if constexpr (A) {
        sincos_core<true>(rand1, &sr, &cr);  // rand1 in [0, 2 pi): ocml's sincos without its range steps
    } else {
        sincos(rand1, &sr, &cr);  // ocml sincos == (sin, cos) bit-for-bit: one shared reduction
    }
}
template <bool A>
__device__ __forceinline__ void hemi_sqrt(float u2, double& r2s, double& rc) {
    const double rand2 = (double)u2;
    // Affine: sqrt's core; rand2 is 0 or a float >= 2^-149, so in its range (and 1 - rand2
    // is in (0, 1]), sqrt(+0) = +0 kept by the select.
    r2s = A ? (rand2 == 0.0 ? 0.0 : sqrt_core(rand2)) : sqrt(rand2);
    rc = A ? sqrt_core(1.0 - rand2) : sqrt(1.0 - rand2);
}

// ... or read from a table (DevScene::hemi, hemi_table_kernel) for uniforms on the grid
// k 2^-16.  noise3D's u = fract(v), v = sin(s) * 43758.5453f, is exact in float and a
// multiple of ulp(v): of 2^-16 or coarser whenever |v| >= 128, i.e. for all but ~0.2 %
// of the draws (|sin| < 0.0029).  Record k holds the four values computed by the code
// above from u = k 2^-16, so a lane reads the bits it would compute (the table kernel
// also counts records where the generic sequences differ -- they never read the table --
// and ptmi_diag_hemi_mismatch reports the count, 0 on this toolchain).  Off-grid draws
// compute; the statistical mode draws its hemisphere uniforms on the grid (xnext16).
#ifndef PTMI_HEMI_TAB_GROUPS
#define PTMI_HEMI_TAB_GROUPS 1  // mesh scenes read the table too (round 5: with the group kernel's colour
                                // state in LDS, 2048 spp: C4 594 -> 577, C5 902 -> 897 ms; in round 4 the
                                // 2 MB table's L2 share had cost C5 ~1.5 % at 512 spp); since round 6 a scene
                                // switch as well (DevScene::hemi_mesh, ptmi_api.cpp; on by default)
#endif
static constexpr int kHemiBits = 16;
static constexpr int kHemiSize = 1 << kHemiBits;
__device__ __forceinline__ int hemi_slot(float u) {  // table record of u, or -1 off the grid
    const float t = u * (float)kHemiSize;  // exact (power of two)
    const int k = (int)t;
    // Every uniform is in [0, 1) (noise3d's fract is at most 0x1.fffffep-1, xnext16 < 1), so k is
    // below kHemiSize whenever t is an integer; a NaN fails the equality.
    if (PTMI_R6_SLOT) return t == (float)k ? k : -1;
    return (t == (float)k && (unsigned)k < (unsigned)kHemiSize) ? k : -1;
}

// The table is two planes (round 6): [0, 2^16) the (sin, cos) pairs, [2^16, 2^17) the (sqrt u,
// sqrt(1 - u)) pairs, 16 B per entry.  A lookup reads one 16-B entry of each plane, as before from two
// unrelated records (u1 and u2 are independent draws); the planes let the mesh kernels keep just the
// 1-MB (sin, cos) plane in the L2 they share with the traversal index and compute the sqrt pair
// (kTabSqrt false): with the whole 2-MB table their HBM traffic was the table's evictions.
#ifndef PTMI_HEMI_SQRT_GROUPS
#define PTMI_HEMI_SQRT_GROUPS 0  // mesh kernels read the sqrt plane too (1) or compute the pair (0)
#endif
// `use` (uniform): the scene lets this kernel read the table (DevScene::hemi_mesh for the mesh kernels).
template <bool A, bool kTab, bool kTabSqrt = kTab>
__device__ __forceinline__ d4 random_hemisphere(const double* __restrict__ tab, d4 nv, float u1, float u2,
                                                bool use = true) {
    double sr, cr, rand2s, rc;
    const int k1 = (kTab && use) ? hemi_slot(u1) : -1;
    if (k1 >= 0) {
        const double2 q = *reinterpret_cast<const double2*>(tab + 2 * k1);
        sr = q.x;
        cr = q.y;
    } else {
        PTMI_WADD(35, 1ull);
        hemi_sincos<A>(u1, sr, cr);
    }
    const int k2 = (kTabSqrt && use) ? hemi_slot(u2) : -1;
    if (k2 >= 0) {
        const double2 q = *reinterpret_cast<const double2*>(tab + 2 * kHemiSize + 2 * k2);
        rand2s = q.x;
        rc = q.y;
    } else {
        PTMI_WADD(36, 1ull);
        hemi_sqrt<A>(u2, rand2s, rc);
    }
    // cross(axis, n) for a unit axis: the fma chains of opencl.bc's cross reduce
    // exactly (up to the sign of exact zeros) to component moves:
    //   cross((0,1,0,0), n) = (n.z, 0, -n.x, 0),  cross((1,0,0,0), n) = (0, -n.z, n.y, 0)
    d4 c = fabs(nv.x) > 0.1 ? mk(nv.z, 0.0, -nv.x, 0.0) : mk(0.0, -nv.z, nv.y, 0.0);
    // |c|^2 >= 0.01 for a unit normal (|n.x| > 0.1 or n.y^2 + n.z^2 >= 0.99): normalize's core
    d4 u = A ? norm3_core(c) : normv<A>(c);
    d4 v = cross4(nv, u);
    return add4(add4(scl4(scl4(u, cr), rand2s), scl4(scl4(v, sr), rand2s)), scl4(nv, rc));
}

// The table: record k = (sin, cos)(2 pi u), sqrt(u), sqrt(1 - u) for u = k 2^-16, from
// the affine sequences; `mismatch` counts records where the generic (full-operator)
// sequences give other bits (ptmi_diag_hemi_mismatch; tests/test_gpu_rng.py expects 0).
__global__ __launch_bounds__(256) void hemi_table_kernel(double* __restrict__ out, int* __restrict__ mismatch) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= kHemiSize) return;
    const float u = (float)k * (1.0f / (float)kHemiSize);
    double a[4], g[4];
    hemi_sincos<true>(u, a[0], a[1]);
    hemi_sqrt<true>(u, a[2], a[3]);
    hemi_sincos<false>(u, g[0], g[1]);
    hemi_sqrt<false>(u, g[2], g[3]);
    bool same = true;
    for (int i = 0; i < 4; i++) {
        out[(i < 2 ? 2 * k : 2 * kHemiSize + 2 * k) + (i & 1)] = a[i];  // the two planes
        same = same && __double_as_longlong(a[i]) == __double_as_longlong(g[i]);
    }
    if (!same) atomicAdd(mismatch, 1);
}

// sunflower (tracer.cl:221-248), randomize == false.
__device__ __noinline__ void sunflower(int amount, int point, double& ox, double& oy) {
    double idx = (double)point;
    double sqp = sqrt((double)amount);
    double b = round(2.0 * sqp);
    const double phi = (sqrt(5.0) + 1.0) / 2.0;
    double n = (double)amount;
    double r = 1.0;
    if (idx <= (n - b)) r = sqrt(idx - 0.5) / sqrt(n - (b + 1.0) / 2.0);
    double theta = 2.0 * kPi * idx / (phi * phi);
    double st, ct;
    sincos(theta, &st, &ct);
    ox = r * ct;
    oy = r * st;
}

// The camera record through a pointer the compiler does not hoist: its fields are
// scalar-loaded where a camera block runs, instead of being held in SGPRs through the
// whole bounce loop -- which spilled them into VGPR lanes (v_writelane / v_readlane, VALU
// instructions) when the loop's other uniform values needed the SGPRs.  C2 / C3 154.85 /
// 160.89 -> 154.46 / 157.35 ms, C4 (512 spp) 165.84 -> 165.15 ms (profiles/r4/cam_reload).
// A *volatile* asm here made every later global load of the loop a vector load (the
// uniform-load analysis treats it as a possible store): C2 264 ms.
#ifndef PTMI_CAM_RELOAD
#define PTMI_CAM_RELOAD 3  // 1: kernels without meshes, 2: mesh kernels, 3: both
#endif
template <bool kReload = true>
__device__ __forceinline__ const DevCamera& camera_ptr(const DevScene& S) {
    if constexpr (!kReload) return S.cam;
    // The constant address space: scalar loads of an invariant record (through a generic
    // pointer the loads were per-lane vector loads: C2 155 -> 264 ms).
    // readfirstlane: a value divergence analysis knows to be uniform, so the loads are
    // scalar (an inline-asm "s" result alone is not).
    typedef const __attribute__((address_space(4))) DevCamera ConstCam;
    const DevCamera* p = S.camg;
    asm("" : "+s"(p));
    const uint64_t a = (uint64_t)p;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
    return *(const DevCamera*)(ConstCam*)u;
}

// rayForPixel (tracer.cl:745-779).  With DoF the aperture offset
// sunflower(S, 2, n) depends only on n: it is read from a per-frame table
// (sunflower_kernel) made with the same arithmetic.
//   origin = mul(inverse, (0,0,0,1)): a frame constant, DevCamera::origin
//   pixel  = mul(inverse, (hw - xo, hh - yo, -1, 1)) where m*(-1) == -m and
//            m*1 == m exactly, so row r = ((m0 a + m1 b) + (-m2)) + m3.
// Everything uniform comes straight from the kernel arguments (scalar
// registers); nothing per-frame is kept live in vector registers across the
// bounce loop.
template <bool kDof, bool A>
__device__ __forceinline__ void ray_for_pixel(const DevCamera& cam, const double* __restrict__ sunf, unsigned x,
                                              unsigned y, float rx, float ry, int sample, d4& ro, d4& rd) {
    double xo = cam.pixel_size * ((double)x + (double)rx);
    double yo = cam.pixel_size * ((double)y + (double)ry);
    const double a = cam.half_width - xo, b = cam.half_height - yo;
    const double* m = cam.inv;
    d4 pixel = mk(((m[0] * a + m[1] * b) + (-m[2])) + m[3], ((m[4] * a + m[5] * b) + (-m[6])) + m[7],
                  ((m[8] * a + m[9] * b) + (-m[10])) + m[11],
                  A ? 1.0 : ((m[12] * a + m[13] * b) + (-m[14])) + m[15]);
    d4 origin = ld4(cam.origin);
    if (A) origin.w = 1.0;
    // Affine scenes have a tame camera (ptmi_api.cpp): |pixel - origin| >= 2^-196, so
    // normalize's core.
    d4 dir = (PTMI_ABLATE & 2) ? sub4(pixel, origin) : A ? norm3_core(sub4(pixel, origin)) : normv<A>(sub4(pixel, origin));
    if (kDof && cam.aperture != 0) {
        d4 pos = add4(origin, scl4(dir, cam.focal_length));
        const double sx = sunf[2 * sample], sy = sunf[2 * sample + 1];
        d4 no = mk(origin.x + (sy * cam.aperture), origin.y + (sx * cam.aperture), origin.z, 1.0);
        dir = sub4(pos, no);
        origin = no;
    }
    ro = origin;
    rd = dir;
}

// Per-lane path state.  A lane walks its chunk of samples as a sequence of
// bounce steps; when a path ends it immediately starts its next sample (path
// regeneration), so lanes of a wave never idle waiting for the wave's longest
// path.  Within a lane the arithmetic and its order are exactly the reference's
// sample loop (tracer.cl:867-1179) with the shading reduction (1116-1176)
// applied as each bounce is produced.
struct PathState {
    d4 ro, rd;
    double mr, mg, mb;  // mask
    double ar, ag, ab;  // accumColor
    unsigned b, effective;  // bounce index (also the reduction's record index x, tracer.cl:1148-1160), effectiveBounces
    bool inside, done;
    // A camera ray with a NaN component (DoF sample 0: sunflowerRadius(0) =
    // sqrt(-0.5), tracer.cl:224) makes every object-space component NaN in the
    // reference (0*NaN = NaN), so it misses everything and the sample adds 0.
    bool dead;
    Xrng rng;  // statistical mode (F_XRNG) only
};

// `dead` is a shortcut only (a NaN path misses and adds 0 either way), taken where
// NaN camera rays occur: DoF scenes.
template <bool A, bool kDof>
__device__ __forceinline__ void start_path(PathState& P, d4 ro, d4 rd) {
    P.ro = ro;
    P.rd = rd;
    P.mr = P.mg = P.mb = 1.0;
    P.ar = P.ag = P.ab = 0.0;
    P.b = P.effective = 0;
    P.inside = P.done = false;
    P.dead = kDof && !(isfinite(ro.x) && isfinite(ro.y) && isfinite(ro.z) && (A || isfinite(ro.w)) &&
                       isfinite(rd.x) && isfinite(rd.y) && isfinite(rd.z) && (A || isfinite(rd.w)));
}

// ---- Textures (tracer.cl:113-213, 829, 907-914, 1077-1092) ----------------------
// gfx950 has no image instructions (read_imagef does not lower for it; DESIGN.md
// "Textures"), so the kernel's sampler -- CLK_NORMALIZED_COORDS_TRUE |
// CLK_ADDRESS_REPEAT | CLK_FILTER_LINEAR on RGBA UNORM8 arrays -- is done here in
// software with the OpenCL 1.2 s8.2 formulas in FP32, separately rounded in a fixed
// order (the CPU oracle restates the same sequence; parity unpinned).
struct Rgb {
    float r, g, b;
};

// Repeat addressing + linear filter along one axis: texel pair and weight.
__device__ __forceinline__ void tex_axis(float s, int n, int& i0, int& i1, float& a) {
    if (!isfinite(s)) s = 0.0f;  // undefined in OpenCL; pinned to 0 here and in the oracle
    const float u = (s - floorf(s)) * (float)n;
    const float um = u - 0.5f;
    const float fl = floorf(um);
    i0 = (int)fl;
    i1 = i0 + 1;
    if (i0 < 0) i0 = n + i0;
    if (i1 > n - 1) i1 = i1 - n;
    a = um - fl;
}

__device__ __forceinline__ Rgb texel(const DevTexArray& T, int layer, int i, int j) {
    const uint32_t p = T.texels[((size_t)layer * (size_t)T.h + (size_t)j) * (size_t)T.w + (size_t)i];
    return Rgb{(float)(p & 0xffu) / 255.0f, (float)((p >> 8) & 0xffu) / 255.0f, (float)((p >> 16) & 0xffu) / 255.0f};
}

// read_imagef(array, sampler, (float4)(s, t, layer, 0)).xyz
__device__ __noinline__ Rgb tex_sample(const DevTexArray T, float s, float t, float layer) {
    if (T.layers <= 0) return Rgb{0.0f, 0.0f, 0.0f};  // the reference's all-zero fake image
    const int l = (int)fminf(fmaxf(rintf(layer), 0.0f), (float)(T.layers - 1));
    int i0, i1, j0, j1;
    float a, b;
    tex_axis(s, T.w, i0, i1, a);
    tex_axis(t, T.h, j0, j1, b);
    const Rgb t00 = texel(T, l, i0, j0), t10 = texel(T, l, i1, j0);
    const Rgb t01 = texel(T, l, i0, j1), t11 = texel(T, l, i1, j1);
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    return Rgb{((w00 * t00.r + w10 * t10.r) + w01 * t01.r) + w11 * t11.r,
               ((w00 * t00.g + w10 * t10.g) + w01 * t01.g) + w11 * t11.g,
               ((w00 * t00.b + w10 * t10.b) + w01 * t01.b) + w11 * t11.b};
}

// OpenCL length(double4) (opencl.bc): sqrt(dot) with range scaling.
__device__ __forceinline__ double length4(d4 v) {
    const double d = dot4(v, v);
    if (d < 0x1p-1022) return sqrt(dot4(scl4(v, 0x1p563), scl4(v, 0x1p563))) * 0x1p-563;
    if (d == __builtin_inf()) return sqrt(dot4(scl4(v, 0x1p-514), scl4(v, 0x1p-514))) * 0x1p514;
    return sqrt(d);
}

// sphericalMap (tracer.cl:178-213) -> (u, v)
__device__ __noinline__ void spherical_map(d4 p, double& u, double& v) {
    const double theta = atan2(p.x, p.z);
    const double radius = length4(mk(p.x, p.y, p.z, 0.0));
    const double phi = acos(p.y / radius);
    const double raw_u = theta / (2.0 * kPi);
    u = 1 - (raw_u + 0.5);
    v = 1 - phi / kPi;
}

// cubeUV (tracer.cl:113-175): the face of a 4x3 cross layout -> (u, v)
__device__ __noinline__ void cube_uv(d4 p, double& u, double& v) {
    const double coord = max3(fabs(p.x), fabs(p.y), fabs(p.z));
    double fu, fv;
    if (coord == p.x) {  // right
        fu = fmod(1.0 - p.z, 2.0) / 2.0, fv = fmod(p.y + 1.0, 2.0) / 2.0;
        u = 0.5 + fu * 0.25, v = 0.6666666 - fv * 0.333333;
    } else if (coord == -p.x) {  // left
        fu = fmod(p.z + 1.0, 2.0) / 2.0, fv = fmod(p.y + 1.0, 2.0) / 2.0;
        u = fu * 0.25, v = 0.6666666 - fv * 0.333333;
    } else if (coord == p.y) {  // up
        fu = fmod(p.x + 1.0, 2.0) / 2.0, fv = fmod(1.0 - p.z, 2.0) / 2.0;
        u = 0.25 + fu * 0.25, v = 1.0 - fv * 0.333333;
    } else if (coord == -p.y) {  // down
        fu = fmod(p.x + 1.0, 2.0) / 2.0, fv = fmod(p.z + 1.0, 2.0) / 2.0;
        u = 0.25 + fu * 0.25, v = fv * 0.333333;
    } else if (coord == p.z) {  // front
        fu = fmod(p.x + 1.0, 2.0) / 2.0, fv = fmod(p.y + 1.0, 2.0) / 2.0;
        u = 0.25 + fu * 0.25, v = 0.6666666 - fv * 0.333333;
    } else {  // back
        fu = fmod(1.0 - p.x, 2.0) / 2.0, fv = fmod(p.y + 1.0, 2.0) / 2.0;
        u = 0.75 + fu * 0.25, v = 0.6666666 - fv * 0.333333;
    }
}

// Texture colour of a textured plane / sphere / cube hit (tracer.cl:1077-1092)
// from T = the array of its type; false for other types (the object colour stays).
template <bool A>
__device__ __noinline__ bool textured_color(const DevTexArray T, const DevObject& ob, d4 pos, double& r, double& g,
                                            double& b) {
    const d4 lp = xpt<A>(ob.inv, ob.st, pos);
    Rgb c;
    if (ob.type == 0) {
        c = tex_sample(T, (float)(lp.x * ob.tex_scale[0]), (float)(lp.z * ob.tex_scale[1]),
                       (float)ob.tex_index);
    } else if (ob.type == 1) {
        double u, v;
        spherical_map(lp, u, v);
        c = tex_sample(T, (float)u, (float)(1.0 - v), (float)ob.tex_index);
    } else if (ob.type == 3) {
        double u, v;
        cube_uv(lp, u, v);
        c = tex_sample(T, (float)u, (float)v, (float)ob.tex_index);
    } else {
        return false;
    }
    r = (double)c.r, g = (double)c.g, b = (double)c.b;
    return true;
}

// Normal-mapped plane: objectNormal = normalize(rgb of the normal map, 0)
// (tracer.cl:907-911).
template <bool A>
__device__ __noinline__ d4 plane_normal_map(const DevTexArray T, const DevObject& ob, d4 pos) {
    const d4 lp = xpt<A>(ob.inv, ob.st, pos);
    const Rgb c = tex_sample(T, (float)(fabs(lp.x) * ob.tex_scale[2]), (float)(fabs(lp.z) * ob.tex_scale[3]),
                             (float)ob.tex_index_nm);
    return normalize4(mk((double)c.r, (double)c.g, (double)c.b, 0.0));
}

// One bounce (tracer.cl:884-1110).  Returns true when the path has ended.
// One bounce of the path given its closest hit h (tracer.cl:886-1110 after
// findClosestIntersection).  Returns true when the path has ended.
// kAccLds: accumColor lives in LDS at acm[0, kBlock, 2 kBlock] instead of P.ar/ag/ab
// (the kernels without meshes; it changes only on bounces that see emission).
// kMaskLds: the path's mask (throughput) lives in LDS at msk[0, kBlock, 2 kBlock] instead of
// P.mr/mg/mb (the mesh kernels, where the 4-wave register budget otherwise spills it with a
// scratch load and store per bounce).
template <int FL, bool kAccLds = false, bool kMaskLds = false>
__device__ __forceinline__ bool bounce_shade(const DevScene& S, PathState& P, const Hit& h, float fgi, uint32_t n,
                                             double* acm = nullptr, double* msk = nullptr) {
    constexpr bool A = !(FL & F_PROJ);
    constexpr bool kX = (FL & F_XRNG) != 0;
    if (h.pk < 0) return true;  // a miss repeats identically until b == 10 in the reference
    PTMI_WADD(44, 1ull);
    const DevObject& ob = S.objs[h.pk & 0xFFFF];
    const int type = ob.type;
    const uint32_t b = P.b;
    d4 pos = add4(P.ro, scl4(P.rd, h.t));
    d4 eye = mk(-P.rd.x, -P.rd.y, -P.rd.z, -P.rd.w);
    // Object normal -> world normal (tracer.cl:903-955).
    d4 nv;
    if (type == 0 && !((FL & F_TEX) && ob.tex_nm)) {
        PTMI_WADD(41, 1ull);
        nv = ld4(ob.plane_n);  // constant per plane: normalize(mul(invT, (0,1,0,0))), w = 0
    } else {
        PTMI_WADD(42, 1ull);
        d4 on;
        if ((FL & F_TEX) && type == 0) {
            on = plane_normal_map<A>(S.tex[0], ob, pos);
        } else if (type == 1) {
            d4 lp = xpt<A>(ob.inv, ob.st, pos);
            on = mk(lp.x - 0.0, lp.y - 0.0, lp.z - 0.0, A ? 0.0 : lp.w - 1.0);
        } else if ((FL & F_CYLCUBE) && type == 2) {
            d4 lp = xpt<A>(ob.inv, ob.st, pos);
            double dist = lp.x * lp.x + lp.z * lp.z;  // pow(v, 2) folds to v*v
            if (dist < 1 && lp.y >= ob.max_y - kEps) on = mk(0.0, 1.0, 0.0, 0.0);
            else if (dist < 1 && lp.y <= ob.min_y + kEps) on = mk(0.0, -1.0, 0.0, 0.0);
            else on = mk(lp.x, 0.0, lp.z, 0.0);
        } else if ((FL & F_CYLCUBE) && type == 3) {
            d4 lp = xpt<A>(ob.inv, ob.st, pos);
            double mc = max3(fabs(lp.x), fabs(lp.y), fabs(lp.z));
            if (mc == fabs(lp.x)) on = mk(lp.x, 0.0, 0.0, 0.0);
            else if (mc == fabs(lp.y)) on = mk(0.0, lp.y, 0.0, 0.0);
            else on = mk(0.0, 0.0, lp.z, 0.0);
        } else {  // group: interpolated vertex normal of the winning triangle (tracer.cl:669, 949)
            const DevTriShade& T = S.tri_shade[h.tri];
            on = add4(add4(scl4(ld4(T.n2), h.u), scl4(ld4(T.n3), h.v)), scl4(ld4(T.n1), 1.0 - h.u - h.v));
        }
        // mul(invT, n) with .w then set to 0: row 3 is dead; diagonal rows 0-2 when invt_diag.
        const double* it = ob.inv_t;
        if (ob.invt_diag) {
            nv = mk(it[0] * on.x, it[5] * on.y, it[10] * on.z, 0.0);
        } else {
            nv.x = (it[0] * on.x + it[1] * on.y) + it[2] * on.z;
            nv.y = (it[4] * on.x + it[5] * on.y) + it[6] * on.z;
            nv.z = (it[8] * on.x + it[9] * on.y) + it[10] * on.z;
            if constexpr (!A) {  // affine: it[3], it[7], it[11] are +-0 and on.w is finite
                nv.x = nv.x + it[3] * on.w;
                nv.y = nv.y + it[7] * on.w;
                nv.z = nv.z + it[11] * on.w;
            }
            nv.w = 0.0;
        }
        // A sphere's normal invT * (a point on the unit sphere) has |nv| >= 2^-196 in a tame
        // scene (ptmi_api.cpp): normalize's core.  Other shapes keep the full normalize.
        if (A && type == 1) nv = norm3_core(nv);
        else nv = normv<A>(nv);
    }
    if (dotv<A>(eye, nv) < 0.0) nv = scl4(nv, -1.0);
    d4 over = add4(pos, scl4(nv, kEps));
    double cosine = 1.0;
    bool entering = false, exiting = false, reflecting = false;
    // Material decision (tracer.cl:973-1061)
    if ((FL & F_MATERIALS) && ob.reflectivity != 0.0 &&
        (kX ? xnext(P.rng) : noise3d(fgi, (float)n, (float)b)) < ob.reflectivity) {
        P.rd = reflect<A>(P.rd, nv);
        reflecting = true;
    } else if ((FL & F_MATERIALS) && ob.refractive_index == -1.0) {
        if (schlick<A>(eye, nv, 1.0, 1.5) < (kX ? xnext(P.rng) : noise3d(fgi, (float)(n * n), (float)b))) {
            over = sub4(pos, scl4(nv, kEps));
        } else {
            P.rd = reflect<A>(P.rd, nv);
            reflecting = true;
        }
    } else if ((FL & F_MATERIALS) && ob.refractive_index != 1.0) {
        const double ri = ob.refractive_index;
        const bool in = P.inside;
        const double sch = in ? schlick<A>(eye, nv, ri, 1.0) : schlick<A>(eye, nv, 1.0, ri);
        if (sch < (kX ? xnext(P.rng) : noise3d(fgi, (float)(n * n), (float)b))) {
            P.rd = in ? refracted<A>(eye, nv, ri, 1.0) : refracted<A>(eye, nv, 1.0, ri);
            over = sub4(pos, scl4(nv, kEps));
            entering = !in;
            exiting = in;
            P.inside = !in;
        } else {
            P.rd = reflect<A>(P.rd, nv);
            reflecting = true;
        }
    } else {
        float u1, u2;
        if constexpr (kX) {
            u1 = xnext16(P.rng);
            u2 = xnext16(P.rng);
        } else if (PTMI_R6_NPAIR == 1 || PTMI_R6_NPAIR == 3) {
            noise3d_pair(fgi, (float)b, (float)n, (float)b, (float)n, fgi, u1, u2);
        } else {
            u1 = noise3d(fgi, (float)b, (float)n);
            u2 = noise3d((float)b, (float)n, fgi);
        }
        // Only affine instantiations read the table: its records are the affine sequences'
        // results, so they equal what such a lane computes by construction.
        P.rd = random_hemisphere<A, A && (PTMI_HEMI_TAB_GROUPS || !(FL & F_GROUPS)),
                                 A && (PTMI_HEMI_SQRT_GROUPS || !(FL & F_GROUPS))>(S.hemi, nv, u1, u2,
                                                                                 !(FL & F_GROUPS) || S.hemi_mesh);
        cosine = dotv<A>(P.rd, nv);
    }
    P.ro = over;
    // Bounce record + reduction step (tracer.cl:1071-1096, 1148-1175).
    if (!P.done && !(entering || exiting)) {
        double er, eg, eb, cr, cg, cb;
        if ((FL & F_GROUPS) && type == 4) {
            const DevTriShade& T = S.tri_shade[h.tri];
            er = eg = eb = 0.0;
            cr = T.color[0];
            cg = T.color[1];
            cb = T.color[2];
        } else {
            er = ob.emission[0];
            eg = ob.emission[1];
            eb = ob.emission[2];
            cr = ob.color[0];
            cg = ob.color[1];
            cb = ob.color[2];
            if constexpr ((FL & F_TEX) != 0) {
                if (ob.tex) textured_color<A>(S.tex[type == 0 ? 0 : type == 1 ? 1 : 2], ob, pos, cr, cg, cb);
            }
        }
        double mr = P.mr, mg = P.mg, mb = P.mb;
        if constexpr (kMaskLds) {
            mr = msk[0 * kBlock];
            mg = msk[1 * kBlock];
            mb = msk[2 * kBlock];
        }
        if constexpr (kAccLds) {
            // accumColor += mask * emission, skipped when every product is +-0: accumColor
            // starts at +0 and is never -0 before its last write (a sum is -0 only if both
            // terms are), so adding +-0 would leave it unchanged.  NaN products are added.
            const double tr = mr * er, tg = mg * eg, tb = mb * eb;
            if (!(tr == 0.0 && tg == 0.0 && tb == 0.0)) {
                acm[0 * kBlock] = acm[0 * kBlock] + tr;
                acm[1 * kBlock] = acm[1 * kBlock] + tg;
                acm[2 * kBlock] = acm[2 * kBlock] + tb;
            }
        } else {
            P.ar = P.ar + mr * er;
            P.ag = P.ag + mg * eg;
            P.ab = P.ab + mb * eb;
        }
        if (er > 0.0) {
            PTMI_WADD(43, 1ull);
            if (b == 0) {  // the reduction's first record (tracer.cl:1160): records are per bounce, so x == b
                if constexpr (kAccLds) {
                    acm[0 * kBlock] = cr;
                    acm[1 * kBlock] = cg;
                    acm[2 * kBlock] = cb;
                } else {
                    P.ar = cr;
                    P.ag = cg;
                    P.ab = cb;
                }
            }
            P.done = true;
        } else {
            mr = mr * cr;
            mg = mg * cg;
            mb = mb * cb;
            mr = mr * cosine;
            mg = mg * cosine;
            mb = mb * cosine;
            if constexpr (kMaskLds) {
                msk[0 * kBlock] = mr;
                msk[1 * kBlock] = mg;
                msk[2 * kBlock] = mb;
            } else {
                P.mr = mr;
                P.mg = mg;
                P.mb = mb;
            }
        }
    }
    if (!entering && !exiting && !reflecting) P.effective++;
    P.b = b + 1;
    // Loop exits of tracer.cl:884 / 1107-1109.
    return ob.emission[0] > 0.0 || P.b >= kMaxBounces || P.effective >= kMaxEffectiveBounces;
}

// Per-launch resources of trace_kernel<FL>: workgroup size and the register budget.
#ifndef PTMI_WAVES
#define PTMI_WAVES 7  // waves/SIMD the register allocation targets (scenes without groups or materials).
                      // Round 6: with the colour sums really in LDS (PTMI_R6_VACC) and the bounce-loop
                      // cuts, C2's kernel fits 72 VGPRs without spill and C3's 72 with 16 B/lane: 7 waves,
                      // C2 150.5 -> 145.1 ms, C3 153.0 -> 152.0 ms (profiles/r6/SUMMARY.md).  Before:
                      // With the sincos constants in SGPRs (ptmi_fp64core.h) C2/C3 fit 95 VGPRs at 5 waves
                      // without spill (C2 2048 spp 178.0 -> 171.6 ms against the old 3-wave budget); 6 waves
                      // (80 VGPRs, 64 B/lane of spilled loop invariants) gain another 2-2.6 % (C2 171.5 ->
                      // 167.9, C3 179.5 -> 174.9 ms); 7 waves (72 VGPRs, 96 B/lane) lose 10 %
#endif
#ifndef PTMI_WAVES_MATERIALS
#define PTMI_WAVES_MATERIALS 5  // ... with reflective / refractive materials: ~95-101 VGPRs since round 3 (LDS colour
                                // sums and accumColor), 0-32 B/lane of spill at 5; 256 spp: transparency 56.7 -> 53.5,
                                // reflection 28.0 -> 24.9, default 37.4 -> 35.6 ms against 3 waves (4: within 1 %)
#endif
#ifndef PTMI_WAVES_GROUPS
#define PTMI_WAVES_GROUPS 4  // ... and with BVH groups: the walk phases need ~155 VGPRs, so 4 waves spill
                             // 80 B/lane, yet beat 3 waves without spill (512 spp: C4 188 -> 176, C5 294 ->
                             // 271 ms); round 2, at a demand of ~183 and 128 B/lane of spill, 4 lost 14 %
#endif

// Work item of a wave (WorkPlan): the tile's pixel of this lane, its sample range and
// where its sums go.  ok == false: the wave has no item.
struct Item {
    bool ok, whole, inside;
    uint32_t c0, c1;
    size_t oslot;  // output: pixel index into sums, or slot of the partial buffer
    uint32_t i;    // pixel index (inside only)
    int px, py;
};
// Sample range [c0, c1) of chunk c (WorkPlan::n_long, tail_len).
__device__ __forceinline__ void chunk_range(const WorkPlan& WP, uint32_t c, uint32_t& c0, uint32_t& c1) {
    const bool lng = c < WP.n_long;
    c0 = WP.s_begin + (lng ? c * WP.chunk_len : WP.n_long * WP.chunk_len + (c - WP.n_long) * WP.tail_len);
    c1 = min(WP.s_end, c0 + (lng ? WP.chunk_len : WP.tail_len));
}
// kList (F_TLIST instantiations): owned tile k is WP.tiles[k] (a scalar load of a uniform
// index) instead of tile_offset + k * tile_stride.
template <bool kList = false>
__device__ __forceinline__ Item work_item(const DevScene& S, const WorkPlan& WP, uint32_t item, int lane) {
    Item it{};
    const int W = S.cam.width, H = S.cam.height;
    const int tiles_x = (W + kTile - 1) / kTile;
    const int tiles_y = (H + kTile - 1) / kTile;
    uint32_t k;
    if (item < WP.n_whole) {
        it.whole = true;
        k = item;
        it.c0 = WP.s_begin;
        it.c1 = WP.s_end;
    } else {
        it.whole = false;
        const uint32_t t = item - WP.n_whole;
        const uint32_t c = t / max(WP.n_tail, 1u), tq = t - c * WP.n_tail;
        if (c >= WP.nchunks) return it;
        const uint32_t tt = WP.order ? WP.order[WP.n_whole + tq] : tq;  // the round's tq-th tile in dispatch order
        k = WP.n_whole + tt;
        chunk_range(WP, c, it.c0, it.c1);
        it.oslot = ((size_t)c * WP.n_tail + tt) * 64 + lane;
    }
    const uint32_t tile = kList ? WP.tiles[k] : WP.tile_offset + k * WP.tile_stride;
    if (tile >= (uint32_t)(tiles_x * tiles_y)) return it;
    it.px = (int)(tile % (uint32_t)tiles_x) * kTile + (lane & 7);
    it.py = (int)(tile / (uint32_t)tiles_x) * kTile + (lane >> 3);
    // A lane outside the image (edge tiles) stays in its wave's loop without samples:
    // the walk pool's cross-lane steps need every lane of the wave.
    it.inside = it.px < W && it.py < H;
    it.i = it.inside ? (uint32_t)it.py * (uint32_t)W + (uint32_t)it.px : 0u;
    if (it.whole) it.oslot = it.i;
    it.ok = true;
    return it;
}

// A whole-tile item writes its pixel's (r, g, b, samples) into the frame sums.  A chunk
// item: kPlanes, its r, g, b into plane k of the partial buffer at
// k * (nchunks * n_tail * 64) + oslot, the sample counts re-derived by reduce_chunks_kernel
// (24 B per lane and item); else the same (r, g, b, samples) record as a whole tile.  The
// stores are non-temporal: written once, read by the reduce after the launch, they should not
// evict the mesh index and the hemisphere table from an XCD's L2.
// Round 3 kept the mesh kernels on records (the plane store then cost them 9 more spill
// reloads in the loop, C4/C5 +2 %; the row layout [(item * 3 + k) * 64 + lane] cost C2
// +0.3 %).  Round 6, where the mesh kernel stores after its loop from a re-derived item:
// planes C4 533.4 / 532.6 -> 529.7 / 531.1 ms, C5 828.5 / 826.8 -> 823.0 / 824.8; planes and
// non-temporal stores 528.9 / 530.8 and 822.2 / 825.5 ms, C2 unchanged (145.2 / 145.0 ->
// 145.2 / 145.1); HBM per launch C4 1.05 -> 0.88 GB, C5 3.71 -> 3.36 GB (profiles/r6/traffic).
#ifndef PTMI_NT_SUMS
#define PTMI_NT_SUMS 1
#endif
template <bool kPlanes>
__device__ __forceinline__ void store_sums(const Item& it, const WorkPlan& WP, double* __restrict__ sums,
                                           double* __restrict__ part, double cr, double cg, double cb) {
    if (!it.inside) return;
    if (kPlanes && !it.whole) {
        const size_t plane = (size_t)WP.nchunks * WP.n_tail * 64;
        if (PTMI_NT_SUMS) {
            __builtin_nontemporal_store(cr, part + it.oslot);
            __builtin_nontemporal_store(cg, part + plane + it.oslot);
            __builtin_nontemporal_store(cb, part + 2 * plane + it.oslot);
            return;
        }
        part[it.oslot] = cr;
        part[plane + it.oslot] = cg;
        part[2 * plane + it.oslot] = cb;
        return;
    }
    double* o = (it.whole ? sums : part) + it.oslot * 4;
    const double ns = (double)(it.c1 > it.c0 ? it.c1 - it.c0 : 0);
    if (PTMI_NT_SUMS) {
        __builtin_nontemporal_store(cr, o + 0);
        __builtin_nontemporal_store(cg, o + 1);
        __builtin_nontemporal_store(cb, o + 2);
        __builtin_nontemporal_store(ns, o + 3);
        return;
    }
    o[0] = cr;
    o[1] = cg;
    o[2] = cb;
    o[3] = ns;
}

// The scene record through an opaque uniform pointer to the kernel's arguments (DevScene is
// trace_kernel's first argument): inside the bounce loop its fields are scalar-loaded where
// they are used instead of being held in SGPRs across the loop (camera_ptr's reasoning):
// fewer SGPRs live across the loop, fewer of them spilled to VGPR lanes (the C2 loop's
// static v_readlane count 32 -> 18).  2048 spp, one MI355X (profiles/r5/SUMMARY.md s6):
// C3 158.4 -> 156.3 ms; with PTMI_HEMI_TAB_GROUPS C4 577 -> 561, C5 897 -> 882 ms; C2 unchanged.
#ifndef PTMI_SCENE_RELOAD
#define PTMI_SCENE_RELOAD 3  // 1: mesh kernels, 2: kernels without meshes, 3: both (0: off)
#endif
template <bool kReload>
__device__ __forceinline__ const DevScene& scene_reload(const DevScene& S) {
    if constexpr (!kReload) return S;
    typedef const __attribute__((address_space(4))) DevScene ConstScene;
    const DevScene* p = (const DevScene*)__builtin_amdgcn_kernarg_segment_ptr();
    asm("" : "+s"(p));
    const uint64_t a = (uint64_t)p;
    const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32);
    return *(const DevScene*)(ConstScene*)u;
}

// trace_kernel's body for scenes with BVH groups: the loop of the other scenes, with
// the BVH walks deferred.  A lane whose ray needs a walk (group_needs_walk) parks
// (pending, keeping its primitives' best in LDS) and the wave walks all parked lanes
// together once S.walk_batch are parked or no lane is ready to shade -- a walk costs the
// whole wave its longest traversal, so it should run with many lanes, not the ~10 % of
// rays that reach a mesh in any one bounce.  Each lane still traces its samples in
// order, and the closest hit does not depend on when or in which order candidates are
// examined (lexicographic minimum, better()).
// Path pool (round 6; every affine mesh kernel: trace_kernel<1|3|5|...>, the F_TLIST and the F_WIDE
// ones).  A mesh work item is one tile's chunk of samples, lane t tracing pixel t's samples
// in order, so a lane that has traced its chunk idled until the wave's slowest lane was done: 5.7 %
// of the one-GPU loop lane-cycles and 12-15 % of an 8-rank tile share's, whose chunks are short
// (C5 at N = 8: 55 chunks of 38 samples; profiles/r5/timeline).  With the pool a wave's lanes take
// the item's (pixel, sample) paths in order from one wave-wide counter -- path j is pixel j mod 64,
// sample c0 + j / 64 -- whenever their camera buffer is empty, idle lanes first, so no lane idles
// before the item's last 64 paths.  Every path is the reference's path of its (pixel, sample), bit
// for bit; a pixel's colour sum adds its paths in completion order (LDS atomic adds, ds_add_f64)
// instead of sample order: an FP64 summation-order difference (~1e-16 relative), deterministic (one
// wave runs the item in lock step) and independent of the item's tile list or dispatch.  The loop
// carries the buffered path's id instead of the lane's pixel, seed values and sample counter; fgi
// is read from a per-tile LDS table at shading, fgi2 recomputed from the seed at the camera refill,
// and the traversal stack takes the 21 entries the index's depth bound needs (ptmi_bvh.cpp), so the
// LDS stays at 16 waves per CU (10,112 B per wave); spill 48 -> 16 B/lane (trace_kernel<5>).
// 2048 spp, one MI355X, same box (profiles/r6/pool): C4 528.3 -> 489.8 ms, C5 822.9 -> 784.3 ms;
// 8-rank shares (tools/shard_balance.py): C5 tile split Sigma/T1 1.195 -> 1.050, projected
// efficiency 0.831 -> 0.941.  (The generic and statistical-RNG mesh kernels keep trace_groups;
// PTMI_POOL=0 builds the diagnostic libraries without the pool.)
#ifndef PTMI_POOL
#define PTMI_POOL 1
#endif
template <int FL>
constexpr bool kPoolOf = PTMI_POOL != 0 && (FL & F_GROUPS) != 0 && !(FL & (F_PROJ | F_XRNG));
template <int FL>
__device__ __forceinline__ void trace_groups(const DevScene& S0, uint32_t samples, const WorkPlan& WP,
                                             const double* __restrict__ seeds, const double* __restrict__ sunf,
                                             double* __restrict__ sums, double* __restrict__ part, uint32_t item) {
    constexpr bool A = !(FL & F_PROJ);
    constexpr bool kDof = (FL & F_DOF) != 0;
    constexpr int kCamComp = (kDof || !A) ? (A ? 6 : 8) : 3;  // see trace_kernel
    const DevScene& S = S0;
    // Per-lane BVH traversal stacks, lane-interleaved (entry k of lane t at
    // [k * kStkStride + t]) so a wave's pushes and pops hit 64 consecutive dwords; the
    // per-pixel colour sums (the same additions in the same order) and a parked lane's
    // primitive best (t, pk), which change once per path or per park, wait in LDS too:
    // registers are what the walk phases need.
    // 16-bit entries unless the scene's codes are wide (F_WIDE: 6 KB per wave, 13.3 KB in all, so
    // LDS then holds 12 waves per CU instead of 16).
    __shared__ StackEntry<A && !(FL & F_WIDE)> stk_lds[kStack * kStkStride];
    __shared__ double acc_lds[3 * kBlock];
    // accumColor of the lane's current path in LDS (bounce_shade kAccLds), as in the kernels
    // without meshes: it changes only on bounces that see emission, and in registers the
    // 4-wave budget spilled it with a load and a store per bounce.
    constexpr bool kAcm = PTMI_GROUP_ACM != 0;
    __shared__ double acm_lds[kAcm ? 3 * kBlock : 1];
    // ... and the path's mask (bounce_shade kMaskLds).
    constexpr bool kMsk = PTMI_GROUP_MASK != 0;
    __shared__ double msk_lds[kMsk ? 3 * kBlock : 1];
    __shared__ double hp_t_lds[kBlock];
    __shared__ int hp_pk_lds[kBlock];
    __shared__ double cam_lds[kCamComp * kBlock];
    const int tid = threadIdx.x, lane = tid & 63;
#if PTMI_STATS
    ptmi_wstat[0][lane] = 0;
#endif
    const Item it = work_item<(FL & F_TLIST) != 0>(S, WP, item, lane);
    if (!it.ok) return;
    const int px = it.px, py = it.py;
    // fgi / fgi2 (tracer.cl:839-841): double division rounded to float.
    const double seed = it.inside ? seeds[it.i] : 0.0;
    const float fgi = (float)(seed / (double)S.n_list);
    const float fgi2 = (float)(seed / (double)samples);
    const XSeed seed_bits = xseed_of((uint64_t)__double_as_longlong(seed));  // statistical mode
    const uint32_t c_end = it.inside ? it.c1 : it.c0;
    auto* stk = lds_ptr(stk_lds + tid);
#if PTMI_R6_VACC  // (the colour sums really in LDS: see trace_kernel)
    volatile __attribute__((address_space(3))) double* acc =
        (volatile __attribute__((address_space(3))) double*)(acc_lds + tid);
#else
    double* acc = acc_lds + tid;
#endif
    acc[0 * kBlock] = 0.0;
    acc[1 * kBlock] = 0.0;
    acc[2 * kBlock] = 0.0;
    double* acm = kAcm ? acm_lds + tid : nullptr;
    double* msk = kMsk ? msk_lds + tid : nullptr;
    uint32_t n_gen = it.c0;
#if PTMI_NCUR_LDS
    // The sample index of the lane's current path waits in LDS (written at path start, read by
    // the shading's noise draws): in registers the 4-wave budget spilled it, a scratch store at
    // nearly every loop iteration.
    __shared__ uint32_t ncur_lds[kBlock];
#else
    uint32_t n_cur = 0;
#endif
    bool buffered = false, active = false, pending = false;
    PathState P;
    PTMI_TSTAMP(t_loop);
    for (;;) {
        if (!__any(active || buffered || n_gen < c_end)) break;
        const DevScene& S = scene_reload<(PTMI_SCENE_RELOAD & 1) != 0>(S0);
        PTMI_TSTAMP(t_a);
        // Camera rays in wave-wide batches (see trace_kernel).
        const bool need = !buffered && n_gen < c_end;
        const int n_need = __popcll(__ballot(need));
        const int n_starve = __popcll(__ballot(!buffered && !active && n_gen < c_end));
        if (n_need >= kRefillNeed || n_starve >= PTMI_REFILL_STARVE_GROUPS || (n_starve > 0 && !__any(active))) {
            const DevCamera& cam = camera_ptr<(PTMI_CAM_RELOAD & 2) != 0>(S);
            if (need) {
                d4 ro, rd;
                float rx, ry;
                camera_offsets<FL>(fgi, fgi2, seed_bits, n_gen, rx, ry);
                ray_for_pixel<kDof, A>(cam, sunf, (unsigned)px, (unsigned)py, rx, ry, (int)n_gen, ro, rd);
                double* cb = cam_lds + tid;
                cb[0 * kBlock] = rd.x;
                cb[1 * kBlock] = rd.y;
                cb[2 * kBlock] = rd.z;
                if constexpr (kCamComp > 3) {
                    cb[3 * kBlock] = ro.x;
                    cb[4 * kBlock] = ro.y;
                    cb[5 * kBlock] = ro.z;
                }
                if constexpr (!A) {
                    cb[6 * kBlock] = ro.w;
                    cb[7 * kBlock] = rd.w;
                }
                n_gen++;
                buffered = true;
            }
        }
        if (!active && buffered) {
            const double* cb = cam_lds + tid;
            const d4 crd = mk(cb[0 * kBlock], cb[1 * kBlock], cb[2 * kBlock], A ? 0.0 : cb[(kCamComp - 1) * kBlock]);
            d4 cro;
            if constexpr (kCamComp > 3)
                cro = mk(cb[3 * kBlock], cb[4 * kBlock], cb[5 * kBlock], A ? 1.0 : cb[(kCamComp - 2) * kBlock]);
            else
                {
                    const double* co = camera_ptr<(PTMI_CAM_RELOAD & 2) != 0>(S).origin;  // ray_for_pixel's origin
                    cro = mk(co[0], co[1], co[2], 1.0);
                }
            start_path<A, kDof>(P, cro, crd);
            if constexpr (kAcm) {
                acm[0 * kBlock] = 0.0;
                acm[1 * kBlock] = 0.0;
                acm[2 * kBlock] = 0.0;
            }
            if constexpr (kMsk) {
                msk[0 * kBlock] = 1.0;
                msk[1 * kBlock] = 1.0;
                msk[2 * kBlock] = 1.0;
            }
#if PTMI_NCUR_LDS
            ncur_lds[tid] = n_gen - 1;
#else
            n_cur = n_gen - 1;
#endif
            if constexpr ((FL & F_XRNG) != 0) P.rng = xseed(seed_bits, n_gen - 1);
            buffered = false;
            active = true;
        }
        PTMI_TADD(12, t_a);
        PTMI_TSTAMP(t_b);
        bool ready = false;
        Hit h;
        if (active && !pending) {
            if (P.dead) {
                h.pk = -1;
                ready = true;
            } else {
                h = find_closest_prims<FL>(S, P.ro, P.rd);
                const bool nw = group_needs_walk<A>(S, P.ro, P.rd, h);
                if (PTMI_ABLATE & 1024) asm volatile("" ::"v"(nw ? 1 : 0));  // DIAGNOSTIC 1024: hull culls kept,
                                                                              // no walks (the mesh is invisible)
                if (!(PTMI_ABLATE & 1024) && nw) {
                    pending = true;
                    hp_t_lds[tid] = h.t;  // find_closest_prims: tri, ti, u, v are constants
                    hp_pk_lds[tid] = h.pk;
                } else {
                    ready = true;
                }
            }
        }
        PTMI_TADD(13, t_b);
        PTMI_TSTAMP(t_c);
        const int n_pend = __popcll(__ballot(pending));
        if (n_pend >= S.walk_batch || (n_pend > 0 && !__any(ready))) {
            PTMI_WADD(8, 1ull);
            PTMI_WADD(9, (unsigned long long)n_pend);
            if (pending) {
                h = Hit{hp_t_lds[tid], hp_pk_lds[tid], -1, -1, 0.0, 0.0};
#if PTMI_CAPTURE
                const unsigned ci = atomicAdd(&ptmi_cap_n, 1u);
                if (ci < ptmi_cap_max)
                    ptmi_cap_req[ci] = WalkReq{{P.ro.x, P.ro.y, P.ro.z}, {P.rd.x, P.rd.y, P.rd.z}, h.t, h.pk, 0};
#endif
                group_walks<A>(S, stk, P.ro, P.rd, h);
#if PTMI_CAPTURE
                if (ci < ptmi_cap_max) ptmi_cap_res[ci] = WalkRes{h.t, h.pk, h.tri, h.ti, 0, h.u, h.v};
#endif
                pending = false;
                ready = true;
            }
        }
        PTMI_TADD(14, t_c);
        PTMI_TSTAMP(t_d);
#if PTMI_NCUR_LDS
        if (ready && bounce_shade<FL, kAcm, kMsk>(S, P, h, fgi, ncur_lds[tid], acm, msk)) {
#else
        if (ready && bounce_shade<FL, kAcm, kMsk>(S, P, h, fgi, n_cur, acm, msk)) {
#endif
            if constexpr (kAcm) {
                acc[0 * kBlock] = acc[0 * kBlock] + acm[0 * kBlock];  // colors += accumColor (tracer.cl:1179)
                acc[1 * kBlock] = acc[1 * kBlock] + acm[1 * kBlock];
                acc[2 * kBlock] = acc[2 * kBlock] + acm[2 * kBlock];
            } else {
                acc[0 * kBlock] = acc[0 * kBlock] + P.ar;
                acc[1 * kBlock] = acc[1 * kBlock] + P.ag;
                acc[2 * kBlock] = acc[2 * kBlock] + P.ab;
            }
            active = false;
        }
        PTMI_TADD(15, t_d);
        PTMI_WADD(10, 1ull);
#if PTMI_STATS == 2
        {  // (timers build: lane-cycles of lanes whose item has no sample left, [27] of [28])
            const unsigned long long dt = clock64() - t_a;
            PTMI_WADD(27, dt * (unsigned long long)__popcll(__ballot(!active && !buffered && n_gen >= c_end)));
            PTMI_WADD(28, dt * 64ull);
        }
#endif
    }
    PTMI_TADD(16, t_loop);
#if PTMI_STATS
    if (PTMI_FIRST_ACTIVE())
        for (int k = 0; k < 64; k++)
            if (ptmi_wstat[0][k]) atomicAdd(&ptmi_stats[k], ptmi_wstat[0][k]);
#endif
    // The work item is re-derived (a few integer operations) rather than kept live across
    // the loop: its fields would hold ~5 VGPRs through every walk phase.
    store_sums<PTMI_MESH_PLANES != 0>(work_item<(FL & F_TLIST) != 0>(S, WP, item, lane), WP, sums, part, acc[0 * kBlock], acc[1 * kBlock], acc[2 * kBlock]);
}

// trace_groups with the path pool (kPoolOf above): the same loop, phases and walks; what
// changes is which (pixel, sample) a lane's next camera ray is for, and where its colour goes.
template <int FL>
__device__ __forceinline__ void trace_groups_pool(const DevScene& S0, uint32_t samples, const WorkPlan& WP,
                                                  const double* __restrict__ seeds, const double* __restrict__ sunf,
                                                  double* __restrict__ sums, double* __restrict__ part,
                                                  uint32_t item) {
    constexpr bool A = true;
    constexpr bool kDof = (FL & F_DOF) != 0;
    constexpr int kCamComp = kDof ? 6 : 3;
    constexpr int kPoolStack = 21;  // ptmi_bvh.cpp kMaxNode4Depth * 3
    static_assert(kPoolStack <= kStack, "pool stack");
    __shared__ StackEntry<!(FL & F_WIDE)> stk_lds[kPoolStack * kStkStride];  // 32-bit codes: F_WIDE
    __shared__ double acc_lds[3 * kBlock];  // colour sum of pixel t of the tile at [k * 64 + t]
    __shared__ double acm_lds[3 * kBlock];  // accumColor / mask of the lane's path (as trace_groups)
    __shared__ double msk_lds[3 * kBlock];
    __shared__ double hp_t_lds[kBlock];
    __shared__ int hp_pk_lds[kBlock];
    __shared__ double cam_lds[kCamComp * kBlock];
    __shared__ uint32_t ncur_lds[kBlock];  // the lane's current path j: pixel j & 63, sample c0 + (j >> 6)
    __shared__ float fgi_lds[kBlock];      // fgi of pixel t of the tile
    const int tid = threadIdx.x, lane = tid & 63;
#if PTMI_STATS
    ptmi_wstat[0][lane] = 0;
#endif
    const Item it = work_item<(FL & F_TLIST) != 0>(S0, WP, item, lane);
    if (!it.ok) return;
    const double seed0 = it.inside ? seeds[it.i] : 0.0;
    fgi_lds[tid] = (float)(seed0 / (double)S0.n_list);
    acc_lds[0 * kBlock + tid] = 0.0;
    acc_lds[1 * kBlock + tid] = 0.0;
    acc_lds[2 * kBlock + tid] = 0.0;
    // The lanes read each other's fgi and add into each other's sums from here on: a wave barrier
    // (one wave per workgroup; LDS serves a wave's operations in program order) keeps the compiler
    // from moving those accesses across the initialisation, and the one after the loop keeps the
    // final reads of the sums after every lane's adds.
    __builtin_amdgcn_wave_barrier();
    // The tile's origin and sample range are the wave's (work_item of lane 0).
    const int tx0 = __builtin_amdgcn_readfirstlane(it.px - (lane & 7));
    const int ty0 = __builtin_amdgcn_readfirstlane(it.py - (lane >> 3));
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)it.c0);
    const uint32_t total = 64u * ((uint32_t)__builtin_amdgcn_readfirstlane((int)it.c1) - c0);
    const int W = S0.cam.width, H = S0.cam.height;
    auto* stk = lds_ptr(stk_lds + tid);
    double* acm = acm_lds + tid;
    double* msk = msk_lds + tid;
    uint32_t j_next = 0;  // the next path of the item (wave-uniform)
    uint32_t buf_id = 0;  // the buffered camera ray's path j
    bool buffered = false, active = false, pending = false;
    PathState P;
    for (;;) {
        if (!__any(active || buffered) && j_next >= total) break;
        const DevScene& S = scene_reload<(PTMI_SCENE_RELOAD & 1) != 0>(S0);
        // Camera rays in wave-wide batches, as trace_groups; the lanes without a buffered ray take
        // the next paths, idle lanes first.
        const uint32_t avail = total - j_next;
        const uint64_t m_idle = __ballot(!buffered && !active), m_busy = __ballot(!buffered && active);
        const uint32_t n_idle = min((uint32_t)__popcll(m_idle), avail);
        const uint32_t n_need = min((uint32_t)(__popcll(m_idle) + __popcll(m_busy)), avail);
        if (n_need >= (uint32_t)kRefillNeed || n_idle >= (uint32_t)PTMI_REFILL_STARVE_GROUPS ||
            (n_idle > 0 && !__any(active))) {
            const uint32_t rank = active ? (uint32_t)__popcll(m_idle) + __builtin_amdgcn_mbcnt_hi(
                                                                            (uint32_t)(m_busy >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m_busy, 0u))
                                         : __builtin_amdgcn_mbcnt_hi((uint32_t)(m_idle >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m_idle, 0u));
            if (!buffered && rank < avail) {
                const uint32_t j = j_next + rank;
                const uint32_t p = j & 63u, n = c0 + (j >> 6);
                const int px = tx0 + (int)(p & 7u), py = ty0 + (int)(p >> 3);
                const bool in = px < W && py < H;
                const double sd = in ? seeds[(uint32_t)py * (uint32_t)W + (uint32_t)px] : 0.0;
                const float fgi2 = (float)(sd / (double)samples);
                const DevCamera& cam = camera_ptr<(PTMI_CAM_RELOAD & 2) != 0>(S);
                d4 ro, rd;
                float rx, ry;
                camera_offsets<FL>(fgi_lds[p], fgi2, XSeed{}, n, rx, ry);
                ray_for_pixel<kDof, A>(cam, sunf, (unsigned)px, (unsigned)py, rx, ry, (int)n, ro, rd);
                double* cb = cam_lds + tid;
                cb[0 * kBlock] = rd.x;
                cb[1 * kBlock] = rd.y;
                cb[2 * kBlock] = rd.z;
                if constexpr (kCamComp > 3) {
                    cb[3 * kBlock] = ro.x;
                    cb[4 * kBlock] = ro.y;
                    cb[5 * kBlock] = ro.z;
                }
                buf_id = j;
                buffered = true;
            }
            j_next += n_need;
        }
        if (!active && buffered) {
            const double* cb = cam_lds + tid;
            const d4 crd = mk(cb[0 * kBlock], cb[1 * kBlock], cb[2 * kBlock], 0.0);
            d4 cro;
            if constexpr (kCamComp > 3) {
                cro = mk(cb[3 * kBlock], cb[4 * kBlock], cb[5 * kBlock], 1.0);
            } else {
                const double* co = camera_ptr<(PTMI_CAM_RELOAD & 2) != 0>(S).origin;
                cro = mk(co[0], co[1], co[2], 1.0);
            }
            start_path<A, kDof>(P, cro, crd);
            acm[0 * kBlock] = 0.0;
            acm[1 * kBlock] = 0.0;
            acm[2 * kBlock] = 0.0;
            msk[0 * kBlock] = 1.0;
            msk[1 * kBlock] = 1.0;
            msk[2 * kBlock] = 1.0;
            ncur_lds[tid] = buf_id;
            buffered = false;
            active = true;
        }
        bool ready = false;
        Hit h;
        if (active && !pending) {
            if (P.dead) {
                h.pk = -1;
                ready = true;
            } else {
                h = find_closest_prims<FL>(S, P.ro, P.rd);
                if (group_needs_walk<A>(S, P.ro, P.rd, h)) {
                    pending = true;
                    hp_t_lds[tid] = h.t;
                    hp_pk_lds[tid] = h.pk;
                } else {
                    ready = true;
                }
            }
        }
        const int n_pend = __popcll(__ballot(pending));
        if (n_pend >= S.walk_batch || (n_pend > 0 && !__any(ready))) {
            if (pending) {
                h = Hit{hp_t_lds[tid], hp_pk_lds[tid], -1, -1, 0.0, 0.0};
                group_walks<A>(S, stk, P.ro, P.rd, h);
                pending = false;
                ready = true;
            }
        }
        if (ready) {
            const uint32_t id = ncur_lds[tid];
            if (bounce_shade<FL, true, true>(S, P, h, fgi_lds[id & 63u], c0 + (id >> 6), acm, msk)) {
                // colors += accumColor (tracer.cl:1179) into the path's pixel; two lanes may finish
                // paths of one pixel in the same step, hence the atomic adds.
                const uint32_t p = id & 63u;
                atomicAdd(&acc_lds[0 * kBlock + p], acm[0 * kBlock]);
                atomicAdd(&acc_lds[1 * kBlock + p], acm[1 * kBlock]);
                atomicAdd(&acc_lds[2 * kBlock + p], acm[2 * kBlock]);
                active = false;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    store_sums<PTMI_MESH_PLANES != 0>(work_item<(FL & F_TLIST) != 0>(S0, WP, item, lane), WP, sums, part, acc_lds[0 * kBlock + tid],
                                      acc_lds[1 * kBlock + tid], acc_lds[2 * kBlock + tid]);
}

// The path pool for the kernels without meshes (PTMI_POOL_FLAT, affine non-DoF parity-mode scenes):
// the loop of trace_kernel's else branch with trace_groups_pool's path hand-out.  Measured and off:
// their items are mostly whole tiles (2048 samples per lane, no per-item drain to remove), and what
// the pool saves in registers (C2: 69 instead of 72 VGPRs at 7 waves, or 8 waves at 64 VGPRs with
// 16 B/lane of spill, 5,120 B of LDS) does not pay for its LDS reads and atomics: 2048 spp, same
// box, C2 144.46 ms -> 146.9 (7 waves) / 145.3 ms (8 waves) (profiles/r6/tune/ab2).
#ifndef PTMI_POOL_FLAT
#define PTMI_POOL_FLAT 0
#endif
#ifndef PTMI_POOL_FGI2_SEED
#define PTMI_POOL_FGI2_SEED 1  // fgi2 recomputed from the seed at the camera refill (no LDS table)
#endif
template <int FL>
constexpr bool kPoolFlatOf = PTMI_POOL_FLAT != 0 && !(FL & (F_GROUPS | F_PROJ | F_XRNG | F_TEX | F_DOF));
template <int FL>
__device__ __forceinline__ void trace_flat_pool(const DevScene& S0, uint32_t samples, const WorkPlan& WP,
                                                const double* __restrict__ seeds, const double* __restrict__ sunf,
                                                double* __restrict__ sums, double* __restrict__ part) {
    constexpr bool A = true;
    constexpr bool kDof = (FL & F_DOF) != 0;
    constexpr int kCamComp = kDof ? 6 : 3;
    __shared__ double acc_lds[3 * kBlock];
    __shared__ double acm_lds[3 * kBlock];
    __shared__ double cam_lds[kCamComp * kBlock];
    __shared__ uint32_t ncur_lds[kBlock];
    __shared__ float fgi_lds[kBlock];
    __shared__ float fgi2_lds[PTMI_POOL_FGI2_SEED ? 1 : kBlock];
    const int tid = threadIdx.x, lane = tid & 63;
    const Item it = work_item(S0, WP, blockIdx.x, lane);
    if (!it.ok) return;
    {
        const double seed0 = it.inside ? seeds[it.i] : 0.0;
        fgi_lds[tid] = (float)(seed0 / (double)S0.n_list);
        if (!PTMI_POOL_FGI2_SEED) fgi2_lds[tid] = (float)(seed0 / (double)samples);
    }
    const int W = S0.cam.width, H = S0.cam.height;
    acc_lds[0 * kBlock + tid] = 0.0;
    acc_lds[1 * kBlock + tid] = 0.0;
    acc_lds[2 * kBlock + tid] = 0.0;
    __builtin_amdgcn_wave_barrier();  // (see trace_groups_pool)
    const int tx0 = __builtin_amdgcn_readfirstlane(it.px - (lane & 7));
    const int ty0 = __builtin_amdgcn_readfirstlane(it.py - (lane >> 3));
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)it.c0);
    const uint32_t total = 64u * ((uint32_t)__builtin_amdgcn_readfirstlane((int)it.c1) - c0);
    double* acm = acm_lds + tid;
    uint32_t j_next = 0, buf_id = 0;
    bool buffered = false, active = false;
    PathState P;
    for (;;) {
        if (!__any(active || buffered) && j_next >= total) break;
        const DevScene& S = scene_reload<(PTMI_SCENE_RELOAD & 2) != 0>(S0);
        const uint32_t avail = total - j_next;
        const uint64_t m_idle = __ballot(!buffered && !active), m_busy = __ballot(!buffered && active);
        const uint32_t n_idle = min((uint32_t)__popcll(m_idle), avail);
        const uint32_t n_need = min((uint32_t)(__popcll(m_idle) + __popcll(m_busy)), avail);
        if (n_need >= (uint32_t)kRefillNeed || n_idle >= (uint32_t)PTMI_REFILL_STARVE || (n_idle > 0 && !__any(active))) {
            const uint32_t rank = active ? (uint32_t)__popcll(m_idle) + __builtin_amdgcn_mbcnt_hi(
                                                                            (uint32_t)(m_busy >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m_busy, 0u))
                                         : __builtin_amdgcn_mbcnt_hi((uint32_t)(m_idle >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m_idle, 0u));
            if (!buffered && rank < avail) {
                const uint32_t j = j_next + rank;
                const uint32_t p = j & 63u, n = c0 + (j >> 6);
                const int px = tx0 + (int)(p & 7u), py = ty0 + (int)(p >> 3);
                float fgi2;
                if (PTMI_POOL_FGI2_SEED) {
                    const double sd = (px < W && py < H) ? seeds[(uint32_t)py * (uint32_t)W + (uint32_t)px] : 0.0;
                    fgi2 = (float)(sd / (double)samples);
                } else {
                    fgi2 = fgi2_lds[p];
                }
                const DevCamera& cam = camera_ptr<(PTMI_CAM_RELOAD & 1) != 0>(S);
                d4 ro, rd;
                float rx, ry;
                camera_offsets<FL>(fgi_lds[p], fgi2, XSeed{}, n, rx, ry);
                ray_for_pixel<kDof, A>(cam, sunf, (unsigned)px, (unsigned)py, rx, ry, (int)n, ro, rd);
                double* cb = cam_lds + tid;
                cb[0 * kBlock] = rd.x;
                cb[1 * kBlock] = rd.y;
                cb[2 * kBlock] = rd.z;
                if constexpr (kCamComp > 3) {
                    cb[3 * kBlock] = ro.x;
                    cb[4 * kBlock] = ro.y;
                    cb[5 * kBlock] = ro.z;
                }
                buf_id = j;
                buffered = true;
            }
            j_next += n_need;
        }
        if (!active && buffered) {
            const double* cb = cam_lds + tid;
            const d4 crd = mk(cb[0 * kBlock], cb[1 * kBlock], cb[2 * kBlock], 0.0);
            d4 cro;
            if constexpr (kCamComp > 3) {
                cro = mk(cb[3 * kBlock], cb[4 * kBlock], cb[5 * kBlock], 1.0);
            } else {
                const double* co = camera_ptr<(PTMI_CAM_RELOAD & 1) != 0>(S).origin;
                cro = mk(co[0], co[1], co[2], 1.0);
            }
            start_path<A, kDof>(P, cro, crd);
            acm[0 * kBlock] = 0.0;
            acm[1 * kBlock] = 0.0;
            acm[2 * kBlock] = 0.0;
            ncur_lds[tid] = buf_id;
            buffered = false;
            active = true;
        }
        if (active) {
            Hit h;
            if (P.dead) h.pk = -1;
            else h = find_closest_prims<FL>(S, P.ro, P.rd);
            const uint32_t id = ncur_lds[tid];
            if (bounce_shade<FL, true>(S, P, h, fgi_lds[id & 63u], c0 + (id >> 6), acm)) {
                const uint32_t p = id & 63u;
                atomicAdd(&acc_lds[0 * kBlock + p], acm[0 * kBlock]);
                atomicAdd(&acc_lds[1 * kBlock + p], acm[1 * kBlock]);
                atomicAdd(&acc_lds[2 * kBlock + p], acm[2 * kBlock]);
                active = false;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    store_sums<true>(work_item(S0, WP, blockIdx.x, lane), WP, sums, part, acc_lds[0 * kBlock + tid],
                     acc_lds[1 * kBlock + tid], acc_lds[2 * kBlock + tid]);
}

// Per-item duration onto its tile's cost accumulator (WorkPlan::cost, tile_order_kernel;
// mesh kernels only).  Off in the product (PTMI_TILE_COST 0): the clock read at an item's
// start (s_memrealtime, an intrinsic with side effects) made the uniform-load analysis treat
// every later global load as clobbered, so the mesh kernel's object and root records went
// from scalar to vector loads (82 of 108 s_loads; HBM writes 3 -> 57 GB per C4 frame from
// the extra VGPR pressure and spill).  Kept in LDS the tick cost the mesh kernel its 16th
// wave per CU; in the kernels without meshes any clock read cost 48 B/lane of spill.
#ifndef PTMI_TILE_COST
#define PTMI_TILE_COST PTMI_STUDY  // the study build measures; the product does not
#endif
__device__ __forceinline__ void item_cost_add(const DevScene& S, const WorkPlan& WP, uint32_t item,
                                              unsigned long long t0) {
    if (WP.cost && threadIdx.x == 0) {
        const Item it = work_item(S, WP, item, 0);
        if (it.ok) {
            const uint32_t tiles_x = ((uint32_t)S.cam.width + kTile - 1) / kTile;
            atomicAdd(&WP.cost[(uint32_t)(it.py / kTile) * tiles_x + (uint32_t)(it.px / kTile)], wall_clock64() - t0);
        }
    }
}

// One wave per workgroup; workgroup b runs work item b of the WorkPlan: an 8x8 tile
// over the whole sample range (sums -> the frame) or a sample chunk of a tail tile
// (sums -> its slot of the partial buffer).  A wave that finishes frees its slot (LDS
// included) at once.  RGB sums, A = #samples.
// Which item a mesh kernel's workgroup runs: PTMI_ITEM_QUEUE 1 -- the next one in dispatch
// order from a per-launch counter (one atomic per workgroup, zeroed before the launch), so
// items go to whichever XCD frees a slot first instead of workgroup b's fixed XCD (b mod 8),
// whose static eighth of the items made the XCDs of an 8-rank C5 share end up to 8 ms apart
// (profiles/r5/timeline).  The scene records the kernel reads after it come through the
// constant address space (cmem), so the atomic does not make them look clobbered to the
// compiler's uniform-load analysis (with plain global reads 18 of trace_kernel<5>'s scalar
// loads became vector loads and the frames lost 5.5 %, profiles/r5/item_queue).  Every item
// writes only its own sums: the frame does not depend on the assignment.  The kernels without
// meshes keep blockIdx.x.
#ifndef PTMI_ITEM_QUEUE
#define PTMI_ITEM_QUEUE 1
#endif
__device__ __forceinline__ uint32_t take_item(uint32_t* __restrict__ ctr) {
#if PTMI_ITEM_QUEUE
    uint32_t v = 0;
    if (threadIdx.x == 0) v = atomicAdd(ctr, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);  // lane 0: every lane is active here
#else
    (void)ctr;
    return blockIdx.x;
#endif
}
template <int FL>
__global__ __launch_bounds__(kBlock, (FL & F_GROUPS)      ? PTMI_WAVES_GROUPS
                                                  : (FL & F_MATERIALS) ? PTMI_WAVES_MATERIALS
                                                                       : PTMI_WAVES) void trace_kernel(DevScene S, uint32_t samples, WorkPlan WP,
                                                    const double* __restrict__ seeds, const double* __restrict__ sunf,
                                                    double* __restrict__ sums, double* __restrict__ part,
                                                    uint32_t* __restrict__ item_ctr) {
#if PTMI_TIMELINE
    const unsigned long long tl0 = wall_clock64();
#endif
    if constexpr ((FL & F_GROUPS) != 0) {
        const uint32_t item = take_item(item_ctr);
#if PTMI_TILE_COST
        const unsigned long long c0 = WP.cost ? wall_clock64() : 0ull;
#endif
        if constexpr (kPoolOf<FL>)
            trace_groups_pool<FL>(S, samples, WP, seeds, sunf, sums, part, item);
        else
            trace_groups<FL>(S, samples, WP, seeds, sunf, sums, part, item);
#if PTMI_TILE_COST
        item_cost_add(S, WP, item, c0);
#endif
#if PTMI_TIMELINE
        if (threadIdx.x == 0 && item < ptmi_tl_max) {
            ptmi_tl[2 * item] = tl0;
            ptmi_tl[2 * item + 1] = wall_clock64();
        }
#endif
    } else if constexpr (kPoolFlatOf<FL>) {
        trace_flat_pool<FL>(S, samples, WP, seeds, sunf, sums, part);
    } else {
        constexpr bool A = !(FL & F_PROJ);
        const int tid = threadIdx.x, lane = tid & 63;
#if PTMI_STATS
        ptmi_wstat[0][lane] = 0;
#endif
        const Item it = work_item(S, WP, blockIdx.x, lane);
        if (!it.ok) return;
        const int px = it.px, py = it.py;
        // fgi / fgi2 (tracer.cl:839-841): double division rounded to float.
        const double seed = it.inside ? seeds[it.i] : 0.0;
        const float fgi = (float)(seed / (double)S.n_list);
        const float fgi2 = (float)(seed / (double)samples);
        const XSeed seed_bits = xseed_of((uint64_t)__double_as_longlong(seed));  // statistical mode
        const uint32_t c_end = it.inside ? it.c1 : it.c0;
        // colors (tracer.cl:1179): one LDS slot per lane, the same additions in the same
        // order; they change once per path, and the registers keep the bounce loop off
        // scratch at the 6-waves/SIMD budget.
        __shared__ double acc_lds[3 * kBlock];
        // volatile (round 6): without it the compiler, seeing no other reader, kept the three
        // sums in registers across the whole loop -- 6 VGPRs and 3 v_mov_b64 per iteration --
        // and wrote the LDS slots only after it.
#if PTMI_R6_VACC
        volatile __attribute__((address_space(3))) double* acc =
            (volatile __attribute__((address_space(3))) double*)(acc_lds + tid);
#else
        double* acc = acc_lds + tid;
#endif
        acc[0 * kBlock] = 0.0;
        acc[1 * kBlock] = 0.0;
        acc[2 * kBlock] = 0.0;
        // accumColor of the lane's current path (bounce_shade kAccLds): 6 VGPRs fewer
        // through the bounce loop.
        __shared__ double acm_lds[3 * kBlock];
        double* acm = acm_lds + tid;
        // Camera rays are produced in wave-wide batches into a one-deep per-lane buffer
        // (LDS) and consumed by path regeneration: generating them at the moment each lane
        // needs one would run the camera block (2 noise3D + the transform) on nearly every
        // bounce iteration with ~1/5 of the lanes active.  Per lane the samples are still
        // traced in order n = c0, c0+1, ..., so the arithmetic and the order of `colors +=`
        // are unchanged.  SoA, component c of lane t at [c * 64 + t]: the direction, then
        // (DoF or non-affine scenes) the origin; affine scenes keep no w lanes.  (2- and
        // 3-deep buffers measured no faster on C2, +1.4 % on the group scenes.)
        constexpr int kCamComp = ((FL & F_DOF) || !A) ? (A ? 6 : 8) : 3;
        constexpr int kWg = kBlock;
        __shared__ double cam_lds[kCamComp * kWg];
        uint32_t n_gen = it.c0;  // next sample whose camera ray is to be generated
        uint32_t n_cur = 0;
        bool buffered = false, active = false;
        PathState P;
        PTMI_TSTAMP(t_loop);
        const DevScene& S0 = S;
        for (;;) {
            if (!__any(active || buffered || n_gen < c_end)) break;
            const DevScene& S = scene_reload<(PTMI_SCENE_RELOAD & 2) != 0>(S0);
            PTMI_TSTAMP(t_a);
            const bool need = !buffered && n_gen < c_end;
            const int n_need = __popcll(__ballot(need));
            const int n_starve = __popcll(__ballot(!buffered && !active && n_gen < c_end));
            if (n_need >= kRefillNeed || n_starve >= PTMI_REFILL_STARVE || (n_starve > 0 && !__any(active))) {
                const DevCamera& cam = camera_ptr<(PTMI_CAM_RELOAD & 1) != 0>(S);
                PTMI_WADD(32, 1ull);
                if (need) {
                    d4 ro, rd;
                    float rx, ry;
                    camera_offsets<FL>(fgi, fgi2, seed_bits, n_gen, rx, ry);
                    ray_for_pixel<(FL & F_DOF) != 0, A>(cam, sunf, (unsigned)px, (unsigned)py, rx, ry, (int)n_gen,
                                                        ro, rd);
                    double* cbuf = cam_lds + tid;
                    cbuf[0 * kWg] = rd.x;
                    cbuf[1 * kWg] = rd.y;
                    cbuf[2 * kWg] = rd.z;
                    if constexpr (kCamComp > 3) {
                        cbuf[3 * kWg] = ro.x;
                        cbuf[4 * kWg] = ro.y;
                        cbuf[5 * kWg] = ro.z;
                    }
                    if constexpr (!A) {
                        cbuf[6 * kWg] = ro.w;
                        cbuf[7 * kWg] = rd.w;
                    }
                    n_gen++;
                    buffered = true;
                }
            }
            if (!active && buffered) {
                const double* cbuf = cam_lds + tid;
                const d4 crd = mk(cbuf[0 * kWg], cbuf[1 * kWg], cbuf[2 * kWg], A ? 0.0 : cbuf[(kCamComp - 1) * kWg]);
                d4 cro;
                if constexpr (kCamComp > 3)
                    cro = mk(cbuf[3 * kWg], cbuf[4 * kWg], cbuf[5 * kWg], A ? 1.0 : cbuf[(kCamComp - 2) * kWg]);
                else
                    {
                    const double* co = camera_ptr<(PTMI_CAM_RELOAD & 1) != 0>(S).origin;  // ray_for_pixel's origin
                    cro = mk(co[0], co[1], co[2], 1.0);
                }
                start_path<A, (FL & F_DOF) != 0>(P, cro, crd);
                acm[0 * kBlock] = 0.0;
                acm[1 * kBlock] = 0.0;
                acm[2 * kBlock] = 0.0;
                n_cur = n_gen - 1;
                if constexpr ((FL & F_XRNG) != 0) P.rng = xseed(seed_bits, n_cur);
                buffered = false;
                active = true;
            }
            PTMI_TADD(12, t_a);
#if PTMI_R6_LOOP
            // The hit lives only inside the active block (round 6): declared outside it, the
            // uninitialised Hit of inactive lanes became loop-carried registers, copied at every
            // iteration (6 v_mov_b64 per bounce).
            if (active) {
                PTMI_TSTAMP(t_b);
                PTMI_WADD(45, 1ull);
                PTMI_WADD(46, (unsigned long long)__popcll(__ballot(1)));
                Hit h;
                if (P.dead) h.pk = -1;
                else h = find_closest_prims<FL>(S, P.ro, P.rd);
                PTMI_TADD(13, t_b);
                PTMI_TSTAMP(t_d);
                if (bounce_shade<FL, true>(S, P, h, fgi, n_cur, acm)) {
                    acc[0 * kBlock] = acc[0 * kBlock] + acm[0 * kBlock];  // colors += accumColor (tracer.cl:1179)
                    acc[1 * kBlock] = acc[1 * kBlock] + acm[1 * kBlock];
                    acc[2 * kBlock] = acc[2 * kBlock] + acm[2 * kBlock];
                    active = false;
                }
                PTMI_TADD(15, t_d);
            }
#else
            PTMI_TSTAMP(t_b);
            Hit h;
            if (active) {
                if (P.dead) h.pk = -1;
                else h = find_closest_prims<FL>(S, P.ro, P.rd);
            }
            PTMI_TADD(13, t_b);
            PTMI_TSTAMP(t_d);
            if (active && bounce_shade<FL, true>(S, P, h, fgi, n_cur, acm)) {
                acc[0 * kBlock] = acc[0 * kBlock] + acm[0 * kBlock];  // colors += accumColor (tracer.cl:1179)
                acc[1 * kBlock] = acc[1 * kBlock] + acm[1 * kBlock];
                acc[2 * kBlock] = acc[2 * kBlock] + acm[2 * kBlock];
                active = false;
            }
            PTMI_TADD(15, t_d);
#endif
            PTMI_WADD(10, 1ull);
        }
        PTMI_TADD(16, t_loop);
#if PTMI_STATS
        if (PTMI_FIRST_ACTIVE())
            for (int k = 0; k < 64; k++)
                if (ptmi_wstat[0][k]) atomicAdd(&ptmi_stats[k], ptmi_wstat[0][k]);
#endif
        store_sums<true>(work_item(S, WP, blockIdx.x, lane), WP, sums, part, acc[0 * kBlock], acc[1 * kBlock],
                   acc[2 * kBlock]);  // the work item re-derived: fewer live VGPRs
#if PTMI_TIMELINE
        if (threadIdx.x == 0 && blockIdx.x < ptmi_tl_max) {
            ptmi_tl[2 * blockIdx.x] = tl0;
            ptmi_tl[2 * blockIdx.x + 1] = wall_clock64();
        }
#endif
    }
}

// scene_reload builds its pointer from the kernel-argument segment: it needs DevScene to be
// trace_kernel's FIRST parameter.  Explicit kernel arguments are laid out from offset 0 in
// declaration order (the hidden arguments follow them, AMDGPU code object v5), so this check on
// the parameter list is what keeps the reload pointing at S.
template <typename F>
struct first_param;
template <typename R, typename P0, typename... Ps>
struct first_param<R (*)(P0, Ps...)> {
    using type = P0;
};
static_assert(std::is_same<first_param<decltype(&trace_kernel<0>)>::type, DevScene>::value &&
                  std::is_same<first_param<decltype(&trace_kernel<F_ALL>)>::type, DevScene>::value,
              "scene_reload: DevScene must be trace_kernel's first parameter (kernarg offset 0)");

#if PTMI_STUDY
// ==== STUDY build only (make study -> build/libptmi_study.so) ==========================
// The standalone walk kernels and the split execution form of the mesh scenes are the
// round-4 measurements behind DESIGN.md s5; they are not part of the product library.
// ---- Standalone BVH walks (round 4) -------------------------------------------------
// The mesh kernels walk inside their bounce loop, with the whole path state live: 4
// waves/SIMD, and a walk phase runs ~24 parked lanes of 64 for as long as the longest
// walk.  These kernels walk a list of requests (WalkReq: world ray + primitive best) with
// nothing else live.  walk_kernel: one request per lane, the same group_walks code.
// walk_pool_kernel: persistent waves, one walk step (a Node4 visit or a leaf) per lane per
// iteration, and a lane whose walk ends takes the next request from a global counter, so
// the wave's lanes stay busy to the end of the list.  Same candidate set, same
// lexicographic minimum, same gate certification: the results equal group_walks'.
#ifndef PTMI_WALK_WAVES
#define PTMI_WALK_WAVES 5
#endif
template <bool A>
__global__ __launch_bounds__(kBlock, PTMI_WALK_WAVES) void walk_kernel(DevScene S, const WalkReq* __restrict__ req,
                                                                      uint32_t n, WalkRes* __restrict__ res) {
    __shared__ int stk_lds[kStack * kStkStride];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const WalkReq q = req[i];
    Hit h{q.t, q.pk, -1, -1, 0.0, 0.0};
    group_walks<A>(S, lds_ptr(stk_lds + threadIdx.x), mk(q.o[0], q.o[1], q.o[2], 1.0), mk(q.d[0], q.d[1], q.d[2], 0.0), h);
    res[i] = WalkRes{h.t, h.pk, h.tri, h.ti, 0, h.u, h.v};
}

#ifndef PTMI_WALK_REFILL
#define PTMI_WALK_REFILL 16  // lanes without a walk that trigger the wave's finish-and-refill step
#endif
template <bool A>
__global__ __launch_bounds__(kBlock, PTMI_WALK_WAVES) void walk_pool_kernel(DevScene S,
                                                                           const WalkReq* __restrict__ req,
                                                                           uint32_t n, WalkRes* __restrict__ res,
                                                                           uint32_t* __restrict__ next) {
    __shared__ int stk_lds[kStack * kStkStride];
    const int lane = threadIdx.x;
    LdsInt* stk = lds_ptr(stk_lds + lane);
    const int j_end = S.run_end[4];
    // Lane phases: kIdle (no request), kWalk (walking object j of request ri), kDone (every
    // object walked: the gate check, barycentrics and result store are pending), kDrained
    // (the list is exhausted).  Finishing and refilling run for all such lanes of the wave
    // together, once PTMI_WALK_REFILL of them wait (their FP64 work then runs on many
    // lanes), or when no lane walks.
    enum : int { kIdle = 0, kWalk = 1, kDone = 2, kDrained = 3 };
    int phase = kIdle;
    uint32_t ri = 0;
    const int lb = S.leaf_bit;
    int j = 0, cur = lb, sp = 0, vchain = -1;
    bool cert = false;
    d4 o = mk(0.0, 0.0, 0.0, 1.0), d = mk(0.0, 0.0, 0.0, 0.0);
    WalkRay W{};
    float lim = 0.0f;
    Hit h{1024.0, -1, -1, -1, 0.0, 0.0};
    // The walk of the first group object from jj on whose hull the segment [eps, best]
    // can meet; kDone when none is left.
    auto start_object = [&](int jj) {
        const WalkReq& q = req[ri];
        const d4 ro = mk(q.o[0], q.o[1], q.o[2], 1.0), rd = mk(q.d[0], q.d[1], q.d[2], 0.0);
        for (; jj < j_end; jj++) {
            const DevObject& ob = S.objs[jj];
            o = xpt<A>(ob.inv, ob.st, ro);
            d = xdir<A>(ob.inv, ob.st, rd);
            const d4 r = mk(rcp_walk(d.x), rcp_walk(d.y), rcp_walk(d.z), 0.0);
            const RootRec& R = S.root_rec[ob.child_base];  // one traversal index per group object
            double tn;
            if (cull_box(o, r, R.hull_mn[0], R.hull_mn[1], R.hull_mn[2], R.hull_mx[0], R.hull_mx[1], R.hull_mx[2],
                         h.t + prune_margin(h.t), tn))
                continue;
            W = walk_setup(o, r, R);
            lim = walk_limit(h.t);
            cur = R.entry;
            sp = 0;
            vchain = -1;
            break;
        }
        j = jj;
        phase = jj < j_end ? kWalk : kDone;
    };
    for (;;) {
        const uint64_t wait_m = __ballot(phase == kIdle || phase == kDone);
        const bool any_walk = __any(phase == kWalk);
        if (__popcll(wait_m) >= PTMI_WALK_REFILL || (wait_m != 0 && !any_walk)) {
            if (phase == kDone) {  // the gate check (group_walks), barycentrics, result
                const WalkReq& q = req[ri];
                const d4 ro = mk(q.o[0], q.o[1], q.o[2], 1.0), rd = mk(q.d[0], q.d[1], q.d[2], 0.0);
                if (h.tri >= 0 && !cert) {
                    const DevObject& ob = S.objs[hit_obj(h)];
                    if (!verify_chain(S, S.tris[h.ti].chain, xpt<A>(ob.inv, ob.st, ro), xdir<A>(ob.inv, ob.st, rd))) {
                        h = Hit{q.t, q.pk, -1, -1, 0.0, 0.0};  // the eager walks
                        group_walks_impl<A, true>(S, stk, ro, rd, h, cert);
                    }
                }
                if (h.tri >= 0) {
                    const DevObject& ob = S.objs[hit_obj(h)];
                    tri_uv(S.tris[h.ti], xpt<A>(ob.inv, ob.st, ro), xdir<A>(ob.inv, ob.st, rd), h.u, h.v);
                }
                res[ri] = WalkRes{h.t, h.pk, h.tri, h.ti, 0, h.u, h.v};
                phase = kIdle;
            }
            // refill: one atomic for the wave, each waiting lane takes the next request
            const uint64_t im = __ballot(phase == kIdle);
            const int first = __ffsll((long long)im) - 1;
            uint32_t base = 0;
            if (lane == first) base = atomicAdd(next, (uint32_t)__popcll(im));
            base = __shfl(base, first);
            if (phase == kIdle) {
                ri = base + __popcll(im & ((1ull << lane) - 1));
                if (ri < n) {
                    const WalkReq& q = req[ri];
                    h = Hit{q.t, q.pk, -1, -1, 0.0, 0.0};
                    cert = false;
                    start_object(S.run_end[3]);
                } else {
                    phase = kDrained;
                }
            }
        }
        if (!__any(phase == kWalk || phase == kDone)) break;
        if (phase == kWalk) {  // one walk step of object j (walk_index's loop body)
            bool down = false;
            if (cur < lb) {
                int nxt;
                down = node_visit(S, stk, cur, sp, W, lim, nxt);
                if (down) cur = nxt;
            } else {
                leaf_visit<false>(S, cur - lb, j, S.objs[j].key, o, d, h, vchain);
                lim = walk_limit(h.t);
            }
            if (!down) {
                if (sp > 0) {
                    cur = stk[(--sp) * kStkStride];
                } else {  // object j walked: certify a winner from it, then the next object
                    if (h.tri >= 0 && hit_obj(h) == j) cert = chain_certified(S, S.tris[h.ti].chain, o, d, h.t);
                    start_object(j + 1);
                }
            }
        }
    }
}

// ---- Split execution of mesh scenes (round 4) -------------------------------------
// The mesh kernel above keeps every path in registers and walks the BVH in wave-wide walk
// phases: ~24 parked lanes walk while the others wait, and parked lanes idle through the
// primitive and shading phases.  Measured on the walks of real frames (tools/walk_bench.py,
// profiles/r4/walk_kernel): the same walks cost 2.1x less in a standalone kernel, and the
// mesh kernel without its walks (the mesh made invisible, hull culls kept) runs C4 / C5 in
// 286 / 330 ms instead of 627 / 966 ms.  The split form runs those two halves as separate
// kernels over a pool of path slots in HBM (SplitBufs), pass by pass:
//   trace_split_kernel: each wave owns B.per_wave slots and hands them to its lanes; a lane
//     resumes a slot's path (applying the walk result of the previous pass), traces it --
//     primitives, hull culls, shading, its next samples -- until its ray needs a walk, then
//     saves the path and the primitive best, appends the slot to the request list and takes
//     the wave's next slot.  A slot whose pixel-chunk is finished claims the next one.
//   walk_split_kernel: group_walks for every request of the pass (the same code as the mesh
//     kernel's walk phases), result to the slot.
// Per slot the samples of a pixel-chunk run in order with the reference's arithmetic, and
// chunk sums go to the same partial records as the mesh kernel's chunk items, so the frame
// equals a mesh-kernel render with the same chunk length bit for bit.
#ifndef PTMI_WAVES_SPLIT
#define PTMI_WAVES_SPLIT 4  // (round 5: 5 waves spilled 208 B/lane, the tracer pass then waited on memory 82 % of
                            // its cycles; 4: 64 B/lane, C4 split frame 2444 -> 1511 ms, profiles/r5/split)
#endif
#ifndef PTMI_SPLIT_BATCH
#define PTMI_SPLIT_BATCH 16  // waiting lanes that trigger a batched slot / claim / camera step
#endif
// A slot yields after starting B.budget samples in one pass (saved at a sample boundary,
// resumed by the next pass): every wave then does about the same work per pass, so a pass
// is not as long as its luckiest wave's run of walk-free samples.
static constexpr uint32_t kFlagYield = 1u << 9;  // path flags: saved at a sample boundary, no walk pending
// Pixel-chunks are claimed by the wave in blocks of one tile-chunk (64 consecutive ids, the
// 64 pixels of one tile for one sample chunk), one global atomic per block.  (One atomic
// per claim, and one per batch of walk requests, on shared counters had left the split
// kernel's waves waiting on the atomic unit most of the pass.)
static constexpr uint32_t kClaimBlock = 64;
template <int FL>
__global__ __launch_bounds__(kBlock, PTMI_WAVES_SPLIT) void trace_split_kernel(DevScene S, uint32_t samples,
                                                                              WorkPlan WP, SplitBufs B,
                                                                              const double* __restrict__ seeds,
                                                                              const double* __restrict__ sunf,
                                                                              double* __restrict__ part) {
    static_assert((FL & F_GROUPS) && !(FL & (F_PROJ | F_TEX | F_XRNG)), "affine parity mesh scenes");
    constexpr bool A = true;
    constexpr bool kDof = (FL & F_DOF) != 0;
    __shared__ double acc_lds[3 * kBlock];
    const int lane = threadIdx.x;
    double* acc = acc_lds + lane;
    // The wave's next slot to hand out: wave-uniform, so every lane keeps its own copy and
    // advances it by the same ballot count (a counter in LDS written by one lane and read
    // by others without synchronisation had let lanes see stale values).
    uint32_t next_slot = 0;
    // Wave-uniform counters, kept identical in every lane: the claimed block of
    // pixel-chunks [cl_next, cl_end), this pass's walk requests and yields.
    uint32_t cl_next = B.wcl[2 * blockIdx.x], cl_end = B.wcl[2 * blockIdx.x + 1], n_req = 0, n_yield = 0;
    bool claims_done = false;
    const uint32_t L = B.L;
    const uint32_t base = blockIdx.x * B.per_wave;
    const uint32_t end = min(base + B.per_wave, L);
    const int W = S.cam.width, H = S.cam.height;
    const int tiles_x = (W + kTile - 1) / kTile, tiles_y = (H + kTile - 1) / kTile;
    const uint32_t n_tiles = max(WP.n_tail, 1u);
    enum : int { kNoSlot = 0, kClaim = 1, kNeedCam = 2, kTrace = 3, kReady = 4, kExhausted = 5 };
    int mode = kNoSlot;
    uint32_t slot = 0, q = 0, n_cur = 0, c_end = 0, spent = 0;
    int px = 0, py = 0;
    float fgi = 0.0f;
    PathState P;
    start_path<A, kDof>(P, mk(0.0, 0.0, 0.0, 1.0), mk(0.0, 0.0, 0.0, 0.0));
    Hit h{1024.0, -1, -1, -1, 0.0, 0.0};
    // Pixel-chunk q -> pixel and sample range; false for a pixel outside the image.
    auto decode = [&](uint32_t qq, uint32_t& c0) -> bool {
        const uint32_t l = qq & 63u, tc = qq >> 6, c = tc / n_tiles, tk = tc - c * n_tiles;
        const uint32_t tile = WP.tile_offset + tk * WP.tile_stride;
        px = (int)(tile % (uint32_t)tiles_x) * kTile + (int)(l & 7u);
        py = (int)(tile / (uint32_t)tiles_x) * kTile + (int)(l >> 3);
        c0 = WP.s_begin + c * WP.chunk_len;
        c_end = min(WP.s_end, c0 + WP.chunk_len);
        return tile < (uint32_t)(tiles_x * tiles_y) && px < W && py < H;
    };
    auto R = [&]() -> SplitRec& { return reinterpret_cast<SplitRec*>(B.rec)[slot]; };
    auto dget = [&](int k) -> double& { return R().d[k]; };
    auto uget = [&](int k) -> uint32_t& { return R().u[k]; };
    for (;;) {
        const bool tr = mode == kTrace || mode == kReady;
        // A. Lanes without a slot take the wave's next ones (batched).
        {
            const uint64_t m = __ballot(mode == kNoSlot);
            if (m && (__popcll(m) >= PTMI_SPLIT_BATCH || !__any(tr || mode == kNeedCam || mode == kClaim))) {
                const uint32_t b0 = next_slot;
                next_slot += (uint32_t)__popcll(m);
                if (mode == kNoSlot) {
                    const uint32_t k = base + b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1));
                    if (k >= end) {
                        mode = kExhausted;
                    } else {
                        slot = k;
                        const uint32_t it = uget(0);
                        if (it == kSlotFree) {
                            spent = 0;
                            mode = kClaim;
                        } else if (it != kSlotDead && (uget(2) & kFlagYield)) {  // yielded between samples
                            q = it;
                            uint32_t c0;
                            decode(q, c0);
                            n_cur = uget(1);
                            acc[0 * kBlock] = dget(12), acc[1 * kBlock] = dget(13), acc[2 * kBlock] = dget(14);
                            fgi = R().f[0];
                            spent = 0;
                            mode = kNeedCam;
                        } else if (it != kSlotDead) {  // a path waiting for its walk result: resume it
                            q = it;
                            spent = 0;
                            uint32_t c0;
                            decode(q, c0);
                            n_cur = uget(1);
                            const uint32_t fl = uget(2);
                            P.ro = mk(dget(0), dget(1), dget(2), 1.0);
                            P.rd = mk(dget(3), dget(4), dget(5), 0.0);
                            P.mr = dget(6), P.mg = dget(7), P.mb = dget(8);
                            P.ar = dget(9), P.ag = dget(10), P.ab = dget(11);
                            acc[0 * kBlock] = dget(12), acc[1 * kBlock] = dget(13), acc[2 * kBlock] = dget(14);
                            P.b = fl & 15u, P.effective = (fl >> 4) & 7u;
                            P.inside = (fl >> 7) & 1u, P.done = (fl >> 8) & 1u, P.dead = false;
                            fgi = R().f[0];
                            const WalkRes r = R().res;
                            h = Hit{r.t, r.pk, r.tri, r.ti, r.u, r.v};
                            mode = kReady;
                        }
                    }
                }
            }
        }
        // B. Slots without a pixel-chunk claim the next ones (batched, one atomic).
        {
            const uint64_t m = __ballot(mode == kClaim);
            if (m && (__popcll(m) >= PTMI_SPLIT_BATCH || !__any(tr || mode == kNeedCam))) {
                if (cl_next >= cl_end && !claims_done) {  // the wave's next block (one atomic)
                    const int first = __ffsll((long long)m) - 1;
                    uint32_t b0 = 0;
                    if (lane == first) b0 = atomicAdd(&B.cnt[1], kClaimBlock);
                    b0 = __shfl(b0, first);
                    cl_next = b0;
                    cl_end = min(b0 + kClaimBlock, B.n_items);
                    claims_done = b0 >= B.n_items;
                }
                const uint32_t avail = cl_next < cl_end ? cl_end - cl_next : 0u;
                const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1));
                cl_next += min(avail, (uint32_t)__popcll(m));
                if (mode == kClaim && rank >= avail) {
                    if (claims_done) {  // every pixel-chunk is claimed: the slot is done for good
                        uget(0) = kSlotDead;
                        mode = kNoSlot;
                    }  // else: claims again from the wave's next block
                } else if (mode == kClaim) {
                    const uint32_t qq = cl_next - min(avail, (uint32_t)__popcll(m)) + rank;
                    {
                        q = qq;
                        uint32_t c0;
                        if (!decode(q, c0)) {
                            mode = kClaim;  // outside the image: nothing to render, claim again
                        } else {
                            uget(0) = q;
                            n_cur = c0;
                            acc[0 * kBlock] = 0.0, acc[1 * kBlock] = 0.0, acc[2 * kBlock] = 0.0;
                            const double seed = seeds[(uint32_t)py * (uint32_t)W + (uint32_t)px];
                            fgi = (float)(seed / (double)S.n_list);  // tracer.cl:840
                            R().f[0] = fgi;
                            R().f[1] = (float)(seed / (double)samples);  // fgi2, tracer.cl:841
                            if (n_cur < c_end) {
                                mode = kNeedCam;
                            } else {  // an empty chunk (the range ends before it)
                                double* o = part + (size_t)q * 4;
                                o[0] = 0.0, o[1] = 0.0, o[2] = 0.0, o[3] = 0.0;
                                uget(0) = kSlotFree;
                                mode = kClaim;
                            }
                        }
                    }
                }
            }
        }
        // C. Camera rays for the lanes starting a sample (batched: the camera block runs for
        //    many lanes at once, as in the mesh kernel's refills).
        {
            const int n_cam = __popcll(__ballot(mode == kNeedCam));
            if (n_cam && (n_cam >= PTMI_SPLIT_BATCH || !__any(tr))) {
                n_yield += (uint32_t)__popcll(__ballot(mode == kNeedCam && spent >= B.budget));
                if (mode == kNeedCam && spent >= B.budget) {  // yield: the next pass goes on from n_cur
                    uget(1) = n_cur;
                    uget(2) = kFlagYield;
                    dget(12) = acc[0 * kBlock], dget(13) = acc[1 * kBlock], dget(14) = acc[2 * kBlock];
                    mode = kNoSlot;
                }
                if (mode == kNeedCam) {
                    spent++;
                    const float fgi2 = R().f[1];
                    float rx, ry;
                    camera_offsets<FL>(fgi, fgi2, XSeed{}, n_cur, rx, ry);  // (parity mode only: no key)
                    d4 ro, rd;
                    ray_for_pixel<kDof, A>(camera_ptr(S), sunf, (unsigned)px, (unsigned)py, rx, ry, (int)n_cur, ro, rd);
                    start_path<A, kDof>(P, ro, rd);
                    mode = kTrace;
                }
            }
        }
        if (!__any(mode != kExhausted)) {
            if (lane == 0) {
                B.wcl[2 * blockIdx.x] = cl_next;
                B.wcl[2 * blockIdx.x + 1] = cl_end;
                B.seg[blockIdx.x] = n_req;
                if (n_req) {
                    atomicAdd(&B.cnt[0], n_req);
                    atomicAdd(&B.cnt[3], n_req);  // all passes (diagnostics)
                }
                if (n_yield) atomicAdd(&B.cnt[2], n_yield);
            }
            break;
        }
        // D. Closest primitive; a ray whose segment can meet a mesh hull saves its path and
        //    asks for a walk.
        bool walk = false;
        if (mode == kTrace) {
            if (P.dead) {
                h.pk = -1;
                mode = kReady;
            } else {
                h = find_closest_prims<FL>(S, P.ro, P.rd);
                if (group_needs_walk<A>(S, P.ro, P.rd, h)) {
                    dget(0) = P.ro.x, dget(1) = P.ro.y, dget(2) = P.ro.z;
                    dget(3) = P.rd.x, dget(4) = P.rd.y, dget(5) = P.rd.z;
                    dget(6) = P.mr, dget(7) = P.mg, dget(8) = P.mb;
                    dget(9) = P.ar, dget(10) = P.ag, dget(11) = P.ab;
                    dget(12) = acc[0 * kBlock], dget(13) = acc[1 * kBlock], dget(14) = acc[2 * kBlock];
                    dget(15) = h.t;
                    uget(1) = n_cur;
                    uget(2) = P.b | (P.effective << 4) | ((P.inside ? 1u : 0u) << 7) | ((P.done ? 1u : 0u) << 8);
                    uget(3) = (uint32_t)h.pk;
                    walk = true;
                    mode = kNoSlot;
                } else {
                    mode = kReady;
                }
            }
        }
        {  // the walk requests of this step, appended to the wave's own segment
            const uint64_t wm = __ballot(walk);
            if (walk) B.req[base + n_req + (uint32_t)__popcll(wm & ((1ull << lane) - 1))] = slot;
            n_req += (uint32_t)__popcll(wm);
        }
        // E. Shading (tracer.cl:886-1110); a finished path adds to the pixel-chunk's sums
        //    (tracer.cl:1179), a finished chunk writes its record (r, g, b, samples).
        if (mode == kReady) {
            if (bounce_shade<FL>(S, P, h, fgi, n_cur)) {
                acc[0 * kBlock] = acc[0 * kBlock] + P.ar;
                acc[1 * kBlock] = acc[1 * kBlock] + P.ag;
                acc[2 * kBlock] = acc[2 * kBlock] + P.ab;
                n_cur++;
                if (n_cur < c_end) {
                    mode = kNeedCam;
                } else {
                    uint32_t c0;
                    decode(q, c0);
                    double* o = part + (size_t)q * 4;
                    o[0] = acc[0 * kBlock], o[1] = acc[1 * kBlock], o[2] = acc[2 * kBlock];
                    o[3] = (double)(c_end - c0);
                    uget(0) = kSlotFree;
                    mode = kClaim;
                }
            } else {
                mode = kTrace;
            }
        }
    }
}

// The walks of one split pass: every request appended by trace_split_kernel.
__global__ __launch_bounds__(kBlock, PTMI_WALK_WAVES) void walk_split_kernel(DevScene S, SplitBufs B) {
    __shared__ int stk_lds[kStack * kStkStride];
    LdsInt* stk = lds_ptr(stk_lds + threadIdx.x);
    const uint32_t nseg = (B.L + B.per_wave - 1) / B.per_wave;
    for (uint32_t w = blockIdx.x; w < nseg; w += gridDim.x)  // tracer wave w's segment
        for (uint32_t i = threadIdx.x, n = B.seg[w]; i - threadIdx.x < n; i += kBlock) {
            if (i >= n) continue;
            const uint32_t slot = B.req[(size_t)w * B.per_wave + i];
            SplitRec& Rs = reinterpret_cast<SplitRec*>(B.rec)[slot];
            const double* d = Rs.d;
            Hit h{d[15], (int)Rs.u[3], -1, -1, 0.0, 0.0};
            group_walks<true>(S, stk, mk(d[0], d[1], d[2], 1.0), mk(d[3], d[4], d[5], 0.0), h);
            Rs.res = WalkRes{h.t, h.pk, h.tri, h.ti, 0, h.u, h.v};
        }
}

bool split_supported(int flags) {
    return (flags & F_GROUPS) && !(flags & (F_PROJ | F_TEX | F_XRNG | F_WIDE));
}

const void* trace_split_symbol(int flags) {
    switch (flags & F_ALL) {
#define K(f) \
    case f: return reinterpret_cast<const void*>(&trace_split_kernel<f>);
        K(1) K(3) K(5) K(7) K(9) K(11) K(13) K(15)
#undef K
    }
    return nullptr;
}
const void* walk_split_symbol() { return reinterpret_cast<const void*>(&walk_split_kernel); }

hipError_t launch_split_pass(const DevScene& S, int flags, uint32_t samples, const WorkPlan& WP, const SplitBufs& B,
                             const double* seeds, const double* sunf, double* part, uint32_t walk_grid,
                             hipStream_t st) {
    if (!split_supported(flags)) return hipErrorInvalidValue;
    const dim3 grid((B.L + B.per_wave - 1) / B.per_wave), block(kBlock);
    switch (flags & F_ALL) {
#define K(f)                                                                                                   \
    case f:                                                                                                    \
        hipLaunchKernelGGL(trace_split_kernel<f>, grid, block, 0, st, S, samples, WP, B, seeds, sunf, part); \
        break;
        K(1) K(3) K(5) K(7) K(9) K(11) K(13) K(15)
#undef K
    default:
        return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(walk_split_kernel, dim3(walk_grid), block, 0, st, S, B);
    return hipGetLastError();
}

hipError_t launch_walk(const DevScene& S, int flags, int mode, const WalkReq* req, uint32_t n, WalkRes* res,
                       uint32_t* next, uint32_t grid, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if ((flags & (F_PROJ | F_TEX | F_WIDE)) || !(flags & F_GROUPS)) return hipErrorInvalidValue;  // affine narrow-code mesh scenes
    if (mode == 0) {
        hipLaunchKernelGGL(walk_kernel<true>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, S, req, n, res);
    } else {
        hipLaunchKernelGGL(walk_pool_kernel<true>, dim3(grid), dim3(kBlock), 0, st, S, req, n, res, next);
    }
    return hipGetLastError();
}

const void* walk_kernel_symbol(int mode) {
    return mode == 0 ? reinterpret_cast<const void*>(&walk_kernel<true>)
                     : reinterpret_cast<const void*>(&walk_pool_kernel<true>);
}
#endif  // PTMI_STUDY

#if PTMI_CAPTURE
hipError_t capture_setup(WalkReq* req, WalkRes* res, uint32_t cap) {
    unsigned z = 0;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_cap_req), &req, sizeof(req));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_cap_res), &res, sizeof(res));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_cap_max), &cap, sizeof(cap));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_cap_n), &z, sizeof(z));
    return e;
}
hipError_t capture_count(uint32_t* n) { return hipMemcpyFromSymbol(n, HIP_SYMBOL(ptmi_cap_n), sizeof(*n)); }
#else
hipError_t capture_setup(WalkReq*, WalkRes*, uint32_t) { return hipErrorNotSupported; }
hipError_t capture_count(uint32_t*) { return hipErrorNotSupported; }
#endif
#if PTMI_TIMELINE
hipError_t timeline_setup(unsigned long long* buf, uint32_t cap) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_tl), &buf, sizeof(buf));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(ptmi_tl_max), &cap, sizeof(cap));
    return e;
}
#else
hipError_t timeline_setup(unsigned long long*, uint32_t) { return hipErrorNotSupported; }
#endif

// DoF aperture offsets sunflower(S, 2, n) for n in [0, S) (tracer.cl:221-248,
// 766): a per-frame table, same arithmetic as the reference.
__global__ void sunflower_kernel(double* __restrict__ out, uint32_t samples) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= samples) return;
    double sx, sy;
    sunflower((int)samples, (int)n, sx, sy);
    out[2 * n] = sx;
    out[2 * n + 1] = sy;
}

hipError_t launch_sunflower(double* out, uint32_t samples, hipStream_t st) {
    hipLaunchKernelGGL(sunflower_kernel, dim3((samples + 255) / 256), dim3(256), 0, st, out, samples);
    return hipGetLastError();
}

// Per-plane constant world normal: the exact arithmetic of tracer.cl:913, 953-955
// for objectNormal = (0,1,0,0), done once per scene with the kernel's own math.
__global__ void plane_normals_kernel(DevObject* objs, int n) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || objs[j].type != 0) return;
    d4 nv = mat_mul(objs[j].inv_t, mk(0.0, 1.0, 0.0, 0.0));
    nv.w = 0.0;
    nv = normalize4(nv);
    objs[j].plane_n[0] = nv.x;
    objs[j].plane_n[1] = nv.y;
    objs[j].plane_n[2] = nv.z;
    objs[j].plane_n[3] = nv.w;
}

hipError_t launch_hemi_table(double* out, int* mismatch, hipStream_t st) {
    hipLaunchKernelGGL(hemi_table_kernel, dim3(kHemiSize / 256), dim3(256), 0, st, out, mismatch);
    return hipGetLastError();
}

hipError_t launch_plane_normals(DevObject* objs, int n, hipStream_t st) {
    hipLaunchKernelGGL(plane_normals_kernel, dim3(1), dim3(64), 0, st, objs, n);
    return hipGetLastError();
}

// The tail tiles' chunk partials (WorkPlan) summed in chunk order (deterministic)
// into the frame; one thread per tail-tile pixel.
__global__ __launch_bounds__(256) void reduce_chunks_kernel(const double* __restrict__ part, double* __restrict__ sums,
                                                            WorkPlan WP, int W, int H, bool planes) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= WP.n_tail * 64) return;
    const uint32_t tt = j >> 6, lane = j & 63;
    const int tiles_x = (W + kTile - 1) / kTile;
    const uint32_t k = WP.n_whole + tt;
    const uint32_t tile = WP.tiles ? WP.tiles[k] : WP.tile_offset + k * WP.tile_stride;
    const int px = (int)(tile % (uint32_t)tiles_x) * kTile + (int)(lane & 7);
    const int py = (int)(tile / (uint32_t)tiles_x) * kTile + (int)(lane >> 3);
    if (px >= W || py >= H) return;
    double r = 0.0, g = 0.0, b = 0.0, a = 0.0;
    for (uint32_t c = 0; c < WP.nchunks; c++) {
        if (planes) {
            const size_t plane = (size_t)WP.nchunks * WP.n_tail * 64;
            const double* p = part + (size_t)c * WP.n_tail * 64 + j;  // store_sums' planes
            r = r + p[0];
            g = g + p[plane];
            b = b + p[2 * plane];
            uint32_t c0, c1;
            chunk_range(WP, c, c0, c1);
            a = a + (double)(c1 > c0 ? c1 - c0 : 0);  // the chunk item's sample count (work_item)
        } else {
            const double* p = part + ((size_t)c * WP.n_tail * 64 + j) * 4;  // records
            r = r + p[0];
            g = g + p[1];
            b = b + p[2];
            a = a + p[3];
        }
    }
    double* o = sums + ((size_t)py * W + px) * 4;
    o[0] = r;
    o[1] = g;
    o[2] = b;
    o[3] = a;
}

// colors * (1.0 / samples), alpha 1 (tracer.cl:837, 1184-1187).
__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ sums, double* __restrict__ out,
                                                       uint32_t npix, uint32_t samples) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const double w = 1.0 / samples;
    out[4 * (size_t)i + 0] = sums[4 * (size_t)i + 0] * w;
    out[4 * (size_t)i + 1] = sums[4 * (size_t)i + 1] * w;
    out[4 * (size_t)i + 2] = sums[4 * (size_t)i + 2] * w;
    out[4 * (size_t)i + 3] = 1.0;
}

// ptmi_trace_multi's device-side combine: out = the partial frames parts[0..nparts)
// (each npix*4 doubles, RGB sums, A = sample count) summed in part order, times 1/S,
// alpha 1 (tracer.cl:1184-1187).  out may alias parts[0].
__global__ __launch_bounds__(256) void combine_kernel(const double* parts, uint32_t nparts, size_t npix,
                                                      double* out, uint32_t samples) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const size_t stride = npix * 4;
    double r = parts[4 * i], g = parts[4 * i + 1], b = parts[4 * i + 2];
    for (uint32_t k = 1; k < nparts; k++) {
        const double* p = parts + k * stride + 4 * i;
        r = r + p[0];
        g = g + p[1];
        b = b + p[2];
    }
    const double w = 1.0 / samples;
    out[4 * i + 0] = r * w;
    out[4 * i + 1] = g * w;
    out[4 * i + 2] = b * w;
    out[4 * i + 3] = 1.0;
}

// Seeds with Go rand.Float64 granularity (k / 2^53) from a SplitMix64 stream.
__global__ __launch_bounds__(256) void seeds_kernel(double* __restrict__ seeds, uint32_t n, uint64_t stream) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = stream + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    seeds[i] = (double)(z >> 11) * 0x1p-53;
}

// ---- host-side launch wrappers (called from ptmi_api.cpp) ----------------------
int trace_block_threads(int flags) { return kBlock; }
int trace_tiles_per_block(int flags) { return 1; }

// The instantiation a scene's flags launch: textured and non-affine scenes take the
// generic ones; F_XRNG exists for the affine instantiations (ptmi_scene_set_rng).
static int kernel_flags(int flags) {
    if (flags & F_TEX) return F_ALL | F_PROJ | F_TEX;
    if (flags & F_PROJ) return F_ALL | F_PROJ;
    if (flags & F_WIDE) return F_ALL | F_WIDE | (flags & F_XRNG);
    if ((flags & F_TLIST) && (flags & F_GROUPS) && !(flags & F_XRNG)) return flags & (F_ALL | F_TLIST);
    return flags & (F_ALL | F_XRNG);
}

int trace_kernel_flags(int flags) { return kernel_flags(flags); }

// Whether a launch with these scene flags can take an owned-tile list (ptmi_api.cpp render).
bool tile_list_supported(int flags) {
    return (flags & F_GROUPS) && !(flags & (F_PROJ | F_TEX | F_XRNG | F_WIDE));
}

const void* trace_kernel_symbol(int flags) {
    switch (kernel_flags(flags)) {
#define K(f) \
    case f: return reinterpret_cast<const void*>(&trace_kernel<f>);
        K(0) K(1) K(2) K(3) K(4) K(5) K(6) K(7) K(8) K(9) K(10) K(11) K(12) K(13) K(14) K(15)
        K(F_ALL | F_PROJ) K(F_ALL | F_PROJ | F_TEX)
        K(64) K(65) K(66) K(67) K(68) K(69) K(70) K(71) K(72) K(73) K(74) K(75) K(76) K(77) K(78) K(79)
        K(129) K(131) K(133) K(135) K(137) K(139) K(141) K(143)
        K(F_ALL | F_WIDE) K(F_ALL | F_WIDE | F_XRNG)
#undef K
    }
    return nullptr;
}

hipError_t launch_trace(const DevScene& S, int flags, uint32_t samples, const WorkPlan& WP, const double* seeds,
                        const double* sunf, double* sums, double* part, uint32_t* item_ctr, hipStream_t st) {
    const uint32_t items = WP.n_whole + WP.n_tail * WP.nchunks;
    if (items == 0) return hipSuccess;
    flags = kernel_flags(flags);
    const int threads = trace_block_threads(flags), wpb = trace_tiles_per_block(flags);
    const dim3 grid((items + wpb - 1) / wpb), block(threads);
    switch (flags) {
#define K(f)                                                                                          \
    case f:                                                                                           \
        hipLaunchKernelGGL(trace_kernel<f>, grid, block, 0, st, S, samples, WP, seeds, sunf, sums, part, item_ctr); \
        break;
        K(0) K(1) K(2) K(3) K(4) K(5) K(6) K(7) K(8) K(9) K(10) K(11) K(12) K(13) K(14) K(15)
        K(F_ALL | F_PROJ) K(F_ALL | F_PROJ | F_TEX)
        K(64) K(65) K(66) K(67) K(68) K(69) K(70) K(71) K(72) K(73) K(74) K(75) K(76) K(77) K(78) K(79)
        K(129) K(131) K(133) K(135) K(137) K(139) K(141) K(143)
        K(F_ALL | F_WIDE) K(F_ALL | F_WIDE | F_XRNG)
#undef K
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_reduce(const double* part, double* sums, const WorkPlan& WP, int W, int H, bool planes,
                         hipStream_t st) {
    if (WP.n_tail == 0) return hipSuccess;
    hipLaunchKernelGGL(reduce_chunks_kernel, dim3((WP.n_tail * 64 + 255) / 256), dim3(256), 0, st, part, sums, WP, W,
                       H, planes);
    return hipGetLastError();
}

#if PTMI_STUDY  // the measured tile order (needs PTMI_TILE_COST)
// The next launch's dispatch order (WorkPlan::order) from the durations the last launch
// measured (WorkPlan::cost): within the whole tiles and within the chunked tiles
// separately, costliest first in 64 half-octave classes, any order within a class (the
// order never changes a result); then the owned tiles' accumulators are cleared.  One
// workgroup; a few microseconds.
__global__ __launch_bounds__(1024) void tile_order_kernel(unsigned long long* __restrict__ cost, uint32_t n_whole,
                                                           uint32_t n_tail, uint32_t stride, uint32_t offset,
                                                           uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[2][64];
    const uint32_t t = threadIdx.x, n = n_whole + n_tail;
    if (t < 128) hist[t >> 6][t & 63] = 0;
    __syncthreads();
    auto cls = [&](uint32_t p) {
        const unsigned long long c = cost[offset + p * stride];
        const int l2 = 63 - __clzll(c | 1ull);              // floor(log2 c)
        const int half = (c >> (l2 > 0 ? l2 - 1 : 0)) & 1;  // next bit: half octaves
        return 63 - min(63, 2 * l2 + half);                 // costliest -> class 0
    };
    for (uint32_t p = t; p < n; p += blockDim.x) atomicAdd(&hist[p < n_whole ? 0 : 1][cls(p)], 1u);
    __syncthreads();
    if (t < 2) {
        uint32_t run = t == 0 ? 0u : n_whole;
        for (int b = 0; b < 64; b++) {
            const uint32_t h = hist[t][b];
            hist[t][b] = run;
            run += h;
        }
    }
    __syncthreads();
    for (uint32_t p = t; p < n; p += blockDim.x) {
        const bool w = p < n_whole;
        order[atomicAdd(&hist[w ? 0 : 1][cls(p)], 1u)] = w ? p : p - n_whole;
    }
    __syncthreads();
    for (uint32_t p = t; p < n; p += blockDim.x) cost[offset + p * stride] = 0ull;
}

hipError_t launch_tile_order(unsigned long long* cost, uint32_t n_whole, uint32_t n_tail, uint32_t stride,
                             uint32_t offset, uint32_t* order, hipStream_t st) {
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, st, cost, n_whole, n_tail, stride, offset, order);
    return hipGetLastError();
}
#endif  // PTMI_STUDY

hipError_t launch_finalize(const double* sums, double* out, uint32_t npix, uint32_t samples, hipStream_t st) {
    hipLaunchKernelGGL(finalize_kernel, dim3((npix + 255) / 256), dim3(256), 0, st, sums, out, npix, samples);
    return hipGetLastError();
}

hipError_t launch_combine(const double* parts, uint32_t nparts, size_t npix, double* out, uint32_t samples,
                          hipStream_t st) {
    hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, parts, nparts, npix, out,
                       samples);
    return hipGetLastError();
}

hipError_t launch_seeds(double* seeds, uint32_t n, uint64_t stream, hipStream_t st) {
    hipLaunchKernelGGL(seeds_kernel, dim3((n + 255) / 256), dim3(256), 0, st, seeds, n, stream);
    return hipGetLastError();
}

}  // namespace ptmi

#if PTMI_STATS
namespace ptmi {
int stats_read(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ptmi_stats), sizeof(unsigned long long) * 80) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[80] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ptmi_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
}  // namespace ptmi
#endif
