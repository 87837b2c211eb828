// sinf_probe.hip -- TEST INFRASTRUCTURE: checks, on the GPU, that the oracle's
// C restatement of ROCm ocml's sin_f32 (oracle/ocml_sinf.h) is bit-identical to
// the device library for EVERY float, and dumps ocml results for a vector set
// the CPU tests replay.  Built by __graft_entry__.build() into tests/gpu_probe/.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#define PT_FN __host__ __device__ static inline
#include "../../oracle/ocml_sinf.h"
#include "../../pathtracer-ocl_amd/csrc/ptmi_sinf.h"  // the product's noise sin (kernel code)
#include "../../pathtracer-ocl_amd/csrc/ptmi_fp64core.h"  // the product's divide / sqrt / rsqrt cores

__global__ void sinf_check(uint64_t base, uint64_t count, unsigned long long* mism, unsigned int* first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t bits = (uint32_t)(base + i);
    float x = pto_bits2f(bits);
    float a = sinf(x);
    float b = pto_sinf(x);
    bool same = (pto_f2bits(a) == pto_f2bits(b)) || (a != a && b != b);
    float fa = a * 43758.5453f;
    float ra = fminf(fa - floorf(fa), 0x1.fffffep-1f);
    float rb = pto_fractf(fa);
    same = same && ((pto_f2bits(ra) == pto_f2bits(rb)) || (fa != fa) || isinf(fa));
    if (!same) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

// The kernel's sin for |x| < 2^19 (ptmi_sinf.h) against the device library.
__global__ void ptmi_sinf_check(uint64_t base, uint64_t count, unsigned long long* mism, unsigned int* first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = (uint32_t)(base + i);
    const float x = pto_bits2f(bits);
    if (!(fabsf(x) < 0x1p19f)) return;
    if (pto_f2bits(sinf(x)) != pto_f2bits(ptmi::sinf_lt19(x))) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

// The kernel's complete noise sin (ptmi_sinf.h noise_sinf: sinf_lt19 below 2^19,
// sinf_cw30 up to 2^30 with ocml's own sin where it declines, ocml above) against the
// device library, for every float; fb counts the [2^19, 2^30) lanes cw30 declines.
__global__ void ptmi_noise_sinf_check(uint64_t base, uint64_t count, unsigned long long* mism, unsigned int* first,
                                      unsigned long long* fb) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = (uint32_t)(base + i);
    const float x = pto_bits2f(bits);
    const float ax = fabsf(x);
    if (ax >= 0x1p19f && ax < 0x1p30f) {
        float t;
        if (!ptmi::sinf_cw30(x, t)) atomicAdd(fb, 1ull);
    }
    const float a = sinf(x);
    const float b = ptmi::noise_sinf(x, [](float v) { return sinf(v); });
    if (pto_f2bits(a) != pto_f2bits(b) && !(a != a && b != b)) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

// Random doubles with a uniform exponent in [emin, emax], random mantissa and sign.
__device__ static inline uint64_t splitmix(uint64_t& z) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t r = z;
    r = (r ^ (r >> 30)) * 0xBF58476D1CE4E5B9ull;
    r = (r ^ (r >> 27)) * 0x94D049BB133111EBull;
    return r ^ (r >> 31);
}
__device__ static inline double rand_double(uint64_t& z, int emin, int emax, bool sign) {
    const uint64_t u = splitmix(z);
    const int e = emin + (int)(splitmix(z) % (uint64_t)(emax - emin + 1));
    const uint64_t bits = ((uint64_t)(e + 1023) << 52) | (u & 0xFFFFFFFFFFFFFull) | (sign ? (u & (1ull << 63)) : 0ull);
    return __longlong_as_double((long long)bits);
}
// ptmi::div_core / sqrt_core / rsqrt_core against the compiler's operators on the
// ranges the kernel relies on: quotients of operands in [2^-500, 2^500]; sqrt of
// [2^-767, 2^1023]; rsqrt of normal [2^-1022, 2^1023].  mism[k] counts op k.
__global__ void fp64core_check(uint64_t seed, uint64_t per_thread, unsigned long long* mism) {
    uint64_t z = seed ^ ((uint64_t)(blockIdx.x * blockDim.x + threadIdx.x) * 0xD1B54A32D192ED03ull);
    unsigned long long m0 = 0, m1 = 0, m2 = 0;
    for (uint64_t k = 0; k < per_thread; k++) {
        const double x = rand_double(z, -500, 500, true), y = rand_double(z, -500, 500, true);
        const double q0 = x / y, q1 = ptmi::div_core(x, y);
        m0 += __double_as_longlong(q0) != __double_as_longlong(q1);
        const double s = rand_double(z, -767, 1022, false);
        const double s0 = sqrt(s), s1 = ptmi::sqrt_core(s);
        m1 += __double_as_longlong(s0) != __double_as_longlong(s1);
        const double r = rand_double(z, -1022, 1022, false);
        const double r0 = rsqrt(r), r1 = ptmi::rsqrt_core(r);
        m2 += __double_as_longlong(r0) != __double_as_longlong(r1);
    }
    if (m0) atomicAdd(&mism[0], m0);
    if (m1) atomicAdd(&mism[1], m1);
    if (m2) atomicAdd(&mism[2], m2);
}

// ptmi::sincos_core (both constant sources) against ocml's sincos for the hemisphere angle of every noise
// value: rand1 = 2 * (double)3.14159265359f * (double)v for each float v in [0, 1)
// (tracer.cl:349, as ptmi_kernels.hip random_hemisphere computes it).
__global__ void sincos_check(unsigned long long* mism, unsigned int* first) {
    const uint32_t bits = blockIdx.x * blockDim.x + threadIdx.x;
    if (bits >= 0x3F800000u) return;
    const double kpi = (double)3.14159265359f;
    const double x = 2.0 * kpi * (double)pto_bits2f(bits);
    double s0, c0, s1, c1, s2, c2;
    sincos(x, &s0, &c0);
    ptmi::sincos_core(x, &s1, &c1);
    ptmi::sincos_core<true>(x, &s2, &c2);  // constants from the __constant__ table (group kernels)
    if (__double_as_longlong(s0) != __double_as_longlong(s1) || __double_as_longlong(c0) != __double_as_longlong(c1) ||
        __double_as_longlong(s0) != __double_as_longlong(s2) || __double_as_longlong(c0) != __double_as_longlong(c2)) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

__global__ void sinf_eval(const float* in, float* out, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = sinf(in[i]);
}

extern "C" int probe_sinf_all(unsigned long long* mismatches, unsigned int* first_bad) {
    unsigned long long* dm;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(sinf_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, chunk, dm, df);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    return 0;
}

extern "C" int probe_ptmi_sinf_all(unsigned long long* mismatches, unsigned int* first_bad) {
    unsigned long long* dm;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(ptmi_sinf_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, chunk, dm, df);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    return 0;
}

extern "C" int probe_fp64core(uint64_t seed, uint64_t total, unsigned long long* mismatches3) {
    unsigned long long* dm;
    if (hipMalloc(&dm, 24)) return -1;
    (void)hipMemset(dm, 0, 24);
    const uint64_t threads = 1ull << 20, per = (total + threads - 1) / threads;
    hipLaunchKernelGGL(fp64core_check, dim3((unsigned)(threads / 256)), dim3(256), 0, 0, seed, per, dm);
    if (hipGetLastError() != hipSuccess) return -2;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches3, dm, 24, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    return 0;
}

extern "C" int probe_sincos_core_all(unsigned long long* mismatches, unsigned int* first_bad) {
    unsigned long long* dm;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    hipLaunchKernelGGL(sincos_check, dim3(0x3F800000u / 256), dim3(256), 0, 0, dm, df);
    if (hipGetLastError() != hipSuccess) return -2;
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    return 0;
}

extern "C" int probe_sinf_eval(const float* in, float* out, uint64_t n) {
    float *din, *dout;
    if (hipMalloc(&din, n * 4) || hipMalloc(&dout, n * 4)) return -1;
    (void)hipMemcpy(din, in, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(sinf_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, din, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(din);
    (void)hipFree(dout);
    return 0;
}

extern "C" int probe_ptmi_noise_sinf_all(unsigned long long* mismatches, unsigned int* first_bad,
                                         unsigned long long* cw30_fallbacks) {
    unsigned long long *dm, *dfb;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4) || hipMalloc(&dfb, 8)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(dfb, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(ptmi_noise_sinf_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, chunk, dm, df,
                           dfb);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cw30_fallbacks, dfb, 8, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    (void)hipFree(dfb);
    return 0;
}

// The paired noise sin (ptmi_sinf.h noise_sinf2, round 6) against noise_sinf for every float in
// the first slot, paired with a second float drawn from the whole bit space (a bijective mix of the
// first's bits, so every float is also checked in the second slot).
__device__ static inline uint32_t pair_mix(uint32_t b) {
    b ^= b >> 16;
    b *= 0x7FEB352Du;
    b ^= b >> 15;
    b *= 0x846CA68Bu;
    b ^= b >> 16;
    return b;
}
__global__ void ptmi_noise_sinf2_check(uint64_t base, uint64_t count, unsigned long long* mism, unsigned int* first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = (uint32_t)(base + i);
    const float x1 = pto_bits2f(bits), x2 = pto_bits2f(pair_mix(bits));
    auto fb = [](float v) { return sinf(v); };
    float o1, o2;
    ptmi::noise_sinf2(x1, x2, fb, o1, o2);
    const float e1 = ptmi::noise_sinf(x1, fb), e2 = ptmi::noise_sinf(x2, fb);
    const bool ok1 = pto_f2bits(o1) == pto_f2bits(e1) || (o1 != o1 && e1 != e1);
    const bool ok2 = pto_f2bits(o2) == pto_f2bits(e2) || (o2 != o2 && e2 != e2);
    if (!(ok1 && ok2)) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

extern "C" int probe_ptmi_noise_sinf2_all(unsigned long long* mismatches, unsigned int* first_bad) {
    unsigned long long* dm;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(ptmi_noise_sinf2_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, chunk, dm, df);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    return 0;
}

// v_fract_f32 (__builtin_amdgcn_fractf) against ocml's fract, min(x - floor(x), 0x1.fffffep-1), for
// every finite float: whether noise3d may use the one instruction (PTMI_R6_FRACT).
__global__ void fract_check(uint64_t base, uint64_t count, unsigned long long* mism, unsigned int* first) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t bits = (uint32_t)(base + i);
    const float x = pto_bits2f(bits);
    if (!isfinite(x)) return;
    const float a = __builtin_amdgcn_fractf(x), b = fminf(x - floorf(x), 0x1.fffffep-1f);
    if (pto_f2bits(a) != pto_f2bits(b)) {
        atomicAdd(mism, 1ull);
        atomicMin(first, bits);
    }
}

extern "C" int probe_fract_all(unsigned long long* mismatches, unsigned int* first_bad) {
    unsigned long long* dm;
    unsigned int* df;
    if (hipMalloc(&dm, 8) || hipMalloc(&df, 4)) return -1;
    (void)hipMemset(dm, 0, 8);
    (void)hipMemset(df, 0xff, 4);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(fract_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, chunk, dm, df);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(mismatches, dm, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(first_bad, df, 4, hipMemcpyDeviceToHost);
    (void)hipFree(dm);
    (void)hipFree(df);
    return 0;
}
