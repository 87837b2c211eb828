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
