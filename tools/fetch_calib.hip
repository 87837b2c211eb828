// DIAGNOSTIC: calibrates the L2 -> fabric read counters (FETCH_SIZE, TCC_EA0_RDREQ*) on access
// patterns of known size, so the mesh kernels' HBM figures can be read in bytes
// (MI355X_MICROARCH.md: "Other access widths are uncalibrated: calibrate on a known byte count").
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc <counters> -- tools/bin/fetch_calib
// Kernels (one dispatch each, over a 1 GiB buffer, 8 Mi 128-B lines):
//   stream16    every byte once, 16 B per lane, coalesced (the guide's calibrated case)
//   line64_scat one 64-B half of every 128-B line, 16 B per lane (4 lanes per half), lines in
//               a scattered (odd-multiplier) order -- a Node4 read
//   line128_scat both halves of every line, as one 128-B read of 8 lanes, scattered
//   word8_scat  one 8-B word per line, scattered (a hemisphere-table or scratch-like read)
// The known byte counts are printed; compare the counters per dispatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr uint64_t kBytes = 1ull << 30;
constexpr uint64_t kLines = kBytes / 128;

__device__ __forceinline__ uint64_t scatter(uint64_t i) { return (i * 0x9E3779B1ull) & (kLines - 1); }

__global__ void stream16(const uint4* __restrict__ p, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 v = p[i];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;
}

__global__ void line64_scat(const uint4* __restrict__ p, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 4 lanes per line
    const uint64_t line = scatter(i >> 2);
    const uint4 v = p[line * 8 + (i & 3)];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;
}

__global__ void line128_scat(const uint4* __restrict__ p, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 8 lanes per line
    const uint64_t line = scatter(i >> 3);
    const uint4 v = p[line * 8 + (i & 7)];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1;
}

__global__ void word8_scat(const uint2* __restrict__ p, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 1 lane per line
    const uint2 v = p[scatter(i) * 16];
    if ((v.x ^ v.y) == 0x12345678u) out[0] = 1;
}

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

int main() {
    void* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc((void**)&out, 256));
    CK(hipMemset(buf, 1, kBytes));
    CK(hipDeviceSynchronize());
    const uint4* p4 = (const uint4*)buf;
    stream16<<<dim3((unsigned)(kBytes / 16 / 256)), dim3(256)>>>(p4, out);
    line64_scat<<<dim3((unsigned)(kLines * 4 / 256)), dim3(256)>>>(p4, out);
    line128_scat<<<dim3((unsigned)(kLines * 8 / 256)), dim3(256)>>>(p4, out);
    word8_scat<<<dim3((unsigned)(kLines / 256)), dim3(256)>>>((const uint2*)buf, out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    printf("stream16     requested %llu B (%llu lines, each whole)\n", (unsigned long long)kBytes,
           (unsigned long long)kLines);
    printf("line64_scat  requested %llu B (%llu lines, one 64-B half each)\n", (unsigned long long)(kBytes / 2),
           (unsigned long long)kLines);
    printf("line128_scat requested %llu B (%llu lines, each whole)\n", (unsigned long long)kBytes,
           (unsigned long long)kLines);
    printf("word8_scat   requested %llu B (%llu lines, one 8-B word each)\n", (unsigned long long)(kLines * 8),
           (unsigned long long)kLines);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
