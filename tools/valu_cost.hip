// DIAGNOSTIC: issue cost of the VALU instruction classes trace_kernel<0> is made of, on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_cost tools/valu_cost.hip && ./build/valu_cost
// Each kernel runs a loop of 16 independent instruction streams (inline asm, so the compiler
// keeps exactly these instructions), one wave per workgroup, W waves per SIMD resident; every wave
// times its loop with s_memtime (shader clock).  Printed: SIMD-cycles per wave64 instruction
// = cycles / (W * instructions per wave), the pipe cost the kernel's instruction mix is priced at
// (profiles/r6/valu_cost.txt).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

enum Op { FMA64, MUL64, ADD64, CND32, ADDU32, MOV32, ADDF32, FMAF32, PKFMA, RCP64, MIX_FMA64_CND, MIX_FMA64_F32,
          MIX_FMA64_SALU, CMP64, CVT64, CND32S, ADDU32S, FMA64S, BFI32, CMPCND, MOV64, MAD64, NOP_OPS };
static const char* kName[] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_cndmask_b32 (vcc)", "v_add_u32", "v_mov_b32",
                              "v_add_f32", "v_fma_f32", "v_pk_fma_f32", "v_rcp_f64", "fma_f64+cndmask (1:1)",
                              "fma_f64+add_f32 (1:1)", "fma_f64+s_add (1:1)", "v_cmp_lt_f64", "v_cvt_f32_f64",
                              "v_cndmask_b32 (s mask)", "v_add_u32 (s operand)", "v_fma_f64 (s operand)", "v_bfi_b32",
                              "v_cmp+v_cndmask (1:1)", "v_mov_b64", "v_mad_u64_u32"};

template <int OP>
__global__ __launch_bounds__(64) void k(unsigned long long* cyc, double* sink, int iters) {
    double d[16];
    float f[16];
    unsigned u[16];
#define INIT(i) d[i] = 1.0 + threadIdx.x * 1e-3 + i; f[i] = 1.0f + i; u[i] = threadIdx.x + i;
    REP16(INIT)
    const double b = 1.0000001, c = 1e-9;
    const float bf = 1.0000001f;
    unsigned s = 0;
    const unsigned long long smask = 0x00000000FFFF0000ull;
    const unsigned s32 = __builtin_amdgcn_readfirstlane(threadIdx.x) + 7;
    const double bs = __builtin_amdgcn_readfirstlane((int)threadIdx.x) + 1.0000001;
    const unsigned vmask = (threadIdx.x & 1) ? 0xFFFF0000u : 0x0000FFFFu;
    asm volatile("v_cmp_gt_u32 vcc, 32, %0" ::"v"(threadIdx.x));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#define STEP(i)                                                                                             \
    if constexpr (OP == FMA64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(b), "v"(c));     \
    if constexpr (OP == MUL64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(b));                  \
    if constexpr (OP == ADD64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(c));                  \
    if constexpr (OP == CND32) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[15 - i]));  \
    if constexpr (OP == ADDU32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[15 - i]));        \
    if constexpr (OP == MOV32) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[15 - i]));             \
    if constexpr (OP == ADDF32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(bf));                \
    if constexpr (OP == FMAF32) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(bf));            \
    if constexpr (OP == PKFMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d[i]) : "v"(b));           \
    if constexpr (OP == RCP64) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));                               \
    if constexpr (OP == MIX_FMA64_CND) {                                                                    \
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(b), "v"(c));                             \
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[15 - i]));                        \
    }                                                                                                       \
    if constexpr (OP == MIX_FMA64_F32) {                                                                    \
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(b), "v"(c));                             \
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(bf));                                        \
    }                                                                                                       \
    if constexpr (OP == MIX_FMA64_SALU) {                                                                   \
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(b), "v"(c));                             \
        asm volatile("s_add_u32 %0, %0, 3" : "+s"(s) : : "scc");                                                      \
    }                                                                                                       \
    if constexpr (OP == CMP64) asm volatile("v_cmp_lt_f64 vcc, %0, %1" ::"v"(d[i]), "v"(b));               \
    if constexpr (OP == CVT64) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));                 \
    if constexpr (OP == CND32S) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[15 - i]), "s"(smask)); \
    if constexpr (OP == ADDU32S) asm volatile("v_add_u32 %0, %1, %0" : "+v"(u[i]) : "s"(s32));               \
    if constexpr (OP == FMA64S) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "s"(bs), "v"(c));     \
    if constexpr (OP == BFI32) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(u[i]) : "v"(vmask), "v"(u[15 - i])); \
    if constexpr (OP == CMPCND) {                                                                             \
        asm volatile("v_cmp_lt_u32 vcc, %0, %1" ::"v"(u[i]), "v"(u[15 - i]) : "vcc");                        \
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[15 - i]));                          \
    }                                                                                                         \
    if constexpr (OP == MOV64) asm volatile("v_mov_b64 %0, %1" : "=v"(d[i]) : "v"(d[15 - i]));               \
    if constexpr (OP == MAD64) asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(d[i]) : "v"(u[i]), "v"(u[15 - i]) : "s100", "s101");
        REP16(STEP)
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double acc = s;
#define SUM(i) acc += d[i] + f[i] + u[i];
    REP16(SUM)
    sink[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(int waves_per_simd, int iters, unsigned long long* dc, double* ds, int ncu) {
    const int grid = ncu * 4 * waves_per_simd;
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(64), 0, 0, dc, ds, 8);  // warm-up
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(64), 0, 0, dc, ds, iters);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(grid);
    hipMemcpy(c.data(), dc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[grid / 2];
    const int per_iter = ((OP >= MIX_FMA64_CND && OP <= MIX_FMA64_SALU) || OP == CMPCND) ? 32 : 16;
    const double insts = (double)iters * per_iter;
    printf("%-24s W=%d  %7.2f cycles per wave-instruction, %5.2f SIMD-cycles per instruction\n", kName[OP],
           waves_per_simd, med / insts, med / (insts * waves_per_simd));
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    printf("%s  %d CUs\n", p.gcnArchName, ncu);
    unsigned long long* dc;
    double* ds;
    hipMalloc(&dc, sizeof(unsigned long long) * ncu * 4 * 8);
    hipMalloc(&ds, sizeof(double) * ncu * 4 * 8 * 64);
    const int iters = 4096;
    for (int w : {1, 4, 8}) {
        run<FMA64>(w, iters, dc, ds, ncu);
        run<MUL64>(w, iters, dc, ds, ncu);
        run<ADD64>(w, iters, dc, ds, ncu);
        run<CND32>(w, iters, dc, ds, ncu);
        run<ADDU32>(w, iters, dc, ds, ncu);
        run<MOV32>(w, iters, dc, ds, ncu);
        run<ADDF32>(w, iters, dc, ds, ncu);
        run<FMAF32>(w, iters, dc, ds, ncu);
        run<PKFMA>(w, iters, dc, ds, ncu);
        run<RCP64>(w, iters, dc, ds, ncu);
        run<CMP64>(w, iters, dc, ds, ncu);
        run<CVT64>(w, iters, dc, ds, ncu);
        run<MIX_FMA64_CND>(w, iters, dc, ds, ncu);
        run<MIX_FMA64_F32>(w, iters, dc, ds, ncu);
        run<MIX_FMA64_SALU>(w, iters, dc, ds, ncu);
        run<CND32S>(w, iters, dc, ds, ncu);
        run<ADDU32S>(w, iters, dc, ds, ncu);
        run<FMA64S>(w, iters, dc, ds, ncu);
        run<BFI32>(w, iters, dc, ds, ncu);
        run<CMPCND>(w, iters, dc, ds, ncu);
        run<MOV64>(w, iters, dc, ds, ncu);
        run<MAD64>(w, iters, dc, ds, ncu);
    }
    return 0;
}
