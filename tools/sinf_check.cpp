// DIAGNOSTIC / verification: ptmi::sinf_lt19 (pathtracer-ocl_amd/csrc/ptmi_sinf.h,
// the kernel's noise sin) against the oracle's restatement of ocml's sin_f32
// (oracle/ocml_sinf.h, itself bit-identical to the device library over all 2^32
// floats) for EVERY float with |x| < 2^19.  Host build, run from tools/:
//   g++ -O2 -fopenmp -ffp-contract=off -mfma -std=c++20 -o /tmp/sinf_check sinf_check.cpp && /tmp/sinf_check
#include <cstdio>
#include <cstdint>
#define PT_FN static inline
#include "../oracle/ocml_sinf.h"
#define PTMI_SINF_FN static inline
#include "../pathtracer-ocl_amd/csrc/ptmi_sinf.h"
int main() {
  unsigned long long bad = 0; uint32_t first = 0xffffffff;
  const uint32_t END = 0x49000000u;  // 2^19
  #pragma omp parallel for reduction(+:bad) schedule(static)
  for (long long i = 0; i < (long long)END; i++) {
    uint32_t b = (uint32_t)i;
    float x = pto_bits2f(b);
    float a = ptmi::sinf_lt19(x), c = pto_sinf(x);
    float xn = -x;
    float an = ptmi::sinf_lt19(xn), cn = pto_sinf(xn);
    if (pto_f2bits(a) != pto_f2bits(c) || pto_f2bits(an) != pto_f2bits(cn)) {
      bad++;
      #pragma omp critical
      { if (b < first) first = b; }
    }
  }
  printf("mismatches %llu first 0x%08x\n", bad, first);
  // ptmi::sinf_cw30 (2^19 <= |x| < 2^30, the glass noise) where it returns a result
  unsigned long long bad2 = 0, fb = 0;
  #pragma omp parallel for reduction(+:bad2, fb) schedule(static)
  for (long long i = 0x49000000ll; i < 0x4E800000ll; i++) {
    for (int sg = 0; sg < 2; sg++) {
      const float x = pto_bits2f((uint32_t)i | (sg ? 0x80000000u : 0u));
      float a;
      if (!ptmi::sinf_cw30(x, a)) { fb++; continue; }
      if (pto_f2bits(a) != pto_f2bits(pto_sinf(x))) bad2++;
    }
  }
  printf("cw30: mismatches %llu fallbacks %llu of %llu\n", bad2, fb, 2ull * (0x4E800000ull - 0x49000000ull));
}
