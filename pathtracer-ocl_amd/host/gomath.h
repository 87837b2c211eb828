// gomath.h -- Go's math.Sin / math.Cos / math.Tan (sin.go, tan.go: Cephes
// polynomials after a 3-part Cody-Waite reduction), evaluated with the same
// IEEE-754 double operations in the same order.  The reference builds its scene
// matrices (geom/rotation.go, camera.go:22) with these, so glibc's sin/cos would
// change the kernel's input bytes.  Compiled with -ffp-contract=off: Go on amd64
// never fuses.  Only |x| < 2^29 (Go's reduceThreshold) is restated.
#pragma once
#include <cmath>
#include <cstdint>
#include <stdexcept>

namespace ptmi_host {
namespace gomath {

constexpr double kSin[6] = {1.58962301576546568060e-10, -2.50507477628578072866e-8, 2.75573136213857245213e-6,
                            -1.98412698295895385996e-4, 8.33333333332211858878e-3, -1.66666666666666307295e-1};
constexpr double kCos[6] = {-1.13585365213876817300e-11, 2.08757008419747316778e-9, -2.75573141792967388112e-7,
                            2.48015872888517045348e-5,  -1.38888888888730564116e-3, 4.16666666666665929218e-2};
constexpr double kTanP[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
constexpr double kTanQ[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6, 2.50083801823357915839e7,
                             -5.38695755929454629881e7};
constexpr double PI4A = 7.85398125648498535156e-1;   // 0x3fe921fb40000000
constexpr double PI4B = 3.77489470793079817668e-8;   // 0x3e64442d00000000
constexpr double PI4C = 2.69515142907905952645e-15;  // 0x3ce8469898cc5170
constexpr double kReduceThreshold = 536870912.0;     // 1 << 29
constexpr double kFourOverPi = 1.2732395447351628;   // Go constant 4/Pi, rounded once

inline void reduce(double x, uint64_t& j, double& z) {
    if (x >= kReduceThreshold) throw std::domain_error("gomath: Payne-Hanek path not restated (|x| >= 2^29)");
    j = (uint64_t)(x * kFourOverPi);
    double y = (double)j;
    if (j & 1) {
        j++;
        y += 1;
    }
    j &= 7;
    z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
}
inline double sinpoly(double z, double zz) {
    return z + z * zz * ((((((kSin[0] * zz) + kSin[1]) * zz + kSin[2]) * zz + kSin[3]) * zz + kSin[4]) * zz + kSin[5]);
}
inline double cospoly(double zz) {
    return 1.0 - 0.5 * zz +
           zz * zz * ((((((kCos[0] * zz) + kCos[1]) * zz + kCos[2]) * zz + kCos[3]) * zz + kCos[4]) * zz + kCos[5]);
}

inline double Sin(double x) {
    if (std::isnan(x) || std::isinf(x)) return NAN;
    if (x == 0) return x;
    bool sign = false;
    if (x < 0) {
        x = -x;
        sign = true;
    }
    uint64_t j;
    double z;
    reduce(x, j, z);
    if (j > 3) {
        sign = !sign;
        j -= 4;
    }
    const double zz = z * z;
    const double y = (j == 1 || j == 2) ? cospoly(zz) : sinpoly(z, zz);
    return sign ? -y : y;
}

inline double Cos(double x) {
    if (std::isnan(x) || std::isinf(x)) return NAN;
    bool sign = false;
    x = std::fabs(x);
    uint64_t j;
    double z;
    reduce(x, j, z);
    if (j > 3) {
        j -= 4;
        sign = !sign;
    }
    if (j > 1) sign = !sign;
    const double zz = z * z;
    const double y = (j == 1 || j == 2) ? sinpoly(z, zz) : cospoly(zz);
    return sign ? -y : y;
}

inline double Tan(double x) {
    if (x == 0 || std::isnan(x)) return x;
    if (std::isinf(x)) return NAN;
    bool sign = false;
    if (x < 0) {
        x = -x;
        sign = true;
    }
    if (x >= kReduceThreshold) throw std::domain_error("gomath: Payne-Hanek path not restated (|x| >= 2^29)");
    uint64_t j = (uint64_t)(x * kFourOverPi);
    double y = (double)j;
    if (j & 1) {
        j++;
        y += 1;
    }
    const double z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
    const double zz = z * z;
    if (zz > 1e-14)
        y = z + z * (zz * (((kTanP[0] * zz) + kTanP[1]) * zz + kTanP[2]) /
                     ((((zz + kTanQ[1]) * zz + kTanQ[2]) * zz + kTanQ[3]) * zz + kTanQ[4]));
    else
        y = z;
    if (j & 2) y = -1 / y;
    return sign ? -y : y;
}

}  // namespace gomath
}  // namespace ptmi_host
