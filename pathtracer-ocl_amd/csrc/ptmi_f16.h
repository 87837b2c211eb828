// ptmi_f16.h -- IEEE binary16 with directed rounding, for the traversal boxes'
// bounds (ptmi_bvh.cpp; tested on the host by tests/test_f16_bounds.py).
#pragma once
#include <stdint.h>

#include <cmath>

namespace ptmi {

// IEEE binary16 for the Node4 bounds.  Finite and infinite patterns are ordered by
// ord(h) = +-(h & 0x7fff) (sign from bit 15), so directed rounding is a search over
// that order with the exact decoder.
constexpr uint16_t kF16Inf = 0x7c00;
inline double f16_value(uint16_t h) {
    const int e = (h >> 10) & 31, f = h & 1023;
    const double mag = e == 31 ? (f ? NAN : HUGE_VAL) : e == 0 ? std::ldexp(f, -24) : std::ldexp(1024 + f, e - 25);
    return (h & 0x8000) ? -mag : mag;
}
inline uint16_t f16_of_ord(int o) { return o >= 0 ? (uint16_t)o : (uint16_t)(0x8000 | -o); }
// The largest binary16 <= v (-infinity below the range).
inline uint16_t f16_down(double v) {
    int lo = -kF16Inf, hi = kF16Inf;  // f16_value(ord lo) <= v holds for every non-NaN v
    if (f16_value(f16_of_ord(hi)) <= v) return kF16Inf;
    while (hi - lo > 1) {  // invariant: value(lo) <= v < value(hi)
        const int mid = lo + (hi - lo) / 2;
        (f16_value(f16_of_ord(mid)) <= v ? lo : hi) = mid;
    }
    return f16_of_ord(lo);
}
// The smallest binary16 >= v (+infinity above the range).
inline uint16_t f16_up(double v) {
    int lo = -kF16Inf, hi = kF16Inf;
    if (f16_value(f16_of_ord(lo)) >= v) return f16_of_ord(lo);
    while (hi - lo > 1) {  // invariant: value(lo) < v <= value(hi)
        const int mid = lo + (hi - lo) / 2;
        (f16_value(f16_of_ord(mid)) >= v ? hi : lo) = mid;
    }
    return f16_of_ord(hi);
}

}  // namespace ptmi
