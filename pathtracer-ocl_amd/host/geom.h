// geom.h -- the reference's host geometry (internal/app/geom): row-major 4x4
// matrices (matrix.go, Mat4x4 [16]float64) and 4-tuples (tuple.go), with the
// same double operations in the same order as the Go source, so the matrices
// that land in CLObject / CLCamera are bit-identical.  -ffp-contract=off.
#pragma once
#include <array>
#include <cmath>

#include "gomath.h"

namespace ptmi_host {

using Mat = std::array<double, 16>;
using Tup = std::array<double, 4>;

inline Mat identity() { return {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}; }
inline Tup point(double x, double y, double z) { return {x, y, z, 1.0}; }
inline Tup vector(double x, double y, double z) { return {x, y, z, 0.0}; }
inline Tup color(double r, double g, double b) { return {r, g, b, 1.0}; }   // geom.NewColor: w = 1
inline Tup tuple3(double r, double g, double b) { return {r, g, b, 0.0}; }  // a Tuple4{r, g, b} literal

// Multiply / multiply4x4 (matrix.go:41-49, 205-211): a0 + a1 + a2 + a3 left to right.
inline Mat multiply(const Mat& m1, const Mat& m2) {
    Mat out{};
    for (int row = 0; row < 4; row++)
        for (int col = 0; col < 4; col++) {
            const double a0 = m1[row * 4 + 0] * m2[0 + col];
            const double a1 = m1[row * 4 + 1] * m2[4 + col];
            const double a2 = m1[row * 4 + 2] * m2[8 + col];
            const double a3 = m1[row * 4 + 3] * m2[12 + col];
            out[row * 4 + col] = a0 + a1 + a2 + a3;
        }
    return out;
}

// MultiplyByTuple (matrix.go:51-61)
inline Tup multiply_by_tuple(const Mat& m, const Tup& t) {
    Tup out{};
    for (int row = 0; row < 4; row++) {
        const double a = m[row * 4 + 0] * t[0];
        const double b = m[row * 4 + 1] * t[1];
        const double c = m[row * 4 + 2] * t[2];
        const double d = m[row * 4 + 3] * t[3];
        out[row] = a + b + c + d;
    }
    return out;
}

inline Mat transpose(const Mat& m) {
    Mat out{};
    for (int col = 0; col < 4; col++)
        for (int row = 0; row < 4; row++) out[row * 4 + col] = m[col * 4 + row];
    return out;
}

namespace detail {
inline double det2(const double* m) { return m[0] * m[3] - m[1] * m[2]; }
inline void sub3(const double* m, int dr, int dc, double* out) {
    int k = 0;
    for (int row = 0; row < 3; row++) {
        if (row == dr) continue;
        for (int col = 0; col < 3; col++) {
            if (col == dc) continue;
            out[k++] = m[row * 3 + col];
        }
    }
}
inline double cof3(const double* m, int row, int col) {
    double s[4];
    sub3(m, row, col, s);
    const double minor = det2(s);
    return ((row + col) % 2 != 0) ? -minor : minor;
}
inline double det3(const double* m) {
    double det = 0.0;
    for (int col = 0; col < 3; col++) det = det + m[col] * cof3(m, 0, col);
    return det;
}
inline void sub4(const double* m, int dr, int dc, double* out) {
    int k = 0;
    for (int row = 0; row < 4; row++) {
        if (row == dr) continue;
        for (int col = 0; col < 4; col++) {
            if (col == dc) continue;
            out[k++] = m[row * 4 + col];
        }
    }
}
inline double cof4(const double* m, int row, int col) {
    double s[9];
    sub4(m, row, col, s);
    const double minor = det3(s);
    return ((row + col) % 2 != 0) ? -minor : minor;
}
inline double det4(const double* m) {
    double det = 0.0;
    for (int col = 0; col < 4; col++) det = det + m[col] * cof4(m, 0, col);
    return det;
}
}  // namespace detail

// Inverse: cofactor expansion (matrix.go:190-203)
inline Mat inverse(const Mat& m) {
    Mat out{};
    const double d4 = detail::det4(m.data());
    for (int row = 0; row < 4; row++)
        for (int col = 0; col < 4; col++) out[col * 4 + row] = detail::cof4(m.data(), row, col) / d4;
    return out;
}

inline Mat translate(double x, double y, double z) {
    Mat m = identity();
    m[3] = x, m[7] = y, m[11] = z;
    return m;
}
inline Mat scale(double x, double y, double z) {
    Mat m = identity();
    m[0] = x, m[5] = y, m[10] = z;
    return m;
}
// rotation.go:5-32
inline Mat rotate_x(double r) {
    Mat m = identity();
    m[5] = gomath::Cos(r);
    m[6] = -gomath::Sin(r);
    m[9] = gomath::Sin(r);
    m[10] = gomath::Cos(r);
    return m;
}
inline Mat rotate_y(double r) {
    Mat m = identity();
    m[0] = gomath::Cos(r);
    m[2] = gomath::Sin(r);
    m[8] = -gomath::Sin(r);
    m[10] = gomath::Cos(r);
    return m;
}
inline Mat rotate_z(double r) {
    Mat m = identity();
    m[0] = gomath::Cos(r);
    m[1] = -gomath::Sin(r);
    m[4] = gomath::Sin(r);
    m[5] = gomath::Cos(r);
    return m;
}

inline Tup sub(const Tup& a, const Tup& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]}; }
inline Tup add(const Tup& a, const Tup& b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]}; }
// Magnitude: 3 components (tuple.go); Normalize divides all 4 by it.
inline double magnitude(const Tup& t) { return std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]); }
inline Tup normalize(const Tup& t) {
    const double m = magnitude(t);
    return {t[0] / m, t[1] / m, t[2] / m, t[3] / m};
}
inline Tup cross(const Tup& a, const Tup& b) {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0], 0.0};
}
// Eq with Epsilon 0.01 (types.go:5-10)
inline bool eq(double a, double b) { return std::fabs(a - b) < 0.01; }
inline bool tuple_equals(const Tup& a, const Tup& b) {
    return eq(a[0], b[0]) && eq(a[1], b[1]) && eq(a[2], b[2]) && eq(a[3], b[3]);
}

}  // namespace ptmi_host
