"""Restatement of the reference's host-side math (internal/app/geom) used to build
the kernel's input records.  Every function performs the same IEEE-754 double
operations in the same order as the Go source so the produced CLObject /
CLCamera / CLTriangle bytes are identical to what ``BuildSceneBufferCL`` emits.

Matrices are row-major 16-float lists (geom/matrix.go:216 ``Mat4x4 [16]float64``),
tuples are 4-float lists (geom/tuple.go ``Tuple4``).
"""
from . import gomath


def identity():
    return [1.0, 0.0, 0.0, 0.0,
            0.0, 1.0, 0.0, 0.0,
            0.0, 0.0, 1.0, 0.0,
            0.0, 0.0, 0.0, 1.0]


def point(x, y, z):
    return [float(x), float(y), float(z), 1.0]


def vector(x, y, z):
    return [float(x), float(y), float(z), 0.0]


def color(r, g, b):
    """geom.NewColor (tuple.go): w = 1."""
    return [float(r), float(g), float(b), 1.0]


def tuple3(r, g, b):
    """A Go ``geom.Tuple4{r, g, b}`` literal: w = 0."""
    return [float(r), float(g), float(b), 0.0]


def multiply(m1, m2):
    """geom.Multiply / multiply4x4 (matrix.go:41-49, 205-211)."""
    out = [0.0] * 16
    for row in range(4):
        for col in range(4):
            a0 = m1[row * 4 + 0] * m2[0 + col]
            a1 = m1[row * 4 + 1] * m2[4 + col]
            a2 = m1[row * 4 + 2] * m2[8 + col]
            a3 = m1[row * 4 + 3] * m2[12 + col]
            out[row * 4 + col] = a0 + a1 + a2 + a3
    return out


def multiply_by_tuple(m1, t):
    """geom.MultiplyByTuple (matrix.go:51-61)."""
    out = [0.0] * 4
    for row in range(4):
        a = m1[row * 4 + 0] * t[0]
        b = m1[row * 4 + 1] * t[1]
        c = m1[row * 4 + 2] * t[2]
        d = m1[row * 4 + 3] * t[3]
        out[row] = a + b + c + d
    return out


def transpose(m1):
    """geom.Transpose (matrix.go:82-90)."""
    out = [0.0] * 16
    for col in range(4):
        for row in range(4):
            out[row * 4 + col] = m1[col * 4 + row]
    return out


def _det2(m):
    return m[0] * m[3] - m[1] * m[2]


def _sub3(m, dr, dc):
    out = []
    for row in range(3):
        if row == dr:
            continue
        for col in range(3):
            if col == dc:
                continue
            out.append(m[row * 3 + col])
    return out


def _cof3(m, row, col):
    minor = _det2(_sub3(m, row, col))
    return -minor if (row + col) % 2 != 0 else minor


def _det3(m):
    det = 0.0
    for col in range(3):
        det = det + m[col] * _cof3(m, 0, col)
    return det


def _sub4(m, dr, dc):
    out = []
    for row in range(4):
        if row == dr:
            continue
        for col in range(4):
            if col == dc:
                continue
            out.append(m[row * 4 + col])
    return out


def _cof4(m, row, col):
    minor = _det3(_sub4(m, row, col))
    return -minor if (row + col) % 2 != 0 else minor


def _det4(m):
    det = 0.0
    for col in range(4):
        det = det + m[col] * _cof4(m, 0, col)
    return det


def inverse(m1):
    """geom.Inverse: cofactor expansion (matrix.go:190-203)."""
    out = [0.0] * 16
    d4 = _det4(m1)
    for row in range(4):
        for col in range(4):
            c = _cof4(m1, row, col)
            out[col * 4 + row] = c / d4
    return out


def translate(x, y, z):
    m = identity()
    m[3], m[7], m[11] = float(x), float(y), float(z)
    return m


def scale(x, y, z):
    m = identity()
    m[0], m[5], m[10] = float(x), float(y), float(z)
    return m


def rotate_x(r):
    m = identity()
    m[5] = gomath.Cos(r)
    m[6] = -gomath.Sin(r)
    m[9] = gomath.Sin(r)
    m[10] = gomath.Cos(r)
    return m


def rotate_y(r):
    m = identity()
    m[0] = gomath.Cos(r)
    m[2] = gomath.Sin(r)
    m[8] = -gomath.Sin(r)
    m[10] = gomath.Cos(r)
    return m


def rotate_z(r):
    m = identity()
    m[0] = gomath.Cos(r)
    m[1] = -gomath.Sin(r)
    m[4] = gomath.Sin(r)
    m[5] = gomath.Cos(r)
    return m


def sub(a, b):
    return [a[i] - b[i] for i in range(4)]


def add(a, b):
    return [a[i] + b[i] for i in range(4)]


def magnitude(t):
    """geom.Magnitude: 3-component (tuple.go)."""
    import math
    return math.sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2])


def normalize(t):
    """geom.Normalize: all 4 components divided by the 3-component magnitude."""
    m = magnitude(t)
    return [t[i] / m for i in range(4)]


def cross(a, b):
    return [a[1] * b[2] - a[2] * b[1],
            a[2] * b[0] - a[0] * b[2],
            a[0] * b[1] - a[1] * b[0],
            0.0]


def eq(a, b):
    """geom.Eq with Epsilon 0.01 (types.go:5-10)."""
    return abs(a - b) < 0.01


def tuple_equals(a, b):
    return eq(a[0], b[0]) and eq(a[1], b[1]) and eq(a[2], b[2]) and eq(a[3], b[3])
