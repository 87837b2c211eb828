"""Bit-faithful restatement of the Go ``math`` trig functions the reference scene
builders call (``math.Sin``/``math.Cos``/``math.Tan`` in camera.go:22 and
geom/rotation.go:5-32).

Go's trig functions are pure Go (Cephes polynomials with a 3-part Cody-Waite
reduction), not the platform libm, so ``math.cos(pi/2)`` in Python (glibc) and
``math.Cos(math.Pi/2)`` in Go differ in the last bits.  The scene matrices are part
of the kernel's input bytes, so the restatement evaluates the same IEEE-754 double
operations in the same order.  Python floats are IEEE doubles with no FMA
contraction, matching the Go gc compiler on amd64 (GOAMD64=v1 never fuses).

Only the |x| < 2**29 path (``reduceThreshold``) is needed by any scene; larger
arguments raise instead of silently deviating.
"""
import math

_SIN = (
    1.58962301576546568060e-10,   # 0x3de5d8fd1fd19ccd
    -2.50507477628578072866e-8,   # 0xbe5ae5e5a9291f5d
    2.75573136213857245213e-6,    # 0x3ec71de3567d48a1
    -1.98412698295895385996e-4,   # 0xbf2a01a019bfdf03
    8.33333333332211858878e-3,    # 0x3f8111111110f7d0
    -1.66666666666666307295e-1,   # 0xbfc5555555555548
)
_COS = (
    -1.13585365213876817300e-11,  # 0xbda8fa49a0861a9b
    2.08757008419747316778e-9,    # 0x3e21ee9d7b4e3f05
    -2.75573141792967388112e-7,   # 0xbe927e4f7eac4bc6
    2.48015872888517045348e-5,    # 0x3efa01a019c844f5
    -1.38888888888730564116e-3,   # 0xbf56c16c16c14f91
    4.16666666666665929218e-2,    # 0x3fa555555555554b
)
_TANP = (
    -1.30936939181383777646e4,    # 0xc0c992d8d24f3f38
    1.15351664838587416140e6,     # 0x413199eca5fc9ddd
    -1.79565251976484877988e7,    # 0xc1711fead3299176
)
_TANQ = (
    1.0,
    1.36812963470692954678e4,     # 0x40cab8a5eeb36572
    -1.32089234440210967447e6,    # 0xc13427bc582abc96
    2.50083801823357915839e7,     # 0x4177d98fc2ead8ef
    -5.38695755929454629881e7,    # 0xc189afe03cbe5a31
)
PI4A = 7.85398125648498535156e-1   # 0x3fe921fb40000000
PI4B = 3.77489470793079817668e-8   # 0x3e64442d00000000
PI4C = 2.69515142907905952645e-15  # 0x3ce8469898cc5170
REDUCE_THRESHOLD = float(1 << 29)
FOUR_OVER_PI = 4.0 / math.pi       # Go constant 4/Pi rounded once to float64

Pi = math.pi  # Go's math.Pi constant rounds to the same float64


def _reduce(x):
    if x >= REDUCE_THRESHOLD:
        raise ValueError("gomath: Payne-Hanek path not restated (|x| >= 2^29)")
    j = int(x * FOUR_OVER_PI)
    y = float(j)
    if j & 1 == 1:
        j += 1
        y += 1
    j &= 7
    z = ((x - y * PI4A) - y * PI4B) - y * PI4C
    return j, z


def _sinpoly(z, zz):
    return z + z * zz * ((((((_SIN[0] * zz) + _SIN[1]) * zz + _SIN[2]) * zz + _SIN[3]) * zz + _SIN[4]) * zz + _SIN[5])


def _cospoly(zz):
    return 1.0 - 0.5 * zz + zz * zz * ((((((_COS[0] * zz) + _COS[1]) * zz + _COS[2]) * zz + _COS[3]) * zz + _COS[4]) * zz + _COS[5])


def Sin(x):
    """Go math.Sin (sin.go)."""
    if math.isnan(x) or math.isinf(x):
        return math.nan
    if x == 0:
        return x
    sign = False
    if x < 0:
        x = -x
        sign = True
    j, z = _reduce(x)
    if j > 3:
        sign = not sign
        j -= 4
    zz = z * z
    y = _cospoly(zz) if j in (1, 2) else _sinpoly(z, zz)
    return -y if sign else y


def Cos(x):
    """Go math.Cos (sin.go)."""
    if math.isnan(x) or math.isinf(x):
        return math.nan
    sign = False
    x = abs(x)
    j, z = _reduce(x)
    if j > 3:
        j -= 4
        sign = not sign
    if j > 1:
        sign = not sign
    zz = z * z
    y = _sinpoly(z, zz) if j in (1, 2) else _cospoly(zz)
    return -y if sign else y


def Tan(x):
    """Go math.Tan (tan.go)."""
    if x == 0 or math.isnan(x):
        return x
    if math.isinf(x):
        return math.nan
    sign = False
    if x < 0:
        x = -x
        sign = True
    if x >= REDUCE_THRESHOLD:
        raise ValueError("gomath: Payne-Hanek path not restated (|x| >= 2^29)")
    j = int(x * FOUR_OVER_PI)
    y = float(j)
    if j & 1 == 1:
        j += 1
        y += 1
    z = ((x - y * PI4A) - y * PI4B) - y * PI4C
    zz = z * z
    if zz > 1e-14:
        y = z + z * (zz * (((_TANP[0] * zz) + _TANP[1]) * zz + _TANP[2])
                     / ((((zz + _TANQ[1]) * zz + _TANQ[2]) * zz + _TANQ[3]) * zz + _TANQ[4]))
    else:
        y = z
    if j & 2 == 2:
        y = -1 / y
    return -y if sign else y
