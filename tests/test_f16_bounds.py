"""Host check of the traversal boxes' binary16 bounds (csrc/ptmi_f16.h, used by
ptmi_bvh.cpp): f16_down / f16_up must round outward -- the largest binary16 <= v and
the smallest >= v, +-infinity past the range -- since a Node4 bound that moved
inward could cull a box the exact ray passes (binary16 bounds).
Checked against numpy's float16 on random doubles over the whole binary16 range and
its edges; the header is compiled here with g++ (no GPU)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HDR = os.path.join(ROOT, "pathtracer-ocl_amd", "csrc")

SRC = r'''
#include "ptmi_f16.h"
extern "C" uint16_t t_down(double v) { return ptmi::f16_down(v); }
extern "C" uint16_t t_up(double v) { return ptmi::f16_up(v); }
extern "C" double t_value(uint16_t h) { return ptmi::f16_value(h); }
'''


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("f16")
    src, so = d / "f16.cpp", d / "libf16.so"
    src.write_text(SRC)
    subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-I", HDR, "-o", str(so), str(src)], check=True)
    L = ctypes.CDLL(str(so))
    L.t_down.restype = L.t_up.restype = ctypes.c_uint16
    L.t_down.argtypes = L.t_up.argtypes = [ctypes.c_double]
    L.t_value.restype = ctypes.c_double
    L.t_value.argtypes = [ctypes.c_uint16]
    return L


def _f16(bits):
    return float(np.array([bits], dtype=np.uint16).view(np.float16)[0])


def test_decoder_matches_numpy_for_every_pattern(lib):
    for h in range(0x10000):
        a, b = lib.t_value(h), _f16(h)
        assert (a == b) or (np.isnan(a) and np.isnan(b)), hex(h)


def _samples():
    rng = np.random.default_rng(16)
    v = [0.0, -0.0, 1.0, -1.0, 65504.0, -65504.0, 65519.99, 65520.0, -65520.0, 1e5, -1e5, 1e300, -1e300,
         2.0 ** -24, -(2.0 ** -24), 2.0 ** -25, -(2.0 ** -25), 2.0 ** -14, 3.4, -3.434, 1e-7, -1e-7]
    mags = np.exp(rng.uniform(np.log(1e-9), np.log(2e5), 20000))
    v += list(mags * rng.choice([-1.0, 1.0], mags.size))
    # values on and next to binary16 grid points
    grid = np.array(rng.integers(0, 0x7c00, 2000), dtype=np.uint16).view(np.float16).astype(np.float64)
    v += list(grid) + list(np.nextafter(grid, np.inf)) + list(np.nextafter(grid, -np.inf)) + list(-grid)
    return v


def test_outward_rounding_is_tight(lib):
    with np.errstate(over="ignore"):  # nextafter from +-65504 outward is +-inf by design
        for v in _samples():
            lo, hi = lib.t_value(lib.t_down(v)), lib.t_value(lib.t_up(v))
            assert lo <= v <= hi, v
            # tight: no binary16 strictly between lo and v, or between v and hi
            assert lo == v or float(np.nextafter(np.float16(lo), np.float16(np.inf))) > v, v
            assert hi == v or float(np.nextafter(np.float16(hi), np.float16(-np.inf))) < v, v
            if abs(v) < 65504.0:
                assert np.isfinite(lo) and np.isfinite(hi), v


def test_past_range_is_infinite(lib):
    assert lib.t_value(lib.t_up(65505.0)) == np.inf
    assert lib.t_value(lib.t_down(-65505.0)) == -np.inf
    assert lib.t_value(lib.t_down(1e5)) == 65504.0
    assert lib.t_value(lib.t_up(-1e5)) == -65504.0
