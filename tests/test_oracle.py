"""The CPU oracle (oracle/pt_oracle.c) against golden vectors produced by THE
REFERENCE KERNEL ITSELF (tracer.cl compiled by ROCm's OpenCL toolchain, run on an
MI355X: tests/golden/make_golden.py).  This is what pins the oracle; every GPU
parity test then compares the product against this oracle and the same goldens.
"""
import numpy as np
import pytest

import pyoracle
from ptmi import layout
from tests.scene_inputs import scene_inputs

TOL = 1e-4  # north_star: image L-inf < 1e-4 per channel vs the reference


def _inputs(z):
    objs, tris, grps, cam = scene_inputs(str(z["scene"]), int(z["width"]), int(z["height"]),
                                         float(z["aperture"]), float(z["focal_length"]))
    return objs, tris, grps, cam


def test_golden_inputs_match_scene_restatement(golden_cases):
    """The records the reference rendered are exactly what ptmi's restatement of
    the Go scene code produces today (no drift in the input side)."""
    assert golden_cases, "no golden vectors found"
    for name, z in golden_cases.items():
        objs, _, _, cam = _inputs(z)
        assert np.array_equal(objs.view(np.uint8).ravel(), z["objects"].ravel()), name
        assert np.array_equal(np.asarray(cam).reshape(1).view(np.uint8).ravel(), z["camera"].ravel()), name


@pytest.mark.parametrize("name", ["ref_64x48_s4", "ref_dof_64x48_s8", "ocl_64x48_s8", "teapot_32x24_s4",
                                  "ref_64x48_s16", "ref_40x30_s3", "ocl_dof_48x32_s5", "gopher_32x24_s4",
                                  "ref_160x120_s4", "transp_48x32_s6", "transp_quad_48x32_s4",
                                  "transp_f_dof_48x32_s5", "reflect_48x32_s6", "glassteapot_32x24_s4"])
def test_oracle_matches_reference_kernel(golden_cases, name):
    if name not in golden_cases:
        pytest.skip("golden %s not generated yet" % name)
    z = golden_cases[name]
    objs, tris, grps, cam = _inputs(z)
    tris, grps = layout.pad_empty(tris, grps)
    out = pyoracle.cpu_trace(objs, tris, grps, cam, int(z["samples"]), z["seeds"])
    ref = z["rgba"]
    assert out.shape == ref.shape
    assert not np.isnan(out).any()
    err = np.abs(out - ref).max()
    assert err < TOL, "%s: L-inf %.3e" % (name, err)
    # In practice the restatement agrees to double rounding noise (~1e-15).
    assert err < 1e-12, "%s: L-inf %.3e (expected rounding-level agreement)" % (name, err)
    assert np.all(ref[3::4] == 1.0)


def test_oracle_sample_split_sums_to_full(golden_cases):
    """Sample ranges use GLOBAL indices (fgi2 = seed/S, sunflower(S, 2, n)), so the
    sum of partial renders equals the full render (the multi-GPU sample split)."""
    z = golden_cases["ref_dof_64x48_s8"]
    objs, tris, grps, cam = _inputs(z)
    tris, grps = layout.pad_empty(tris, grps)
    S = int(z["samples"])
    parts = [pyoracle.cpu_trace(objs, tris, grps, cam, S, z["seeds"], sample_begin=a, sample_end=b)
             for a, b in ((0, 3), (3, 5), (5, 8))]
    tot = sum(parts)
    assert np.all(tot[3::4] == S)
    rgb = tot.reshape(-1, 4)[:, :3] * (1.0 / S)
    ref = z["rgba"].reshape(-1, 4)[:, :3]
    assert np.abs(rgb - ref).max() < 1e-12


def test_oracle_row_window_matches_full(golden_cases):
    z = golden_cases["ref_64x48_s4"]
    objs, tris, grps, cam = _inputs(z)
    tris, grps = layout.pad_empty(tris, grps)
    w = int(z["width"])
    part = pyoracle.cpu_trace(objs, tris, grps, cam, int(z["samples"]), z["seeds"], row0=10, rows=7)
    assert np.array_equal(part, z["rgba"][10 * w * 4:17 * w * 4]) or \
        np.abs(part - z["rgba"][10 * w * 4:17 * w * 4]).max() < 1e-12


def test_dof_sample_zero_is_black():
    """sunflowerRadius(0, ...) = sqrt(-0.5) = NaN (tracer.cl:224, 766): with DoF the
    n = 0 camera ray is NaN, misses everything and contributes exactly 0."""
    objs, tris, grps, cam = scene_inputs("reference", 16, 12, 0.15, 1.6)
    tris, grps = layout.pad_empty(tris, grps)
    seeds = layout.seeds_go_float64(16 * 12, 5)
    s0 = pyoracle.cpu_trace(objs, tris, grps, cam, 4, seeds, sample_begin=0, sample_end=1)
    assert np.all(s0.reshape(-1, 4)[:, :3] == 0.0)


def test_textured_object_without_textures_is_black():
    """A textured object with no texture arrays samples the reference's all-zero
    fake image (ocltracer.go:249-251): its bounce colour becomes (0, 0, 0)."""
    objs, tris, grps, cam = scene_inputs("reference", 16, 12)
    tris, grps = layout.pad_empty(tris, grps)
    seeds = layout.seeds_go_float64(16 * 12, 5)
    tex = objs.copy()
    tex["is_textured"][1] = 1  # the floor plane
    black = objs.copy()
    black["color"][1][:3] = 0.0
    a = pyoracle.cpu_trace(tex, tris, grps, cam, 2, seeds)
    b = pyoracle.cpu_trace(black, tris, grps, cam, 2, seeds)
    assert np.array_equal(a, b)


def test_golden_cases_stay_inside_reference_ctx(golden_cases):
    """Every golden case records at most 64 candidates per line in the reference's ctx
    arrays (tracer.cl:97-99), so the reference's image is defined there; the adversarial
    "bumpy" mesh goes past them (it is an oracle-only case) and "big" does not."""
    for name, z in golden_cases.items():
        objs, tris, grps, cam = _inputs(z)
        seeds = np.asarray(z["seeds"], dtype=np.float64)
        t2, g2 = layout.pad_empty(tris, grps)
        n = pyoracle.max_candidates(objs, t2, g2, cam, 1, seeds, rows=4)
        assert 0 < n <= 64, (name, n)
    from tests import adversarial
    for kind, past in (("big", False), ("bumpy", True)):
        objs, tris, grps, cam = adversarial.scene_inputs(kind, 64, 48)
        t2, g2 = layout.pad_empty(tris, grps)
        n = pyoracle.max_candidates(objs, t2, g2, cam, 2, layout.seeds_go_float64(64 * 48, 404))
        assert (n > 64) == past, (kind, n)
