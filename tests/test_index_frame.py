"""The traversal index's per-root frame (ptmi_bvh.cpp, RootRec ctr / sc): Node4
bounds are binary16 values of (bound - ctr) / 2^s, so a mesh far from the origin or larger
than binary16's range keeps boxes as tight as the same mesh at the origin.  Host only
(ptmi_index_stats builds the index on the CPU); the GPU parity of moved meshes against the
live reference is in tests/test_gpu_parity.py."""
import pytest

from ptmi import api
from tests.moved_mesh import moved
from tests.scene_inputs import scene_inputs


@pytest.fixture(scope="module")
def teapot():
    return scene_inputs("teapot", 64, 48)


def _stats(objs, tris, grps, cam):
    return api.index_stats(objs, tris, grps, cam)


def test_index_stats_of_the_teapot(teapot):
    st = _stats(*teapot)
    assert st["roots"] == 1 and st["nodes4"] > 100 and st["slots"] > st["nodes4"]
    assert st["inf_bounds"] == 0 and st["max_scale_exp"] == 0


@pytest.mark.parametrize("offset,tol", [((1.0e3, 0.0, 0.0), 0.005), ((1.0e4, 0.0, 0.0), 0.02),
                                        ((-3.0e4, 2.0e4, 7.5e3), 0.05)])
def test_offset_mesh_keeps_its_boxes(teapot, offset, tol):
    """Translated in object space by 1e3-3e4 units (an OBJ in millimetres, say): the
    decoded boxes' total surface area stays close to the mesh's at the origin.  In a frame
    at the origin the binary16 rounding near |x| = 1e4 alone is 4-8 units on this mesh,
    which is ~7 units across, and past 65504 every bound on that axis is infinite.  What
    is left is the index's widening, 1e-7 x the largest |coordinate| (it covers hit-point
    rounding, which grows with the coordinates): 0.1 % / 1.5 % / 4.4 % more box area
    here."""
    objs, tris, grps, cam = teapot
    base = _stats(objs, tris, grps, cam)
    st = _stats(*moved(objs, tris, grps, offset=offset), cam)
    assert st["nodes4"] == base["nodes4"] and st["inf_bounds"] == 0
    assert abs(st["box_area"] / base["box_area"] - 1.0) < tol, (st, base)


@pytest.mark.parametrize("scale,offset", [(1.0e5, (0.0, 0.0, 0.0)), (3.0e5, (1.0e9, 0.0, -2.0e9))])
def test_large_mesh_gets_finite_scaled_bounds(teapot, scale, offset):
    """Scaled past binary16's range (extent up to ~1e7 units): the root scale 2^s keeps
    every bound finite, and box areas scale with the mesh (within 2 %)."""
    objs, tris, grps, cam = teapot
    base = _stats(objs, tris, grps, cam)
    st = _stats(*moved(objs, tris, grps, offset=offset, scale=scale), cam)
    assert st["inf_bounds"] == 0 and st["max_scale_exp"] > 0, st
    assert abs(st["box_area"] / (base["box_area"] * scale * scale) - 1.0) < 0.02, (st, base)


@pytest.mark.parametrize("scene", ["teapot", "gopher", "adv:flat", "adv:stairs", "adv:dupes", "adv:far"])
def test_node4_chains_fit_the_walk_stack(scene):
    """The walk's LDS stack holds 3 entries per Node4 level (kStack >= 21 in
    ptmi_kernels.hip): every index the builder emits has chains of <= 7 Node4s, on the
    bench meshes and on the adversarial ones (tests/adversarial.py)."""
    if scene.startswith("adv:"):
        from tests import adversarial
        objs, tris, grps, cam = adversarial.scene_inputs(scene[4:], 32, 24, 0.0, 0.0)
    else:
        objs, tris, grps, cam = scene_inputs(scene, 64, 48)
    st = _stats(objs, tris, grps, cam)
    assert 1 <= st["depth"] <= 7, st


def _tile_cost(objs, tris, grps, cam, w, h):
    import ctypes
    import numpy as np
    from ptmi.api import _ptr, _records, load_library
    lib = load_library()
    lib.ptmi_diag_tile_cost.restype = ctypes.c_int
    lib.ptmi_diag_tile_cost.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32, ctypes.c_char_p,
                                        ctypes.c_size_t]
    objs, tris, grps, cam = _records(objs, tris, grps, cam)
    n = ((w + 7) // 8) * ((h + 7) // 8)
    out = (ctypes.c_uint8 * n)()
    err = ctypes.create_string_buffer(512)
    rc = lib.ptmi_diag_tile_cost(_ptr(objs), len(objs), _ptr(tris), len(tris), _ptr(grps), len(grps), _ptr(cam),
                                 out, n, err, len(err))
    assert rc == 0, err.value
    return np.frombuffer(bytes(out), dtype=np.uint8).reshape((h + 7) // 8, (w + 7) // 8)


@pytest.mark.parametrize("scene", ["teapot", "gopher"])
def test_mesh_tile_classes_mark_the_mesh(scene):
    """The static dispatch classes of a rank's first launch (ptmi_api.cpp mesh_tile_cost):
    0..9 camera rays of 9 per tile pass the mesh hulls' cull.  The mesh covers a block of
    these frames (the teapot's hull 8 %, the gopher's 13 % of the tiles at 320x240), some
    tiles fully, the frame's corners not at all; the classes only order work items
    (tests/test_gpu_order.py checks the image)."""
    w, h = 320, 240
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    c = _tile_cost(objs, tris, grps, cam, w, h)
    assert c.max() == 9 and (c == 9).sum() >= 20, c
    assert c[0, 0] == 0 and c[-1, -1] == 0 and c[0, -1] == 0
    assert 0.02 < (c > 0).mean() < 0.9


def test_tile_classes_are_zero_without_meshes():
    w, h = 64, 48
    objs, tris, grps, cam = scene_inputs("reference", w, h)
    assert _tile_cost(objs, tris, grps, cam, w, h).max() == 0


def test_child_codes_narrow_for_the_baseline_meshes(teapot):
    """Teapot and gopher child codes fit 16 bits: the affine kernels' LDS stack holds them
    (ptmi_bvh.cpp finalize_index_codes)."""
    assert _stats(*teapot)["leaf_bit"] == 0x8000
    assert _stats(*scene_inputs("gopher", 32, 24))["leaf_bit"] == 0x8000


def test_child_codes_wide_past_16_bits():
    """34,848 triangles do not fit 15-bit triangle indices: wide codes (leaf bit 2^30)."""
    from tests import adversarial
    st = _stats(*adversarial.scene_inputs("big", 16, 12))
    assert st["leaf_bit"] == 0x40000000 and st["depth"] <= 7
