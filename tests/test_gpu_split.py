"""The split form of the mesh scenes (ptmi_kernels.hip trace_split_kernel + walk_split_kernel,
DESIGN.md section 5) against the one-kernel form: same chunking -> the same frame sums bit
for bit (every sample of a pixel-chunk runs in order with the same arithmetic; the walks are
group_walks either way).  The split form is a measured alternative, off by default (DESIGN.md
section 5); the product's one-kernel form is pinned to the reference by test_gpu_parity.py and
test_gpu_fullres.py, so equality with it pins the split form too.  The split form lives in
the study library (make -C pathtracer-ocl_amd study), not in the product."""
import os

import numpy as np
import pytest
import torch

from ptmi import api, layout
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu


def _study():
    if not os.path.exists(api.STUDY_LIB_PATH):
        pytest.fail("libptmi_study.so not built (make -C pathtracer-ocl_amd study)")
    return api.load_library(api.STUDY_LIB_PATH)


def test_product_has_no_split_form():
    objs, tris, grps, cam = scene_inputs("teapot", 64, 48)
    scene = api.Scene(0, objs, tris, grps, cam)
    assert not scene.set_split(True)
    assert scene.set_split(False)
    scene.close()


def _sums(scene, S, seeds, chunks, split, w, h, s0=0, s1=None, stride=1, off=0):
    assert scene.set_split(split)
    sums = torch.zeros(w * h * 4, dtype=torch.float64, device="cuda")
    scene.render(S, s0, S if s1 is None else s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=stride,
                 tile_offset=off, chunks=chunks)
    torch.cuda.synchronize()
    return sums.cpu().numpy()


@pytest.mark.parametrize("name,w,h,S,chunks,ap", [
    ("teapot", 128, 96, 48, 4, 0.0),
    ("gopher", 96, 64, 40, 5, 0.0),
    ("teapot", 64, 48, 24, 3, 0.15),
    ("transparent_teapot", 64, 48, 16, 2, 0.0),
])
def test_split_equals_one_kernel_form(name, w, h, S, chunks, ap):
    objs, tris, grps, cam = scene_inputs(name, w, h, ap, 1.6 if ap else 0.0)
    scene = api.Scene(0, objs, tris, grps, cam, lib=_study())
    seeds = torch.tensor(layout.seeds_go_float64(w * h, 77), dtype=torch.float64, device="cuda")
    a = _sums(scene, S, seeds, chunks, True, w, h)
    assert scene.split_passes() > 1
    b = _sums(scene, S, seeds, chunks, False, w, h)
    scene.close()
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), "max |diff| %.3e" % np.abs(a - b).max()


def test_split_sample_range_and_tile_split():
    """Sample sub-ranges and tile ownership (the multi-GPU shards) in the split form."""
    w, h, S = 96, 64, 32
    objs, tris, grps, cam = scene_inputs("teapot", w, h)
    scene = api.Scene(0, objs, tris, grps, cam, lib=_study())
    seeds = torch.tensor(layout.seeds_go_float64(w * h, 78), dtype=torch.float64, device="cuda")
    # (stride 5: 12 tiles per row do not divide by it, so the one-kernel form keeps the raster
    # ownership the split form uses -- with 3 it would take the diagonal one, ptmi_api.cpp render)
    for kw in ({"s0": 8, "s1": 24}, {"stride": 5, "off": 1}):
        a = _sums(scene, S, seeds, 2, True, w, h, **kw)
        b = _sums(scene, S, seeds, 2, False, w, h, **kw)
        assert np.array_equal(a.view(np.int64), b.view(np.int64)), kw
    scene.close()


def test_split_pool_smaller_than_the_work():
    """More pixel-chunks than slots (640x480 x 8 chunks = 2.46 M > the 1.3 M-slot pool):
    slots claim chunk after chunk across passes, and a wave's claimed block survives the
    pass it was claimed in."""
    w, h, S = 640, 480, 64
    objs, tris, grps, cam = scene_inputs("teapot", w, h)
    scene = api.Scene(0, objs, tris, grps, cam, lib=_study())
    seeds = torch.tensor(layout.seeds_go_float64(w * h, 79), dtype=torch.float64, device="cuda")
    a = _sums(scene, S, seeds, 8, True, w, h)
    b = _sums(scene, S, seeds, 8, False, w, h)
    scene.close()
    assert np.array_equal(a.view(np.int64), b.view(np.int64)), "max |diff| %.3e" % np.abs(a - b).max()
