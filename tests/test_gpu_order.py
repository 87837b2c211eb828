"""Mesh scenes dispatch their chunked tiles costliest first (ptmi_api.cpp render: the static
hull-hit classes; in the study library also the order tile_order_kernel derives from the
last launch's measured item durations).  Only the order in which work items run changes:
each tile keeps its partial slots and the reduction's chunk order, so every launch's sums
must equal the raster-order launch's bit for bit, whatever the order was."""
import os

import numpy as np
import pytest

from ptmi import api, layout
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu


def _renders(order, scene, w, h, spp, n, stride=1, offset=0, chunks=0, lib=None):
    import torch
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    sc = api.Scene(0, objs, tris, grps, cam, lib=lib)
    assert sc.set_knob(api.KNOB_TILE_ORDER, order) == api.PTMI_OK
    seeds = torch.tensor(layout.seeds_go_float64(w * h, 77), dtype=torch.float64, device="cuda")
    out = []
    for _ in range(n):
        sums = torch.empty(w * h * 4, dtype=torch.float64, device="cuda")
        sc.render(spp, 0, spp, seeds.data_ptr(), sums.data_ptr(), tile_stride=stride, tile_offset=offset,
                  chunks=chunks)
        torch.cuda.synchronize()
        out.append(sums.cpu().numpy())
    sc.close()
    return out


@pytest.mark.parametrize("scene", ["teapot", "gopher"])
@pytest.mark.parametrize("stride,offset", [(1, 0), (3, 1)])
def test_tile_order_never_changes_the_sums(scene, stride, offset):
    w, h, spp = 320, 240, 48
    raster = _renders(0, scene, w, h, spp, 1, stride, offset, chunks=4)[0]
    static = _renders(1, scene, w, h, spp, 2, stride, offset, chunks=4)
    for m in static:
        assert np.array_equal(raster, m)


def test_measured_order_is_study_only():
    """The product library has no item timing: the measured order (2) is refused."""
    objs, tris, grps, cam = scene_inputs("teapot", 64, 48)
    sc = api.Scene(0, objs, tris, grps, cam)
    assert sc.set_knob(api.KNOB_TILE_ORDER, 2) == api.PTMI_ERR_UNSUPPORTED
    sc.close()


@pytest.mark.parametrize("scene", ["teapot", "gopher"])
def test_measured_order_never_changes_the_sums(scene):
    """Study library: launches 2 and 3 run the order measured by the launch before."""
    if not os.path.exists(api.STUDY_LIB_PATH):
        pytest.fail("libptmi_study.so not built (make -C pathtracer-ocl_amd study)")
    study = api.load_library(api.STUDY_LIB_PATH)
    w, h, spp = 320, 240, 48
    # (the study library is built without the product's path pool: its raster launch is the reference)
    raster = _renders(0, scene, w, h, spp, 1, 3, 1, chunks=4, lib=study)[0]
    measured = _renders(2, scene, w, h, spp, 3, 3, 1, chunks=4, lib=study)
    for m in measured:  # launch 1: static order; launches 2, 3: orders from measured costs
        assert np.array_equal(raster, m)
