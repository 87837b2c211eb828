"""Mesh scenes dispatch their chunked tiles costliest first (ptmi_api.cpp render: the static
hull-hit classes on a rank's first launch, then the order tile_order_kernel derives from the
last launch's measured item durations).  Only the order in which work items run changes:
each tile keeps its partial slots and the reduction's chunk order, so every launch's sums
must equal the raster-order launch's bit for bit, whatever the measured order was."""
import numpy as np
import pytest

from ptmi import api, layout
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu


def _renders(monkeypatch, order, scene, w, h, spp, n, stride=1, offset=0, chunks=0):
    import torch
    monkeypatch.setenv("PTMI_TILE_ORDER", str(order))
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    sc = api.Scene(0, objs, tris, grps, cam)
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
def test_tile_order_never_changes_the_sums(monkeypatch, scene, stride, offset):
    w, h, spp = 320, 240, 48
    raster = _renders(monkeypatch, 0, scene, w, h, spp, 1, stride, offset, chunks=4)[0]
    static = _renders(monkeypatch, 1, scene, w, h, spp, 1, stride, offset, chunks=4)[0]
    measured = _renders(monkeypatch, 2, scene, w, h, spp, 3, stride, offset, chunks=4)
    assert np.array_equal(raster, static)
    for m in measured:  # launch 1: static order; launches 2, 3: orders from measured costs
        assert np.array_equal(raster, m)
