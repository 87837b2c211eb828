"""The cgo binding's call sequence on the GPU (go/ocltracer_hip.go).

This image has no Go toolchain, so tests/go_abi/go_sequence.c makes the binding's C
calls instead: ptmi_trace with `&slice[0]` records (NULL for empty slices), W*H
seeds, an all-zero ptmi_textures, a caller-owned output and a 512-byte error buffer;
the deviceIndex contract (ocltracer.go:135-140); then ptmi_trace_multi with a
C-allocated device list, tile and sample split.  Its frame must equal the Python
binding's ptmi_trace on the same records and seeds bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from ptmi import api
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
BIN = os.path.join(ROOT, "tests", "go_abi", "build", "go_sequence")


@pytest.mark.parametrize("scene,w,h,spp", [("reference", 96, 64, 24), ("default", 64, 48, 16)])
def test_go_call_sequence(tmp_path, scene, w, h, spp):
    if not os.path.exists(BIN):
        pytest.fail("tests/go_abi/build/go_sequence not built (__graft_entry__.build())")
    r = subprocess.run([BIN, scene, str(w), str(h), str(spp), str(tmp_path)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    ld = lambda n: np.fromfile(os.path.join(tmp_path, n), dtype=np.float64)  # noqa: E731
    seeds, trace, tile, smp = ld("seeds.f64"), ld("trace.f64"), ld("multi_tile.f64"), ld("multi_sample.f64")
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    want = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.array_equal(trace, want)
    assert np.array_equal(tile, want)
    assert np.abs(smp - want).max() < 1e-12
