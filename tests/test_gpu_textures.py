"""Textures on the GPU: the HIP kernel's software sampler and UV maps against the
CPU oracle's restatement (oracle/pt_oracle.c), on the reference's three textured
scenes (textures / envmap / cubemap) with synthetic images of the same roles
(tests/textures_synth.py; the reference's image assets are not in its checkout).

PARITY UNPINNED against the reference kernel: its read_imagef cannot run on
gfx950 (no image instructions; DESIGN.md "Textures").  The HIP kernel and the
oracle run the same FP32 sampler sequence and the same double UV arithmetic;
they differ only where sphericalMap calls atan2/acos (ocml on the GPU, glibc on
the CPU: last-ulp differences that the float cast of u/v absorbs).  Tolerance
1e-9, stated here; observed agreement is reported in the assertion messages.
"""
import ctypes

import numpy as np
import pytest

import pyoracle
from ptmi import api, layout
from tests import textures_synth
from tests.scene_inputs import scene_inputs

pytestmark = pytest.mark.gpu
TOL_TEX = 1e-9


@pytest.mark.parametrize("scene,w,h,spp,ap,seed", [
    ("textures", 64, 48, 4, 0.0, 201),
    ("textures", 48, 32, 3, 0.15, 202),
    ("envmap", 64, 48, 4, 0.0, 203),
    ("cubemap", 48, 32, 3, 0.0, 204),
])
def test_hip_textures_match_cpu_oracle(scene, w, h, spp, ap, seed):
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, 1.6 if ap else 0.0)
    tex = textures_synth.scene_textures(scene)
    seeds = layout.seeds_go_float64(w * h, seed)
    t2, g2 = layout.pad_empty(tris, grps)
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds, textures=tex)
    out = api.Trace(objs, tris, grps, 0, spp, cam, *tex, seeds=seeds)
    err = np.abs(out - ora).max()
    assert err < TOL_TEX, "%s: L-inf %.3e vs CPU oracle" % (scene, err)
    # the textures are visible: without them (the all-zero fake image) the frame changes
    blank = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(out - blank).max() > 1e-3


def test_hip_missing_textures_are_the_zero_image():
    """No texture arrays with textured objects = the reference's 1024x1024 all-zero
    fake image (ocltracer.go:249-251): black colours, zero normal maps."""
    w, h, spp = 40, 24, 3
    objs, tris, grps, cam = scene_inputs("textures", w, h)
    seeds = layout.seeds_go_float64(w * h, 205)
    t2, g2 = layout.pad_empty(tris, grps)
    ora = pyoracle.cpu_trace(objs, t2, g2, cam, spp, seeds)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(out - ora).max() < TOL_TEX


def test_hip_uniform_texture_equals_object_colour():
    w, h, spp = 48, 32, 3
    objs, tris, grps, cam = scene_inputs("envmap", w, h)
    seeds = layout.seeds_go_float64(w * h, 206)
    c = (51, 153, 204)
    sky = [np.tile(np.array(list(c) + [255], np.uint8), (4, 8, 1))]
    plain = objs.copy()
    plain["color"][1][:3] = np.float32(np.array(c) / 255.0).astype(np.float64)
    plain["is_textured"][1] = 0
    a = api.Trace(objs, tris, grps, 0, spp, cam, None, sky, None, seeds=seeds)
    b = api.Trace(plain, tris, grps, 0, spp, cam, seeds=seeds)
    assert np.abs(a - b).max() < 1e-5


def test_hip_textured_scene_sample_split():
    """Resident-scene API with textures: sample ranges sum to the full frame."""
    import torch
    w, h, S = 40, 24, 6
    objs, tris, grps, cam = scene_inputs("textures", w, h)
    tex = textures_synth.scene_textures("textures")
    sc = api.Scene(0, objs, tris, grps, cam, *tex)
    n = w * h
    seeds = torch.tensor(layout.seeds_go_float64(n, 207), dtype=torch.float64, device="cuda")
    full = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    part = torch.empty_like(full)
    sc.render(S, 0, S, seeds.data_ptr(), full.data_ptr())
    acc = torch.zeros_like(full)
    for a, b in ((0, 2), (2, 6)):
        sc.render(S, a, b, seeds.data_ptr(), part.data_ptr(), chunks=2)
        acc += part
    torch.cuda.synchronize()
    assert (acc - full).abs().max().item() < 1e-12


def test_hip_texture_argument_errors():
    objs, tris, grps, cam = scene_inputs("textures", 8, 8)
    lib = api.load_library()
    from ptmi.textures import PtmiTextures
    t = PtmiTextures()
    t.count[0], t.width[0], t.height[0] = 1, 4, 4  # NULL pixels
    out = np.empty(8 * 8 * 4)
    err = ctypes.create_string_buffer(256)
    rc = lib.ptmi_trace(objs.ctypes.data, len(objs), None, 0, None, 0, 0, 1, np.asarray(cam).ctypes.data, None, 1,
                        ctypes.cast(ctypes.pointer(t), ctypes.c_void_p), out.ctypes.data, err, 256)
    assert rc == api.PTMI_ERR_ARG and b"texture array 0" in err.value
