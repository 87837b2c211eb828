"""End to end on the GPU: the Go-free CLI (pathtracer-ocl_amd/build/pt, the
cmd/pt counterpart) builds a scene natively, renders through ptmi_trace and
writes the reference's PNG / .raw; its pixels equal the clamped frame that the
Python mirror of ocl.Trace renders from the same records and seeds."""
import os
import struct
import subprocess

import numpy as np
import pytest

from ptmi import api
from tests.scene_inputs import scene_inputs
from tests.test_host import _clamp, _read_png

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PT = os.path.join(ROOT, "pathtracer-ocl_amd", "build", "pt")


@pytest.mark.parametrize("scene,w,h,spp,ap", [("reference", 64, 48, 8, 0.0), ("transparency", 40, 30, 6, 0.15),
                                              ("default", 33, 17, 4, 0.0)])
def test_cli_matches_trace(tmp_path, scene, w, h, spp, ap):
    if not os.path.exists(PT):
        pytest.fail("pt CLI not built")
    png, raw = tmp_path / "o.png", tmp_path / "o.raw"
    fl = 1.6 if ap else 0.0
    cmd = [PT, "--scene", scene, "--width", str(w), "--height", str(h), "--samples", str(spp), "--aperture",
           repr(ap), "--focal-length", repr(fl), "--seed", "4242", "--out", str(png), "--raw", str(raw)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    ref = api.Trace(objs, tris, grps, 0, spp, cam, seed_stream=4242).reshape(h, w, 4)
    px = _read_png(str(png))
    assert np.array_equal(px[..., :3], _clamp(ref[..., :3]))
    body = open(raw, "rb").read()
    assert struct.unpack(">iiii", body[:16]) == (1, 0, w, h)
    assert np.array_equal(np.frombuffer(body[16:], ">f4").reshape(h, w, 3), ref[..., :3].astype(np.float32))


def test_cli_lists(tmp_path):
    r = subprocess.run([PT, "--list-scenes"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "reference" in r.stdout.split()
    r = subprocess.run([PT, "--list-devices"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "Index: 0" in r.stdout


def test_cli_multi_device_flags(tmp_path):
    """--gpus / --split run ptmi_trace_multi (one GPU here: --gpus 1 only)."""
    png = tmp_path / "m.png"
    r = subprocess.run([PT, "--scene", "reference", "--width", "24", "--height", "16", "--samples", "3", "--gpus", "1",
                        "--split", "tile", "--seed", "3", "--out", str(png)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert os.path.getsize(png) > 0


@pytest.mark.parametrize("scene,w,h,spp", [("textures", 48, 32, 4), ("envmap", 40, 30, 4)])
def test_cli_textured_scene(tmp_path, scene, w, h, spp):
    """Textured scenes end to end: images loaded from --assets (PNG stand-ins of
    the reference's missing assets, the .jpg one as a same-stem .png), packed as
    prepareTextures does and sampled on the GPU == api.Trace with the same arrays."""
    from ptmi import scenes
    from tests import textures_synth
    from tests.test_host_images import write_png
    tex = textures_synth.scene_textures(scene)
    for k, key in enumerate(("textures", "sphereTextures", "cubeTextures")):
        for name, img in zip(scenes.TEXTURE_ASSETS[scene].get(key, []), tex[k] or []):
            stem = name.rsplit(".", 1)[0]
            write_png(tmp_path / (stem + ".png"), img.astype(np.int64), 6, 8)
    png = tmp_path / "o.png"
    cmd = [PT, "--scene", scene, "--width", str(w), "--height", str(h), "--samples", str(spp), "--seed", "77",
           "--assets", str(tmp_path), "--out", str(png)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    ref = api.Trace(objs, tris, grps, 0, spp, cam, *tex, seed_stream=77).reshape(h, w, 4)
    assert np.array_equal(_read_png(str(png))[..., :3], _clamp(ref[..., :3]))
    # without the images the CLI fails loudly, as LoadImage panics
    r = subprocess.run(cmd[:-4] + ["--assets", str(tmp_path / "none"), "--out", str(png)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0 and "cannot read" in r.stderr
