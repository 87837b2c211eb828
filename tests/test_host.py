"""The native host side (libptmi_host.so, include/ptmi_host.h; SURVEY.md 8f rows
3-4) on CPU: its C++ restatement of the Go scene build produces the SAME record
bytes as ptmi's Python restatement -- which the reference-kernel goldens pin --
for every scene, and its writers follow pathtracer.go:40-59 (PNG clamp) and
raw/writer.go:11-35 (.raw)."""
import ctypes
import os
import struct
import zlib

import numpy as np
import pytest

from ptmi import layout, scenes
from tests.scene_inputs import MESH_SCENES, scene_inputs

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "pathtracer-ocl_amd", "build", "libptmi_host.so")
ASSETS = scenes.ASSETS


class Records(ctypes.Structure):
    _fields_ = [("objects", ctypes.c_void_p), ("n_obj", ctypes.c_uint32), ("triangles", ctypes.c_void_p),
                ("n_tri", ctypes.c_uint32), ("groups", ctypes.c_void_p), ("n_grp", ctypes.c_uint32),
                ("camera", ctypes.c_uint8 * 256)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libptmi_host.so not built: run __graft_entry__.build() / make -C pathtracer-ocl_amd")
    lib = ctypes.CDLL(LIB)
    lib.ptmi_host_build_scene.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_char_p, ctypes.POINTER(Records),
                                          ctypes.c_char_p, ctypes.c_size_t]
    lib.ptmi_host_free_records.argtypes = [ctypes.POINTER(Records)]
    lib.ptmi_host_scene_names.restype = ctypes.c_char_p
    for f in (lib.ptmi_host_write_png, lib.ptmi_host_write_raw):
        f.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    return lib


def _build(lib, name, w, h, ap=0.0, fl=0.0, assets=ASSETS):
    r = Records()
    err = ctypes.create_string_buffer(512)
    rc = lib.ptmi_host_build_scene(name.encode(), w, h, ap, fl, assets.encode(), ctypes.byref(r), err, 512)
    if rc:
        raise RuntimeError("rc=%d: %s" % (rc, err.value.decode()))

    def take(p, n, dt):
        if n == 0:
            return np.zeros(0, dt)
        return np.frombuffer(ctypes.string_at(p, n * dt.itemsize), dtype=dt).copy()
    out = (take(r.objects, r.n_obj, layout.OBJECT_DTYPE), take(r.triangles, r.n_tri, layout.TRIANGLE_DTYPE),
           take(r.groups, r.n_grp, layout.GROUP_DTYPE), bytes(r.camera))
    lib.ptmi_host_free_records(ctypes.byref(r))
    return out


def test_scene_names(lib):
    names = lib.ptmi_host_scene_names().decode().split()
    assert set(names) == set(scenes.SCENES)


@pytest.mark.parametrize("name", sorted(set(scenes.SCENES) - set(MESH_SCENES) - {"glass"}))
@pytest.mark.parametrize("w,h,ap,fl", [(64, 48, 0.0, 0.0), (37, 91, 0.15, 1.6)])
def test_records_match_python_restatement(lib, name, w, h, ap, fl):
    objs, tris, grps, cam = _build(lib, name, w, h, ap, fl)
    po, pt, pg, pc = scene_inputs(name, w, h, ap, fl)
    assert objs.tobytes() == po.tobytes()
    assert tris.tobytes() == pt.tobytes()
    assert grps.tobytes() == pg.tobytes()
    assert cam == np.asarray(pc).reshape(1).tobytes()


@pytest.mark.parametrize("name", MESH_SCENES)
def test_mesh_records_match_fixtures(lib, name):
    if not os.path.exists(os.path.join(ASSETS, "teapot.obj")):
        pytest.skip("OBJ assets not present (reference checkout)")
    objs, tris, grps, cam = _build(lib, name, 64, 48)
    po, pt, pg, pc = scene_inputs(name, 64, 48)  # fixture records (shared meshes resolved)
    assert objs.tobytes() == po.tobytes()
    assert tris.tobytes() == pt.tobytes()
    assert grps.tobytes() == pg.tobytes()
    assert cam == np.asarray(pc).reshape(1).tobytes()


def test_glass_scene_needs_its_missing_mesh(lib):
    """GlassScene reads assets/glass.obj, which the reference does not ship: both
    restatements fail loudly, as the Go os.ReadFile panic does."""
    with pytest.raises(RuntimeError, match="glass.obj"):
        _build(lib, "glass", 16, 12)
    with pytest.raises(FileNotFoundError):
        scenes.SCENES["glass"](16, 12)


def test_errors(lib):
    with pytest.raises(RuntimeError, match="unknown scene"):
        _build(lib, "no-such-scene", 8, 8)
    with pytest.raises(RuntimeError, match="cannot read"):
        _build(lib, "teapot", 8, 8, assets="/nonexistent")


def _clamp(v):  # pathtracer.go:50-59 (math.Round: half away from zero)
    r = np.floor(np.abs(v) * 255.0 + 0.5) * np.sign(v)
    return np.clip(r, 0, 255).astype(np.uint8)


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body)
        if typ == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert (depth, ctype) == (8, 6)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * 4 + 1)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 4)


def test_png_and_raw_writers(lib, tmp_path):
    w, h = 13, 7
    rng = np.random.default_rng(0)
    img = rng.uniform(-0.2, 1.3, (h, w, 4))
    img[0, 0, :3] = [0.5 / 255, 1.5 / 255, 254.5 / 255]  # halves round away from zero
    buf = np.ascontiguousarray(img.ravel())
    err = ctypes.create_string_buffer(256)
    png, raw = str(tmp_path / "x.png"), str(tmp_path / "x.raw")
    assert lib.ptmi_host_write_png(png.encode(), buf.ctypes.data, w, h, err, 256) == 0
    px = _read_png(png)
    assert np.array_equal(px[..., :3], _clamp(img[..., :3])) and (px[..., 3] == 255).all()
    assert lib.ptmi_host_write_raw(raw.encode(), buf.ctypes.data, w, h, err, 256) == 0
    want = struct.pack(">iiii", 1, 0, w, h) + img[..., :3].astype(">f4").tobytes()
    assert open(raw, "rb").read() == want
