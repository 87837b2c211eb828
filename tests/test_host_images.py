"""Texture image loading of the native host side (libptmi_host.so images.cpp):
LoadImage (scene.go:30-56) = image/png decode + draw.Draw into NRGBA, and
prepareTextures packing (ocltracer.go:228-254).

PNG files are written here by a small independent encoder covering every colour
type / bit depth Go's reader accepts, all five filters, tRNS and Adam7; the
expected NRGBA bytes follow Go 1.19's image/color conversions (spelled out in
``_expected``).  No reference image ships with the reference checkout, so the
cases are synthetic."""
import ctypes
import os
import struct
import zlib

import numpy as np
import pytest

from tests.test_host import LIB

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


class Tex(ctypes.Structure):
    _fields_ = [("pixels", ctypes.c_void_p * 3), ("width", ctypes.c_uint32 * 3), ("height", ctypes.c_uint32 * 3),
                ("count", ctypes.c_uint32 * 3)]


@pytest.fixture(scope="module")
def lib():
    lib = ctypes.CDLL(LIB)
    lib.ptmi_host_load_image.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.c_char_p, ctypes.c_size_t]
    lib.ptmi_host_free_image.argtypes = [ctypes.c_void_p]
    lib.ptmi_host_load_scene_textures.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Tex),
                                                  ctypes.c_char_p, ctypes.c_size_t]
    lib.ptmi_host_free_textures.argtypes = [ctypes.POINTER(Tex)]
    return lib


def load(lib, path):
    p, w, h = ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_uint32()
    err = ctypes.create_string_buffer(512)
    rc = lib.ptmi_host_load_image(str(path).encode(), ctypes.byref(p), ctypes.byref(w), ctypes.byref(h), err, 512)
    if rc:
        raise RuntimeError(err.value.decode())
    out = np.frombuffer(ctypes.string_at(p, w.value * h.value * 4), np.uint8).reshape(h.value, w.value, 4).copy()
    lib.ptmi_host_free_image(p)
    return out


# ---- a minimal PNG encoder ------------------------------------------------------
def _chunk(t, body):
    return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xffffffff)


def _pack_rows(samples, depth):
    """samples: (h, w*channels) ints -> (h, rowbytes) uint8."""
    h, n = samples.shape
    if depth == 16:
        return samples.astype(">u2").view(np.uint8).reshape(h, n * 2)
    if depth == 8:
        return samples.astype(np.uint8)
    per = 8 // depth
    rb = (n + per - 1) // per
    out = np.zeros((h, rb), np.uint8)
    for i in range(n):
        out[:, i // per] |= (samples[:, i].astype(np.uint8) << (8 - depth * (i % per + 1))).astype(np.uint8)
    return out


def _filter(rows, bpp, ftype):
    out = []
    prev = np.zeros(rows.shape[1], np.int32)
    for y, r in enumerate(rows.astype(np.int32)):
        f = ftype if ftype is not None else y % 5
        a = np.concatenate([np.zeros(bpp, np.int32), r[:-bpp]]) if len(r) > bpp else np.zeros_like(r)
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]]) if len(r) > bpp else np.zeros_like(r)
        if f == 0:
            d = r
        elif f == 1:
            d = r - a
        elif f == 2:
            d = r - prev
        elif f == 3:
            d = r - (a + prev) // 2
        else:
            p = a + prev - c
            pa, pb, pc = abs(p - a), abs(p - prev), abs(p - c)
            d = r - np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
        out.append(bytes([f]) + (d & 0xff).astype(np.uint8).tobytes())
        prev = r
    return b"".join(out)


def write_png(path, samples, ctype, depth, palette=None, trns=None, interlace=False, ftype=None):
    """samples: (h, w, channels) ints at `depth`."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    if interlace:
        data = b""
        for x0, y0, dx, dy in ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.size:
                data += _filter(_pack_rows(sub.reshape(sub.shape[0], -1), depth), bpp, ftype)
    else:
        data = _filter(_pack_rows(samples.reshape(h, -1), depth), bpp, ftype)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        png += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).ravel()))
    if trns is not None:
        png += _chunk(b"tRNS", trns)
    png += _chunk(b"IDAT", zlib.compress(data)) + _chunk(b"IEND", b"")
    open(path, "wb").write(png)


# ---- Go 1.19 image/color semantics ------------------------------------------------
def _model(r, g, b, a):  # color.NRGBAModel of premultiplied 16-bit values
    if a == 0xffff:
        return [r >> 8, g >> 8, b >> 8, 0xff]
    if a == 0:
        return [0, 0, 0, 0]
    return [((r * 0xffff) // a) >> 8, ((g * 0xffff) // a) >> 8, ((b * 0xffff) // a) >> 8, a >> 8]


def _nrgba8(R, G, B, A):  # color.NRGBA.RGBA()
    f = lambda c: ((c | c << 8) * A) // 0xff  # noqa: E731
    return _model(f(R), f(G), f(B), A | A << 8)


def _nrgba16(R, G, B, A):  # color.NRGBA64.RGBA()
    return _model(R * A // 0xffff, G * A // 0xffff, B * A // 0xffff, A)


def _expected(samples, ctype, depth, palette=None, trns_key=None):
    h, w, _ = samples.shape
    out = np.zeros((h, w, 4), np.int64)
    scale = {1: 0xff, 2: 0x55, 4: 0x11, 8: 1}
    for y in range(h):
        for x in range(w):
            s = [int(v) for v in samples[y, x]]
            if ctype == 0:
                if depth == 16:
                    out[y, x] = _nrgba16(s[0], s[0], s[0], 0) if s[0] == trns_key else [s[0] >> 8] * 3 + [255]
                else:
                    g = s[0] * scale[depth]
                    out[y, x] = [g, g, g, 0 if s[0] == trns_key else 255]
            elif ctype == 2:
                if depth == 16:
                    out[y, x] = _nrgba16(*s, 0) if tuple(s) == trns_key else [v >> 8 for v in s] + [255]
                else:
                    out[y, x] = s + [0 if tuple(s) == trns_key else 255]
            elif ctype == 3:
                c = list(palette[s[0]]) if s[0] < len(palette) else [0, 0, 0, 255]
                out[y, x] = _nrgba8(*c)
            elif ctype == 4:
                out[y, x] = _nrgba16(s[0], s[0], s[0], s[1]) if depth == 16 else [s[0]] * 3 + [s[1]]
            else:
                out[y, x] = _nrgba16(*s) if depth == 16 else s
    return out.astype(np.uint8)


CASES = [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16), (2, 8), (2, 16), (3, 1), (3, 2), (3, 4), (3, 8), (4, 8), (4, 16),
         (6, 8), (6, 16)]


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ctype,depth", CASES)
def test_png_decode_matches_go_semantics(lib, tmp_path, ctype, depth, interlace):
    rng = np.random.default_rng(ctype * 100 + depth + 7 * interlace)
    w, h = 13, 11
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    hi = (1 << depth) - 1
    samples = rng.integers(0, hi + 1, size=(h, w, ch))
    palette, trns, key, pal_rgba = None, None, None, None
    if ctype == 3:
        n = min(1 << depth, 6)
        palette = rng.integers(0, 256, size=(n, 3))
        alphas = rng.integers(0, 256, size=n - 2)  # tRNS for the first n-2 entries
        trns = bytes(alphas.astype(np.uint8))
        pal_rgba = [list(palette[i]) + [int(alphas[i]) if i < n - 2 else 255] for i in range(n)]
        samples[0, 0, 0] = hi if hi >= n else samples[0, 0, 0]  # an index past the palette when possible
    elif ctype in (0, 2):
        key = tuple(int(v) for v in samples[1, 2]) if ctype == 2 else int(samples[1, 2, 0])
        vals = key if ctype == 2 else (key,)
        trns = b"".join(struct.pack(">H", v) for v in vals)
    path = tmp_path / "t.png"
    write_png(path, samples, ctype, depth, palette, trns, interlace, ftype=None)
    got = load(lib, path)
    want = _expected(samples, ctype, depth, pal_rgba, key)
    assert np.array_equal(got, want)


def test_jpeg_assets_need_a_png_stand_in(lib, tmp_path):
    s = np.random.default_rng(1).integers(0, 256, size=(4, 5, 3))
    with pytest.raises(RuntimeError, match="JPEG decoding"):
        load(lib, tmp_path / "x.jpg")
    write_png(tmp_path / "x.png", s, 2, 8)
    assert np.array_equal(load(lib, tmp_path / "x.jpeg")[..., :3], s)
    with pytest.raises(RuntimeError, match="cannot read"):
        load(lib, tmp_path / "none.png")
    (tmp_path / "bad.png").write_bytes(b"not a png")
    with pytest.raises(RuntimeError, match="not a PNG"):
        load(lib, tmp_path / "bad.png")


def test_scene_textures_are_packed_like_prepare_textures(lib, tmp_path):
    """texturedplanets: 4 textures (the first image's size; Pix concatenated, a
    shorter image zero-filled) and 2 sphere textures; envmap: 1 sphere texture."""
    rng = np.random.default_rng(3)
    imgs = {}
    for name, (w, h) in {"concrete_squares.png": (6, 4), "seamless-cobblestone-texture.png": (6, 4),
                         "floor_boards.png": (3, 2), "concrete_squares_nm2.png": (6, 4), "planet.png": (8, 4),
                         "jupiter2_6k_contrast.png": (8, 4)}.items():
        a = rng.integers(0, 256, size=(h, w, 4))
        write_png(tmp_path / name, a, 6, 8)
        imgs[name] = a.astype(np.uint8)
    t = Tex()
    err = ctypes.create_string_buffer(512)
    assert lib.ptmi_host_load_scene_textures(b"textures", str(tmp_path).encode(), ctypes.byref(t), err, 512) == 0, \
        err.value
    assert list(t.count) == [4, 2, 0] and list(t.width) == [6, 8, 0] and list(t.height) == [4, 4, 0]
    got = np.frombuffer(ctypes.string_at(t.pixels[0], 4 * 6 * 4 * 4), np.uint8)
    cat = np.concatenate([imgs[n].ravel() for n in ("concrete_squares.png", "seamless-cobblestone-texture.png",
                                                    "floor_boards.png", "concrete_squares_nm2.png")])
    want = np.zeros(4 * 6 * 4 * 4, np.uint8)
    want[:cat.size] = cat
    assert np.array_equal(got, want)
    lib.ptmi_host_free_textures(ctypes.byref(t))
    assert list(t.count) == [0, 0, 0]
    assert lib.ptmi_host_load_scene_textures(b"reference", str(tmp_path).encode(), ctypes.byref(t), err, 512) == 0
    assert list(t.count) == [0, 0, 0]
    assert lib.ptmi_host_load_scene_textures(b"envmap", str(tmp_path).encode(), ctypes.byref(t), err, 512) != 0
    assert b"alps_field_8k.png" in err.value
