"""Synthetic texture arrays for the textured scenes (textures / envmap / cubemap).

The Go scenes load their images from ./assets (scene.go:30-56), and none of those
files is in the reference checkout, so the parity cases use deterministic
stand-ins of the same roles and aspect ratios: NRGBA8 H x W x 4 images (row 0 at
the top, alpha 255 as a decoded opaque PNG/JPEG converted by draw.Draw).  Sizes
are small and deliberately unequal in w and h so that both sampler axes wrap
differently.  A normal map (texture 3 of the "textures" scene) holds
((n + 1) / 2) * 255 of a bumpy unit normal, as a tangent-space map is stored.
"""
import numpy as np


def _rng(tag):
    return np.random.default_rng(sum(map(ord, tag)) * 7919)  # stable across runs (no hash())


def _opaque(rgb):
    h, w, _ = rgb.shape
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = np.clip(rgb, 0, 255).astype(np.uint8)
    out[..., 3] = 255
    return out


def checker(w, h, cell, c0, c1, noise=0, tag="checker"):
    y, x = np.mgrid[0:h, 0:w]
    m = ((x // cell + y // cell) % 2).astype(bool)
    rgb = np.where(m[..., None], np.array(c1, float), np.array(c0, float))
    if noise:
        rgb = rgb + _rng(tag).integers(-noise, noise + 1, size=rgb.shape)
    return _opaque(rgb)


def gradient(w, h, tag="gradient"):
    y, x = np.mgrid[0:h, 0:w]
    rgb = np.stack([255.0 * x / max(w - 1, 1), 255.0 * y / max(h - 1, 1), 128 + 100 * np.sin(x * 0.3 + y * 0.2)],
                   axis=-1)
    return _opaque(rgb + _rng(tag).integers(-6, 7, size=rgb.shape))


def normal_map(w, h):
    y, x = np.mgrid[0:h, 0:w]
    nx = 0.35 * np.sin(2 * np.pi * x / w * 3)
    nz = 0.35 * np.cos(2 * np.pi * y / h * 2)
    ny = np.ones_like(nx)
    n = np.stack([nx, ny, nz], axis=-1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    return _opaque(np.rint((n + 1.0) * 0.5 * 255.0))


def cube_cross(w, h):
    """4:3 cross layout (cubeUV, tracer.cl:113-175): each face a distinct tint."""
    img = gradient(w, h, tag="cube").astype(float)
    fw, fh = w // 4, h // 3
    tints = {(1, 0): (1.0, .6, .6), (0, 1): (.6, 1.0, .6), (1, 1): (.6, .6, 1.0), (2, 1): (1.0, 1.0, .5),
             (3, 1): (.5, 1.0, 1.0), (1, 2): (1.0, .5, 1.0)}
    for (cx, cy), t in tints.items():
        img[cy * fh:(cy + 1) * fh, cx * fw:(cx + 1) * fw, :3] *= t
    return _opaque(img[..., :3])


def scene_textures(name, scale=1):
    """[textures, sphereTextures, cubeTextures] for a textured scene (None: untextured)."""
    s = int(scale)
    if name == "textures":
        w, h = 48 * s, 40 * s
        return [[checker(w, h, 6, (200, 60, 40), (240, 220, 200), noise=12, tag="squares"),
                 checker(w, h, 5, (90, 90, 90), (170, 160, 150), noise=30, tag="cobble"),
                 gradient(w, h, tag="boards"),
                 normal_map(w, h)],
                [gradient(64 * s, 32 * s, tag="planet"), checker(64 * s, 32 * s, 4, (180, 120, 60), (240, 200, 150),
                                                                 noise=20, tag="jupiter")],
                None]
    if name == "envmap":
        return [None, [gradient(96 * s, 48 * s, tag="alps")], None]
    if name == "cubemap":
        return [None, None, [cube_cross(64 * s, 48 * s)]]
    return None
