"""Texture arrays for ``Trace`` / ``Scene``: the Python side of ``ptmi_textures``.

The reference passes ``textures, sphereTextures, cubeTextures []image.Image``
(ocltracer.go:100) and ``prepareTextures`` (ocltracer.go:228-254) turns each list
into one RGBA UNORM8 ``image2d_array``: width/height of the first image, the
``image.NRGBA.Pix`` bytes of every image concatenated.  Here an image is an
``H x W x 4`` uint8 array of NRGBA pixels (row 0 = top, as ``Pix``); every image
of one list must have the first image's size (the OpenCL image array requires
it; the reference would read past a smaller one).
"""
import ctypes

import numpy as np


class PtmiTextures(ctypes.Structure):
    """include/ptmi.h ``ptmi_textures``."""
    _fields_ = [("pixels", ctypes.c_void_p * 3), ("width", ctypes.c_uint32 * 3), ("height", ctypes.c_uint32 * 3),
                ("count", ctypes.c_uint32 * 3)]


def pack_array(images):
    """One texture list -> (contiguous uint8 [n, H, W, 4] array or None, W, H, n)."""
    if images is None or len(images) == 0:
        return None, 0, 0, 0
    imgs = [np.asarray(im) for im in images]
    h, w = imgs[0].shape[:2]
    for k, im in enumerate(imgs):
        if im.dtype != np.uint8 or im.ndim != 3 or im.shape[2] != 4:
            raise TypeError("texture %d: expected an H x W x 4 uint8 NRGBA image, got %s %s" % (k, im.dtype, im.shape))
        if im.shape[:2] != (h, w):
            raise ValueError("texture %d: %dx%d, but the array's first image is %dx%d (image2d_array layers share "
                             "one size, ocltracer.go:233-236)" % (k, im.shape[1], im.shape[0], w, h))
    return np.ascontiguousarray(np.stack(imgs)), w, h, len(imgs)


class TextureSet:
    """The three texture arrays, packed once; ``.struct`` is the ``ptmi_textures``
    to pass (NULL-equivalent when every list is empty); the arrays stay alive
    with this object."""

    def __init__(self, textures=None, sphereTextures=None, cubeTextures=None):
        self.arrays = [pack_array(t) for t in (textures, sphereTextures, cubeTextures)]
        self.struct = PtmiTextures()
        for k, (a, w, h, n) in enumerate(self.arrays):
            self.struct.pixels[k] = a.ctypes.data if a is not None else None
            self.struct.width[k], self.struct.height[k], self.struct.count[k] = w, h, n

    @property
    def empty(self):
        return all(n == 0 for _, _, _, n in self.arrays)

    def pointer(self):
        return None if self.empty else ctypes.cast(ctypes.pointer(self.struct), ctypes.c_void_p)

    def oracle_args(self):
        """(pixels*, w*, h*, n*) for oracle/pt_oracle.c pto_trace_tex."""
        pix = (ctypes.c_void_p * 3)(*[a.ctypes.data if a is not None else None for a, _, _, _ in self.arrays])
        w = (ctypes.c_uint32 * 3)(*[x[1] for x in self.arrays])
        h = (ctypes.c_uint32 * 3)(*[x[2] for x in self.arrays])
        n = (ctypes.c_uint32 * 3)(*[x[3] for x in self.arrays])
        return pix, w, h, n
