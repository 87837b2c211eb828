"""ctypes binding of libptmi.so (include/ptmi.h).

``Trace`` mirrors the reference's Go entry point
``internal/ocl.Trace(objects, triangles, groups, deviceIndex, samples, camera,
textures, sphereTextures, cubeTextures) []float64`` (ocltracer.go:98-226): same
argument meaning, same record bytes, same float64 RGBA result.  Where the Go code
calls ``logrus.Fatalf`` this raises ``PtmiError`` (the library returned an error
code; nothing falls back to another implementation).

``Scene`` exposes the resident-scene API (scene uploaded to HBM once, frames
rendered from device buffers on a caller's HIP stream) used by bench.py and
the multi-GPU driver; device buffers are passed as raw pointers (e.g.
``tensor.data_ptr()``), so the C ABI stays free of torch types.
"""
import ctypes
import os

import numpy as np

from . import _runtime, layout
from .textures import TextureSet

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTMI_LIB", os.path.join(_HERE, "..", "build", "libptmi.so"))
# DIAGNOSTIC study library (make -C pathtracer-ocl_amd study): the product plus the split
# execution form, the standalone walk kernels and the measured tile order.
STUDY_LIB_PATH = os.path.join(_HERE, "..", "build", "libptmi_study.so")

PTMI_OK, PTMI_ERR_ARG, PTMI_ERR_DEVICE, PTMI_ERR_HIP, PTMI_ERR_UNSUPPORTED, PTMI_ERR_NOMEM = 0, -1, -2, -3, -4, -5
RNG_NOISE3D, RNG_XOSHIRO = 0, 1  # ptmi_scene_set_rng: parity (default) / opt-in statistical mode
# ptmi_diag_set_knob (include/ptmi_diag.h): work-plan knobs of a resident scene
(KNOB_TAIL_TILES, KNOB_TAIL_ITEMS, KNOB_MESH_ITEMS, KNOB_MIN_CHUNK, KNOB_TILE_ORDER, KNOB_SPLIT_CHUNK,
 KNOB_SPLIT_SLOTS, KNOB_SPLIT_SYNC, KNOB_SPLIT_BUDGET, KNOB_TAIL_SPLIT, KNOB_MESH_ITEMS_SHARE, KNOB_TAIL_MIN,
 KNOB_WALK_BATCH, KNOB_HEMI_MESH) = range(1, 15)

EXPORTS = ("ptmi_trace", "ptmi_device_count", "ptmi_device_name", "ptmi_scene_create", "ptmi_scene_destroy",
           "ptmi_scene_size", "ptmi_scene_render", "ptmi_finalize", "ptmi_fill_seeds", "ptmi_build_info",
           "ptmi_scene_set_timing", "ptmi_scene_kernel_time", "ptmi_trace_multi", "ptmi_scene_create_textured",
           "ptmi_trace_multi_timed", "ptmi_sample_split_point", "ptmi_combine_frames",
           "ptmi_scene_set_rng", "ptmi_index_stats")


class MultiTiming(ctypes.Structure):
    """ptmi_multi_timing (include/ptmi.h): wall-clock phases of ptmi_trace_multi, ms."""
    _fields_ = [(n, ctypes.c_double) for n in ("prepare_ms", "render_ms", "combine_ms", "readback_ms", "total_ms")] + \
        [("peer_direct", ctypes.c_int32), ("peer_staged", ctypes.c_int32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class PtmiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libptmi error %d: %s" % (code, msg))
        self.code = code


_lib = None


def load_library(path=None):
    """Load libptmi.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = os.path.abspath(path or LIB_PATH)
    _runtime.preload()
    if not os.path.exists(p):
        raise FileNotFoundError("libptmi.so not built (%s): run `make -C pathtracer-ocl_amd`" % p)
    lib = ctypes.CDLL(p)
    vp, u32, i32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
    cp = ctypes.c_char_p
    lib.ptmi_trace.restype = i32
    lib.ptmi_trace.argtypes = [vp, u32, vp, u32, vp, u32, i32, u32, vp, vp, ctypes.c_uint64, vp, vp, cp, sz]
    lib.ptmi_trace_multi.restype = i32
    lib.ptmi_trace_multi.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, i32, u32, vp, vp, ctypes.c_uint64, vp, vp,
                                     cp, sz]
    lib.ptmi_trace_multi_timed.restype = i32
    lib.ptmi_trace_multi_timed.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, i32, u32, vp, vp, ctypes.c_uint64, vp,
                                           vp, ctypes.POINTER(MultiTiming), cp, sz]
    if hasattr(lib, "ptmi_combine_frames"):
        lib.ptmi_combine_frames.restype = i32
        lib.ptmi_combine_frames.argtypes = [vp, u32, u32, vp, u32, vp, cp, sz]
    lib.ptmi_sample_split_point.restype = u32
    lib.ptmi_sample_split_point.argtypes = [i32, i32, u32]
    lib.ptmi_device_count.restype = i32
    lib.ptmi_device_count.argtypes = []
    lib.ptmi_device_name.restype = i32
    lib.ptmi_device_name.argtypes = [i32, cp, sz]
    lib.ptmi_scene_create.restype = i32
    lib.ptmi_scene_create.argtypes = [i32, vp, u32, vp, u32, vp, u32, vp, ctypes.POINTER(vp), cp, sz]
    lib.ptmi_scene_create_textured.restype = i32
    lib.ptmi_scene_create_textured.argtypes = [i32, vp, u32, vp, u32, vp, u32, vp, vp, ctypes.POINTER(vp), cp, sz]
    lib.ptmi_scene_destroy.restype = None
    lib.ptmi_scene_destroy.argtypes = [vp]
    lib.ptmi_scene_size.restype = i32
    lib.ptmi_scene_size.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32)]
    lib.ptmi_scene_render.restype = i32
    lib.ptmi_scene_render.argtypes = [vp, u32, u32, u32, u32, u32, vp, vp, u32, vp, cp, sz]
    lib.ptmi_finalize.restype = i32
    lib.ptmi_finalize.argtypes = [vp, vp, u32, u32, vp, cp, sz]
    lib.ptmi_fill_seeds.restype = i32
    lib.ptmi_fill_seeds.argtypes = [vp, u32, ctypes.c_uint64, vp, cp, sz]
    if hasattr(lib, "ptmi_scene_set_rng"):  # (older diagnostic builds lack it; tests/test_abi.py checks the product)
        lib.ptmi_scene_set_rng.restype = i32
        lib.ptmi_scene_set_rng.argtypes = [vp, i32, cp, sz]
    lib.ptmi_scene_set_timing.restype = i32
    lib.ptmi_scene_set_timing.argtypes = [vp, i32]
    lib.ptmi_scene_kernel_time.restype = i32
    lib.ptmi_scene_kernel_time.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u32), cp, sz]
    lib.ptmi_build_info.restype = cp
    lib.ptmi_build_info.argtypes = []
    if hasattr(lib, "ptmi_index_stats"):
        lib.ptmi_index_stats.restype = i32
        lib.ptmi_index_stats.argtypes = [vp, u32, vp, u32, vp, u32, vp, ctypes.POINTER(ctypes.c_double), i32, cp, sz]
    for name, args in (("ptmi_diag_set_knob", [vp, i32, i32]), ("ptmi_diag_force_flags", [i32]),
                       ("ptmi_diag_hemi_mismatch", [vp]), ("ptmi_diag_set_split", [vp, i32]),
                       ("ptmi_diag_split_passes", [vp]), ("ptmi_diag_scene_flags", [vp]),
                       ("ptmi_diag_tile_ownership", [vp, u32])):
        if hasattr(lib, name):  # (diagnostic libraries of earlier rounds lack some)
            getattr(lib, name).restype = i32
            getattr(lib, name).argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check(rc, err):
    if rc != PTMI_OK:
        raise PtmiError(rc, err.value.decode(errors="replace"))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and len(a) else None


def _records(objects, triangles, groups, camera):
    objects = np.ascontiguousarray(objects)
    triangles = np.ascontiguousarray(triangles) if triangles is not None else np.zeros(0, layout.TRIANGLE_DTYPE)
    groups = np.ascontiguousarray(groups) if groups is not None else np.zeros(0, layout.GROUP_DTYPE)
    camera = np.ascontiguousarray(np.asarray(camera).reshape(1))
    for arr, dt, name in ((objects, layout.OBJECT_DTYPE, "objects"), (triangles, layout.TRIANGLE_DTYPE, "triangles"),
                          (groups, layout.GROUP_DTYPE, "groups"), (camera, layout.CAMERA_DTYPE, "camera")):
        if arr.dtype.itemsize != dt.itemsize:
            raise TypeError("%s: expected %d-byte records, got %d" % (name, dt.itemsize, arr.dtype.itemsize))
    return objects, triangles, groups, camera


def device_count():
    return load_library().ptmi_device_count()


def device_name(i):
    buf = ctypes.create_string_buffer(256)
    rc = load_library().ptmi_device_name(i, buf, len(buf))
    if rc:
        raise PtmiError(rc, "no device %d" % i)
    return buf.value.decode()


def Trace(objects, triangles, groups, deviceIndex, samples, camera, textures=None, sphereTextures=None,
          cubeTextures=None, seeds=None, seed_stream=0):
    """Drop-in for ocl.Trace (ocltracer.go:98-100).  Returns float64 RGBA, len W*H*4.

    ``seeds``: W*H per-pixel seeds (the Go side's rand.Float64() per pixel); None
    lets the library generate them from ``seed_stream``.  ``textures`` /
    ``sphereTextures`` / ``cubeTextures``: lists of H x W x 4 uint8 NRGBA images
    (ptmi/textures.py), or None.
    """
    tex = TextureSet(textures, sphereTextures, cubeTextures)
    lib = load_library()
    objects, triangles, groups, camera = _records(objects, triangles, groups, camera)
    w, h = int(camera["width"][0]), int(camera["height"][0])
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.float64)
        if seeds.size != w * h:
            raise ValueError("seeds: expected %d values, got %d" % (w * h, seeds.size))
    out = np.empty(w * h * 4, dtype=np.float64)
    err = ctypes.create_string_buffer(1024)
    rc = lib.ptmi_trace(_ptr(objects), len(objects), _ptr(triangles), len(triangles), _ptr(groups), len(groups),
                        int(deviceIndex), int(samples), _ptr(camera), _ptr(seeds), int(seed_stream), tex.pointer(),
                        out.ctypes.data_as(ctypes.c_void_p), err, len(err))
    _check(rc, err)
    return out


def TraceMulti(objects, triangles, groups, devices, split, samples, camera, textures=None, sphereTextures=None,
               cubeTextures=None, seeds=None, seed_stream=0):
    """ptmi_trace_multi_timed: the frame over `devices` (an index may repeat) with a
    sample (split="sample") or 8x8-tile (split="tile") split, combined on device.
    Returns (float64 RGBA of len W*H*4, {phase: ms})."""
    tex = TextureSet(textures, sphereTextures, cubeTextures)
    lib = load_library()
    objects, triangles, groups, camera = _records(objects, triangles, groups, camera)
    w, h = int(camera["width"][0]), int(camera["height"][0])
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.float64)
        if seeds.size != w * h:
            raise ValueError("seeds: expected %d values, got %d" % (w * h, seeds.size))
    if split not in ("sample", "tile"):
        raise ValueError("split must be 'sample' or 'tile'")
    devs = (ctypes.c_int * len(devices))(*devices)
    out = np.empty(w * h * 4, dtype=np.float64)
    timing = MultiTiming()
    err = ctypes.create_string_buffer(1024)
    rc = lib.ptmi_trace_multi_timed(_ptr(objects), len(objects), _ptr(triangles), len(triangles), _ptr(groups),
                                    len(groups), devs, len(devices), 0 if split == "sample" else 1, int(samples),
                                    _ptr(camera), _ptr(seeds), int(seed_stream), tex.pointer(),
                                    out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(timing), err, len(err))
    _check(rc, err)
    return out, timing.as_dict()


def combine_frames(parts_ptr, n_parts, n_pixels, out_ptr, samples, stream=0):
    """ptmi_combine_frames: n_parts partial frames (device memory, back to back) summed
    in part order and normalised into out_ptr (may equal parts_ptr)."""
    err = ctypes.create_string_buffer(256)
    _check(load_library().ptmi_combine_frames(ctypes.c_void_p(parts_ptr), int(n_parts), int(n_pixels),
                                              ctypes.c_void_p(out_ptr), int(samples), ctypes.c_void_p(stream),
                                              err, len(err)), err)


def index_stats(objects, triangles, groups, camera):
    """ptmi_index_stats (host only): summary of the traversal index the library builds
    for these records -- {nodes4, slots, box_area, inf_bounds, max_scale_exp, roots, depth}."""
    objects, triangles, groups, camera = _records(objects, triangles, groups, camera)
    out = (ctypes.c_double * 8)()
    err = ctypes.create_string_buffer(1024)
    _check(load_library().ptmi_index_stats(_ptr(objects), len(objects), _ptr(triangles), len(triangles),
                                           _ptr(groups), len(groups), _ptr(camera), out, 8, err, len(err)), err)
    return dict(zip(("nodes4", "slots", "box_area", "inf_bounds", "max_scale_exp", "roots", "depth", "leaf_bit"),
                    list(out)))


class force_flags:
    """Context manager (ptmi_diag_force_flags): scenes created inside it -- by Trace or
    Scene -- launch the kernel instantiation `flags` instead of their own (test hook for
    the generic instantiations)."""

    def __init__(self, flags, lib=None):
        self.flags, self.lib = int(flags), lib or load_library()

    def __enter__(self):
        _check(self.lib.ptmi_diag_force_flags(self.flags), ctypes.create_string_buffer(b"bad flags"))
        return self

    def __exit__(self, *exc):
        self.lib.ptmi_diag_force_flags(-1)
        return False


def sample_split_point(g, n, samples):
    """The library's cost-balanced sample split (ptmi_sample_split_point)."""
    return load_library().ptmi_sample_split_point(int(g), int(n), int(samples))


class Scene:
    """A scene resident on one device (ptmi_scene_*)."""

    def __init__(self, device_index, objects, triangles, groups, camera, textures=None, sphereTextures=None,
                 cubeTextures=None, lib=None):
        # lib: another build of the library (e.g. load_library(STUDY_LIB_PATH)); default the product
        self._lib = lib or load_library()
        objects, triangles, groups, camera = _records(objects, triangles, groups, camera)
        tex = TextureSet(textures, sphereTextures, cubeTextures)
        handle = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = self._lib.ptmi_scene_create_textured(int(device_index), _ptr(objects), len(objects), _ptr(triangles),
                                                  len(triangles), _ptr(groups), len(groups), _ptr(camera),
                                                  tex.pointer(), ctypes.byref(handle), err, len(err))
        _check(rc, err)
        self._h = handle
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        self._lib.ptmi_scene_size(self._h, ctypes.byref(w), ctypes.byref(h))
        self.width, self.height = w.value, h.value

    def render(self, samples, sample_begin, sample_end, seeds_ptr, sums_ptr, tile_stride=1, tile_offset=0,
               chunks=0, stream=0):
        err = ctypes.create_string_buffer(1024)
        rc = self._lib.ptmi_scene_render(self._h, samples, sample_begin, sample_end, tile_stride, tile_offset,
                                         ctypes.c_void_p(seeds_ptr), ctypes.c_void_p(sums_ptr), chunks,
                                         ctypes.c_void_p(stream), err, len(err))
        _check(rc, err)

    def finalize(self, sums_ptr, out_ptr, samples, stream=0):
        err = ctypes.create_string_buffer(1024)
        rc = self._lib.ptmi_finalize(ctypes.c_void_p(sums_ptr), ctypes.c_void_p(out_ptr),
                                     self.width * self.height, samples, ctypes.c_void_p(stream), err, len(err))
        _check(rc, err)

    def set_rng(self, mode):
        """RNG_NOISE3D (default, the reference's noise3D bit for bit) or RNG_XOSHIRO (the
        opt-in statistical mode: images converge to the same expectation, not equal)."""
        err = ctypes.create_string_buffer(256)
        _check(self._lib.ptmi_scene_set_rng(self._h, int(mode), err, len(err)), err)

    def set_split(self, enable=True):
        """Diagnostics (include/ptmi_diag.h): mesh scenes in the split form (study library
        only) or the (default) one-kernel form.  Returns False when the library lacks it."""
        if not hasattr(self._lib, "ptmi_diag_set_split"):
            return False
        return self._lib.ptmi_diag_set_split(self._h, 1 if enable else 0) == 0

    def split_passes(self):
        return self._lib.ptmi_diag_split_passes(self._h)

    def set_knob(self, knob, value):
        """ptmi_diag_set_knob: a work-plan knob (KNOB_*); returns the library's status code
        (PTMI_ERR_UNSUPPORTED for a knob or value this build lacks)."""
        return self._lib.ptmi_diag_set_knob(self._h, int(knob), int(value))

    def hemi_mismatch(self):
        """ptmi_diag_hemi_mismatch: hemisphere-table records where the generic operator
        sequences differ from the affine ones the table holds (0 expected)."""
        return self._lib.ptmi_diag_hemi_mismatch(self._h)

    def kernel_flags(self):
        """ptmi_diag_scene_flags: F_* flags of the trace_kernel instantiation this scene launches."""
        return self._lib.ptmi_diag_scene_flags(self._h)

    def tile_ownership(self, tile_stride):
        """ptmi_diag_tile_ownership: 'diagonal' or 'raster', the tile ownership a tile-split render
        with this stride uses (the library's own decision; ptmi/dist.py tile_owner_mask takes it)."""
        r = self._lib.ptmi_diag_tile_ownership(self._h, int(tile_stride))
        if r < 0:
            raise PtmiError(PTMI_ERR_ARG, "tile_ownership: bad stride %r" % (tile_stride,))
        return "diagonal" if r == 1 else "raster"

    def set_timing(self, enable=True):
        self._lib.ptmi_scene_set_timing(self._h, 1 if enable else 0)

    def kernel_time(self):
        """(summed trace_kernel ms, launches) since the last call (waits for them)."""
        ms, n = ctypes.c_double(), ctypes.c_uint32()
        err = ctypes.create_string_buffer(512)
        _check(self._lib.ptmi_scene_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(n), err, len(err)), err)
        return ms.value, n.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ptmi_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_seeds(seeds_ptr, n, seed_stream, stream=0):
    lib = load_library()
    err = ctypes.create_string_buffer(256)
    _check(lib.ptmi_fill_seeds(ctypes.c_void_p(seeds_ptr), n, seed_stream, ctypes.c_void_p(stream), err, len(err)),
           err)
