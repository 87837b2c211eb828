"""ctypes front-end of the two oracles -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
The product path (libptmi.so) never links or calls anything under oracle/.

* ``ref_trace``  -- the reference kernel itself (tracer.cl compiled by ROCm's OpenCL
  toolchain, oracle/_ref/tracer_ref.hsaco) dispatched on a GPU through HSA.
* ``cpu_trace``  -- the C restatement of the same algorithm (oracle/pt_oracle.c,
  oracle/build/libptoracle.so), multithreaded with OpenMP.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_HSACO = os.path.join(HERE, "_ref", "tracer_ref.hsaco")
REF_LIB = os.path.join(HERE, "_ref", "libptref.so")
CPU_LIB = os.path.join(HERE, "build", "libptoracle.so")

_ref = None
_cpu = None


def ref_available():
    return os.path.exists(REF_HSACO) and os.path.exists(REF_LIB) and os.path.exists(REF_HSACO + ".args")


def _as_bytes_ptr(a):
    a = np.ascontiguousarray(a)
    return a, a.ctypes.data_as(ctypes.c_void_p)


def ref_trace(objects, triangles, groups, camera, samples, seeds, device_index=0, wg_size=None,
              timeout_s=600.0):
    """Run the reference OpenCL kernel on the GPU; returns float64 RGBA [H*W*4]."""
    global _ref
    if _ref is None:
        try:  # share the process's HIP/HSA runtime with torch (see ptmi/_runtime.py)
            import torch  # noqa: F401
        except ImportError:
            pass
        _ref = ctypes.CDLL(REF_LIB)
        _ref.ptref_trace.restype = ctypes.c_int
        _ref.ptref_trace.argtypes = [ctypes.c_char_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_double, ctypes.c_char_p, ctypes.c_size_t]
    cam = np.asarray(camera).reshape(())
    w, h = int(cam["width"]), int(cam["height"])
    n = w * h
    if wg_size is None:
        wg_size = next(g for g in (256, 128, 64, 32, 16, 8, 4, 2, 1) if n % g == 0)
    seeds = np.ascontiguousarray(seeds, dtype=np.float64)
    assert seeds.size == n
    out = np.zeros(n * 4, dtype=np.float64)
    objects, po = _as_bytes_ptr(objects)
    triangles, pt = _as_bytes_ptr(triangles)
    groups, pg = _as_bytes_ptr(groups)
    cam_arr, pc = _as_bytes_ptr(cam)
    err = ctypes.create_string_buffer(512)
    rc = _ref.ptref_trace(REF_HSACO.encode(), device_index, po, len(objects), pt, len(triangles),
                          pg, len(groups), pc, samples, seeds.ctypes.data_as(ctypes.c_void_p), n,
                          wg_size, out.ctypes.data_as(ctypes.c_void_p), timeout_s, err, len(err))
    if rc != 0:
        raise RuntimeError("ptref_trace rc=%d: %s" % (rc, err.value.decode(errors="replace")))
    return out


def cpu_available():
    return os.path.exists(CPU_LIB)


def _cpu_lib():
    global _cpu
    if _cpu is None:
        _cpu = ctypes.CDLL(CPU_LIB)
        _cpu.pto_trace.restype = ctypes.c_int
        _cpu.pto_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        _cpu.pto_trace_tex.restype = ctypes.c_int
        _cpu.pto_trace_tex.argtypes = _cpu.pto_trace.argtypes[:-1] + [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
        _cpu.pto_tex_sample.restype = None
        _cpu.pto_tex_sample.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        for f in (_cpu.pto_spherical_map, _cpu.pto_cube_uv):
            f.restype = None
            f.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
        _cpu.pto_ray_box.restype = ctypes.c_int
        _cpu.pto_ray_box.argtypes = [ctypes.c_void_p] * 4
        _cpu.pto_noise3d.restype = ctypes.c_float
        _cpu.pto_noise3d.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float]
        _cpu.pto_sinf32.restype = ctypes.c_float
        _cpu.pto_sinf32.argtypes = [ctypes.c_float]
        _cpu.pto_sinf_many.restype = None
        _cpu.pto_sinf_many.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    return _cpu


def _tex_arrays(tex_lists):
    """[textures, sphereTextures, cubeTextures] (lists of H x W x 4 uint8 NRGBA
    images) -> stacked arrays (kept alive by the caller) + ctypes arguments."""
    keep, pix = [], (ctypes.c_void_p * 3)()
    w, h, n = (ctypes.c_uint32 * 3)(), (ctypes.c_uint32 * 3)(), (ctypes.c_uint32 * 3)()
    for k, imgs in enumerate(tex_lists or (None, None, None)):
        if imgs is None or len(imgs) == 0:
            continue
        a = np.ascontiguousarray(np.stack([np.asarray(i, dtype=np.uint8) for i in imgs]))
        keep.append(a)
        pix[k] = a.ctypes.data
        n[k], h[k], w[k] = a.shape[0], a.shape[1], a.shape[2]
    return keep, (pix, w, h, n)


def tex_sample(images, s, t, layer):
    """The restated sampler alone: read_imagef(array, sampler, (s, t, layer, 0)).xyz."""
    keep, (pix, w, h, n) = _tex_arrays([images, None, None])
    out = (ctypes.c_float * 3)()
    _cpu_lib().pto_tex_sample(pix[0], w[0], h[0], n[0], s, t, layer, out)
    return tuple(out)


def spherical_map(x, y, z):
    uv = (ctypes.c_double * 2)()
    _cpu_lib().pto_spherical_map(x, y, z, uv)
    return uv[0], uv[1]


def cube_uv(x, y, z):
    uv = (ctypes.c_double * 2)()
    _cpu_lib().pto_cube_uv(x, y, z, uv)
    return uv[0], uv[1]


def cpu_trace(objects, triangles, groups, camera, samples, seeds, row0=0, rows=None,
              sample_begin=0, sample_end=None, threads=0, textures=None):
    """C restatement of the reference kernel.  Returns float64 RGBA for rows
    [row0, row0+rows).  ``sample_begin/end`` select a sub-range of the S samples
    (global indices, as a multi-GPU sample split passes them); with a partial
    range the result is the un-normalised sum (like one GPU's partial frame).
    ``textures``: [textures, sphereTextures, cubeTextures] image lists or None."""
    lib = _cpu_lib()
    cam = np.asarray(camera).reshape(())
    w, h = int(cam["width"]), int(cam["height"])
    rows = h - row0 if rows is None else rows
    sample_end = samples if sample_end is None else sample_end
    seeds = np.ascontiguousarray(seeds, dtype=np.float64)
    assert seeds.size == w * h
    out = np.zeros(w * rows * 4, dtype=np.float64)
    objects, po = _as_bytes_ptr(objects)
    triangles, pt = _as_bytes_ptr(triangles)
    groups, pg = _as_bytes_ptr(groups)
    cam_arr, pc = _as_bytes_ptr(cam)
    keep, (tp, tw, th, tn) = _tex_arrays(textures)
    rc = lib.pto_trace_tex(po, len(objects), pt, len(triangles), pg, len(groups), pc, samples,
                           seeds.ctypes.data_as(ctypes.c_void_p), row0, rows, sample_begin, sample_end,
                           threads, tp, tw, th, tn, out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise RuntimeError("pto_trace rc=%d" % rc)
    return out


def max_candidates(objects, triangles, groups, camera, samples, seeds, row0=0, rows=None):
    """The most entries the reference would record in its 64-entry ctx arrays
    (tracer.cl:97-99) in one findClosestIntersection call of this trace: every
    candidate with t != 0, negative t included (the oracle's counting build, which
    streams them).  A scene past 64 overflows the reference's arrays (undefined
    behaviour; the live reference kernel faults on such scenes), so it can be checked
    against this restatement only."""
    lib = ctypes.CDLL(os.path.join(os.path.dirname(CPU_LIB), "libptoracle_count.so"))
    lib.pto_trace.restype = ctypes.c_int
    lib.pto_trace.argtypes = _cpu_lib().pto_trace.argtypes
    lib.pto_max_candidates.restype = ctypes.c_int
    cam = np.asarray(camera).reshape(())
    w, h = int(cam["width"]), int(cam["height"])
    rows = h - row0 if rows is None else rows
    seeds = np.ascontiguousarray(seeds, dtype=np.float64)
    out = np.zeros(w * rows * 4, dtype=np.float64)
    objects, po = _as_bytes_ptr(objects)
    triangles, pt = _as_bytes_ptr(triangles)
    groups, pg = _as_bytes_ptr(groups)
    cam_arr, pc = _as_bytes_ptr(cam)
    rc = lib.pto_trace(po, len(objects), pt, len(triangles), pg, len(groups), pc, samples,
                       seeds.ctypes.data_as(ctypes.c_void_p), row0, rows, 0, samples, 0,
                       out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise RuntimeError("pto_trace rc=%d" % rc)
    return int(lib.pto_max_candidates())


def ray_box(origin, direction, bb_min, bb_max):
    """intersectRayWithBox (tracer.cl:270-280): origin/direction 4-tuples, box corners 3-tuples."""
    a = [np.ascontiguousarray(v, dtype=np.float64) for v in (origin, direction, bb_min, bb_max)]
    return bool(_cpu_lib().pto_ray_box(*[x.ctypes.data_as(ctypes.c_void_p) for x in a]))


def noise3d(x, y, z):
    return _cpu_lib().pto_noise3d(x, y, z)


def sinf(x):
    return _cpu_lib().pto_sinf32(x)
