"""The kernel ABI records, byte-for-byte as the reference defines them, and the
scene flattening that fills them.

Record layouts (packed, little endian) -- the C-ABI consumes exactly these bytes:

* ``CLObject``   1024 B  ocltracer.go:25-51  == tracer.cl:37-63  ``object``
* ``CLGroup``     256 B  ocltracer.go:53-64  == tracer.cl:24-35  ``group``
* ``CLTriangle``  512 B  ocltracer.go:66-78  == tracer.cl:82-93  ``triangle``
* ``CLCamera``    256 B  ocltracer.go:85-96  == tracer.cl:6-17   ``camera``

``build_scene_buffer_cl`` restates ``BuildSceneBufferCL`` / ``BuildCLGroup``
(internal/ocl/scene.go:14-155) without its package-level globals.
"""
import numpy as np

from . import shapes

OBJECT_DTYPE = np.dtype([
    ("transform", "<f8", 16), ("inverse", "<f8", 16), ("inverse_transpose", "<f8", 16),
    ("color", "<f8", 4), ("emission", "<f8", 4),
    ("refractive_index", "<f8"), ("type", "<i8"), ("min_y", "<f8"), ("max_y", "<f8"),
    ("reflectivity", "<f8"),
    ("texture_scale_x", "<f8"), ("texture_scale_y", "<f8"),
    ("texture_scale_x_nm", "<f8"), ("texture_scale_y_nm", "<f8"),
    ("bb_min", "<f8", 4), ("bb_max", "<f8", 4),
    ("child_count", "<i4"), ("children", "<i4", 64),
    ("is_textured", "u1"), ("texture_index", "u1"), ("is_textured_nm", "u1"),
    ("texture_index_nm", "u1"), ("is_env_map", "u1"),
    ("label", "u1", 8), ("padding5", "u1", 167),
])
GROUP_DTYPE = np.dtype([
    ("bb_min", "<f8", 4), ("bb_max", "<f8", 4), ("color", "<f8", 4), ("emission", "<f8", 4),
    ("tri_offset", "<i4"), ("tri_count", "<i4"), ("child_group_count", "<i4"),
    ("children", "<i4", 2), ("padding", "u1", 108),
])
TRIANGLE_DTYPE = np.dtype([
    ("p1", "<f8", 4), ("p2", "<f8", 4), ("p3", "<f8", 4), ("e1", "<f8", 4), ("e2", "<f8", 4),
    ("n1", "<f8", 4), ("n2", "<f8", 4), ("n3", "<f8", 4), ("color", "<f8", 4),
    ("padding", "u1", 224),
])
CAMERA_DTYPE = np.dtype([
    ("width", "<i4"), ("height", "<i4"), ("fov", "<f8"), ("pixel_size", "<f8"),
    ("half_width", "<f8"), ("half_height", "<f8"), ("aperture", "<f8"), ("focal_length", "<f8"),
    ("inverse", "<f8", 16), ("padding", "u1", 72),
])
assert OBJECT_DTYPE.itemsize == 1024 and GROUP_DTYPE.itemsize == 256
assert TRIANGLE_DTYPE.itemsize == 512 and CAMERA_DTYPE.itemsize == 256
assert OBJECT_DTYPE.fields["child_count"][1] == 584 and OBJECT_DTYPE.fields["label"][1] == 849

TYPE_PLANE, TYPE_SPHERE, TYPE_CYLINDER, TYPE_CUBE, TYPE_GROUP, TYPE_IGNORED = 0, 1, 2, 3, 4, 999
MAX_OBJECTS = 16     # tracer.cl:846 ``__local object objects[16]``


def _label_bytes(s, n):
    b = s.encode("utf-8")[:n]
    return list(b) + [0] * (n - len(b))


def build_scene_buffer_cl(objects):
    """BuildSceneBufferCL (scene.go:14-86) -> (objects[n], triangles[m], groups[k])."""
    objs = np.zeros(len(objects), dtype=OBJECT_DTYPE)
    tris, grps = [], []

    def build_cl_group(group):
        """BuildCLGroup (scene.go:96-155): preorder node numbering, node triangles
        contiguous at triOffset, children[] == 0 means 'absent'."""
        gid = len(grps)
        rec = np.zeros((), dtype=GROUP_DTYPE)
        grps.append(rec)
        rec["bb_min"] = group.bbox[0]
        rec["bb_max"] = group.bbox[1]
        lbl = group.label.encode("utf-8")
        if len(lbl) > 108:
            raise ValueError("group label longer than the 108-byte pad (scene.go:108 panics)")
        rec["padding"][:len(lbl)] = list(lbl)
        rec["tri_offset"] = len(tris)
        n = 0
        for c in group.children:
            if isinstance(c, shapes.Triangle):
                t = np.zeros((), dtype=TRIANGLE_DTYPE)
                for f in ("p1", "p2", "p3", "e1", "e2", "n1", "n2", "n3"):
                    t[f] = getattr(c, f)
                t["color"] = c.material.color
                tris.append(t)
                n += 1
        rec["tri_count"] = n
        k = 0
        for c in group.children:
            if isinstance(c, shapes.Group):
                if k >= 2:
                    raise ValueError("BuildCLGroup: more than 2 sub-groups (scene.go:143 index out of range)")
                rec["children"][k] = build_cl_group(c)
                k += 1
        rec["child_group_count"] = k if k > 0 else -1
        return gid

    for i, s in enumerate(objects):
        o = objs[i]
        o["label"] = _label_bytes(s.label, 8)
        o["transform"] = s.transform
        o["inverse"] = s.inverse
        o["inverse_transpose"] = s.inverse_transpose
        m = s.material
        o["color"] = m.color
        o["emission"] = m.emission
        o["refractive_index"] = m.refractive_index
        o["children"] = -1
        if m.textured:
            o["is_textured"] = 1
            o["texture_index"] = m.texture_id
            o["texture_scale_x"] = m.texture_scale_x
            o["texture_scale_y"] = m.texture_scale_y
        if m.textured_nm:
            o["is_textured_nm"] = 1
            o["texture_index_nm"] = m.texture_id_nm
            o["texture_scale_x_nm"] = m.texture_scale_x_nm
            o["texture_scale_y_nm"] = m.texture_scale_y_nm
        o["is_env_map"] = 1 if m.is_env_map else 0
        if isinstance(s, shapes.Group):
            o["type"] = TYPE_GROUP
            o["bb_min"] = s.bbox[0]
            o["bb_max"] = s.bbox[1]
            idx = 0
            for c in s.children:
                if isinstance(c, shapes.Group):
                    o["children"][idx] = build_cl_group(c)
                    idx += 1
                    o["child_count"] += 1
        elif isinstance(s, (shapes.Plane, shapes.Sphere, shapes.Cylinder, shapes.Cube)):
            o["type"] = s.TYPE
            if isinstance(s, shapes.Cylinder):
                o["min_y"] = s.min_y
                o["max_y"] = s.max_y
        else:
            o["type"] = TYPE_IGNORED
        o["reflectivity"] = m.reflectivity
    tri_arr = np.array(tris, dtype=TRIANGLE_DTYPE) if tris else np.zeros(0, TRIANGLE_DTYPE)
    grp_arr = np.array(grps, dtype=GROUP_DTYPE) if grps else np.zeros(0, GROUP_DTYPE)
    return objs, tri_arr, grp_arr


def camera_record(cam):
    """CLCamera as filled by renderPixelPathTracer (renderer.go:44-56)."""
    c = np.zeros((), dtype=CAMERA_DTYPE)
    c["width"] = cam.width
    c["height"] = cam.height
    c["fov"] = cam.fov
    c["pixel_size"] = cam.pixel_size
    c["half_width"] = cam.half_width
    c["half_height"] = cam.half_height
    c["aperture"] = cam.aperture
    c["focal_length"] = cam.focal_length
    c["inverse"] = cam.inverse
    return c


def pad_empty(triangles, groups):
    """Trace's dummy records for scenes without meshes (ocltracer.go:106-120)."""
    if len(triangles) == 0:
        triangles = np.zeros(1, TRIANGLE_DTYPE)
    if len(groups) == 0:
        groups = np.zeros(1, GROUP_DTYPE)
    return triangles, groups


def seeds_go_float64(n, seed=1234):
    """Per-pixel seeds with Go ``rand.Float64`` granularity (k / 2^53), from a fixed
    PCG64 stream so parity runs are reproducible (the reference uses a time-seeded
    math/rand source, ocltracer.go:260-263)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.random(n, dtype=np.float64)
