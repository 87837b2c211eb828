"""Kernel input records for the benchmark / parity scenes.

Scenes without meshes are built on the fly by ptmi's scene restatement.
``teapot`` / ``gopher`` / ``transparent_teapot`` load the records pre-built from the OBJ
assets (tests/golden/scene_*.npz, tests/golden/make_scenes.py) because the assets
live in the reference checkout, which the GPU box does not have; only the camera
record (a function of W/H/aperture/focal) is rebuilt.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pathtracer-ocl_amd"))
from ptmi import layout, scenes  # noqa: E402

_cache = {}
# records from tests/golden/scene_<name>.npz (cubemap / gopher-window / christian
# store only their objects and reuse their base mesh's triangles and groups)
MESH_SCENES = ("teapot", "gopher", "transparent_teapot", "cubemap", "gopher-window", "christian")


def _load_mesh_scene(name):
    if name not in _cache:
        z = np.load(os.path.join(HERE, "golden", "scene_%s.npz" % name.replace("-", "_")))
        if "mesh" in z.files:
            _, tris, grps = _load_mesh_scene(str(z["mesh"]))
        else:
            tris = z["triangles"].view(layout.TRIANGLE_DTYPE).copy()
            grps = z["groups"].view(layout.GROUP_DTYPE).copy()
        _cache[name] = (z["objects"].view(layout.OBJECT_DTYPE).copy(), tris, grps)
    return _cache[name]


def scene_inputs(name, width, height, aperture=0.0, focal_length=0.0):
    """-> (objects, triangles, groups, camera) records (triangles/groups may be empty)."""
    if name in MESH_SCENES:
        objs, tris, grps = _load_mesh_scene(name)
        cam = scenes.CAMERAS.get(name, scenes._std_camera)(width, height, aperture, focal_length)
        return objs, tris, grps, layout.camera_record(cam)
    sc = scenes.SCENES[name](width, height, aperture, focal_length)
    objs, tris, grps = layout.build_scene_buffer_cl(sc.objects)
    return objs, tris, grps, layout.camera_record(sc.camera)
