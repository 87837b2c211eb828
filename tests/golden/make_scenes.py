"""Generate the committed BVH scene records (inputs, not reference code).

The teapot / gopher / transparent_teapot scenes are built by ptmi's restatement of the reference's OBJ
parser + BVH build from the OBJ assets in the reference checkout
(/root/reference/assets, this container only).  The resulting kernel input
records (CLObject / CLTriangle / CLGroup bytes, layout.py) are saved so tests and
bench.py on the GPU box -- where /root/reference does not exist -- use the same
inputs.  The camera record is not stored: it depends only on W/H/aperture/focal and
is rebuilt by ``ptmi.scenes`` at run time.

    python tests/golden/make_scenes.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "pathtracer-ocl_amd"))
from ptmi import layout, scenes  # noqa: E402


# Scenes whose triangle / group records are byte-identical to a base mesh scene's
# (same OBJ, same Divide threshold: Divide works in the group's own space, so only
# the CLObject records differ); only their objects are stored, plus the base name.
SHARED_MESH = {"cubemap": "gopher", "gopher-window": "gopher", "christian": "teapot"}


def main():
    bases_first = ("teapot", "gopher", "transparent_teapot")
    for name in bases_first:
        if not os.path.exists(os.path.join(HERE, "scene_%s.npz" % name)):
            raise SystemExit("build the base scenes first (they are committed)")
    for name, base in SHARED_MESH.items():
        sc = scenes.SCENES[name](64, 48)
        objs, tris, grps = layout.build_scene_buffer_cl(sc.objects)
        b = np.load(os.path.join(HERE, "scene_%s.npz" % base))
        assert np.array_equal(tris.view(np.uint8), b["triangles"]) and np.array_equal(grps.view(np.uint8), b["groups"])
        out = os.path.join(HERE, "scene_%s.npz" % name.replace("-", "_"))
        np.savez_compressed(out, objects=objs.view(np.uint8), mesh=np.array(base))
        print(out, os.path.getsize(out), len(objs), "(+ %s triangles/groups)" % base)
    for name in ("teapot", "gopher", "transparent_teapot"):
        sc = scenes.SCENES[name](64, 48)
        objs, tris, grps = layout.build_scene_buffer_cl(sc.objects)
        out = os.path.join(HERE, "scene_%s.npz" % name)
        np.savez_compressed(out, objects=objs.view(np.uint8), triangles=tris.view(np.uint8),
                            groups=grps.view(np.uint8))
        print(out, os.path.getsize(out), len(objs), len(tris), len(grps))


if __name__ == "__main__":
    main()
