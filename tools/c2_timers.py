"""DIAGNOSTIC: phase clocks of the non-group trace kernel (libptmi_timers.so, PTMI_STATS=2).
    PTMI_LIB=pathtracer-ocl_amd/build/libptmi_timers.so python tools/c2_timers.py [scene] [spp]"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402,F401
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "reference"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W, H = 1280, 960
lib = api.load_library()
buf = (ctypes.c_ulonglong * 80)()
lib.ptmi_stats_read(buf, 1)
objs, tris, grps, cam = scene_inputs(scene, W, H)
api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 3))
lib.ptmi_stats_read(buf, 1)
v = list(buf)
lp = max(v[16], 1)
print("%s spp %d: loop iterations %d, cycles per iteration %.0f" % (scene, spp, v[10], v[16] / max(v[10], 1)))
for i, n in ((12, "camera refill + path start"), (13, "closest hit (prims)"), (14, "walk phases"), (15, "shade")):
    print("  %-28s %.3f of loop cycles, %.0f cycles per iteration" % (n, v[i] / lp, v[i] / max(v[10], 1)))
