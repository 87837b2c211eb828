"""DIAGNOSTIC: phase timing of ptmi_trace_multi (the in-process multi-device path of
`pt --gpus N`) on the C2 frame, device 0 repeated N times on a one-GPU box.
    python tools/multi_timing.py [spp]"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402,F401
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
objs, tris, grps, cam = scene_inputs("reference", 1280, 960)
seeds = layout.seeds_go_float64(1280 * 960, 1234)
for n in (1, 2, 4, 8):
    for split in ("sample", "tile"):
        api.TraceMulti(objs, tris, grps, [0] * n, split, spp, cam, seeds=seeds)  # warm-up
        _, t = api.TraceMulti(objs, tris, grps, [0] * n, split, spp, cam, seeds=seeds)
        print("devices %d %-6s %s" % (n, split, " ".join("%s %.2f" % kv for kv in t.items())), flush=True)
