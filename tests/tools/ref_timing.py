"""Time the reference kernel (oracle/_ref, HSA launch) against ptmi on large frames,
so the full-resolution parity tests can be sized.  Test tooling (GPU box).

    python tests/tools/ref_timing.py [case ...]      case = scene:W:H:spp[:aperture]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import pyoracle  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

cases = sys.argv[1:] or ["reference:640:480:4", "reference:1280:960:8", "reference:1280:960:8:0.15",
                         "teapot:1280:960:1", "gopher:1280:960:1", "reference:1280:960:64"]
for c in cases:
    f = c.split(":")
    scene, w, h, spp = f[0], int(f[1]), int(f[2]), int(f[3])
    ap = float(f[4]) if len(f) > 4 else 0.0
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, 1.6 if ap else 0.0)
    seeds = layout.seeds_go_float64(w * h, 1234)
    t2, g2 = layout.pad_empty(tris, grps)
    t0 = time.time()
    ref = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds, timeout_s=900)
    t_ref = time.time() - t0
    t0 = time.time()
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
    t_hip = time.time() - t0
    print("%-32s ref %8.2f s  ptmi %7.3f s  L-inf %.3e  (ref %.1f Msamples/s)"
          % (c, t_ref, t_hip, float(np.abs(out - ref).max()), w * h * spp / t_ref / 1e6), flush=True)
