"""DIAGNOSTIC: time one leg of tests/test_gpu_parity.py's wide-code case on its own.
    python tools/diag_big.py ref|hip [w h spp]
ref = the live reference kernel (oracle/_ref), hip = ptmi_trace; prints the time and a checksum."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pathtracer-ocl_amd")]
import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests import adversarial  # noqa: E402

leg = sys.argv[1]
w, h, spp = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (64, 48, 2)
objs, tris, grps, cam = adversarial.scene_inputs("big", w, h)
print("stats", api.index_stats(objs, tris, grps, cam), flush=True)
seeds = layout.seeds_go_float64(w * h, 404)
t0 = time.time()
if leg == "ref":
    t2, g2 = layout.pad_empty(tris, grps)
    out = pyoracle.ref_trace(objs, t2, g2, cam, spp, seeds)
else:
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=seeds)
print(leg, "%.3f s" % (time.time() - t0), "sum %.17g" % float(np.asarray(out).sum()), flush=True)
np.save(os.path.join(ROOT, "gpurun_out", "big_%s.npy" % leg), np.asarray(out))
