"""DIAGNOSTIC: the statistical RNG mode against the parity mode on one scene.
    python tools/xrng_check.py [scene] [W] [H] [spp]"""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "reference"
W, H, S = (int(a) for a in (sys.argv[2:5] if len(sys.argv) > 4 else (160, 120, 256)))
objs, tris, grps, cam = scene_inputs(scene, W, H)
sc = api.Scene(0, objs, tris, grps, cam)
n = W * H
out = {}
for tag, mode, seed in (("parity", 0, 1), ("xrng", 1, 1), ("xrng2", 1, 2)):
    seeds = torch.tensor(layout.seeds_go_float64(n, seed), dtype=torch.float64, device="cuda")
    sums = torch.empty(n * 4, dtype=torch.float64, device="cuda")
    sc.set_rng(mode)
    sc.render(S, 0, S, seeds.data_ptr(), sums.data_ptr())
    torch.cuda.synchronize()
    t0 = time.time()
    sc.render(S, 0, S, seeds.data_ptr(), sums.data_ptr())
    torch.cuda.synchronize()
    out[tag] = (sums.cpu().numpy().reshape(H, W, 4)[..., :3] / S, time.time() - t0)
for k, (img, t) in out.items():
    print("%-7s mean %s  %.3f s" % (k, img.mean(axis=(0, 1)), t))
d_fp = out["xrng"][0] - out["parity"][0]
d_ff = out["xrng"][0] - out["xrng2"][0]
print("rms pixel diff xrng-parity %.4e, xrng-xrng2 %.4e" % (np.sqrt((d_fp ** 2).mean()), np.sqrt((d_ff ** 2).mean())))
