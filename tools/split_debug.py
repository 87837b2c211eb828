"""DIAGNOSTIC: split vs one-kernel vs the live reference on a tiny mesh frame."""
import sys, os
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import torch
from ptmi import api, layout
from tests.scene_inputs import scene_inputs
import pyoracle

w, h, S = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
chunks = int(sys.argv[4]) if len(sys.argv) > 4 else 1
objs, tris, grps, cam = scene_inputs("teapot", w, h)
seeds_h = layout.seeds_go_float64(w * h, 77)
scene = api.Scene(0, objs, tris, grps, cam)
seeds = torch.tensor(seeds_h, dtype=torch.float64, device="cuda")
res = {}
for sp in (True, False):
    scene.set_split(sp)
    sums = torch.zeros(w * h * 4, dtype=torch.float64, device="cuda")
    scene.render(S, 0, S, seeds.data_ptr(), sums.data_ptr(), chunks=chunks)
    torch.cuda.synchronize()
    res[sp] = sums.cpu().numpy().reshape(-1, 4)
    if sp:
        print("passes", scene.split_passes())
t2, g2 = layout.pad_empty(tris, grps)
ref = pyoracle.ref_trace(objs, t2, g2, cam, S, seeds_h).reshape(-1, 4) if pyoracle.ref_available() else None
for name, a in (("split", res[True]), ("one", res[False])):
    img = a[:, :3] / S
    e = np.abs(img - ref[:, :3]).max() if ref is not None else -1
    print(name, "vs ref L-inf %.3e" % e, "samples", np.unique(a[:, 3]))
d = np.where(np.any(res[True] != res[False], axis=1))[0]
print("differing pixels", len(d), d[:20])
for i in d[:5]:
    print(i, res[True][i], res[False][i], ref[i] * S if ref is not None else None)
