"""DIAGNOSTIC: kernel time of one 256-sample slice of the C2 frame (S = 2048) at
several sample offsets -- the per-rank work of an 8-GPU sample split; with a
third argument G, the ranges of ptmi.dist's cost-balanced split over G ranks.
    python tools/sample_cost.py [scene] [slice] [G]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pathtracer-ocl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene_name = sys.argv[1] if len(sys.argv) > 1 else "reference"
sl = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W, H, S = 1280, 960, 2048
objs, tris, grps, cam = scene_inputs(scene_name, W, H)
sc = api.Scene(0, objs, tris, grps, cam)
seeds = torch.tensor(layout.seeds_go_float64(W * H, 1234), dtype=torch.float64, device="cuda")
sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
sc.render(S, 0, sl, seeds.data_ptr(), sums.data_ptr())
torch.cuda.synchronize()
if len(sys.argv) > 3:
    from ptmi import dist
    G = int(sys.argv[3])
    ranges = [(dist.sample_split_point(g, G, S), dist.sample_split_point(g + 1, G, S)) for g in range(G)]
else:
    ranges = [(s0, s0 + sl) for s0 in range(0, S, sl)]
for s0, s1 in ranges:
    ts = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print("samples [%4d, %4d): %.2f ms" % (s0, s1, 1e3 * min(ts)), flush=True)
