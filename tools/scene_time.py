"""DIAGNOSTIC: trace_kernel time of one frame of any scene (resident API, HIP events).
    [PTMI_LIB=...] python tools/scene_time.py <scene> [spp] [W H] [frames]
Prints the scene, the kernel ms per frame (mean of `frames` after one warm-up)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene_name = sys.argv[1]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1280
H = int(sys.argv[4]) if len(sys.argv) > 4 else 960
frames = int(sys.argv[5]) if len(sys.argv) > 5 else 2
objs, tris, grps, cam = scene_inputs(scene_name, W, H)
scene = api.Scene(0, objs, tris, grps, cam)
seeds = torch.tensor(layout.seeds_go_float64(W * H, 1234), dtype=torch.float64, device="cuda")
sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
scene.render(spp, 0, spp, seeds.data_ptr(), sums.data_ptr(), stream=stream)
torch.cuda.synchronize()
scene.set_timing(True)
for _ in range(frames):
    scene.render(spp, 0, spp, seeds.data_ptr(), sums.data_ptr(), stream=stream)
torch.cuda.synchronize()
ms, n = scene.kernel_time()
print("%s %dx%d %d spp: %.3f ms per frame (%d launches)" % (scene_name, W, H, spp, ms / max(n, 1), n))
scene.close()
