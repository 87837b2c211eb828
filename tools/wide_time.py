"""DIAGNOSTIC: the wide-code mesh scene (tests/adversarial.py "big", 34,848 triangles, child codes
past 16 bits) on its affine F_WIDE instantiation (round 6) against the generic instantiation it
took in round 5 (forced with ptmi_diag_force_flags(31)): trace_kernel ms per frame, median of 3.
    python tools/wide_time.py [W H spp]"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests import adversarial  # noqa: E402

W, H, S = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (640, 480, 64)
objs, tris, grps, cam = adversarial.scene_inputs("big", W, H)
seeds = torch.tensor(layout.seeds_go_float64(W * H, 404), dtype=torch.float64, device="cuda")
sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
res = {}
for name, force in (("affine F_WIDE (round 6)", None), ("generic, forced 31 (round 5's path)", 31)):
    if force is None:
        sc = api.Scene(0, objs, tris, grps, cam)
    else:
        with api.force_flags(force):
            sc = api.Scene(0, objs, tris, grps, cam)
    stream = torch.cuda.current_stream().cuda_stream
    sc.render(S, 0, S, seeds.data_ptr(), sums.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    sc.kernel_time()
    sc.set_timing(True)
    t = []
    for _ in range(3):
        sc.render(S, 0, S, seeds.data_ptr(), sums.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        ms, n = sc.kernel_time()
        t.append(ms / max(n, 1))
    img = sums.clone()
    res[name] = (sorted(t)[1], sc.kernel_flags(), img)
    sc.close()
base = None
for name, (ms, fl, img) in res.items():
    print("%-38s flags %3d  %8.2f ms per %dx%d x %d spp frame" % (name, fl, ms, W, H, S))
a, b = [v[2] for v in res.values()]
print("images bit-identical:", bool(torch.equal(a, b)), " max |diff| of the sums: %.3e" % (a - b).abs().max().item())
