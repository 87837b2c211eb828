"""DIAGNOSTIC: walk-pool counters of the group kernels (libptmi_timers.so, PTMI_STATS=2).
    PTMI_LIB=pathtracer-ocl_amd/build/libptmi_timers.so python tools/pool_stats.py [scene] [spp] [stride]
Counters are per wave (summed over waves): clocks are shader cycles of that wave.  stride > 1:
one rank's tile split share (tiles t with t mod stride = 0) instead of the whole frame."""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "teapot"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 1
W, H = 1280, 960
lib = api.load_library()
buf = (ctypes.c_ulonglong * 80)()
lib.ptmi_stats_read(buf, 1)
objs, tris, grps, cam = scene_inputs(scene, W, H)
if stride > 1:
    sc = api.Scene(0, objs, tris, grps, cam)
    seeds = torch.tensor(layout.seeds_go_float64(W * H, 3), dtype=torch.float64, device="cuda")
    sums = torch.zeros(W * H * 4, dtype=torch.float64, device="cuda")
    sc.render(spp, 0, spp, seeds.data_ptr(), sums.data_ptr(), tile_stride=stride, tile_offset=0)
    torch.cuda.synchronize()
else:
    api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 3))
lib.ptmi_stats_read(buf, 1)
v = list(buf)
names = {8: "tracer_sleeps", 10: "tracer_loop_iterations", 12: "cyc_camera", 13: "cyc_prims_shadeprep",
         14: "cyc_results_and_sleeps", 15: "cyc_shade", 16: "cyc_tracer_loop", 18: "cyc_walker_loop",
         19: "inner_iterations", 21: "walking_lanes_sum", 22: "walker_sleeps", 23: "walker_outer_iterations",
         24: "claims", 26: "cyc_walker_sleep"}
print(scene, "spp", spp)
for i, n in names.items():
    print("  %-26s %16d" % (n, v[i]))
print("  walking lanes per inner iteration %.1f, inner iterations per outer %.2f, claims per outer %.1f" % (
    v[21] / max(v[19], 1), v[19] / max(v[23], 1), v[24] / max(v[23], 1)))
wl = max(v[18], 1)
print("  walker: sleeping %.3f of its cycles, cycles per inner iteration %.0f" % (
    v[26] / wl, (v[18] - v[26]) / max(v[19], 1)))
lp = max(v[16], 1)
print("  tracers: share of loop cycles camera %.3f, prims %.3f, results+sleep %.3f, shade %.3f; sleeps per iteration %.3f"
      % (v[12] / lp, v[13] / lp, v[14] / lp, v[15] / lp, v[8] / max(v[10], 1)))
print("  walker loop cycles / tracer loop cycles per wave: %.3f" % (v[18] / lp * 3))
print("  lanes with a finished item: %.3f of the loop's lane-cycles" % (v[27] / max(v[28], 1)))
