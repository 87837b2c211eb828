"""DIAGNOSTIC: traversal counters of the BVH path (libptmi_stats.so, PTMI_STATS).
    PTMI_LIB=pathtracer-ocl_amd/build/libptmi_stats.so python tools/bvh_stats.py [scene] [spp]
"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402,F401
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "teapot"
if scene.startswith("adv:"):
    from tests import adversarial
    scene_inputs = lambda n, w, h: adversarial.scene_inputs(n[4:], w, h)  # noqa: E731
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
W, H = 1280, 960
lib = api.load_library()
buf = (ctypes.c_ulonglong * 40)()
lib.ptmi_stats_read(buf, 1)
objs, tris, grps, cam = scene_inputs(scene, W, H)
api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 3))
lib.ptmi_stats_read(buf, 1)
names = ["walks", "node4", "leaves", "tri_tests", "verifies", "gate_rejects", "obj_gate_pass", "group_obj_tests",
         "walk_phases", "lanes_in_phases", "wave_iterations", "eager_rewalks",
         "cyc_refill", "cyc_prims_gate", "cyc_walk_phases", "cyc_shade", "cyc_loop", "exact_chain_verifies",
         "cyc_walk_loops", "walk_loop_wave_iters", "walks_no_leaf", "walks_root_only", "walks_improving", "x23",
         "ww_walker_iters", "ww_walker_lanes", "ww_walker_cycles", "ww_walker_admin_cycles", "ww_walks_posted",
         "ww_walker_empty_iters", "ww_tracer_iters", "ww_tracer_pending", "ww_tracer_ready", "ww_tracer_cycles",
         "ww_tracer_idle_iters"]
v = dict(zip(names, buf))
n = W * H * spp
print(scene, "spp", spp)
print("  lanes per walk phase %.1f, wave iterations per walk phase %.1f" % (
    v["lanes_in_phases"] / max(v["walk_phases"], 1), v["wave_iterations"] / max(v["walk_phases"], 1)))
for k in names:
    print("  %-16s %14d  per sample %8.3f  per walk %8.3f" % (k, v[k], v[k] / n, v[k] / max(v["walks"], 1)))
tot = max(v["cyc_loop"], 1)
for k in ("cyc_refill", "cyc_prims_gate", "cyc_walk_phases", "cyc_shade"):
    print("  share %-16s %.3f" % (k, v[k] / tot))
print("  cycles per walk phase %.0f, per wave iteration %.0f" % (
    v["cyc_walk_phases"] / max(v["walk_phases"], 1), v["cyc_loop"] / max(v["wave_iterations"], 1)))
print("  walk-loop cycles per phase %.0f, loop iterations per phase %.1f, cycles per loop iteration %.0f" % (
    v["cyc_walk_loops"] / max(v["walk_phases"], 1), v["walk_loop_wave_iters"] / max(v["walk_phases"], 1),
    v["cyc_walk_loops"] / max(v["walk_loop_wave_iters"], 1)))
print("  camera/prims/shade cycles per non-walk wave iteration %.0f" % (
    (v["cyc_refill"] + v["cyc_prims_gate"] + v["cyc_shade"]) / max(v["wave_iterations"], 1)))
if v["ww_walker_iters"]:
    print("  walker: lanes walking per iteration %.1f, admin share of walker cycles %.3f, cycles per iteration %.0f, "
          "empty-pool iterations %.3f" % (v["ww_walker_lanes"] / v["ww_walker_iters"],
                                          v["ww_walker_admin_cycles"] / max(v["ww_walker_cycles"], 1),
                                          v["ww_walker_cycles"] / v["ww_walker_iters"],
                                          v["ww_walker_empty_iters"] / v["ww_walker_iters"]))
    print("  tracer: pending lanes per iteration %.1f, ready lanes per iteration %.1f, iterations without a ready "
          "lane %.3f, cycles per iteration %.0f" % (v["ww_tracer_pending"] / v["ww_tracer_iters"],
                                                     v["ww_tracer_ready"] / v["ww_tracer_iters"],
                                                     v["ww_tracer_idle_iters"] / v["ww_tracer_iters"],
                                                     v["ww_tracer_cycles"] / v["ww_tracer_iters"]))
