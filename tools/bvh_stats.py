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
buf = (ctypes.c_ulonglong * 80)()
lib.ptmi_stats_read(buf, 1)
objs, tris, grps, cam = scene_inputs(scene, W, H)
api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 3))
lib.ptmi_stats_read(buf, 1)
names = ["walks", "node4", "leaves", "tri_tests", "verifies", "gate_rejects", "obj_gate_pass", "group_obj_tests",
         "walk_phases", "lanes_in_phases", "wave_iterations", "eager_rewalks",
         "cyc_refill", "cyc_prims_gate", "cyc_walk_phases", "cyc_shade", "cyc_loop", "exact_chain_verifies",
         "cyc_walk_loops", "walk_loop_wave_iters", "walks_no_leaf", "walks_root_only", "walks_improving", "x23",
         "lanes_ready", "lanes_pending", "lanes_starving", "lanes_finished", "lanes_prims", "cyc_walk_node",
         "cyc_walk_leaf", "walk_leaf_sections"]
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
it = max(v["wave_iterations"], 1)
print("  lanes per wave iteration: shade %.1f, pending %.1f, starving %.1f, finished %.1f, prims %.1f" % (
    v["lanes_ready"] / it, v["lanes_pending"] / it, v["lanes_starving"] / it, v["lanes_finished"] / it,
    v["lanes_prims"] / it))
print("  walk loop: node-section cycles %.3f, leaf-section cycles %.3f of walk-loop cycles; leaf sections per "
      "wave loop iteration %.2f" % (v["cyc_walk_node"] / max(v["cyc_walk_loops"], 1),
                                     v["cyc_walk_leaf"] / max(v["cyc_walk_loops"], 1),
                                     v["walk_leaf_sections"] / max(v["walk_loop_wave_iters"], 1)))
