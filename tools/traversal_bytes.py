"""Executed traversal work per primary sample of the BVH configs (C4, C5), counted
by the kernel's own stats build (libptmi_stats.so, PTMI_STATS=1), for bench.py's
HBM roofline of those configs (bytes per sample).  Bytes per visit
follow the device layouts (csrc/ptmi_device.h): a Node4 64 B, a DevTri 80 B, a
winning triangle's DevTriShade 128 B.
    on the GPU box:  PTMI_LIB=pathtracer-ocl_amd/build/libptmi_stats.so \
                     python tools/traversal_bytes.py run gpurun_out/traversal.json [spp]
    here:            python tools/traversal_bytes.py merge gpurun_out/traversal.json
(merge writes them into profiles/alg_counts.json as workloads[*]["traversal"])."""
import ctypes
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
NODE4_B, TRI_B, SHADE_B = 64, 80, 128
CONFIGS = {"c4_teapot_1280x960": "teapot", "c5_gopher_1280x960": "gopher"}


def run(out_path, spp):
    import torch  # noqa: F401
    from ptmi import api, layout
    from tests.scene_inputs import scene_inputs
    lib = api.load_library()
    buf = (ctypes.c_ulonglong * 80)()
    res = {}
    for key, scene in CONFIGS.items():
        W, H = 1280, 960
        objs, tris, grps, cam = scene_inputs(scene, W, H)
        lib.ptmi_stats_read(buf, 1)  # reset
        api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(W * H, 1234))
        lib.ptmi_stats_read(buf, 1)
        n = W * H * spp
        c = {"walks": buf[0], "node4": buf[1], "leaves": buf[2], "tri_tests": buf[3], "tri_winners": buf[4]}
        per = {k: v / n for k, v in c.items()}
        per["bytes_per_sample"] = per["node4"] * NODE4_B + per["tri_tests"] * TRI_B + per["tri_winners"] * SHADE_B
        per["sample"] = "%dx%d, %d spp, seeds PCG64(1234)" % (W, H, spp)
        res[key] = per
        print(key, json.dumps(per))
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


def merge(in_path):
    p = os.path.join(ROOT, "profiles", "alg_counts.json")
    with open(p) as f:
        ac = json.load(f)
    with open(in_path) as f:
        tr = json.load(f)
    for key, per in tr.items():
        per["basis"] = ("executed by ptmi's traversal index (kernel stats build): Node4 %d B, DevTri %d B, "
                        "DevTriShade %d B per visit" % (NODE4_B, TRI_B, SHADE_B))
        ac["workloads"][key]["traversal"] = per
    with open(p, "w") as f:
        json.dump(ac, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 16)
    else:
        merge(sys.argv[2])
