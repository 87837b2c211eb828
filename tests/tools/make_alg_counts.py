"""Freeze the algorithmic work per primary sample of the benchmark workloads into
profiles/alg_counts.json (read by bench.py for roofline.achieved).

Runs the oracle's event-counting build (oracle/build/libptoracle_count.so) over a
sample of each workload (full frame width, every k-th row band, fixed seeds) and
applies the cost model in ptmi/flops.py.  Test/measurement tooling only.

    python tests/tools/make_alg_counts.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
from ptmi import flops, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

WORKLOADS = {
    "c2_reference_1280x960": ("reference", 1280, 960, 2048, 0.0, 0.0),
    "c3_reference_dof_1280x960": ("reference", 1280, 960, 2048, 0.15, 1.6),
    "c4_teapot_1280x960": ("teapot", 1280, 960, 2048, 0.0, 0.0),
    "c5_gopher_1280x960": ("gopher", 1280, 960, 2048, 0.0, 0.0),
}


def main(rows=24, spp_sample=8):
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libptoracle_count.so"))
    lib.pto_trace.restype = ctypes.c_int
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.pto_trace.argtypes = [vp, u32, vp, u32, vp, u32, vp, u32, vp, u32, u32, u32, u32, ctypes.c_int, vp]
    lib.pto_event_counts.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    out = {"model": "ptmi/flops.py", "bytes_model": "ptmi/flops.py BYTES (reference visit rules)", "sample": "rows every H/%d, %d spp of the frame's sample range" % (rows, spp_sample),
           "workloads": {}}
    for name, (scene, w, h, spp, ap, fl) in WORKLOADS.items():
        objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
        tris, grps = layout.pad_empty(tris, grps)
        seeds = layout.seeds_go_float64(w * h, 1234)
        tot = np.zeros(len(flops.EVENTS), dtype=np.uint64)
        t0 = time.time()
        for band in range(rows):
            r = band * (h // rows) + (h // rows) // 2
            # spread the sample indices over [0, spp): n = k * spp / spp_sample
            for k in range(spp_sample):
                n0 = k * (spp // spp_sample)
                buf = np.zeros(w * 4)
                rc = lib.pto_trace(objs.ctypes.data, len(objs), tris.ctypes.data, len(tris), grps.ctypes.data,
                                   len(grps), np.asarray(cam).reshape(1).ctypes.data, spp, seeds.ctypes.data, r, 1,
                                   n0, n0 + 1, 0, buf.ctypes.data)
                assert rc == 0
                c = (ctypes.c_uint64 * len(flops.EVENTS))()
                lib.pto_event_counts(c, len(flops.EVENTS))
                tot += np.frombuffer(c, dtype=np.uint64)
        counts = {e: int(v) for e, v in zip(flops.EVENTS, tot)}
        f64, f32 = flops.flops_per_sample(counts)
        out["workloads"][name] = {"scene": scene, "width": w, "height": h, "samples": spp, "aperture": ap,
                                  "focal_length": fl, "events": counts, "fp64_flops_per_sample": f64,
                                  "fp32_flops_per_sample": f32,
                                  "bytes_per_sample": flops.bytes_per_sample(counts),
                                  "bounces_per_sample": counts["hit"] / counts["sample"],
                                  "obj_tests_per_sample": counts["obj_test"] / counts["sample"]}
        print("%-28s %7.1f s  fp64 flops/sample %8.1f  hits/sample %.3f  tri tests/sample %.1f" % (
            name, time.time() - t0, f64, counts["hit"] / counts["sample"], counts["tri_det"] / counts["sample"]))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "alg_counts.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
