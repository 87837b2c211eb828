"""Generate golden vectors from THE REFERENCE KERNEL ITSELF.

Runs /root/reference/internal/ocl/tracer.cl -- compiled unmodified (two
preprocessor flags, see oracle/Makefile) by ROCm's OpenCL toolchain into
oracle/_ref/tracer_ref.hsaco -- on an MI355X through the HSA launcher
(oracle/ref_launch.c), on the scene records ptmi builds, with fixed seeds.
Each case is written as tests/golden/<case>.npz: inputs (records, seeds,
samples) and the reference's float64 RGBA output.

Run on a GPU box (oracle/_ref is built here and travels with the snapshot):
    python tests/golden/make_golden.py --out gpurun_out/golden [--cases a,b]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "pathtracer-ocl_amd"))
sys.path.insert(0, ROOT)
from ptmi import layout, scenes  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

# name: (scene, W, H, samples, aperture, focal, seed)
CASES = {
    "ref_64x48_s4": ("reference", 64, 48, 4, 0.0, 0.0, 11),
    "ref_64x48_s16": ("reference", 64, 48, 16, 0.0, 0.0, 12),
    "ref_40x30_s3": ("reference", 40, 30, 3, 0.0, 0.0, 13),
    "ref_dof_64x48_s8": ("reference", 64, 48, 8, 0.15, 1.6, 14),
    "ocl_64x48_s8": ("default", 64, 48, 8, 0.0, 0.0, 15),
    "ocl_dof_48x32_s5": ("default", 48, 32, 5, 0.15, 1.6, 16),
    "teapot_32x24_s4": ("teapot", 32, 24, 4, 0.0, 0.0, 17),
    "gopher_32x24_s4": ("gopher", 32, 24, 4, 0.0, 0.0, 18),
    "ref_160x120_s4": ("reference", 160, 120, 4, 0.0, 0.0, 19),
    # material paths: glass (RI 1.52) / diffuse RI 1.57 / mirror / thin glass (RI -1)
    "transp_48x32_s6": ("transparency", 48, 32, 6, 0.0, 0.0, 20),
    "transp_quad_48x32_s4": ("transparency_quad_lights", 48, 32, 4, 0.0, 0.0, 21),
    "transp_f_dof_48x32_s5": ("transparency_f_light", 48, 32, 5, 0.15, 1.6, 22),
    "reflect_48x32_s6": ("reflection", 48, 32, 6, 0.0, 0.0, 23),
    "glassteapot_32x24_s4": ("transparent_teapot", 32, 24, 4, 0.0, 0.0, 24),
}


def run_case(name, out_dir):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    scene, w, h, spp, ap, fl, seed = CASES[name]
    objs, tris, grps, cam = scene_inputs(scene, w, h, ap, fl)
    tris_p, grps_p = layout.pad_empty(tris, grps)
    seeds = layout.seeds_go_float64(w * h, seed)
    t = time.time()
    out = pyoracle.ref_trace(objs, tris_p, grps_p, cam, spp, seeds)
    dt = time.time() - t
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), scene=scene, width=w, height=h,
                        samples=spp, aperture=ap, focal_length=fl, seed=seed,
                        objects=objs.view(np.uint8), camera=np.asarray(cam).reshape(1).view(np.uint8),
                        seeds=seeds, rgba=out)
    img = out.reshape(h, w, 4)
    print("%-20s %5.2fs  mean rgb %s  nan %d" % (name, dt, img[..., :3].mean(axis=(0, 1)),
                                                  int(np.isnan(out).sum())), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "golden"))
    ap.add_argument("--cases", default=",".join(CASES))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for c in a.cases.split(","):
        run_case(c, a.out)


if __name__ == "__main__":
    main()
