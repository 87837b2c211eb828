"""DIAGNOSTIC: compare two builds of libptmi.so on one small frame (subprocess per build).
    python tools/ab_diff.py <libA> <libB> <scene> <w> <h> <spp> [seed]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if len(sys.argv) > 1 and sys.argv[1] == "--render":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
    import torch  # noqa: F401
    from ptmi import api, layout
    from tests.scene_inputs import scene_inputs
    scene, w, h, spp, seed, outp = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), sys.argv[7]
    objs, tris, grps, cam = scene_inputs(scene, w, h)
    out = api.Trace(objs, tris, grps, 0, spp, cam, seeds=layout.seeds_go_float64(w * h, seed))
    np.save(outp, out)
    sys.exit(0)
a, b, scene, w, h, spp = sys.argv[1:7]
seed = sys.argv[7] if len(sys.argv) > 7 else "105"
imgs = []
for k, lib in enumerate((a, b)):
    o = "/tmp/ab_%d.npy" % k
    subprocess.run([sys.executable, __file__, "--render", scene, w, h, spp, seed, o], check=True,
                   env=dict(os.environ, PTMI_LIB=lib))
    imgs.append(np.load(o).reshape(int(h), int(w), 4))
d = np.abs(imgs[0] - imgs[1]).max(axis=2)
ys, xs = np.nonzero(d > 1e-9)
print(scene, "max diff %.3e, pixels > 1e-9: %d of %d" % (d.max(), len(ys), d.size))
for y, x in list(zip(ys, xs))[:20]:
    print("  (%d,%d) tile %d lane %d: %s vs %s" % (x, y, (y // 8) * ((int(w) + 7) // 8) + x // 8, (y % 8) * 8 + x % 8,
                                                 imgs[0][y, x, :3], imgs[1][y, x, :3]))
