"""The premise of the kernel's hemisphere table (DESIGN.md §2 item 9,
ptmi_kernels.hip random_hemisphere / hemi_table_kernel): a noise3D uniform
(tracer.cl:314-317) is fract(v) with v = sin(s) * 43758.5453f, an exact float
difference and so a multiple of ulp(v) -- on the table's 2^-16 grid whenever
|v| >= 128.  Checked on the CPU restatement of noise3D over the hemisphere's own
argument pattern (noise3D(fgi, b, n) and noise3D(b, n, fgi), tracer.cl:1057)."""
import numpy as np

import pyoracle


def _grid(u):
    t = np.float32(u) * np.float32(65536.0)
    return float(t) == float(np.floor(t))


def test_hemisphere_uniforms_mostly_on_the_table_grid():
    rng = np.random.default_rng(11)
    fgis = rng.random(40).astype(np.float32)
    on = total = 0
    for fgi in fgis:
        for n in range(0, 2048, 41):
            for b in range(0, 10, 3):
                for x, y, z in ((fgi, b, n), (b, n, fgi)):
                    # the calls the kernel makes: noise3d(fgi, b, n) and noise3d(b, n, fgi)
                    u = pyoracle.noise3d(float(np.float32(x)), float(np.float32(y)), float(np.float32(z)))
                    total += 1
                    on += _grid(u)
                    if not _grid(u):
                        # off the grid only when |v| < 128, i.e. |sin| < 128 / 43758.5453
                        s = np.float32(np.float32(x) * np.float32(112.9898)) + np.float32(np.float32(y) * np.float32(179.233))
                        s = np.float32(s + np.float32(np.float32(z) * np.float32(237.212)))
                        assert abs(pyoracle.sinf(float(s))) < 128.0 / 43758.5453 * (1 + 1e-6)
    assert total > 10000
    assert on / total > 0.99, "only %.4f of the hemisphere uniforms are on the 2^-16 grid" % (on / total)
