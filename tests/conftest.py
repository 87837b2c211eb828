import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "pathtracer-ocl_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_cases():
    import glob
    import numpy as np
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz"))):
        name = os.path.basename(f)[:-4]
        if name.startswith("scene_") or name.startswith("sinf_"):
            continue
        out[name] = dict(np.load(f))
    return out
