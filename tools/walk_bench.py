"""DIAGNOSTIC: standalone BVH walk kernels against the mesh kernel's
in-loop walk phases, on the walks of a real frame.

  PTMI_LIB=pathtracer-ocl_amd/build/libptmi_capture.so \
      python tools/walk_bench.py capture <scene> <s0> <s1> [out.json]
      -> renders samples [s0, s1) of the 1280x960 2048-spp frame while capturing every walk
         of the walk phases (ray, primitive best, result), then walks the captured requests
         with walk_kernel (mode 0, one per lane) and walk_pool_kernel (mode 1, persistent
         with refill), 3 timed runs each, and checks their results bit for bit against
         the mesh kernel's own.
  PTMI_LIB=<product or timers lib> python tools/walk_bench.py frame <scene> <s0> <s1> [out.json]
      -> kernel time of the same sample range (3 runs); with the timers library
         (PTMI_STATS=2) also the walk phases' share of the loop clock.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402

mode, scene_name, s0, s1 = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
out_path = sys.argv[5] if len(sys.argv) > 5 else None
W, H, S = 1280, 960, 2048
lib = api.load_library()
objs, tris, grps, cam = scene_inputs(scene_name, W, H)
scene = api.Scene(0, objs, tris, grps, cam)
seeds = torch.tensor(layout.seeds_go_float64(W * H, 1234), dtype=torch.float64, device="cuda")
sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
err = ctypes.create_string_buffer(512)
res = {"scene": scene_name, "samples": [s0, s1], "frame_spp": S, "lib": os.environ.get("PTMI_LIB", "product")}


def render():
    scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), stream=stream)


if mode == "frame":
    render()
    torch.cuda.synchronize()
    scene.kernel_time()
    has_stats = hasattr(lib, "ptmi_stats_read")
    buf = (ctypes.c_ulonglong * 80)()
    if has_stats:
        lib.ptmi_stats_read.restype = ctypes.c_int
        lib.ptmi_stats_read(buf, 1)
    scene.set_timing(True)
    for _ in range(3):
        render()
    torch.cuda.synchronize()
    ms, n = scene.kernel_time()
    res["kernel_ms"] = ms / n
    if has_stats:
        lib.ptmi_stats_read(buf, 1)
        v = list(buf)
        lp = max(v[16], 1)
        res["timers"] = {"walk_phase_share": v[14] / lp, "prims_share": v[13] / lp, "shade_share": v[15] / lp,
                         "camera_share": v[12] / lp, "walk_phases": v[8] / 3, "lanes_in_phases": v[9] / 3}
else:
    cap = 1 << 24
    for f in ("ptmi_diag_capture_setup", "ptmi_diag_capture_count", "ptmi_diag_walk"):
        assert hasattr(lib, f), "library lacks %s (use the capture build)" % f
    lib.ptmi_diag_capture_setup.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p,
                                            ctypes.c_size_t]
    lib.ptmi_diag_capture_count.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_size_t]
    lib.ptmi_diag_walk.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_char_p,
                                   ctypes.c_size_t]
    req = torch.zeros(cap * 64, dtype=torch.uint8, device="cuda")
    ref = torch.zeros(cap * 48, dtype=torch.uint8, device="cuda")
    rc = lib.ptmi_diag_capture_setup(ctypes.c_void_p(req.data_ptr()), ctypes.c_void_p(ref.data_ptr()), cap, err,
                                     len(err))
    assert rc == 0, err.value
    render()
    torch.cuda.synchronize()
    cnt = ctypes.c_uint32(0)
    assert lib.ptmi_diag_capture_count(ctypes.byref(cnt), err, len(err)) == 0, err.value
    n = min(cnt.value, cap)
    res["walks_in_range"] = cnt.value
    res["walks_measured"] = n
    counter = torch.zeros(4, dtype=torch.int32, device="cuda")
    refv = ref[: n * 48].view(n, 48)
    for m in (0, 1):
        times = []
        mism = None
        for rep in range(3):
            got = torch.zeros(n * 48, dtype=torch.uint8, device="cuda")
            ms = ctypes.c_float(0)
            rc = lib.ptmi_diag_walk(scene._h, m,
                                    ctypes.c_void_p(req.data_ptr()), n, ctypes.c_void_p(got.data_ptr()),
                                    ctypes.c_void_p(counter.data_ptr()), ctypes.c_void_p(stream), ctypes.byref(ms),
                                    err, len(err))
            assert rc == 0, err.value
            times.append(ms.value)
            if rep == 0:
                gv = got.view(n, 48)
                # t, pk, tri, ti (bytes 0..20) and u, v (24..40): bit for bit
                diff = (gv[:, 0:20] != refv[:, 0:20]).any(1) | (gv[:, 24:40] != refv[:, 24:40]).any(1)
                mism = int(diff.sum().item())
            del got
        best = min(times)
        res["mode%d" % m] = {"ms": times, "ns_per_walk_chip": best * 1e6 / max(n, 1), "mismatches": mism}
    t = np.frombuffer(ref[: n * 48].cpu().numpy().tobytes(), dtype=np.int32).reshape(n, 12)
    res["winner_is_triangle"] = float((t[:, 3] >= 0).mean())
print(json.dumps(res))
if out_path:
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
