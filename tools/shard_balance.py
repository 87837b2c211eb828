"""Per-rank shares of the multi-GPU splits, timed on one GPU.

    python tools/shard_balance.py [out.json] [--configs c2,c3,c4,c5] [--worlds 2,4,8]

For each BASELINE config and world size N, every rank's share of the full frame (the
sample ranges of ptmi/dist.py's cost-balanced sample split, or the round-robin 8x8 tiles
of the tile split) is rendered on device 0 exactly as bench.py's rank would render it
(ptmi_scene_render with that rank's range / tile ownership, its own work plan), and the
trace_kernel time is recorded (HIP events, median of 3).  Reported per (config, N): the
share times, max / mean, the one-GPU frame time T1, and the projected strong-scaling
efficiency T1 / (N * (max share + reduce)), with the reduce of the W*H*4-double frame
priced at 39.3 MB over one xGMI link (~153 GB/s, MI355X_MICROARCH.md) -- a projection from
one-GPU timings, not a scaling measurement.
"""
import argparse
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pathtracer-ocl_amd")]
import torch  # noqa: E402
from ptmi import api, layout  # noqa: E402
from ptmi import dist as pdist  # noqa: E402
from tests.scene_inputs import scene_inputs  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out", nargs="?", default="")
ap.add_argument("--configs", default="c2,c3,c4,c5")
ap.add_argument("--worlds", default="2,4,8")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--split", default="", help="sample|tile: override every config's split")
ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                help="a work-plan knob of every scene (ptmi_diag_set_knob), as bench.py --knob")
a = ap.parse_args()
knobs = [(getattr(api, "KNOB_" + kv.split("=")[0].strip().upper()), int(kv.split("=")[1])) for kv in a.knob]
XGMI_GBS = 153.0
res = {"what": __doc__.strip().splitlines()[0], "device": api.device_name(0), "knobs": a.knob, "configs": {}}
for cfg in a.configs.split(","):
    scene_name, W, H, S, aper, focal, split, _, desc = bench.CONFIGS[cfg]
    split = a.split or split
    objs, tris, grps, cam = scene_inputs(scene_name, W, H, aper, focal)
    scene = api.Scene(0, objs, tris, grps, cam)
    for k, v in knobs:
        assert scene.set_knob(k, v) == api.PTMI_OK, (k, v)
    seeds = torch.tensor(layout.seeds_go_float64(W * H, 1234), dtype=torch.float64, device="cuda")
    sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def timed(s0, s1, stride, off):
        scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=stride, tile_offset=off, stream=stream)
        torch.cuda.synchronize()
        scene.kernel_time()
        scene.set_timing(True)
        t = []
        for _ in range(a.reps):
            scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=stride, tile_offset=off,
                         stream=stream)
            torch.cuda.synchronize()
            ms, n = scene.kernel_time()
            t.append(ms / max(n, 1))
        scene.set_timing(False)
        return sorted(t)[len(t) // 2]

    t1 = timed(0, S, 1, 0)
    reduce_ms = W * H * 4 * 8 / (XGMI_GBS * 1e9) * 1e3
    entry = {"workload": desc, "split": split, "t1_ms": round(t1, 3), "reduce_ms_model": round(reduce_ms, 3),
             "worlds": {}}
    for n in [int(x) for x in a.worlds.split(",")]:
        shares = []
        for r in range(n):
            s0, s1, stride, off = pdist.shard(r, n, S, split)
            shares.append(round(timed(s0, s1, stride, off), 3))
        mx, mean = max(shares), sum(shares) / n
        entry["worlds"][str(n)] = {"share_ms": shares, "max_over_mean": round(mx / mean, 4),
                                   "sum_over_t1": round(sum(shares) / t1, 4),
                                   "projected_efficiency": round(t1 / (n * (mx + reduce_ms)), 4)}
        print(cfg, n, "max/mean %.4f" % (mx / mean), "sum/T1 %.4f" % (sum(shares) / t1),
              "proj eff %.3f" % (t1 / (n * (mx + reduce_ms))), flush=True)
    res["configs"][cfg] = entry
    scene.close()
print(json.dumps(res))
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
