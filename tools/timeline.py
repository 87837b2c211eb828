"""DIAGNOSTIC: work-item timeline of one trace_kernel launch (the timeline build).

  PTMI_LIB=pathtracer-ocl_amd/build/libptmi_timeline.so \
      python tools/timeline.py <config> [--samples S] [--range s0,s1] [--stride N --offset K] [out.json]

Renders the config's frame (bench.CONFIGS) once to warm up, then once with every work
item's start and end wall-clock ticks recorded (100 MHz).  Reports the launch span, the
item durations, the number of items in flight over time (its plateau = the resident
wave slots), and the slot-time lost to the ramp at the start and the drain at the end:
    lost = 1 - (sum of item durations) / (plateau x span).
"""
import argparse
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
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config")
ap.add_argument("out", nargs="?", default="")
ap.add_argument("--samples", type=int, default=0)
ap.add_argument("--range", default="")
ap.add_argument("--stride", type=int, default=1)
ap.add_argument("--offset", type=int, default=0)
a = ap.parse_args()
scene_name, W, H, S, aper, focal, _, _, desc = bench.CONFIGS[a.config]
S = a.samples or S
s0, s1 = (int(x) for x in a.range.split(",")) if a.range else (0, S)
lib = api.load_library()
assert hasattr(lib, "ptmi_diag_timeline_setup"), "library lacks ptmi_diag_timeline_setup"
lib.ptmi_diag_timeline_setup.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
objs, tris, grps, cam = scene_inputs(scene_name, W, H, aper, focal)
scene = api.Scene(0, objs, tris, grps, cam)
seeds = torch.tensor(layout.seeds_go_float64(W * H, 1234), dtype=torch.float64, device="cuda")
sums = torch.empty(W * H * 4, dtype=torch.float64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
cap = 1 << 21
buf = torch.zeros(2 * cap, dtype=torch.int64, device="cuda")
err = ctypes.create_string_buffer(512)


def render():
    scene.render(S, s0, s1, seeds.data_ptr(), sums.data_ptr(), tile_stride=a.stride, tile_offset=a.offset,
                 stream=stream)
    torch.cuda.synchronize()


render()
assert lib.ptmi_diag_timeline_setup(ctypes.c_void_p(buf.data_ptr()), cap, err, len(err)) == 0, err.value
render()
assert lib.ptmi_diag_timeline_setup(None, 0, err, len(err)) == 0, err.value
t = buf.cpu().numpy().reshape(cap, 2)
idx = np.nonzero(t[:, 1] > 0)[0]
t = t[idx].astype(np.float64)
n = len(t)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) * 1e-5, (t[:, 1] - t0) * 1e-5  # ms (100 MHz ticks)
span = en.max()
dur = en - st
# items in flight over time, 1000 bins
edges = np.linspace(0.0, span, 1001)
ev = np.concatenate([st, en])
sign = np.concatenate([np.ones(n), -np.ones(n)])
order = np.argsort(ev, kind="stable")
inflight = np.cumsum(sign[order])
bins = np.searchsorted(ev[order], edges[:-1], side="right") - 1
act = np.where(bins >= 0, inflight[np.clip(bins, 0, None)], 0)
plateau = float(np.percentile(act, 50))
busy = dur.sum()
last_start = st.max()
res = {"config": a.config, "workload": desc, "samples": [s0, s1], "frame_spp": S, "stride": a.stride,
       "items": int(n), "span_ms": round(float(span), 3), "plateau_items": plateau,
       "item_ms": {"mean": round(float(dur.mean()), 3), "p50": round(float(np.median(dur)), 3),
                   "p99": round(float(np.percentile(dur, 99)), 3), "max": round(float(dur.max()), 3)},
       "last_start_ms": round(float(last_start), 3), "drain_ms": round(float(span - last_start), 3),
       "ramp_ms": round(float(edges[np.argmax(act >= 0.95 * plateau)]), 3),
       "lost_slot_fraction": round(float(1.0 - busy / (plateau * span)), 4),
       "tail_below_90pct_ms": round(float(span - edges[np.nonzero(act >= 0.9 * plateau)[0].max()]), 3),
       # items in flight at 200 instants, and the start / end of the items by kind (whole
       # tile or chunk: the longest tenth of the items vs the rest)
       "curve": [[round(float(edges[i]), 3), int(act[i])] for i in range(0, 1000, 5)],
       # the first items in dispatch order (whole tiles in the kernels without meshes)
       "first_6144_items_ms_p0_p10_p50_p90_p100": [round(float(np.percentile(dur[:6144], q)), 3)
                                                   for q in (0, 10, 50, 90, 100)],
       # per XCD, assuming the round-robin placement of workgroups (blockIdx mod 8): the
       # summed item time and the last end
       "xcd_busy_over_mean": [round(float(dur[idx % 8 == x].sum() / (dur.sum() / 8)), 4) for x in range(8)],
       "xcd_last_end_ms": [round(float(en[idx % 8 == x].max()), 3) for x in range(8)],
       "long_items": {"count": int((dur >= np.percentile(dur, 90)).sum()),
                      "ms_p0_p10_p50_p90_p100": [round(float(np.percentile(dur[dur >= np.percentile(dur, 90)], q)), 3)
                                                 for q in (0, 10, 50, 90, 100)],
                      "last_end_ms": round(float(en[dur >= np.percentile(dur, 90)].max()), 3),
                      "last_start_ms": round(float(st[dur >= np.percentile(dur, 90)].max()), 3)}}
print(json.dumps({k: v for k, v in res.items() if k != "curve"}))
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
scene.close()
