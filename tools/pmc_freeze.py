"""Freeze the rocprofv3 PMC measurements of one profiling round into
profiles/pmc_measured.json, which bench.py reads for the measured levels of its
roofline (HBM bytes per trace_kernel launch; L2 requests and hit rate; VALU issue).

    python tools/pmc_freeze.py profiles/r3 [--out profiles/pmc_measured.json]

Inputs in the round directory, per config c in c2..c5 (all optional):
  pmc_<c>.json   tools/pmc_traffic.py output (FETCH_SIZE x2 + WRITE_SIZE per launch)
  l2_<c>.json    tools/pmc_l2_summary.py output (TCP->TCC read requests, TCC hit/miss)
  valu_<c>.json  tools/pmc_summary.py --json output (VALU issue / lane utilisation)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import build_id  # noqa: E402

KEYS = {"c2": "c2_reference_1280x960", "c3": "c3_reference_dof_1280x960", "c4": "c4_teapot_1280x960",
        "c5": "c5_gopher_1280x960"}


def _load(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("round_dir")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                                  "pmc_measured.json"))
    ap.add_argument("--spp", type=int, default=2048, help="samples per pixel of the profiled frames")
    ap.add_argument("--build", default=None, help="build id of the profiled library (default: this tree's)")
    a = ap.parse_args()
    out = {"what": "rocprofv3 PMC measurements per trace_kernel launch of one full %d-spp frame, "
                   "frozen from %s by tools/pmc_freeze.py" % (a.spp, os.path.normpath(a.round_dir)),
           "build": a.build or build_id(), "spp": a.spp,
           "build_note": "bench.py reports these counters only for the build they were measured on "
                         "(bench.build_id: a hash of the kernel sources)",
           "workloads": {}}
    for c, key in KEYS.items():
        w = {}
        t = _load(os.path.join(a.round_dir, "pmc_%s.json" % c))
        if t:
            w["hbm_bytes_per_launch"] = t["hbm_bytes_per_launch"]
        l2 = _load(os.path.join(a.round_dir, "l2_%s.json" % c))
        if l2:
            w["l2_read_bytes_per_launch"] = l2["l2_read_bytes_per_launch"]
            w["l2_hit_rate"] = l2["l2_hit_rate"]
        v = _load(os.path.join(a.round_dir, "valu_%s.json" % c))
        if v:
            w["valu"] = v
        if w:
            w["source"] = os.path.join(os.path.normpath(a.round_dir), "{pmc,l2,valu}_%s.json" % c)
            out["workloads"][key] = w
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
