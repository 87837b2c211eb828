"""Summarise tools/pmc_stall.sh: a wave-cycle table for trace_kernel.

    python tools/pmc_stall.py <dir> [--json out.json]

SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready but
not issued: dependency or pipe busy) + SQ_ACTIVE_INST_ANY (issuing), all in quad-cycles
(MI355X_MICROARCH.md, rocprofv3 PMC slots).  Per-instruction-type cycles are the
SQ_ACTIVE_INST_* buckets; instruction counts the SQ_INSTS_* counters.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--json")
a = ap.parse_args()
vals = defaultdict(float)
disp = defaultdict(set)
for f in glob.glob(os.path.join(a.dir, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "trace_kernel" not in r.get("Kernel_Name", ""):
                continue
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r.get("Dispatch_Id"))
v = vals
for k in sorted(v):
    print("%-24s %20.0f  (dispatches %d)" % (k, v[k], len(disp[k])))
res = {}
wc = v.get("SQ_WAVE_CYCLES", 0.0)
if wc:
    print("\nshare of wave cycles:")
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_FLAT",
              "SQ_WAIT_INST_LDS"):
        if k in v:
            res[k.lower() + "_frac"] = v[k] / wc
            print("  %-22s %.3f" % (k, v[k] / wc))
vi = v.get("SQ_INSTS_VALU", 0.0)
if vi:
    print("\nper VALU instruction:")
    for k in ("SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD",
              "SQ_INSTS_VMEM_WR", "SQ_LDS_BANK_CONFLICT"):
        if k in v:
            res[k.lower() + "_per_valu"] = v[k] / vi
            print("  %-22s %.4f" % (k, v[k] / vi))
if v.get("SQ_INSTS_LDS"):
    res["lds_bank_conflict_per_lds_inst"] = v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_INSTS_LDS"]
if v.get("GRBM_GUI_ACTIVE") and wc:
    n = max(len(disp["GRBM_GUI_ACTIVE"]), 1)
    cyc = v["GRBM_GUI_ACTIVE"] / n / 8.0
    res["resident_waves_per_simd"] = wc / max(len(disp["SQ_WAVE_CYCLES"]), 1) * 4 / (cyc * 1024)
    print("resident waves / SIMD    %.2f" % res["resident_waves_per_simd"])
if a.json:
    with open(a.json, "w") as f:
        json.dump(res, f, indent=1)
