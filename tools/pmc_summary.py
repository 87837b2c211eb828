"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh, tools/pmc_l2.sh) for trace_kernel.

    python tools/pmc_summary.py <pmc_dir> [--valu-json out.json] [--l2-json out.json]

Per-launch figures divide the summed counters by the number of trace_kernel
dispatches seen for that counter.  Issue rate: VALU wave-instructions per SIMD-cycle,
with the frame's cycles = GRBM_GUI_ACTIVE / 8 XCDs and 1024 SIMDs (wave64 peak 0.5 on
gfx950's SIMD-32: one wave64 VALU instruction per 2 cycles; FP64 FMA takes 4).
L2: TCP->TCC read requests x 64 B (uncalibrated request size) and the TCC hit rate.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--valu-json")
ap.add_argument("--l2-json")
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
for k in sorted(vals):
    print("%-28s %18.0f  (dispatches %d)" % (k, vals[k], len(disp[k])))
v = vals


def per(k):
    return v[k] / max(len(disp[k]), 1)


res = {}
if v.get("SQ_WAVES"):
    res["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
    print("VALU insts / wave        %.0f" % res["valu_insts_per_wave"])
if v.get("SQ_INSTS_VALU"):
    res["valu_insts_per_launch"] = per("SQ_INSTS_VALU")
if v.get("SQ_THREAD_CYCLES_VALU") and v.get("SQ_ACTIVE_INST_VALU"):
    res["lane_utilisation"] = v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"])
    print("VALU lane utilisation    %.3f" % res["lane_utilisation"])
f64 = sum(v.get(k, 0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                               "SQ_INSTS_VALU_TRANS_F64"))
if f64 and v.get("SQ_INSTS_VALU"):
    res["fp64_share"] = f64 / v["SQ_INSTS_VALU"]
    print("FP64 share of VALU insts %.3f" % res["fp64_share"])
    # FP64 flops the kernel executed: (ADD + MUL + TRANS + 2 FMA) wave-instructions x 64 lanes x
    # the VALU lane utilisation (the FP64 instructions' own lane mask is not counted separately)
    ops = sum(per(k) for k in ("SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")) + \
        2 * per("SQ_INSTS_VALU_FMA_F64")
    res["fp64_wave_ops_per_launch"] = ops
    if res.get("lane_utilisation"):
        res["fp64_flops_executed_per_launch"] = ops * 64 * res["lane_utilisation"]
        print("FP64 flops executed / launch %.4g (lane-utilisation weighted)" % res["fp64_flops_executed_per_launch"])
if v.get("GRBM_GUI_ACTIVE") and v.get("SQ_INSTS_VALU"):
    cyc = per("GRBM_GUI_ACTIVE") / 8.0
    res["frame_cycles"] = cyc
    res["valu_insts_per_simd_cycle"] = per("SQ_INSTS_VALU") / (cyc * 1024)
    print("VALU insts / SIMD-cycle  %.4f" % res["valu_insts_per_simd_cycle"])
    if v.get("SQ_WAVE_CYCLES"):
        res["resident_waves_per_simd"] = per("SQ_WAVE_CYCLES") * 4 / (cyc * 1024)
        print("resident waves / SIMD    %.2f" % res["resident_waves_per_simd"])
for k in ("FETCH_SIZE", "WRITE_SIZE"):
    if k in v:
        print("%s (KB, summed)  %.0f" % (k, v[k]))
l2 = {}
if v.get("TCC_HIT_sum") is not None and (v.get("TCC_HIT_sum", 0) + v.get("TCC_MISS_sum", 0)) > 0:
    l2["l2_hit_rate"] = v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
    print("L2 hit rate              %.4f" % l2["l2_hit_rate"])
if v.get("TCP_TCC_READ_REQ_sum"):
    l2["tcp_tcc_read_req_per_launch"] = per("TCP_TCC_READ_REQ_sum")
    l2["l2_read_bytes_per_launch"] = 64.0 * l2["tcp_tcc_read_req_per_launch"]
    l2["request_bytes"] = "64 B per TCP->TCC read request (uncalibrated)"
    print("TCP->TCC read req/launch %.0f" % l2["tcp_tcc_read_req_per_launch"])
if v.get("TCP_TOTAL_CACHE_ACCESSES_sum") and v.get("TCP_TCC_READ_REQ_sum"):
    l2["l1_to_l2_fraction"] = v["TCP_TCC_READ_REQ_sum"] / v["TCP_TOTAL_CACHE_ACCESSES_sum"]
if a.valu_json and res:
    with open(a.valu_json, "w") as f:
        json.dump(res, f, indent=1)
if a.l2_json and l2:
    with open(a.l2_json, "w") as f:
        json.dump(l2, f, indent=1)
