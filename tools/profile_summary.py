"""Summarise a tools/profile_final.sh output directory into profiles/<round>/:
kernel_stats_<cfg>.csv, bench_<cfg>.json, pmc_c2*.{csv,json} and SUMMARY.md, plus
the derived VALU metrics of tools/pmc.sh output directories given as cfg=dir.
    python tools/profile_summary.py gpurun_out/prof_r1b profiles/r1 [c2=gpurun_out/pmc_c2 ...]
"""
import csv
import json
import os
import re
import shutil
import sys

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def valu_metrics(summary_txt):
    """VALU-active fraction, resident waves per SIMD, lane utilisation and FP64 share
    of one trace_kernel launch from tools/pmc.sh's summary (MI355X: 8 XCDs x 32 CUs x
    4 SIMDs; SQ_*_CYCLES count quad-cycles, GRBM_GUI_ACTIVE is summed over XCDs)."""
    v = {}
    with open(summary_txt) as f:
        for line in f:
            m = re.match(r"(\w+)\s+([\d.]+)\s+\(dispatches", line)
            if m:
                v[m.group(1)] = float(m.group(2))
    simd_cycles = 256 * 4 * v["GRBM_GUI_ACTIVE"] / 8
    return {"valu_active": 4 * v["SQ_ACTIVE_INST_VALU"] / simd_cycles,
            "waves_per_simd": 4 * v["SQ_WAVE_CYCLES"] / simd_cycles,
            "lane_util": v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"]),
            "fp64_share": sum(v.get(k, 0.0) for k in F64) / v["SQ_INSTS_VALU"],
            "valu_insts_per_wave": v["SQ_INSTS_VALU"] / v["SQ_WAVES"]}

CMDS = {"c2": "python3 bench.py --config c2 --steps 2 --warmup 1",
        "c4": "python3 bench.py --config c4 --samples 256 --steps 1 --warmup 1 --no-cpu-baseline --no-trace-call",
        "c5": "python3 bench.py --config c5 --samples 256 --steps 1 --warmup 1 --no-cpu-baseline --no-trace-call"}


def main(src, dst, pmc_dirs=()):
    os.makedirs(dst, exist_ok=True)
    lines = ["# rocprofv3 --kernel-trace --stats summaries (tools/profile_final.sh, one MI355X)", ""]
    for c, cmd in CMDS.items():
        shutil.copy(os.path.join(src, c, "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats_%s.csv" % c))
        shutil.copy(os.path.join(src, "bench_%s.json" % c), os.path.join(dst, "bench_%s.json" % c))
        lines.append("## %s: `%s`" % (c, cmd))
        with open(os.path.join(dst, "kernel_stats_%s.csv" % c)) as f:
            for r in csv.DictReader(f):
                if "ptmi" not in r["Name"]:
                    continue
                name = r["Name"].split("(")[0].replace("void ", "")
                lines.append("  %-36s calls %3s  avg %12.3f ms  total %12.3f ms" % (
                    name, r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
        with open(os.path.join(dst, "bench_%s.json" % c)) as f:
            b = json.load(f)
        rf = b["roofline"]
        lines.append("  bench: value %.2f Msamples/s  kernel_ms_avg (HIP events) %.3f  achieved %.3f TF/s  frac %.4f"
                     % (b["value"], rf["kernel_ms_avg"], rf["achieved"], rf["frac"]))
        if b.get("ptmi_trace_call"):
            tc = b["ptmi_trace_call"]
            lines.append("  ptmi_trace call (PCIe-inclusive, scene upload + BVH build): %.1f ms = %.2f Msamples/s"
                         % (tc["ms"], tc["value"]))
        if b.get("cpu_baseline"):
            cb = b["cpu_baseline"]
            lines.append("  cpu_baseline: %.2f %s on %d cores (%s; %s)" % (cb["value"], cb["unit"], cb["cores"],
                                                                         cb["kind"], cb["sample"]))
        lines.append("")
    for cfg, what in (("c2", "1 frame, 2048 spp"), ("c4", "1 frame, 256 spp")):
        if not os.path.exists(os.path.join(src, "pmc_%s.json" % cfg)):
            continue
        shutil.copy(os.path.join(src, "pmc_%s.json" % cfg), os.path.join(dst, "pmc_%s.json" % cfg))
        for k in ("fetch", "write"):
            shutil.copy(os.path.join(src, "%s_%s" % (cfg, k), "run_counter_collection.csv"),
                        os.path.join(dst, "pmc_%s_%s.csv" % (cfg, k)))
        with open(os.path.join(dst, "pmc_%s.json" % cfg)) as f:
            p = json.load(f)
        lines.append("## %s HBM traffic (separate --pmc passes, %s): FETCH_SIZE %.1f KB (x2 gfx950 correction), "
                     "WRITE_SIZE %.1f KB -> %.1f MB per launch" % (cfg, what, p["fetch_size_kb_raw_per_launch"],
                                                                 p["write_size_kb_per_launch"],
                                                                 p["hbm_bytes_per_launch"] / 1e6))
    if pmc_dirs:
        lines += ["", "## trace_kernel VALU counters (tools/pmc.sh, separate --pmc passes; c2 one 2048-spp frame,"
                  " c4 / c5 one 256-spp frame)", "",
                  "| config | VALU active | resident waves/SIMD | VALU lane utilisation | FP64 share of VALU insts |",
                  "|---|---|---|---|---|"]
    for arg in pmc_dirs:
        cfg, d = arg.split("=", 1)
        shutil.copy(os.path.join(d, "summary.txt"), os.path.join(dst, "pmc_valu_%s.txt" % cfg))
        m = valu_metrics(os.path.join(d, "summary.txt"))
        lines.append("| %s | %.3f | %.2f | %.3f | %.3f |" % (cfg, m["valu_active"], m["waves_per_simd"],
                                                            m["lane_util"], m["fp64_share"]))
    with open(os.path.join(dst, "SUMMARY.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
