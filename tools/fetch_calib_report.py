"""DIAGNOSTIC: tables of tools/fetch_calib.sh's passes -- every counter per dispatch of the
calibration kernels (with the bytes each requested) and of the mesh frames' trace_kernel.
    python3 tools/fetch_calib_report.py <outdir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

REQ = {"stream16": 1 << 30, "line64_scat": 1 << 29, "line128_scat": 1 << 30, "word8_scat": (1 << 23) * 8}
LINES = 1 << 23


def load(d):
    rows = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            rows[(int(r["Dispatch_Id"]), name)][r["Counter_Name"]] = float(r["Counter_Value"])
    return rows


def main():
    out = sys.argv[1]
    for sub in sorted(os.listdir(out)):
        d = os.path.join(out, sub)
        if not os.path.isdir(d):
            continue
        rows = load(d)
        if not rows:
            continue
        print("==", sub)
        for (disp, name), cs in sorted(rows.items()):
            short = name.split("::")[-1]
            if not (short in REQ or short.startswith("trace_kernel")):
                continue
            line = "  %-26s" % short[:26]
            for k, v in sorted(cs.items()):
                line += "  %s %.4g" % (k, v)
            if short in REQ:
                line += "  | requested %.4g B, %d lines" % (REQ[short], LINES)
                if "FETCH_SIZE" in cs:
                    line += ", FETCH_SIZE*1024/requested %.3f, per line %.1f B" % (
                        cs["FETCH_SIZE"] * 1024 / REQ[short], cs["FETCH_SIZE"] * 1024 / LINES)
                for k, v in sorted(cs.items()):
                    if k.startswith("TCC_"):
                        line += ", %s per line %.3f" % (k, v / LINES)
            print(line)


if __name__ == "__main__":
    main()
