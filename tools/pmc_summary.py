"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) for trace_kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(float)
disp = defaultdict(set)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "trace_kernel" not in r.get("Kernel_Name", ""):
                continue
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r.get("Dispatch_Id"))
for k in sorted(vals):
    print("%-28s %18.0f  (dispatches %d)" % (k, vals[k], len(disp[k])))
v = vals
if v.get("SQ_WAVES"):
    print("VALU insts / wave        %.0f" % (v["SQ_INSTS_VALU"] / v["SQ_WAVES"]))
if v.get("SQ_THREAD_CYCLES_VALU") and v.get("SQ_ACTIVE_INST_VALU"):
    print("VALU lane utilisation    %.3f" % (v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"])))
f64 = sum(v.get(k, 0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                               "SQ_INSTS_VALU_TRANS_F64"))
if f64 and v.get("SQ_INSTS_VALU"):
    print("FP64 share of VALU insts %.3f" % (f64 / v["SQ_INSTS_VALU"]))
for k in ("FETCH_SIZE", "WRITE_SIZE"):
    if k in v:
        print("%s (KB, summed)  %.0f" % (k, v[k]))
