#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4f; mkdir -p $OUT
A="--config c4 --samples 256 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
P="SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
for sp in 1 0; do
  PTMI_SPLIT_SLOTS=8 PTMI_SPLIT=$sp timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $OUT/s$sp -o run -- python3 bench.py $A > $OUT/s$sp.log 2>&1
  python3 - <<PY
import csv,glob,collections
v=collections.defaultdict(float); n=collections.defaultdict(int)
for f in glob.glob("$OUT/s$sp/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k=r["Kernel_Name"]
        if "ptmi::" not in k: continue
        key=k.split("(")[0][:40]
        v[(key,r["Counter_Name"])]+=float(r["Counter_Value"])
for (k,c),x in sorted(v.items()): print("split=$sp", k, c, "%.4g"%x)
PY
done
