#!/bin/bash
# DIAGNOSTIC: L2 (TCC) hit / miss and L1 (TCP) -> L2 read counters of trace_kernel, one
# --pmc pass each.  usage (GPU box, repo root): bash tools/pmc_l2.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc_l2}; shift || true
ARGS=${@:---config c5 --steps 1 --warmup 0 --samples 64 --no-cpu-baseline --no-trace-call}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for P in "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $OUT --l2-json $OUT/l2.json > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt
