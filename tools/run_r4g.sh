#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4g; mkdir -p $OUT
PTMI_SPLIT_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- python3 bench.py --config c4 --samples 512 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/c4.json 2> $OUT/c4.err
grep "split:" $OUT/c4.err
find $OUT -name "*kernel_stats.csv" -exec grep -E "split|trace_kernel" {} \; | cut -c1-200
bash tools/split_sweep.sh gpurun_out/sw3 512 "c4" "s2:PTMI_SPLIT_SLOTS=2 s1:PTMI_SPLIT_SLOTS=1 b2:PTMI_SPLIT_BUDGET=2 b8:PTMI_SPLIT_BUDGET=8 c32:PTMI_SPLIT_CHUNK=32 c128:PTMI_SPLIT_CHUNK=128 y32:PTMI_SPLIT_SYNC=32"
