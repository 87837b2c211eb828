#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4e; mkdir -p $OUT
PTMI_SPLIT_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- python3 bench.py --config c4 --samples 128 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/c4.json 2> $OUT/c4.err
grep "split:" $OUT/c4.err
find $OUT -name "*kernel_stats.csv" -exec cat {} \;
