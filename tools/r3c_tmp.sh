#!/bin/bash
# DIAGNOSTIC scratch: tail-item sweep with write traffic
set -e -o pipefail
O=gpurun_out/r3k; mkdir -p $O
bash tools/diag_ab.sh $O 2048 "c2" "base base:PTMI_TAIL_ITEMS=6 base:PTMI_TAIL_ITEMS=5 base base:PTMI_TAIL_ITEMS=6 base:PTMI_TAIL_ITEMS=5"
export TMPDIR=/tmp
for v in 6 5; do
PTMI_TAIL_ITEMS=$v timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$v -o run -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $O/w$v.log 2>&1
PTMI_TAIL_ITEMS=$v timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$v -o run -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $O/f$v.log 2>&1
done
grep -h "trace_kernel" $O/w6/run_counter_collection.csv $O/w5/run_counter_collection.csv $O/f6/run_counter_collection.csv $O/f5/run_counter_collection.csv | awk -F, '{print $(NF-2), $(NF-1)}'
