#!/bin/bash
# WRITE_SIZE of the C4 launch under each tile order (one --pmc pass each, no tracing domains).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wr
A="--config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
for o in 0 1 2; do
  PTMI_TILE_ORDER=$o timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wr/o$o -o run -- python3 bench.py $A > gpurun_out/wr/o$o.log 2>&1 || { tail -5 gpurun_out/wr/o$o.log; exit 1; }
  python3 - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('gpurun_out/wr/o$o/**/run_counter_collection.csv', recursive=True)[0])))
v=[float(r['Counter_Value']) for r in rows if 'trace_kernel' in r['Kernel_Name']]
print('order $o WRITE_SIZE KB per trace launch', v)
PY
done
