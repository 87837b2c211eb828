#!/bin/bash
# WRITE_SIZE of the C4 launch: product vs the round-3 build vs no camera reload in the mesh kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wr2
A="--config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
for v in ${VARS:-base r3 cam1}; do
  if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
  PTMI_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wr2/$v -o run -- python3 bench.py $A > gpurun_out/wr2/$v.log 2>&1 || { tail -5 gpurun_out/wr2/$v.log; exit 1; }
  python3 - <<PY
import csv,glob
rows=list(csv.DictReader(open(glob.glob('gpurun_out/wr2/$v/**/run_counter_collection.csv', recursive=True)[0])))
v=[float(r['Counter_Value']) for r in rows if 'trace_kernel' in r['Kernel_Name']]
print('$v WRITE_SIZE KB per trace launch', v)
PY
done
