#!/bin/bash
# Memory-instruction counts of the C4 launch across builds (one SQ --pmc pass each).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
A="--config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
for v in ${VARS:-r3 b349779 base}; do
  if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
  PTMI_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_SALU --output-format csv -d gpurun_out/sq/$v -o run -- python3 bench.py $A > gpurun_out/sq/$v.log 2>&1 || { tail -5 gpurun_out/sq/$v.log; exit 1; }
  python3 - <<PY
import csv,glob,collections
rows=list(csv.DictReader(open(glob.glob('gpurun_out/sq/$v/**/run_counter_collection.csv', recursive=True)[0])))
d=collections.defaultdict(float)
for r in rows:
    if 'trace_kernel' in r['Kernel_Name']: d[r['Counter_Name']]+=float(r['Counter_Value'])
print('$v', {k: '%.4g'%v for k,v in sorted(d.items())})
PY
done
