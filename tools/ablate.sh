#!/bin/bash
# DIAGNOSTIC: time the product lib and each ablation lib on the bench workload.
OUT=${1:-gpurun_out/ablate}; mkdir -p $OUT
for a in base 1 2 4 8 16; do
  if [ $a = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/libptmi_ablate_$a.so; fi
  PTMI_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu-baseline --extra none --steps 2 --warmup 1 > $OUT/$a.json 2>$OUT/$a.err || echo "ablate $a failed"
  python3 -c "import json,sys; d=json.load(open('$OUT/$a.json')); print('$a', d['value'], d['roofline']['kernel_ms_avg'])"
done
