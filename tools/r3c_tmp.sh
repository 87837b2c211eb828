#!/bin/bash
# DIAGNOSTIC scratch: material variants at 5 waves (product) vs 6; parity
set -e -o pipefail
O=gpurun_out/r3s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
for sc in transparency reflection default; do
  for v in base m6 base; do
    L=pathtracer-ocl_amd/build/libptmi.so; [ $v != base ] && L=pathtracer-ocl_amd/build/exp/libptmi_$v.so
    echo -n "$v: "; PTMI_LIB=$L timeout -k 10 120 python tools/scene_time.py $sc 256 2>&1 | grep spp
  done
done
