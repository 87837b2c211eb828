#!/bin/bash
# DIAGNOSTIC (round 6): C5 HBM traffic and frame time for the hemisphere table in the mesh kernels
# (base) against none (build/exp/libptmi_notab.so) and against fewer chunk items (mesh_items=24).
set -e -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
A="--config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
run() {  # name lib extra-args
  PTMI_LIB=$2 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$1_fetch -o run -- python3 bench.py $A $3 > $OUT/$1_fetch.log 2>&1
  PTMI_LIB=$2 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$1_write -o run -- python3 bench.py $A $3 > $OUT/$1_write.log 2>&1
  python3 tools/pmc_traffic.py $OUT/$1_fetch $OUT/$1_write $OUT/pmc_$1.json
  python3 -c "import json;d=json.load(open('$OUT/pmc_$1.json'));print('$1', 'HBM GB', round(d['hbm_bytes_per_launch']/1e9,3), 'write GB', round(d['write_size_kb_per_launch']*1024/1e9,3))"
}
run base pathtracer-ocl_amd/build/libptmi.so ""
run notab pathtracer-ocl_amd/build/exp/libptmi_notab.so ""
run mi24 pathtracer-ocl_amd/build/libptmi.so "--knob mesh_items=24"
bash tools/diag_ab.sh $OUT/ab 2048 "c5" "base notab base@mesh_items=24 base notab base@mesh_items=24"
