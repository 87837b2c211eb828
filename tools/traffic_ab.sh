#!/bin/bash
# DIAGNOSTIC: HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.py) of one
# full-frame launch per config and library variant.  usage:
#   bash tools/traffic_ab.sh <outdir> "<configs>" "<variants>"
# variant: base (the product build) or <name> (build/exp/libptmi_<name>.so, tools/build_variant.sh).
set -e -o pipefail
OUT=$1; CFGS=$2; VARS=$3
export TMPDIR=/tmp
mkdir -p $OUT
for c in $CFGS; do
  for v in $VARS; do
    if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
    A="--config $c --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
    PTMI_LIB=$L timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${c}_${v}_fetch -o run -- python3 bench.py $A > $OUT/${c}_${v}_fetch.log 2>&1
    PTMI_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${c}_${v}_write -o run -- python3 bench.py $A > $OUT/${c}_${v}_write.log 2>&1
    python3 tools/pmc_traffic.py $OUT/${c}_${v}_fetch $OUT/${c}_${v}_write $OUT/pmc_${c}_${v}.json > /dev/null
    python3 -c "import json;d=json.load(open('$OUT/pmc_${c}_${v}.json'));print('$c $v fetch(raw) %.4f GB write %.4f GB hbm %.4f GB' % (d['fetch_size_kb_raw_per_launch']*1024/1e9, d['write_size_kb_per_launch']*1024/1e9, d['hbm_bytes_per_launch']/1e9))"
  done
done
