#!/bin/bash
# DIAGNOSTIC (round 4): split-form knobs on C4/C5 frames, study library.
#   bash tools/split_sweep.sh <out> <spp> "<cfgs>" "<specs>"
#   spec: name:knob=VAL,knob=VAL (bench.py --knob names, e.g. split_slots=8,split_budget=4)
set -o pipefail
OUT=$1; SPP=$2; CFGS=$3; SPECS=$4
mkdir -p $OUT
for c in $CFGS; do
  for spec in $SPECS; do
    tag=${spec%%:*}; e=${spec#*:}; [ "$e" = "$spec" ] && e=""
    kn=""; for kv in ${e//,/ }; do kn="$kn --knob $kv"; done
    PTMI_LIB=pathtracer-ocl_amd/build/libptmi_study.so PTMI_SPLIT_DEBUG=1 timeout -k 10 300 python3 bench.py --split $kn --config $c --samples $SPP --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > $OUT/${c}_$tag.json 2> $OUT/${c}_$tag.err || { echo "$c $tag FAILED"; tail -3 $OUT/${c}_$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${c}_$tag.json'));print('$c $tag', d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
    grep "split:" $OUT/${c}_$tag.err | tail -1
  done
done
