#!/bin/bash
# DIAGNOSTIC: A/B one-frame timings on one box.  usage:
#   bash tools/diag_ab.sh <outdir> <spp> "<configs>" "<variant specs>"
# variant spec: name[@knob=val[@knob=val]][:ENV=VAL] -- the library build/exp/libptmi_<name>.so (base =
# the product build), bench.py --knob for each @knob=val, and an env setting for that run.
set -e -o pipefail
OUT=$1; SPP=$2; CFGS=$3; VARS=$4
mkdir -p $OUT
for c in $CFGS; do
  for spec in $VARS; do
    v=${spec%%:*}; e=""; [ "$spec" != "$v" ] && e=${spec#*:}
    k=""; IFS=@ read -r -a parts <<< "$v"; v=${parts[0]}
    for kv in "${parts[@]:1}"; do k="$k --knob $kv"; done
    if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
    tag=${spec//[:=@]/_}
    env $e PTMI_LIB=$L timeout -k 10 300 python bench.py --config $c --samples $SPP --steps 2 --warmup 1 \
      --no-cpu-baseline --no-trace-call $k > $OUT/${c}_$tag.json 2> $OUT/${c}_$tag.err
    python3 -c "import json;d=json.load(open('$OUT/${c}_$tag.json'));print('$c $tag', d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
