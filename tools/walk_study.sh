#!/bin/bash
# DIAGNOSTIC (round 4): the standalone-walk measurement of VERDICT r3 item 1 on one box.
#   bash tools/walk_study.sh <outdir> [s1]
set -e -o pipefail
OUT=${1:-gpurun_out/walk}; S1=${2:-32}
B=pathtracer-ocl_amd/build
NOWALK=${NOWALK:-}
mkdir -p $OUT
for sc in teapot gopher; do
  for v in libptmi_capture exp/libptmi_capture_w4 exp/libptmi_capture_w6; do
    tag=$(basename $v .so)
    PTMI_LIB=$B/$v.so timeout -k 10 240 python3 tools/walk_bench.py capture $sc 0 $S1 $OUT/${sc}_$tag.json > $OUT/${sc}_$tag.log 2>&1
    echo "$sc $tag done"
  done
  PTMI_LIB=$B/libptmi.so timeout -k 10 240 python3 tools/walk_bench.py frame $sc 0 $S1 $OUT/${sc}_frame.json > $OUT/${sc}_frame.log 2>&1
  PTMI_LIB=$B/libptmi_timers.so timeout -k 10 240 python3 tools/walk_bench.py frame $sc 0 $S1 $OUT/${sc}_timers.json > $OUT/${sc}_timers.log 2>&1
  for v in $NOWALK; do  # DIAGNOSTIC ablation: the mesh kernel without walks (tracer-only estimate)
    PTMI_LIB=$B/exp/libptmi_$v.so timeout -k 10 240 python3 tools/walk_bench.py frame $sc 0 $S1 $OUT/${sc}_$v.json > $OUT/${sc}_$v.log 2>&1
  done
  echo "$sc frame done"
done
