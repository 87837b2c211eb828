#!/bin/bash
# DIAGNOSTIC (round 6): work-item timelines of the final build's C5 frame and one 8-rank C5 tile share.
set -e -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
L=pathtracer-ocl_amd/build/libptmi_timeline.so
PTMI_LIB=$L timeout -k 10 200 python3 tools/timeline.py c5 $OUT/c5.json > $OUT/c5.log 2>&1; tail -1 $OUT/c5.log | cut -c1-400
PTMI_LIB=$L timeout -k 10 200 python3 tools/timeline.py c5 $OUT/c5s8.json --stride 8 --offset 3 > $OUT/c5s8.log 2>&1; tail -1 $OUT/c5s8.log | cut -c1-400
