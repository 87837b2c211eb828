#!/bin/bash
# DIAGNOSTIC: rocprofv3 PC sampling of one bench.py workload (dynamic instruction hot spots).
#   bash tools/pcsamp.sh <outdir> <method: stochastic|host_trap> <interval> [bench args ...]
# stochastic: interval in shader cycles (power of two); host_trap: interval in microseconds.
# The samples are mapped to kernel phases by tools/pc_phases.py.
set -o pipefail
OUT=$1; METHOD=$2; IV=$3; shift 3
UNIT=cycles; [ "$METHOD" = host_trap ] && UNIT=time
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
  --pc-sampling-interval $IV --output-format csv -d $OUT -o run -- python3 bench.py "$@" --extra none \
  --no-cpu-baseline --no-trace-call > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "pcsamp $METHOD rc=$rc"
ls -la $OUT | head -20
exit $rc
