#!/bin/bash
# DIAGNOSTIC: read-counter calibration (tools/fetch_calib.hip) and the same counters on the mesh
# frames.  usage: bash tools/fetch_calib.sh <outdir> [configs]
# Needs tools/bin/fetch_calib (built here: see fetch_calib.hip).  Every pass is its own
# rocprofv3 run with at most 4 TCC counters (FETCH_SIZE takes 3).
set -e -o pipefail
OUT=$1; CFGS=${2:-c4 c5}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
# the request-size counters this ROCm knows for gfx950 (at most 4 TCC counters per pass)
C=""
for n in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_BUBBLE TCC_EA0_RDREQ_64B; do
  if grep -qw "$n" $OUT/avail.txt; then C="$C ${n}_sum"; fi
done
echo "request counters:$C"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o run -- tools/bin/fetch_calib > $OUT/calib.log 2>&1
echo "calib fetch done"
if [ -n "$C" ]; then
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/calib_req -o run -- tools/bin/fetch_calib >> $OUT/calib.log 2>&1
  echo "calib req done"
  for c in $CFGS; do
    timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $OUT/${c}_req -o run -- \
      python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/${c}_req.log 2>&1
    echo "$c req done"
  done
fi
python3 tools/fetch_calib_report.py $OUT
