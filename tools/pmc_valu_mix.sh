#!/bin/bash
# DIAGNOSTIC: VALU instruction mix of trace_kernel (integer / conversion / total), one --pmc pass.
#   bash tools/pmc_valu_mix.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc_mix}; shift || true
ARGS=${@:---config c2 --steps 1 --warmup 0 --samples 256 --no-cpu-baseline --no-trace-call}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
    --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt
