#!/bin/bash
# Collect rocprofv3 PMC counters for trace_kernel (separate passes; no tracing
# domains combined with --pmc).  Run on the GPU box from the repo root:
#   bash tools/pmc.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 1 --warmup 0 --samples 64 --no-cpu-baseline --extra none}
export TMPDIR=/tmp
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32"
P3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || echo "pass $i failed ($P)" >> $OUT/failed.txt
done
python3 tools/pmc_summary.py $OUT --valu-json $OUT/valu.json > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt
