#!/bin/bash
# DIAGNOSTIC: where trace_kernel's wave cycles go (round 4).  Three
# --pmc passes of SQ counters only (no tracing domains), then tools/pmc_stall.py.
#   bash tools/pmc_stall.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/stall}; shift || true
ARGS=${@:---config c2 --steps 1 --warmup 0 --samples 256 --no-cpu-baseline --no-trace-call --extra none}
export TMPDIR=/tmp
mkdir -p $OUT
S1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAVES"
S3="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$S1" "$S2" "$S3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
done
python3 tools/pmc_stall.py $OUT > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt
