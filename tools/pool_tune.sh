#!/bin/bash
# DIAGNOSTIC (round 6): the pooled kernels' tail floor and walk batch; the wide-code scene with and without the pool.
set -e -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/shard_balance.py $OUT/sh_new.json --configs c4,c5 --worlds 4,8 > $OUT/sh_new.log 2>&1
grep -E "^c[0-9] " $OUT/sh_new.log | sed "s/^/tailmin=auto /"
timeout -k 10 300 python3 tools/shard_balance.py $OUT/sh_old.json --configs c4,c5 --worlds 4,8 --knob tail_min=32 > $OUT/sh_old.log 2>&1
grep -E "^c[0-9] " $OUT/sh_old.log | sed "s/^/tailmin=32 /"
bash tools/diag_ab.sh $OUT/ab 2048 "c4 c5" "base wb28 wb32 base wb28 wb32"
timeout -k 10 200 python3 tools/wide_time.py 1280 960 64 > $OUT/wide_pool.txt 2>&1; tail -3 $OUT/wide_pool.txt
PTMI_LIB=pathtracer-ocl_amd/build/exp/libptmi_nopool.so timeout -k 10 200 python3 tools/wide_time.py 1280 960 64 > $OUT/wide_nopool.txt 2>&1; tail -3 $OUT/wide_nopool.txt
# the pool in the C2 kernel (PTMI_POOL_FLAT, non-DoF scenes without meshes) at 7 and 8 waves/SIMD
bash tools/diag_ab.sh $OUT/ab2 2048 "c2" "base pf7 pf8 base pf7 pf8"
