#!/bin/bash
# DIAGNOSTIC: the tile-split path pool (round 6) against the same build without it (build/exp/libptmi_nopool.so):
# rank-share timings of C5 (tile split) and C4 (tile split forced) at N = 4, 8 on one GPU.
set -e -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for v in base nopool; do
  L=pathtracer-ocl_amd/build/libptmi.so; [ $v = nopool ] && L=pathtracer-ocl_amd/build/exp/libptmi_nopool.so
  PTMI_LIB=$L timeout -k 10 300 python3 tools/shard_balance.py $OUT/shards_c5_$v.json --configs c5 --worlds 4,8 > $OUT/shards_c5_$v.log 2>&1
  grep -E "^c[0-9] " $OUT/shards_c5_$v.log | sed "s/^/$v /"
  PTMI_LIB=$L timeout -k 10 300 python3 tools/shard_balance.py $OUT/shards_c4t_$v.json --configs c4 --worlds 8 --split tile > $OUT/shards_c4t_$v.log 2>&1
  grep -E "^c[0-9] " $OUT/shards_c4t_$v.log | sed "s/^/$v tile /"
done
# one-GPU frames with the pool in every affine mesh kernel (build/exp/libptmi_poolall.so, PTMI_POOL=2)
bash tools/diag_ab.sh $OUT/ab 2048 "c4 c5" "base poolall base poolall"
