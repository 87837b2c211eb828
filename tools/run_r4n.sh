#!/bin/bash
set -o pipefail
timeout -k 10 400 python3 tools/shard_balance.py gpurun_out/shards_c45_order.json --configs c4,c5 > gpurun_out/shards_c45_order.log 2>&1 || { tail -5 gpurun_out/shards_c45_order.log; exit 1; }
grep -v amdgpu gpurun_out/shards_c45_order.log | grep -v "^{"
mkdir -p gpurun_out/order512
bash tools/diag_ab.sh gpurun_out/order512 512 "c4 c5" "base base:PTMI_TILE_ORDER=0" > gpurun_out/order512.log 2>&1 || { cat gpurun_out/order512.log; exit 1; }
cat gpurun_out/order512.log
