#!/bin/bash
# Diagonal tile-split ownership: tile-split parity and shard tests, then the C5 8-rank balance with and without it.
set -o pipefail
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py tests/test_gpu_split.py tests/test_gpu_fullres.py -x -q --timeout 700 --timeout-method thread -k "tile or shard or split or order or multi" > gpurun_out/parity_r4y.log 2>&1 || { tail -8 gpurun_out/parity_r4y.log; exit 1; }
tail -1 gpurun_out/parity_r4y.log
timeout -k 10 300 python3 tools/shard_balance.py gpurun_out/shards_skew.json --configs c5 --worlds 2,4,8 > gpurun_out/shards_skew.log 2>&1 || { tail -5 gpurun_out/shards_skew.log; exit 1; }
echo skew; grep -v amdgpu gpurun_out/shards_skew.log | grep -v "^{"
PTMI_TILE_SKEW=0 timeout -k 10 300 python3 tools/shard_balance.py gpurun_out/shards_noskew.json --configs c5 --worlds 8 > gpurun_out/shards_noskew.log 2>&1 || { tail -5 gpurun_out/shards_noskew.log; exit 1; }
echo noskew; grep -v amdgpu gpurun_out/shards_noskew.log | grep -v "^{"
