#!/bin/bash
set -o pipefail
for mc in 64 128; do
  PTMI_MIN_CHUNK=$mc timeout -k 10 300 python3 tools/shard_balance.py gpurun_out/shards_order_mc$mc.json --configs c4,c5 --worlds 2,8 \
    > gpurun_out/shards_order_mc$mc.log 2>&1 || { tail -5 gpurun_out/shards_order_mc$mc.log; exit 1; }
  echo "min_chunk $mc"; grep -v amdgpu gpurun_out/shards_order_mc$mc.log | grep -v "^{"
done
