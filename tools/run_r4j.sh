#!/bin/bash
# Round-4: camera reload through scalar loads (cc1 / cc3) and the chunk-length floor for rank shares.
set -o pipefail
mkdir -p gpurun_out/cam2
bash tools/diag_ab.sh gpurun_out/cam2 2048 "c2 c3" "base cc1" > gpurun_out/cam2.log 2>&1 || { cat gpurun_out/cam2.log; exit 1; }
bash tools/diag_ab.sh gpurun_out/cam2 512 "c4" "base cc3" >> gpurun_out/cam2.log 2>&1 || { cat gpurun_out/cam2.log; exit 1; }
cat gpurun_out/cam2.log
timeout -k 10 300 python3 tools/shard_balance.py gpurun_out/shards_c23.json --configs c2,c3 > gpurun_out/shards_c23.log 2>&1 || { tail -5 gpurun_out/shards_c23.log; exit 1; }
grep -v amdgpu gpurun_out/shards_c23.log | grep -v "^{"
for mc in 64 128 256; do
  PTMI_MIN_CHUNK=$mc timeout -k 10 300 python3 tools/shard_balance.py gpurun_out/shards_mc$mc.json --configs c4,c5 --worlds 8 \
    > gpurun_out/shards_mc$mc.log 2>&1 || { tail -5 gpurun_out/shards_mc$mc.log; exit 1; }
  echo "min_chunk $mc"; grep -v amdgpu gpurun_out/shards_mc$mc.log | grep -v "^{"
  python3 -c "import json;d=json.load(open('gpurun_out/shards_mc$mc.json'));print({c:e['t1_ms'] for c,e in d['configs'].items()})"
done
