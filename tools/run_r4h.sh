#!/bin/bash
set -o pipefail
OUT=gpurun_out/r4h; mkdir -p $OUT
for sp in 1 0; do
  PTMI_SPLIT=$sp PTMI_SPLIT_SLOTS=1 PTMI_SPLIT_DEBUG=1 timeout -k 10 300 python3 bench.py --config c4 --chunks 32 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none --save-image $OUT/c4_s$sp.npy > $OUT/c4_s$sp.json 2> $OUT/c4_s$sp.err || exit 1
  grep "split:" $OUT/c4_s$sp.err
done
python3 -c "
import numpy as np
a=np.load('$OUT/c4_s1.npy'); b=np.load('$OUT/c4_s0.npy')
print('C4 2048spp chunks 32: split vs one-kernel identical', np.array_equal(a.view(np.int64), b.view(np.int64)), 'max diff %.3e'%np.abs(a-b).max())
"
