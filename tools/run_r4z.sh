#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4z
bash tools/diag_ab.sh gpurun_out/r4z 2048 "c4 c5 c3" "base noskew base noskew" > gpurun_out/r4z.log 2>&1 || { cat gpurun_out/r4z.log; exit 1; }
cat gpurun_out/r4z.log
