#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/wb
bash tools/diag_ab.sh gpurun_out/wb 2048 "c4 c5" "base wb20 wb28 base wb20 wb28" > gpurun_out/wb.log 2>&1 || { cat gpurun_out/wb.log; exit 1; }
cat gpurun_out/wb.log
