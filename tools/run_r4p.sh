#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/items
bash tools/diag_ab.sh gpurun_out/items 2048 "c4 c5" "base base:PTMI_MESH_ITEMS=16 base:PTMI_MESH_ITEMS=24 base:PTMI_MESH_ITEMS=48" > gpurun_out/items.log 2>&1 || { cat gpurun_out/items.log; exit 1; }
cat gpurun_out/items.log
