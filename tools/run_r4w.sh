#!/bin/bash
# Static tile order with the mesh kernel's scalar loads restored vs the measured order (cost build).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4w
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4w.log 2>&1 || { tail -8 gpurun_out/parity_r4w.log; exit 1; }
tail -1 gpurun_out/parity_r4w.log
bash tools/diag_ab.sh gpurun_out/r4w 2048 "c4 c5" "base cost:PTMI_TILE_ORDER=2 base cost:PTMI_TILE_ORDER=2" > gpurun_out/r4w.log 2>&1 || { cat gpurun_out/r4w.log; exit 1; }
cat gpurun_out/r4w.log
VARS="base" bash tools/run_r4u.sh
