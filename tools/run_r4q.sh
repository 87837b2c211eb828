#!/bin/bash
# Round-4: measured-cost tile order (PTMI_TILE_ORDER=2) -- invariance, parity, A/B, timelines.
set -o pipefail
mkdir -p gpurun_out/order2 gpurun_out/tl
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4q.log 2>&1 || { tail -8 gpurun_out/parity_r4q.log; exit 1; }
tail -1 gpurun_out/parity_r4q.log
bash tools/diag_ab.sh gpurun_out/order2 2048 "c4 c5" "base base:PTMI_TILE_ORDER=1 base:PTMI_TILE_ORDER=0" > gpurun_out/order2.log 2>&1 || { cat gpurun_out/order2.log; exit 1; }
cat gpurun_out/order2.log
L=pathtracer-ocl_amd/build/libptmi_timeline.so
run() { PTMI_LIB=$L timeout -k 10 120 python3 tools/timeline.py "$@" 2>&1 | grep -v amdgpu | tail -1; }
run c4 gpurun_out/tl/c4_order2.json || exit 1
run c5 gpurun_out/tl/c5_order2.json || exit 1
