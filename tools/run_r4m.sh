#!/bin/bash
# Round-4: mesh tiles dispatched costliest first (PTMI_TILE_ORDER) -- parity, A/B, timelines.
set -o pipefail
mkdir -p gpurun_out/order gpurun_out/tl
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4m.log 2>&1 || { tail -5 gpurun_out/parity_r4m.log; exit 1; }
tail -1 gpurun_out/parity_r4m.log
bash tools/diag_ab.sh gpurun_out/order 2048 "c4 c5" "base base:PTMI_TILE_ORDER=0" > gpurun_out/order.log 2>&1 || { cat gpurun_out/order.log; exit 1; }
cat gpurun_out/order.log
L=pathtracer-ocl_amd/build/libptmi_timeline.so
run() { PTMI_LIB=$L timeout -k 10 120 python3 tools/timeline.py "$@" 2>&1 | grep -v amdgpu | tail -1; }
run c4 gpurun_out/tl/c4_order.json || exit 1
run c5 gpurun_out/tl/c5_order.json || exit 1
run c4 gpurun_out/tl/c4_share8_order.json --range 0,256 || exit 1
run c5 gpurun_out/tl/c5_share8_order.json --stride 8 --offset 0 || exit 1
run c2 gpurun_out/tl/c2_curve.json || exit 1
