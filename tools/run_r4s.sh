#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r4s
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4s.log 2>&1 || { tail -8 gpurun_out/parity_r4s.log; exit 1; }
tail -1 gpurun_out/parity_r4s.log
bash tools/diag_ab.sh gpurun_out/r4s 2048 "c2 c4 c5" "base prev base prev" > gpurun_out/r4s.log 2>&1 || { cat gpurun_out/r4s.log; exit 1; }
cat gpurun_out/r4s.log
