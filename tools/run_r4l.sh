#!/bin/bash
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4l.log 2>&1 || { tail -5 gpurun_out/parity_r4l.log; exit 1; }
tail -1 gpurun_out/parity_r4l.log
bash tools/run_r4k.sh
