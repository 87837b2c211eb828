#!/bin/bash
# DIAGNOSTIC scratch: parity subset + A/B timings for the current change
set -e -o pipefail
O=gpurun_out/r3c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rng_mode.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
bash tools/diag_ab.sh $O 512 "c2" "head base w7 w5"
bash tools/diag_ab.sh $O 512 "c4 c5" "head base"
