#!/bin/bash
# DIAGNOSTIC scratch: parity subset + A/B timings for the current change
set -e -o pipefail
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rng.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
bash tools/diag_ab.sh $O 512 "c2 c3" "head base nopair"
bash tools/diag_ab.sh $O 512 "c4 c5" "head base"
