#!/bin/bash
# DIAGNOSTIC scratch: parity + A/B for the partial-layout split
set -e -o pipefail
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres.py -x -q --timeout 600 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
bash tools/diag_ab.sh $O 512 "c4 c5" "p475 base"
bash tools/diag_ab.sh $O 2048 "c2" "head base"
