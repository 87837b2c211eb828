#!/bin/bash
# DIAGNOSTIC scratch: parity subset + A/B timings for the current change
set -e -o pipefail
O=gpurun_out/r3f; mkdir -p $O


bash tools/diag_ab.sh $O 512 "c4 c5" "base lf4 lf2"
