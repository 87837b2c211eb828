#!/bin/bash
# DIAGNOSTIC scratch: A/B timings for the current change
set -e -o pipefail
O=gpurun_out/r3e; mkdir -p $O
bash tools/diag_ab.sh $O 512 "c2 c3" "base w7"
bash tools/diag_ab.sh $O 512 "c4 c5" "base gnotab"
bash tools/diag_ab.sh $O 512 "c5" "base gnotab"
