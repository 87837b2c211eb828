#!/bin/bash
# Round 3: correctness of the pooled BVH walks, then A/B frame times (GPU box, repo root).
#   bash tools/r3_pool_check.sh <outdir> <spp> "<variants>"
set -e -o pipefail
OUT=${1:-gpurun_out/r3b}; SPP=${2:-512}; VARS=${3:-"head base w2"}
mkdir -p $OUT
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -k "golden" -x -q --timeout 120 --timeout-method thread > $OUT/golden.log 2>&1
tail -2 $OUT/golden.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres.py -m "gpu and not slow" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
bash tools/diag_ab.sh $OUT/ab $SPP "c4 c5" "$VARS"
