#!/bin/bash
# The sample index in LDS in the mesh kernels (PTMI_NCUR_LDS=1) against the product.
set -o pipefail
mkdir -p gpurun_out/r4x
PTMI_LIB=pathtracer-ocl_amd/build/exp/libptmi_ncur.so timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4x.log 2>&1 || { tail -8 gpurun_out/parity_r4x.log; exit 1; }
tail -1 gpurun_out/parity_r4x.log
bash tools/diag_ab.sh gpurun_out/r4x 2048 "c4 c5" "base ncur base ncur" > gpurun_out/r4x.log 2>&1 || { cat gpurun_out/r4x.log; exit 1; }
cat gpurun_out/r4x.log
