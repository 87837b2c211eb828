#!/bin/bash
# Round-4: work-item timelines (ramp / drain) of full frames and of N=8 rank shares.
set -o pipefail
mkdir -p gpurun_out/tl
L=pathtracer-ocl_amd/build/libptmi_timeline.so
run() { PTMI_LIB=$L timeout -k 10 120 python3 tools/timeline.py "$@" 2>&1 | grep -v amdgpu | tail -1; }
run c2 gpurun_out/tl/c2.json || exit 1
run c4 gpurun_out/tl/c4.json || exit 1
run c5 gpurun_out/tl/c5.json || exit 1
run c4 gpurun_out/tl/c4_share8.json --range 0,256 || exit 1
run c5 gpurun_out/tl/c5_share8.json --stride 8 --offset 0 || exit 1
run c2 gpurun_out/tl/c2_share8.json --range 0,256 || exit 1
