#!/bin/bash
# DIAGNOSTIC scratch: traversal counters + group-kernel knobs at 4 waves/SIMD
set -e -o pipefail
O=gpurun_out/r3q; mkdir -p $O
PTMI_LIB=pathtracer-ocl_amd/build/libptmi_stats.so timeout -k 10 200 python tools/bvh_stats.py teapot 16 > $O/teapot_stats.txt 2>&1
PTMI_LIB=pathtracer-ocl_amd/build/libptmi_stats.so timeout -k 10 200 python tools/bvh_stats.py gopher 16 > $O/gopher_stats.txt 2>&1
grep -h "walks \|node4\|walks_no_leaf\|walks_root_only\|lanes per walk\|tri_tests" $O/teapot_stats.txt $O/gopher_stats.txt
bash tools/diag_ab.sh $O 512 "c4 c5" "base rpt wb20 wb28 base:PTMI_MESH_ITEMS=16 base:PTMI_MESH_ITEMS=64 base"
