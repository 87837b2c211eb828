#!/bin/bash
# DIAGNOSTIC: build libptmi.so from a git revision's sources into
# pathtracer-ocl_amd/build/exp/libptmi_<name>.so, for A/B runs with tools/exp_variants.sh.
#   bash tools/build_ref_variant.sh <rev> <name> [extra hipcc flags]
set -e
REV=$1; NAME=$2; shift 2
T=$(mktemp -d)
mkdir -p $T/pathtracer-ocl_amd/csrc $T/include
for f in $(git ls-tree --name-only $REV pathtracer-ocl_amd/csrc/); do git show $REV:$f > $T/$f; done
for f in $(git ls-tree --name-only $REV include/); do git show $REV:$f > $T/$f; done
mkdir -p pathtracer-ocl_amd/build/exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-result "$@" \
    -shared -o pathtracer-ocl_amd/build/exp/libptmi_$NAME.so \
    $T/pathtracer-ocl_amd/csrc/ptmi_kernels.hip $T/pathtracer-ocl_amd/csrc/ptmi_api.cpp $T/pathtracer-ocl_amd/csrc/ptmi_bvh.cpp
rm -rf $T
