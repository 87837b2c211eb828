#!/bin/bash
# DIAGNOSTIC: VGPRs / scratch / occupancy of each trace_kernel<FL> instantiation.
#   bash tools/resources.sh [extra hipcc flags]
cd "$(dirname "$0")/../pathtracer-ocl_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-result "$@" \
  -c csrc/ptmi_kernels.hip -o /tmp/ptmi_res.o -Rpass-analysis=kernel-resource-usage 2>&1 | \
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' | awk '/Function Name:/{n=$NF} /VGPRs:/{v=$NF} /ScratchSize/{s=$NF} /Occupancy/{if (n ~ /trace_kernel/) {sub(/.*ILi/,"",n); sub(/EE.*/,"",n); printf "FL=%-3s VGPR %-4s scratch %-4s waves %s\n", n, v, s, $NF}}'
