# DIAGNOSTIC: build an experimental libptmi.so from the working tree with extra
# defines.  usage: bash tools/build_variant.sh <name> [-DNAME=VAL ...]
#   -> pathtracer-ocl_amd/build/exp/libptmi_<name>.so   (tools/exp_variants.sh times it)
# <name> = head: the HEAD commit's sources instead of the working tree.
set -e
NAME=$1; shift
cd "$(dirname "$0")/../pathtracer-ocl_amd"
mkdir -p build/exp
SRC=csrc
REV=${REV:-HEAD}
if [ "$NAME" = head ] || [ -n "$FROMREV" ]; then
  SRC=$(mktemp -d)/csrc; mkdir -p $SRC
  for f in ptmi_kernels.hip ptmi_api.cpp ptmi_bvh.cpp ptmi_bvh.h ptmi_device.h ptmi_sinf.h ptmi_fp64core.h ptmi_f16.h; do
    git show $REV:pathtracer-ocl_amd/csrc/$f > $SRC/$f
  done
  mkdir -p $(dirname $SRC)/../include
  for f in ptmi.h ptmi_diag.h ptmi_host.h; do
    git show $REV:include/$f > $(dirname $SRC)/../include/$f 2>/dev/null || true
  done
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-result \
  "$@" -shared -o build/exp/libptmi_$NAME.so $SRC/ptmi_kernels.hip $SRC/ptmi_api.cpp $SRC/ptmi_bvh.cpp
