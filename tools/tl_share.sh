set -e -o pipefail
OUT=gpurun_out/tl2; mkdir -p $OUT
export TMPDIR=/tmp
L=pathtracer-ocl_amd/build/libptmi_timeline.so
PTMI_LIB=$L timeout -k 10 200 python3 tools/timeline.py c5 $OUT/c5s8.json --stride 8 --offset 3 > $OUT/c5s8.log 2>&1; tail -12 $OUT/c5s8.log
for k in mesh_items=16 mesh_items=24 mesh_items=48 mesh_items=64 min_chunk=32 min_chunk=128; do
  timeout -k 10 200 python3 tools/shard_balance.py $OUT/sh_$k.json --configs c5 --worlds 8 --knob $k > $OUT/sh_$k.log 2>&1
  grep -E "^c5 " $OUT/sh_$k.log | sed "s/^/$k /"
done
bash tools/diag_ab.sh $OUT/ab 2048 "c4 c5" "base wb28 wb20 base wb28 wb20"
