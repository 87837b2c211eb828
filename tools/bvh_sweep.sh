# DIAGNOSTIC: frame time vs the traversal index's SAH triangle cost and leaf size
# (PTMI_BVH_CTRI / PTMI_BVH_LEAF, read by the study library's ptmi_bvh.cpp at scene upload).
#   bash tools/bvh_sweep.sh "<configs>" "<ctri values>" "<leaf sizes>" [spp]
set -e
for c in $1; do
  for ct in $2; do
    for lf in $3; do
      PTMI_LIB=pathtracer-ocl_amd/build/libptmi_study.so PTMI_BVH_CTRI=$ct PTMI_BVH_LEAF=$lf timeout -k 10 200 python bench.py --config $c --samples ${4:-256} --steps 2 \
          --warmup 1 --no-cpu-baseline --no-trace-call > gpurun_out/bv_${c}_${ct}_${lf}.json 2>/dev/null
      python3 -c "import json;d=json.load(open('gpurun_out/bv_${c}_${ct}_${lf}.json'));print('$c ctri=$ct leaf=$lf', d['ms_per_step'])"
    done
  done
done
