# DIAGNOSTIC: time experimental builds of libptmi.so (pathtracer-ocl_amd/build/exp/libptmi_<v>.so)
# against the product build.  usage: bash tools/exp_variants.sh "<variants>" "<configs>" [samples]
set -e
mkdir -p gpurun_out
VARS=${1:-base}
CFGS=${2:-c4}
SPP=${3:-256}
for c in $CFGS; do
  for v in $VARS; do
    if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
    PTMI_LIB=$L timeout -k 10 300 python bench.py --config $c --samples $SPP --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call \
      > gpurun_out/exp_${c}_$v.json 2> gpurun_out/exp_${c}_$v.err
    python3 -c "import json;d=json.load(open('gpurun_out/exp_${c}_$v.json'));print('$c $v', d['ms_per_step'], d['roofline']['frac'])"
  done
done
