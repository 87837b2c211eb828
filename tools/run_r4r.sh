#!/bin/bash
# Round-4: whole-tile order support + mesh-only item timing (C2 kernel spill 16 -> 0 B) vs the previous commit.
set -o pipefail
mkdir -p gpurun_out/r4r
timeout -k 10 500 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_rng_mode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_r4r.log 2>&1 || { tail -8 gpurun_out/parity_r4r.log; exit 1; }
tail -1 gpurun_out/parity_r4r.log
bash tools/diag_ab.sh gpurun_out/r4r 2048 "c2 c3 c4" "base prev base prev" > gpurun_out/r4r.log 2>&1 || { cat gpurun_out/r4r.log; exit 1; }
cat gpurun_out/r4r.log
for v in base prev; do
  if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
  PTMI_LIB=$L timeout -k 10 300 python bench.py --config c2 --rng xoshiro --steps 2 --warmup 1 --no-cpu-baseline \
    --no-trace-call > gpurun_out/r4r/c2x_$v.json 2> gpurun_out/r4r/c2x_$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r4r/c2x_$v.json'));print('c2x $v', d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
