#!/bin/bash
# Round-4 A/B: accumColor in LDS for the mesh kernels (acm, acm21), camera reload, mesh items.
set -o pipefail
mkdir -p gpurun_out
PTMI_LIB=pathtracer-ocl_amd/build/exp/libptmi_acm21.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/parity_acm21.log 2>&1 || { tail -5 gpurun_out/parity_acm21.log; exit 1; }
tail -2 gpurun_out/parity_acm21.log
bash tools/diag_ab.sh gpurun_out/cam 512 "c4 c5" "base acm acm21 cam3 base:PTMI_MESH_ITEMS=44" > gpurun_out/cam.log 2>&1 || { cat gpurun_out/cam.log; exit 1; }
bash tools/diag_ab.sh gpurun_out/cam 2048 "c2 c3" "base cam0" >> gpurun_out/cam.log 2>&1 || { cat gpurun_out/cam.log; exit 1; }
cat gpurun_out/cam.log
timeout -k 10 400 python3 tools/shard_balance.py gpurun_out/shards.json > gpurun_out/shards.log 2>&1 || { tail -5 gpurun_out/shards.log; exit 1; }
grep -v amdgpu gpurun_out/shards.log | grep -v "^{" | tail -14
PTMI_LIB=pathtracer-ocl_amd/build/libptmi.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rng_mode.py -x -q \
  --timeout 200 --timeout-method thread -s > gpurun_out/rng_mode.log 2>&1 || { tail -5 gpurun_out/rng_mode.log; exit 1; }
grep -E "ratio|passed|failed" gpurun_out/rng_mode.log
for v in base xs64; do
  if [ $v = base ]; then L=pathtracer-ocl_amd/build/libptmi.so; else L=pathtracer-ocl_amd/build/exp/libptmi_$v.so; fi
  PTMI_LIB=$L timeout -k 10 300 python bench.py --config c2 --rng xoshiro --steps 2 --warmup 1 --no-cpu-baseline \
    --no-trace-call > gpurun_out/cam/c2x_$v.json 2> gpurun_out/cam/c2x_$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/cam/c2x_$v.json'));print('c2x $v', d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
