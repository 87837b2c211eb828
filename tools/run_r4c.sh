set -o pipefail
B=pathtracer-ocl_amd/build
mkdir -p gpurun_out/r4c
for c in c4 c5; do
  PTMI_LIB=$B/exp/libptmi_nowalk_g4.so timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > gpurun_out/r4c/${c}_nowalk.json 2> gpurun_out/r4c/${c}_nowalk.err
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > gpurun_out/r4c/${c}_base.json 2> gpurun_out/r4c/${c}_base.err
  echo "$c done"
done
for m in 1 4; do
  PTMI_WALK_GRID_MULT=$m PTMI_LIB=$B/libptmi_capture.so timeout -k 10 240 python3 tools/walk_bench.py capture teapot 0 32 gpurun_out/r4c/teapot_grid$m.json > gpurun_out/r4c/teapot_grid$m.log 2>&1
done
