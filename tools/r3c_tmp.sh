set -o pipefail
OUT=gpurun_out/r3h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/pcs -o run --output-format csv -- python3 bench.py --config c2 --samples 128 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/pcs.log 2>&1
echo "pcs rc=$?"
ls -R $OUT/pcs | head -20
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -5 $OUT/gpu_tests.log
