set -e -o pipefail
OUT=gpurun_out/r3f; mkdir -p $OUT
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -k "golden or adversarial or live_reference" -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_rng_mode.py tests/test_gpu_go_abi.py -x -q --timeout 200 --timeout-method thread > $OUT/tests2.log 2>&1 || true
tail -15 $OUT/tests2.log
bash tools/diag_ab.sh $OUT/ab 512 "c2 c4 c5" "head base"
