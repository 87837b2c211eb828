set -e -o pipefail
OUT=gpurun_out/r3e; mkdir -p $OUT
timeout -k 10 150 env PTMI_LIB=pathtracer-ocl_amd/build/exp/libptmi_w2.so python -u -m pytest tests/test_gpu_parity.py -k "golden or adversarial or live_reference" -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
bash tools/diag_ab.sh $OUT/ab 512 "c4 c5" "head r32 r16 w2 t2w2 t4w2"
