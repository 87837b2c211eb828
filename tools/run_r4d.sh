#!/bin/bash
# round 4: split-form checks and timings (one GPU call)
set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > $OUT/split_test.log 2>&1 || { echo "split test failed"; tail -30 $OUT/split_test.log; exit 1; }
echo "split tests ok"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
echo "parity ok"
for c in c4 c5; do
  for sp in 1 0; do
    PTMI_SPLIT=$sp timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > $OUT/${c}_split$sp.json 2> $OUT/${c}_split$sp.err || { echo "bench $c $sp failed"; tail $OUT/${c}_split$sp.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${c}_split$sp.json'));print('$c split=$sp', d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
