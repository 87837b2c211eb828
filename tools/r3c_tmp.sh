#!/bin/bash
# DIAGNOSTIC scratch: statistical-mode tests + timing, then the L2/VALU passes
set -e -o pipefail
O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rng_mode.py -x -q --timeout 300 --timeout-method thread > $O/rng.log 2>&1
tail -2 $O/rng.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > $O/c2.json 2> $O/c2.err
python3 -c "import json;d=json.load(open('$O/c2.json'));print('c2', d['ms_per_step'], 'stat', d.get('statistical_rng',{}).get('ms_per_step'))"
STAGES="l2 valu" bash tools/profile_round3.sh gpurun_out/prof3
