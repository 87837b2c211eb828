#!/bin/bash
# Round evidence on the GPU box (run from the repo root):  bash tools/profile_round2.sh <outdir>
# 1. rocprofv3 --kernel-trace --stats of the default bench command (C2, as the driver runs it)
# 2. kernel-trace stats of full 2048-spp frames of C3, C4, C5 (one timed frame each)
# 3. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no tracing domains): one C2 and one C4 frame
# 4. VALU counter passes (tools/pmc.sh) for one C2 and one C4 frame
set -e -o pipefail
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run -- \
    python3 bench.py --steps 3 --warmup 1 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
for c in c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c -o run -- \
      python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-trace-call --extra none > $OUT/bench_$c.json 2> $OUT/bench_$c.err
done
for c in c2 c4; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${c}_fetch -o run -- \
      python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/${c}_fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${c}_write -o run -- \
      python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none > $OUT/${c}_write.log 2>&1
  python3 tools/pmc_traffic.py $OUT/${c}_fetch $OUT/${c}_write $OUT/pmc_$c.json
done
timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_valu_c2 --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none
timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_valu_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none
timeout -k 10 600 bash tools/pmc.sh $OUT/pmc_valu_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none
find $OUT -name "*kernel_stats.csv" | sort
