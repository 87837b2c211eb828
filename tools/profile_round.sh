#!/bin/bash
# Round evidence on the GPU box (run from the repo root):
#   bash tools/profile_round.sh <outdir>
# 1. rocprofv3 --kernel-trace --stats of the default bench command (C2) -> kernel stats + the bench line
# 2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no tracing domains), 1 frame of C2
# 3. kernel-trace stats of C4 / C5 (256 spp frames: same kernel, 1/8 of the samples)
# 4. FETCH_SIZE / WRITE_SIZE of one C4 256-spp frame (BVH scene traffic)
set -e -o pipefail
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run -- \
    python3 bench.py --config c2 --steps 2 --warmup 1 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o run -- \
    python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call > $OUT/c2_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o run -- \
    python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call > $OUT/c2_write.log 2>&1
python3 tools/pmc_traffic.py $OUT/c2_fetch $OUT/c2_write $OUT/pmc_c2.json
for c in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c -o run -- \
      python3 bench.py --config $c --samples 256 --steps 1 --warmup 1 --no-cpu-baseline --no-trace-call > $OUT/bench_$c.json 2> $OUT/bench_$c.err
done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4_fetch -o run -- \
    python3 bench.py --config c4 --samples 256 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call > $OUT/c4_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c4_write -o run -- \
    python3 bench.py --config c4 --samples 256 --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call > $OUT/c4_write.log 2>&1
python3 tools/pmc_traffic.py $OUT/c4_fetch $OUT/c4_write $OUT/pmc_c4.json
find $OUT -name "*kernel_stats.csv" | sort
