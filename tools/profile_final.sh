#!/bin/bash
# A round's final evidence on the GPU box (repo root):  bash tools/profile_final.sh <outdir>
# 1. rocprofv3 --kernel-trace --stats of the driver's default bench command (C2 headline,
#    then the C3/C4/C5 extras and the statistical-RNG C2 frames in the same process)
# 2. kernel-trace stats of one full 2048-spp frame of each of C2..C5 on its own
# 3. FETCH_SIZE / WRITE_SIZE (separate --pmc passes, no tracing domains) for C2, C4, C5
# 4. L2 passes (TCC hit/miss, TCP->TCC read requests) for C4, C5
# 5. VALU passes (tools/pmc.sh) for C2, C4, C5 and the C2 frame in the statistical RNG mode
# 6. wave-cycle (stall) passes (tools/pmc_stall.sh) for C2 and the statistical RNG mode
# then tools/pmc_freeze.py -> profiles/pmc_measured.json is run by hand on the copies.
# STAGES (env, default all): any of "trace traffic l2 valu", so a call fits gpurun's limit.
set -e -o pipefail
OUT=${1:-gpurun_out/prof4}
STAGES=${STAGES:-trace traffic l2 valu stall}
has() { case " $STAGES " in *" $1 "*) return 0;; esac; return 1; }
export TMPDIR=/tmp
mkdir -p $OUT
ONE="--steps 1 --warmup 1 --no-cpu-baseline --no-trace-call --extra none"
if has trace; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/default -o run -- \
    python3 bench.py --steps 5 --warmup 2 > $OUT/bench_default.json 2> $OUT/bench_default.err
echo "default done"
for c in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c -o run -- \
      python3 bench.py --config $c $ONE > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  echo "$c trace done"
done
fi
P="--config CFG --steps 1 --warmup 0 --no-cpu-baseline --no-trace-call --extra none"
has traffic && for c in c2 c4 c5; do
  A=${P/CFG/$c}
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${c}_fetch -o run -- python3 bench.py $A > $OUT/${c}_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${c}_write -o run -- python3 bench.py $A > $OUT/${c}_write.log 2>&1
  python3 tools/pmc_traffic.py $OUT/${c}_fetch $OUT/${c}_write $OUT/pmc_$c.json
  echo "$c traffic done"
done
has l2 && for c in c4 c5; do
  A=${P/CFG/$c}
  timeout -k 10 400 bash tools/pmc_l2.sh $OUT/l2_$c $A > $OUT/l2_$c.txt 2>&1
  cp $OUT/l2_$c/l2.json $OUT/l2_$c.json
  echo "$c l2 done"
done
has valu && for c in c2 c4 c5 c2x; do
  A=${P/CFG/${c%x}}
  [ "$c" = c2x ] && A="$A --rng xoshiro"
  timeout -k 10 700 bash tools/pmc.sh $OUT/valu_$c $A > $OUT/valu_$c.txt 2>&1
  cp $OUT/valu_$c/valu.json $OUT/valu_$c.json
  echo "$c valu done"
done
has stall && for c in c2 c2x; do
  A=${P/CFG/c2}
  [ "$c" = c2x ] && A="$A --rng xoshiro"
  timeout -k 10 400 bash tools/pmc_stall.sh $OUT/stall_$c $A > $OUT/stall_$c.txt 2>&1
  echo "$c stall done"
done
find $OUT -name "*kernel_stats.csv" | sort
true
