#!/bin/bash
# DIAGNOSTIC: the round's GPU sessions as a list of named steps, run in order on the box
# (gpurun -- bash tools/gpu_steps.sh <out> <step> ...); the first failing step ends the run.
#   tests                      full `pytest -m gpu` of the product build
#   parity:<lib>               tests/test_gpu_parity.py against build/exp/libptmi_<lib>.so
#   ab:<spp>:<cfgs>:<variants> tools/diag_ab.sh (cfgs / variants comma-separated)
#   bench                      the default bench command (the driver's)
#   prof:<cfg>                 rocprofv3 --kernel-trace --stats of bench.py --config <cfg> --extra none
#   profx:<name>:<lib>:<args>  the same for build/<lib>.so and bench args (comma-separated), e.g. the split form
#   pmc:<cfg>:<counters>       one rocprofv3 --pmc pass (counters comma-separated) of the same
#   pmcx:<name>:<lib>:<ctrs>:<args>  one --pmc pass of any bench command with build/<lib>.so
#   shards:<cfgs>:<worlds>     tools/shard_balance.py (comma-separated lists)
#   shardsk:<tag>:<cfgs>:<worlds>:<knobs>  the same with work-plan knobs (NAME=VALUE, comma-separated)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  echo "== $step ($(date +%T))"
  case $kind in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 \
        || { tail -30 $OUT/tests.log; exit 1; }
      tail -1 $OUT/tests.log ;;
    parity)
      PTMI_LIB=pathtracer-ocl_amd/build/exp/libptmi_$a.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
        -x -q --timeout 200 --timeout-method thread > $OUT/parity_$a.log 2>&1 || { tail -30 $OUT/parity_$a.log; exit 1; }
      tail -1 $OUT/parity_$a.log ;;
    ab)
      bash tools/diag_ab.sh $OUT/ab $a "${b//,/ }" "${c//,/ }" || exit 1 ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'],{k:v['ms_per_step'] for k,v in d.get('extra_configs',{}).items()})" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$a -o run -- python3 bench.py --config $a --steps 3 \
        --warmup 1 --extra none --no-cpu-baseline --no-trace-call > $OUT/prof_$a.json 2> $OUT/prof_$a.err \
        || { tail -20 $OUT/prof_$a.err; exit 1; } ;;
    profx)  # profx:<name>:<lib>:<bench args, comma-separated>: kernel trace of any bench command
      L=pathtracer-ocl_amd/build/${b}.so
      PTMI_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$a -o run -- python3 bench.py \
        ${c//,/ } --extra none --no-cpu-baseline --no-trace-call > $OUT/prof_$a.json 2> $OUT/prof_$a.err \
        || { tail -20 $OUT/prof_$a.err; exit 1; } ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc ${b//,/ } --output-format csv -d $OUT/pmc_${a}_${b//,/_} -o run -- python3 bench.py --config $a \
        --steps 1 --warmup 1 --extra none --no-cpu-baseline --no-trace-call > /dev/null 2> $OUT/pmc_$a.err \
        || { tail -20 $OUT/pmc_$a.err; exit 1; } ;;
    pmcx)  # pmcx:<name>:<lib>:<counters>:<bench args>, all comma-separated lists
      IFS=: read -r kind a b c d <<< "$step"
      PTMI_LIB=pathtracer-ocl_amd/build/${b}.so timeout -s KILL 400 rocprofv3 --pmc ${c//,/ } --output-format csv \
        -d $OUT/pmcx_${a} -o run -- python3 bench.py ${d//,/ } --extra none --no-cpu-baseline --no-trace-call \
        > $OUT/pmcx_$a.json 2> $OUT/pmcx_$a.err || { tail -20 $OUT/pmcx_$a.err; exit 1; } ;;
    shards)  # shards:<configs>:<worlds>: every rank's share timed on this GPU (tools/shard_balance.py)
      timeout -k 10 600 python3 tools/shard_balance.py $OUT/shards.json --configs $a --worlds $b > $OUT/shards.log 2>&1 \
        || { tail -20 $OUT/shards.log; exit 1; }
      tail -12 $OUT/shards.log ;;
    shardsk)  # shardsk:<tag>:<cfgs>:<worlds>:<knobs, comma-separated NAME=VALUE>
      IFS=: read -r kind a b c d <<< "$step"
      kn=""; for kv in ${d//,/ }; do case $kv in split=*) kn="$kn --split ${kv#split=}";; *) kn="$kn --knob $kv";; esac; done
      timeout -k 10 600 python3 tools/shard_balance.py $OUT/shards_$a.json --configs $b --worlds $c $kn \
        > $OUT/shards_$a.log 2>&1 || { tail -20 $OUT/shards_$a.log; exit 1; }
      grep -E "^c[0-9] " $OUT/shards_$a.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
