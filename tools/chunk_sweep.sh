# DIAGNOSTIC: frame time vs the sample-chunk count of the trace launch (bench.py --chunks;
# 0 = ptmi's automatic choice).  usage: bash tools/chunk_sweep.sh "<configs>" "<chunk counts>" [spp]
set -e
for c in $1; do
  for k in $2; do
    timeout -k 10 200 python bench.py --config $c ${3:+--samples $3} --steps 2 --warmup 1 --no-cpu-baseline \
        --no-trace-call --chunks $k > gpurun_out/ch_${c}_$k.json 2>/dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/ch_${c}_$k.json'));print('$c chunks=$k', d['ms_per_step'], d['roofline']['frac'])"
  done
done
