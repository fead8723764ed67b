#!/bin/bash
# SAC per-launch timings (profiles/sac_micro.py) and the default bench line, twice
# each. Usage: bash profiles/order_ab.sh <tag>
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python -u profiles/sac_micro.py --steps 10 > $OUT/micro_$i.json 2> $OUT/micro_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 1
done
python profiles/summ.py $OUT/bench_1.json $OUT/bench_2.json $OUT/micro_1.json $OUT/micro_2.json
