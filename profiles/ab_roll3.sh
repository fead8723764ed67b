#!/bin/bash
# Rollout-only A/B of the production library against tagged variants (alternating
# bench lines). Usage: bash profiles/ab_roll3.sh <out> <variant-tag>...
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
D=$PWD/distributional-reachability-policy-optimization_amd
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/base_$i.json 2> $OUT/base_$i.err || exit 1
  for v in "$@"; do
    DRPO_LIB_OVERRIDE=$D/libdrpo_hip_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit 1
  done
done
python profiles/summ.py $OUT/base_*.json
for v in "$@"; do python profiles/summ.py $OUT/${v}_*.json; done
