#!/bin/bash
# Full default bench (rollout + SAC + fit) of the production library against tagged
# variants, alternating, N rounds. Usage: bash profiles/ab_full.sh <out> <rounds> <variant-tag>...
OUT=gpurun_out/$1
N=$2
shift 2
mkdir -p $OUT
export TMPDIR=/tmp
D=$PWD/distributional-reachability-policy-optimization_amd
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/base_$i.json 2> $OUT/base_$i.err || exit 1
  for v in "$@"; do
    DRPO_LIB_OVERRIDE=$D/libdrpo_hip_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/${v}_$i.json 2> $OUT/${v}_$i.err || exit 1
  done
done
python profiles/summ.py $OUT/base_*.json
for v in "$@"; do python profiles/summ.py $OUT/${v}_*.json; done
