#!/bin/bash
# A/B of the production library against a tagged variant build (same sources, other -D
# macros: build_lib.py --tag T -D ...), alternating default bench lines (and SAC
# per-launch timings). Usage: bash profiles/ab_lib.sh <out-tag> <variant-tag> [rounds]
OUT=gpurun_out/$1
VAR=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_$2.so
N=${3:-2}
mkdir -p $OUT
export TMPDIR=/tmp
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/base_$i.json 2> $OUT/base_$i.err || exit 1
  DRPO_LIB_OVERRIDE=$VAR timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/var_$i.json 2> $OUT/var_$i.err || exit 1
done
python profiles/summ.py $OUT/base_*.json $OUT/var_*.json
