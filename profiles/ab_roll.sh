#!/bin/bash
# Rollout-only A/B of the production library against a tagged variant (alternating
# bench lines), plus config-2 stamps of the stamps build. Usage: bash profiles/ab_roll.sh <out> <variant> [rounds]
OUT=gpurun_out/$1
VAR=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_$2.so
N=${3:-3}
mkdir -p $OUT
export TMPDIR=/tmp
for i in $(seq $N); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/base_$i.json 2> $OUT/base_$i.err || exit 1
  DRPO_LIB_OVERRIDE=$VAR timeout -k 10 200 python -u bench.py --no-cpu-baseline --rollout-only > $OUT/var_$i.json 2> $OUT/var_$i.err || exit 1
done
if [ -f distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so ]; then
  DRPO_STAMPS_H=3 DRPO_STAMPS_CONFIG=2 DRPO_LIB_OVERRIDE=$PWD/distributional-reachability-policy-optimization_amd/libdrpo_hip_stamps.so DRPO_STAMPS_ROLLOUT=fused timeout -k 10 120 python profiles/stamps.py > $OUT/stamps_c2.txt 2>&1
  cat $OUT/stamps_c2.txt
fi
python profiles/summ.py $OUT/base_*.json $OUT/var_*.json
