#!/bin/bash
# Fit-step A/B (profiles/fit_profile.py, 3000 steps) of the production library against
# tagged variants, alternating, N rounds. Usage: bash profiles/ab_fit.sh <out> <rounds> <variant-tag>...
OUT=gpurun_out/$1
N=$2
shift 2
mkdir -p $OUT
export TMPDIR=/tmp
D=$PWD/distributional-reachability-policy-optimization_amd
for i in $(seq $N); do
  FIT_STEPS=3000 timeout -k 10 120 python -u profiles/fit_profile.py >> $OUT/base.txt 2>&1 || exit 1
  for v in "$@"; do
    DRPO_LIB_OVERRIDE=$D/libdrpo_hip_$v.so FIT_STEPS=3000 timeout -k 10 120 python -u profiles/fit_profile.py >> $OUT/$v.txt 2>&1 || exit 1
  done
done
for f in $OUT/*.txt; do echo "$f: $(grep -o '[0-9.]* ms per fit step' $f | tr '\n' ' ')"; done
