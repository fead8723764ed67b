#!/bin/bash
# Round 5: fused fit kernel epilogue-order A/B (fit wall time, phase stamps incl. the
# weight-gradient + Adam launch).
OUT=gpurun_out/${1:-r05l}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
for rep in 1 2; do
  for v in "" "DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_epif.so"; do
    env $v FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
    echo "[$v]: $(tail -1 $OUT/fit.log)"
  done
done
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps_epif.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps_epif.txt 2>&1 || exit 1
cat $OUT/fit_stamps.txt; echo EPIF; grep -v "^/opt" $OUT/fit_stamps_epif.txt | head -20
