#!/bin/bash
# Round 5: member-affine XCD placement of the fit's two launches (fit_fb + wgrad/Adam):
# parity, fit wall-time A/B, phase stamps.
OUT=gpurun_out/${1:-r05m}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_wgrad.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fit or wgrad" > $OUT/pytest_fb.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest_fb.log; tail -4 $OUT/pytest_fb.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in "" "DRPO_WGRAD_AFFINE=0" "DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_noaff.so" "DRPO_WGRAD_AFFINE=0 DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_noaff.so"; do
    env $v FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
    echo "[$v]: $(tail -1 $OUT/fit.log)"
  done
done
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
grep -v "^/opt" $OUT/fit_stamps.txt
