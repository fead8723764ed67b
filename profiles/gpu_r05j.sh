#!/bin/bash
# Round 5: fused fit kernel with cross-phase weight prefetch: parity, fit wall time
# (default ring 6 / ring 8 / two-launch path), phase stamps.
OUT=gpurun_out/${1:-r05j}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fit_fb or full_width_fit or fused_adam" > $OUT/pytest_fb.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest_fb.log; tail -4 $OUT/pytest_fb.log
[ $rc -eq 0 ] || exit 1
for v in "DRPO_FIT_FB=1" "DRPO_FIT_FB=1 DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_pf8.so" "DRPO_FIT_FB=0"; do
  for rep in 1 2; do
    env $v FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
    echo "$v: $(tail -1 $OUT/fit.log)"
  done
done
DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_stamps.so timeout -k 10 120 python -u profiles/fit_stamps.py > $OUT/fit_stamps.txt 2>&1 || exit 1
cat $OUT/fit_stamps.txt
