#!/bin/bash
# Round 5: fused fit kernel with deferred coalesced saves (DRPO_FIT_DEFER): fit parity
# tests, then fit wall time A/B, three alternating rounds.
OUT=gpurun_out/${1:-r05aa}
mkdir -p $OUT
export TMPDIR=/tmp
LIBD=$PWD/distributional-reachability-policy-optimization_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fit" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest.log; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for t in base fitnd; do
    if [ $t = base ]; then L=""; else L="DRPO_LIB_OVERRIDE=$LIBD/libdrpo_hip_$t.so"; fi
    env $L FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit.log 2>&1 || exit 1
    echo "$t: $(tail -1 $OUT/fit.log)"
  done
done
