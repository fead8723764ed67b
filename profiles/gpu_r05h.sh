#!/bin/bash
# Round 5: fused fit forward + NLL + backward-data (drpo_ens_fit_fb): its parity tests
# first, the fit A/B (one launch vs two) wall time and kernel stats, then the GPU suite.
OUT=gpurun_out/${1:-r05h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fit_fb or full_width_fit or fused_adam" > $OUT/pytest_fb.log 2>&1
rc=$?; echo "pytest rc $rc" >> $OUT/pytest_fb.log; tail -15 $OUT/pytest_fb.log
[ $rc -eq 0 ] || exit 1
for fb in 1 0; do
  DRPO_FIT_FB=$fb FIT_STEPS=300 timeout -k 10 120 python -u profiles/fit_profile.py > $OUT/fit_fb$fb.log 2>&1 || exit 1
  echo "fb=$fb $(tail -1 $OUT/fit_fb$fb.log)"
done
for fb in 1 0; do
  DRPO_FIT_FB=$fb FIT_STEPS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/prof_fb$fb -o fit -- python3 profiles/fit_profile.py > $OUT/prof_fb$fb.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $OUT/pytest.log 2>&1
echo "pytest rc $?" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
